#!/bin/bash
set -o pipefail
# The round's final measurements part 1 (scripts/final_r04a.sh: smoke, suite,
# bench line + its kernel stats, PMC traffic)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out; cd $R
bash scripts/final_r04a.sh
