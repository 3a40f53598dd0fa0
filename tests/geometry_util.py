"""Reference lengths per K_parse tally mode, asked of the library's own planner
(host-only: mpc_plan_create + mpc_plan_info, no device), so the parity tests
cover every LDS / HBM tally mode whatever the planner's current thresholds."""
import functools
import importlib


@functools.lru_cache(maxsize=None)
def mode_lengths():
    """{tally_mode: [reference lengths]} for two strands x 1000 reads, scanning
    1-140 kb; every mode the planner uses below the HBM-state mode 4 appears."""
    eng = importlib.import_module("minion-plasmid-consensus_amd").engine
    out = {}
    for n in list(range(1000, 20001, 500)) + list(range(20000, 140001, 2500)):
        m = eng.geometry([n, n], [1000, 1000], n * 240)["tally_mode"]
        out.setdefault(m, []).append(n)
    return out


def first_length(mode, above=0):
    """The shortest reference (> ``above``) the planner runs in ``mode``."""
    return next(n for n in mode_lengths()[mode] if n > above)
