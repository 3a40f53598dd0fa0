"""Bit-exact parity at the BASELINE configs' FULL size (the pipeline's depth
regime, >= 10^5x coverage: /root/reference/README.md:32, :240).

Every config of bench.py, exactly as bench.py builds it at N=1, through the
C-ABI: the full pileup (min_depth_factor = -1: every slot emitted) against the
C oracle call by call, and the configured thresholds (0.1 / 5, config.yaml:38-39)
against the oracle's full pileup filtered by the reference's two tests
(depth_util.derive).  Matches mapped_paf_read_parser.py:292-439 at depth.

Plus the 16-bit LDS tally bound of K_parse: batches whose parse workgroups
hold exactly the reads-per-workgroup cap (mpc_plan_info), in every LDS tally
mode (tm 1 12-byte, tm 2 10-byte packed, tm 3 depth-only + substitution events).
"""
import importlib

import numpy as np
import pytest

import depth_util as du

pytestmark = pytest.mark.gpu

CONFIG_CASES = ["c1", "c2", "c3", "c4", "c5_slice", "c5"]


def _samples(pkg, case):
    bench = importlib.import_module("bench")
    if case == "c5_slice":  # 2 plasmids x 2 strands x 10k reads of 30 kb
        n, reads, _, profile, seed, anti, _ = bench.CONFIGS["c5"]
        out = []
        for k in range(2):
            syn = pkg.synth.Synth(n=n, n_reads=reads, profile=profile, seed=seed + k, antisense=anti)
            out += [syn.sample(0), syn.sample(1)]
        return out
    return bench.shard_samples(pkg, case, 0, 1)[0]


def _check(pkg, samples, tag, mode=None):
    full_exp = du.oracle_many(samples, -1.0, 1.0)
    runner = pkg.engine.Runner(samples)
    if mode is not None:
        assert runner.plan.info()["tally_mode"] == mode, runner.plan.info()
    runner.step(-1.0, 1.0)
    runner.check()
    for s, (got, exp) in enumerate(zip(runner.fetch(), full_exp)):
        du.compare(got, exp, (tag, s, "full"))
    for mdf, gtf in ((0.1, 5.0), (0.5, 2.5)):
        runner.step(mdf, gtf)
        runner.check()
        for s, (got, full) in enumerate(zip(runner.fetch(), full_exp)):
            du.compare(got, du.derive(full, mdf, gtf), (tag, s, mdf, gtf))
    return runner


@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", CONFIG_CASES)
def test_config_full_size(pkg, case):
    samples = _samples(pkg, case)
    _check(pkg, samples, case)


def _tiny_reads_batch(pkg, n_tiny, big_n, big_reads=100):
    """One ``big_n`` bp sample with a few reads (sets the tally mode) and one
    30 bp sample with ``n_tiny`` reads: its parse workgroups fill up to the
    reads-per-workgroup cap; high substitution / deletion rates and partial
    reads put many updates on every position's 16-bit counters."""
    a = pkg.synth.Synth(n=big_n, n_reads=big_reads, profile="default", seed=61, antisense=False)
    b = pkg.synth.Synth(n=30, n_reads=n_tiny, profile="default", seed=62, antisense=False, frac_partial=0.5,
                        flank=(0, 6), p_sub=0.4, p_del=0.1, p_ins=0.1, del_len=(1, 2), ins_len=(1, 2))
    return [a.sample(0), b.sample(0)]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", [2, 3])
def test_workgroup_cap_packed_tallies(pkg, mode):
    """Tally modes 2 (10-byte packed LDS tallies) and 3 (LDS depth, substitution
    events): 16383 reads per workgroup (the reference length that puts the
    planner in each mode: tests/geometry_util.py)."""
    import geometry_util as geo
    samples = _tiny_reads_batch(pkg, 16383 * 300, geo.first_length(mode))
    info = pkg.engine.Plan(pkg.engine.Batch(samples)).info()
    assert info["tally_mode"] == mode and info["max_reads_per_workgroup"] == info["reads_per_workgroup_cap"] == 16383
    _check(pkg, samples, "cap_tm%d" % mode, mode)


@pytest.mark.timeout(600)
def test_workgroup_cap_wide_tallies(pkg):
    """Tally mode 1 (12-byte LDS tallies: C1 / C2): 32767 reads per workgroup."""
    syn = pkg.synth.Synth(n=30, n_reads=32767 * 260, profile="default", seed=63, antisense=False, frac_partial=0.5,
                          flank=(0, 4), p_sub=0.4, p_del=0.1, p_ins=0.05, del_len=(1, 2), ins_len=(1, 2))
    samples = [syn.sample(0)]
    info = pkg.engine.Plan(pkg.engine.Batch(samples)).info()
    assert info["tally_mode"] == 1 and info["max_reads_per_workgroup"] == info["reads_per_workgroup_cap"] == 32767
    _check(pkg, samples, "cap_tm1", 1)


@pytest.mark.timeout(600)
def test_golden_depth_cli(tmp_path):
    """The drop-in CLI on the inputs of every tests/golden_depth case (the
    reference's own outputs at 10^3-10^4x depth) reproduces them byte for byte."""
    import depth_golden as dg
    cli = importlib.import_module("minion-plasmid-consensus_amd.mapped_paf_read_parser")
    for case in dg.cases():
        dg.check_cli(case, str(tmp_path / case), cli)
