"""Parity of the HIP path (through the C-ABI) with the reference and the oracle.

  * every golden case (outputs of the reference script itself) through the
    drop-in CLI: identical bytes in all three files and identical exit status
  * seeded synthetic batches vs the C oracle, call by call, with
    min_depth_factor = -1 (every pileup slot is emitted: full-pileup parity)
"""
import importlib
import os

import numpy as np
import pytest

import geometry_util as geo
import golden_util as gu
import oracle

pytestmark = pytest.mark.gpu

KEYS = ("base", "chrom1", "chrom2", "count", "count2", "total")


@pytest.fixture(scope="module")
def cli():
    return importlib.import_module("minion-plasmid-consensus_amd.mapped_paf_read_parser")


@pytest.mark.parametrize("case", gu.cases())
def test_cli_matches_reference(case, tmp_path, cli):
    ref, reads, paf = gu.materialize(case, str(tmp_path))
    for k, run, exp in gu.runs(case):
        outs = [str(tmp_path / f"o{k}_{x}") for x in ("c.fa", "ch.tsv", "acc.tsv")]
        rc = cli.main(["--ref", ref, "--reads", reads, "--paf", paf, "--consensus", outs[0], "--chromat", outs[1],
                       "--accuracies", outs[2], "--min_depth_factor", repr(run["mdf"]),
                       "--global_threshold_factor", repr(run["gtf"])])
        if case in gu.DIVERGENT:  # pinned divergence: the reference writes files, the drop-in rejects
            assert run["exit"] == 0 and rc == 1, (case, k, gu.DIVERGENT[case])
            assert not any(os.path.exists(o) for o in outs)
            continue
        assert rc == run["exit"], (case, k)
        if rc == 0:
            for o, f in zip(outs, ("c.fa", "ch.tsv", "acc.tsv")):
                assert open(o, "rb").read() == exp[f], (case, k, f)
        else:
            assert not any(os.path.exists(o) for o in outs), "no partial outputs on failure"


def test_cli_jobs_own_reads_one_launch(tmp_path, cli):
    """--job (a batch of plasmids, each with its OWN reads file, one launch):
    every job's three files equal the reference's golden outputs of its case."""
    cases = ["r01_default_sense", "r03_indel_antisense", "t2a_order", "r06_smallref_sense"]
    argv, outs, exps = [], [], []
    run_of = {}
    for c in cases:
        d = tmp_path / c
        d.mkdir()
        ref, reads, paf = gu.materialize(c, str(d))
        k, run, exp = next(iter(gu.runs(c)))
        run_of[c] = run
        o = [str(d / f"o_{x}") for x in ("c.fa", "ch.tsv", "acc.tsv")]
        argv += ["--job", ref, paf, reads, *o]
        outs.append(o)
        exps.append(exp)
    mdfs = {(r["mdf"], r["gtf"]) for r in run_of.values()}
    assert len(mdfs) == 1, mdfs  # one (mdf, gtf) per launch
    mdf, gtf = mdfs.pop()
    assert cli.main(argv + ["--min_depth_factor", repr(mdf), "--global_threshold_factor", repr(gtf)]) == 0
    for c, o, exp in zip(cases, outs, exps):
        for path, f in zip(o, ("c.fa", "ch.tsv", "acc.tsv")):
            assert open(path, "rb").read() == exp[f], (c, f)


@pytest.mark.parametrize("stem", ["r01_default", "r03_indel"])
def test_cli_both_strands_one_launch(stem, tmp_path, cli):
    """--also (sense + antisense in one launch, same reads file) and --revcomp
    (rule revcomp_antisense_consensus): every file equals the golden per-strand
    outputs of the reference, the revcomp file the rule applied to them."""
    (ts, s), (ta, a) = [(tmp_path / x, f"{stem}_{x}") for x in ("sense", "antisense")]
    ts.mkdir()
    ta.mkdir()
    ref_s, reads, paf_s = gu.materialize(s, str(ts))
    ref_a, _, paf_a = gu.materialize(a, str(ta))
    for (k, run, exp_s), (_, run_a, exp_a) in zip(gu.runs(s), gu.runs(a)):
        assert (run["mdf"], run["gtf"]) == (run_a["mdf"], run_a["gtf"])
        o_s = [str(ts / f"o{k}_{x}") for x in ("c.fa", "ch.tsv", "acc.tsv")]
        o_a = [str(ta / f"o{k}_{x}") for x in ("c.fa", "ch.tsv", "acc.tsv")]
        rc_path = str(ta / f"o{k}_rc.fa")
        rc = cli.main(["--ref", ref_s, "--reads", reads, "--paf", paf_s, "--consensus", o_s[0], "--chromat", o_s[1],
                       "--accuracies", o_s[2], "--min_depth_factor", repr(run["mdf"]),
                       "--global_threshold_factor", repr(run["gtf"]), "--also", ref_a, paf_a, *o_a,
                       "--revcomp", o_a[0], rc_path])
        assert rc == 0, (stem, k)
        for outs, exp in ((o_s, exp_s), (o_a, exp_a)):
            for o, f in zip(outs, ("c.fa", "ch.tsv", "acc.tsv")):
                assert open(o, "rb").read() == exp[f], (stem, k, f)
        seq = exp_a["c.fa"].decode().split("\n")[1]
        comp = {"A": "T", "T": "A", "C": "G", "G": "C", "N": "N"}
        assert open(rc_path).read() == ">consensus\n" + "".join(comp[b] for b in reversed(seq))


def _oracle(s, mdf, gtf):
    return oracle.run_packed(s["ref"], s["cs"], s["cs_off"], s["tstart"], s["up"], s["up_off"], s["down"],
                             s["down_off"], mdf, gtf)


def _cmp(got, exp, tag):
    assert got["max_depth"] == exp["max_depth"], tag
    for k in KEYS:
        a = np.asarray(got[k], dtype=np.int64)
        b = np.asarray(exp[k], dtype=np.int64)
        assert a.shape == b.shape, (tag, k, a.shape, b.shape)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0][:5]
            raise AssertionError(f"{tag} {k} differs at {bad.tolist()}: {a[bad].tolist()} vs {b[bad].tolist()}")


SYNTH = [
    dict(n=2686, n_reads=3000, profile="default", seed=2, frac_partial=0.02),
    dict(n=1500, n_reads=2000, profile="default", seed=21, frac_partial=0.4),
    dict(n=1000, n_reads=1500, profile="indel", seed=4, frac_partial=0.1),
    dict(n=700, n_reads=800, profile="indel", seed=41, frac_partial=0.6, ins_len=(1, 12), del_len=(1, 30),
         flank=(0, 200)),
    dict(n=50, n_reads=2000, profile="c1probe", seed=7, frac_partial=0.5, flank=(0, 8)),
    dict(n=3000, n_reads=500, profile="default", seed=9, frac_partial=0.3, ins_len=(1, 1500), del_len=(1, 1200),
         p_ins=0.0005, p_del=0.0005, flank=(0, 3000)),
    # K_flank: 64 reads' flanks around its 2032-byte per-wave stage (some waves
    # one stage, some two: the owner carry across the stage boundary)
    dict(n=900, n_reads=6000, profile="indel", seed=73, frac_partial=0.5, flank=(0, 64)),
    # every K_parse tally mode the planner uses (tests/geometry_util.py): the
    # shortest reference in each LDS mode, mode 3 also with 3 substitution
    # windows (> 2 x 16384 positions), and the global-atomic mode 0
]
SYNTH += [dict(n=geo.first_length(m), n_reads=1000, profile="default" if m != 3 else "indel", seed=43 + m,
               frac_partial=0.2) for m in (1, 2, 3)]
SYNTH += [dict(n=geo.first_length(3, 2 * 16384), n_reads=150, profile="indel", seed=47, frac_partial=0.3),
          dict(n=geo.first_length(0), n_reads=60, profile="default", seed=46, frac_partial=0.3)]


def test_every_tally_mode_planned():
    """The planner still reaches every mode at some reference length."""
    assert {0, 1, 2, 3} <= set(geo.mode_lengths())


@pytest.mark.parametrize("spec", SYNTH, ids=lambda s: f"n{s['n']}_N{s['n_reads']}_{s['profile']}_s{s['seed']}")
def test_synthetic_full_pileup(pkg, spec):
    syn = pkg.synth.Synth(**spec)
    samples = [syn.sample(0), syn.sample(1)]
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0), (0.5, 2.5)):
        res = pkg.engine.pileup(samples, mdf, gtf)
        for s, (smp, r) in enumerate(zip(samples, res)):
            _cmp(r, _oracle(smp, mdf, gtf), (spec["seed"], s, mdf, gtf))


def test_flank_chunk_ranges_across_samples(pkg):
    """K_flank with more read chunks than blocks (each block a contiguous range
    of chunks, its LDS windows re-placed where the range crosses into another
    sample's hot gaps), long flanks around the per-wave stage, four samples."""
    specs = [dict(n=600, n_reads=70_000, profile="indel", seed=81, frac_partial=0.3, flank=(0, 64)),
             dict(n=450, n_reads=70_000, profile="default", seed=82, frac_partial=0.3, flank=(0, 40))]
    samples = []
    for sp in specs:
        syn = pkg.synth.Synth(**sp)
        samples += [syn.sample(0), syn.sample(1)]
    n_reads = sum(len(smp["tstart"]) for smp in samples)
    assert (n_reads + 511) // 512 > 512  # more 512-read chunks than K_flank's 512 blocks
    res = pkg.engine.pileup(samples, -1.0, 1.0)
    for s, (smp, r) in enumerate(zip(samples, res)):
        _cmp(r, _oracle(smp, -1.0, 1.0), ("flank_ranges", s))


def test_repeat_launches_identical(pkg):
    """Integer atomics: the result does not depend on wave scheduling."""
    syn = pkg.synth.Synth(n=1200, n_reads=4000, profile="indel", seed=77, frac_partial=0.3)
    samples = [syn.sample(0)]
    batch = pkg.engine.Batch(samples)
    plan = pkg.engine.Plan(batch, row_cap=200000)
    first = None
    for _ in range(5):
        plan.run(-1.0, 1.0)
        got = plan.fetch()[0]
        if first is None:
            first = got
            _cmp(got, _oracle(samples[0], -1.0, 1.0), "repeat")
        else:
            _cmp(got, first, "repeat")


@pytest.mark.parametrize("parse_cus,R", [(0, 2), (40, 2), (48, 3)])
def test_batches_in_flight_on_two_streams(pkg, parse_cus, R):
    """bench.py --inflight: independent plans on R streams, steps interleaved
    without host synchronisation, each equal to the oracle (the look-back status
    words of concurrent launches carry different epochs); with the parse grid
    sized for fewer CUs (mpc_input.parse_cus) as bench.py does."""
    import torch
    syn = pkg.synth.Synth(n=2686, n_reads=6000, profile="default", seed=91, frac_partial=0.2)
    samples = [syn.sample(0), syn.sample(1)]
    runners = [pkg.engine.Runner(samples, parse_cus=parse_cus) for _ in range(R)]
    if parse_cus:
        assert runners[0].plan.info()["parse_workgroups"] <= parse_cus
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(R - 1)]
    for k in range(4 * R):
        with torch.cuda.stream(streams[k % R]):
            runners[k % R].step(0.1, 5.0)
    torch.cuda.synchronize()
    exp = [_oracle(s, 0.1, 5.0) for s in samples]
    for r in runners:
        r.check()
        for s, (got, e) in enumerate(zip(r.fetch(), exp)):
            _cmp(got, e, ("in flight", s))


def test_capacity_replan(pkg):
    syn = pkg.synth.Synth(n=400, n_reads=500, profile="default", seed=3, frac_partial=0.5, flank=(0, 100))
    samples = [syn.sample(0)]
    res = pkg.engine.pileup(samples, -1.0, 1.0, row_cap=10)
    _cmp(res[0], _oracle(samples[0], -1.0, 1.0), "replan")


def test_many_samples_one_launch(pkg):
    samples, exp = [], []
    for k in range(12):
        syn = pkg.synth.Synth(n=300 + 37 * k, n_reads=200 + 20 * k, profile="indel" if k % 2 else "default",
                              seed=100 + k, frac_partial=0.2, antisense=False)
        samples.append(syn.sample(0))
    res = pkg.engine.pileup(samples, 0.1, 5.0)
    for k, (s, r) in enumerate(zip(samples, res)):
        _cmp(r, _oracle(s, 0.1, 5.0), ("multi", k))


SHARDED = [(SYNTH[0], 2), (SYNTH[1], 3), (SYNTH[2], 2), (SYNTH[3], 3), (SYNTH[4], 4), (SYNTH[5], 2)]


@pytest.mark.parametrize("spec,n_shards", SHARDED,
                         ids=lambda x: f"{x}" if isinstance(x, int) else f"n{x['n']}_{x['profile']}_s{x['seed']}")
def test_sharded_matches_oracle(pkg, spec, n_shards):
    """Reads split into contiguous shards (multi-GPU protocol of dist.py, all
    shards on this GPU, exchanges in-process): every shard ends with the
    single-pileup result, bit-exact."""
    dist = importlib.import_module("minion-plasmid-consensus_amd.dist")
    syn = pkg.synth.Synth(**spec)
    samples = [syn.sample(0), syn.sample(1)]
    sp = dist.ShardedPileup(dist.split_samples(samples, n_shards), [0] * n_shards)
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
        sp.step(mdf, gtf)
        exp = [_oracle(s, mdf, gtf) for s in samples]
        for k, plan in enumerate(sp.plans):
            for s, (r, e) in enumerate(zip(plan.fetch(), exp)):
                _cmp(r, e, ("shard", k, s, mdf))


def _packed(ref, css, tstarts, flank_seed=0):
    """A sample dict (synth layout) from explicit cs strings."""
    rng = np.random.default_rng(flank_seed)
    cs_b = [c.encode() for c in css]
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    ups = [rng.choice(acgt, int(rng.integers(0, 6))).tobytes() for _ in css]
    dns = [rng.choice(acgt, int(rng.integers(0, 6))).tobytes() for _ in css]
    off = lambda xs: np.concatenate([[0], np.cumsum([len(x) for x in xs])]).astype(np.int64)
    arr = lambda xs: np.frombuffer(b"".join(xs) or b"", dtype=np.uint8).copy()
    return dict(ref=np.frombuffer(ref, dtype=np.uint8).copy(), cs=arr(cs_b), cs_off=off(cs_b),
                tstart=np.asarray(tstarts, dtype=np.int64), up=arr(ups), up_off=off(ups), down=arr(dns),
                down_off=off(dns))


def _dense_cs(rng, n, ts):
    """Valid cs made of 1-3 byte tokens (empty ':' operands are skipped by the
    reference unless last): up to one boundary per byte, so 2 KiB windows hit
    their unit cap, and ':'+op pairs sit at every distance and lane seam."""
    out, i = ["Z:"], ts
    stop = int(rng.integers(n // 2, n - 3))
    while True:
        r = rng.random()
        if r < 0.25:
            out.append(":")
        elif r < 0.45 and i < n - 1:
            k = int(rng.integers(1, 3))
            out.append(":%d" % k); i += k
        elif r < 0.6:
            out.append("+" + "".join(rng.choice(list("acgtACGT"), int(rng.integers(1, 3)))))
        elif r < 0.75 and i < n - 2:
            out.append("-" + "".join(rng.choice(list("acgt"), 1))); i += 1
        elif r < 0.9 and i < n - 1:
            out.append("*a" + str(rng.choice(list("cgtCGT")))); i += 1
        if i >= stop:
            out.append(":1")
            return "".join(out)


@pytest.mark.parametrize("seed", [1, 2])
def test_dense_tokens_match_oracle(pkg, seed):
    rng = np.random.default_rng(seed)
    n = 3000
    ref = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()
    ts = [int(rng.integers(0, 40)) for _ in range(300)]
    css = [_dense_cs(rng, n, t) for t in ts]
    smp = _packed(ref, css, ts, seed)
    assert max(np.diff(smp["cs_off"])) > 2048  # reads span several windows
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
        _cmp(pkg.engine.pileup([smp], mdf, gtf)[0], _oracle(smp, mdf, gtf), ("dense", seed, mdf))


def _mixed_cs(rng, n, ts, p_odd, exotic=False):
    """Valid cs of canonical units (':'-digits + '*' / '+' / '-' with 1-4 byte
    operands) with, at rate p_odd per unit, a valid token the per-unit fast
    decode does not take: a ':' of 5-6 digits (leading zeros), a 5-7 base
    insertion, a deletion of non-base bytes, a '*' whose first byte is not a
    base, a 'Z' with an operand, an empty op right after a ':' prefix, ':0'.
    exotic adds a ':' of 9 digits and a '*' with a 5-byte operand."""
    out, i = ["Z::"], ts
    stop = int(rng.integers(n // 2, n - 60))
    while i < stop:
        out.append(":%d" % int(rng.integers(1, 30)))
        i += int(out[-1][1:])
        if rng.random() < p_odd:
            k = int(rng.integers(0, 9 if exotic else 7))
            if k == 0:
                out.append(":%05d" % int(rng.integers(0, 9))); i += int(out[-1][1:])
            elif k == 1:
                out.append("+" + "".join(rng.choice(list("acgtACGT"), int(rng.integers(5, 8)))))
            elif k == 2:
                out.append("-" + "".join(rng.choice(list("nNxq"), int(rng.integers(1, 4))))); i += len(out[-1]) - 1
            elif k == 3:
                out.append("*n" + str(rng.choice(list("acgt")))); i += 1
            elif k == 4:
                out.append("Z" + "".join(rng.choice(list("acgt"), int(rng.integers(1, 4)))))
            elif k == 5:
                out.append("*")  # empty: nothing, the ':' before it still advances
            elif k == 6:
                out.append(":0")
            elif k == 7:
                out.append(":%09d" % int(rng.integers(0, 9))); i += int(out[-1][1:])
            else:
                out.append("*" + "".join(rng.choice(list("acgt"), 5))); i += 1
        else:
            r = rng.random()
            if r < 0.5:
                out.append("*" + str(rng.choice(list("acgt"))) + str(rng.choice(list("acgtACGT")))); i += 1
            elif r < 0.75:
                out.append("+" + "".join(rng.choice(list("acgtACGT"), int(rng.integers(1, 5)))))
            else:
                k = int(rng.integers(1, 5))
                out.append("-" + "".join(rng.choice(list("acgt"), k))); i += k
    out.append(":1")
    return "".join(out)


@pytest.mark.parametrize("n,p_odd,exotic", [(4000, 0.0, False), (4000, 0.002, False), (4000, 0.02, False),
                                             (12000, 0.0, False), (12000, 0.02, False), (4000, 0.002, True),
                                             (12000, 0.02, True)])
def test_mixed_canonical_windows_match_oracle(pkg, n, p_odd, exotic):
    """Canonical units only, and rounds holding a few valid tokens the fast
    decode does not take (they are redone on the general decode): bit-exact
    against the oracle, full pileup and at the pipeline's thresholds."""
    eng = pkg.engine
    rng = np.random.default_rng(int(p_odd * 1000) + n + exotic)
    ref = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()
    ts = [int(rng.integers(0, 200)) for _ in range(400)]
    css = [_mixed_cs(rng, n, t, p_odd, exotic) for t in ts]
    smp = _packed(ref, css, ts, 11)
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
        _cmp(eng.pileup([smp], mdf, gtf)[0], _oracle(smp, mdf, gtf), ("mixed", n, p_odd, exotic, mdf))


def test_two_byte_substitutions_mode3(pkg):
    """'*' tokens of two bytes ("*a": valid, :96 writes operand[-1]) packed
    densely in tally mode 3, where substitutions travel as 2-byte events in a
    per-chunk region sized from the chunk's cs bytes: one event per two bytes
    must fit (round 5's regions assumed three bytes per '*' and overran)."""
    rng = np.random.default_rng(96)
    n = geo.first_length(3) + 500
    ref = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()
    ts = [int(rng.integers(0, 50)) for _ in range(300)]
    css = []
    for t in ts:
        k = int(rng.integers(n // 3, n - t - 2))
        css.append("Z::" + "".join("*" + str(rng.choice(list("acgtACGT"))) for _ in range(k)) + ":1")
    smp = _packed(ref, css, ts, 5)
    plan = pkg.engine.Plan(pkg.engine.Batch([smp]))
    assert plan.info()["tally_mode"] == 3
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
        _cmp(pkg.engine.pileup([smp], mdf, gtf)[0], _oracle(smp, mdf, gtf), ("star2", mdf))


@pytest.mark.parametrize("mode,reads", [(1, 400), (3, 300), (1, 1), (3, 2)])
def test_deferred_placement_dense_insertions(pkg, mode, reads):
    """Insertions queued per wave in LDS and placed 64 at a time
    (mpc_kernels.hip MPC_DEFER_PLACE; mpc_plan_info.deferred_placement): reads
    of dense 1-4 base '+' tokens (every round fills the queue, bucket pages
    open during the flushes) plus longer ones (the overflow list, not queued),
    and single reads whose few events wait in the queue until the last flush."""
    rng = np.random.default_rng(400 + mode + reads)
    n = 3000 if mode == 1 else geo.first_length(3) + 500
    ref = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()
    css, ts = [], []
    for r in range(reads):
        t = int(rng.integers(0, 50))
        parts, i = ["Z"], t
        stop = n - 60 if reads > 2 else t + 40
        while i < stop:
            m = int(rng.integers(1, 4))
            parts.append(":%d" % m)
            i += m
            k = int(rng.integers(1, 5)) if rng.random() < 0.9 else int(rng.integers(5, 9))
            parts.append("+" + "".join(rng.choice(list("acgt"), k)))
        css.append("".join(parts) + ":2")
        ts.append(t)
    smp = _packed(ref, css, ts, 7)
    info = pkg.engine.Plan(pkg.engine.Batch([smp])).info()
    assert info["tally_mode"] == mode and info["deferred_placement"] == 1, info
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
        _cmp(pkg.engine.pileup([smp], mdf, gtf)[0], _oracle(smp, mdf, gtf), ("defer", mode, reads, mdf))


@pytest.mark.parametrize("n,mode,reads", [(300_000, 0, 40), (400_000, 4, 40), (1_500_000, 4, 16)])
def test_long_reference(pkg, n, mode, reads):
    """A 300 kb reference (parse state in LDS, tally mode 0), a 400 kb one past
    the LDS budget (tally mode 4: LEFT bitmap, insertion-bucket counters and
    event-sort cursors in HBM) and a 1.5 Mb one (coordinates past 2^20):
    bit-exact full pileup and at the pipeline's thresholds, against the
    oracle (the reference takes any length, mapped_paf_read_parser.py:161-184)."""
    syn = pkg.synth.Synth(n=n, n_reads=reads, profile="default", seed=48, frac_partial=0.5, antisense=True)
    samples = [syn.sample(0), syn.sample(1)]
    assert len(samples[0]["ref"]) == n
    plan = pkg.engine.Plan(pkg.engine.Batch(samples))
    assert plan.info()["tally_mode"] == mode
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
        res = pkg.engine.pileup(samples, mdf, gtf)
        for s, r in zip(samples, res):
            _cmp(r, _oracle(s, mdf, gtf), ("long_ref", n, mdf))


@pytest.mark.timeout(300)
def test_long_reference_mode4_many_reads(pkg):
    """Tally mode 4 under load: a 400 kb reference with 1,500
    indel-heavy reads, so the parse spans many workgroups and every chunk group,
    with thousands of insertion events per bucket placed through the HBM
    scatter cursors (parse_epilogue_big: other waves' device atomics seen after
    the barrier).  Bit-exact full pileup vs the oracle, and repeat launches give
    identical calls (the order of a bucket's events may vary, the counts may not)."""
    syn = pkg.synth.Synth(n=400_000, n_reads=1500, profile="indel", seed=49, frac_partial=0.9, antisense=False)
    samples = [syn.sample(0)]
    run = pkg.engine.Runner(samples)
    info = run.plan.info()
    assert info["tally_mode"] == 4 and info["parse_workgroups"] >= 8, info
    exp = _oracle(samples[0], -1.0, 1.0)
    first = None
    for rep in range(3):
        run.step(-1.0, 1.0)
        run.check()
        got = run.fetch()[0]
        if first is None:
            first = got
            _cmp(got, exp, "mode4_many")
        else:
            _cmp(got, first, ("mode4_repeat", rep))


@pytest.mark.timeout(300)
def test_max_reference_dense_windows(pkg):
    """the 32-bit coordinate bound at the largest reference
    (2^22 - 2 bases, tally mode 4) with parse windows packed with
    maximal advances -- 63 reads per window of "Z::4194302" (the window
    prefix of advances reaches ~63 x 2^22), long deletions, a substitution
    and a negative start -- bit-exact full pileup vs the oracle."""
    n = (1 << 22) - 2
    rng = np.random.default_rng(11)
    ref = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)].copy()
    cs, ts = [], []
    for k in range(130):
        cs.append(b"Z::%d" % n); ts.append(0)
    for k in range(6):
        cs.append(b"Z::1000-" + b"a" * 1000 + b":%d" % (n - 2000)); ts.append(0)
        cs.append(b"Z::2097150*" + b"gat"[k % 3: k % 3 + 1] + b"g" + b":%d" % (n - 2097151)); ts.append(0)
    cs.append(b"Z::%d" % (n + 1)); ts.append(-1)  # matches below 0 write nothing
    cs.append(b"Z::%d" % (n - 3)); ts.append(3)
    off = np.concatenate([[0], np.cumsum([len(c) for c in cs])]).astype(np.int64)
    z = np.zeros(len(cs) + 1, np.int64)
    smp = {"ref": ref, "cs": np.frombuffer(b"".join(cs), np.uint8).copy(), "cs_off": off,
           "tstart": np.array(ts, np.int64), "up": np.zeros(0, np.uint8), "up_off": z, "down": np.zeros(0, np.uint8),
           "down_off": z.copy()}
    plan = pkg.engine.Plan(pkg.engine.Batch([smp]))
    assert plan.info()["tally_mode"] == 4
    got = pkg.engine.pileup([smp], -1.0, 1.0)[0]
    exp = _oracle(smp, -1.0, 1.0)
    assert exp["max_depth"] == 130 + 12 + 2
    _cmp(got, exp, "max_ref_dense")
    # an advance past the 2^22 clamp from a negative coordinate: its true end
    # (here exactly n) is not representable -> rejected, never a wrong count
    bad = dict(smp, cs=np.frombuffer(b"Z::%d" % (n + 5), np.uint8).copy(), cs_off=np.array([0, 10], np.int64),
               tstart=np.array([-5], np.int64), up_off=np.zeros(2, np.int64), down_off=np.zeros(2, np.int64))
    with pytest.raises(pkg.engine.DataError) as e:
        pkg.engine.pileup([bad], -1.0, 1.0)
    assert e.value.flags & pkg.engine.DE_UNSUPPORTED


@pytest.mark.parametrize("seed", [5, 6])
def test_negative_starts_random(pkg, seed):
    """seeded batches with ~5 % negative target starts --
    upstream flanks, '+' insertions and downstream flanks that Python's
    negative wrap writes into ODD positions (:57-61, :67-71, :81-87, :300-303,
    :323), several per position in different read orders, between the
    one-base writes of the reads covering them -- call by call against the
    oracle, with a sample without negative starts in the same launch."""
    import neg_util
    samples = [neg_util.neg_sample(seed), neg_util.neg_sample(seed + 100, n=500, n_reads=1500, frac_neg=0.06)]
    syn = pkg.synth.Synth(n=700, n_reads=600, profile="indel", seed=seed, frac_partial=0.3, antisense=False)
    samples.append(syn.sample(0))
    batch = pkg.engine.Batch(samples)
    assert batch.neg_reads > 0
    run = pkg.engine.Runner(samples)
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0), (0.5, 2.5)):
        run.step(mdf, gtf)
        run.check()
        st = run.plan.status()
        assert st[pkg.engine.MPC_ST_WRAP_EVENTS] > 0 and st[pkg.engine.MPC_ST_WRAP_POS] > 0
        for k, (got, smp) in enumerate(zip(run.fetch(), samples)):
            _cmp(got, _oracle(smp, mdf, gtf), ("negative starts", seed, k, mdf))


def test_negative_starts_need_declaring(pkg):
    """A plan told there are no negative starts (mpc_input.neg_reads = 0)
    reports one as MPC_DE_UNSUPPORTED instead of writing anything out of range."""
    import neg_util
    smp = neg_util.neg_sample(5, n_reads=400)
    batch = pkg.engine.Batch([smp])
    batch.neg_reads = batch.neg_cs_bytes = 0
    plan = pkg.engine.Plan(batch)
    plan.run(-1.0, 1.0)
    with pytest.raises(pkg.engine.DataError) as e:
        plan.fetch()
    assert e.value.flags & pkg.engine.DE_UNSUPPORTED


def test_reference_past_coordinate_limit(pkg):
    """2^22 - 1 bases: beyond the coordinate scheme (mpc.h), rejected."""
    long = {"ref": np.zeros((1 << 22) - 1, dtype=np.uint8) + ord("A"), "cs": np.frombuffer(b"Z::1", np.uint8).copy(),
            "cs_off": np.array([0, 4], np.int64), "tstart": np.array([0], np.int64),
            "up": np.zeros(0, np.uint8), "up_off": np.zeros(2, np.int64), "down": np.zeros(0, np.uint8),
            "down_off": np.zeros(2, np.int64)}
    with pytest.raises(pkg.engine.MpcError):
        pkg.engine.Plan(pkg.engine.Batch([long]))


@pytest.mark.parametrize("spec,lo,hi", [
    # K_rsort's three paths by the count M of mixed RIGHT events (status word
    # MPC_ST_MIXED): LDS (M <= 8192), register (<= 32768 entries of one word),
    # HBM ping-pong beyond
    (dict(n=400, n_reads=4000, profile="indel", seed=4, frac_partial=0.5), 1, 8192),
    (dict(n=1000, n_reads=30000, profile="indel", seed=5, frac_partial=0.5), 8193, 32768),
    (dict(n=3000, n_reads=60000, profile="indel", seed=6, frac_partial=0.6), 32769, 10 ** 9),
], ids=["lds", "registers", "hbm"])
def test_mixed_right_sort_paths(pkg, spec, lo, hi):
    syn = pkg.synth.Synth(antisense=False, **spec)
    samples = [syn.sample(0)]
    runner = pkg.engine.Runner(samples)
    runner.step(-1.0, 1.0)
    runner.check()
    m = int(runner.plan.status()[pkg.engine.MPC_ST_MIXED])
    assert lo <= m <= hi, m
    _cmp(runner.fetch()[0], _oracle(samples[0], -1.0, 1.0), ("rsort", m))


@pytest.mark.parametrize("spec,lo,hi,path", [
    # more than 512 K_rsplit blocks: the multi-workgroup sort (K_rscan, K_rscatter,
    # K_rsegsort) -- gaps of up to 64 events -- and its fallback to K_rsort
    # (a gap with more); the path taken is read back (MPC_ST_RSORT_PATH)
    (dict(n=2000, n_reads=600_000, profile="default", seed=8, frac_partial=0.05), 8193, 600_000, 1),
    (dict(n=500, n_reads=600_000, profile="indel", seed=9, frac_partial=0.3), 8193, 600_000, 2),
], ids=["multi", "multi_fallback"])
def test_mixed_right_sort_many_reads(pkg, spec, lo, hi, path):
    syn = pkg.synth.Synth(antisense=False, **spec)
    samples = [syn.sample(0)]
    runner = pkg.engine.Runner(samples)
    runner.step(-1.0, 1.0)
    runner.check()
    m = int(runner.plan.status()[pkg.engine.MPC_ST_MIXED])
    assert lo <= m <= hi, m
    assert int(runner.plan.status()[pkg.engine.MPC_ST_RSORT_PATH]) == path
    _cmp(runner.fetch()[0], _oracle(samples[0], -1.0, 1.0), ("rsort many", m))


def test_mode3_windows_with_an_empty_sample(pkg):
    """Tally mode 3 with two substitution windows per sample (K_subs slab rows
    summed by K_subsum per sample and window) and a sample without reads in
    the same launch (no K_subs blocks, no K_subsum work: its tallies stay the
    cleared zeros)."""
    n = geo.first_length(3, 16384 + 100)
    syn = pkg.synth.Synth(n=n, n_reads=300, profile="indel", seed=71, frac_partial=0.3, antisense=False)
    full = syn.sample(0)
    empty = dict(full)
    empty.update(cs=np.zeros(0, np.uint8), cs_off=np.zeros(1, np.int64), tstart=np.zeros(0, np.int64),
                 up=np.zeros(0, np.uint8), up_off=np.zeros(1, np.int64), down=np.zeros(0, np.uint8),
                 down_off=np.zeros(1, np.int64), aligned=np.zeros(0, np.int64))
    samples = [full, empty, full]
    runner = pkg.engine.Runner(samples)
    assert runner.plan.info()["tally_mode"] == 3
    for mdf, gtf in ((-1.0, 1.0), (0.1, 5.0)):
        runner.step(mdf, gtf)
        runner.check()
        for k, (got, smp) in enumerate(zip(runner.fetch(), samples)):
            _cmp(got, _oracle(smp, mdf, gtf), ("mode3 empty", k, mdf))
