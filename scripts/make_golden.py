#!/usr/bin/env python3
"""Generate tests/golden/ by running the REFERENCE script on seeded inputs.

Run in the build container only (the reference is never shipped anywhere):
    python3 scripts/make_golden.py [--ref-script /root/reference/src/mapped_paf_read_parser.py]

Each case directory holds the CLI inputs (ref.fa, reads.fa, in.paf; gzip'd when
larger than 4 KB), and for every (min_depth_factor, global_threshold_factor)
run the reference's exit status and its three output files.  The reference is
run as a subprocess with ``python3 -B`` (no bytecode written into the
read-only reference tree).  Fixtures are data: inputs and expected outputs.
"""
import argparse
import gzip
import importlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
synth = importlib.import_module("minion-plasmid-consensus_amd.synth")

GOLDEN = os.path.join(REPO, "tests", "golden")


def wfile(path, data):
    if isinstance(data, str):
        data = data.encode()
    if len(data) > 4096:
        with open(path + ".gz", "wb") as raw:
            with gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0, filename="") as f:
                f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)


def run_ref(script, d, mdf, gtf):
    out = {}
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    cmd = [sys.executable, "-B", script, "--ref", "ref.fa", "--reads", "reads.fa", "--paf", "in.paf",
           "--consensus", "c.fa", "--chromat", "ch.tsv", "--accuracies", "acc.tsv",
           "--min_depth_factor", repr(mdf), "--global_threshold_factor", repr(gtf)]
    for f in ("c.fa", "ch.tsv", "acc.tsv"):
        if os.path.exists(os.path.join(d, f)):
            os.remove(os.path.join(d, f))
    p = subprocess.run(cmd, cwd=d, env=env, capture_output=True, text=True)
    out["exit"] = p.returncode
    last = p.stderr.strip().splitlines()[-1] if p.stderr.strip() else ""
    out["error"] = last
    for f in ("c.fa", "ch.tsv", "acc.tsv"):
        fp = os.path.join(d, f)
        out[f] = open(fp, "rb").read() if os.path.exists(fp) else None
    return out


def emit_case(script, name, ref_fa, reads_fa, paf, runs, note=""):
    cdir = os.path.join(GOLDEN, name)
    if os.path.exists(cdir):
        shutil.rmtree(cdir)
    os.makedirs(cdir)
    with tempfile.TemporaryDirectory() as tmp:
        for fn, data in (("ref.fa", ref_fa), ("reads.fa", reads_fa), ("in.paf", paf)):
            with open(os.path.join(tmp, fn), "wb") as f:
                f.write(data if isinstance(data, bytes) else data.encode())
            wfile(os.path.join(cdir, fn), data)
        manifest = {"note": note, "runs": []}
        for k, (mdf, gtf) in enumerate(runs):
            r = run_ref(script, tmp, mdf, gtf)
            ent = {"mdf": mdf, "gtf": gtf, "exit": r["exit"], "error": r["error"], "files": {}}
            for f in ("c.fa", "ch.tsv", "acc.tsv"):
                if r[f] is not None:
                    ent["files"][f] = f"run{k}_{f}"
                    wfile(os.path.join(cdir, f"run{k}_{f}"), r[f])
            manifest["runs"].append(ent)
    with open(os.path.join(cdir, "case.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    codes = [e["exit"] for e in manifest["runs"]]
    print(f"{name}: exits {codes}")


def paf_line(name, qlen, qs, qe, strand, ts, te, cs, n=10, extra=""):
    return f"{name}\t{qlen}\t{qs}\t{qe}\t{strand}\tref\t{n}\t{ts}\t{te}\t0\t0\t60{extra}\tcs:Z:{cs}\n"


def hand_cases(script):
    R = ">ref\nACGTACGTAC\n"
    # t1: mixed strands, sub/ins/del, flanks, duplicate PAF line, top tie
    reads = ">r1\nGGACGTACGTACTT\n>r2\nACGTTGTACGTACTT\n>r3\nTTGTACGTAA\n"
    # r3 is '-' strand: revcomp(TTGTACGTAA) = TTACGTACAA ; qs'=qlen-qe
    paf = (paf_line("r1", 14, 2, 12, "+", 0, 10, ":10")
           + paf_line("r2", 15, 0, 12, "+", 0, 10, ":3*ta:3+tt:1-g:1")
           + paf_line("r3", 10, 1, 8, "-", 2, 9, ":7")
           + paf_line("r1", 14, 2, 12, "+", 0, 10, ":5"))
    emit_case(script, "t1_mixed", R, reads, paf, [(0.1, 1), (0.1, 5), (0, 1), (-1, 1)], "SURVEY App.B t1")
    # t2a / t2b: LEFT vs RIGHT order dependence at one even position
    ra = paf_line("a", 7, 0, 5, "+", 0, 5, ":5")
    rb = paf_line("b", 13, 0, 13, "+", 0, 10, ":5+ttt:5")
    reads = ">a\nACGTAGG\n>b\nACGTATTTCGTAC\n"
    emit_case(script, "t2a_order", R, reads, ra + rb, [(0, 1), (-1, 5)], "RIGHT then LEFT at even 10")
    emit_case(script, "t2b_order", R, reads, rb + ra, [(0, 1), (-1, 5)], "LEFT then RIGHT at even 10")
    # t5: second-base tie -> N with summed count
    R3 = ">r\nAAA\n"
    lines, rd = [], []
    for k in range(11):
        b2 = "A" if k < 7 else ("C" if k < 10 else "G")
        b3 = "A" if k < 7 else ("C" if k < 9 else "G")
        seq = "A" + b2 + b3
        cs = ":1" + (":1" if b2 == "A" else f"*a{b2.lower()}") + (":1" if b3 == "A" else f"*a{b3.lower()}")
        lines.append(paf_line(f"q{k}", 3, 0, 3, "+", 0, 3, cs, n=3))
        rd.append(f">q{k}\n{seq}\n")
    emit_case(script, "t5_ties", R3, "".join(rd), "".join(lines), [(0, 1), (0.5, 2.5), (0, 5)], "second-base tie")
    # error exits
    emit_case(script, "t3_N_in_flank", R, ">r1\nNGACGTACGTAC\n", paf_line("r1", 12, 2, 12, "+", 0, 10, ":10"),
              [(0.1, 5)], "N in upstream flank -> KeyError")
    emit_case(script, "t4_missing_read", R, ">zz\nACGT\n", paf_line("r1", 10, 0, 10, "+", 0, 10, ":10"),
              [(0.1, 5)], "PAF read absent from FASTA -> KeyError")
    emit_case(script, "e_empty_paf", R, ">r1\nACGT\n", "", [(0.1, 5)], "empty PAF")
    emit_case(script, "e_unknown_op", R, ">r1\nACGTACGTAC\n",
              "r1\t10\t0\t10\t+\tref\t10\t0\t10\t0\t0\t60\tcs:10\n", [(0.1, 5)], "cs without Z: -> unknown operator")
    emit_case(script, "e_past_end", R, ">r1\nACGTACGTACGG\n", paf_line("r1", 12, 0, 12, "+", 0, 10, ":12"),
              [(0.1, 5)], "match runs past reference end -> IndexError")
    emit_case(script, "e_minus_badchar", R, ">r1\nGTACGTRCGT\n", paf_line("r1", 10, 0, 10, "-", 0, 10, ":10"),
              [(0.1, 5)], "minus-strand read with R -> KeyError in revcomp")
    emit_case(script, "e_plus_N_aligned", R, ">r1\nACGTNCGTAC\n>r2\nACGTACGTAC\n",
              paf_line("r1", 10, 0, 10, "+", 0, 10, ":4*an:5").replace("*an", "*ac")
              + paf_line("r2", 10, 0, 10, "+", 0, 10, ":10"),
              [(0, 1)], "N inside a plus-strand aligned part is never written")
    emit_case(script, "e_multi_ref_lower", ">a\nacgt\n>b desc\nACGtac\n  \n", ">r1\nACGTACGTAC\n",
              paf_line("r1", 10, 0, 10, "+", 0, 10, ":10"), [(0, 1)], "multi-record + lowercase reference")
    emit_case(script, "e_pyint", R, ">r1\nACGTACGTAC\n>r2\nACGTACGTAC\n",
              paf_line("r1", 10, 0, 10, "+", 0, 10, ":1_0") + paf_line("r2", 10, 0, 10, "+", 0, 10, ":0010"),
              [(0, 1)], "int() accepts 1_0 and leading zeros")
    emit_case(script, "e_pyint_bad", R, ">r1\nACGTACGTAC\n", paf_line("r1", 10, 0, 10, "+", 0, 10, ":1__0"),
              [(0, 1)], "int('1__0') -> ValueError")
    emit_case(script, "e_star_long", R, ">r1\nACGTACGTAC\n", paf_line("r1", 10, 0, 10, "+", 0, 10, ":2*cagt:7"),
              [(0, 1)], "'*' uses the LAST operand character")
    emit_case(script, "e_consec_ins", R, ">r1\nTTGACAACGTACGTCCAAG\n>r2\nACGTACGTACAAA\n",
              paf_line("r1", 19, 2, 17, "+", 0, 10, "+ga+c:5+AA:5+cc") + paf_line("r2", 13, 0, 10, "+", 0, 10, ":10+aaa"),
              [(0, 1), (-1, 1)], "consecutive insertions, insertion at gap 0 after flank, at gap n")
    emit_case(script, "e_zero_len", R, ">r1\nGGTT\n>r2\nACGTACGTAC\n",
              paf_line("r1", 4, 2, 2, "+", 4, 4, ":0") + paf_line("r2", 10, 0, 10, "+", 0, 10, ":10"),
              [(0, 1), (-1, 1)], "zero-length alignment: LEFT then RIGHT at one gap")
    emit_case(script, "e_empty_cs", R, ">r1\nACGT\n", paf_line("r1", 4, 0, 4, "+", 0, 4, ""), [(0, 1)],
              "cs:Z: -> int('') ValueError")
    emit_case(script, "e_trailing_star", R, ">r1\nACGT\n", paf_line("r1", 4, 0, 4, "+", 0, 4, ":3*"), [(0, 1)],
              "trailing '*' -> IndexError")
    emit_case(script, "e_trailing_ops", R, ">r1\nACGT\n>r2\nACGT\n>r3\nACGT\n",
              paf_line("r1", 4, 0, 4, "+", 0, 4, ":4+") + paf_line("r2", 4, 0, 4, "+", 0, 4, ":4-")
              + paf_line("r3", 4, 0, 4, "+", 0, 4, ":4Z"), [(0, 1)], "trailing empty + - Z are no-ops")
    emit_case(script, "e_del_past_end_ok", R, ">r1\nACGTA\n", paf_line("r1", 5, 0, 5, "+", 0, 5, ":5-acgtacgtacgt"),
              [(0, 1)], "deletion past the end with empty downstream is fine")
    emit_case(script, "e_del_past_end_bad", R, ">r1\nACGTAGG\n", paf_line("r1", 7, 0, 5, "+", 0, 5, ":5-acgtacgtacgt"),
              [(0, 1)], "deletion past the end then downstream flank -> IndexError")
    emit_case(script, "e_sub_same", R, ">r1\nACGTACGTAC\n", paf_line("r1", 10, 0, 10, "+", 0, 10, ":3*tt:6"),
              [(0, 1)], "substitution to the reference base")
    emit_case(script, "e_crlf", R.replace("\n", "\r\n"), ">r1\r\nGGACGTACGTACTT\r\n",
              paf_line("r1", 14, 2, 12, "+", 0, 10, ":10").replace("\n", "\r\n"), [(0, 1)], "CRLF line endings")
    emit_case(script, "e_blank_paf_line", R, ">r1\nACGTACGTAC\n", paf_line("r1", 10, 0, 10, "+", 0, 10, ":10") + "\n",
              [(0, 1)], "blank PAF line -> IndexError")
    emit_case(script, "e_ref_N_sub_ok", ">r\nACGNACGTAC\n", ">r1\nACGTACGTAC\n",
              paf_line("r1", 10, 0, 10, "+", 0, 10, ":3*nt:6"), [(0, 1)], "N in the reference only substituted")
    emit_case(script, "e_ref_N_match_bad", ">r\nACGNACGTAC\n", ">r1\nACGTACGTAC\n",
              paf_line("r1", 10, 0, 10, "+", 0, 10, ":10"), [(0, 1)], "match over N in the reference -> KeyError")
    emit_case(script, "e_header_space", R, ">r1 extra\nACGTACGTAC\n", paf_line("r1", 10, 0, 10, "+", 0, 10, ":10"),
              [(0, 1)], "FASTA name is the whole header line -> missing -> KeyError")
    emit_case(script, "e_strand_dot", R, ">r1\nGGACGTACGTACTT\n", paf_line("r1", 14, 2, 12, ".", 0, 10, ":10"),
              [(0, 1)], "strand other than '-' is treated as '+'")
    emit_case(script, "e_slice_clamp", R, ">r1\nACGTACGTAC\n>r2\nACGTACGTAC\n",
              paf_line("r1", 8, 0, 10, "-", 0, 10, ":10") + paf_line("r2", 10, 12, 15, "+", 0, 10, ":10"),
              [(0, 1), (-1, 1)], "PAF coordinates that disagree with the read: Python slice semantics")
    emit_case(script, "e_dup_fasta", R, ">r1\nTTTTACGTACGTAC\n>r1\nGGACGTACGTACTT\n",
              paf_line("r1", 14, 2, 12, "+", 0, 10, ":10"), [(0, 1)], "duplicate FASTA record: last wins")
    emit_case(script, "e_thresholds", R, ">r1\nACGTACGTAC\n>r2\nACGTTCGTAC\n>r3\nACGTACGTAC\n",
              paf_line("r1", 10, 0, 10, "+", 0, 10, ":10") + paf_line("r2", 10, 0, 10, "+", 0, 10, ":4*at:5")
              + paf_line("r3", 10, 0, 5, "+", 0, 5, ":5"),
              [(1, 1), (0.5, 2), (0.666, 2.0), (0, 0), (-0.5, 100), (float("inf"), 1), (0, float("inf")),
               (float("nan"), 1)], "threshold edges incl. inf/nan")


def unicode_cases(script):
    """Non-ASCII text: the reference reads str, so coordinates
    count characters, str.upper() may change lengths, int() takes Unicode
    digits, and a non-ACGT character only fails where it is written."""
    R = ">ref\nACGTACGTAC\n"
    one = lambda cs, qlen=10, qs=0, qe=10, ts=0, te=10: paf_line("r1", qlen, qs, qe, "+", ts, te, cs)
    # reference: non-ASCII where no read writes (uncovered tail) -> fine; 'ß'.upper() == 'SS' shifts coordinates
    emit_case(script, "u_ref_tail", ">ref \u00e9t\u00e9\nACGTACGTAC\u00e9\u00df\u4e2d\n", ">r1\nACGTACGTAC\n",
              one(":10"), [(0, 1), (-1, 1)], "non-ASCII reference characters no read covers")
    emit_case(script, "u_ref_sharp_s", ">ref\nAC\u00dfGTACGT\n", ">r1\nGTACGT\n",
              one(":6", qlen=6, qs=0, qe=6, ts=4, te=10), [(0, 1), (-1, 1)], "upper() lengthens the reference")
    emit_case(script, "u_ref_matched", ">ref\nACGT\u00e9CGTAC\n", ">r1\nACGTACGTAC\n", one(":10"), [(0, 1)],
              "a matched non-ASCII reference base: KeyError")
    emit_case(script, "u_ref_subbed", ">ref\nACGT\u00e9CGTAC\n", ">r1\nACGTACGTAC\n", one(":4*\u00e9a:5"),
              [(0, 1), (-1, 1)], "a substituted non-ASCII reference base is never written")
    # cs operands
    emit_case(script, "u_del_operand", R, ">r1\nACGTCGTAC\n", one(":3-\u00e9:6", qlen=9, qe=9), [(0, 1), (-1, 1)],
              "deletion of a non-ASCII character counts one")
    emit_case(script, "u_del_cjk", R, ">r1\nACGTAC\n", one(":2-\u4e2d\u00fc\u00e9\u00df:4", qlen=6, qe=6), [(0, 1), (-1, 1)],
              "deletion operand of 4 non-ASCII characters")
    emit_case(script, "u_colon_fullwidth", R, ">r1\nACGTTCGTAC\n", one(":\uff14*at:\uff15"), [(0, 1), (-1, 1)],
              "int() of fullwidth digits")
    emit_case(script, "u_colon_arabic", R, ">r1\nACGTACGTAC\n", one(":\u0661\u0660"), [(0, 1)],
              "int() of Arabic-Indic digits (10)")
    emit_case(script, "u_colon_bad", R, ">r1\nACGTACGTAC\n", one(":1\u00e9"), [(0, 1)], "int() ValueError")
    emit_case(script, "u_sub_first", R, ">r1\nACGTTCGTAC\n", one(":4*\u00e9t:5"), [(0, 1), (-1, 1)],
              "only operand[-1] of '*' is written")
    emit_case(script, "u_sub_last", R, ">r1\nACGTTCGTAC\n", one(":4*a\u00e9:5"), [(0, 1)], "KeyError")
    emit_case(script, "u_ins", R, ">r1\nACGTTTCGTAC\n", one(":4+\u00e9:6", qlen=11, qe=11), [(0, 1)], "KeyError")
    emit_case(script, "u_z_operand", R, ">r1\nACGTACGTAC\n", one(":4Z\u00e9\u00e9:6"), [(0, 1), (-1, 1)],
              "'Z' ignores its operand")
    # reads: names, aligned part (never written), flanks (written)
    emit_case(script, "u_read_name", R, ">r\u00e9 x\nACGTACGTAC\n",
              paf_line("r\u00e9 x", 10, 0, 10, "+", 0, 10, ":10"), [(0, 1)], "non-ASCII read name")
    emit_case(script, "u_read_aligned", R, ">r1\nGGACGT\u00e9\u00dfCGTACTT\n",
              one(":10", qlen=16, qs=2, qe=13), [(0, 1), (-1, 1)], "non-ASCII inside the aligned part; 'ß' -> 'SS'")
    emit_case(script, "u_flank", R, ">r1\n\u00e9ACGTACGTAC\n", one(":10", qlen=11, qs=1, qe=11), [(0, 1)],
              "non-ASCII upstream flank base: KeyError")


def random_cases(script):
    specs = [
        # name, n, reads, profile, seed, frac_partial, flank, ins_len, del_len
        ("r01_default", 1200, 150, "default", 11, 0.02, (0, 40), (1, 3), (1, 3)),
        ("r02_partial", 1500, 160, "default", 12, 0.35, (0, 40), (1, 3), (1, 3)),
        ("r03_indel", 1000, 120, "indel", 13, 0.05, (0, 40), (1, 3), (1, 3)),
        ("r04_c1probe", 2000, 100, "c1probe", 14, 0.10, (0, 40), (1, 3), (1, 3)),
        ("r05_longins", 800, 120, "default", 15, 0.30, (0, 300), (1, 25), (1, 400)),
        ("r06_smallref", 60, 400, "indel", 16, 0.50, (0, 12), (1, 6), (1, 4)),
        ("r07_highdepth", 300, 500, "default", 17, 0.02, (0, 40), (1, 3), (1, 3)),
        ("r08_partial_indel", 900, 200, "indel", 18, 0.60, (0, 60), (1, 8), (1, 8)),
    ]
    sweep = [(0, 1), (0.1, 5), (0.5, 2.5), (0.1, 1), (0, 5), (0.5, 1)]
    with tempfile.TemporaryDirectory() as tmp:
        for name, n, nr, prof, seed, fp, flank, il, dl in specs:
            s = synth.Synth(n=n, n_reads=nr, profile=prof, seed=seed, frac_partial=fp, flank=flank,
                            ins_len=il, del_len=dl, antisense=True)
            p = lambda f: os.path.join(tmp, f)
            s.write_files(p("ref.fa"), p("reads.fa"), p("s.paf"), p("ras.fa"), p("as.paf"))
            rd = open(p("reads.fa"), "rb").read()
            emit_case(script, name + "_sense", open(p("ref.fa"), "rb").read(), rd, open(p("s.paf"), "rb").read(),
                      sweep, f"synth n={n} N={nr} {prof} seed={seed} partial={fp}")
            emit_case(script, name + "_antisense", open(p("ras.fa"), "rb").read(), rd,
                      open(p("as.paf"), "rb").read(), sweep[:3], "same reads vs revcomp reference")


def negative_cases(script):
    """PAF target starts below 0 (minimap2 never writes one; the reference then
    indexes refarr / obsarr with Python's negative wrap, :222, :300-303,
    :57-61, :79, :87, :96).  Pins what the reference does: a match or deletion
    at a negative coordinate >= -(n+1) is a no-op (the wrapped refarr index is
    even, i.e. ''), a '*' writes a one-base LEFT string at the wrapped even
    index, a '+' / flank writes slots into a wrapped ODD position."""
    R = ">ref\nACGTACGTAC\n"
    ok = paf_line("r1", 10, 0, 10, "+", 0, 10, ":10")
    two = ">r1\nACGTACGTAC\n>r2\nACGTACGTAC\n"
    emit_case(script, "n_neg_match", R, two, ok + paf_line("r2", 10, 0, 10, "+", -3, 7, ":10"),
              [(0, 1), (-1, 1)], "negative tstart, matches only: the ones below 0 are no-ops")
    emit_case(script, "n_neg_del", R, ">r1\nACGTACGTAC\n>r2\nACGTACGT\n",
              ok + paf_line("r2", 8, 0, 8, "+", -2, 8, "-ac:8"), [(0, 1), (-1, 1)],
              "negative tstart, a deletion crossing 0")
    emit_case(script, "n_neg_far_del", R, ">r1\nACGTACGTAC\n>r2\nACGTA\n",
              ok + paf_line("r2", 5, 0, 5, "+", -15, 5, "-" + "a" * 15 + ":5"), [(0, 1)],
              "negative tstart below -(n+1), deletion only: no index is taken")
    emit_case(script, "n_neg_far_match", R, two, ok + paf_line("r2", 10, 0, 10, "+", -12, 8, ":20"), [(0, 1)],
              "a match below -(n+1): IndexError")
    emit_case(script, "n_neg_sub", R, two, ok + paf_line("r2", 10, 0, 10, "+", -2, 8, "*ag:9"), [(0, 1), (-1, 1)],
              "'*' at a negative coordinate: a one-base LEFT string at the wrapped even index")
    emit_case(script, "n_neg_ins", R, ">r1\nACGTACGTAC\n>r2\nAAACGTACGTAC\n",
              ok + paf_line("r2", 12, 0, 12, "+", -1, 9, "+aa:10"), [(0, 1), (-1, 1)],
              "'+' at a negative coordinate: slots in a wrapped odd position")
    emit_case(script, "n_neg_flank", R, ">r1\nACGTACGTAC\n>r2\nGGACGTACGT\n",
              ok + paf_line("r2", 10, 2, 10, "+", -2, 6, ":8"), [(0, 1), (-1, 1)],
              "upstream flank at a negative tstart: slots in a wrapped odd position")
    emit_case(script, "n_neg_end", R, ">r1\nACGTACGTAC\n>r2\nACGTT\n",
              ok + paf_line("r2", 5, 0, 3, "+", -8, -5, ":3"), [(0, 1), (-1, 1)],
              "a read ending below 0 with a downstream flank: slots appended to a wrapped odd position")


def long_reference_cases(script):
    """A reference one base past the engine's coordinate limit (include/mpc.h:
    n <= 2^22 - 2 = 4,194,302; the reference takes any length, :161-184), with
    a handful of reads at its start, middle and end.  The reference exits 0;
    the drop-in rejects the plan and exits 1 (tests/golden_util.py DIVERGENT).
    The sequence repeats a 1020-base unit with a few point changes, so the
    gzip'd fixture stays small."""
    import random
    rng = random.Random(22)
    n = (1 << 22) - 1
    unit = "".join(rng.choice("ACGT") for _ in range(1020))  # 17 lines of 60: gzip sees the repeats
    ref = list((unit * (n // 1020 + 1))[:n])
    for k in range(40):
        ref[rng.randrange(n)] = rng.choice("ACGT")
    ref = "".join(ref)
    R = ">big\n" + "\n".join(ref[i:i + 60] for i in range(0, n, 60)) + "\n"
    reads, paf = [], []

    def add(name, ts, cs_ops, up, down):
        # query = upstream + aligned bases (matches copy the reference, '*' y, '+' s) + downstream
        q, i = [up], ts
        for op, v in cs_ops:
            if op == ":":
                q.append(ref[i:i + v]); i += v
            elif op == "*":
                q.append(v[1].upper()); i += 1
            elif op == "+":
                q.append(v.upper())
            elif op == "-":
                i += len(v)
        q.append(down)
        seq = "".join(q)
        cs = "".join(op + (str(v) if op == ":" else v) for op, v in cs_ops)
        reads.append(">%s\n%s\n" % (name, seq))
        paf.append(paf_line(name, len(seq), len(up), len(seq) - len(down), "+", ts, i, cs))

    add("r1", 0, [(":", 120), ("*", "ag"), (":", 40)], "", "TTGCA")
    add("r2", 2_097_000, [(":", 60), ("+", "tta"), (":", 30), ("-", "ac"), (":", 70)], "GGA", "CAT")
    add("r3", 2_097_010, [(":", 200)], "AC", "")
    add("r4", n - 150, [(":", 80), ("*", "ct"), (":", 69)], "ACGTT", "GATTACA")
    add("r5", n - 100, [(":", 100)], "", "CCCC")
    emit_case(script, "l_ref_past_limit", R, "".join(reads), "".join(paf), [(0.1, 5), (0, 1)],
              "reference of 2^22 - 1 bases, one past the engine's coordinate limit")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref-script", default="/root/reference/src/mapped_paf_read_parser.py")
    ap.add_argument("--only", default="", help="'unicode' / 'negative' / 'long': regenerate only the non-ASCII / negative-tstart / "
                                            "past-the-length-limit cases")
    a = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)
    if a.only == "unicode":
        unicode_cases(a.ref_script)
        return
    if a.only == "negative":
        negative_cases(a.ref_script)
        return
    if a.only == "long":
        long_reference_cases(a.ref_script)
        return
    hand_cases(a.ref_script)
    unicode_cases(a.ref_script)
    negative_cases(a.ref_script)
    long_reference_cases(a.ref_script)
    random_cases(a.ref_script)


if __name__ == "__main__":
    main()
