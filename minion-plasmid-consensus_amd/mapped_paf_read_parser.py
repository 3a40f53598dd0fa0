"""Drop-in CLI for src/mapped_paf_read_parser.py (reference v5.1, :108-465).

Same flags, same output files, same exit status; Steps 4-6 run on an MI355X
through libmpc.so.  The Snakemake rule `consensus` (Snakefile:401-423) only has
to point ``params.script`` here.

Extra, optional flags (defaults keep the reference behaviour):
  --device N         HIP device index (default 0)
  --also REF PAF CONSENSUS CHROMAT ACCURACIES
                     run another (assembly, PAF) pair against the same --reads in
                     the SAME launch (e.g. the antisense strand); repeatable
  --revcomp SRC DST  after writing, reverse-complement consensus SRC into DST
                     (Snakefile rule revcomp_antisense_consensus, :425-450);
                     repeatable
  --job REF PAF READS CONSENSUS CHROMAT ACCURACIES
                     another job with its OWN reads file, same launch (a batch of
                     plasmids: BASELINE configs[4]); repeatable.  With --job the
                     primary --ref/--paf/--reads/... flags may be omitted.
"""
import argparse
import importlib
import os
import sys
import time

TITLE = "Mapped PAF Read Parser"


def statprint(msg, msg_type="STATUS"):
    print("{} [{}]: {}".format(msg_type, time.strftime("%Y/%m/%d %T"), msg), flush=True)


def _pkg():
    if __package__:
        return importlib.import_module(__package__)
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    return importlib.import_module(os.path.basename(here))


def build_parser():
    p = argparse.ArgumentParser(description=TITLE)
    p.add_argument("--ref", dest="REF", help="Reference fasta file of plasmid sequence", type=str)
    p.add_argument("--reads", dest="READS", help="Raw reads fasta file", type=str)
    p.add_argument("--paf", dest="PAF", help="Mapped reads .paf file", type=str)
    p.add_argument("--consensus", help="Consensus output file", type=str)
    p.add_argument("--chromat", help="Chromatogram data output file", type=str)
    p.add_argument("--accuracies", help="Per position consensus accuracies output file", type=str)
    p.add_argument("--min_depth_factor", dest="MIN_DEPTH_FACTOR", type=float,
                   help="Minimum number of reads needed to call a base is set to max_depth*MIN_DEPTH_FACTOR")
    p.add_argument("--global_threshold_factor", dest="GLOBAL_THRESHOLD_FACTOR", type=float,
                   help="Value of minimum most frequent to second most frequent base ratio to make call")
    p.add_argument("-d", "--debug", action="store_true", dest="DEBUG", help="Flag for setting debug/test state.")
    p.add_argument("-v", "--verbose", action="store_true", dest="VERB", help="Flag for setting verbose output.")
    p.add_argument("--device", type=int, default=0, help="HIP device index")
    p.add_argument("--also", nargs=5, action="append", default=[],
                   metavar=("REF", "PAF", "CONSENSUS", "CHROMAT", "ACCURACIES"),
                   help="additional (assembly, PAF) job against the same reads, same launch")
    p.add_argument("--revcomp", nargs=2, action="append", default=[], metavar=("SRC", "DST"),
                   help="reverse-complement a written consensus file (rule revcomp_antisense_consensus)")
    p.add_argument("--job", nargs=6, action="append", default=[],
                   metavar=("REF", "PAF", "READS", "CONSENSUS", "CHROMAT", "ACCURACIES"),
                   help="additional job with its own reads file, same launch")
    return p


def _ingest_and_pileup(ingest, engine, jobs, args, tm):
    """Steps 1-6 of every job.  Jobs sharing a reads file are ingested together
    (one scan of it); a group's pileup runs on the device (a worker thread: the
    native ingest and the HIP calls release the GIL) while the next group is
    ingested.  Errors as the jobs would raise them in order: the first job
    (in job order) the ingest rejects, else the first group's device error.
    Returns the per-job call dicts, or None when --min_depth_factor is missing
    (every file is still read first, as the reference does).  ``tm`` receives
    the phase walls: ingest (all groups), device (what the ingest did not
    hide)."""
    import concurrent.futures as cf
    mdf, gtf = args.MIN_DEPTH_FACTOR, args.GLOBAL_THRESHOLD_FACTOR
    triples = [(ref, paf, reads) for ref, paf, reads, *_ in jobs]
    groups = ingest.job_groups(triples)
    packed, futs, t_ing = [None] * len(jobs), [], 0.0
    with cf.ThreadPoolExecutor(max_workers=1) as dev:
        for idx in groups:
            t = time.perf_counter()
            got = ingest.pack_group([triples[j] for j in idx])
            t_ing += time.perf_counter() - t
            for j, x in zip(idx, got):
                packed[j] = x
            ok = not any(isinstance(x, Exception) for x in got)
            if ok:
                for x in got:
                    statprint("There were {} mapped reads.".format(x["n_alignments"]))
            if ok and mdf is not None:
                if not futs:
                    statprint("Pileup and consensus on device {}...".format(args.device))
                futs.append((idx, dev.submit(engine.pileup, got, mdf, 1.0 if gtf is None else gtf, args.device)))
        t1 = time.perf_counter()
        tm["ingest"] = t_ing
        errs = [x for x in packed if isinstance(x, Exception)]
        if errs:
            for _, f in futs:  # let launched pileups finish before reporting
                f.exception()
            raise errs[0]
        if mdf is None:
            return None
        results = [None] * len(jobs)
        # reads of every job, and the job-order prefix: a device error is
        # reported as the read index in the launch of all jobs in JOB order
        n_of = [len(packed[j]["tstart"]) for j in range(len(jobs))]
        before = [sum(n_of[:j]) for j in range(len(jobs))]
        first = None  # (job, read within it, flags) of the earliest failing job
        for idx, f in futs:
            try:
                res = f.result()
            except engine.DataError as e:
                # the group's samples are its jobs in idx order: map the launch's
                # read index back to (job, read in the job)
                r = e.read
                for k, j in enumerate(idx):
                    if r < n_of[j] or k == len(idx) - 1:
                        break
                    r -= n_of[j]
                if first is None or j < first[0]:
                    first = (j, r, e.flags)
                continue
            for j, r in zip(idx, res):
                results[j] = r
        if first is not None:
            j, r, flags = first
            raise engine.DataError(flags, before[j] + r)
    tm["device"] = time.perf_counter() - t1
    return results


def main(argv=None, timings=None):
    """CLI entry.  ``timings`` (a dict, optional) receives the wall seconds of
    the phases: ingest, device (H2D + kernels + D2H), write."""
    t_main = time.perf_counter()
    args = build_parser().parse_args(argv)
    tm = timings if timings is not None else {}
    pkg = _pkg()
    ingest, engine, writers = pkg.ingest, pkg.engine, pkg.writers
    print("=======================================================")
    print("Python version: {}".format(sys.version))
    print("Python environment: {}".format(sys.prefix))
    print("Server: {}".format(os.uname()[1]))
    print("Current directory: {}".format(os.getcwd()))
    print("Command: {}".format(" ".join(sys.argv)))
    print("Time: {}".format(time.strftime("%Y/%m/%d %T")))
    print("Engine: libmpc (HIP, gfx950)")
    print("=======================================================\n")
    # (ref, paf, reads, consensus, chromat, accuracies) per job
    jobs = [] if (args.job and args.REF is None) else \
        [(args.REF, args.PAF, args.READS, args.consensus, args.chromat, args.accuracies)]
    jobs += [(r, p, args.READS, c, ch, a) for r, p, c, ch, a in args.also] + [tuple(j) for j in args.job]
    t0 = time.perf_counter()
    tm["setup"] = t0 - t_main
    try:
        for ref, paf, reads, *_ in jobs:
            statprint(f"Ingesting {paf} against {ref}...")
        results = _ingest_and_pileup(ingest, engine, jobs, args, tm)
        if results is None:  # (:338) max_depth * None, after every file was read
            raise ingest.IngestError("TypeError: --min_depth_factor is required")
        if args.GLOBAL_THRESHOLD_FACTOR is None and any(len(r["count"]) or r["max_depth"] for r in results):
            raise ingest.IngestError("TypeError: --global_threshold_factor is required")  # (:421)
    except (ingest.IngestError, engine.DataError, OSError, UnicodeDecodeError) as e:
        print("Error: {}".format(e), file=sys.stderr)
        return 1
    except engine.MpcError as e:  # input past the engine's limits (e.g. a reference over 2^22 - 2 bases)
        print("Error: {}".format(e), file=sys.stderr)
        return 1
    t2 = time.perf_counter()
    for (ref, paf, _, c, ch, acc), res in zip(jobs, results):
        statprint("Max depth is {}.".format(res["max_depth"]))
        statprint("DEPTH_THRESHOLD is {}.".format(res["max_depth"] * args.MIN_DEPTH_FACTOR))
        statprint("Writing consensus, chromatogram data and per-position consensus accuracies...")
        try:
            writers.write_outputs(res, c, ch, acc)
        except OSError as e:  # WriteError included: the reference's open()/write() raise -> exit 1
            print("Error: {}".format(e), file=sys.stderr)
            return 1
    tm["write"] = time.perf_counter() - t2
    for src, dst in args.revcomp:
        statprint("Reverse-complementing {} into {}...".format(src, dst))
        try:
            writers.revcomp_consensus(src, dst)
        except (writers.RevcompError, OSError, UnicodeDecodeError) as e:
            print("Error: {}".format(e), file=sys.stderr)
            return 1
    statprint("Done.")
    tm["main"] = time.perf_counter() - t_main
    return 0


if __name__ == "__main__":
    sys.exit(main())
