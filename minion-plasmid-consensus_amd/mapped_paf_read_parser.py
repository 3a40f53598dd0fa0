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


def main(argv=None, timings=None):
    """CLI entry.  ``timings`` (a dict, optional) receives the wall seconds of
    the phases: ingest, device (H2D + kernels + D2H), write."""
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
    try:
        for ref, paf, reads, *_ in jobs:
            statprint(f"Ingesting {paf} against {ref}...")
        # jobs sharing a reads file are ingested together (one scan of it)
        samples = ingest.pack_samples([(ref, paf, reads) for ref, paf, reads, *_ in jobs])
        for s in samples:
            statprint("There were {} mapped reads.".format(s["n_alignments"]))
        t1 = time.perf_counter()
        tm["ingest"] = t1 - t0
        if args.MIN_DEPTH_FACTOR is None:
            raise ingest.IngestError("TypeError: --min_depth_factor is required")  # max_depth*None (:338)
        gtf = args.GLOBAL_THRESHOLD_FACTOR
        statprint("Pileup and consensus on device {}...".format(args.device))
        results = engine.pileup(samples, args.MIN_DEPTH_FACTOR, 1.0 if gtf is None else gtf, device=args.device)
        tm["device"] = time.perf_counter() - t1
        if gtf is None and any(len(r["count"]) or r["max_depth"] for r in results):
            raise ingest.IngestError("TypeError: --global_threshold_factor is required")  # (:421)
    except (ingest.IngestError, engine.DataError, OSError, UnicodeDecodeError) as e:
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
    return 0


if __name__ == "__main__":
    sys.exit(main())
