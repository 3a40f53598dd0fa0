/*
 * mpc_ingest.h -- C-ABI of libmpc_ingest.so: the native host I/O of the drop-in
 * CLI -- ingest (Steps 1-3 of /root/reference/src/mapped_paf_read_parser.py)
 * and the Step 7 writers.
 *
 *   reference                                     replaced by
 *   --------------------------------------------  ----------------------------------
 *   Step 1 reference FASTA          :161-184      mpc_ingest(): ref
 *   Step 2 PAF, first alignment per read :192-245 mpc_ingest(): cs, tstart, qs/qe flip
 *   Step 3 reads FASTA, revcomp, flanks :253-277  mpc_ingest(): up, down
 *   Step 7 writers                  :446-463      mpc_write_calls()
 *   src/pseudopair_reads.py         :92-140       mpc_pseudopair()
 *
 * Same results as minion-plasmid-consensus_amd/ingest.py (the Python
 * restatement of those steps): memory-mapped files, multi-threaded line
 * parsing, first-occurrence dedup of PAF records, last-wins for duplicate
 * FASTA names, Python slicing for the flanks.
 *
 * status
 *   MPC_INGEST_OK        outputs valid
 *   MPC_INGEST_ERROR     the reference raises on this input (exit 1); message says why
 *   MPC_INGEST_FALLBACK  an input feature this parser does not restate (non-ASCII bytes,
 *                        '\r' line ends, integers Python accepts that are not plain digits):
 *                        the caller uses the Python ingest, which has the exact semantics
 * Outputs are owned by the library: release them with mpc_ingest_free().
 */
#ifndef MPC_INGEST_H
#define MPC_INGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPC_INGEST_OK 0
#define MPC_INGEST_ERROR 1
#define MPC_INGEST_FALLBACK 2
/* lowest PAF target start passed on to the engine (same value as mpc.h) */
#ifndef MPC_TSTART_MIN
#define MPC_TSTART_MIN (-(1 << 28))
#endif

typedef struct {
  uint8_t* ref;         /* concatenated, rstrip()ed, upper-cased reference (:163-165) */
  int64_t ref_len;
  uint8_t* cs;          /* cs tags after "cs:" (:231-234), retained reads in PAF first-occurrence order */
  int64_t* cs_off;      /* [n_reads + 1] */
  int64_t* tstart;      /* [n_reads] PAF column 8 (:222) */
  uint8_t* up;          /* upstream flanks seq[:qs'] (:264) */
  int64_t* up_off;      /* [n_reads + 1] */
  uint8_t* down;        /* downstream flanks seq[qe':] (:265) */
  int64_t* down_off;    /* [n_reads + 1] */
  int64_t* aligned;     /* [n_reads] qe' - qs' (aligned bases) */
  int64_t n_reads;      /* retained reads (first alignment per name, :237-243) */
  int64_t n_alignments; /* PAF lines (:213) */
  int32_t status;       /* MPC_INGEST_* */
  char message[256];
} mpc_ingest_out;

int mpc_ingest_version(void);

/* Step 7 writers (:446-463), native (csrc/writers.cpp).  calls = ONE sample's
 * calls exactly as the device returns them (MPC_BUF_CALLS rows of include/mpc.h:
 * uint32 x4 = {base | chrom1 << 8 | chrom2 << 16, count, count2, total}).
 * Writes the consensus FASTA, the chromatogram TSV and the accuracies TSV in
 * the reference's formats (accuracy = Python repr of 100 * (count / total) in
 * f64); n_threads <= 0: all hardware threads.  0 on success, -1 with msg set. */
int mpc_write_calls(const uint32_t* calls, int64_t n_calls, const char* consensus_path, const char* chromat_path,
                    const char* accuracies_path, int n_threads, char* msg, int msg_len);
/* Python's repr() of a float into out (NUL-terminated): its length, or -1 if out_len is too small. */
int mpc_py_float_repr(double x, char* out, int out_len);

/* src/pseudopair_reads.py:92-140 (rule pseudopair_reads, Snakefile:211-228), native
 * (csrc/pseudopair.cpp): reads the PAF, writes the "fwd rev" pairs to out_path.
 * has_min = 0: --min_align_length not given (TypeError in the script once reads
 * remain).  Returns stats->status (MPC_INGEST_*; FALLBACK: use the Python
 * restatement, minion-plasmid-consensus_amd/pseudopair_reads.py). */
typedef struct {
  int64_t n_fwd, n_rev;            /* tables after the PAF pass (:117) */
  int64_t n_fwd_kept, n_rev_kept;  /* after the length filter (:135) */
  int64_t n_pairs;
  int32_t status;
  char message[256];
} mpc_pseudopair_stats;
int mpc_pseudopair(const char* paf_path, int64_t min_align_length, int has_min, const char* out_path, int n_threads,
                   mpc_pseudopair_stats* stats);
/* n_threads <= 0: all hardware threads.  Returns out->status. */
int mpc_ingest(const char* ref_path, const char* paf_path, const char* reads_path, int n_threads,
               mpc_ingest_out* out);
/* Several (assembly, PAF) jobs against ONE reads FASTA (sense + antisense of a
 * sample, Snakefile:401-423): the reads file is scanned once for all of them.
 * outs[j] is exactly what mpc_ingest(ref_paths[j], paf_paths[j], reads_path)
 * returns (each has its own status); returns outs[0].status. */
int mpc_ingest_multi(int n_jobs, const char* const* ref_paths, const char* const* paf_paths, const char* reads_path,
                     int n_threads, mpc_ingest_out* outs);
void mpc_ingest_free(mpc_ingest_out* out);

#ifdef __cplusplus
}
#endif
#endif /* MPC_INGEST_H */
