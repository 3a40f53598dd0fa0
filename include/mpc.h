/*
 * mpc.h -- C-ABI of libmpc.so, the MI355X (gfx950) pileup + consensus engine.
 *
 * Drop-in boundary.  The reference has no FFI: its interface is the CLI of
 * src/mapped_paf_read_parser.py (:111-121) and three output files (:446-463).
 * The build keeps that CLI (minion-plasmid-consensus_amd/mapped_paf_read_parser.py)
 * and moves the work of the reference's Step 4-6 onto the GPU behind this ABI:
 *
 *   reference (mapped_paf_read_parser.py)          replaced by
 *   ---------------------------------------------  -----------------------------
 *   Step 4 cs tokenizer + processOperation :285-323, :74-104
 *                                                  mpc_parse()           (K_parse)
 *   processBaseString_leftIndel/rightIndel :37-72  mpc_index() .. mpc_rows()
 *                                                  (even-slot layout, tallies: K_rsplit, K_left,
 *                                                  K_layout, K_ins, K_flank)
 *   Step 5 max depth :332-341                      mpc_consensus()       (K_call)
 *   Step 6 consensus/threshold :348-439            mpc_consensus()       (K_call, K_select)
 *   whole Step 4-6                                 mpc_run()
 *
 * Steps 1-3 (FASTA/PAF ingest, :161-277) and Step 7 (writers) stay on the host.
 *
 * Conventions
 *   - Plain C types only; every buffer is owned by the caller.  The caller
 *     allocates ONE device workspace of mpc_plan_workspace_bytes() bytes and
 *     passes it to mpc_plan_bind(); the library never allocates device memory.
 *   - All device work is enqueued on the caller's stream (hipStream_t passed as
 *     void*); no call synchronizes the device.
 *   - Return value: MPC_OK (0) or a negative MPC_E_* code.  Input DATA errors
 *     (what makes the reference raise and exit 1) are not return codes: they are
 *     reported in the status words (MPC_BUF_STATUS) after the run, see MPC_DE_*.
 *   - Threading: one plan per device / stream; plans share no state.
 */
#ifndef MPC_H
#define MPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPC_ABI_VERSION 9  /* 9: mpc_plan_info.deferred_placement (struct grew) */

/* return codes */
#define MPC_OK 0
#define MPC_E_ARG (-1)       /* bad argument or unsupported size (see mpc_last_error) */
#define MPC_E_HIP (-2)       /* HIP runtime error */
#define MPC_E_WORKSPACE (-3) /* workspace smaller than mpc_plan_workspace_bytes() */
#define MPC_E_STATE (-4)     /* phase called out of order / plan not bound */

/* data-error bits in status[MPC_ST_FLAGS]; any bit => the reference exits 1 */
#define MPC_DE_OP 1u       /* cs does not start with an operator (sys.exit "Unknown operator", :100-102) */
#define MPC_DE_VALUE 2u    /* int() of a ':' operand fails (ValueError, :77) */
#define MPC_DE_INDEX 4u    /* write past the reference end / '*' without operand (IndexError) */
#define MPC_DE_KEY 8u      /* written base not in ACGT (KeyError, :61 / :71) */
#define MPC_DE_CAPACITY 16u /* row capacity too small: re-plan with status[MPC_ST_ROWS_NEEDED] */
#define MPC_DE_INTERNAL 32u /* invariant violated (bug) */
#define MPC_DE_UNSUPPORTED 64u /* input the reference accepts but this engine does not: a ':' / '-' advance
                                  of 2^22 or more from a negative coordinate; tstart < MPC_TSTART_MIN; a
                                  write into a wrapped ODD position (below) in a plan that declared no
                                  negative starts (mpc_input.neg_reads = 0) or with n_shards > 1 */

/* Lowest target start the engine takes.  Negative starts (minimap2 never
 * writes one) follow the reference's Python negative indexing (:222,
 * :300-303): matches and deletions below 0 write nothing, a '*' below 0 writes
 * a one-base LEFT string at gap n + 1 + i, an index below -(2n+1) raises
 * IndexError.  An upstream flank or '+' insertion at a coordinate i in [-n, 0)
 * (:303, :81-87 -> obsarr[2i] = odd position n + i) and the downstream flank of
 * a read ending there (:323) add slots to a reference-base position: its
 * slot list is replayed like a gap's (:37-72) over those strings and the
 * one-base writes of the reads covering it, in read order (single shard;
 * the plan sizes the event list from mpc_input.neg_reads / neg_cs_bytes). */
#ifndef MPC_TSTART_MIN
#define MPC_TSTART_MIN (-(1 << 28))
#endif

/* status words (uint32) at buffer MPC_BUF_STATUS */
#define MPC_ST_FLAGS 0       /* OR of MPC_DE_* */
#define MPC_ST_FIRST_READ 1  /* smallest local read index with a data error (0xFFFFFFFF if none) */
#define MPC_ST_ROWS_NEEDED 2 /* rows (pileup slots incl. empty odd positions) the layout needs */
#define MPC_ST_MIXED 3       /* downstream (RIGHT) events at gaps that also hold LEFT events */
#define MPC_ST_UNITS 4       /* internal: work units of the bucketed event tallies */
#define MPC_ST_RSORT_PATH 5  /* internal: sort of the mixed RIGHT events -- 0 one workgroup (planned), 1 the
                               multi-workgroup path ran, 2 it was planned but fell back to one workgroup */
#define MPC_ST_WRAP_EVENTS 6 /* strings written into wrapped odd positions (negative starts, see above) */
#define MPC_ST_WRAP_POS 7    /* internal: odd positions that received them */
#define MPC_ST_WORDS 8

/* Per-read inputs, already in HBM.  One sample = one (assembly, PAF) pair, e.g.
 * the sense and antisense consensus jobs of Snakefile:401-423 in one launch.
 * Reads are grouped by sample (sample[] nondecreasing) and, within a sample,
 * are in the reference's iteration order: first-occurrence order of the PAF
 * (:237-243, :292). */
typedef struct {
  /* ---- device pointers ---- */
  const uint8_t* ref;      /* concatenated upper-cased references (:163-165) */
  const int64_t* ref_off;  /* [n_samples+1] offsets into ref */
  const uint8_t* cs;       /* cs tag text after "cs:" (e.g. "Z::120*ag:7+tt"), concatenated (:231-234) */
  const int64_t* cs_off;   /* [n_reads+1]; the cs buffer must stay readable up to cs_off[n_reads]+2048 */
  const int32_t* tstart;   /* [n_reads] PAF column 8, target start (:222); >= MPC_TSTART_MIN */
  const uint8_t* up;       /* upstream flanks (read bases before the alignment, :264); up and down
                              must stay readable 16 bytes past their last offset */
  const int64_t* up_off;   /* [n_reads+1] */
  const uint8_t* down;     /* downstream flanks (:265) */
  const int64_t* down_off; /* [n_reads+1] */
  const int32_t* sample;   /* [n_reads] sample id */
  /* ---- host-side sizes ---- */
  int32_t n_samples;
  const int64_t* h_ref_len;    /* host [n_samples] reference lengths n_s (0 <= n_s <= 4194302 = 2^22 - 2: 32-bit
                                  coordinates with the advance clamp, 22-bit gaps in the insertion events; up
                                  to ~312 kb the parse keeps its per-gap state in LDS, beyond it in HBM (tally
                                  mode 4); mpc_plan_create fails with MPC_E_ARG past 2^22 - 2) */
  const int64_t* h_read_begin; /* host [n_samples+1] local reads of sample s: [h_read_begin[s], h_read_begin[s+1]) */
  int64_t n_reads;             /* local reads */
  int64_t cs_bytes;            /* cs_off[n_reads] - cs_off[0] */
  int64_t cs_base;             /* cs_off[0] */
  /* multi-GPU read sharding (single GPU: 0, n_reads, 0, 1).  Shards own
   * CONTIGUOUS global read ranges in shard order (the slot layout at gaps with
   * both LEFT and RIGHT events depends on read order). */
  int64_t read_offset;         /* global index of local read 0 */
  int64_t n_reads_global;
  int32_t shard;               /* this shard's index */
  int32_t n_shards;            /* number of shards (0 is taken as 1) */
  /* optional host copy of cs_off ([n_reads+1], same values as the device one):
   * the planner then splits the parse work (workgroups and the waves inside
   * them) by cs BYTES instead of by read count, so no wave waits for a longer
   * neighbour at the end of the parse.  NULL: split by read count. */
  const int64_t* h_cs_off;
  /* CUs the parse grid is sized for (0: all 256).  With several batches in
   * flight on separate streams, a parse that leaves CUs free lets the other
   * batches' post-parse kernels run beside it (they cannot share a CU with the
   * parse, which holds every VGPR of the CUs it runs on). */
  int32_t parse_cus;
  /* reads with tstart < 0 and their cs bytes (host counts; 0, 0 when there
   * are none).  They bound the strings Python's negative wrap writes into odd
   * positions (upstream / downstream flanks, '+' insertions at i in [-n, 0));
   * a plan sized with 0 reports such a write as MPC_DE_UNSUPPORTED. */
  int64_t neg_reads;
  int64_t neg_cs_bytes;
} mpc_input;

typedef struct mpc_plan mpc_plan;

/* named workspace buffers (byte offset + element count via mpc_plan_buffer) */
enum {
  MPC_BUF_STATUS = 0,   /* uint32[MPC_ST_WORDS] */
  MPC_BUF_CALLS,        /* uint32[rows][4]: {base | chrom1<<8 | chrom2<<16, count, count2, total} */
  MPC_BUF_NCALLS,       /* int32[n_samples+1]: calls of sample s are [ncalls[s], ncalls[s+1]) */
  MPC_BUF_MAXDEPTH,     /* uint32[n_samples] */
  MPC_BUF_ROWS,         /* uint32[rows][4]: per-slot A,T,C,G tallies in output order */
  MPC_BUF_ROWMETA,      /* uint8[rows] bit0 odd position, bit1 first slot of its position */
  MPC_BUF_RIGHT_CNT,    /* int32[gaps] this shard's mixed RIGHT events per gap     (exchange: all-gather) */
  MPC_BUF_RIGHT_CNT_ALL,/* int32[n_shards][gaps] all shards' MPC_BUF_RIGHT_CNT   (exchange: target)     */
  MPC_BUF_HASLEFT,      /* uint32[(gaps+31)/32 + 1] bitmap: gap holds a LEFT event (exchange: OR)         */
  MPC_BUF_MAXR,         /* int32[gaps] longest RIGHT event at RIGHT-only gaps       (exchange: MAX, span)  */
  MPC_BUF_RUN_M,        /* int32[n_reads_global + gaps] longest LEFT event per run  (exchange: MAX, span)  */
  MPC_BUF_RUN_R,        /* int32[n_reads_global + gaps] length of the RIGHT event closing each run (MAX, span) */
  MPC_BUF_DIFF,         /* int32[gaps] this shard's read-span/deletion difference array (not exchanged)    */
  MPC_BUF_SUB,          /* uint32[gaps][4] this shard's substitution tallies        (not exchanged)        */
  MPC_BUF_COUNT
};

int mpc_version(void);
/* Measurement switches this library was compiled with (0 in the product
 * build, tests/test_abi.py): MPC_BF_STAMPS s_memtime stamp build, MPC_BF_TUNING
 * planner overrides from the environment, MPC_BF_VARIANT a kernel variant
 * (a tuning macro set on the compiler command line). */
#define MPC_BF_STAMPS 1
#define MPC_BF_TUNING 2
#define MPC_BF_VARIANT 4
int mpc_build_flags(void);
const char* mpc_last_error(void);

/* Plan for one input shape.  row_cap = capacity of the pileup-row buffers; the
 * exact need is only known on device after the layout phase (status word
 * MPC_ST_ROWS_NEEDED) -- if it is exceeded, MPC_DE_CAPACITY is raised and the
 * caller re-plans with a larger row_cap.  Host-only, no device work. */
int mpc_plan_create(const mpc_input* in, int64_t row_cap, mpc_plan** plan);
int mpc_plan_destroy(mpc_plan* plan);
/* Host copies of the parse work split (tests / tools; no device work):
 * work   n_wg x {sample, first read, end read, chunks} (int32)
 * chunks n_wg x (MPC_PARSE_CHUNKS + 1) read boundaries: the workgroup's reads cut
 *        into contiguous chunks that its waves take in turn.
 * Either pointer may be NULL.  Returns n_wg (>= 0) or a negative MPC_E_*. */
#define MPC_PARSE_CHUNKS 48
int mpc_plan_parse_tables(const mpc_plan* plan, int32_t* work, int32_t* chunks);

int mpc_plan_workspace_bytes(const mpc_plan* plan, size_t* bytes);
int mpc_plan_bind(mpc_plan* plan, void* workspace, size_t bytes);
int mpc_plan_buffer(const mpc_plan* plan, int which, size_t* byte_offset, int64_t* count);
/* Geometry the planner chose (host-only; tests and bench records).  K_parse
 * keeps per-position tallies in LDS as 16-bit counters: tally_mode 1 = 12 B per
 * position, 2 = 10 B (biased depth half), 3 = depth in LDS + global
 * substitution atomics, 0 = global atomics only.  A parse workgroup never
 * holds more than reads_per_workgroup_cap reads (16-bit exactness bound). */
typedef struct {
  int32_t tally_mode;
  int32_t parse_window;            /* cs bytes per wave window */
  int32_t parse_waves;             /* waves per parse workgroup */
  int32_t parse_lds_bytes;
  int32_t parse_workgroups;
  int32_t overrides;               /* MPC_OVR_* bits: a measurement override changed this plan (only in
                                      libraries built with -DMPC_TUNING_OVERRIDES; product builds: 0) */
  int64_t max_reads_per_workgroup;
  int64_t reads_per_workgroup_cap;
  int64_t workspace_bytes;
  int32_t deferred_placement;      /* 1: K_parse queues insertion events per wave in LDS and places them
                                      64 at a time (2 KiB windows, tally mode 1 or 3 with one
                                      substitution window, when the queues fit the LDS budget) */
  int32_t reserved;
} mpc_plan_info;
int mpc_plan_get_info(const mpc_plan* plan, mpc_plan_info* info);
#define MPC_OVR_GEOMETRY 1 /* MPC_PARSE_GEOMETRY="tm,win,nw" picked the parse geometry */
#define MPC_OVR_WGS 2      /* MPC_PARSE_WGS=k set the parse workgroup target */

/* Layout of mpc_input as this library was compiled (bindings check their own
 * struct against it, tests/test_abi.py): returns sizeof(mpc_input) and, when
 * offsets != NULL, writes the byte offset of the first min(cap, field count)
 * fields in declaration order into offsets[].  Field count: MPC_INPUT_FIELDS. */
#define MPC_INPUT_FIELDS 24
size_t mpc_input_layout(size_t* offsets, int cap);
/* update the per-read device pointers (same shape) without re-planning */
int mpc_plan_set_input(mpc_plan* plan, const mpc_input* in);

/* Phases (single GPU: mpc_run() = all of them, in this order).  With
 * n_shards > 1 the host inserts these collectives (Multi-GPU):
 *   mpc_parse    ; OR  HASLEFT
 *   mpc_index    ; ALL-GATHER RIGHT_CNT -> RIGHT_CNT_ALL
 *   mpc_runs     (global run index space, RIGHT length per run)
 *   mpc_tally    ; MAX over the span MAXR .. RUN_R (MAXR, RUN_M, RUN_R lie in this order
 *                  in the workspace, with padding between them: one collective)
 *   mpc_layout   (identical on every shard)
 *   mpc_rows     ; SUM ROWS  (every shard's rows hold its own reads' counts, odd
 *                  positions included: DIFF / SUB are never exchanged)
 *   mpc_consensus (identical on every shard) */
int mpc_parse(mpc_plan* plan, void* stream);        /* clear; cs -> i_end, LEFT gap bits, tallies, insertion events */
int mpc_index(mpc_plan* plan, void* stream);        /* downstream (RIGHT) events at mixed gaps, stable (gap, read) sort; insertion work units */
int mpc_runs(mpc_plan* plan, void* stream);         /* shards > 1: global run index space            */
int mpc_tally(mpc_plan* plan, void* stream);        /* longest LEFT string per run (M)               */
int mpc_layout(mpc_plan* plan, void* stream);       /* per-gap replay of the slot layout, row counts, row offsets, depth, odd rows */
int mpc_rows(mpc_plan* plan, void* stream);         /* insertion and flank tallies onto the slot rows */
int mpc_consensus(mpc_plan* plan, double min_depth_factor, double global_threshold_factor,
                  void* stream);                    /* max depth, calls, compaction            */
int mpc_run(mpc_plan* plan, double min_depth_factor, double global_threshold_factor, void* stream);

/* Measurement hook (bench.py): enqueue ONE launch of a single kernel with the
 * same grid as inside the pipeline, so it can be bracketed by HIP events.
 * The plan must have completed mpc_run() once; the status words are stale
 * until the next mpc_run() (the long-insertion counter keeps growing). */
#define MPC_K_PARSE 0
#define MPC_K_LEFT 2
#define MPC_K_FLANK 3
#define MPC_K_INS 4  /* consumes (and zeroes) the run tallies K_left left: time it after a K_LEFT */
#define MPC_K_RSORT 5 /* re-sorts the mixed RIGHT events of the last K_rsplit (idempotent) */
int mpc_profile_kernel(mpc_plan* plan, int which, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MPC_H */
