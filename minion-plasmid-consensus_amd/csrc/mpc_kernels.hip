// libmpc: MI355X (gfx950) pileup + consensus for the consensus rule of the
// MinION plasmid pipeline.  Hot path = Steps 4-6 of
// /root/reference/src/mapped_paf_read_parser.py (include/mpc.h maps every
// reference function to its replacement; DESIGN.md has layouts and rooflines).
//
// Pipeline (one stream, no host synchronization):
//   parse     K_clear        zero the per-launch state
//             K_parse        per workgroup: contiguous reads of one sample.  cs
//                            ':'+op units -> substitution / deletion / span
//                            tallies (LDS), insertion events (64-event pages
//                            per 64-gap bucket, written once), i_end, LEFT-event
//                            gap bitmap, error flags
//             K_subs/K_subsum tally mode 3: substitution events -> tallies
//   index     K_rsplit_units RIGHT events: mixed gaps -> sort keys, RIGHT-only
//                            gaps -> longest flank; insertion work units
//             K_rsort        stable (gap, read) order of the mixed RIGHT events
//             K_rstart       per-gap ranges in the sorted list, RIGHT run lengths
//   runs      K_runs, K_runR (several shards) global run index space
//   tally     K_left         longest LEFT string per run (insertions, upstream flanks)
//   layout    K_layout       per-gap replay of the slot-layout state of
//                            processBaseString_* (:37-72) -> row counts, then
//                            row offsets + depth (look-back scan), odd rows
//   rows      K_ins, K_flank insertion / flank bases onto their slot rows
//   consensus K_call         per-slot top/second/tie/N (:363-439), max depth
//             K_select       threshold test + ordered compaction of the calls
//                            (look-back scan)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "mpc.h"
#include "mpc_device.h"

// What this library was compiled with (mpc_build_flags): product builds set
// none of the measurement switches below on the command line.  Recorded before
// the #ifndef defaults further down give them their product values.
#if defined(MPC_STAMPS) || defined(MPC_STAMPS_LEFT)
#define MPC_BF_STAMPS_ 1
#else
#define MPC_BF_STAMPS_ 0
#endif
#if defined(MPC_TUNING_OVERRIDES)
#define MPC_BF_TUNING_ 2
#else
#define MPC_BF_TUNING_ 0
#endif
#if defined(MPC_PARSE_DMA) || defined(MPC_FAST_DECODE_MODES) || defined(MPC_LDS_BASE_MODES) || defined(MPC_EPI_U) || \
    defined(MPC_SUBS_SLAB) || defined(MPC_LAYOUT_GAPS) || defined(MPC_LOOKBACK_U) ||     \
    defined(MPC_FLANK_BLOCKS_MAX) || defined(MPC_BPERM_BASE_MODES) || defined(MPC_FLANK_WAVES) || defined(MPC_CS_NT) || defined(MPC_SUB1) || defined(MPC_EARLY_PLACE) || defined(MPC_FLANK_SMALL_BELOW) || \
    defined(MPC_PREFETCH_CS_MODES) || defined(MPC_INT_CHECK_MODES) || defined(MPC_DEFER_PLACE) || defined(MPC_DEFER_SUBEV) || defined(MPC_LEFT_INTERP) || defined(MPC_FLUSH_X2)
#define MPC_BF_VARIANT_ 4
#else
#define MPC_BF_VARIANT_ 0
#endif

using namespace mpc;

namespace {

constexpr uint32_t DE_OP = MPC_DE_OP, DE_VALUE = MPC_DE_VALUE, DE_INDEX = MPC_DE_INDEX,
                   DE_KEY = MPC_DE_KEY, DE_CAP = MPC_DE_CAPACITY, DE_INTERNAL = MPC_DE_INTERNAL,
                   DE_UNSUP = MPC_DE_UNSUPPORTED;

constexpr int kBlk = 1024;          // cs bytes staged per wave iteration (64 lanes x 16 B)
constexpr int kInsInline = 4;       // insertions up to this length travel as one event word
// 32-bit coordinates: a unit's advances are clamped at kAdvCap > n (a clamped
// advance still leaves i past the end).  An advance of 2^22 takes at least 8 cs
// bytes (':' + 7 digits; a '-' advances by its operand bytes), so a window's
// prefix of advances stays below (WIN / 8) * 2^22 <= 2^30 at the largest
// window, and a coordinate (a read base <= kICap plus that prefix plus one
// unit's advance) below 2^31 (static_assert below).  The insertion event word
// holds the gap in 22 bits (kNullGap).
constexpr int kMaxRefLen = (1 << 22) - 2;
constexpr int kAdvCap = 1 << 22;    // > any reference length: a clamped advance keeps i past the end
constexpr int kICap = 1 << 28;      // saturation of the running coordinate i
constexpr int kMaxWin = 2048;       // largest parse window (bytes)
static_assert((int64_t)kICap + (int64_t)(kMaxWin / 8) * kAdvCap + 2 * (int64_t)kAdvCap < (int64_t)INT32_MAX,
              "32-bit coordinates: read base + window prefix of advances + one unit");
static_assert((int64_t)MPC_TSTART_MIN - (int64_t)(kMaxWin / 8) * kAdvCap > (int64_t)INT32_MIN,
              "32-bit coordinates below 0 (negative target starts)");
constexpr int kBW = 64;             // gaps per insertion bucket (K_left workgroup)
static_assert(kBW <= 64 && (kBW & (kBW - 1)) == 0, "sorted insertion events hold the gap within its bucket in 6 bits");
constexpr int kKMax = 8;            // runs per gap tallied in K_left's LDS (others go to HBM)
constexpr uint32_t kNullGap = 0x3fffffu;
// decoupled look-back status words (K_layout, K_select): flag in bits 62-63
// (1 = a block's own sum, 2 = its inclusive prefix), the launch epoch in bits
// 32-61, the 32-bit value below
constexpr uint64_t kSelAgg = 1ull << 62, kSelPre = 2ull << 62, kSelTag = 0x3fffffffull << 32;
// look-back predecessors per lane and step (1: 64 per step)
#ifndef MPC_LOOKBACK_U
#define MPC_LOOKBACK_U 1
#endif

// Decoupled look-back, called by ONE wave of block b: publishes the block's NV
// values (own[k], flag 1), sums its predecessors' values back to the nearest
// inclusive prefix, publishes its own inclusive prefix (flag 2) and returns the
// exclusive prefixes in pre[k].  Block b's NV words are st[NV*b .. NV*b+NV-1]; a
// predecessor counts once all its words carry this launch's tag and the same
// flag.  Each step reads 64 x U predecessors (U per lane).  The launches use
// U = 1 (MPC_LOOKBACK_U, 64 per step): U = 4 (256 per step, 11 instead of 44
// dependent steps over C5's 2.8 k blocks) measured the same within +-4 us
// (profiles/r03_experiments/lookback_variants.txt).  Blocks are dispatched in index order, so the blocks
// waited on are running or done; the spin is bounded anyway (DE_INTERNAL).
template <int NV, int U>
__device__ void lookback(uint64_t* st, int64_t b, uint64_t tag, const int32_t* own, int64_t* pre, uint32_t* flags) {
  const int l = lane();
  if (l == 0)
    for (int k = NV - 1; k >= 0; --k)
      __hip_atomic_store(st + NV * b + k, (b == 0 ? kSelPre : kSelAgg) | tag | (uint32_t)own[k], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  int64_t acc[NV];
  for (int k = 0; k < NV; ++k) acc[k] = 0;
  int spins = 0;
  for (int64_t j0 = b - 1; j0 >= 0;) {
    uint64_t x[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = j0 - 64 * u - l;  // distance 64 u + l; before block 0: prefixes of 0
#pragma unroll
      for (int k = 0; k < NV; ++k)
        x[u][k] = j >= 0 ? __hip_atomic_load(st + NV * j + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (kSelPre | tag);
    }
    // windows u = 0.. in order of distance: every predecessor up to the nearest
    // prefix must be ready
    bool ok = true, found = false;
    uint64_t need[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bool ready = (x[u][0] & kSelTag) == tag && (x[u][0] >> 62) != 0;
#pragma unroll
      for (int k = 1; k < NV; ++k) ready = ready && (x[u][k] & kSelTag) == tag && (x[u][k] >> 62) == (x[u][0] >> 62);
      const uint64_t rdy = ballot(ready), pfx = ballot(ready && (x[u][0] >> 62) == 2);
      need[u] = found ? 0ull : (pfx ? (pfx & (0 - pfx)) * 2 - 1 : ~0ull);
      ok = ok && (rdy & need[u]) == need[u];
      found = found || pfx != 0;
    }
    if (!ok) {
      if (++spins > (1 << 22)) {  // never expected: in-order dispatch
        if (l == 0) atomicOr(flags, (uint32_t)MPC_DE_INTERNAL);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      int32_t v = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) v += ((need[u] >> l) & 1ull) ? (int32_t)(uint32_t)x[u][k] : 0;
      acc[k] += wave_sum(v);
    }
    if (found) break;
    j0 -= 64 * U;
  }
  if (l == 0 && b > 0)
    for (int k = NV - 1; k >= 0; --k)
      __hip_atomic_store(st + NV * b + k, kSelPre | tag | (uint32_t)(int32_t)(acc[k] + own[k]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  for (int k = 0; k < NV; ++k) pre[k] = acc[k];
}

struct Ovf {  // long insertion (len > kInsInline), tallied by K_flank
  int64_t off;  // absolute byte offset of the inserted bases in cs
  int32_t read;
  int32_t gap;  // local gap index (i), sample implied by read
  int32_t len;
  int32_t pad[3];
};

// A string Python's negative index wrap writes into an ODD position: with i in
// [-n, 0), obsarr[2 i] is obsarr[2 (n + i) + 1], the reference base n + i.  An
// upstream flank at tstart = i (:303) or a '+' at i (:81-87) is a LEFT string
// there, the downstream flank of a read ending at i (:323) a RIGHT string.
// K_parse lists them (rare: minimap2 never writes a negative start); the
// position's slot list is then replayed like a gap's (K_woprep, K_wocover,
// K_layout<true>, K_worows).
enum { kWoUp = 0, kWoIns = 1, kWoDown = 2 };  // (order within one read: upstream, cs, downstream)
struct WoEv {
  int32_t g;     // global index of the odd position: gbase[s] + (n + i)
  int32_t read;  // local read
  int32_t len;   // '+': operand bytes (flanks: from the read's offsets)
  int32_t type;  // kWo*
  int64_t src;   // '+': absolute cs offset of the operand
};
struct WoPos {   // one odd position holding such strings
  int32_t g, beg, end;  // its events [beg, end) in the sorted list
  int32_t run0, nrun;   // its runs (LEFT events between consecutive RIGHT ones)
  int32_t lo, F, row0;  // replayed lo, slots, first row (K_layout<true>)
};
struct WoRun {
  int32_t M, R;         // longest LEFT string of the run / RIGHT string closing it
  int32_t hiR, loR;     // replayed hi seen by its LEFT events / lo seen by its RIGHT event
  uint32_t C[4];        // one-base LEFT writes of the reads covering the position (:79, :96)
};
constexpr int64_t kWoCapMax = 1 << 22;  // event list bound (the single-workgroup sort)

// Insertion events (what K_left reads): 4 bytes, bases (8 bits, 2 per base in
// string order) | (len-1) << 8 | gap within its kBW-gap bucket << 10 | read
// relative to the parse workgroup's first read << 16 (< 2^15: wg_reads_cap);
// bit 31 clear.  The bucket and the workgroup are implied by the PAGE the
// event lies in: K_parse places every event once, into 64-event pages of its
// (workgroup, bucket), allocated as they fill (parse_place_event); the
// epilogue lists every bucket's pages, all full but the last (pg_list).
constexpr int kPgEv = 64;                    // events per page (256 B)
constexpr int kPgBits = 12;                  // bucket word: page << 12 | fill
constexpr uint32_t kPgNone = 0xFFFFFu;       // page field of a bucket with no page yet
constexpr uint32_t kPgOvf = kPgNone - 1u;    // ... of a bucket whose workgroup ran out of pages (DE_INTERNAL)
constexpr uint32_t kPgInit = (kPgNone << kPgBits) | (uint32_t)kPgEv;  // first event opens a page
constexpr uint32_t kPgMark = 0xFFFFFFFFu;    // pg_own of a bucket's last page (placed by the epilogue)
static_assert(kPgEv + 1024 < (1 << kPgBits), "fill field: a full page plus every thread of a block waiting");
__device__ __forceinline__ uint32_t ins_word(int gap, int len, uint32_t bases, int rel_read) {
  return bases | ((uint32_t)(len - 1) << 8) | (((uint32_t)gap % (uint32_t)kBW) << 10) | ((uint32_t)rel_read << 16);
}
// page base (in pages) of parse workgroup wg: its events are at most half its
// cs bytes plus 3 per read (an insertion takes >= 2 cs bytes), i.e. at most
// bytes / 128 + 3 reads / 64 full pages, plus one partial page per bucket
__host__ __device__ inline int64_t parse_page_base(int64_t cs_rel, int64_t r, int64_t wg, int nbs) {
  return cs_rel / 128 + (3 * r) / 64 + wg * (int64_t)(nbs + 4);
}

struct Dev {  // device-side views of the plan for the small kernels (passed by value)
  const uint8_t* ref; const int64_t* ref_off;
  const uint8_t* cs; const int64_t* cs_off;
  const int32_t* tstart;
  const uint8_t* up; const int64_t* up_off;
  const uint8_t* down; const int64_t* down_off;
  const int32_t* sample;
  int64_t N, Ng, read_offset, cs_base;
  int32_t S, G;
  const int32_t* n_of; const int32_t* gbase;
  uint32_t* status;
  int32_t* i_end;
  Ovf* ovf; uint32_t* ovf_cnt; int64_t ovf_cap;
  uint32_t* hasleft;                 // bitmap over gaps
  int32_t* maxR;
  uint32_t* keys_in; int32_t* vals_in; uint32_t* keys_out; int32_t* vals_out;
  uint32_t* keys_tmp; int32_t* vals_tmp; int32_t* bcnt; int32_t* bpre;  // K_rsplit -> K_rsort
  int32_t* gcnt; int32_t* kslot;     // multi-workgroup sort: [G+1] mixed events per gap, [N] slot in its gap
  int32_t* rsflag;                   // [4] its path word, scan partials follow (K_rscan)
  int32_t* rlen;                     // [Ng] downstream length by global read
  int32_t* rpos;                     // [N] local read -> position of its mixed RIGHT event in the sorted list
  int32_t* right_start;              // [G+1] mixed RIGHT events (all shards) with gap < g
  int32_t* rsl;                      // [G+1] the same over this shard's sorted list (== right_start on 1 GPU)
  int32_t* roff;                     // [G+1] mixed RIGHT events at gap g on lower shards
  int32_t* rcnt;                     // [G] this shard's mixed RIGHT events per gap (exchange)
  const int32_t* rcnt_all;           // [n_shards][G] all shards' counts (exchange)
  int32_t shard, n_shards;
  int32_t* diff;                     // [G]
  uint32_t* sub;                     // [G][4]
  int32_t* M;                        // [Ng+G] per run: longest LEFT string
  int32_t* runR;                     // [Ng+G] per run: length of the RIGHT string closing it
  int32_t* hiR; int32_t* loR;        // [Ng+G] per run: hi seen by its LEFT events, lo seen by its RIGHT event
  int32_t* lo_f; int32_t* rowcnt; int32_t* row_base;
  int32_t* bsum;                     // [2 * ceil(G / kGB)] x 8 B: K_layout's look-back words (rows, diff)
  uint32_t* rows; uint8_t* meta; int64_t row_cap;
  uint32_t* runt;                    // [Ng+G][4][4] per run: inline insertion bases by slot from the right end
  uint32_t* res; int32_t* keep; int32_t* ksum; uint32_t* calls; int32_t* ncalls; uint32_t* maxdepth;
  int32_t* srow;                     // [S] first row of every sample (K_layout)
  // strings in wrapped odd positions (negative starts; wo_cap 0: none planned)
  WoEv* wo; uint64_t* wo_key; uint32_t* wo_idx; int32_t* wo_erun; WoPos* wo_pos; WoRun* wo_run;
  int64_t wo_cap, wo_p2;             // list capacity, its power-of-two sort size
  double mdf, gtf;
};

// Dict code of a written base after .upper() (:87, :96): A0 T1 C2 G3, -1 if not ACGT.
// (c|0x20) maps exactly {A,a}->a, {C,c}->c, {G,g}->g, {T,t}->t; h=(lc>>1)&3 is a
// perfect hash a0 c1 t2 g3, bit-swapped into dict order.
__device__ __forceinline__ int code_upper(uint32_t c) {
  const uint32_t lc = c | 0x20u;
  const uint32_t h = (lc >> 1) & 3u;
  const uint32_t expect = (0x67746361u >> (8 * h)) & 0xffu;
  const int code = (int)(((h & 1u) << 1) | (h >> 1));
  return lc == expect ? code : -1;
}

// special-character bits of a lane's 16 staged bytes, restricted to [lo, hi)
__device__ __forceinline__ uint32_t special_mask16(uint4 v, int lo, int hi) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t c = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
    const bool sp = (c == 0x3Au) | (c == 0x5Au) | (((c - 0x2Au) <= 3u) & (c != 0x2Cu));  // : Z * + -
    m |= (uint32_t)sp << k;
  }
  hi = hi < 0 ? 0 : (hi > 16 ? 16 : hi);
  lo = lo < 0 ? 0 : (lo > 16 ? 16 : lo);
  return m & ((1u << hi) - 1u) & ~((1u << lo) - 1u);
}

// x * 2561 (= 2^11 + 2^9 + 1) as two full-rate shift-adds; the compiler would
// fold the shifts back into the quarter-rate v_mul_lo_u32
__device__ __forceinline__ uint32_t mul2561(uint32_t x) {
  uint32_t y, z;
  asm("v_lshl_add_u32 %0, %1, 9, %1" : "=v"(y) : "v"(x));
  asm("v_lshl_add_u32 %0, %1, 11, %2" : "=v"(z) : "v"(x), "v"(y));
  return z;
}

__device__ __forceinline__ int64_t readlane64(int64_t x, int j) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)x, j);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), j);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Diagnostic build only (-DMPC_STAMPS, scripts/kparse_stamps.py): s_memtime
// stamps around K_parse's segments, summed per wave in scalar registers and
// stored once per wave into g_stamps (nothing else reads them).  The product
// build compiles none of this.
// -DMPC_STAMPS_LEFT: the same stamps around K_left's segments instead
// (scripts/kleft_stamps.py).
#if defined(MPC_STAMPS) || defined(MPC_STAMPS_LEFT)
constexpr int kStampSeg = 8, kStampWaves = 1 << 16;
__device__ uint64_t g_stamps[kStampWaves * kStampSeg];
#define MPC_STAMP(t)                                                                   \
  do {                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");        \
    __builtin_amdgcn_sched_barrier(0);                                               \
  } while (0)
#define MPC_SEG_ALWAYS(k)           \
  do {                              \
    uint64_t t_;                    \
    MPC_STAMP(t_);                  \
    st_acc[k] += t_ - st_prev;      \
    st_prev = t_;                   \
  } while (0)
#endif
#ifdef MPC_STAMPS
#define MPC_SEG(k) MPC_SEG_ALWAYS(k)
#else
#define MPC_SEG(k) do {} while (0)
#endif
#ifdef MPC_STAMPS_LEFT
#define MPC_LSEG(k) MPC_SEG_ALWAYS(k)
#else
#define MPC_LSEG(k) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// K_parse: Step 4 of the reference (:285-323 tokenizer, :74-104 processOperation)
// ---------------------------------------------------------------------------
constexpr int kSlots = 64;              // reads touching a window (slot 0 = read carried in)
constexpr int kMaxPW = 16;              // waves per workgroup (runtime: blockDim.x / 64)
constexpr uint32_t kFar = 0x7fffu;      // sentinel: the window's only token ends beyond the window
constexpr int kMaxCh = MPC_PARSE_CHUNKS;  // read chunks per parse workgroup, taken dynamically by its waves

// units per window (tok list capacity): a 2 KiB window is cut early when it
// would hold more (LDS budget), smaller windows never hold more than WIN
template <int WIN> constexpr int tok_cap() { return WIN <= 1024 ? WIN : 1024; }

// K_parse may stage a window's cs bytes by LDS-DMA (global_load_lds_dwordx4,
// no VGPRs) into the other of two per-wave stage buffers while the current
// window's rounds run.  Off: measured slower at every config (C1 +15 %, C5
// +14 %, C2-C4 +1 %; profiles/r04_experiments/kparse_variants.txt) -- the
// consumer's vmcnt(0) also waits for every event store the rounds issued.
#ifndef MPC_PARSE_DMA
#define MPC_PARSE_DMA 0
#endif
template <int WIN> constexpr bool parse_dma() { return MPC_PARSE_DMA && WIN >= 1024; }

// K_parse tally modes (bit TM) whose rounds try the fast decode first.  Round
// 4: modes 3-4 only (C4 -4.5 %, C5 -2 %, C3 +0.6 %, C2 (mode 1) +8 %: every
// read starts with the empty tokens "Z" ":", which sent its round to the
// general decode).  Round 5, with those tokens decoded as no-ops on the fast
// path: every mode (C2 parse 137.9 -> 133.7 us, C1 -1 %, modes 3-4 +-0.2 %;
// profiles/r05_experiments/place2_fdall_*.log)
#ifndef MPC_FAST_DECODE_MODES
#define MPC_FAST_DECODE_MODES 0x1f
#endif
template <int TM> constexpr bool fast_decode() { return (MPC_FAST_DECODE_MODES >> TM) & 1; }
// Tally mode 3 with ONE substitution window (references up to 16384 bases:
// C3, C4): the K_parse<3, WIN, NK, true> instantiation takes the round's
// substitution slots from a wave-uniform count -- no loop over windows, no
// count kept in a VGPR lane (C3 -1.3 to -1.9 %, C4 -2.2 %); plans with more
// windows (C5) keep the loop, in a kernel that compiles nothing else
#ifndef MPC_SUB1
#define MPC_SUB1 1
#endif
// ... and the returning add that takes an insertion event's page slot is
// issued before the round's other effects (their issue hides its latency)
#ifndef MPC_EARLY_PLACE
#define MPC_EARLY_PLACE 0
#endif
// ... and tally modes (bit TM) whose next window's cs bytes are loaded before
// this window's rounds (registers live across them) instead of after
#ifndef MPC_PREFETCH_CS_MODES
#define MPC_PREFETCH_CS_MODES 0x00
#endif
template <int TM> constexpr bool prefetch_cs() { return (MPC_PREFETCH_CS_MODES >> TM) & 1; }
// ... and tally modes (bit TM) whose per-unit canonical check is computed as
// VALU integers with one compare (a '*' then needs all its operand bytes to be
// bases, not only the last: the others take the general decode)
#ifndef MPC_INT_CHECK_MODES
#define MPC_INT_CHECK_MODES 0x00
#endif
template <int TM> constexpr bool int_check() { return (MPC_INT_CHECK_MODES >> TM) & 1; }
// ... and insertion events are queued per wave in LDS (kDefQ entries) and
// placed 64 at a time, one per lane, instead of in every round that holds one
// (2 KiB windows, tally modes 1 and 3 with one substitution window, when the
// queues fit the LDS budget)
#ifndef MPC_DEFER_PLACE
#define MPC_DEFER_PLACE 1
#endif
constexpr int kDefQ = 128;  // queue entries per wave (a power of 2, >= 127)
// ... and the epilogue flushes the LDS substitution tallies (tally modes 1, 2)
// with one 64-bit atomic per two codes of a position (off: bit-exact, C1 +6 %,
// C2 +-0; profiles/r06_experiments/kparse_flush_x2.txt)
#ifndef MPC_FLUSH_X2
#define MPC_FLUSH_X2 0
#endif
// ... and (tally mode 3 with one substitution window) the 2-byte substitution
// events too: a ring of kSubQ per wave, written out 128 at a time (two
// consecutive events per lane) instead of one global store per round
// (off: bit-exact, but C3 +7.7 %, C4 +6.5 % -- 120 instead of 89 SGPR spills;
// profiles/r06_experiments/kparse_deferred_subev.txt)
#ifndef MPC_DEFER_SUBEV
#define MPC_DEFER_SUBEV 0
#endif
constexpr int kSubQ = 256;  // substitution-event ring per wave (a power of 2, >= 191)
__host__ __device__ constexpr int defer_bytes(int nw, bool subq) {
  return nw * (kDefQ * 8 + (subq ? kSubQ * 2 : 0));
}
// ... and tally modes whose rounds find a unit's read base by an LDS round trip
// (slot base written by the read's start lane, read back by every lane) instead
// of a scalar pass over the round's read starts: short reads (C1 / C2) start
// several reads per round
#ifndef MPC_LDS_BASE_MODES
#define MPC_LDS_BASE_MODES 0x07
#endif
// ... or by one ds_bpermute from the round's last read-start lane (no LDS slot,
// no fence; takes precedence over the two above)
#ifndef MPC_BPERM_BASE_MODES
#define MPC_BPERM_BASE_MODES 0x00
#endif
template <int TM> constexpr bool bperm_base() { return (MPC_BPERM_BASE_MODES >> TM) & 1; }
template <int TM> constexpr bool lds_base() { return !bperm_base<TM>() && ((MPC_LDS_BASE_MODES >> TM) & 1); }
__host__ __device__ constexpr bool lds_base_rt(int tm) {
  return !((MPC_BPERM_BASE_MODES >> tm) & 1) && ((MPC_LDS_BASE_MODES >> tm) & 1);
}
template <int WIN> constexpr int stage_bufs() { return parse_dma<WIN>() ? 2 : 1; }

template <int WIN, bool SV>              // SV: the read-base slots (lds_base modes)
struct alignas(16) WaveLds {            // per-wave LDS of K_parse
  int32_t s_val[SV ? kSlots : 0];       // read base: i = s_val + window prefix of advances
  int32_t s_ts[kSlots];                 // tstart (clamped to [MPC_TSTART_MIN, kICap])
  int32_t s_read[kSlots];               // local read index
  int32_t s_iend[kSlots];               // i_end | bit 30: read has a downstream flank
  int64_t s_end[kSlots];                // cs offset of the read's end
  uint8_t stage[stage_bufs<WIN>()][WIN + 16];  // window bytes (+16: word reads past the end)
  uint8_t ra[WIN / 8];                  // read-start bits, bit = byte
  uint16_t tok[tok_cap<WIN>() + 2 + 64];  // unit starts in [P, C), then the sentinel C; bits 12-14: ':' prefix
                                        // operand length, bit 15: read start (+64: unconditional loads)
};

struct ParseArgs {  // slim argument block (no SGPR spills)
  const uint8_t* cs; const int64_t* cs_off; const int32_t* tstart;
  const int64_t* up_off; const int64_t* down_off; const int32_t* n_of; const int32_t* gbase;
  const int4* work;  // per workgroup: {sample, first read, end read, chunks}
  const int32_t* wave_tab;  // per workgroup: kMaxCh + 1 read boundaries of its chunks (planner: by cs bytes)
  int64_t cs_base, ovf_cap, read_offset, n_reads;
  int32_t nbs;       // bucket slots per parse workgroup (max buckets)
  int32_t* i_end; uint32_t* ins_sorted; uint32_t* pg_own; uint32_t* pg_list; int32_t* bk_cnt; int32_t* bk_off;
  int64_t* rbase;
  uint32_t* bk_cur;  // tally mode 4 only: per (workgroup, bucket) page words in HBM
  Ovf* ovf; uint32_t* ovf_cnt; uint32_t* hasleft; uint32_t* status;
  int32_t* diff; uint32_t* sub;
  // tally mode 3: substitutions as 2-byte events per (wave, position window),
  // tallied by K_subs (0 windows: global atomics)
  uint16_t* subev; uint32_t* subev_cnt; int64_t subev_cap; int32_t sub_wins;
  WoEv* wo; int64_t wo_cap;  // strings written into wrapped odd positions (negative starts only)
  int32_t defer_off;  // deferred placement (K_parse DP): LDS byte offset of the per-wave event queues
};

// Substitution events (tally mode 3, references too long for LDS substitution
// tallies): position within a kSubWin-position window << 2 | code, per wave and
// window in the wave's region [(cs_off[ra] - cs_base) / kSubEvBytes + 2 ra, ...)
// of window w's slice; K_subs tallies them per window in LDS.  A '*' token takes
// at least 2 cs bytes ('*' and the base it writes, :96 -- minimap2 writes 3,
// "*ag", but "*a" is valid: round 5 sized the regions by 3 bytes, which two-byte
// tokens overran)
constexpr int kSubWinBits = 14, kSubWin = 1 << kSubWinBits, kMaxSubWins = 4;
constexpr int kSubEvBytes = 2;

__host__ __device__ inline int parse_hl_words(int n) { return (n + 1 + 31) / 32; }
// the chunk table (cs offset, read), the chunk counter and the page counter
__host__ __device__ constexpr int parse_misc_bytes() { return (kMaxCh + 2) * 8 + (kMaxCh + 4) * 4 + 16; }
static_assert(parse_misc_bytes() % 16 == 0 && kMaxCh % 4 == 0, "parse LDS misc area alignment");
template <int WIN>
// position tallies of K_parse: 0 = global atomics, 4 = global atomics AND the
// LEFT bitmap / insertion-bucket counters / event-sort cursors in HBM (references
// too long for any LDS mode, up to kMaxRefLen), 1 = LDS, 12 B per position
// (sub 4 x u16, depth decrements | increments u16), 2 = LDS, 10 B per position
// (the depth difference as one biased 16-bit half), 3 = depth differences in
// LDS (2 B per position), substitutions global: references up to ~40 kb
__host__ __device__ inline int parse_lds_bytes(int n_max, int tm, int nbmax, int nw) {
  const int wl = lds_base_rt(tm) ? (int)sizeof(WaveLds<WIN, true>) : (int)sizeof(WaveLds<WIN, false>);
  if (tm == 4) return nw * wl + parse_misc_bytes();  // per-gap state in HBM
  const int tallies = tm == 0 ? 0 : tm == 1 ? 12 * (n_max + 1) : tm == 2 ? 8 * (n_max + 1) + 4 * ((n_max + 2) / 2)
                                                                 : 4 * ((n_max + 2) / 2);
  const int buckets = 16 * nbmax + 4;  // epilogue: counts, cursors, chunk counts, chunk offsets
  return nw * wl + parse_misc_bytes() + 4 * parse_hl_words(n_max) + 4 * nbmax +
         (tallies > buckets ? tallies : buckets);
}

// reads per parse workgroup that keep the 16-bit LDS tallies exact: a read adds
// at most 2 to a position's depth counters; modes 2 / 3 keep the depth
// difference as one half biased by 0x8000 (|sum| <= 2 * 16383 < 0x8000),
// mode 1 keeps decrements and increments apart (2 * 32767 < 2^16)
__host__ __device__ constexpr int64_t wg_reads_cap(int tm) { return tm == 2 || tm == 3 ? 16383 : 32767; }

struct TokInfo { int adv; int kind; uint32_t pay; uint32_t err; };

// Semantics of one token that do not depend on its coordinate, operand read
// from HBM: the slow path for rare tokens (a token longer than the window,
// long insertions / substitution operands, ':' operands that are not 1-4 plain digits).
__device__ __noinline__ TokInfo analyze_long(const uint8_t* cs, int64_t s, int64_t e, bool is_last) {
  TokInfo r{0, 0, 0u, 0u};
  const uint32_t op = cs[s];
  if (!is_special(op)) { r.err = DE_OP; return r; }
  const int64_t olen = e - s - 1;
  if (!(olen > 0 || is_last)) return r;
  if (op == ':') {
    int64_t vv = 0;
    if (!py_int(cs + s + 1, olen, &vv)) r.err |= DE_VALUE;
    else r.adv = vv <= 0 ? 0 : (vv < kAdvCap ? (int)vv : kAdvCap);
    r.kind = r.adv > 0 ? 1 : 0;
  } else if (op == '*') {
    if (olen == 0) { r.err |= DE_INDEX; return r; }
    const int cd = code_upper(cs[e - 1]);
    if (cd < 0) r.err |= DE_KEY;
    r.pay = (uint32_t)(cd & 3); r.adv = 1; r.kind = 2;
  } else if (op == '+') {
    if (olen == 0) return r;
    bool ok = true;
    for (int64_t x = s + 1; x < e; ++x) ok &= code_upper(cs[x]) >= 0;
    if (!ok) r.err |= DE_KEY;
    r.kind = 3;
  } else if (op == '-') {
    r.adv = olen < kAdvCap ? (int)olen : kAdvCap;
    r.kind = olen > 0 ? 4 : 0;
  }
  return r;
}

// first special character in cs[x0, bound) (x0 16-aligned), else bound: all lanes, 1 KiB per step.
// Inlined: a call in the window loop pins the values live across it to the
// callee-saved registers (K_parse<3, 2048> 127 -> 120 VGPRs inlined)
__device__ __forceinline__ int64_t scan_special_wave(const uint8_t* cs, int64_t x0, int64_t bound) {
  for (int64_t x = x0; x < bound; x += 1024) {
    const int64_t y = x + 16 * lane();
    uint32_t m = 0;
    if (y < bound) {
      const uint4 v = *reinterpret_cast<const uint4*>(cs + y);
      const int64_t lim = bound - y;
      m = special_mask16(v, 0, lim > 16 ? 16 : (int)lim);
    }
    const uint64_t b = ballot(m != 0);
    if (b) {
      const int f = __ffsll((unsigned long long)b) - 1;
      const uint32_t mf = (uint32_t)__builtin_amdgcn_readlane((int)m, f);
      return x + 16 * f + __ffs(mf) - 1;
    }
  }
  return bound;
}

__device__ __forceinline__ void push_ovf(const ParseArgs& a, int64_t off, int64_t r, int gap, int len) {
  const uint32_t slot = atomicAdd(a.ovf_cnt, 1u);
  if ((int64_t)slot < a.ovf_cap) {
    Ovf o; o.off = off; o.read = (int32_t)r; o.gap = gap; o.len = len;
    o.pad[0] = o.pad[1] = o.pad[2] = 0;
    a.ovf[slot] = o;
  } else {
    atomicOr(&a.status[MPC_ST_FLAGS], DE_INTERNAL);
  }
}

// a string into a wrapped odd position (WoEv); returns the data error to flag:
// none, or DE_UNSUP when the plan has no room (declared no negative starts,
// several shards)
__device__ __forceinline__ uint32_t push_wo(const ParseArgs& a, int g, int64_t r, int type, int len, int64_t src) {
  if (a.wo_cap <= 0) return DE_UNSUP;
  const uint32_t slot = atomicAdd(&a.status[MPC_ST_WRAP_EVENTS], 1u);
  if ((int64_t)slot >= a.wo_cap) return DE_UNSUP;
  WoEv e;
  e.g = g; e.read = (int32_t)r; e.len = len; e.type = type; e.src = src;
  a.wo[slot] = e;
  return 0u;
}

__device__ __forceinline__ void flag_read(const ParseArgs& a, uint32_t err, int64_t r) {
  atomicOr(&a.status[MPC_ST_FLAGS], err);
  atomicMin(&a.status[MPC_ST_FIRST_READ], (uint32_t)r);
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lanes_below(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Per-byte character classes of a lane's staged bytes, SWAR per 32-bit word
// (no per-byte compares: those pin 2 SGPRs per byte): bit k of sp = byte k is
// special (: Z * + -), of cm = ':'.  The ops that may follow a ':' prefix in
// one unit are sp & ~cm ('Z' included: a unit ':n' + 'Z' decodes as the two
// tokens it is, so only two masks are compacted per word).
__device__ __forceinline__ uint32_t byte_hits(uint32_t w, uint32_t pat) {  // bit 7 of byte k: byte k == pat's
  const uint32_t t = w ^ pat;
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
__device__ __forceinline__ uint32_t hit_nibble(uint32_t z) {  // bits 7, 15, 23, 31 -> bits 0..3
  z >>= 7;
  z |= z >> 7;
  z |= z >> 14;
  return z & 0xfu;
}
// Special bytes by two v_perm table lookups per word: a byte c = (hi, lo) is
// special iff lo >= 8, c < 0x80 and bit hi of T1[lo & 7] is set -- T1[2] (lo
// 0xA) = {2, 3, 5} for '*' ':' 'Z', T1[3] (lo 0xB) = {2} for '+', T1[5] (lo
// 0xD) = {2} for '-' -- i.e. T1[lo & 7] & (1 << hi) != 0, the second lookup
// giving 1 << (hi & 7).  That AND is 8 exactly for ':' (hi 3), so both masks
// come from one pair of lookups.
template <int NW>
__device__ __forceinline__ void word_classes(const uint32_t* w, uint32_t* sp, uint32_t* cm) {
  uint32_t s_ = 0, c_ = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t c = w[i];
    const uint32_t t1 = __builtin_amdgcn_perm(0x00000400u, 0x042C0000u, c & 0x07070707u);
    const uint32_t t2 = __builtin_amdgcn_perm(0x80402010u, 0x08040201u, (c >> 4) & 0x07070707u);
    const uint32_t y = t1 & t2;                   // per byte: 0, or the single bit 1 << hi (<= 0x20)
    const uint32_t ok = (c << 4) & ~c;            // bit 7 of a byte: lo >= 8 and c < 0x80
    const uint32_t zs = (y + 0x7F7F7F7Fu) & ok & 0x80808080u;  // bit 7: y != 0 (no carry out: y <= 0x20)
    const uint32_t zc = (y << 4) & ok & 0x80808080u;           // bit 7: y == 8 (':')
    s_ |= hit_nibble(zs) << (4 * i);
    c_ |= hit_nibble(zc) << (4 * i);
  }
  *sp = s_;
  *cm = c_;
}
struct alignas(16) U8x32 { uint4 a, b; };  // a lane's 32 bytes of a 2 KiB window
__device__ __forceinline__ void chunk_classes(uint2 v, uint32_t* sp, uint32_t* cm) {
  const uint32_t w[2] = {v.x, v.y};
  word_classes<2>(w, sp, cm);
}
__device__ __forceinline__ void chunk_classes(uint4 v, uint32_t* sp, uint32_t* cm) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  word_classes<4>(w, sp, cm);
}
__device__ __forceinline__ void chunk_classes(U8x32 v, uint32_t* sp, uint32_t* cm) {
  const uint32_t w[8] = {v.a.x, v.a.y, v.a.z, v.a.w, v.b.x, v.b.y, v.b.z, v.b.w};
  word_classes<8>(w, sp, cm);
}
// bits [0, x) set, x in [0, 32]
__device__ __forceinline__ uint32_t lowmask(int x) { return x >= 32 ? 0xffffffffu : (1u << x) - 1u; }
// a lane's CH boundary / read-start bits in the per-wave LDS bit arrays
template <int CH>
__device__ __forceinline__ void put_lane_bits(uint8_t* arr, int l, uint32_t v) {
  if (CH == 32) reinterpret_cast<uint32_t*>(arr)[l] = v;
  else if (CH == 16) reinterpret_cast<uint16_t*>(arr)[l] = (uint16_t)v;
  else arr[l] = (uint8_t)v;
}
template <int CH>
__device__ __forceinline__ uint32_t get_lane_bits(const uint8_t* arr, int l) {
  if (CH == 32) return reinterpret_cast<const uint32_t*>(arr)[l];
  if (CH == 16) return reinterpret_cast<const uint16_t*>(arr)[l];
  return arr[l];
}
// lane l gets x of lane l-1 (0 on lane 0) / of lane l+1 (0 on lane 63)
__device__ __forceinline__ uint32_t from_lane_below(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, true);  // wave_shr:1
}
__device__ __forceinline__ uint32_t from_lane_above(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, true);  // wave_shl:1
}


// One window's prefetched inputs: WIN/64 cs bytes per lane and the offsets /
// tstart of reads rs0 + lane.
template <int CH> struct Chunk;
template <> struct Chunk<16> { using T = uint4; };
template <> struct Chunk<8> { using T = uint2; };
template <> struct Chunk<32> { using T = U8x32; };
template <int CH>
struct WinIn {
  typename Chunk<CH>::T d;
  int64_t o;
  uint32_t uo, dno;  // low words of the flank offsets: only the lengths' signs are needed
  int32_t ts;
};
// A lane's cs bytes of a window.  The cs stream is read exactly once:
// MPC_CS_NT loads it non-temporally (evict-first in the caches), so it does not
// push the insertion pages being filled out of L2 before their lines are whole.
#ifndef MPC_CS_NT
#define MPC_CS_NT 1
#endif
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 nt_load16(const uint8_t* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <int CH>
__device__ __forceinline__ typename Chunk<CH>::T cs_load(const uint8_t* p) {
  if constexpr (!MPC_CS_NT) {
    return *reinterpret_cast<const typename Chunk<CH>::T*>(p);
  } else if constexpr (CH == 32) {
    U8x32 v;
    v.a = nt_load16(p);
    v.b = nt_load16(p + 16);
    return v;
  } else if constexpr (CH == 16) {
    return nt_load16(p);
  } else {
    const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(p));
    return make_uint2(v.x, v.y);
  }
}
template <int CH, bool DATA = true>
__device__ __forceinline__ WinIn<CH> fetch_window(const ParseArgs& a, int64_t P, int64_t rs0, int l) {
  WinIn<CH> f;
  const int64_t A = P & ~(int64_t)15;
  if (DATA) f.d = cs_load<CH>(a.cs + A + CH * l);
  const int64_t r = rs0 + l;
  const bool ok = r <= a.n_reads;
  f.o = ok ? a.cs_off[r] : INT64_MAX;
  f.uo = ok ? reinterpret_cast<const uint32_t*>(a.up_off)[2 * r] : 0u;
  f.dno = ok ? reinterpret_cast<const uint32_t*>(a.down_off)[2 * r] : 0u;
  f.ts = r < a.n_reads ? a.tstart[r] : 0;
  return f;
}
// 1 KiB of global memory at src (16 B per lane) into LDS at dst (wave-uniform
// byte address), by LDS-DMA: no VGPR destination; the hardware counts it on
// vmcnt, the compiler does not (the consumer waits vmcnt(0) itself).  M0 is
// written and restored inside the one statement (cdna_hip_programming.md).
__device__ __forceinline__ void dma_1k(const uint8_t* src, uint32_t dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src + 16 * lane()), "s"(dst) : "memory");
}
template <int WIN>
__device__ __forceinline__ void dma_window(const uint8_t* src, uint8_t* stage) {
  const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)stage);
#pragma unroll
  for (int k = 0; k < WIN / 1024; ++k) dma_1k(src + 1024 * k, dst + 1024u * k);
}
__device__ __forceinline__ void chunk_load(const uint8_t* p, uint4& v) { v = *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ void chunk_load(const uint8_t* p, uint2& v) { v = *reinterpret_cast<const uint2*>(p); }
__device__ __forceinline__ void chunk_load(const uint8_t* p, U8x32& v) {
  v.a = reinterpret_cast<const uint4*>(p)[0];
  v.b = reinterpret_cast<const uint4*>(p)[1];
}
__device__ __forceinline__ void chunk_store(uint8_t* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }
__device__ __forceinline__ void chunk_store(uint8_t* p, uint2 v) { *reinterpret_cast<uint2*>(p) = v; }
__device__ __forceinline__ void chunk_store(uint8_t* p, U8x32 v) {
  reinterpret_cast<uint4*>(p)[0] = v.a;
  reinterpret_cast<uint4*>(p)[1] = v.b;
}

// One insertion event into its (workgroup, bucket) page (every lane with an
// event calls it; wave-uniform loop).  The bucket word W = page << 12 | fill:
// a returning add takes slot `fill`; the lane that takes slot 64 of a full page
// opens the next one (page counter npg, owner pg_own) and publishes it with
// fill 1 (its own event in slot 0); lanes that found the page full meanwhile
// (slot > 64, their adds are discarded by the publish) wait for the new page
// and try again.  W lives in LDS (tally modes 0-3) or HBM (mode 4).  Every
// wave reaches the loop's end: an opener never waits.
// EARLY: the returning add was issued by the caller (`old`), ahead of the
// round's other effects, so its LDS latency overlaps them.
template <bool GLOBAL_W, bool EARLY = false>
__device__ __forceinline__ void parse_place_event(const ParseArgs& a, bool has, uint32_t* W, uint32_t* npg,
                                                  int64_t pbase, uint32_t* pg0, uint32_t pcap, int b, uint32_t word,
                                                  uint32_t old = 0u) {
  // common case straight-line: the add gives a slot of the current page
  // (pg0 = the workgroup's first page: 32-bit offsets from a scalar base)
  if constexpr (!EARLY) old = has ? atomicAdd(W, 1u) : 0u;
  const bool fast = has && (old & ((1u << kPgBits) - 1u)) < (uint32_t)kPgEv;
  if (fast) pg0[(old >> kPgBits) * kPgEv + (old & ((1u << kPgBits) - 1u))] = word;
  bool need = has && !fast;
  if (!ballot(need)) return;
  // the page is full: open the next one, or wait for its opener.  A waiting
  // lane looks at W once per pass of the wave-uniform loop, so an opener lane
  // of the SAME wave (whose branch the compiler may place after the waiting
  // lanes' code in one pass) has published before the next look
  bool waiting = false, first = true;
  uint32_t wpg = 0;
  int spins = 0;
  while (ballot(need)) {
    if (need && waiting) {
      const uint32_t cur = GLOBAL_W ? __hip_atomic_load(W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : __hip_atomic_load(W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      waiting = (cur >> kPgBits) == wpg;
      if (waiting && ++spins > (1 << 22)) {  // bounded: never expected
        atomicOr(&a.status[MPC_ST_FLAGS], DE_INTERNAL);
        need = false;
      }
    }
    if (need && !waiting) {
      if (!first) old = atomicAdd(W, 1u);
      first = false;
      const uint32_t slot = old & ((1u << kPgBits) - 1u), pg = old >> kPgBits;
      if (pg == kPgOvf && slot > (uint32_t)kPgEv) {
        // the region ran out of pages (flagged by the opener): the event is
        // dropped, and the word reset so its fill never carries into the page field
        atomicExch(W, (kPgOvf << kPgBits) | (uint32_t)kPgEv);
        need = false;
      } else if (slot < (uint32_t)kPgEv) {
        pg0[pg * kPgEv + slot] = word;
        need = false;
      } else if (slot == (uint32_t)kPgEv) {
        const uint32_t np = atomicAdd(npg, 1u);
        if (np >= pcap) {  // never expected: the page region bound (parse_page_base)
          // publish the overflow page, so waiting lanes leave (dropping their events)
          atomicOr(&a.status[MPC_ST_FLAGS], DE_INTERNAL);
          atomicExch(W, (kPgOvf << kPgBits) | (uint32_t)kPgEv);
        } else {
          a.pg_own[pbase + np] = (uint32_t)b;
          pg0[np * kPgEv] = word;
          atomicExch(W, (np << kPgBits) | 1u);
        }
        need = false;
      } else {
        waiting = true;  // the page filled meanwhile: wait for its opener
        wpg = pg;
      }
    }
  }
}

// End of a parse workgroup: flush the LDS position tallies and the LEFT-gap
// bitmap with contiguous atomics (tally modes 1-3), then list every bucket's
// pages: bk_cnt = its events, bk_off = where its page list starts in
// pg_list[pbase ...] -- the pages (global page numbers) in any order but the bucket's current
// (possibly partial) page LAST, so event e of the bucket is in page
// pg_list[pbase + bk_off + e / 64] at slot e % 64.  W (page words), cnt and cur
// are LDS for modes 0-3 (cnt, cur alias the flushed tallies) and HBM for mode 4
// (W = bk_cur, cnt = bk_cnt zeroed by K_clear, cur = bk_cur once read).  Every
// thread of the block calls it.
template <int TM>
__device__ void parse_epilogue(const ParseArgs& a, int n, int gb, int nbk, uint32_t* hl, uint32_t* W, uint32_t* uni,
                               const uint32_t* npg, int64_t pbase, uint32_t pcap) {
  constexpr bool big = TM == 4;
  constexpr bool fused = TM >= 1 && TM <= 3;
  constexpr bool lds_sub = TM == 1 || TM == 2;
  constexpr bool packed = TM == 2 || TM == 3;
  const int l = lane();
  const int nsub = lds_sub ? 2 * (n + 1) : 0;
  const uint32_t* sub_l = uni;
  const uint32_t* del_l = uni + nsub;
  // ---- flush LDS tallies and the LEFT-gap bitmap ----
  if (fused) {
    // one word per lane, consecutive lanes on consecutive words: a wave's
    // atomics cover contiguous bytes (memory-side atomics run at full rate
    // only on contiguous segments)
    for (int p = threadIdx.x; p <= n; p += blockDim.x) {
      int32_t dv;
      if (packed) dv = (int32_t)((del_l[p >> 1] >> (16 * (p & 1))) & 0xffffu) - 0x8000;
      else { const uint32_t dl = del_l[p]; dv = (int32_t)(dl >> 16) - (int32_t)(dl & 0xffffu); }
      if (dv) atomicAdd(a.diff + gb + p, dv);
    }
    uint32_t* sg = a.sub + (int64_t)gb * 4;
    if (MPC_FLUSH_X2) {
      // two codes per 64-bit add (LDS word k = position k/2, codes 2 (k&1) + {0, 1}
      // = global words 2k, 2k + 1): a position's count of one code never
      // reaches 2^32, so the low half never carries into the high one
      for (int k = threadIdx.x; lds_sub && k < 2 * (n + 1); k += blockDim.x) {
        const uint32_t w2 = sub_l[k];
        if (w2) atomicAdd(reinterpret_cast<unsigned long long*>(sg) + k,
                          (unsigned long long)(w2 & 0xffffu) | ((unsigned long long)(w2 >> 16) << 32));
      }
    } else {
      for (int k = threadIdx.x; lds_sub && k < 4 * (n + 1); k += blockDim.x) {  // word k = position k/4, code k%4
        const uint32_t w2 = sub_l[2 * (k >> 2) + ((k >> 1) & 1)];
        const uint32_t v = (k & 1) ? (w2 >> 16) : (w2 & 0xffffu);
        if (v) atomicAdd(sg + k, v);
      }
    }
  }
  for (int k = threadIdx.x; !big && k < parse_hl_words(n); k += blockDim.x) {
    const uint32_t v = hl[k];
    if (!v) continue;
    const int g0 = gb + 32 * k;  // global bit of local bit 0 of this word
    atomicOr(a.hasleft + (g0 >> 5), v << (g0 & 31));
    if (g0 & 31) atomicOr(a.hasleft + (g0 >> 5) + 1, v >> (32 - (g0 & 31)));
  }
  const int64_t wgb = (int64_t)blockIdx.x * a.nbs;
  uint32_t* cnt = big ? reinterpret_cast<uint32_t*>(a.bk_cnt) + wgb : uni;       // non-last pages per bucket
  uint32_t* cur = big ? a.bk_cur + wgb : uni + nbk;                               // list cursors
  auto wload = [&](int b) -> uint32_t {
    return big ? __hip_atomic_load(W + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : W[b];
  };
  __syncthreads();  // (LDS tallies flushed: cnt / cur may alias them)
  const uint32_t np_all = min(*npg, pcap);  // (the counter runs past pcap only after DE_INTERNAL)
  // A: mark every bucket's last page (it goes to the end of the bucket's list)
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) {
    const uint32_t w = wload(b);
    if ((w >> kPgBits) < pcap) a.pg_own[pbase + (w >> kPgBits)] = kPgMark;
    if (!big) cnt[b] = 0;
  }
  __syncthreads();
  // B: the other pages per bucket
  for (uint32_t p = threadIdx.x; p < np_all; p += blockDim.x) {
    const uint32_t b = a.pg_own[pbase + p];
    if (b != kPgMark) atomicAdd(cnt + b, 1u);
  }
  __syncthreads();
  // C: one wave -- list offsets (exclusive scan of the page counts), event
  // counts, the last page at the end of each list, the list cursors
  if (threadIdx.x < 64) {
    int carry = 0;
    for (int c0 = 0; c0 < nbk; c0 += 64) {
      const int b = c0 + l;
      uint32_t w = kPgInit, c = 0;
      if (b < nbk) {
        w = wload(b);
        c = big ? (uint32_t)__hip_atomic_load(cnt + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : cnt[b];
      }
      const bool has = (w >> kPgBits) < pcap;  // (not kPgNone, not kPgOvf)
      const int np = (int)c + (has ? 1 : 0);
      const int inc = wave_scan_i32(np);
      const int off = carry + inc - np;
      if (b < nbk) {
        a.bk_cnt[wgb + b] = has ? (int32_t)(c * kPgEv + (w & ((1u << kPgBits) - 1u))) : 0;
        a.bk_off[wgb + b] = off;
        if (has) a.pg_list[pbase + off + np - 1] = (uint32_t)(pbase + (w >> kPgBits));
        if (big) __hip_atomic_store(cur + b, (uint32_t)off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else cur[b] = (uint32_t)off;
      }
      carry += wave_last_i32(inc);
    }
  }
  if (threadIdx.x == 0) a.rbase[blockIdx.x] = pbase;
  __syncthreads();
  // D: place the other pages
  for (uint32_t p = threadIdx.x; p < np_all; p += blockDim.x) {
    const uint32_t b = a.pg_own[pbase + p];
    if (b != kPgMark) a.pg_list[pbase + atomicAdd(cur + b, 1u)] = (uint32_t)(pbase + p);
  }
}

// Workgroup = contiguous reads of ONE sample (host work table); wave w takes
// the w-th part of them and streams their cs bytes in windows of WIN bytes
// (WIN/64 per lane, coalesced).  Token boundaries (special characters and read starts) are bits
// of an LDS mask.  A window is cut at its LAST boundary C, so every token in
// [P, C) ends inside the window (no lookahead halo); the next window starts at
// C.  The token starts are compacted into a list of UNITS -- a ':' token
// with 1-4 digits and the op token right after it in the same read form one
// unit (minimap2's short cs alternates them, so this halves the list) -- and
// processed ONE UNIT PER LANE, 64 per round: branch-free SWAR decode of the
// operand words, one DPP scan of the advances for the coordinates i (reads
// are segments: per-read bases in a slot table), ballot/mbcnt for the read
// slot.  Effects: substitution / deletion / span tallies (LDS in tally modes
// 1-3), insertion events placed once into 64-event pages of their (workgroup,
// bucket) (parse_place_event), LEFT-gap bits (LDS bitmap).  Epilogue: flush
// the tallies, list every bucket's pages (parse_epilogue).
// NK: the plan holds reads with a negative tstart (mpc_input.neg_reads): the
// kernel carries the rounds of Python's negative index wrap (NEG below),
// taken by the workgroups that hold such a read; without NK nothing of it is
// compiled in (its registers would bound every plan's kernel), and a negative
// tstart is MPC_DE_UNSUPPORTED (parsed from 0, never an out-of-range write).
// S1: tally mode 3 with one substitution window (MPC_SUB1 above).
template <int TM, int WIN, bool NK, bool S1 = false, bool DP = false>
__global__ __launch_bounds__(kMaxPW * 64) void K_parse(ParseArgs a) {
  static_assert(!S1 || TM == 3, "one substitution window: tally mode 3 only");
  static_assert(!DP || TM != 4, "deferred placement: bucket words in LDS");
  constexpr int CH = WIN / 64;
  static_assert(WIN <= kMaxWin, "coordinate bound (kMaxWin)");
  using WL = WaveLds<WIN, lds_base<TM>()>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int l = lane();
  const int nw = (int)(blockDim.x >> 6);
  const int w = uniform_i32((int)(threadIdx.x >> 6));
  WL& W = *reinterpret_cast<WL*>(lds + w * (int)sizeof(WL));
  int64_t* cbo = reinterpret_cast<int64_t*>(lds + nw * (int)sizeof(WL));        // [kMaxCh + 1] chunk bounds: cs offset
  int32_t* cbr = reinterpret_cast<int32_t*>(cbo + kMaxCh + 2);                  // [kMaxCh + 1] ... and read
  uint32_t* cnext = reinterpret_cast<uint32_t*>(cbr + kMaxCh + 4);              // next chunk to take
  uint32_t* hl = cnext + 4;                                                      // LEFT gaps bitmap
  const int4 wk = a.work[blockIdx.x];
#ifdef MPC_STAMPS
  uint64_t st_acc[kStampSeg] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev;
  MPC_STAMP(st_prev);
#endif
  const int smp = wk.x;
  const int64_t r0 = wk.y, r1 = wk.z;
  const int n = a.n_of[smp];
  const int gb = a.gbase[smp];
  const int nbk = (n + 1 + kBW - 1) / kBW;  // insertion buckets
  constexpr bool big = TM == 4;             // per-gap state (LEFT bitmap, bucket page words) in HBM
  // [nbk] page word of every insertion bucket (page << 12 | fill, parse_place_event)
  uint32_t* bkw = big ? a.bk_cur + (int64_t)blockIdx.x * a.nbs : hl + parse_hl_words(n);
  uint32_t* uni = hl + parse_hl_words(n) + nbk;
  uint32_t* npg = cnext + 1;                // pages opened by the workgroup
  // the workgroup's page region [pbase, pnext) (parse_page_base)
  const int64_t pbase = parse_page_base(a.cs_off[r0] - a.cs_base, r0, blockIdx.x, a.nbs);
  const int64_t pnext = parse_page_base(a.cs_off[r1] - a.cs_base, r1, blockIdx.x + 1, a.nbs);
  const uint32_t pcap = (uint32_t)min(pnext - pbase, (int64_t)kPgOvf);
  uint32_t* const pg0 = a.ins_sorted + pbase * kPgEv;  // the region's first event slot
  constexpr bool fused = TM >= 1 && TM <= 3;  // depth differences in LDS (one address space per instantiation)
  constexpr bool lds_sub = TM == 1 || TM == 2;  // substitution tallies in LDS too
  constexpr bool packed = TM == 2 || TM == 3;
  const int nsub = lds_sub ? 2 * (n + 1) : 0;
  uint32_t* sub_l = uni;                    // [2 (n+1)] (TM 1, 2): A | T << 16, C | G << 16
  // TM 1:    [n+1] depth-decrement count | depth-increment count << 16
  // TM 2, 3: [(n+2)/2] depth difference of position p in half p&1 of word p>>1,
  //          biased by 0x8000: at most 16383 reads per workgroup and 2 per read and
  //          position keep every partial sum inside (0, 0xffff): no carry across halves
  uint32_t* del_l = uni + nsub;
  for (int k = threadIdx.x; !big && k < parse_hl_words(n); k += blockDim.x) hl[k] = 0;
  for (int k = threadIdx.x; !big && k < nbk; k += blockDim.x) bkw[k] = kPgInit;  // (mode 4: K_clear)
  if (threadIdx.x == 0) { *cnext = (uint32_t)nw; *npg = 0u; cnext[2] = 0u; }  // chunks 0..nw-1 go to waves 0..nw-1
  const int nch = wk.w;
  for (int k = threadIdx.x; k <= nch; k += blockDim.x) {
    const int32_t r = a.wave_tab[(int64_t)blockIdx.x * (kMaxCh + 1) + k];
    cbr[k] = r;
    cbo[k] = a.cs_off[r];
  }
  if (fused)
    for (int k = threadIdx.x; k < nsub + (packed ? (n + 2) / 2 : n + 1); k += blockDim.x)
      uni[k] = (packed && k >= nsub) ? 0x80008000u : 0u;
  // a read with a negative tstart in the workgroup: its chunks take the rounds
  // that follow Python's negative index wrap (NEG below; the others compile
  // none of it)
  // (an OR through cnext[2], not __syncthreads_or: that one takes static LDS
  // the planner's budget does not hold)
  bool wg_neg = false;
  if constexpr (NK) {
    bool has_neg = false;
    for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) has_neg |= a.tstart[r] < 0;
    __syncthreads();
    if (ballot(has_neg) && lane() == 0) atomicOr(cnext + 2, 1u);
    __syncthreads();
    wg_neg = uniform_i32((int)cnext[2]) != 0;
  } else {
    __syncthreads();  // the chunk table, counters and cleared tallies above are in place
  }

  auto odd_sub = [&](int pos, int code) {
    if (lds_sub) atomicAdd(sub_l + 2 * pos + (code >> 1), 1u << (16 * (code & 1)));
    else atomicAdd(a.sub + (int64_t)(gb + pos) * 4 + code, 1u);
  };
  auto depth_dec = [&](int pos) {  // diff[pos] -= 1
    if (packed) atomicSub(del_l + (pos >> 1), 1u << (16 * (pos & 1)));
    else if (fused) atomicAdd(del_l + pos, 1u);
    else atomicAdd(a.diff + gb + pos, -1);
  };
  auto depth_inc = [&](int pos) {  // diff[pos] += 1
    if (packed) atomicAdd(del_l + (pos >> 1), 1u << (16 * (pos & 1)));
    else if (fused) atomicAdd(del_l + pos, 1u << 16);
    else atomicAdd(a.diff + gb + pos, 1);
  };

  auto left_bit = [&](int pos) {  // gap pos holds a LEFT event
    if (big) atomicOr(a.hasleft + ((gb + pos) >> 5), 1u << ((gb + pos) & 31));
    else atomicOr(hl + (pos >> 5), 1u << (pos & 31));
  };
  // The workgroup's reads come in chunks (planner: contiguous, by cs bytes,
  // 5/8 of the bytes in the first nw chunks, smaller ones after); wave w
  // starts on chunk w and takes the next free one when it is done, so all
  // waves reach the epilogue barrier within about one small chunk of each
  // other (a static share per wave left them waiting there ~20 % of their
  // time: profiles/r03_stamps).  The chunk table sits in LDS (one load per
  // chunk bound per workgroup).  A chunk is a stream of its own: event
  // regions, i_end.
  // take the next chunk: every lane adds (lane 0 one, the others zero), so no
  // divergent region guards the atomic (a lane-0-only atomic in the loop head
  // was compiled into a loop exit that only lane 0 took: the wave never left)
  auto take_chunk = [&]() {
    const uint32_t v = atomicAdd(cnext, l == 0 ? 1u : 0u);
    return uniform_i32(__builtin_amdgcn_readlane((int)v, 0));
  };
  // deferred placement: the wave's queue of (bucket, event word) in LDS, a ring
  // of kDefQ entries between dq_tail and dq_head (wave-uniform counters); a
  // round appends its events, and 64 at a time are placed after it (<= 63 wait
  // before a round, <= 127 after one)
  uint2* const dq = DP ? reinterpret_cast<uint2*>(lds + a.defer_off) + w * kDefQ : nullptr;
  uint32_t dq_head = 0, dq_tail = 0;
  // ... and the chunk's substitution events (S1): ring index = event index in
  // the chunk's region; sq_tail of them are in HBM (nsub_s = the head)
  constexpr bool DQS = DP && S1 && MPC_DEFER_SUBEV;
  uint16_t* const sq = DQS ? reinterpret_cast<uint16_t*>(lds + a.defer_off + nw * kDefQ * 8) + w * kSubQ : nullptr;
  auto defer_flush = [&](const int cnt) {  // the cnt (<= 64) oldest events, one per lane
    wave_sync_lds();
    const bool has = l < cnt;
    const uint2 e = has ? dq[(dq_tail + l) & (kDefQ - 1)] : make_uint2(0u, 0u);
    parse_place_event<big>(a, has, bkw + e.x, npg, pbase, pg0, pcap, (int)e.x, e.y);
    dq_tail += (uint32_t)cnt;
  };
  auto chunks = [&](auto negc) {
  constexpr bool NEG = decltype(negc)::value;
  for (int chk = w < nch ? w : nch; chk < nch; chk = take_chunk()) {
  const int64_t ra = uniform_i32(cbr[chk]), rb = uniform_i32(cbr[chk + 1]);
  const int64_t wend = readlane64(cbo[chk + 1], 0);
  int64_t P = readlane64(cbo[chk], 0);
  const int64_t sev_base = (P - a.cs_base) / kSubEvBytes + 2 * ra;  // ... and its substitution-event regions (TM 3)
  uint32_t nsub_v = 0;                                    // lane k: substitution events of window k
  uint32_t nsub_s = 0;                                    // ... of the only window (S1, wave-uniform)
  uint32_t sq_tail = 0;                                   // (DQS) ... written to the region
  auto sub_flush = [&](const uint32_t cnt) {  // the cnt (<= 128) oldest queued events, two per lane
    wave_sync_lds();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t k = sq_tail + 2u * (uint32_t)l + (uint32_t)h;
      if (k < sq_tail + cnt) a.subev[sev_base + k] = sq[k & (kSubQ - 1)];
    }
    sq_tail += cnt;
  };  int64_t rs0 = ra;         // first read whose cs starts at or after P
  bool carry = false;       // slot 0 holds a read continuing into this window
  int32_t c_base = 0;       // ... and its coordinate base (wave-uniform): i = base + window prefix of advances
  constexpr bool dma = parse_dma<WIN>();
  int sb = 0;               // stage buffer of the current window
  if (dma && P < wend) dma_window<WIN>(a.cs + (P & ~(int64_t)15), W.stage[0]);
  WinIn<CH> cur = fetch_window<CH, !dma>(a, P, rs0, l);
  while (P < wend) {
    const int64_t A = P & ~(int64_t)15;
    // ---- window: at most 63 read starts in [P, E) ----
    int64_t E = A + WIN < wend ? A + WIN : wend;
    const int64_t o63 = readlane64(cur.o, 63);
    if (o63 < E) E = o63;
    MPC_SEG(0);
    // the next read's offsets (lane l + 1, by DPP; lane 63 is never a read of the window)
    const int64_t o_nx = (int64_t)(((uint64_t)from_lane_above((uint32_t)((uint64_t)cur.o >> 32)) << 32) |
                                   from_lane_above((uint32_t)cur.o));
    const uint32_t uo_nx = from_lane_above(cur.uo);
    const uint32_t dno_nx = from_lane_above(cur.dno);
    if (E <= P) {
      // reads rs0 .. rs0+62 all start at P: 63 empty cs (processOperation('', ''))
      if (l < 63) {
        flag_read(a, DE_OP, rs0 + l);
        a.i_end[rs0 + l] = cur.ts < 0 ? 0 : (cur.ts > n ? n + 1 : cur.ts);
      }
      rs0 += 63;
      cur = fetch_window<CH, !dma>(a, P, rs0, l);  // (same P: the staged bytes stay)
      continue;
    }
    // ---- stage bytes, boundary bits ----
    if (dma) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this window's LDS-DMA has landed
      chunk_load(W.stage[sb] + CH * l, cur.d);
    } else {
      chunk_store(W.stage[0] + CH * l, cur.d);
    }
    uint32_t spm, cm_own;
    chunk_classes(cur.d, &spm, &cm_own);
    const uint32_t om_own = spm & ~cm_own;
    put_lane_bits<CH>(W.ra, l, 0u);
    wave_sync_lds();
    {  // read-start bits of every read starting inside the window (incl. E)
      const int64_t rel = cur.o - A;
      if (rel >= 0 && rel < WIN) atomicOr(reinterpret_cast<uint32_t*>(W.ra) + (rel >> 5), 1u << (rel & 31));
    }
    wave_sync_lds();
    const int64_t cA = A + CH * l;
    const uint32_t ra_own = get_lane_bits<CH>(W.ra, l);
    const uint32_t em_own = spm | ra_own;  // boundaries: special characters and read starts
    // ---- cut C: E if E is a boundary (a read start), else the last boundary in (P, E) ----
    const bool e_rs = (E == wend) || (E == o63);
    int64_t C;
    bool c_rs;
    bool far = false;
    if (e_rs) { C = E; c_rs = true; }
    else {
      int lo = (int)(P + 1 - cA), hi = (int)(E - cA);
      lo = lo < 0 ? 0 : (lo > CH ? CH : lo);
      hi = hi < 0 ? 0 : (hi > CH ? CH : hi);
      const uint32_t m = em_own & lowmask(hi) & ~lowmask(lo);
      const uint64_t b = ballot(m != 0);
      if (b) {
        const int f = 63 - __clzll((long long)b);
        const uint32_t mf = (uint32_t)__builtin_amdgcn_readlane((int)m, f);
        const uint32_t rf = (uint32_t)__builtin_amdgcn_readlane((int)ra_own, f);
        const int k = 31 - __clz(mf);
        C = A + CH * f + k;
        c_rs = (rf >> k) & 1u;
      } else {
        // one token runs past the window: its end is the next special character
        // or the next read start (the first read start after P)
        const uint64_t bn = ballot(cur.o > P);
        const int fo = bn ? __ffsll((unsigned long long)bn) - 1 : 63;
        const int64_t bound = readlane64(cur.o, fo) < wend ? readlane64(cur.o, fo) : wend;
        C = scan_special_wave(a.cs, A + WIN, bound);
        c_rs = C == bound;
        far = true;
      }
    }
    if (WIN > tok_cap<WIN>() && !far) {
      // more than tok_cap tokens in [P, C): cut at the tok_cap-th boundary after P
      int lo = (int)(P - cA), hi = (int)(C - cA);
      lo = lo < 0 ? 0 : (lo > CH ? CH : lo);
      hi = hi < 0 ? 0 : (hi > CH ? CH : hi);
      const uint32_t m = em_own & lowmask(hi) & ~lowmask(lo);
      const int cb = __popc(m);
      // at most tok_cap / 64 boundaries in every lane: no cut (the usual case, no scan)
      const bool may = ballot(cb > tok_cap<WIN>() / 64) != 0;
      const int inc = may ? wave_scan_i32(cb) : 0;
      if (may && wave_last_i32(inc) > tok_cap<WIN>()) {
        const int f = __ffsll((unsigned long long)ballot(inc > tok_cap<WIN>())) - 1;
        uint32_t mf = (uint32_t)__builtin_amdgcn_readlane((int)m, f);
        const int j = tok_cap<WIN>() - (__builtin_amdgcn_readlane(inc, f) - __builtin_amdgcn_readlane(cb, f));
        for (int u = 0; u < j; ++u) mf &= mf - 1;  // drop the j lowest boundaries of lane f
        const int k = __ffs(mf) - 1;
        C = A + CH * f + k;
        c_rs = (((uint32_t)__builtin_amdgcn_readlane((int)ra_own, f)) >> k) & 1u;
      }
    }
    const bool inwin = l < 63 && cur.o < C;  // read rs0+l starts in [P, C)
    const int nst = __popcll(ballot(inwin));
    // ---- per-read slots ----
    if (inwin) {
      const int q = l + 1;
      const bool up = uo_nx != cur.uo, dn = dno_nx != cur.dno;  // flank lengths < 2^32
      uint32_t derr = 0;
      // (a kernel without the negative rounds parses a negative start from 0, flagged)
      const int ts = !NEG && cur.ts < 0 ? 0 : cur.ts;
      if (!NEG && cur.ts < 0) derr |= DE_UNSUP;
      // obsarr[2 tstart] (:303) with Python's negative wrap: below -n past the
      // front (IndexError), in [-n, 0) a LEFT string at the wrapped ODD
      // position n + tstart (listed; only NEG chunks see a negative tstart)
      if (up && ts < 0) {
        if (ts + n < 0) derr |= DE_INDEX;
        else if constexpr (NEG) derr |= push_wo(a, gb + ts + n, rs0 + l, kWoUp, 0, 0);
        else derr |= DE_INTERNAL;
      }
      if (ts < MPC_TSTART_MIN) derr |= DE_UNSUP;
      if (up && ts > n) derr |= DE_INDEX;             // leftIndel(2*i) past the end
      if (o_nx <= cur.o) derr |= DE_OP;               // processOperation('', '')
      if (derr) flag_read(a, derr, rs0 + l);
      if (up && ts >= 0 && ts <= n) left_bit(ts);  // upstream flank: LEFT at gap tstart
      W.s_end[q] = o_nx;
      W.s_ts[q] = ts < MPC_TSTART_MIN ? MPC_TSTART_MIN : (ts > kICap ? kICap : ts);
      W.s_read[q] = (int32_t)(rs0 + l);
      W.s_iend[q] = (ts < 0 ? 0 : (ts > n ? n + 1 : ts)) | (dn ? 1 << 30 : 0);
    }
    // ---- the next window starts at C: its bytes go by LDS-DMA into the other
    // stage buffer now, behind this window's rounds (its read records load
    // after the rounds: holding them across the rounds costs VGPRs) ----
    const int64_t Pn = C, rsn = rs0 + nst;
    if (dma && Pn < wend) dma_window<WIN>(a.cs + (Pn & ~(int64_t)15), W.stage[sb ^ 1]);
    // (prefetch_cs: the next window's cs bytes load now, behind the rounds,
    // into registers that stay live across them; its read records after them)
    typename Chunk<CH>::T nxt_d{};
    if (prefetch_cs<TM>() && !dma && Pn < wend) nxt_d = cs_load<CH>(a.cs + (Pn & ~(int64_t)15) + CH * l);
    // ---- token list: starts in [P, C) (bit 15 = read start), then the sentinel ----
    int T;
    {
      int tlo = (int)(P - cA), thi = (int)(C - cA);
      tlo = tlo < 0 ? 0 : (tlo > CH ? CH : tlo);
      thi = thi < 0 ? 0 : (thi > CH ? CH : thi);
      const uint32_t rng = lowmask(thi) & ~lowmask(tlo);
      const uint32_t tm = em_own & rng;
      // Units: a ':' token with 1-4 operand bytes and the op token right after
      // it in the same read, both in [P, C), are ONE list entry (bits 12-14: the
      // ':' operand length); every other token is its own entry.  Bit-parallel
      // on 32-bit masks: bit k of at(m, d) = bit k + d of this lane's mask m
      // continued by the next lane's, so a ':' at k has operand length d - 1
      // when the first boundary after it is an op at k + d (d = 2..5).
      const uint32_t cmr = cm_own & rng, omr = om_own & ~ra_own & rng;
      const uint32_t em_nx = from_lane_above(em_own), om_nx = from_lane_above(omr);
      auto at = [&](uint32_t own, uint32_t nx, int d) -> uint32_t {
        if constexpr (CH == 32) return __builtin_amdgcn_alignbit(nx, own, (uint32_t)d);
        else return (own | (nx << CH)) >> d;
      };
      const uint32_t n1 = ~at(em_own, em_nx, 1), n2 = n1 & ~at(em_own, em_nx, 2);
      const uint32_t n3 = n2 & ~at(em_own, em_nx, 3), n4 = n3 & ~at(em_own, em_nx, 4);
      const uint32_t p2 = cmr & n1 & at(omr, om_nx, 2);  // ':' whose op is 2 bytes on
      const uint32_t p3 = cmr & n2 & at(omr, om_nx, 3);
      const uint32_t p4 = cmr & n3 & at(omr, om_nx, 4);
      const uint32_t p5 = cmr & n4 & at(omr, om_nx, 5);
      const uint32_t pl0 = p2 | p4, pl1 = p3 | p4;        // operand length d - 1 in 3 bit planes
      // the absorbed ops: here, or (carried) in the next lane
      uint32_t ab_own, ab_hi;
      if constexpr (CH == 32) {
        ab_own = (p2 << 2) | (p3 << 3) | (p4 << 4) | (p5 << 5);
        ab_hi = (p2 >> 30) | (p3 >> 29) | (p4 >> 28) | (p5 >> 27);
      } else {
        const uint32_t ab = (p2 << 2) | (p3 << 3) | (p4 << 4) | (p5 << 5);
        ab_own = ab & lowmask(CH);
        ab_hi = ab >> CH;
      }
      ab_own |= from_lane_below(ab_hi);
      const uint32_t tu = tm & ~ab_own;
      const int cnt = __popc(tu);
      const int incl = wave_scan_i32(cnt);
      T = wave_last_i32(incl);
      const int base = CH * l;
      auto entry = [&](int k) -> uint16_t {
        return (uint16_t)((uint32_t)(base + k) | (((pl0 >> k) & 1u) << 12) | (((pl1 >> k) & 1u) << 13) |
                          (((p5 >> k) & 1u) << 14) | (((ra_own >> k) & 1u) << 15));
      };
      uint32_t m = tu;
      int idx = incl - cnt;
      while (m) {
        const int k = __ffs(m) - 1;
        m &= m - 1;
        W.tok[idx++] = entry(k);
      }
      if (l == 0) W.tok[T] = far ? (uint16_t)(kFar | (c_rs ? 0x8000u : 0u)) : (uint16_t)((C - A) | (c_rs ? 0x8000u : 0u));
    }
    wave_sync_lds();
    MPC_SEG(1);

    // ---- rounds: one token per lane ----
    const int far_c = (int)(C - A < (1 << 30) ? C - A : (1 << 30));  // wave-uniform
    int32_t G = 0;  // advances of the window's earlier rounds
    int qc = 0;     // read starts of the window's earlier rounds
    int32_t cb = c_base;  // coordinate base of the open read (wave-uniform)
    // one round (64 units, one per lane): GEN = the general decode; without it
    // the fast decode, and false (nothing applied) when a unit is not canonical
    auto round = [&](const int t0, auto genc) -> bool {
      constexpr bool GEN = decltype(genc)::value;
      const int t = t0 + l;
      const bool v = t < T;
      const uint32_t t0r = W.tok[t], t1r = W.tok[t + 1];  // in bounds for every lane (+64 padding)
      const uint32_t e0 = v ? t0r : 0u, e1 = v ? t1r : 0u;
      const int s0 = (int)(e0 & 0xfffu);         // unit start
      const int pl = (int)((e0 >> 12) & 7u);     // ':' operand length of a unit's prefix (0: none)
      const int sx = pl ? s0 + pl + 1 : s0;      // the unit's main token
      const bool lfar = v && ((e1 & 0x7fffu) == kFar);
      // far: the token ends at C (beyond the window); 32-bit here (far_c saturates
      // at 2^30 > kAdvCap + the window), 64-bit only on the slow path
      const int ex32 = lfar ? far_c : (int)(e1 & 0xfffu);
      const int ex = ex32 - sx - 1 < kAdvCap ? ex32 : sx + 1 + kAdvCap;
      const bool is_rs = v && (e0 >> 15);
      const bool last = v && (e1 >> 15);
      const uint64_t brs = ballot(is_rs);
      const int q = qc + lanes_below(brs) + (is_rs ? 1 : 0);
      // the read's slot (tstart, read, i_end), loaded before the decode
      const int32_t q_ts = W.s_ts[q], q_read = W.s_read[q], q_iend = W.s_iend[q];
      // ---- decode.  Fast path: every unit of the round is canonical -- an
      // optional absorbed ':' prefix of 1-4 digits, then ':' + 1-4 digits, '*' +
      // 1-4 bytes ending in a base, '+' + 1-4 bases or '-' + 1-4 bytes, ending
      // inside the window -- so no data error can arise but the coordinate
      // checks; branch-free from two 8-byte LDS reads.  A round holding any
      // other unit ('Z', empty / long operands, non-digits, non-bases, a token
      // past the window, a read not starting with an operator) takes the
      // general decode below for all its lanes.
      const uint32_t* b32 = reinterpret_cast<const uint32_t*>(W.stage[sb]);
      int adv0, adv, kind, olen_e;
      uint32_t pay, err = 0u;
      bool fast = false;
      if constexpr (!GEN) {
        const uint32_t sh = (uint32_t)(sx & 3);
        uint32_t m0 = b32[sx >> 2], m1 = b32[(sx >> 2) + 1];  // bytes sx .. sx + 4 (sh + 4 <= 7)
        const int pa = (s0 + 1) >> 2;
        uint32_t p0 = b32[pa], p1 = b32[pa + 1];
        // (opaque: both 8-byte reads issue together, unconditionally -- the
        // compiler would otherwise sink the prefix read into a branch on pl)
        asm volatile("" : "+v"(m0), "+v"(m1), "+v"(p0), "+v"(p1));
        const uint32_t op = __builtin_amdgcn_alignbyte(m1, m0, sh) & 0xffu;
        const uint32_t ow = sh == 3u ? m1 : __builtin_amdgcn_alignbyte(m1, m0, sh + 1u);  // operand bytes
        const uint32_t pw = __builtin_amdgcn_alignbyte(p1, p0, (uint32_t)((s0 + 1) & 3));  // ':' prefix
        const int olen = ex32 - sx - 1;
        const int ol4 = olen < 0 ? 0 : (olen > 4 ? 4 : olen);
        const bool colon = op == ':', star = op == '*', plus = op == '+', minus = op == '-';
        const int cl = pl ? pl : (colon ? ol4 : 0);  // digits of the unit's ':' operand
        const uint32_t cw = pl ? pw : ow;
        const uint32_t cvm = cl == 4 ? 0xffffffffu : ((1u << (8 * cl)) - 1u);
        const uint32_t Tx = cw ^ 0x30303030u;
        const bool dig = ((((Tx & 0x7F7F7F7Fu) + 0x76767676u) | Tx) & 0x80808080u & cvm) == 0;
        uint32_t X = (Tx & cvm & 0x0F0F0F0Fu) << ((32 - 8 * cl) & 31);  // right-aligned digits (cl = 0: 0)
        X = mul2561(X) >> 8;
        X = ((X & 0x00FF00FFu) * 6553601u) >> 16;
        const int val = (int)(X & 0xffffu);
        //   bases: (c|0x20) must equal "acgt"[h] with h = (lc>>1)&3 (v_perm table lookup)
        const uint32_t lc = ow | 0x20202020u;
        const uint32_t hh = (lc >> 1) & 0x03030303u;
        const uint32_t bad = lc ^ __builtin_amdgcn_perm(0u, 0x67746361u, hh);
        const uint32_t codes = ((hh & 0x01010101u) << 1) | ((hh >> 1) & 0x01010101u);  // dict order A0 T1 C2 G3
        const uint32_t shl = 8u * (uint32_t)((ol4 - 1) & 3);
        const uint32_t vm = ol4 == 4 ? 0xffffffffu : ((1u << (8 * ol4)) - 1u);
        uint32_t pk = (codes | (codes >> 6)) & 0x000f000fu;
        pk = (pk | (pk >> 12)) & ((1u << (2 * ol4)) - 1u);
        // a special token with an empty operand that is not its read's last --
        // the 'Z' and ':' every read's cs starts with ("Z::12*ag") -- is a no-op
        // (:309: the operator is only applied to a non-empty operand); no prefix
        // can precede it ('Z' / ':' / '*' / '+' / '-' are never absorbed digits)
        const bool nop = (olen == 0) & !last & (pl == 0) & (colon | star | plus | minus | (op == 'Z'));
        if constexpr (int_check<TM>()) {  // VALU integers and one compare
          const uint32_t not4 = (uint32_t)(olen - 1) >> 2;  // 0 iff 1 <= olen <= 4
          const uint32_t dbad = (((Tx & 0x7F7F7F7Fu) + 0x76767676u) | Tx) & 0x80808080u & cvm;
          const uint32_t bbad = (star | plus) ? (bad & vm) : 0u;
          const uint32_t obad = (colon | star | plus | minus) ? 0u : 1u;
          fast = !v | (!lfar & (((not4 | dbad | bbad | obad) == 0u) | nop));
          (void)dig;
        } else {
          fast = !v | (!lfar & ((olen >= 1) & (olen <= 4) & dig &
                                (colon | minus | (star & (((bad >> shl) & 0xffu) == 0u)) | (plus & ((bad & vm) == 0u))) |
                                nop));
        }
        // branch-free: '*' 0x2A -> 2, '+' 0x2B -> 3, '-' 0x2D -> 4 from op & 7;
        // ':' -> 1 when it matches at least one base (:77); a no-op: 0
        const int mv = -(int)(v & !nop), mc = -(int)colon;
        const int o7 = (int)(op & 7u);
        kind = mv & ((mc & (int)(val > 0)) | (~mc & (o7 - (o7 >> 2))));
        adv = mv & ((mc & val) | (int)star | (-(int)minus & ol4));
        adv0 = mv & (-(int)(pl != 0)) & val;
        const uint32_t ms = 0u - (uint32_t)star;
        pay = (ms & ((codes >> shl) & 3u)) | (~ms & pk);
        olen_e = ol4;
        if (ballot(!fast)) return false;  // (before any effect: the round restarts on the general decode)
      }
      if constexpr (GEN) {  // general decode of the whole round
        const int a4 = sx >> 2;
        const uint32_t sh = (uint32_t)(sx & 3);
        const uint32_t d0 = b32[a4], d1 = b32[a4 + 1], d2 = b32[a4 + 2];
        const uint32_t x0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
        const uint32_t x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
        const uint32_t op = x0 & 0xffu;
        const uint32_t w0 = __builtin_amdgcn_alignbyte(x1, x0, 1u);
        const int olen = ex - sx - 1;
        // branch-free decode: op class, 4 operand bytes at once (SWAR)
        const bool colon = op == ':', star = op == '*', plus = op == '+', minus = op == '-';
        const bool spec = colon | star | plus | minus | (op == 'Z');
        const bool act = v & spec & ((olen > 0) | last);  // empty operand: skipped unless last (:309, :320)
        const int ol4 = olen < 0 ? 0 : (olen > 4 ? 4 : olen);
        const uint32_t vm = ol4 == 4 ? 0xffffffffu : ((1u << (8 * ol4)) - 1u);  // operand bytes in w0
        //   the unit's ':' operand -- its prefix (pl bytes after s0) or the main
        //   token's own operand -- up to 4 digits: right-align, SWAR decimal
        const bool pre = pl != 0;
        const int pa = (s0 + 1) >> 2;
        const uint32_t pw = __builtin_amdgcn_alignbyte(b32[pa + 1], b32[pa], (uint32_t)((s0 + 1) & 3));
        const int cl = pre ? pl : (colon ? ol4 : 0);
        const uint32_t cw = pre ? pw : w0;
        const uint32_t cvm = cl == 4 ? 0xffffffffu : ((1u << (8 * cl)) - 1u);
        const uint32_t Tx = cw ^ 0x30303030u;
        const bool cdig = ((((Tx & 0x7F7F7F7Fu) + 0x76767676u) | Tx) & 0x80808080u & cvm) == 0;
        uint32_t X = cl == 0 ? 0u : (Tx & cvm & 0x0F0F0F0Fu) << (8 * (4 - cl));
        X = mul2561(X) >> 8;
        X = ((X & 0x00FF00FFu) * 6553601u) >> 16;
        const int adv_c = (int)(X & 0xffffu);
        adv0 = pre ? adv_c : 0;
        const bool dig_ok = (olen >= 1) & (olen <= 4) & cdig;  // main ':' token
        //   bases: (c|0x20) must equal "acgt"[h] with h = (lc>>1)&3 (v_perm table lookup)
        const uint32_t lc = w0 | 0x20202020u;
        const uint32_t hh = (lc >> 1) & 0x03030303u;
        const uint32_t bad = lc ^ __builtin_amdgcn_perm(0u, 0x67746361u, hh);
        const uint32_t codes = ((hh & 0x01010101u) << 1) | ((hh >> 1) & 0x01010101u);  // dict order A0 T1 C2 G3
        const int shl = 8 * ((olen - 1) & 3);
        const bool last_ok = ((bad >> shl) & 0xffu) == 0;  // '*': written base = operand[-1] (:96)
        uint32_t pk = codes;
        pk = (pk | (pk >> 6)) & 0x000f000fu;
        pk = (pk | (pk >> 12)) & 0xffu;
        const uint32_t mstar = 0u - (uint32_t)star;
        pay = (mstar & ((codes >> shl) & 3u)) | (~mstar & (pk & ((1u << (2 * ol4)) - 1u)));
        const bool slow = lfar | (pre & !cdig) | (act & ((colon & !dig_ok) | ((star | plus) & (olen > 4))));
        const int kop = ((int)star << 1) | ((int)plus * 3) | ((int)minus << 2);  // exclusive classes
        const int mcol = -(int)colon;
        kind = (-(int)act) & ((mcol & (int)(adv_c > 0)) | (~mcol & (-(int)(olen > 0) & kop)));
        adv = (-(int)(kind == 1) & adv_c) | (int)(kind == 2) | (-(int)(kind == 4) & (olen < kAdvCap ? olen : kAdvCap));
        err = (v & !spec) ? DE_OP : 0u;  // cs does not start with an operator (:100-102)
        if (act & star & (olen == 0)) err |= DE_INDEX;  // operand[-1] of '' (:96)
        if ((kind == 2) & !last_ok) err |= DE_KEY;
        if ((kind == 3) & ((bad & vm) != 0)) err |= DE_KEY;
        olen_e = olen;
        if (slow) {  // rare: decode from HBM
          const int64_t s = A + sx, e = A + (lfar ? C - A : (int64_t)(e1 & 0xfffu));
          const TokInfo ti = analyze_long(a.cs, s, e, last);
          adv = ti.adv; kind = ti.kind; pay = ti.pay; err = ti.err;
          olen_e = (int)(e - s - 1 < kAdvCap ? e - s - 1 : kAdvCap);
          if (pl) {
            const TokInfo tp = analyze_long(a.cs, A + s0, s, false);
            adv0 = tp.adv;
            err |= tp.err;
          }
        }
      }
      MPC_SEG(2);
      // ---- coordinates ----
      const int advu = adv0 + adv;            // unit advance <= 2^23: 64 lanes stay < 2^29
      const int ainc = wave_scan_i32(advu);
      const int aex = ainc - advu;
      const int atot = wave_last_i32(ainc);
      // read bases, i = base + G + aex: lanes before the round's first read
      // start continue the open read (base cb); a read starting at lane j has
      // base tstart - (G + aex_j) on lanes j.. up to the next start.  One
      // scalar pass over the start lanes (about one per round: reads hold tens
      // to hundreds of units) instead of an LDS write, fence and read back
      int bv = cb;
      if constexpr (bperm_base<TM>()) {
        // the last read start at or below this lane (its base by one
        // ds_bpermute), else the read open since an earlier round (cb)
        const uint64_t le = brs & (~0ull >> (63 - l));
        const int mine = q_ts - (G + aex);
        const int ls = le ? 63 - __clzll((long long)le) : 0;
        const int sv = __builtin_amdgcn_ds_bpermute(ls << 2, mine);
        bv = le ? sv : cb;
        if (brs) cb = __builtin_amdgcn_readlane(mine, 63 - __clzll((long long)brs));
      } else if constexpr (lds_base<TM>()) {
        if (is_rs) W.s_val[q] = q_ts - (G + aex);
        wave_sync_lds();
        const int sv = W.s_val[q];
        bv = q == 0 ? cb : sv;  // slot 0: the read open since an earlier window
      } else {
        for (uint64_t m = brs; m; m &= m - 1) {
          const int j = __ffsll((unsigned long long)m) - 1;
          cb = __builtin_amdgcn_readlane(q_ts, j) - (G + __builtin_amdgcn_readlane(aex, j));
          bv = l >= j ? cb : bv;
        }
      }
      const int iu = bv + G + aex;  // coordinate at the unit start
      const int i = iu + adv0;                // ... and at its main token
      MPC_SEG(3);
      // ---- effects ----
      // data errors and effects as flat predicates (no nested exec-mask regions)
      // IndexError (refarr / obsarr past the end): a ':' prefix writes [iu, i),
      // ':' [i, i + adv), '*' [i, i + 1), '+' the gap i: every kind 1-3 needs
      // 0 <= i and i + adv <= n (adv = 1 for '*', 0 for '+'); sign of an OR
      bool bad_i = ((adv0 > 0) & ((iu | (n - i)) < 0)) | (((uint32_t)(kind - 1) <= 2u) & ((i | (n - adv - i)) < 0));
      // Negative coordinates (a negative tstart; chunks that hold one only):
      // refarr / obsarr take index x at len + x for x in [-(2n+1), 0)
      // (Python list indexing).  A ':' or '-' there writes nothing
      // (the wrapped refarr index is even: ''); a '*' at i < 0 writes its base
      // as a one-base LEFT string at gap n + 1 + i; a '+' at i in [-n, 0) is a
      // LEFT string at the wrapped ODD position n + i (listed, push_wo)
      bool wrap = false, unsup = false, wo_ins = false;
      int di = i, gi = i, li = olen_e;  // deletion start, LEFT gap and length
      if constexpr (NEG) {
        const bool mat = (kind == 1) | (kind == 2);
        bad_i = ((adv0 > 0) & (((iu + n + 1) | (n - i)) < 0)) | (mat & (((i + n + 1) | (n - adv - i)) < 0)) |
                ((kind == 3) & (((i + n) | (n - i)) < 0));
        // an advance clamped at kAdvCap from a negative coordinate (its true
        // end may still be <= n)
        unsup = ((adv0 >= kAdvCap) & (iu < 0)) | ((adv >= kAdvCap) & (i < 0) & ((kind == 1) | (kind == 4)));
        wo_ins = (kind == 3) & (i < 0) & (i + n >= 0);
        wrap = (kind == 2) & (i < 0);
        di = i < 0 ? 0 : i;
        gi = wrap ? i + n + 1 : i;
        li = wrap ? 1 : olen_e;
      }
      uint32_t te = err | (bad_i ? DE_INDEX : 0u) | (unsup ? DE_UNSUP : 0u);
      const int rl = q_read;
      if (NEG && wo_ins && te == 0) te |= push_wo(a, gb + i + n, rl, kWoIns, olen_e, A + sx + 1);
      const bool ok = te == 0 && !wo_ins;
      const bool ins_inline = ((kind == 3 && olen_e <= kInsInline) || wrap) && ok;
      const bool any_ins = ballot(ins_inline) != 0;  // (wave-uniform)
      uint32_t pold = 0u;
      if (!DP && MPC_EARLY_PLACE && any_ins && ins_inline) pold = atomicAdd(bkw + gi / kBW, 1u);  // slot in its bucket's page
      if (ok & (kind == 2) & !wrap & (TM != 3 || (!S1 && a.sub_wins == 0))) odd_sub(i, (int)pay);  // (S1: one window)
      const bool del = NEG ? ok & (kind == 4) & (di < n) & (i + olen_e > di) : ok & (kind == 4) & (i >= 0) & (i < n);
      if (del) {
        depth_dec(di);
        depth_inc(i + olen_e < n ? i + olen_e : n);
      }
      if (ok & ((kind == 3) | wrap)) left_bit(gi);
      if (ok & (kind == 3) & (olen_e > kInsInline)) push_ovf(a, A + sx + 1, rl, i, olen_e);
      if (S1) {  // one substitution window: a wave-uniform count
        const bool sev = ok && kind == 2 && !wrap;
        const uint64_t bw = ballot(sev);
        const uint16_t ev = (uint16_t)(((uint32_t)i << 2) | pay);
        if (DQS) {
          if (sev) sq[(nsub_s + lanes_below(bw)) & (kSubQ - 1)] = ev;
        } else {
          if (sev) a.subev[sev_base + nsub_s + lanes_below(bw)] = ev;
        }
        nsub_s += (uint32_t)__popcll(bw);
      } else if (TM == 3 && a.sub_wins > 0) {  // substitution events, wave-aggregated per window
        const bool sev = ok && kind == 2 && !wrap;
        const int win = i >> kSubWinBits;
        uint16_t* wp = a.subev + sev_base;  // window ww's region of this wave
        for (int ww = 0; ww < a.sub_wins; ++ww, wp += a.subev_cap) {
          const bool mine = sev && win == ww;
          const uint64_t bw = ballot(mine);
          if (!bw) continue;
          const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)nsub_v, ww);
          if (mine) wp[n0 + lanes_below(bw)] = (uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay);
          if (l == ww) nsub_v += (uint32_t)__popcll(bw);
        }
      }
      if (DP) {  // the event into the wave's queue
        const uint64_t bi = ballot(ins_inline);
        if (ins_inline)
          dq[(dq_head + lanes_below(bi)) & (kDefQ - 1)] = make_uint2((uint32_t)(gi / kBW), ins_word(gi, li, pay, rl - (int)r0));
        dq_head += (uint32_t)__popcll(bi);
      } else if (any_ins) {  // the event into its bucket's page (written once)
        parse_place_event<big, MPC_EARLY_PLACE != 0>(a, ins_inline, bkw + gi / kBW, npg, pbase, pg0, pcap, gi / kBW,
                                                     ins_word(gi, li, pay, rl - (int)r0), pold);
      }
      if (last) {  // the read's last operation: i_end, downstream check, span
        const int ia = i + adv;
        const int ie = ia < 0 ? 0 : (ia > n ? n + 1 : ia);
        const int dnf = q_iend & (1 << 30);
        if (dnf && ia > n) te |= DE_INDEX;   // rightIndel(2*i) past the end
        // ... or, wrapped, past the front, or a RIGHT string at the odd
        // position n + ia (listed; i_end n + 1: no gap row for it)
        int iw = ie;
        if (NEG && dnf && ia < 0) {
          if (ia + n < 0) te |= DE_INDEX;
          else { te |= push_wo(a, gb + ia + n, rl, kWoDown, 0, 0); iw = n + 1; }
        }
        W.s_iend[q] = iw | dnf;
        const int ts = NEG && q_ts < 0 ? 0 : q_ts;  // matches below 0 write nothing
        const int e2 = ie > n ? n : ie;
        if (ts < e2) { depth_inc(ts); depth_dec(e2); }
      }
      if (te) flag_read(a, te, rl);
      G += atot;
      qc += __popcll(brs);
      MPC_SEG(4);
      return true;
    };
    // canonical rounds take the fast decode; a round holding any other unit is
    // redone on the general decode (one loop: measured against a loop per kind
    // and against per-window canonical checks, profiles/r06_experiments/)
    for (int t0 = 0; t0 < T; t0 += 64) {
      if (!fast_decode<TM>() || !round(t0, std::false_type{})) round(t0, std::true_type{});
      if (DP && dq_head - dq_tail >= 64u) defer_flush(64);
      if (DQS && nsub_s - sq_tail >= 128u) sub_flush(128u);
    }
    wave_sync_lds();
    // ---- reads that ended in this window: i_end; carry the open one ----
    if (l <= nst && (l > 0 || carry) && W.s_end[l] <= C) a.i_end[W.s_read[l]] = W.s_iend[l] & ~(1 << 30);
    const bool cont = (nst > 0 || carry) && W.s_end[nst] > C;
    if constexpr (lds_base<TM>())
      if (nst > 0) cb = uniform_i32(W.s_val[nst]);  // the base of the window's last read start
    if (cont) {
      const int64_t v = (int64_t)cb + G;
      c_base = (int32_t)(v > kICap ? kICap : v);
    }
    if (cont && l == 0) {
      W.s_end[0] = W.s_end[nst];
      W.s_ts[0] = W.s_ts[nst];
      W.s_read[0] = W.s_read[nst];
      W.s_iend[0] = W.s_iend[nst];
    }
    carry = cont;
    wave_sync_lds();
    P = Pn;
    rs0 = rsn;
    sb ^= dma ? 1 : 0;
    if (Pn < wend) {
      if (prefetch_cs<TM>() && !dma) {
        cur = fetch_window<CH, false>(a, Pn, rsn, l);
        cur.d = nxt_d;
      } else {
        cur = fetch_window<CH, !dma>(a, Pn, rsn, l);
      }
    }
    MPC_SEG(5);
  }
  // reads starting at the range end have an empty cs
  for (int64_t r = rs0 + l; r < rb; r += 64) {
    const int ts = a.tstart[r];
    flag_read(a, DE_OP, r);
    a.i_end[r] = ts < 0 ? 0 : (ts > n ? n + 1 : ts);
  }
  if (DQS && nsub_s != sq_tail) sub_flush(nsub_s - sq_tail);  // (<= 127)
  if (TM == 3 && l < a.sub_wins)
    a.subev_cnt[((int64_t)blockIdx.x * kMaxCh + chk) * kMaxSubWins + l] = S1 ? nsub_s : nsub_v;
  }  // chunks
  };
  if constexpr (NK) {
    if (wg_neg) chunks(std::true_type{});
    else chunks(std::false_type{});
  } else {
    chunks(std::false_type{});
  }
  if (DP && dq_head != dq_tail) defer_flush((int)(dq_head - dq_tail));  // (<= 63)
  MPC_SEG(5);
  // every LDS-DMA was waited for by the window after it (one is issued only
  // when another window follows); drain anyway before the LDS is reused
  if (parse_dma<WIN>()) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  MPC_SEG(6);
  parse_epilogue<TM>(a, n, gb, nbk, hl, bkw, uni, npg, pbase, pcap);
#ifdef MPC_STAMPS
  MPC_SEG(7);
  const int64_t gw = (int64_t)blockIdx.x * kMaxPW + w;
  if (l < kStampSeg && gw < kStampWaves) {
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < kStampSeg; ++k) v = l == k ? st_acc[k] : v;
    g_stamps[gw * kStampSeg + l] = v;
  }
#endif
}


// ---------------------------------------------------------------------------
// K_subs (tally mode 3): the substitution events of a sample's parse waves for
// one kSubWin-position window, tallied in LDS as 16-bit counters (the event
// word IS the counter index: position << 2 | code; a block's chunk holds at most
// 65535 reads, and a read substitutes a position at most once) and flushed with
// contiguous atomics.  One block
// per (sample, window, chunk of <= kSubsWG parse workgroups); wave v walks the
// chunk's regions v, v + 16, ... (8 loads in flight per lane).
// ---------------------------------------------------------------------------
constexpr int kSubsWG = 32;  // parse workgroups per K_subs block, at most
// K_subs blocks store their 16-bit tallies in a slab row each, reduced per
// (sample, window) by K_subsum (instead of every block adding its ~4 n counters
// into the same words with global atomics)
#ifndef MPC_SUBS_SLAB
#define MPC_SUBS_SLAB 1
#endif
struct SubsArgs {
  const int4* work;    // {sample, window, first parse workgroup, end}
  const int4* pwork;   // parse work table {sample, r0, r1, 0}
  const int32_t* wave_tab;  // the parse chunks' read ranges (kMaxCh + 1 boundaries per workgroup)
  const int64_t* cs_off; int64_t cs_base;
  const uint16_t* subev; const uint32_t* subev_cnt; int64_t subev_cap;
  const int32_t* n_of; const int32_t* gbase; uint32_t* sub;
  uint32_t* slab;  // MPC_SUBS_SLAB: [K_subs block][kSubWin * 2] packed tallies
  int32_t nw_parse;
};
__global__ __launch_bounds__(1024) void K_subs(SubsArgs a) {
  __shared__ uint32_t cnt[kSubWin * 2];  // (position, code pair): codes 2h | 2h+1 in the halves
  const int4 wk = a.work[blockIdx.x];
  const int smp = wk.x, win = wk.y, pw0 = wk.z, pw1 = wk.w;
  const int nreg = (pw1 - pw0) * kMaxCh, l = lane(), v = threadIdx.x >> 6, nv = blockDim.x >> 6;
  for (int k = threadIdx.x; k < kSubWin * 2; k += blockDim.x) cnt[k] = 0;
  __syncthreads();
  for (int rg = v; rg < nreg; rg += nv) {
    const int pw = pw0 + rg / kMaxCh, ww = rg % kMaxCh;  // parse workgroup, chunk
    if (ww >= a.pwork[pw].w) continue;
    const int64_t ra = a.wave_tab[(int64_t)pw * (kMaxCh + 1) + ww];  // the chunk's first read
    const int c = (int)a.subev_cnt[((int64_t)pw * kMaxCh + ww) * kMaxSubWins + win];
    const uint16_t* src = a.subev + (int64_t)win * a.subev_cap + (a.cs_off[ra] - a.cs_base) / kSubEvBytes + 2 * ra;
    auto tally = [&](uint32_t ev) { atomicAdd(&cnt[ev >> 1], 1u << (16 * (ev & 1u))); };
    // 16-byte loads (8 events per lane each, 4 in flight): the region's events up
    // to the first 16-byte boundary and after the last whole group one per lane
    const int head = min(c, (int)(((16u - ((uint32_t)(uintptr_t)src & 15u)) & 15u) >> 1));
    if (l < head) tally(src[l]);
    const uint4* body = reinterpret_cast<const uint4*>(src + head);
    const int ng = (c - head) >> 3;
    for (int q0 = 0; q0 < ng; q0 += 4 * 64) {
      uint4 g[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = q0 + l + 64 * u;
        g[u] = q < ng ? body[q] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (q0 + l + 64 * u >= ng) continue;
        const uint32_t w4[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
#pragma unroll
        for (int h = 0; h < 4; ++h) { tally(w4[h] & 0xffffu); tally(w4[h] >> 16); }
      }
    }
    const int t0 = head + 8 * ng;
    if (t0 + l < c) tally(src[t0 + l]);  // (< 8 events)
  }
  __syncthreads();
  const int64_t p0 = (int64_t)win * kSubWin, n = a.n_of[smp];
  if (MPC_SUBS_SLAB) {  // the window's positions (< n), two words each, coalesced
    uint32_t* row = a.slab + (int64_t)blockIdx.x * (kSubWin * 2);
    const int nw2 = (int)(2 * (n - p0 < kSubWin ? n - p0 : kSubWin));
    for (int j = threadIdx.x; j < nw2; j += blockDim.x) row[j] = cnt[j];
    return;
  }
  uint32_t* dst = a.sub + ((int64_t)a.gbase[smp] + p0) * 4;
  for (int j = threadIdx.x; j < kSubWin * 4; j += blockDim.x) {  // consecutive lanes, consecutive words
    const uint32_t x = (cnt[j >> 1] >> (16 * (j & 1))) & 0xffffu;
    if (x && p0 + (j >> 2) < n) atomicAdd(dst + j, x);
  }
}

// K_subsum: per (sample, window, 256 slab words): the sum over the window's
// K_subs blocks (4 groups of rows per thread column, 8 loads in flight each,
// LDS reduce), stored into the substitution tallies (the only writer of a mode-3
// window's words).  work: {sample, window, first block, end block}.
constexpr int kSumCols = 256;
template <int RG>  // row groups: 4 when windows have many slab rows (C3: 256), else 1 (C5: ~5)
__global__ __launch_bounds__(kSumCols * RG) void K_subsum(const int4* work, const uint32_t* slab, const int32_t* n_of,
                                                          const int32_t* gbase, uint32_t* sub) {
  __shared__ uint32_t part[RG][kSumCols][2];
  constexpr int kChunks = kSubWin * 2 / kSumCols;
  const int4 wk = work[blockIdx.x / kChunks];
  const int x = threadIdx.x & (kSumCols - 1), y = threadIdx.x / kSumCols;
  const int64_t p0 = (int64_t)wk.y * kSubWin, n = n_of[wk.x];
  const int nw2 = (int)(2 * (n - p0 < kSubWin ? n - p0 : kSubWin));
  const int j = (int)(blockIdx.x % kChunks) * kSumCols + x;
  uint32_t lo = 0, hi = 0;
  if (j < nw2) {
    for (int b0 = wk.z + y; b0 < wk.w; b0 += RG * 8) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int b = b0 + RG * u;
        v[u] = b < wk.w ? slab[(int64_t)b * (kSubWin * 2) + j] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) { lo += v[u] & 0xffffu; hi += v[u] >> 16; }
    }
  }
  part[y][x][0] = lo;
  part[y][x][1] = hi;
  __syncthreads();
  if (y == 0 && j < nw2) {
    lo = 0;
    hi = 0;
#pragma unroll
    for (int r = 0; r < RG; ++r) { lo += part[r][x][0]; hi += part[r][x][1]; }
    uint32_t* dst = sub + ((int64_t)gbase[wk.x] + p0) * 4 + 2 * j;  // word j: position j / 2, codes 2 (j & 1) + {0, 1}
    dst[0] = lo;
    dst[1] = hi;
  }
}

// ---------------------------------------------------------------------------
// Downstream (RIGHT) events.  A gap holding only RIGHT events needs only its
// longest downstream flank (slot bi = base bi, :64-72).  Gaps that also hold a
// LEFT event ("mixed") need the RIGHT events in read order -> sort keys.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool has_left(const uint32_t* bm, int64_t g) { return (bm[g >> 5] >> (g & 31)) & 1u; }

__device__ __forceinline__ bool l_is(int j) { return lane() == j; }
__device__ __forceinline__ void rsplit_block(const Dev& d, int64_t b) {
  __shared__ int64_t s_key;
  __shared__ int32_t s_val;
  __shared__ int32_t s_w[16];
  const int64_t r = b * blockDim.x + threadIdx.x;
  const bool in = r < d.N;
  int64_t g = -1;
  int32_t len = 0;
  bool mixed = false;
  const int64_t rg = d.read_offset + r;
  if (in) {
    const int s = d.sample[r];
    const int64_t n = d.n_of[s];
    const int64_t ie = d.i_end[r];
    const int64_t L = d.down_off[r + 1] - d.down_off[r];
    len = L > 0x7fffffff ? 0x7fffffff : (int32_t)L;
    if (len > 0 && ie <= n) {
      g = d.gbase[s] + ie;
      mixed = has_left(d.hasleft, g);
    }
    d.rlen[rg] = len;
  }
  // block-local stable compaction of the mixed events (read order), for K_rsort
  const int f = mixed ? 1 : 0;
  const int inc = wave_scan_i32(f);
  const int w = threadIdx.x >> 6;
  if (lane() == 63) s_w[w] = inc;
  __syncthreads();
  int wpre = 0;
  for (int k = 0; k < w; ++k) wpre += s_w[k];
  if (mixed) {
    const int64_t o = b * blockDim.x + wpre + inc - 1;
    d.keys_in[o] = (uint32_t)g;
    d.vals_in[o] = (int32_t)rg;
  }
  if (d.gcnt) {  // multi-workgroup sort: the event's slot within its gap (any order), one atomic per gap per wave
    for (uint64_t act = ballot(mixed); act;) {
      const int lead = __ffsll((unsigned long long)act) - 1;
      const int32_t gl = __builtin_amdgcn_readlane((int)g, lead);
      const uint64_t same = ballot(mixed && (int32_t)g == gl);
      int32_t base = 0;
      if (l_is(lead)) base = atomicAdd(d.gcnt + gl, __popcll(same));
      base = __builtin_amdgcn_readlane(base, lead);
      if (mixed && (int32_t)g == gl) d.kslot[b * blockDim.x + wpre + inc - 1] = base + lanes_below(same);
      act &= ~same;
    }
  }
  if (threadIdx.x == blockDim.x - 1) d.bcnt[b] = wpre + inc;
  block_atomic_max(d.maxR, g < 0 ? 0 : g, len, in && g >= 0 && !mixed, &s_key, &s_val);
}

// ---------------------------------------------------------------------------
// K_rsort: the mixed RIGHT events (partial reads ending at gaps that also hold
// LEFT events: few) sorted by (gap, read).  One workgroup: gather the per-block
// lists of K_rsplit (in read order), then a stable LSD radix sort on the gap
// (8-bit digits, a contiguous segment per wave, wave multi-split ranks) -- in
// LDS when the list fits, else ping-ponging through HBM (same code, generic
// pointers).
// ---------------------------------------------------------------------------
constexpr int kSortLds = 8192;
constexpr int kRsuLds = 2;  // K_rsort chunks in flight in LDS (measured 1/2/4/8 at C1/C2/C4: 2)
constexpr int kGatherLds = 2048;  // source blocks whose prefix stays in LDS (entry-parallel gather)

// One stable LSD pass of K_rsort over digit (key >> sh) & 255: wave w owns the
// contiguous segment [s0, s1) of the list (read order); per-wave digit
// histograms, one scan -> per (wave, digit) start, then every wave walks ITS
// segment in order, 64 entries at a time: stable ranks by wave multi-split,
// the digit's cursor in the wave's own LDS row (no barrier inside the walk:
// 4 per pass).  Force-inlined at call sites whose buffers are all LDS or all
// HBM, so the accesses compile to ds_* / global_* instead of flat.
constexpr int kRS = 1024;
template <int U>  // chunks of 64 entries in flight per wave (HBM: latency; LDS: few)
__device__ __forceinline__ void rsort_pass(const uint32_t* sk, const int32_t* sv, uint32_t* dk, int32_t* dv, int sh,
                                           int64_t s0, int64_t s1, int32_t (*wc)[256], int32_t* hb) {
  constexpr int NW = kRS / 64;
  const int tid = threadIdx.x, l = lane(), w = tid >> 6;
  const uint64_t lt = (1ull << l) - 1ull;
  for (int k = l; k < 256; k += 64) wc[w][k] = 0;
  for (int64_t i0 = s0; i0 < s1; i0 += U * 64) {
    uint32_t kk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + 64 * u + l;
      kk[u] = i < s1 ? sk[i] : ~0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (kk[u] != ~0u) atomicAdd(&wc[w][(kk[u] >> sh) & 255u], 1);
  }
  __syncthreads();
  if (tid < 256) {
    int t = 0;
    for (int k = 0; k < NW; ++k) t += wc[k][tid];
    hb[tid] = t;
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the 256 digit totals (4 per lane)
    const int x0 = hb[4 * tid], x1 = hb[4 * tid + 1], x2 = hb[4 * tid + 2], x3 = hb[4 * tid + 3];
    const int t4 = x0 + x1 + x2 + x3;
    const int e = wave_scan_i32(t4) - t4;
    hb[4 * tid] = e; hb[4 * tid + 1] = e + x0; hb[4 * tid + 2] = e + x0 + x1; hb[4 * tid + 3] = e + x0 + x1 + x2;
  }
  __syncthreads();
  if (tid < 256) {  // per (wave, digit) start: digit start + the digit's entries in lower waves
    int run = hb[tid];
    for (int k = 0; k < NW; ++k) { const int c = wc[k][tid]; wc[k][tid] = run; run += c; }
  }
  __syncthreads();
  for (int64_t i0 = s0; i0 < s1; i0 += U * 64) {
    uint32_t kk[U];
    int32_t vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + 64 * u + l;
      kk[u] = i < s1 ? sk[i] : 0u;
      vv[u] = i < s1 ? sv[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool v = i0 + 64 * u + l < s1;
      const uint32_t dg = (kk[u] >> sh) & 255u;
      uint64_t m = ballot(v);
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const uint64_t bb = ballot(((dg >> bit) & 1u) != 0);
        m &= ((dg >> bit) & 1u) ? bb : ~bb;
      }
      const int rank = __popcll(m & lt);
      const int base = v ? wc[w][dg] : 0;
      if (v) { dk[base + rank] = kk[u]; dv[base + rank] = vv[u]; }
      if (v && rank == 0) wc[w][dg] = base + __popcll(m);  // after every lane's read (in order: one wave)
    }
  }
  __syncthreads();
}

// Register path of K_rsort (more entries than the LDS path holds, up to
// kRS * kRegE): an entry is ONE word, gap << sb | its index in read order (sb
// bits), so the stable gap passes keep read order and need one LDS buffer: the
// entries of a pass's source order sit in VGPRs (wave w: positions s0 + 64 u +
// lane), the scatter writes the new order into LDS, and every wave reloads its
// positions from there.  The values (global reads) wait in HBM at their index.
constexpr int kRegE = 32;
__device__ __forceinline__ void rsort_reg_pass(uint32_t (&e)[kRegE], int64_t s0, int64_t s1, int sh, uint32_t* buf,
                                               int32_t (*wc)[256], int32_t* hb, bool reload) {
  constexpr int NW = kRS / 64;
  const int tid = threadIdx.x, l = lane(), w = tid >> 6;
  const uint64_t lt = (1ull << l) - 1ull;
  for (int k = l; k < 256; k += 64) wc[w][k] = 0;
#pragma unroll
  for (int u = 0; u < kRegE; ++u)
    if (s0 + 64 * u + l < s1) atomicAdd(&wc[w][(e[u] >> sh) & 255u], 1);
  __syncthreads();
  if (tid < 256) {
    int t = 0;
    for (int k = 0; k < NW; ++k) t += wc[k][tid];
    hb[tid] = t;
  }
  __syncthreads();
  if (tid < 64) {
    const int x0 = hb[4 * tid], x1 = hb[4 * tid + 1], x2 = hb[4 * tid + 2], x3 = hb[4 * tid + 3];
    const int t4 = x0 + x1 + x2 + x3;
    const int ex = wave_scan_i32(t4) - t4;
    hb[4 * tid] = ex; hb[4 * tid + 1] = ex + x0; hb[4 * tid + 2] = ex + x0 + x1; hb[4 * tid + 3] = ex + x0 + x1 + x2;
  }
  __syncthreads();
  if (tid < 256) {
    int run = hb[tid];
    for (int k = 0; k < NW; ++k) { const int c = wc[k][tid]; wc[k][tid] = run; run += c; }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kRegE; ++u) {
    const bool v = s0 + 64 * u + l < s1;
    if (ballot(v) == 0) break;  // (wave-uniform) the wave's positions are used up
    const uint32_t dg = (e[u] >> sh) & 255u;
    uint64_t m = ballot(v);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const uint64_t bb = ballot(((dg >> bit) & 1u) != 0);
      m &= ((dg >> bit) & 1u) ? bb : ~bb;
    }
    const int rank = __popcll(m & lt);
    const int base = v ? wc[w][dg] : 0;
    if (v) buf[base + rank] = e[u];
    if (v && rank == 0) wc[w][dg] = base + __popcll(m);
  }
  __syncthreads();
  if (reload) {
#pragma unroll
    for (int u = 0; u < kRegE; ++u)
      if (s0 + 64 * u + l < s1) e[u] = buf[s0 + 64 * u + l];
  }
}

__global__ __launch_bounds__(kRS) void K_rsort(Dev d, int32_t nblocks, int32_t end_bit) {
  if (d.rsflag && d.rsflag[0] == 1) return;  // the multi-workgroup path sorted them
  __shared__ uint32_t pool[4 * kSortLds];  // LDS path: keys and values, two buffers each; register path: one buffer
  uint32_t (*lk)[kSortLds] = reinterpret_cast<uint32_t (*)[kSortLds]>(pool);
  int32_t (*lv)[kSortLds] = reinterpret_cast<int32_t (*)[kSortLds]>(pool + 2 * kSortLds);
  __shared__ int32_t wc[kRS / 64][256];
  __shared__ int32_t hb[256];
  __shared__ int32_t s_w[kRS / 64];
  __shared__ int32_t s_carry;
  __shared__ int32_t s_bpre[kGatherLds + 1];
  const int tid = threadIdx.x, l = lane(), w = tid >> 6;
  const bool pre_lds = nblocks <= kGatherLds;
  // exclusive prefix of the per-block counts -> bpre[0..nblocks]
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (int c0 = 0; c0 < nblocks; c0 += kRS) {
    const int b = c0 + tid;
    const int v = b < nblocks ? d.bcnt[b] : 0;
    const int inc = wave_scan_i32(v);
    if (l == 63) s_w[w] = inc;
    __syncthreads();
    int pre = s_carry;
    for (int k = 0; k < w; ++k) pre += s_w[k];
    if (b < nblocks) {
      d.bpre[b] = pre + inc - v;
      if (pre_lds) s_bpre[b] = pre + inc - v;
    }
    __syncthreads();
    if (tid == kRS - 1) s_carry = pre + inc;
    __syncthreads();
  }
  const int64_t M = s_carry;
  if (tid == 0) { d.bpre[nblocks] = (int32_t)M; d.status[MPC_ST_MIXED] = (uint32_t)M; }
  if (M == 0) return;
  const int passes = (end_bit + 7) / 8;
  const bool in_lds = M <= kSortLds;
  const int sb = 32 - __clz((uint32_t)(M - 1) | 1u);  // bits of an entry index (register path)
  if (!in_lds && M <= (int64_t)kRS * kRegE && end_bit + sb <= 32) {
    // ---- register path: gather gap << sb | index into LDS (values to HBM), one source block per thread ----
    for (int b = tid; b < nblocks; b += kRS) {
      const int c = d.bcnt[b];
      const int o = d.bpre[b];
      const uint32_t* ks = d.keys_in + (int64_t)b * kRS;
      const int32_t* vs = d.vals_in + (int64_t)b * kRS;
      for (int j0 = 0; j0 < c; j0 += 8) {
        uint32_t kk[8];
        int32_t vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = j0 + u < c ? j0 + u : c - 1;
          kk[u] = ks[j];
          vv[u] = vs[j];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (j0 + u < c) { pool[o + j0 + u] = kk[u] << sb | (uint32_t)(o + j0 + u); d.vals_tmp[o + j0 + u] = vv[u]; }
      }
    }
    __syncthreads();
    constexpr int NW = kRS / 64;
    const int64_t s0 = M * w / NW, s1 = M * (w + 1) / NW;  // <= 64 kRegE positions per wave
    uint32_t e[kRegE];
#pragma unroll
    for (int u = 0; u < kRegE; ++u) e[u] = s0 + 64 * u + l < s1 ? pool[s0 + 64 * u + l] : 0u;
    __syncthreads();  // every wave holds its entries before the first scatter
    for (int p = 0; p < passes; ++p) rsort_reg_pass(e, s0, s1, sb + 8 * p, pool, wc, hb, p + 1 < passes);
    const uint32_t im = (1u << sb) - 1u;  // (sb <= 15 here)
    for (int64_t i0 = 0; i0 < M; i0 += 4 * kRS) {
      uint32_t x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { const int64_t i = i0 + tid + u * kRS; x[u] = i < M ? pool[i] : 0u; }
      int32_t vv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { const int64_t i = i0 + tid + u * kRS; vv[u] = i < M ? d.vals_tmp[x[u] & im] : 0; }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + tid + u * kRS;
        if (i < M) { d.keys_out[i] = x[u] >> sb; d.vals_out[i] = vv[u]; }
      }
    }
    return;
  }
  uint32_t* kb[2];
  int32_t* vb[2];
  if (in_lds) { kb[0] = lk[0]; kb[1] = lk[1]; vb[0] = lv[0]; vb[1] = lv[1]; }
  else {
    kb[passes & 1] = d.keys_out; vb[passes & 1] = d.vals_out;
    kb[(passes + 1) & 1] = d.keys_tmp; vb[(passes + 1) & 1] = d.vals_tmp;
  }
  __syncthreads();
  // gather (read order) into buffer 0.  Few source blocks: entry-parallel, the
  // source block of entry i by a search of the LDS prefix, 8 loads in flight
  // per thread; else one source block per thread, 8 loads in flight per batch
  // (the copies are independent; a serial loop would wait a full memory
  // latency per entry)
  for (int64_t i0 = 0; pre_lds && i0 < M; i0 += 8 * kRS) {
    uint32_t kk[8];
    int32_t vv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = i0 + tid + (int64_t)u * kRS;
      kk[u] = 0u; vv[u] = 0;
      if (i < M) {
        int lo = 0, hi = nblocks - 1;  // last block with s_bpre <= i (it holds >= 1 entry)
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (s_bpre[mid] <= i) lo = mid; else hi = mid - 1;
        }
        const int64_t src = (int64_t)lo * kRS + (i - s_bpre[lo]);
        kk[u] = d.keys_in[src];
        vv[u] = d.vals_in[src];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = i0 + tid + (int64_t)u * kRS;
      if (i < M) {
        if (in_lds) { lk[0][i] = kk[u]; lv[0][i] = vv[u]; }
        else { kb[0][i] = kk[u]; vb[0][i] = vv[u]; }
      }
    }
  }
  for (int b = tid; !pre_lds && b < nblocks; b += kRS) {
    const int c = d.bcnt[b];
    const int o = d.bpre[b];
    const uint32_t* ks = d.keys_in + (int64_t)b * kRS;
    const int32_t* vs = d.vals_in + (int64_t)b * kRS;
    for (int j0 = 0; j0 < c; j0 += 8) {
      uint32_t kk[8];
      int32_t vv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u < c ? j0 + u : c - 1;
        kk[u] = ks[j];
        vv[u] = vs[j];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (j0 + u < c) { kb[0][o + j0 + u] = kk[u]; vb[0][o + j0 + u] = vv[u]; }
    }
  }
  __syncthreads();
  constexpr int NW = kRS / 64;
  const int64_t s0 = M * w / NW, s1 = M * (w + 1) / NW;
  if (in_lds) {  // LDS -> LDS passes, the last one LDS -> HBM
    for (int p = 0; p + 1 < passes; ++p) rsort_pass<kRsuLds>(lk[p & 1], lv[p & 1], lk[(p + 1) & 1], lv[(p + 1) & 1], 8 * p, s0, s1, wc, hb);
    rsort_pass<kRsuLds>(lk[(passes - 1) & 1], lv[(passes - 1) & 1], d.keys_out, d.vals_out, 8 * (passes - 1), s0, s1, wc, hb);
  } else {
    for (int p = 0; p < passes; ++p) {  // buffer (passes - p) & 1 is keys_out / vals_out: the last pass lands there
      const bool src_out = ((passes - p) & 1) == 0;
      rsort_pass<8>(src_out ? d.keys_out : d.keys_tmp, src_out ? d.vals_out : d.vals_tmp, src_out ? d.keys_tmp : d.keys_out,
                 src_out ? d.vals_tmp : d.vals_out, 8 * p, s0, s1, wc, hb);
    }
  }
}

// ---------------------------------------------------------------------------
// Multi-workgroup sort of the mixed RIGHT events (many reads: K_rsort's one
// workgroup took 88 us at C3's 19k events, all of it latency).  K_rsplit gave
// every event a slot within its gap (atomics: any order); K_rscan scans the
// per-gap counts (two launches: block sums, then block scans with the sum of
// the blocks before), K_rscatter puts every event at rsl[gap] + slot, and
// K_rsegsort restores read order inside each gap (a wave's bitonic sort of up
// to 64 reads).  A gap with more than 64 events, or few events overall, sends
// the launch to K_rsort instead (path word rsflag[0]: 1 = this path).
// ---------------------------------------------------------------------------
constexpr int64_t kRsortMultiBlocks = 512;      // K_rsplit blocks (of 1024 reads) above which the plan takes this path
constexpr int kScanPer = 8;                     // gaps per thread of K_rscan
constexpr int kScanBlk = 1024 * kScanPer;       // gaps per K_rscan block
constexpr int kSegMax = 64;

__global__ __launch_bounds__(1024) void K_rscan1(Dev d) {
  __shared__ int32_t s_s[16], s_m[16];
  const int64_t g0 = (int64_t)blockIdx.x * kScanBlk + (int64_t)threadIdx.x * kScanPer;
  int32_t sum = 0, mx = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int32_t c = g0 + k <= d.G ? d.gcnt[g0 + k] : 0;
    sum += c;
    mx = c > mx ? c : mx;
  }
  sum = wave_sum(sum);
  for (int o = 32; o; o >>= 1) { const int32_t y = __shfl_xor(mx, o, 64); mx = y > mx ? y : mx; }
  const int w = threadIdx.x >> 6;
  if (lane() == 0) { s_s[w] = sum; s_m[w] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t t = 0, m = 0;
    for (int k = 0; k < 16; ++k) { t += s_s[k]; m = s_m[k] > m ? s_m[k] : m; }
    d.rsflag[4 + 2 * blockIdx.x] = t;
    d.rsflag[5 + 2 * blockIdx.x] = m;
  }
}

__global__ __launch_bounds__(1024) void K_rscan2(Dev d, int32_t nblk_scan) {
  __shared__ int32_t s_w[16];
  __shared__ int32_t s_pre, s_tot, s_max;
  const int tid = threadIdx.x, l = lane(), w = tid >> 6;
  if (tid < 64) {  // blocks before this one, and the totals
    int32_t pre = 0, tot = 0, mx = 0;
    for (int k = tid; k < nblk_scan; k += 64) {
      const int32_t c = d.rsflag[4 + 2 * k], m = d.rsflag[5 + 2 * k];
      tot += c;
      if (k < (int)blockIdx.x) pre += c;
      mx = m > mx ? m : mx;
    }
    pre = wave_sum(pre);
    tot = wave_sum(tot);
    for (int o = 32; o; o >>= 1) { const int32_t y = __shfl_xor(mx, o, 64); mx = y > mx ? y : mx; }
    if (tid == 0) { s_pre = pre; s_tot = tot; s_max = mx; }
  }
  __syncthreads();
  const int64_t g0 = (int64_t)blockIdx.x * kScanBlk + (int64_t)tid * kScanPer;
  int32_t c[kScanPer], sum = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) { c[k] = g0 + k <= d.G ? d.gcnt[g0 + k] : 0; sum += c[k]; }
  const int inc = wave_scan_i32(sum);
  if (l == 63) s_w[w] = inc;
  __syncthreads();
  int32_t run = s_pre + inc - sum;
  for (int k = 0; k < w; ++k) run += s_w[k];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (g0 + k <= d.G) d.rsl[g0 + k] = run;  // (K_rstart writes the same values again)
    run += c[k];
  }
  if (blockIdx.x == 0 && tid == 0) {
    const bool multi = s_tot > kSortLds && s_max <= kSegMax;
    d.rsflag[0] = multi ? 1 : 0;
    d.status[MPC_ST_RSORT_PATH] = multi ? 1u : 2u;
    if (multi) d.status[MPC_ST_MIXED] = (uint32_t)s_tot;
  }
}

__global__ __launch_bounds__(kRS) void K_rscatter(Dev d) {
  if (d.rsflag[0] != 1) return;
  const int64_t b = blockIdx.x;
  const int c = d.bcnt[b];
  if ((int)threadIdx.x >= c) return;
  const int64_t o = b * kRS + threadIdx.x;
  const uint32_t g = d.keys_in[o];
  const int64_t pos = (int64_t)d.rsl[g] + d.kslot[o];
  d.keys_out[pos] = g;
  d.vals_out[pos] = d.vals_in[o];
}

// one wave per gap: its (<= 64) reads in ascending order, bitonic over the lanes
__global__ __launch_bounds__(256) void K_rsegsort(Dev d) {
  if (d.rsflag[0] != 1) return;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g > d.G) return;
  const int32_t c = d.gcnt[g];
  if (c < 2) return;  // (wave-uniform)
  const int l = lane();
  const int64_t a0 = d.rsl[g];
  int32_t v = l < c ? d.vals_out[a0 + l] : INT32_MAX;
  for (int k = 2; k <= 64; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int32_t y = __shfl_xor(v, j, 64);
      const bool up = (l & k) == 0, low = (l & j) == 0;
      v = (low == up) ? (v < y ? v : y) : (v > y ? v : y);
    }
  }
  if (l < c) d.vals_out[a0 + l] = v;
}

// rsl[g] = #mixed RIGHT events of this shard with gap < g; rpos[local read] =
// its position in the shard's sorted list (so consumers need no search).  One
// shard: right_start = rsl, roff = 0, and the RIGHT length of run t + g (the run
// that this event closes) is filled here.  Several: per-gap counts for the
// exchange (K_runs / K_runR).
__global__ __launch_bounds__(256) void K_rstart(Dev d) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t M = d.status[MPC_ST_MIXED];
  if (t <= d.G) {
    const int32_t v = (int32_t)lower_bound_u32(d.keys_out, 0, M, (uint32_t)t);
    d.rsl[t] = v;
    if (d.n_shards == 1) { d.right_start[t] = v; d.roff[t] = 0; }
    if (t < d.G) d.rcnt[t] = (int32_t)lower_bound_u32(d.keys_out, 0, M, (uint32_t)t + 1) - v;
  }
  if (t < M) {
    const uint32_t g = d.keys_out[t];
    const int64_t rg = d.vals_out[t];
    const int64_t lr = rg - d.read_offset;
    if (lr >= 0 && lr < d.N) d.rpos[lr] = (int32_t)t;
    if (d.n_shards == 1) d.runR[t + g] = d.rlen[rg];
  }
}

// Several shards: global right_start and roff from all shards' per-gap counts:
// 1024 gaps per block, the blocks' sums chained by a decoupled look-back
// (K_layout's status words, which it re-tags with its own epoch later in the
// step; one workgroup over all gaps took C2 x 8 shards 18 us)
constexpr int kRunsGB = 1024;
__global__ __launch_bounds__(kRunsGB) void K_runs(Dev d, uint32_t epoch) {
  __shared__ int32_t s_w[kRunsGB / 64];
  __shared__ int64_t s_pre;
  const int l = lane(), w = threadIdx.x >> 6;
  const int64_t b = blockIdx.x;
  const int64_t g = b * kRunsGB + threadIdx.x;
  int32_t tot = 0, below = 0;
  if (g < d.G)
    for (int k = 0; k < d.n_shards; ++k) {
      const int32_t c = d.rcnt_all[(int64_t)k * d.G + g];
      tot += c;
      below += k < d.shard ? c : 0;
    }
  const int inc = wave_scan_i32(tot);
  if (l == 63) s_w[w] = inc;
  __syncthreads();
  int32_t wpre = 0, bt = 0;
  for (int k = 0; k < kRunsGB / 64; ++k) {
    wpre += k < w ? s_w[k] : 0;
    bt += s_w[k];
  }
  if (w == 0) {
    int64_t pre;
    lookback<1, MPC_LOOKBACK_U>(reinterpret_cast<uint64_t*>(d.bsum), b, (uint64_t)(epoch & 0x3fffffffu) << 32, &bt, &pre,
                                &d.status[MPC_ST_FLAGS]);
    if (l == 0) s_pre = pre;
  }
  __syncthreads();
  if (g <= d.G) {
    d.right_start[g] = (int32_t)(s_pre + wpre + inc - tot);
    d.roff[g] = below;
  }
}

// Several shards: RIGHT length of the run each of this shard's mixed RIGHT
// events closes, in the global run index space (exchange: MAX over shards).
__global__ __launch_bounds__(256) void K_runR(Dev d) {
  const int64_t nml = d.rsl[d.G];
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nml; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = d.keys_out[t];
    const int64_t run = (int64_t)d.right_start[g] + g + d.roff[g] + (t - d.rsl[g]);
    d.runR[run] = d.rlen[d.vals_out[t]];
  }
}

// Global run index of a LEFT event of (this shard's) global read rg at global
// gap g: runs of gap g are [right_start[g] + g, right_start[g+1] + g + 1); run
// k precedes the k-th mixed RIGHT event of the gap, k = RIGHT events of lower
// shards + this shard's RIGHT events of earlier reads.
__device__ __forceinline__ int64_t run_left(const int32_t* rs, const int32_t* rsl, const int32_t* roff,
                                            const int32_t* vals_out, int64_t g, int64_t rg) {
  const int64_t a = rsl[g], b = rsl[g + 1];
  int64_t k = roff[g];
  if (b > a) k += lower_bound_i32(vals_out, a, b, (int32_t)rg) - a;
  return rs[g] + g + k;
}

// ---------------------------------------------------------------------------
// Bucketed event work units.  K_parse leaves, per parse workgroup, its
// insertion events counting-sorted into buckets of 16 gaps.  Entries of the
// host table `bc` are (sample, bucket, chunk of <= 256 parse workgroups);
// K_units cuts every entry's events into units of <= kUnit events (hot
// buckets become many units) and appends them to one list.
// ---------------------------------------------------------------------------
constexpr int kUB = 1024;             // threads of K_ins and of K_left's default geometry
// K_left: interpolation probes before the binary search of a gap's staged
// RIGHT reads (ranges over 16); off: bit-exact, C3 +9 us, C4 +13 us, C2 / C5 +-2 us
// (profiles/r06_experiments/k_left_search_ablations.txt)
#ifndef MPC_LEFT_INTERP
#define MPC_LEFT_INTERP 0
#endif

constexpr int kLeftVals = 4096;       // mixed RIGHT reads of a bucket staged in K_left's LDS
constexpr int kEPT = 16;         // events per thread per unit (loads batched)
constexpr int kUnit = kUB * kEPT;     // events per work unit (K_left<kUB>; K_left<512>: half)

struct UnitArgs {
  const int4* bc;  // {sample, bucket, pw0, pw1}
  const int32_t* n_of; const int32_t* gbase;
  const int32_t* bk_cnt; int4* units; uint32_t* status;  // units: 2 int4 per unit (see load_unit)
  int64_t n_bc, units_cap;
  int32_t nbs;
  int32_t unit;  // pages per work unit (K_left's threads x kEPT / 64: one page per wave and step)
};

// kUE consecutive table entries per wave (one wave per entry at a time), one
// add to the unit counter per block: a single counter word serializes its
// atomics (~90 per us), and C5 has 45k entries
constexpr int kUE = 4;
constexpr int kUnitEntriesPerBlock = (kRS / 64) * kUE;
__device__ __forceinline__ void units_block(const UnitArgs& a, int64_t blk) {
  __shared__ int32_t s_wu[kRS / 64];
  __shared__ uint32_t s_ubase;
  const int l = lane(), w = threadIdx.x >> 6;
  const int64_t ent0 = blk * kUnitEntriesPerBlock + (int64_t)w * kUE;
  int ts[kUE], nus[kUE], wsum = 0;
  int4 bcs[kUE];
#pragma unroll
  for (int e = 0; e < kUE; ++e) {
    const int64_t ent = ent0 + e;
    int t = 0;
    bcs[e] = make_int4(0, 0, 0, 0);
    if (ent < a.n_bc) {  // wave-uniform
      const int4 bc = a.bc[ent];
      bcs[e] = bc;
      for (int pw = bc.z + l; pw < bc.w; pw += 64) t += (a.bk_cnt[(int64_t)pw * a.nbs + bc.y] + kPgEv - 1) / kPgEv;
      t = wave_sum(t);  // the entry's pages
    }
    ts[e] = t;
    nus[e] = (t + a.unit - 1) / a.unit;
    wsum += nus[e];
  }
  if (l == 0) s_wu[w] = wsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int k = 0; k < kRS / 64; ++k) { const int v = s_wu[k]; s_wu[k] = tot; tot += v; }
    s_ubase = tot ? atomicAdd(&a.status[MPC_ST_UNITS], (uint32_t)tot) : 0u;
  }
  __syncthreads();
  int64_t u0 = (int64_t)s_ubase + s_wu[w];
#pragma unroll
  for (int e = 0; e < kUE; ++e) {
    const int nu = nus[e];
    if (nu == 0) continue;
    if (u0 + nu > a.units_cap) {
      if (l == 0) atomicOr(&a.status[MPC_ST_FLAGS], DE_INTERNAL);
      return;
    }
    const int n = a.n_of[bcs[e].x], gb = a.gbase[bcs[e].x];
    for (int i = l; i < nu; i += 64) {
      const int e0 = i * a.unit;
      a.units[2 * (u0 + i)] = bcs[e];
      a.units[2 * (u0 + i) + 1] = make_int4(e0, ts[e] - e0 < a.unit ? ts[e] - e0 : a.unit, n, gb);
    }
    u0 += nu;
  }
}

// One launch for two independent jobs after the parse: blocks [0, nrb) split
// the RIGHT events (one read per thread), the rest cut the insertion work
// units (one table entry per wave).  Block-uniform branch.
__global__ __launch_bounds__(kRS) void K_rsplit_units(Dev d, UnitArgs ua, int32_t nrb) {
  if ((int32_t)blockIdx.x < nrb) rsplit_block(d, blockIdx.x);
  else units_block(ua, (int64_t)blockIdx.x - nrb);
}

struct UnitView { int smp, bucket, p0, np, n, gb, g0, gl, nsl; };
// A unit record (2 int4, written by units_block): {sample, bucket, pw0, pw1},
// {p0, np, n, gbase}: pages [p0, p0 + np) of the entry's page sequence (its
// slices -- parse workgroups pw0.. -- in order, each slice's pages as its list
// in pg_list holds them: global page numbers, all full but the last).  One
// round trip loads, per slice, its events, its list base and its workgroup's
// first read, and the bucket's per-gap tables (global run range, this shard's
// sorted-RIGHT range); a block scan gives the slices' first pages (s_ppre).
// Wave w then takes the unit's pages w, w + NW, ... (unit_page: the slice of a
// wave-uniform page by a search of s_ppre, its global page from pg_list), one
// event per lane.
__device__ __forceinline__ UnitView load_unit(const int4* units, int64_t u, const int32_t* bk_cnt,
                                              const int32_t* bk_off, const int64_t* rbase, int nbs,
                                              const int32_t* right_start, const int32_t* rsl, const int32_t* roff,
                                              const int4* pwork, int32_t* s_ppre, int32_t* s_cnt, int64_t* s_src,
                                              int32_t* s_r0, int32_t* s_wsum, int32_t* s_rs, int32_t* s_rsl,
                                              int32_t* s_roff) {
  const int4 ua = units[2 * u], ub = units[2 * u + 1];
  UnitView v;
  v.smp = ua.x; v.bucket = ua.y; v.p0 = ub.x; v.np = ub.y; v.n = ub.z; v.gb = ub.w; v.nsl = ua.w - ua.z;
  v.g0 = v.bucket * kBW;
  v.gl = v.g0 + kBW - 1 < v.n ? v.g0 + kBW - 1 : v.n;  // last gap of the bucket
  const int l = lane(), w = threadIdx.x >> 6;
  const int tid = (int)threadIdx.x;
  int cnt = 0, r0 = 0;
  int64_t src = 0;
  if (tid < 256) {  // <= 256 slices (parse workgroups) per table entry
    const int pw = ua.z + tid;
    if (pw < ua.w) {
      const int64_t slot = (int64_t)pw * nbs + v.bucket;
      cnt = bk_cnt[slot];
      src = rbase[pw] + bk_off[slot];  // the slice's page list in pg_list
      r0 = pwork[pw].y;
    }
  }
  const int64_t gg = (int64_t)v.gb + v.g0 + tid;
  if (tid <= v.gl + 1 - v.g0) { s_rs[tid] = right_start[gg]; s_rsl[tid] = rsl[gg]; s_roff[tid] = roff[gg]; }
  const int npg = (cnt + kPgEv - 1) / kPgEv;
  if (tid < 256) {
    const int inc = wave_scan_i32(npg);
    if (l == 63) s_wsum[w] = inc;
    s_ppre[tid] = inc - npg;
    s_cnt[tid] = cnt;
    s_src[tid] = src;
    s_r0[tid] = r0;
  }
  __syncthreads();
  if (tid < 256) {
    int wpre = 0;
    for (int k = 0; k < w; ++k) wpre += s_wsum[k];
    s_ppre[tid] += wpre;
  }
  __syncthreads();
  return v;
}
// page P of the unit's entry: its global page, events and slice's first read
struct UnitPage { uint32_t page; int cnt, r0; };
__device__ __forceinline__ UnitPage unit_page(const uint32_t* pg_list, const int32_t* s_ppre, const int32_t* s_cnt,
                                              const int64_t* s_src, const int32_t* s_r0, int P) {
  int j = 0;
#pragma unroll
  for (int h = 128; h >= 1; h >>= 1) j = s_ppre[j + h] <= P ? j + h : j;
  const int k = P - s_ppre[j];
  UnitPage r;
  r.page = pg_list[s_src[j] + k];
  r.cnt = min(kPgEv, s_cnt[j] - kPgEv * k);
  r.r0 = s_r0[j];
  return r;
}

// ---------------------------------------------------------------------------
// K_left: LEFT events -> per-run max length M (the slot layout's input; the
// bases themselves are tallied on rows once the layout is known).
//  * insertions: persistent workgroups over the work units; a unit's events
//    all lie in one kBW-gap bucket, so its (gap, run) maxima live in LDS (runs
//    k < kKMax; rarer runs go to HBM) and are flushed with atomics
//  * long insertions and upstream flanks (one per read, LEFT at gap tstart,
//    :303): grid-stride, wave-aggregated atomicMax (most reads share gap 0)
// ---------------------------------------------------------------------------
struct LeftArgs {
  const int64_t* up_off; const int32_t* sample; const int32_t* tstart;
  const int32_t* n_of; const int32_t* gbase;
  const int4* bc; const int4* units; const uint32_t* status;
  const uint32_t* ins_sorted; const uint32_t* pg_list; const int32_t* bk_cnt; const int32_t* bk_off;
  const int64_t* rbase;
  const int4* pwork;  // parse work table {sample, r0, r1, 0}: a slice's first read
  int64_t N, read_offset, ovf_cap;
  int32_t nbs;
  const int32_t* right_start; const int32_t* rsl; const int32_t* roff; const int32_t* vals_out;
  int32_t* M; uint32_t* runt;
  const Ovf* ovf; const uint32_t* ovf_cnt;
};

// Resident blocks per CU, so that the per-unit latency chains overlap:
// UB = 1024 at most 64 VGPRs, two 16-wave blocks (LDS ~57 KB each; C3 K_left
// 312 -> 227 us, C4 387 -> 286 us; 5 VGPRs spill); UB = 512 at most 80 VGPRs
// and a smaller RIGHT-read stage, three 8-wave blocks (C5 285 -> 218 us)
#ifdef MPC_LEFT_DIAG  // diagnostic builds only: K_left event paths (mpc_diag_left)
__device__ unsigned long long g_left_diag[8];
#endif
template <int UB>  // threads per block; work units of UB * kEPT events
__global__ __launch_bounds__(UB) __attribute__((amdgpu_waves_per_eu(UB == 1024 ? 8 : 6))) void K_left(LeftArgs a) {
  __shared__ int64_t s_key;
  __shared__ int32_t s_val;
  // strides padded to odd word counts: every gap of the bucket starts on a
  // different bank (unpadded, all gaps' run-0 counters shared 16 banks)
  constexpr int kMs = kKMax + 1, kTs = kKMax * 16 + 1;
  __shared__ uint32_t Ml[kBW * kMs];
  __shared__ int32_t s_rs[kBW + 1], s_rsl[kBW + 1], s_roff[kBW + 1];  // per gap of the bucket (K_left)
  __shared__ int32_t s_ppre[257], s_cnt[256], s_r0[256], s_wsum[4];   // per slice: first page, events, first read
  __shared__ int64_t s_src[256];                                      // ... and its page list in pg_list
  // 1024-thread blocks (C1-C4: few, large units) stage the unit's pages once,
  // all threads in parallel (one barrier); 512-thread blocks (C5: many small
  // units) look each page up in the wave that takes it (no barrier)
  constexpr bool kStage = UB == 1024;
  constexpr int kUP = kStage ? UB * kEPT / kPgEv : 1;
  __shared__ uint4 s_pe[kUP];             // staged: {global page, events, first read, 0}
  __shared__ uint32_t Tl[kBW * kTs];  // per (gap, run): inline bases [bi from the 3' end][code]
  // 512-thread blocks: a smaller stage, so three blocks fit a CU's LDS
  constexpr int kLV = UB == 512 ? 3072 : kLeftVals;
  __shared__ int32_t s_vals[kLV];         // the bucket's mixed RIGHT reads (vals_out), searched per event
  // (K_units raises DE_INTERNAL instead of overrunning the unit list)
#ifdef MPC_STAMPS_LEFT
  uint64_t st_acc[kStampSeg] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev;
  MPC_STAMP(st_prev);
#endif
  const int64_t nunits = (a.status[MPC_ST_FLAGS] & DE_INTERNAL) ? 0 : a.status[MPC_ST_UNITS];
  // 512-thread blocks (plans with many small buckets, C5): the tallies are
  // zeroed once and every unit flushes (and re-zeroes) only the runs it can
  // touch (s_kn), and short slices are searched for all events at once -- C5
  // K_left 215 -> 189 us; on the 1024-thread plans (C2-C4) the same code was
  // slower (profiles/r04_experiments/k_left_variants.txt: l_kfpa)
  constexpr bool kLean = UB == 512;
  __shared__ int32_t s_kn;
  if constexpr (kLean) {
    for (int k = threadIdx.x; k < kBW * kMs; k += blockDim.x) Ml[k] = 0;
    for (int k = threadIdx.x; k < kBW * kTs; k += blockDim.x) Tl[k] = 0;
  }
  for (int64_t u = blockIdx.x; u < nunits; u += gridDim.x) {
    if constexpr (kLean) {
      if (threadIdx.x == 0) s_kn = 0;  // ordered before its atomics by load_unit's barriers
    } else {
      for (int k = threadIdx.x; k < kBW * kMs; k += blockDim.x) Ml[k] = 0;
      for (int k = threadIdx.x; k < kBW * kTs; k += blockDim.x) Tl[k] = 0;
    }
    MPC_LSEG(0);
    const UnitView uv = load_unit(a.units, u, a.bk_cnt, a.bk_off, a.rbase, a.nbs, a.right_start, a.rsl, a.roff,
                                  a.pwork, s_ppre, s_cnt, s_src, s_r0, s_wsum, s_rs, s_rsl, s_roff);
    MPC_LSEG(1);
    const int n = uv.n;
    const int gb = uv.gb;
    const int g0 = uv.g0;
    uint32_t evs[kEPT];
    int32_t r0q[kEPT];  // the first read of each event's parse workgroup
    // all loads first (latency), then the tallies: wave w takes the unit's
    // pages w, w + NW, ... (wave-uniform: their slice searches and page numbers
    // are uniform), lane l the page's event l
    constexpr int NW = UB / 64;
    const int wv = uniform_i32((int)(threadIdx.x >> 6)), ln = lane();
    if constexpr (kStage) {
      for (int t = threadIdx.x; t < min(uv.np, kUP); t += UB) {
        const UnitPage pg = unit_page(a.pg_list, s_ppre, s_cnt, s_src, s_r0, uv.p0 + t);
        s_pe[t] = make_uint4(pg.page, (uint32_t)pg.cnt, (uint32_t)pg.r0, 0u);
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < kEPT; ++q) {
      const int t = wv + NW * q;
      evs[q] = ~0u;
      r0q[q] = 0;
      if (t < uv.np) {
        UnitPage pg;
        if constexpr (kStage) {
          const uint4 e = s_pe[t];
          pg.page = e.x; pg.cnt = (int)e.y; pg.r0 = (int)e.z;
        } else {
          pg = unit_page(a.pg_list, s_ppre, s_cnt, s_src, s_r0, uv.p0 + t);
        }
        r0q[q] = __builtin_amdgcn_readfirstlane(pg.r0);  // wave-uniform: SGPRs (K_left<1024> spilled 12 VGPRs)
        if (ln < pg.cnt) evs[q] = a.ins_sorted[(int64_t)pg.page * kPgEv + ln];
      }
    }
    // the run of an event at a mixed gap is a search of the gap's RIGHT reads:
    // stage the bucket's (contiguous in vals_out) in LDS, so no event waits on
    // a chain of dependent global loads
    const int32_t v0 = s_rsl[0], vn = s_rsl[uv.gl + 1 - g0] - v0;
    const bool vl = vn <= kLV;
    for (int k = threadIdx.x; vl && k < vn; k += blockDim.x) s_vals[k] = a.vals_out[v0 + k];
    if constexpr (kLean) {
      // LDS runs this unit can touch: an event at gap p has run k in
      // [roff, roff + its mixed RIGHT reads]; the flush covers runs < s_kn
      if (threadIdx.x < kBW && (int)threadIdx.x <= uv.gl - g0) {
        const int p = (int)threadIdx.x;
        atomicMax(&s_kn, min(s_rsl[p + 1] - s_rsl[p], kKMax - 1) + 1);
      }
    }
    MPC_LSEG(2);
    __syncthreads();
    MPC_LSEG(3);
#pragma unroll
    for (int q = 0; q < kEPT; ++q) {
      const uint32_t ev = evs[q];
      if (ev == ~0u) continue;
      const int gap = g0 + (int)((ev >> 10) & (kBW - 1));
      const int64_t g = (int64_t)gb + gap;
      const int32_t rg = (int32_t)a.read_offset + r0q[q] + (int32_t)(ev >> 16);  // global reads < 2^30
      const int L = (int)((ev >> 8) & 3u) + 1;
      const int p = gap - g0;
      // run of the event within its gap: this shard's runs of the gap start at
      // roff (the RIGHT events of lower shards); k counts from there
      const int32_t la = s_rsl[p], lb = s_rsl[p + 1];
      int32_t k = 0;
      if (lb > la) {
        if (vl) {  // 32-bit search of the staged RIGHT reads
          int lo = la - v0, hi = lb - v0;
          const int l0 = lo;
          if (MPC_LEFT_INTERP && hi - lo > 16) {
            // interpolation probes first (a gap's RIGHT reads are spread over
            // the batch's read indices): the range's end values, then up to two
            // probes at the interpolated index; [lo, hi) keeps
            // s_vals[< lo] < rg <= s_vals[>= hi], so any probe is exact
            int32_t vL = s_vals[lo], vH = s_vals[hi - 1];
            if (rg <= vL) {
              hi = lo;
            } else if (rg > vH) {
              lo = hi;
            } else {  // vL < rg <= vH
              int aL = lo, aH = hi - 1;
              lo = aL + 1;
              hi = aH;
#pragma unroll
              for (int it = 0; it < 2; ++it) {
                if (hi - lo <= 8) break;
                const float f = __fdividef((float)(rg - vL), (float)(vH - vL));
                const int g = min(max(aL + (int)(f * (float)(aH - aL)), lo), hi - 1);
                const int32_t vg = s_vals[g];
                if (vg < rg) { aL = g; vL = vg; lo = g + 1; } else { aH = g; vH = vg; hi = g; }
              }
            }
          }
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_vals[mid] < rg) lo = mid + 1; else hi = mid;
          }
          k += lo - l0;
        } else {
          k += lower_bound_i32(a.vals_out, la, lb, rg) - la;
        }
      }
      // the bases too, run-relative (LEFT: base bi from the 3' end lands on the
      // run's slot hi_run - 1 - bi, :37-62): K_ins maps them to rows after the layout
      // LDS slots: the shard's runs of the gap (as many as on one GPU); the
      // global run is s_rs[p] + g + roff + k
#ifdef MPC_LEFT_DIAG
      {  // [0] events [1] searched (mixed gap) [2] run k >= kKMax [3] sum of searched ranges [4] k >= 16 [5] k >= 32
        atomicAdd(&g_left_diag[0], 1ull);
        if (lb > la) { atomicAdd(&g_left_diag[1], 1ull); atomicAdd(&g_left_diag[3], (unsigned long long)(lb - la)); }
        if (k >= kKMax) atomicAdd(&g_left_diag[2], 1ull);
        if (k >= 16) atomicAdd(&g_left_diag[4], 1ull);
        if (k >= 32) atomicAdd(&g_left_diag[5], 1ull);
      }
#endif
      if (k < kKMax) {
        // the run's longest LEFT string: UB = 1024 takes it from the highest
        // slot holding a base at the flush (one LDS atomic less per event: C4
        // K_left 230 -> 220 us); UB = 512 (C5: +5 us that way) per event
        if constexpr (kLean) atomicMax(&Ml[p * kMs + k], (uint32_t)L);
        uint32_t* tp = Tl + p * kTs + k * 16;
#pragma unroll
        for (int j = 0; j < kInsInline; ++j)  // straight-line: bases j < L
          if (j < L) atomicAdd(tp + 4 * (L - 1 - j) + (int)((ev >> (2 * j)) & 3u), 1u);
      } else {
        const int64_t run = s_rs[p] + g + (int64_t)s_roff[p] + k;
        atomicMax(a.M + run, L);
        uint32_t* rt = a.runt + run * 16;
        for (int j = 0; j < L; ++j) atomicAdd(rt + 4 * (L - 1 - j) + (int)((ev >> (2 * j)) & 3u), 1u);
      }
    }
    MPC_LSEG(4);
    __syncthreads();
    MPC_LSEG(5);
    if constexpr (kLean) {  // runs k < s_kn of every gap (k-major), read and re-zeroed
      const int kn = s_kn;
      for (int q = threadIdx.x; q < kBW * kn; q += blockDim.x) {
        const int p = q & (kBW - 1), k = q / kBW;
        const uint32_t m = Ml[p * kMs + k];
        if (m) {
          atomicMax(a.M + s_rs[p] + (int64_t)gb + g0 + p + s_roff[p] + k, (int32_t)m);
          Ml[p * kMs + k] = 0;
        }
      }
      for (int q = threadIdx.x; q < kBW * kn * 16; q += blockDim.x) {  // contiguous per (gap, run)
        const int p = (q >> 4) & (kBW - 1), k = q / (kBW * 16);
        const uint32_t v = Tl[p * kTs + k * 16 + (q & 15)];
        if (v) {
          atomicAdd(a.runt + (s_rs[p] + (int64_t)gb + g0 + p + s_roff[p] + k) * 16 + (q & 15), v);
          Tl[p * kTs + k * 16 + (q & 15)] = 0;
        }
      }
      __syncthreads();
      MPC_LSEG(6);
      continue;
    }
    for (int q = threadIdx.x; q < kBW * kKMax * 16; q += blockDim.x) {  // contiguous per (gap, run)
      const int k = (q >> 4) % kKMax, p = (q >> 4) / kKMax;
      const uint32_t v = Tl[p * kTs + k * 16 + (q & 15)];
      if (v) {
        atomicAdd(a.runt + (s_rs[p] + (int64_t)gb + g0 + p + s_roff[p] + k) * 16 + (q & 15), v);
        atomicMax(&Ml[p * kMs + k], (uint32_t)((q & 15) >> 2) + 1u);  // slot bi holds a base: M > bi
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < kBW * kKMax; q += blockDim.x) {
      const int k = q % kKMax, p = q / kKMax;
      const uint32_t m = Ml[p * kMs + k];
      if (m) atomicMax(a.M + s_rs[p] + (int64_t)gb + g0 + p + s_roff[p] + k, (int32_t)m);
    }
    __syncthreads();
    MPC_LSEG(6);
  }
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  // the per-read parts start at the first block that had no unit (rotated
  // block index), so they run beside the unit blocks instead of after them
  const int64_t fb = ((int64_t)blockIdx.x + gridDim.x - nunits % gridDim.x) % gridDim.x;
  const int64_t tid = fb * blockDim.x + threadIdx.x;
  // long insertions
  const int64_t nov = *a.ovf_cnt < (uint32_t)a.ovf_cap ? *a.ovf_cnt : a.ovf_cap;
  for (int64_t t = tid; t < nov; t += nthreads) {
    const Ovf o = a.ovf[t];
    const int64_t g = (int64_t)a.gbase[a.sample[o.read]] + o.gap;
    atomicMax(a.M + run_left(a.right_start, a.rsl, a.roff, a.vals_out, g, a.read_offset + o.read), o.len);
  }
  // upstream flanks (block-uniform trips: block_atomic_max synchronizes the block)
  for (int64_t r0 = fb * blockDim.x; r0 < a.N; r0 += nthreads) {
    const int64_t r = r0 + threadIdx.x;
    int64_t run = 0;
    int32_t L = 0;
    bool ok = false;
    if (r < a.N) {
      const int64_t ul = a.up_off[r + 1] - a.up_off[r];
      const int s = a.sample[r];
      const int ts = a.tstart[r];
      if (ul > 0 && ts >= 0 && ts <= a.n_of[s]) {
        const int64_t g = (int64_t)a.gbase[s] + ts;
        run = a.right_start[g + 1] > a.right_start[g]
                  ? run_left(a.right_start, a.rsl, a.roff, a.vals_out, g, a.read_offset + r)
                  : (int64_t)a.right_start[g] + g;
        L = ul > 0x7fffffff ? 0x7fffffff : (int32_t)ul;
        ok = true;
      }
    }
    block_atomic_max(a.M, run, L, ok, &s_key, &s_val);
  }
#ifdef MPC_STAMPS_LEFT
  MPC_LSEG(7);
  const int64_t gw = (int64_t)blockIdx.x * (UB / 64) + (threadIdx.x >> 6);
  if (lane() < kStampSeg && gw < kStampWaves) {
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < kStampSeg; ++k) v = lane() == k ? st_acc[k] : v;
    g_stamps[gw * kStampSeg + lane()] = v;
  }
#endif
}

// ---------------------------------------------------------------------------
// Wrapped odd positions (negative target starts; WoEv).  An odd position that
// receives LEFT strings (upstream flanks :303, '+' insertions :81-87) or
// RIGHT strings (downstream flanks :323) through Python's negative index wrap
// grows a slot list like a gap's (:37-72), and its one-base writes -- the
// match or substitution of every read covering the reference base (:79, :96)
// -- are LEFT strings of length 1 in the same replay.  Its runs are split at
// its RIGHT strings in read order (a read's own LEFT strings there precede its
// RIGHT one; a read ending at n + i < 0 never reaches the base itself).
//   K_woprep       one workgroup: sorts the list by (position, read, kind);
//                  the positions, their runs, each string's run, the longest
//                  LEFT / the closing RIGHT string per run
//   K_wocover      one thread per read: walks its cs (:306-320) and counts its
//                  one-base write at every listed position it covers into the
//                  run it falls in
//   K_layout<true> replays each listed position's runs (F slots, F rows)
//   K_worows       the strings and the one-base counts onto those rows
// None of it runs in plans without negative starts (mpc_input.neg_reads).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wo_sort_key(const WoEv& e) {
  return ((uint64_t)(uint32_t)e.g << 32) | ((uint64_t)(uint32_t)e.read << 2) | (uint64_t)(uint32_t)e.type;
}
__device__ __forceinline__ int64_t wo_key_read(uint64_t k) { return (int64_t)((k >> 2) & 0x3fffffffu); }

// exclusive scan of x[0, n) in place by one workgroup; returns the total
__device__ int64_t block_scan_excl(int32_t* x, int64_t n, int32_t* s_w) {
  int64_t carry = 0;
  const int w = threadIdx.x >> 6, l = lane(), nw = (int)(blockDim.x >> 6);
  for (int64_t b0 = 0; b0 < n; b0 += blockDim.x) {
    const int64_t k = b0 + threadIdx.x;
    const int v = k < n ? x[k] : 0;
    const int inc = wave_scan_i32(v);
    if (l == 63) s_w[w] = inc;
    __syncthreads();
    int pre = 0, tot = 0;
    for (int j = 0; j < nw; ++j) { pre += j < w ? s_w[j] : 0; tot += s_w[j]; }
    if (k < n) x[k] = (int32_t)(carry + pre + inc - v);
    carry += tot;
    __syncthreads();
  }
  return carry;
}

// first listed position with g >= x among [0, np)
__device__ __forceinline__ int wo_lower(const WoPos* pos, int np, int64_t x) {
  int lo = 0, hi = np;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (pos[mid].g < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int32_t wo_len(const Dev& d, const WoEv& e) {
  if (e.type == kWoIns) return e.len;
  const int64_t* off = e.type == kWoUp ? d.up_off : d.down_off;
  const int64_t L = off[e.read + 1] - off[e.read];
  return L > 0x7fffffff ? 0x7fffffff : (int32_t)L;
}

__global__ __launch_bounds__(1024) void K_woprep(Dev d) {
  __shared__ int32_t s_w[16];
  const int64_t n = min<int64_t>((int64_t)d.status[MPC_ST_WRAP_EVENTS], d.wo_cap);
  if (n == 0) {
    if (threadIdx.x == 0) d.status[MPC_ST_WRAP_POS] = 0u;
    return;
  }
  int64_t P2 = 1;
  while (P2 < n) P2 <<= 1;
  uint64_t* key = d.wo_key;
  uint32_t* idx = d.wo_idx;
  for (int64_t k = threadIdx.x; k < P2; k += blockDim.x) {
    key[k] = k < n ? wo_sort_key(d.wo[k]) : ~0ull;
    idx[k] = (uint32_t)k;
  }
  __syncthreads();
  // bitonic sort of (key, idx): keys are distinct but for a read's '+' strings
  // at one position, which are LEFT strings of one run (any order)
  for (int64_t size = 2; size <= P2; size <<= 1)
    for (int64_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (int64_t t = threadIdx.x; t < P2 / 2; t += blockDim.x) {
        const int64_t lo = 2 * stride * (t / stride) + (t % stride), hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const uint64_t a = key[lo], b = key[hi];
        if ((a > b) == asc && a != b) {
          key[lo] = b; key[hi] = a;
          const uint32_t x = idx[lo]; idx[lo] = idx[hi]; idx[hi] = x;
        }
      }
      __syncthreads();
    }
  // positions: segments of equal g
  int32_t* tmp = d.wo_erun + d.wo_cap;
  auto starts = [&](int64_t k) { return k == 0 || (key[k] >> 32) != (key[k - 1] >> 32); };
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) tmp[k] = starts(k) ? 1 : 0;
  __syncthreads();
  const int64_t npos = block_scan_excl(tmp, n, s_w);  // tmp[k] = positions starting before k
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
    const bool st = starts(k);
    const int32_t p = st ? tmp[k] : tmp[k] - 1;
    if (st) { d.wo_pos[p].g = (int32_t)(key[k] >> 32); d.wo_pos[p].beg = (int32_t)k; }
    if (k == n - 1 || starts(k + 1)) d.wo_pos[p].end = (int32_t)(k + 1);
  }
  __syncthreads();
  // runs per position: one more than its RIGHT strings
  for (int64_t p = threadIdx.x; p < npos; p += blockDim.x) {
    int32_t m = 0;
    for (int32_t e = d.wo_pos[p].beg; e < d.wo_pos[p].end; ++e) m += (int32_t)(key[e] & 3u) == kWoDown;
    d.wo_pos[p].nrun = m + 1;
    tmp[p] = m + 1;
  }
  __syncthreads();
  block_scan_excl(tmp, npos, s_w);
  for (int64_t p = threadIdx.x; p < npos; p += blockDim.x) {
    WoPos& P = d.wo_pos[p];
    const int32_t run0 = tmp[p];
    P.run0 = run0;
    for (int32_t j = 0; j < P.nrun; ++j) {
      WoRun z;
      z.M = 0; z.R = 0; z.hiR = 0; z.loR = 0; z.C[0] = z.C[1] = z.C[2] = z.C[3] = 0u;
      d.wo_run[run0 + j] = z;
    }
    int32_t j = 0;
    for (int32_t e = P.beg; e < P.end; ++e) {
      d.wo_erun[e] = j;  // RIGHT strings before it: its run (a RIGHT string closes run j)
      const WoEv ev = d.wo[idx[e]];
      const int32_t L = wo_len(d, ev);
      WoRun& R = d.wo_run[run0 + j];
      if (ev.type == kWoDown) { R.R = L; ++j; }
      else if (L > R.M) R.M = L;
    }
  }
  if (threadIdx.x == 0) d.status[MPC_ST_WRAP_POS] = (uint32_t)npos;
}

// one thread per read: the read's one-base writes (:79 matches, :96
// substitutions) at the listed positions, counted per run
__device__ void wo_cover_read(const Dev& d, int np, int64_t r);
__global__ __launch_bounds__(256) void K_wocover(Dev d) {
  const int np = (int)d.status[MPC_ST_WRAP_POS];
  if (np == 0) return;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < d.N; r += (int64_t)gridDim.x * blockDim.x)
    wo_cover_read(d, np, r);
}
__device__ void wo_cover_read(const Dev& d, int np, int64_t r) {
  const int s = d.sample[r];
  const int64_t n = d.n_of[s], gb = d.gbase[s];
  const int pa = wo_lower(d.wo_pos, np, gb), pb = wo_lower(d.wo_pos, np, gb + n);
  if (pa == pb) return;
  const uint8_t* ref = d.ref + d.ref_off[s];
  auto hit = [&](int p, int code) {
    const WoPos P = d.wo_pos[p];
    int lo = P.beg, hi = P.end;  // the position's first string from a read >= r
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (wo_key_read(d.wo_key[mid]) < r) lo = mid + 1; else hi = mid;
    }
    const int32_t j = lo < P.end ? d.wo_erun[lo] : P.nrun - 1;
    atomicAdd(&d.wo_run[P.run0 + j].C[code], 1u);
  };
  // the tokenizer of :306-320: an operator applies to the operand gathered
  // after it when the next operator comes with a non-empty operand, the last
  // one unconditionally.  Data errors were flagged by K_parse: stop there.
  const int64_t b = d.cs_off[r], e = d.cs_off[r + 1];
  int64_t i = d.tstart[r], o0 = b, olen = 0;
  uint32_t op = 0;
  for (int64_t x = b;; ++x) {
    const bool end = x >= e;
    const uint32_t c = end ? 0u : d.cs[x];
    const bool sp = !end && (c == ':' || c == 'Z' || c == '+' || c == '-' || c == '*');
    if (!end && !sp) { ++olen; continue; }
    if (end || olen > 0) {
      if (op == ':') {
        int64_t m = 0;
        if (olen == 0) return;
        for (int64_t y = o0; y < o0 + olen; ++y) {
          const uint32_t dc = (uint32_t)d.cs[y] - 0x30u;
          if (dc > 9u) return;
          m = m * 10 + dc;
          if (m > (1ll << 40)) m = 1ll << 40;
        }
        const int64_t k0 = i < 0 ? 0 : i, k1 = i + m < n ? i + m : n;
        for (int p = k0 < k1 ? wo_lower(d.wo_pos, np, gb + k0) : pb; p < pb && d.wo_pos[p].g < gb + k1; ++p) {
          const int code = base_code_exact(ref[d.wo_pos[p].g - gb]);
          if (code >= 0) hit(p, code);  // (else KeyError: K_layout flags it)
        }
        i += m;
      } else if (op == '*') {
        if (olen == 0) return;
        if (i >= 0 && i < n) {
          const int p = wo_lower(d.wo_pos, np, gb + i);
          if (p < pb && d.wo_pos[p].g == gb + i) {
            const int code = code_upper(d.cs[o0 + olen - 1]);
            if (code >= 0) hit(p, code);
          }
        }
        i += 1;
      } else if (op == '-') {
        i += olen;
      } else if (op != '+' && op != 'Z') {
        return;  // unknown operator (:100-102)
      }
      if (i >= n) return;  // any later one-base write is past the end
    }
    if (end) break;
    op = c;
    o0 = x + 1;
    olen = 0;
  }
}

// ---------------------------------------------------------------------------
// Layout: replay of processBaseString_leftIndel / _rightIndel slot creation.
// Per gap the list grows at the front (LEFT, right-justified) and at the back
// (RIGHT, left-justified).  State: lo = slots prepended, hi = slots appended.
//   LEFT  len L : base bi -> absolute hi-1-bi ; lo = max(lo, L-hi)
//   RIGHT len R : base bi -> absolute -lo+bi  ; hi = max(hi, R-lo)
// Within a run of LEFT events hi is constant, so only the run's longest LEFT
// string matters (M); run k is closed by the gap's k-th mixed RIGHT event
// (length runR).  One thread per gap replays its runs; the row counts and the
// depth difference array are then scanned in the same launch (K_layout).
// ---------------------------------------------------------------------------
#ifndef MPC_LAYOUT_GAPS
#define MPC_LAYOUT_GAPS 256
#endif
constexpr int kGB = MPC_LAYOUT_GAPS;  // gaps per K_layout block (fewer blocks: a shorter look-back chain)

// K_layout = K_replay + K_assemble in ONE launch: the per-gap replay, then the
// row offsets and depths as block scans chained across blocks by a decoupled
// look-back (per block two 64-bit status words, rows and depth difference, each
// {flag, launch epoch, value}: flag 1 = the block's own sum, 2 = its inclusive
// prefix).  Blocks are dispatched in index order, so a block waits only on
// running or finished blocks; the spin is bounded (DE_INTERNAL, never a hang).
// The row capacity is checked per gap (rows that do not fit are not written);
// the last block sets ROWS_NEEDED and DE_CAP for the re-plan.
// WO: the plan lists wrapped odd positions (K_woprep); such a position after
// gap g is replayed here too and takes F rows instead of one.
template <bool WO>
__global__ __launch_bounds__(kGB) void K_layout(Dev d, uint32_t epoch) {
  __shared__ int32_t s_w[2][kGB / 64];
  __shared__ int64_t s_pre[2];
  const int64_t b = blockIdx.x;
  const int64_t nb = (d.G + kGB - 1) / kGB;
  const int64_t g = b * kGB + threadIdx.x;
  int32_t rc = 0, dv = 0;
  int32_t F = 1, wop = -1;  // rows of the odd position after the gap; its listed index
  int s = 0;
  int64_t p = 0;
  if (g < d.G) {
    const int64_t r0 = (int64_t)d.right_start[g] + g, r1 = (int64_t)d.right_start[g + 1] + g + 1;  // runs of gap g
    int32_t lo = 0, hi = 0;
    for (int64_t t = r0; t < r1; ++t) {
      d.hiR[t] = hi;                          // hi seen by the run's LEFT events
      const int32_t m = d.M[t];
      if (m - hi > lo) lo = m - hi;
      if (t + 1 < r1) {
        d.loR[t] = lo;                        // lo seen by the RIGHT event closing the run
        const int32_t R = d.runR[t];
        if (R - lo > hi) hi = R - lo;
      }
    }
    // RIGHT-only gaps: their flanks were not sorted; slot bi = base bi
    const int32_t mr = d.maxR[g];
    if (mr - lo > hi) hi = mr - lo;
    d.lo_f[g] = lo;
    int lo_s = 0, hi_s = d.S - 1;  // sample of gap g
    while (lo_s < hi_s) {
      const int mid = (lo_s + hi_s + 1) >> 1;
      if (d.gbase[mid] <= g) lo_s = mid; else hi_s = mid - 1;
    }
    s = lo_s;
    p = g - d.gbase[s];
    if constexpr (WO) {
      const int np = (int)d.status[MPC_ST_WRAP_POS];
      const int k = wo_lower(d.wo_pos, np, g);
      if (p < d.n_of[s] && k < np && d.wo_pos[k].g == g) {
        // lo / hi of the odd position over its runs; a run's one-base writes
        // are a LEFT string of length 1
        const WoPos P = d.wo_pos[k];
        int32_t wl = 0, wh = 0;
        for (int32_t j = 0; j < P.nrun; ++j) {
          WoRun& R = d.wo_run[P.run0 + j];
          const int32_t c1 = (R.C[0] | R.C[1] | R.C[2] | R.C[3]) != 0u ? 1 : 0;
          const int32_t m = R.M > c1 ? R.M : c1;
          R.hiR = wh;
          if (m - wh > wl) wl = m - wh;
          if (j + 1 < P.nrun) {
            R.loR = wl;
            if (R.R - wl > wh) wh = R.R - wl;
          }
        }
        F = wl + wh;
        wop = k;
        d.wo_pos[k].lo = wl;
        d.wo_pos[k].F = F;
      }
    }
    rc = lo + hi + (p < d.n_of[s] ? F : 0);  // rows of a gap = its slots + the odd position after it
    d.rowcnt[g] = rc;
    dv = d.diff[g];
  }
  const int w = threadIdx.x >> 6, l = lane();
  const int ir = wave_scan_i32(rc), id = wave_scan_i32(dv);
  if (l == 63) { s_w[0][w] = ir; s_w[1][w] = id; }
  __syncthreads();
  int32_t wr = 0, wd = 0, br = 0, bd = 0;
  for (int k = 0; k < kGB / 64; ++k) {
    if (k < w) { wr += s_w[0][k]; wd += s_w[1][k]; }
    br += s_w[0][k];
    bd += s_w[1][k];
  }
  const uint64_t tag = (uint64_t)(epoch & 0x3fffffffu) << 32;
  if (w == 0) {  // [2 nb] words: block b's rows word, diff word
    const int32_t own[2] = {br, bd};
    int64_t pre[2];
    lookback<2, MPC_LOOKBACK_U>(reinterpret_cast<uint64_t*>(d.bsum), b, tag, own, pre, &d.status[MPC_ST_FLAGS]);
    if (l == 0) { s_pre[0] = pre[0]; s_pre[1] = pre[1]; }
  }
  __syncthreads();
  const int64_t pre_r = s_pre[0], pre_d = s_pre[1];
  if (b == nb - 1 && threadIdx.x == 0) {
    const int64_t tot = pre_r + br;
    d.status[MPC_ST_ROWS_NEEDED] = (uint32_t)tot;
    if (tot > d.row_cap) atomicOr(&d.status[MPC_ST_FLAGS], DE_CAP);
  }
  if (g >= d.G) return;
  const int64_t rb = pre_r + wr + ir - rc;  // exclusive
  const int64_t dep = pre_d + wd + id;      // inclusive
  d.row_base[g] = (int32_t)rb;
  if (p == 0) d.srow[s] = (int32_t)rb;  // the consensus kernels' sample table (one load, no gbase chain)
  if (rb + rc > d.row_cap) return;      // does not fit: the last block flags DE_CAP (re-plan)
  const int64_t n = d.n_of[s];
  const int64_t nslots = (int64_t)rc - (p < n ? F : 0);
  if (nslots > 0) d.meta[rb] = 2;  // first slot of the gap
  if (p < n) {
    // each shard: its own reads' depth and substitutions (rows are summed over shards)
    // odd position p: depth = reads covering p with a match or substitution
    const uint32_t* sb = d.sub + g * 4;
    const uint32_t s0 = sb[0], s1 = sb[1], s2 = sb[2], s3 = sb[3];
    const int64_t match = dep - (int64_t)s0 - s1 - s2 - s3;
    uint32_t c[4] = {s0, s1, s2, s3};
    uint32_t fl = 0;
    if (match < 0) fl |= DE_INTERNAL;
    else if (match > 0) {
      const int rcode = base_code_exact(d.ref[d.ref_off[s] + p]);
      if (rcode < 0) fl |= DE_KEY;  // refarr base not in the dict (:61)
      else c[rcode] += (uint32_t)match;
    }
    if (fl) atomicOr(&d.status[MPC_ST_FLAGS], fl);
    if (WO && wop >= 0) d.wo_pos[wop].row0 = (int32_t)(rb + nslots);  // rows by K_worows
    else reinterpret_cast<uint4*>(d.rows)[rb + nslots] = make_uint4(c[0], c[1], c[2], c[3]);
    d.meta[rb + nslots] = 3;  // odd row, first slot of its position
  }
}

// ---------------------------------------------------------------------------
// Slot tallies of the even positions (:37-72 applied to insertion strings).
// A LEFT string's base bi (from the 3' end) lands on slot hi_run - 1 - bi of
// its gap, so K_left tallies the inline insertions per (run, bi, base) and
// K_ins maps every run onto its rows once the layout gives hi_run.  A
// grid-stride tail adds the long insertions (bases re-read from cs).
// ---------------------------------------------------------------------------

struct InsArgs {
  uint32_t* status; const int32_t* sample; const int32_t* gbase;
  int64_t read_offset, ovf_cap, G;
  const int32_t* right_start; const int32_t* rsl; const int32_t* roff; const int32_t* vals_out;
  const int32_t* row_base; const int32_t* lo_f; const int32_t* hiR;
  uint32_t* rows; const Ovf* ovf; const uint32_t* ovf_cnt; const uint8_t* cs;
  uint32_t* runt;
};

__global__ __launch_bounds__(kUB) void K_ins(InsArgs a) {
  const int l = lane();
  const int w = uniform_i32((int)(threadIdx.x >> 6));
  const bool cap = (a.status[MPC_ST_FLAGS] & DE_CAP) != 0;  // rows too small: only clear runt
  // inline insertions: K_left left their bases per run, indexed by the slot
  // from the run's right end; the layout gives the run's rows (one thread per
  // gap, over the gap's runs; LEFT base bi -> row row_base + lo_f + hi_run - 1 - bi)
  // wave-interleaved over the blocks (64 consecutive gaps per wave, consecutive
  // waves on different CUs): a few thousand gaps must not land on a few CUs
  // a gap with ONE run and no long insertions anywhere: its inline-insertion
  // rows get contributions from this thread only (rows are zero before K_ins;
  // K_flank adds after it), so a 16-byte store per non-empty slot replaces four
  // scattered atomics (C5: ~6 M atomics, 300 of K_ins' 330 us)
  const bool no_ovf = *a.ovf_cnt == 0;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t gw = (int64_t)w * gridDim.x + blockIdx.x; gw * 64 < a.G; gw += nwaves) {
    const int64_t g = gw * 64 + l;
    if (g >= a.G) continue;
    // this shard's runs of the gap (one GPU: all of them): a shard's LEFT
    // events fall into the runs its own reads span, [roff, roff + its mixed
    // RIGHT events of the gap]; K_left wrote nothing into the others
    const int64_t t0 = (int64_t)a.right_start[g] + g + a.roff[g], t1 = t0 + (a.rsl[g + 1] - a.rsl[g]) + 1;
    const int64_t top = (int64_t)a.row_base[g] + a.lo_f[g] - 1;
    const bool excl = no_ovf && t1 - t0 == 1;
    for (int64_t t = t0; t < t1; ++t) {
      uint4* rt = reinterpret_cast<uint4*>(a.runt + t * 16);
      uint4 v[4];
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) v[bi] = rt[bi];
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) rt[bi] = make_uint4(0u, 0u, 0u, 0u);  // runt is zero for the next K_left
      if (cap) continue;
      const int64_t rtop = top + a.hiR[t];
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) {
        uint32_t* row = a.rows + (rtop - bi) * 4;
        if (excl) {
          if (v[bi].x | v[bi].y | v[bi].z | v[bi].w) *reinterpret_cast<uint4*>(row) = v[bi];
          continue;
        }
        if (v[bi].x) atomicAdd(row + 0, v[bi].x);
        if (v[bi].y) atomicAdd(row + 1, v[bi].y);
        if (v[bi].z) atomicAdd(row + 2, v[bi].z);
        if (v[bi].w) atomicAdd(row + 3, v[bi].w);
      }
    }
  }
  if (cap) return;
  // long insertions (grid-stride over waves, LEFT like the short ones)
  const int64_t nov = *a.ovf_cnt < (uint32_t)a.ovf_cap ? *a.ovf_cnt : a.ovf_cap;
  for (int64_t t = (int64_t)blockIdx.x * (kUB / 64) + w; t < nov; t += (int64_t)gridDim.x * (kUB / 64)) {
    const Ovf o = a.ovf[t];
    const int64_t g = a.gbase[a.sample[o.read]] + o.gap;
    const int64_t run = run_left(a.right_start, a.rsl, a.roff, a.vals_out, g, a.read_offset + o.read);
    const int64_t rb = (int64_t)a.row_base[g] + a.lo_f[g] + a.hiR[run] - 1;
    for (int64_t bi = l; bi < o.len; bi += 64) {
      const int c = code_upper(a.cs[o.off + o.len - 1 - bi]);
      atomicAdd(a.rows + (rb - bi) * 4 + (c < 0 ? 0 : c), 1u);
    }
  }
}

// ---------------------------------------------------------------------------
// Flank tallies.  Every read's upstream flank (LEFT at gap tstart, :303 ->
// :37-62) and downstream flank (RIGHT at gap i_end, :323 -> :64-72) map
// LINEARLY onto rows once the layout is known: byte j of the flank goes to row
// rowstart + j, with
//   upstream   rowstart = row_base + lo_f + hi_run - L
//   downstream rowstart = row_base + lo_f - lo_at
// (hi_run / lo_at = 0 unless the gap is mixed).  Each WAVE owns 64
// consecutive reads (one per lane: its record, its two row starts); their
// flank bytes are contiguous, so the wave stages them in its LDS with 16-byte
// loads (both sides before any tally) and walks them in 256-byte segments,
// consecutive lanes on consecutive bytes.  The owner of a byte needs no block
// barrier: the lane of a flank starting in the segment marks its start byte
// in the wave's LDS row, and a max-scan over the segment (a byte's owner is
// the last flank starting at or before it) gives every byte its flank's lane,
// whose row offset one ds_bpermute fetches.  Rows of the hot gaps (voted per
// chunk of reads: for full-length reads gap 0 upstream, gap n downstream) are
// tallied in LDS windows, everything else with global atomics.  Block
// barriers: one per chunk (after its records load), and the flush (at the
// end, or when a block's chunk range crosses into another sample's gaps).
// ---------------------------------------------------------------------------
#ifndef MPC_FLANK_WAVES
#define MPC_FLANK_WAVES 8
#endif
constexpr int kFW = MPC_FLANK_WAVES;  // waves per block (64 reads each): C2's 200k reads fit one round of resident blocks
constexpr int kFWSmall = 2;     // ... when kFW-wave blocks would not give every CU one (C1)
constexpr int kWinRows = 256;   // LDS window rows per flank side
constexpr int kFSeg = 256;      // flank bytes per wave step (4 per lane)
constexpr int kFStageLd = 2;    // 16-byte loads per lane per staged side (2 KiB per wave)
constexpr int kFStage = kFStageLd * 1024 - 16;  // flank bytes per side staged per wave (C3: 64 reads x 0-40 B, mean 1280)
// K_flank blocks at most (two per CU): beyond, a block takes a contiguous range of
// chunks (C3: 1954 one-chunk blocks 135 us, 512 blocks of ~4 chunks 110 us)
#ifndef MPC_FLANK_BLOCKS_MAX
#define MPC_FLANK_BLOCKS_MAX 512
#endif

struct FlankArgs {
  uint32_t* status; const int32_t* sample; const int32_t* n_of; const int32_t* gbase;
  const int32_t* tstart; const int32_t* i_end;
  const int64_t* up_off; const uint8_t* up; const int64_t* down_off; const uint8_t* down;
  const int32_t* right_start; const int32_t* rsl; const int32_t* roff; const int32_t* vals_out; const int32_t* rpos;
  const int32_t* row_base; const int32_t* lo_f; const int32_t* hiR; const int32_t* loR;
  uint32_t* rows;
  int64_t N, read_offset;
};

// dict code of an exact-case base (flanks are upper-cased at ingest, :270):
// h = (c >> 1) & 3 is a perfect hash A0 C1 T2 G3 on "ACTG", bit-swapped to A0 T1 C2 G3
__device__ __forceinline__ int code_exact(uint32_t c) {
  const uint32_t h = (c >> 1) & 3u;
  const uint32_t expect = (0x47544341u >> (8 * h)) & 0xffu;
  const int code = (int)(((h & 1u) << 1) | (h >> 1));
  return c == expect ? code : -1;
}

// gap of read r's flank on one side (-1: empty flank or no row), for the window vote
__device__ __forceinline__ int32_t flank_gap(const FlankArgs& a, int64_t r, int side) {
  const int64_t* off = side ? a.down_off : a.up_off;
  if (off[r + 1] <= off[r]) return -1;
  const int s = a.sample[r];
  const int x = side ? a.i_end[r] : a.tstart[r];
  return (x >= 0 && x <= a.n_of[s]) ? a.gbase[s] + x : -1;
}

template <int NW, bool MULTI>  // waves per block; blocks take several chunks (grid capped)
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(MULTI || NW < kFW ? 4 : 6))) void K_flank(FlankArgs a) {
  // row r, code c at word 5 r + c: consecutive rows (the bytes of one flank,
  // on consecutive lanes) fall on distinct banks
  __shared__ uint32_t win[2][kWinRows * 5];
  __shared__ __attribute__((aligned(16))) uint32_t own[NW][kFSeg];  // per wave: 1 + lane of the flank starting at each byte
  __shared__ __attribute__((aligned(16))) uint8_t stg[NW][2][kFStageLd * 64 * 16];  // per wave and side: staged flank bytes
  // the windows' first rows: placed, and voted for the chunk (by chunk parity: a
  // wave still comparing chunk k's vote never sees chunk k + 1's)
  __shared__ int64_t s_w0[2], s_wn[2][2];
  if (a.status[MPC_ST_FLAGS] & (DE_CAP | DE_INTERNAL)) return;
  const int tid = threadIdx.x, l = lane();
  const int w = uniform_i32(tid >> 6);
  const int64_t tot = a.status[MPC_ST_ROWS_NEEDED];
  constexpr int64_t RB = NW * 64;
  for (int k = tid; k < 2 * kWinRows * 5; k += blockDim.x) (&win[0][0])[k] = 0;
  const int64_t nchunks = (a.N + RB - 1) / RB;
  // the block's chunks: a contiguous range (one sample's reads but at sample
  // boundaries), so its windows are flushed once per range, not per chunk --
  // every block's flush adds into the same hot rows (C3: 1954 one-chunk blocks)
  const int64_t cpb = MULTI ? (nchunks + gridDim.x - 1) / gridDim.x : 1;
  const int64_t ck0 = (int64_t)blockIdx.x * cpb, ck1 = ck0 + cpb < nchunks ? ck0 + cpb : nchunks;
  auto flush = [&]() {
    for (int side = 0; side < 2; ++side) {
      const int64_t w0 = s_w0[side];
      for (int k = tid; k < kWinRows * 4; k += blockDim.x) {
        const uint32_t v = win[side][(k >> 2) * 5 + (k & 3)];
        if (v) atomicAdd(a.rows + w0 * 4 + k, v);
      }
    }
  };
  uint32_t lerr = 0;
  int64_t lread = INT64_MAX;
  uint32_t* ow_w = own[w];
#pragma unroll 1
  for (int64_t ck = ck0; ck < ck1; ++ck) {
    if (tid < 2) {  // LDS window: rows of the gap most of the chunk's reads use (vote of 3)
      const int64_t c0 = ck * RB;
      const int64_t nr = a.N - c0 < RB ? a.N - c0 : RB;
      const int32_t x = flank_gap(a, c0, tid), y = flank_gap(a, c0 + nr / 2, tid), z = flank_gap(a, c0 + nr - 1, tid);
      const int32_t gw = (x == y || x == z) ? x : y;
      s_wn[ck & 1][tid] = gw >= 0 ? (int64_t)a.row_base[gw] : (int64_t)INT32_MIN;
      if (ck == ck0) s_w0[tid] = s_wn[ck & 1][tid];  // the first placement (windows zeroed above)
    }
    const int64_t rb = ck * RB + (int64_t)w * 64;  // the wave's first read
    const int64_t r = rb + l;
    const bool live = r < a.N;
    // per-read records: flank byte ranges and the row of byte 0 of each flank,
    // kept in 32 bits past this point (rows < 2^31; a flank longer than 2^31 - 1
    // bytes takes the HBM path below with its 64-bit offsets reloaded): fewer
    // VGPRs, more resident waves -- the other batches' kernels in flight get
    // the CUs K_flank does not hold
    int64_t off0 = 0, off1 = 0;
    int32_t L0 = 0, L1 = 0, rw0 = -1, rw1 = -1;
    if (live) {
      const int s = a.sample[r], ts = a.tstart[r], ie = a.i_end[r];
      off0 = a.up_off[r];
      off1 = a.down_off[r];
      const int64_t ul = a.up_off[r + 1] - off0, dl = a.down_off[r + 1] - off1;
      const int n = a.n_of[s];
      const int64_t gb = a.gbase[s];
      if (ul > 0 && ts >= 0 && ts <= n) {  // LEFT at gap tstart
        const int64_t g = gb + ts;
        int64_t hi = 0;
        if (a.right_start[g + 1] > a.right_start[g])
          hi = a.hiR[run_left(a.right_start, a.rsl, a.roff, a.vals_out, g, a.read_offset + r)];
        const int64_t rs = (int64_t)a.row_base[g] + a.lo_f[g] + hi - ul;
        if (rs >= 0 && rs + ul > tot) lerr |= DE_INTERNAL;
        else rw0 = (int32_t)rs;
      }
      if (dl > 0 && ie >= 0 && ie <= n) {  // RIGHT at gap i_end
        const int64_t g = gb + ie;
        int64_t lo_at = 0;
        if (a.right_start[g + 1] > a.right_start[g]) {
          const int64_t t = a.rpos[r];
          lo_at = a.loR[(int64_t)a.right_start[g] + g + a.roff[g] + (t - a.rsl[g])];
        }
        const int64_t rs = (int64_t)a.row_base[g] + a.lo_f[g] - lo_at;
        if (rs >= 0 && rs + dl > tot) lerr |= DE_INTERNAL;
        else rw1 = (int32_t)rs;
      }
      L0 = ul < INT32_MAX ? (int32_t)ul : INT32_MAX;
      L1 = dl < INT32_MAX ? (int32_t)dl : INT32_MAX;
    }
    __syncthreads();  // the vote is in; every wave is done with the previous chunk
    const int64_t* wn_ = s_wn[ck & 1];
    if (MULTI && (wn_[0] != s_w0[0] || wn_[1] != s_w0[1])) {  // (block-uniform) windows move: flush, clear, place
      flush();
      __syncthreads();
      for (int k = tid; k < 2 * kWinRows * 5; k += blockDim.x) (&win[0][0])[k] = 0;
      if (tid < 2) s_w0[tid] = wn_[tid];
      __syncthreads();
    }
    if (rb >= a.N) continue;
    const int last = a.N - 1 - rb < 63 ? (int)(a.N - 1 - rb) : 63;  // the wave's last read
    // the wave's flank bytes of both sides: [Bw, Bw + nb)
    const int64_t Bw0 = readlane64(off0, 0), nb0 = readlane64(off0 + L0, last) - Bw0;
    const int64_t Bw1 = readlane64(off1, 0), nb1 = readlane64(off1 + L1, last) - Bw1;
    // byte offsets in the wave's range (32-bit whenever the range is below 2^30)
    const int32_t xo0 = live ? (int32_t)(off0 - Bw0) : (int32_t)min(nb0, (int64_t)INT32_MAX);
    const int32_t xo1 = live ? (int32_t)(off1 - Bw1) : (int32_t)min(nb1, (int64_t)INT32_MAX);
    // stage [Bw + c0, Bw + c0 + kFStage) of a side in the wave's LDS (16-byte
    // loads from the aligned-down start).  The first stage of BOTH sides is
    // loaded before any tally: a load issued after a global atomic waits for
    // that atomic too (vmcnt retires in order), so loads between the atomics
    // serialized the wave on them)
    auto stage_load = [&](const uint8_t* src, int64_t B, int64_t nb, int64_t c0, uint4 (&v)[kFStageLd]) {
      const int64_t A = (B + c0) & ~(int64_t)15;
      const int64_t cnt = nb - c0 < kFStage ? nb - c0 : kFStage;
      const int n16 = (int)(((B + c0 - A) + cnt + 15) >> 4);
#pragma unroll
      for (int j = 0; j < kFStageLd; ++j)
        v[j] = l + 64 * j < n16 ? *reinterpret_cast<const uint4*>(src + A + 16 * (l + 64 * j)) : make_uint4(0u, 0u, 0u, 0u);
    };
    auto stage_store = [&](uint8_t* st, const uint4 (&v)[kFStageLd]) {
#pragma unroll
      for (int j = 0; j < kFStageLd; ++j) *reinterpret_cast<uint4*>(st + 16 * (l + 64 * j)) = v[j];
    };
    {
      uint4 v0[kFStageLd], v1[kFStageLd];
      if (nb0 > 0) stage_load(a.up, Bw0, nb0, 0, v0);
      if (nb1 > 0) stage_load(a.down, Bw1, nb1, 0, v1);
      if (nb0 > 0) stage_store(stg[w][0], v0);
      if (nb1 > 0) stage_store(stg[w][1], v1);
    }
#pragma unroll 1
    for (int side = 0; side < 2; ++side) {
      const uint8_t* src = side ? a.down : a.up;
      // (selects, not arrays indexed by side: a runtime index would put them in scratch)
      const int32_t L = side ? L1 : L0, frs = side ? rw1 : rw0, xo = side ? xo1 : xo0;
      const int64_t Bw = side ? Bw1 : Bw0, nb = side ? nb1 : nb0;
      if (nb <= 0) continue;
      const int32_t w032 = s_w0[side] >= 0 ? (int32_t)s_w0[side] : -(1 << 30);  // no window: never a hit
      uint32_t* wn = win[side];
      uint8_t* st = stg[w][side];
      if (nb >= (1 << 30)) {  // (huge flanks: every lane walks its own from HBM; rows < 2^31)
        const int64_t fo = live ? (side ? a.down_off[r] : a.up_off[r]) : 0;
        const int64_t fl = live ? (side ? a.down_off[r + 1] : a.up_off[r + 1]) - fo : 0;
        for (int64_t j = 0; frs >= 0 && j < fl; ++j) {
          const int code = code_exact(src[fo + j]);
          if (code < 0) { lerr |= DE_KEY; lread = r < lread ? r : lread; continue; }
          const int32_t row = (int32_t)(frs + j);
          const uint32_t wr = (uint32_t)(row - w032);
          if (wr < (uint32_t)kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
          else atomicAdd(a.rows + (int64_t)row * 4 + code, 1u);
        }
        continue;
      }
      // wave-relative byte x of lane l's flank: row = x + rowoff (rs + L <= tot < 2^31;
      // no row: rowoff = INT32_MIN, so every row of the flank is negative)
      const int32_t rowoff = (live && frs >= 0) ? frs - xo : INT32_MIN;
      const bool ne = live && L > 0;
      const int nb32 = (int)nb;
      int carry = 0;  // owner (1 + lane) of the previous byte group's last byte
#pragma unroll 1
      for (int c0 = 0; c0 < nb32; c0 += kFStage) {
        if (c0 > 0) {  // (a wave with more than kFStage bytes on this side)
          uint4 v[kFStageLd];
          stage_load(src, Bw, nb, c0, v);
          stage_store(st, v);
        }
        wave_sync_lds();
        const int sh = (int)((Bw + c0) & 15);
        const int c1 = nb32 - c0 < kFStage ? nb32 : c0 + kFStage;
#pragma unroll 1
        for (int S = c0; S < c1; S += kFSeg) {
          // lane l takes bytes S + 64 k + l (k < 4): consecutive lanes on
          // consecutive bytes, so a flank's bytes (consecutive rows) leave as few
          // 64-B atomic requests as they can (4 bytes per lane put every lane's
          // row atomic in a segment of its own: C3 K_flank +30 %)
          *reinterpret_cast<uint4*>(ow_w + 4 * l) = make_uint4(0u, 0u, 0u, 0u);
          wave_sync_lds();
          // non-empty flanks start on distinct bytes; only starts in this
          // stage (< c1): a later one would enter the carry into the next
          // stage ahead of the bytes before it
          if (ne && xo >= S && xo < S + kFSeg && xo < c1) ow_w[xo - S] = (uint32_t)(l + 1);
          wave_sync_lds();
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int x = S + 64 * k + l;
            const int inc = max(wave_scan_max_i32((int)ow_w[64 * k + l]), carry);
            carry = wave_last_i32(inc);
            // the row offset of the byte's flank (owner 0: bytes past the wave's range)
            const int32_t q = __builtin_amdgcn_ds_bpermute(4 * max(inc - 1, 0), rowoff);
            if (x >= c1 || inc == 0) continue;
            const int32_t row = x + q;
            if (row < 0) continue;  // flank without a row
            const int code = code_exact(st[sh + (x - c0)]);
            if (code < 0) {
              lerr |= DE_KEY;
              const int64_t rr = rb + inc - 1;
              lread = rr < lread ? rr : lread;
              continue;
            }
            const uint32_t wr = (uint32_t)(row - w032);
            if (wr < (uint32_t)kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
            else atomicAdd(a.rows + (int64_t)row * 4 + code, 1u);
          }
        }
        wave_sync_lds();  // (the stage is reloaded for the next kFStage bytes)
      }
    }
  }
  __syncthreads();
  if (ck1 > ck0) flush();
  if (lerr) {
    atomicOr(&a.status[MPC_ST_FLAGS], lerr);
    if (lread != INT64_MAX) atomicMin(&a.status[MPC_ST_FIRST_READ], (uint32_t)lread);
  }
}

// The rows of the listed wrapped odd positions (K_layout<true> placed them at
// row0, lo = the replayed slots prepended): a run's one-base writes go to slot
// lo + hiR - 1; a LEFT string's base bi from its 3' end to lo + hiR - 1 - bi
// (:55-61), a RIGHT string's base bi to lo - loR + bi (:67-71).  One wave per
// position (its runs) / per string (its bases on the lanes).
__global__ __launch_bounds__(256) void K_worows(Dev d) {
  const int np = (int)d.status[MPC_ST_WRAP_POS];
  if (np == 0 || (d.status[MPC_ST_FLAGS] & DE_CAP)) return;
  const int64_t n_ev = min<int64_t>((int64_t)d.status[MPC_ST_WRAP_EVENTS], d.wo_cap);
  const int l = lane();
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  for (int64_t p = gw; p < np; p += nwaves) {
    const WoPos P = d.wo_pos[p];
    for (int32_t j = l; j < P.nrun; j += 64) {
      const WoRun R = d.wo_run[P.run0 + j];
      uint32_t* row = d.rows + ((int64_t)P.row0 + P.lo + R.hiR - 1) * 4;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (R.C[c]) atomicAdd(row + c, R.C[c]);
    }
  }
  uint32_t err = 0;
  int64_t eread = INT64_MAX;
  for (int64_t e = gw; e < n_ev; e += nwaves) {
    const WoEv ev = d.wo[d.wo_idx[e]];
    const WoPos P = d.wo_pos[wo_lower(d.wo_pos, np, ev.g)];
    const WoRun R = d.wo_run[P.run0 + d.wo_erun[e]];
    const int64_t L = wo_len(d, ev);
    const uint8_t* src = ev.type == kWoIns ? d.cs + ev.src
                       : ev.type == kWoUp  ? d.up + d.up_off[ev.read]
                                           : d.down + d.down_off[ev.read];
    for (int64_t bi = l; bi < L; bi += 64) {
      int code;
      int64_t slot;
      if (ev.type == kWoDown) {
        code = code_exact(src[bi]);
        slot = (int64_t)P.lo - R.loR + bi;
      } else {
        const uint32_t c = src[L - 1 - bi];
        code = ev.type == kWoIns ? code_upper(c) : code_exact(c);
        slot = (int64_t)P.lo + R.hiR - 1 - bi;
      }
      if (code < 0) {  // KeyError (:61, :71); a '+' base K_parse flagged too
        err |= DE_KEY;
        eread = ev.read < eread ? ev.read : eread;
        continue;
      }
      atomicAdd(d.rows + ((int64_t)P.row0 + slot) * 4 + code, 1u);
    }
  }
  if (err) {
    atomicOr(&d.status[MPC_ST_FLAGS], err);
    atomicMin(&d.status[MPC_ST_FIRST_READ], (uint32_t)eread);
  }
}

// ---------------------------------------------------------------------------
// Consensus (Steps 5-6, :332-439)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int sample_of_row(const Dev& d, int64_t row) {
  int lo = 0, hi = d.S - 1;  // last sample whose first row <= row
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d.srow[mid] <= row) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// first row of every sample in LDS (kSmpLds samples; beyond that the global search)
constexpr int kSmpLds = 512;
__device__ __forceinline__ void load_sample_rows(const Dev& d, int32_t* srow) {
  for (int s = threadIdx.x; s < d.S && s < kSmpLds; s += blockDim.x) srow[s] = d.srow[s];
}
__device__ __forceinline__ int sample_of_row_lds(const Dev& d, const int32_t* srow, int64_t row) {
  if (d.S > kSmpLds) return sample_of_row(d, row);
  int lo = 0, hi = d.S - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (srow[mid] <= row) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// rows per thread of K_call: 1 while the grid is small (the kernel is
// latency-bound: more blocks), kCRBig for large pileups, where every block's
// max-depth atomic on the few maxdepth words serializes (C5: 5.7k blocks)
constexpr int kCRBig = 8;
constexpr int64_t kCallBlocksMax = 512;  // (the 70 kb parity case takes the kCRBig path)

// per slot: sorted(tuples in dict order, key=count)[::-1] -> top / second / tie -> N (:363-423).
// The stable descending sort of the reverse-dict-ordered (base, count) list
// is a descending sort of the keys count << 2 | dict index; bases with count
// 0 are not in the list (they sort last, and no positive count ties them).
// Branch-free: a 5-exchange sorting network (no register-indexed arrays: the
// insertion sort put them in scratch, K_call<8> spilled 18 VGPRs).
__device__ __forceinline__ uint4 call_slot(uint4 cv, double gtf, uint32_t* total_out) {
  const uint32_t total = cv.x + cv.y + cv.z + cv.w;  // A, T, C, G
  *total_out = total;
  if (total == 0) return make_uint4(0, 0, 0, 0);
  uint64_t k0 = ((uint64_t)cv.x << 2) | 0u, k1 = ((uint64_t)cv.y << 2) | 1u;
  uint64_t k2 = ((uint64_t)cv.z << 2) | 2u, k3 = ((uint64_t)cv.w << 2) | 3u;
  auto cx = [](uint64_t& a, uint64_t& b) {  // a >= b after
    const uint64_t hi = a > b ? a : b, lo = a > b ? b : a;
    a = hi; b = lo;
  };
  cx(k0, k1); cx(k2, k3); cx(k0, k2); cx(k1, k3); cx(k1, k2);
  const uint32_t c0 = (uint32_t)(k0 >> 2), c1 = (uint32_t)(k1 >> 2), c2 = (uint32_t)(k2 >> 2), c3 = (uint32_t)(k3 >> 2);
  // 'A' 'T' 'C' 'G' by dict index
  auto name = [](uint64_t k) -> uint32_t { return (0x47435441u >> (8 * (uint32_t)(k & 3u))) & 0xffu; };
  const uint32_t m = (c0 > 0) + (c1 > 0) + (c2 > 0) + (c3 > 0);  // c0 > 0 (total > 0)
  // ties of the first / second count (every tied count is positive: c0 > 0, and c1 is tested only when m >= 2)
  const uint32_t tie0 = c0 * (1u + (c1 == c0) + (c2 == c0) + (c3 == c0));
  const uint32_t tie1 = c1 * ((c0 == c1) + 1u + (c2 == c1) + (c3 == c1));
  const bool one = m == 1 || c0 > c1;
  uint32_t base = one ? name(k0) : 'N';
  const uint32_t count = one ? c0 : tie0;
  const bool two = m == 2 || c1 > c2;
  const uint32_t base2 = m <= 1 ? 'X' : (two ? name(k1) : 'N');
  const uint32_t count2 = m <= 1 ? 0u : (two ? c1 : tie1);
  const uint32_t chrom1 = base;
  if ((double)count < gtf * (double)count2) base = 'N';   // :421
  return make_uint4(base | (chrom1 << 8) | (base2 << 16) | (1u << 24), count, count2, total);
}

// calls of every row + max depth over slot 0 (:332-341); rows t + 256 k of the block
template <int kCR>  // (kCR rows in flight per thread: up to 128 VGPRs, no spills)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kCR > 1 ? 4 : 8))) void K_call(Dev d, int64_t R) {
  constexpr int kCB = 256 * kCR;  // rows per block
  __shared__ int32_t srow[kSmpLds];
  __shared__ int32_t s_blk[2], s_w[4];
  const bool cap = (d.status[MPC_ST_FLAGS] & DE_CAP) != 0;
  const int64_t need0 = cap ? 0 : (int64_t)d.status[MPC_ST_ROWS_NEEDED];
  const int64_t need = need0 < R ? need0 : R;
  load_sample_rows(d, srow);
  const int64_t b0 = (int64_t)blockIdx.x * kCB;
  __syncthreads();
  if (threadIdx.x < 2) {
    const int64_t rr = threadIdx.x == 0 ? b0 : (b0 + kCB < need ? b0 + kCB : need) - 1;
    s_blk[threadIdx.x] = rr >= 0 ? sample_of_row_lds(d, srow, rr) : 0;
  }
  uint4 cv[kCR];
  uint8_t mt[kCR];
#pragma unroll
  for (int k = 0; k < kCR; ++k) {  // all loads first (in bounds: rows < R), in parallel with the status word
    const int64_t row = b0 + threadIdx.x + 256 * k;
    cv[k] = row < R ? reinterpret_cast<const uint4*>(d.rows)[row] : make_uint4(0, 0, 0, 0);
    mt[k] = row < R ? d.meta[row] : 0;
  }
#pragma unroll
  for (int k = 0; k < kCR; ++k)
    if (b0 + threadIdx.x + 256 * k >= need) { cv[k] = make_uint4(0, 0, 0, 0); mt[k] = 0; }
  __syncthreads();
  int32_t dep[kCR];  // slot-0 depth of the row (:336), -1: none
#pragma unroll
  for (int k = 0; k < kCR; ++k) {
    const int64_t row = b0 + threadIdx.x + 256 * k;
    uint32_t total = 0;
    const uint4 out = call_slot(cv[k], d.gtf, &total);
    if (row < R) reinterpret_cast<uint4*>(d.res)[row] = out;
    dep[k] = (total > 0 && (mt[k] & 2u)) ? (int32_t)total : -1;
  }
  // one atomic per (block, sample): atomics on the few maxdepth words serialize
  for (int sb = s_blk[0]; sb <= s_blk[1]; ++sb) {  // block-uniform
    int32_t mx = -1;
#pragma unroll
    for (int k = 0; k < kCR; ++k) {
      const int64_t row = b0 + threadIdx.x + 256 * k;
      if (dep[k] > mx && (s_blk[0] == s_blk[1] || sample_of_row_lds(d, srow, row) == sb)) mx = dep[k];
    }
    mx = wave_max(mx);
    __syncthreads();
    if (lane() == 0) s_w[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int32_t m = max(max(s_w[0], s_w[1]), max(s_w[2], s_w[3]));
      // skip the atomic when a value of this run already covers m (the maxima
      // only grow; a cached read is never above the true one): all blocks'
      // atomics on the few maxdepth words serialize (C5: 6k blocks)
      if (m >= 0 && (uint32_t)m > __hip_atomic_load(d.maxdepth + sb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMax(d.maxdepth + sb, (uint32_t)m);
    }
  }
}

constexpr int kKB = 1024;  // rows per K_select block (4 per thread)

// keep[row] = emitted (:428) and the ordered compaction of the kept calls in
// ONE launch: every block publishes its kept count, then chains the counts of
// the blocks before it by a decoupled look-back (one 64-bit status word per
// block, {flag, launch epoch, value}: flag 1 = the block's own count, 2 = its
// inclusive prefix; wave 0 reads 64 predecessors per step and stops at the
// nearest prefix).  Blocks are dispatched in index order, so a block only ever
// waits on blocks that are already running or done; the spin is bounded anyway
// (DE_INTERNAL instead of a hang).  Replaces K_keep + K_emit (two launches and
// a read of every block count by every block).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void K_select(Dev d, int64_t R, uint32_t epoch) {
  __shared__ int32_t srow[kSmpLds];
  __shared__ uint32_t smd[kSmpLds];
  __shared__ int32_t s_w[4];
  __shared__ int64_t s_pre;
  load_sample_rows(d, srow);
  for (int s = threadIdx.x; s < d.S && s < kSmpLds; s += blockDim.x) smd[s] = d.maxdepth[s];
  const int64_t b = blockIdx.x;
  const int64_t nb = (R + kKB - 1) / kKB;
  const int64_t base = b * kKB + 4 * threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = base + k < R ? reinterpret_cast<const uint4*>(d.res)[base + k] : make_uint4(0, 0, 0, 0);
  __syncthreads();
  int c = 0;
  uint32_t bits = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (v[k].x >> 24) {
      const int s = sample_of_row_lds(d, srow, base + k);
      const double thr = (double)(s < kSmpLds ? smd[s] : d.maxdepth[s]) * d.mdf;  // :338
      if ((double)v[k].y > thr) { ++c; bits |= 1u << k; }  // :428
    }
  }
  const int w = threadIdx.x >> 6, l = lane();
  const int inc = wave_scan_i32(c);
  if (l == 63) s_w[w] = inc;
  __syncthreads();
  int32_t wpre = 0, bt = 0;
  for (int k = 0; k < 4; ++k) { wpre += k < w ? s_w[k] : 0; bt += s_w[k]; }
  const uint64_t tag = (uint64_t)(epoch & 0x3fffffffu) << 32;
  if (w == 0) {
    int64_t pr;
    lookback<1, MPC_LOOKBACK_U>(reinterpret_cast<uint64_t*>(d.ksum), b, tag, &bt, &pr, &d.status[MPC_ST_FLAGS]);
    if (l == 0) s_pre = pr;
  }
  __syncthreads();
  const int64_t pre = s_pre;
  int64_t pos = pre + wpre + inc - c;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (bits & (1u << k)) {
      const uint4 x = v[k];
      reinterpret_cast<uint4*>(d.calls)[pos++] = make_uint4(x.x & 0xffffffu, x.y, x.z, x.w);
    }
  // ncalls[s] = calls before the first row of sample s; ncalls[S] = all
  const int64_t b0 = b * kKB, all = pre + bt;
  for (int s = 0; s < d.S; ++s) {
    const int64_t rb = s < kSmpLds ? srow[s] : d.srow[s];
    if (rb >= b0 && rb < b0 + kKB && (rb - b0) / 4 == threadIdx.x) {
      int64_t q = pre + wpre + inc - c;
      for (int k = 0; k < (int)((rb - b0) & 3); ++k) q += (bits >> k) & 1u;
      d.ncalls[s] = (int32_t)q;
    }
    if (b == nb - 1 && threadIdx.x == 0 && rb >= nb * kKB) d.ncalls[s] = (int32_t)all;
  }
  if (b == nb - 1 && threadIdx.x == 0) d.ncalls[d.S] = (int32_t)all;
}

}  // namespace

// ===========================================================================
// Host side: plan, workspace layout, phases, C-ABI
// ===========================================================================
static thread_local std::string g_err;
// look-back launch epochs (K_layout, K_select): one process-wide sequence, so a
// status word another plan left in reused memory never carries a live tag; 0 is
// never used (zeroed words)
static uint32_t next_epoch() {
  static std::atomic<uint32_t> e{0};
  uint32_t v;
  do v = (e.fetch_add(1) + 1) & 0x3fffffffu; while (v == 0);
  return v;
}
static int fail(int code, const std::string& msg) { g_err = msg; return code; }

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) return fail(MPC_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct mpc_plan {
  mpc_input in;
  std::vector<int64_t> ref_len, read_begin;
  std::vector<int32_t> h_n, h_gbase;
  int64_t N = 0, Ng = 0, G = 0, row_cap = 0, runs_cap = 0, ins_cap = 0, ovf_cap = 0, pages_cap = 0;
  int64_t wo_cap = 0, wo_p2 = 1;  // strings into wrapped odd positions (negative starts): list bound, sort size
  int32_t S = 0;
  int32_t overrides = 0;  // MPC_OVR_* (experiment builds only)
  uint32_t sentinel = 0;
  int end_bit = 0;
  bool rsort_multi = false;  // mixed RIGHT events sorted by K_rscan / K_rscatter / K_rsegsort (many reads)
  size_t ws_bytes = 0;
  uint8_t* ws = nullptr;
  std::vector<int32_t> work_parse, work_bc, work_sub;  // int4 records
  std::vector<int32_t> work_subsum;                   // int4 {sample, window, first K_subs block, end}
  int subsum_rows = 0;                                // most K_subs blocks of one (sample, window)
  std::vector<int32_t> work_wave;                     // per parse workgroup: kMaxPW + 1 wave boundaries
  int32_t sub_wins = 0;                               // tally mode 3: substitution-event windows
  int64_t subev_cap = 0;
  int n_parse_wg = 0, parse_lds = 0, nbmax = 1, parse_win = 1024, parse_nw = 8;
  int defer_off = 0;                                  // K_parse deferred placement: its queues' LDS offset (0: off)
  int64_t n_bc = 0, units_cap = 0, max_wg_reads = 0;
  int32_t left_ub = 1024;  // K_left threads per block
  int32_t shard = 0, n_shards = 1;
  int tally_mode = 0;  // K_parse TM
  enum {
    B_STATUS, B_NOF, B_GBASE, B_IEND, B_PGOWN, B_INSSORT, B_BKCNT, B_BKOFF, B_RBASE, B_OVF, B_OVFCNT,
    B_HASLEFT, B_KIN, B_VIN, B_KOUT, B_VOUT, B_KTMP, B_VTMP, B_BCNT, B_BPRE, B_RLEN, B_RPOS, B_RSTART, B_RSLOC, B_ROFF, B_RCNT, B_RCNTALL,
    // MAXR, M, RUNR adjacent and in this order: one MAX exchange over their span (mpc.h)
    B_DIFF, B_SUB, B_MAXR, B_M, B_RUNR, B_HIR, B_LOR, B_LOF, B_ROWCNT, B_ROWBASE, B_BSUM, B_ROWS,
    B_META, B_RES, B_KEEP, B_KSUM, B_CALLS, B_NCALLS, B_MAXD, B_SROW, B_WPARSE, B_WBC, B_UNITS, B_RUNT,
    B_SUBEV, B_SUBCNT, B_WSUB, B_BKCUR, B_WWAVE, B_SUBSLAB, B_WSUBSUM, B_GCNT, B_KSLOT, B_RSFLAG, B_PGLIST,
    B_WOEV, B_WOKEY, B_WOIDX, B_WOERUN, B_WOPOS, B_WORUN, B_COUNT
  };
  size_t off[B_COUNT];
  size_t sz[B_COUNT];
  int64_t cnt[B_COUNT];
  bool bound = false;
  bool runt_dirty = true;  // runt may hold tallies: K_clear zeroes it (K_ins zeroes what it maps)
  Dev dev() const;
};


template <class T>
static T* at(const mpc_plan* p, int b) { return reinterpret_cast<T*>(p->ws + p->off[b]); }

Dev mpc_plan::dev() const {
  Dev d{};
  d.ref = in.ref; d.ref_off = in.ref_off; d.cs = in.cs; d.cs_off = in.cs_off; d.tstart = in.tstart;
  d.up = in.up; d.up_off = in.up_off; d.down = in.down; d.down_off = in.down_off; d.sample = in.sample;
  d.N = N; d.Ng = Ng; d.read_offset = in.read_offset; d.cs_base = in.cs_base; d.S = S; d.G = (int32_t)G;
  d.n_of = at<int32_t>(this, B_NOF); d.gbase = at<int32_t>(this, B_GBASE);
  d.status = at<uint32_t>(this, B_STATUS); d.i_end = at<int32_t>(this, B_IEND);
  d.ovf = at<Ovf>(this, B_OVF); d.ovf_cnt = at<uint32_t>(this, B_OVFCNT); d.ovf_cap = ovf_cap;
  d.hasleft = at<uint32_t>(this, B_HASLEFT); d.maxR = at<int32_t>(this, B_MAXR);
  d.keys_in = at<uint32_t>(this, B_KIN); d.vals_in = at<int32_t>(this, B_VIN);
  d.keys_out = at<uint32_t>(this, B_KOUT); d.vals_out = at<int32_t>(this, B_VOUT);
  d.keys_tmp = at<uint32_t>(this, B_KTMP); d.vals_tmp = at<int32_t>(this, B_VTMP);
  d.bcnt = at<int32_t>(this, B_BCNT); d.bpre = at<int32_t>(this, B_BPRE);
  d.gcnt = rsort_multi ? at<int32_t>(this, B_GCNT) : nullptr;
  d.kslot = rsort_multi ? at<int32_t>(this, B_KSLOT) : nullptr;
  d.rsflag = rsort_multi ? at<int32_t>(this, B_RSFLAG) : nullptr;
  d.rlen = at<int32_t>(this, B_RLEN); d.rpos = at<int32_t>(this, B_RPOS); d.right_start = at<int32_t>(this, B_RSTART);
  d.rsl = at<int32_t>(this, B_RSLOC); d.roff = at<int32_t>(this, B_ROFF); d.rcnt = at<int32_t>(this, B_RCNT);
  d.rcnt_all = at<int32_t>(this, B_RCNTALL); d.shard = shard; d.n_shards = n_shards;
  d.diff = at<int32_t>(this, B_DIFF); d.sub = at<uint32_t>(this, B_SUB);
  d.M = at<int32_t>(this, B_M); d.runR = at<int32_t>(this, B_RUNR); d.runt = at<uint32_t>(this, B_RUNT);
  d.hiR = at<int32_t>(this, B_HIR); d.loR = at<int32_t>(this, B_LOR);
  d.lo_f = at<int32_t>(this, B_LOF); d.rowcnt = at<int32_t>(this, B_ROWCNT); d.row_base = at<int32_t>(this, B_ROWBASE);
  d.bsum = at<int32_t>(this, B_BSUM);
  d.rows = at<uint32_t>(this, B_ROWS); d.meta = at<uint8_t>(this, B_META);
  d.row_cap = row_cap;
  d.res = at<uint32_t>(this, B_RES); d.keep = at<int32_t>(this, B_KEEP); d.ksum = at<int32_t>(this, B_KSUM);
  d.calls = at<uint32_t>(this, B_CALLS); d.ncalls = at<int32_t>(this, B_NCALLS); d.maxdepth = at<uint32_t>(this, B_MAXD);
  d.srow = at<int32_t>(this, B_SROW);
  d.wo = at<WoEv>(this, B_WOEV); d.wo_key = at<uint64_t>(this, B_WOKEY); d.wo_idx = at<uint32_t>(this, B_WOIDX);
  d.wo_erun = at<int32_t>(this, B_WOERUN); d.wo_pos = at<WoPos>(this, B_WOPOS); d.wo_run = at<WoRun>(this, B_WORUN);
  d.wo_cap = wo_cap; d.wo_p2 = wo_p2;
  return d;
}

static ParseArgs parse_args(const mpc_plan* p, const Dev& d) {
  ParseArgs a;
  a.cs = d.cs; a.cs_off = d.cs_off; a.tstart = d.tstart; a.up_off = d.up_off; a.down_off = d.down_off;
  a.n_of = d.n_of; a.gbase = d.gbase;
  a.work = reinterpret_cast<const int4*>(p->ws + p->off[mpc_plan::B_WPARSE]);
  a.wave_tab = at<const int32_t>(p, mpc_plan::B_WWAVE);
  a.cs_base = d.cs_base; a.ovf_cap = d.ovf_cap; a.read_offset = d.read_offset; a.n_reads = d.N;
  a.nbs = p->nbmax;
  a.i_end = d.i_end;
  a.ins_sorted = at<uint32_t>(p, mpc_plan::B_INSSORT);
  a.pg_own = at<uint32_t>(p, mpc_plan::B_PGOWN); a.pg_list = at<uint32_t>(p, mpc_plan::B_PGLIST);
  a.bk_cnt = at<int32_t>(p, mpc_plan::B_BKCNT); a.bk_off = at<int32_t>(p, mpc_plan::B_BKOFF);
  a.rbase = at<int64_t>(p, mpc_plan::B_RBASE); a.bk_cur = at<uint32_t>(p, mpc_plan::B_BKCUR);
  a.ovf = d.ovf; a.ovf_cnt = d.ovf_cnt; a.hasleft = d.hasleft; a.status = d.status;
  a.diff = d.diff; a.sub = d.sub;
  a.subev = at<uint16_t>(p, mpc_plan::B_SUBEV); a.subev_cnt = at<uint32_t>(p, mpc_plan::B_SUBCNT);
  a.subev_cap = p->subev_cap; a.sub_wins = p->tally_mode == 3 ? p->sub_wins : 0;
  a.wo = d.wo; a.wo_cap = d.wo_cap;
  a.defer_off = p->defer_off;
  return a;
}

// instantiated (tally mode, window) pairs; packed modes only with 1 and 2 KiB windows
template <bool NK>
static const void* parse_kernel_t(int tm, int win, bool s1) {
  if (tm == 4) return (const void*)K_parse<4, 1024, NK>;
  if (tm == 2) return win == 1024 ? (const void*)K_parse<2, 1024, NK> : (const void*)K_parse<2, 2048, NK>;
  if (tm == 3 && s1)
    return win == 1024 ? (const void*)K_parse<3, 1024, NK, true> : (const void*)K_parse<3, 2048, NK, true>;
  if (tm == 3) return win == 1024 ? (const void*)K_parse<3, 1024, NK> : (const void*)K_parse<3, 2048, NK>;
  if (win == 512) return tm ? (const void*)K_parse<1, 512, NK> : (const void*)K_parse<0, 512, NK>;
  if (win == 2048) return tm ? (const void*)K_parse<1, 2048, NK> : (const void*)K_parse<0, 2048, NK>;
  return tm ? (const void*)K_parse<1, 1024, NK> : (const void*)K_parse<0, 1024, NK>;
}
// the plan's K_parse: with the negative-start rounds only when it holds such reads
static const void* parse_kernel(const mpc_plan* p) {
  const bool s1 = MPC_SUB1 && p->tally_mode == 3 && p->sub_wins == 1;
  if (p->defer_off > 0)  // (planner: 2 KiB windows, tally mode 1 or 3 with s1, no negative starts)
    return p->tally_mode == 1 ? (const void*)K_parse<1, 2048, false, false, true>
                              : (const void*)K_parse<3, 2048, false, true, true>;
  return p->in.neg_reads > 0 ? parse_kernel_t<true>(p->tally_mode, p->parse_win, s1)
                             : parse_kernel_t<false>(p->tally_mode, p->parse_win, s1);
}
static void launch_subs(const mpc_plan* p, const Dev& d, hipStream_t st) {
  if (p->work_sub.empty()) return;
  SubsArgs a;
  a.work = at<const int4>(p, mpc_plan::B_WSUB); a.pwork = at<const int4>(p, mpc_plan::B_WPARSE);
  a.cs_off = d.cs_off; a.cs_base = d.cs_base;
  a.subev = at<uint16_t>(p, mpc_plan::B_SUBEV); a.subev_cnt = at<uint32_t>(p, mpc_plan::B_SUBCNT);
  a.subev_cap = p->subev_cap; a.n_of = d.n_of; a.gbase = d.gbase; a.sub = d.sub; a.nw_parse = p->parse_nw;
  a.wave_tab = at<const int32_t>(p, mpc_plan::B_WWAVE);
  a.slab = at<uint32_t>(p, mpc_plan::B_SUBSLAB);
  hipLaunchKernelGGL(K_subs, dim3((unsigned)(p->work_sub.size() / 4)), dim3(1024), 0, st, a);
  if (MPC_SUBS_SLAB) {
    const dim3 g((unsigned)(p->work_subsum.size() / 4 * (kSubWin * 2 / kSumCols)));
    if (p->subsum_rows > 8)
      hipLaunchKernelGGL(K_subsum<4>, g, dim3(4 * kSumCols), 0, st, at<const int4>(p, mpc_plan::B_WSUBSUM),
                         (const uint32_t*)a.slab, d.n_of, d.gbase, d.sub);
    else
      hipLaunchKernelGGL(K_subsum<1>, g, dim3(kSumCols), 0, st, at<const int4>(p, mpc_plan::B_WSUBSUM),
                         (const uint32_t*)a.slab, d.n_of, d.gbase, d.sub);
  }
}
static void launch_parse(const mpc_plan* p, const Dev& d, hipStream_t st) {
  ParseArgs a = parse_args(p, d);
  void* args[] = {&a};
  (void)hipLaunchKernel(parse_kernel(p), dim3(p->n_parse_wg), dim3(p->parse_nw * 64), args, (size_t)p->parse_lds, st);
}

static LeftArgs left_args(const mpc_plan* p, const Dev& d) {
  LeftArgs a;
  a.up_off = d.up_off; a.sample = d.sample; a.tstart = d.tstart; a.n_of = d.n_of; a.gbase = d.gbase;
  a.bc = at<const int4>(p, mpc_plan::B_WBC); a.units = at<const int4>(p, mpc_plan::B_UNITS); a.status = d.status;
  a.ins_sorted = at<uint32_t>(p, mpc_plan::B_INSSORT); a.pg_list = at<uint32_t>(p, mpc_plan::B_PGLIST);
  a.bk_cnt = at<int32_t>(p, mpc_plan::B_BKCNT); a.bk_off = at<int32_t>(p, mpc_plan::B_BKOFF);
  a.rbase = at<int64_t>(p, mpc_plan::B_RBASE); a.pwork = at<const int4>(p, mpc_plan::B_WPARSE);
  a.N = d.N; a.read_offset = d.read_offset; a.ovf_cap = d.ovf_cap; a.nbs = p->nbmax;
  a.right_start = d.right_start; a.rsl = d.rsl; a.roff = d.roff; a.vals_out = d.vals_out; a.M = d.M; a.runt = d.runt;
  a.ovf = d.ovf; a.ovf_cnt = d.ovf_cnt;
  return a;
}

static UnitArgs unit_args(const mpc_plan* p, const Dev& d) {
  UnitArgs a;
  a.bc = at<const int4>(p, mpc_plan::B_WBC); a.bk_cnt = at<int32_t>(p, mpc_plan::B_BKCNT);
  a.units = at<int4>(p, mpc_plan::B_UNITS); a.status = d.status;
  a.n_of = d.n_of; a.gbase = d.gbase;
  a.n_bc = p->n_bc; a.units_cap = p->units_cap; a.nbs = p->nbmax; a.unit = p->left_ub * kEPT / kPgEv;

  return a;
}
// K_left's geometry (planner: left_ub)
static void launch_left(const mpc_plan* p, const Dev& d, hipStream_t st);
// two (1024-thread) or three (512-thread) resident blocks per CU
static int64_t left_grid(const mpc_plan* p) {
  return std::max<int64_t>(1, std::min<int64_t>(p->units_cap, p->left_ub == 512 ? 768 : 512));
}
static LeftArgs left_args(const mpc_plan* p, const Dev& d);
static void launch_left(const mpc_plan* p, const Dev& d, hipStream_t st) {
  if (p->left_ub == 512) hipLaunchKernelGGL(K_left<512>, dim3(left_grid(p)), dim3(512), 0, st, left_args(p, d));
  else hipLaunchKernelGGL(K_left<kUB>, dim3(left_grid(p)), dim3(kUB), 0, st, left_args(p, d));
}
static int64_t ins_grid(const mpc_plan* p) { return std::max<int64_t>(1, std::min<int64_t>(p->units_cap, 512)); }
// 2-wave blocks only when 8-wave blocks would leave most CUs idle (C1's 20 k
// reads: 40 blocks); a C3 shard of 125 k reads (244 blocks of 8 waves) took
// 47.8 us in 2-wave blocks and 26.6 us in 8-wave ones (threshold 256 -> 128;
// C1, C2, C3 / 4 shards unchanged: profiles/r06_experiments/k_flank_small_blocks.txt)
#ifndef MPC_FLANK_SMALL_BELOW
#define MPC_FLANK_SMALL_BELOW 128
#endif
static int flank_waves(const mpc_plan* p) {
  return (p->N + kFW * 64 - 1) / (kFW * 64) < MPC_FLANK_SMALL_BELOW ? kFWSmall : kFW;
}
// K_flank blocks: one per chunk of flank_waves * 64 reads, at most kFlankBlocksMax
constexpr int64_t kFlankBlocksMax = MPC_FLANK_BLOCKS_MAX;
static int64_t flank_grid(const mpc_plan* p) {
  const int64_t fr = flank_waves(p) * 64;
  return std::max<int64_t>(1, std::min<int64_t>(kFlankBlocksMax, (p->N + fr - 1) / fr));
}

static InsArgs ins_args(const mpc_plan* p, const Dev& d) {
  InsArgs a;
  a.status = d.status; a.sample = d.sample; a.gbase = d.gbase;
  a.read_offset = d.read_offset; a.ovf_cap = d.ovf_cap; a.G = p->G;
  a.right_start = d.right_start; a.rsl = d.rsl; a.roff = d.roff; a.vals_out = d.vals_out;
  a.row_base = d.row_base; a.lo_f = d.lo_f; a.hiR = d.hiR;
  a.rows = d.rows; a.ovf = d.ovf; a.ovf_cnt = d.ovf_cnt; a.cs = d.cs;
  a.runt = d.runt;
  return a;
}

static FlankArgs flank_args(const mpc_plan* p, const Dev& d) {
  (void)p;
  FlankArgs a;
  a.status = d.status; a.sample = d.sample; a.n_of = d.n_of; a.gbase = d.gbase;
  a.tstart = d.tstart; a.i_end = d.i_end;
  a.up_off = d.up_off; a.up = d.up; a.down_off = d.down_off; a.down = d.down;
  a.right_start = d.right_start; a.rsl = d.rsl; a.roff = d.roff; a.vals_out = d.vals_out; a.rpos = d.rpos;
  a.row_base = d.row_base; a.lo_f = d.lo_f; a.hiR = d.hiR; a.loR = d.loR;
  a.rows = d.rows; a.N = d.N; a.read_offset = d.read_offset;
  return a;
}
static void launch_flank(const mpc_plan* p, const Dev& d, hipStream_t st) {
  const int nw = flank_waves(p);
  const dim3 grid((unsigned)flank_grid(p)), block((unsigned)(nw * 64));
  const bool multi = flank_grid(p) < (p->N + nw * 64 - 1) / (nw * 64);  // blocks take chunk ranges
  const FlankArgs fa = flank_args(p, d);
  if (nw == kFWSmall) {
    if (multi) hipLaunchKernelGGL((K_flank<kFWSmall, true>), grid, block, 0, st, fa);
    else hipLaunchKernelGGL((K_flank<kFWSmall, false>), grid, block, 0, st, fa);
  } else {
    if (multi) hipLaunchKernelGGL((K_flank<kFW, true>), grid, block, 0, st, fa);
    else hipLaunchKernelGGL((K_flank<kFW, false>), grid, block, 0, st, fa);
  }
}

// One launch clears every accumulator of a run (status, bitmaps, tallies, rows).
struct ClearArgs {
  uint32_t* ptr[24];
  int64_t words[24];
  uint32_t value[24];
  int32_t n;
};
__global__ __launch_bounds__(256) void K_clear(ClearArgs c) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int k = 0; k < c.n; ++k) {
    uint32_t* p = c.ptr[k];
    const uint32_t v = c.value[k];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.words[k]; i += stride) p[i] = v;
  }
}

static inline unsigned nblk(int64_t n, int b = 256) {
  int64_t g = (n + b - 1) / b;
  if (g < 1) g = 1;
  if (g > 65535 * 16) g = 65535 * 16;
  return (unsigned)g;
}

extern "C" {

int mpc_version(void) { return MPC_ABI_VERSION; }
#ifdef MPC_LEFT_DIAG
int mpc_diag_left(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_left_diag), sizeof(g_left_diag)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_left_diag), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

int mpc_build_flags(void) { return MPC_BF_STAMPS_ | MPC_BF_TUNING_ | MPC_BF_VARIANT_; }

size_t mpc_input_layout(size_t* off, int cap) {
#define MPC_F(f) offsetof(mpc_input, f)
  static const size_t o[] = {MPC_F(ref), MPC_F(ref_off), MPC_F(cs), MPC_F(cs_off), MPC_F(tstart), MPC_F(up),
                             MPC_F(up_off), MPC_F(down), MPC_F(down_off), MPC_F(sample), MPC_F(n_samples),
                             MPC_F(h_ref_len), MPC_F(h_read_begin), MPC_F(n_reads), MPC_F(cs_bytes), MPC_F(cs_base),
                             MPC_F(read_offset), MPC_F(n_reads_global), MPC_F(shard), MPC_F(n_shards),
                             MPC_F(h_cs_off), MPC_F(parse_cus), MPC_F(neg_reads), MPC_F(neg_cs_bytes)};
#undef MPC_F
  static_assert(sizeof(o) / sizeof(o[0]) == MPC_INPUT_FIELDS, "mpc_input field table");
  for (int k = 0; off && k < cap && k < MPC_INPUT_FIELDS; ++k) off[k] = o[k];
  return sizeof(mpc_input);
}
const char* mpc_last_error(void) { return g_err.c_str(); }

int mpc_plan_create(const mpc_input* in, int64_t row_cap, mpc_plan** out) {
  if (!in || !out) return fail(MPC_E_ARG, "null argument");
  if (in->n_samples <= 0) return fail(MPC_E_ARG, "n_samples must be > 0");
  auto* p = new mpc_plan();
  p->in = *in;
  p->S = in->n_samples;
  p->N = in->n_reads;
  p->Ng = in->n_reads_global > 0 ? in->n_reads_global : in->n_reads;
  p->n_shards = in->n_shards > 0 ? in->n_shards : 1;
  p->shard = in->shard;
  if (p->shard < 0 || p->shard >= p->n_shards) { delete p; return fail(MPC_E_ARG, "shard out of range"); }
  if (p->Ng < p->N || in->read_offset < 0 || in->read_offset + p->N > p->Ng) {
    delete p;
    return fail(MPC_E_ARG, "read shard [read_offset, read_offset + n_reads) outside [0, n_reads_global)");
  }
  p->ref_len.assign(in->h_ref_len, in->h_ref_len + p->S);
  p->read_begin.assign(in->h_read_begin, in->h_read_begin + p->S + 1);
  p->h_n.resize(p->S);
  p->h_gbase.resize(p->S + 1);
  int64_t g = 0;
  for (int s = 0; s < p->S; ++s) {
    if (p->ref_len[s] < 0 || p->ref_len[s] > kMaxRefLen) { delete p; return fail(MPC_E_ARG, "reference length out of range (at most 2^22 - 2 bases)"); }
    p->h_n[s] = (int32_t)p->ref_len[s];
    p->h_gbase[s] = (int32_t)g;
    g += p->ref_len[s] + 1;
  }
  p->h_gbase[p->S] = (int32_t)g;
  p->G = g;
  if (p->G >= (1ll << 30)) { delete p; return fail(MPC_E_ARG, "too many positions"); }
  if (p->Ng >= (1ll << 30)) { delete p; return fail(MPC_E_ARG, "too many reads (event words hold 30-bit read indices)"); }
  p->row_cap = row_cap > 0 ? row_cap : 1;
  if (p->row_cap >= (1ll << 31)) { delete p; return fail(MPC_E_ARG, "row capacity must be < 2^31"); }
  p->runs_cap = p->Ng + p->G;
  p->ins_cap = in->cs_bytes / 2 + 3 * p->N + 16;  // insertions (>= 2 cs bytes each) + slack per read
  p->ovf_cap = in->cs_bytes / 6 + 16;
  // strings Python's negative wrap writes into odd positions: <= 2 flanks per
  // read with a negative start plus its '+' insertions (>= 2 cs bytes each);
  // one shard only (the replay needs every string of a position)
  if (in->neg_reads < 0 || in->neg_cs_bytes < 0) { delete p; return fail(MPC_E_ARG, "negative neg_reads / neg_cs_bytes"); }
  p->wo_cap = p->n_shards == 1 && in->neg_reads > 0 ? std::min<int64_t>(kWoCapMax, 2 * in->neg_reads + in->neg_cs_bytes / 2 + 16) : 0;
  while (p->wo_p2 < p->wo_cap) p->wo_p2 <<= 1;
  int eb = 1;
  while ((1ll << eb) <= p->G + 1) ++eb;
  p->end_bit = eb;
  p->sentinel = (uint32_t)((1ull << eb) - 1);
  // ---- work tables ----
  {
    int64_t n_max = 0;
    for (int s = 0; s < p->S; ++s) {
      n_max = std::max<int64_t>(n_max, p->ref_len[s]);
      p->nbmax = std::max<int>(p->nbmax, (int)((p->ref_len[s] + 1 + kBW - 1) / kBW));
    }
    // parse geometry: tally mode, window and waves per workgroup that give the
    // most resident waves per CU (ties: the earlier candidate -- LDS tallies,
    // larger windows, the 12-byte tallies)
    const int lds_cap = 160 * 1024;
    const int max_waves_cu = 16;  // VGPR budget of K_parse (<= 128 VGPRs -> 4 waves per SIMD)
    auto lds_of = [&](int win, int tm, int nw) {
      return win == 512    ? parse_lds_bytes<512>((int)n_max, tm, p->nbmax, nw)
             : win == 2048 ? parse_lds_bytes<2048>((int)n_max, tm, p->nbmax, nw)
                           : parse_lds_bytes<1024>((int)n_max, tm, p->nbmax, nw);
    };
    // score = resident waves x window efficiency (measured at C2: 512 B windows
    // cost ~25 % more per byte than 2 KiB ones, 1 KiB ~5 %).  Tally mode 3 keeps
    // only depth in LDS; its substitutions are window events (K_subs) while the
    // reference fits kMaxSubWins windows, and then it competes on score: at C3 /
    // C4 (10 kb) its 16 waves beat tm 2's 12 (parse 3060 -> 2947 us, 3396 ->
    // 3004 us), at C2 tm 1 with 16 waves wins the tie (167 vs 197 us).  Beyond
    // that its substitutions are global atomics: only when tm 1 / 2 do not fit.
    const bool sub_events = n_max <= (int64_t)kSubWin * kMaxSubWins;
    static const int cand[10][2] = {{1, 2048}, {2, 2048}, {1, 1024}, {2, 1024}, {3, 2048}, {3, 1024},
                                    {1, 512}, {0, 2048}, {0, 1024}, {0, 512}};
    int best = -1, per_cu = 1;
    // tuning override for measurements: MPC_PARSE_GEOMETRY="tm,win,nw" takes that
    // candidate when it fits the LDS budget (else the planner's choice)
    int o_tm = -1, o_win = -1, o_nw = -1;
#ifdef MPC_TUNING_OVERRIDES  // experiment builds only (scripts/geom_ab.py); reported in mpc_plan_info.overrides
    if (const char* e = getenv("MPC_PARSE_GEOMETRY")) sscanf(e, "%d,%d,%d", &o_tm, &o_win, &o_nw);
#endif
    for (const auto& c : cand)
      for (int nw : {16, 12, 8}) {
        if (c[0] == 3 && !sub_events && best > 0) break;  // global-atomic tm 3 only when nothing else fits
        if (c[0] == 0 && best > 0) break;                  // tm 0 only when no LDS mode fits
        const int lds = lds_of(c[1], c[0], nw);
        if (lds > lds_cap) continue;
        const int wgs = std::max(1, std::min(lds_cap / lds, max_waves_cu / nw));
        int score = wgs * nw * (c[1] == 512 ? 75 : c[1] == 1024 ? 95 : 100);
        const bool forced = c[0] == o_tm && c[1] == o_win && nw == o_nw;
        if (forced) score = 1 << 30;
        if (score > best) {
          best = score; p->tally_mode = c[0]; p->parse_win = c[1]; p->parse_nw = nw; per_cu = wgs;
          p->overrides = forced ? (p->overrides | MPC_OVR_GEOMETRY) : (p->overrides & ~MPC_OVR_GEOMETRY);
        }
      }
    if (best < 0) {
      // references beyond every LDS mode (~312 kb): per-gap parse state in HBM
      for (int nw : {16, 12, 8}) {
        const int lds = parse_lds_bytes<1024>((int)n_max, 4, p->nbmax, nw);
        if (lds > lds_cap) continue;
        const int wgs = std::max(1, std::min(lds_cap / lds, max_waves_cu / nw));
        if (wgs * nw > best) { best = wgs * nw; p->tally_mode = 4; p->parse_win = 1024; p->parse_nw = nw; per_cu = wgs; }
      }
    }
    if (best < 0) { delete p; return fail(MPC_E_ARG, "reference too long for the LDS budget"); }
    p->parse_lds = lds_of(p->parse_win, p->tally_mode, p->parse_nw);
    // workgroups per sample: the smallest largest-chunk R with sum_s ceil(ns / R)
    // <= the resident slots (256 CUs x per_cu), so that the parse is one balanced
    // wave of workgroups (C5: 24 samples x 10 instead of x 11 = 264 > 256 slots,
    // whose 8 second-wave workgroups doubled K_parse); >= 64 reads per workgroup
    const int cus = in->parse_cus > 0 && in->parse_cus < 256 ? in->parse_cus : 256;
    int64_t target = (int64_t)cus * per_cu;
#ifdef MPC_TUNING_OVERRIDES
    if (const char* e = getenv("MPC_PARSE_WGS")) {  // measurement override
      target = std::max<int64_t>(1, atoll(e));
      p->overrides |= MPC_OVR_WGS;
    }
#endif
    const int64_t wcap = wg_reads_cap(p->tally_mode);
    auto chunks = [&](int64_t ns, int64_t R) {
      int64_t ch = (ns + R - 1) / R;
      ch = std::min<int64_t>(ch, (ns + 63) / 64);
      return std::max<int64_t>(ch, (ns + wcap - 1) / wcap);
    };
    int64_t R_lo = 1, R_hi = std::max<int64_t>(p->N, 1);
    while (R_lo < R_hi) {
      const int64_t mid = (R_lo + R_hi) / 2;
      int64_t tot = 0;
      for (int s = 0; s < p->S; ++s) tot += chunks(p->read_begin[s + 1] - p->read_begin[s], mid);
      if (tot <= target) R_hi = mid; else R_lo = mid + 1;
    }
    // boundaries of [a, b) cut into k parts: equal cs BYTES when the host copy
    // of cs_off is given (the parse time of a read range follows its bytes, not
    // its read count: a count split left waves idle at the epilogue barrier 22 %
    // of their time, profiles/r03_stamps), else equal read counts
    const int64_t* hco = in->h_cs_off;
    auto cut = [&](int64_t a, int64_t b, int64_t k, std::vector<int64_t>& out) {
      out.assign((size_t)k + 1, a);
      out[(size_t)k] = b;
      for (int64_t c = 1; c < k; ++c) {
        int64_t x = a + (b - a) * c / k;
        if (hco) {
          const int64_t tgt = hco[a] + (hco[b] - hco[a]) * c / k;
          x = std::lower_bound(hco + a, hco + b + 1, tgt) - hco;
        }
        out[(size_t)c] = std::min(std::max(x, out[(size_t)c - 1]), b);
      }
    };
    std::vector<int64_t> bnd;
    std::vector<int> pw_begin(p->S + 1, 0);
    for (int s = 0; s < p->S; ++s) {
      pw_begin[s] = (int)(p->work_parse.size() / 4);
      const int64_t a = p->read_begin[s], b = p->read_begin[s + 1], ns = b - a;
      if (ns <= 0) continue;
      const int64_t ch = chunks(ns, R_lo);
      cut(a, b, ch, bnd);
      bool capped = true;  // the byte split must keep the 16-bit tallies' reads-per-workgroup cap
      for (int64_t c = 0; c < ch; ++c) capped &= bnd[(size_t)c + 1] - bnd[(size_t)c] <= wcap;
      for (int64_t c = 0; c < ch; ++c) {
        const int64_t x = capped ? bnd[(size_t)c] : a + ns * c / ch;
        const int64_t y = capped ? bnd[(size_t)c + 1] : a + ns * (c + 1) / ch;
        if (y > x) p->work_parse.insert(p->work_parse.end(), {s, (int32_t)x, (int32_t)y, 0});
        p->max_wg_reads = std::max<int64_t>(p->max_wg_reads, y - x);
      }
    }
    // the chunks of every workgroup (its waves take them in turn): nw chunks
    // with 5/8 of the bytes, then nw with a quarter and nw with the last
    // eighth, so the last chunks taken are the small ones (measured against 4
    // groups of 1/2..1/8, 2 groups, equal quarters and one chunk per wave:
    // DESIGN.md "Parse work split")
    {
      constexpr int kGroups = 3;
      const int nw = p->parse_nw, nch = std::min(kMaxCh, kGroups * nw);
      std::vector<int64_t> part;
      for (size_t k = 0; k < p->work_parse.size(); k += 4) {
        const int64_t a = p->work_parse[k + 1], b = p->work_parse[k + 2];
        std::vector<int64_t> cb{a};
        static constexpr double grp[kGroups] = {0.625, 0.25, 0.125};
        // groups only while the smallest chunks still hold about half a window
        // (else one chunk per wave: C1's 3 KiB per wave ran 11 % slower cut in three)
        const int64_t wg_bytes = hco ? hco[b] - hco[a] : (b - a) * (in->cs_bytes / std::max<int64_t>(1, p->N));
        const int ng = wg_bytes >= 4 * (int64_t)nw * p->parse_win ? kGroups : 1;
        int64_t lo = a;
        double acc = 0;
        for (int g = 0; g < ng && (int)cb.size() - 1 < nch; ++g) {
          acc += grp[g];
          int64_t hi = b;
          if (g < ng - 1) {  // group end: the read where the cumulative byte fraction is reached
            if (hco) hi = std::lower_bound(hco + a, hco + b + 1, hco[a] + (int64_t)((hco[b] - hco[a]) * acc)) - hco;
            else hi = a + (int64_t)((b - a) * acc);
            hi = std::min(std::max(hi, lo), b);
          }
          cut(lo, hi, nw, part);
          for (int c = 1; c <= nw; ++c) cb.push_back(part[(size_t)c]);
          lo = hi;
        }
        p->work_parse[k + 3] = (int32_t)(cb.size() - 1);
        for (int c = 0; c <= kMaxCh; ++c) p->work_wave.push_back((int32_t)cb[(size_t)std::min<int>(c, (int)cb.size() - 1)]);
      }
    }
    pw_begin[p->S] = (int)(p->work_parse.size() / 4);
    p->n_parse_wg = pw_begin[p->S];
    // tally mode 3: substitutions as events per kSubWin-position window (K_subs)
    p->sub_wins = 0;
    if (p->tally_mode == 3 && sub_events) {
      p->sub_wins = (int32_t)((n_max + kSubWin - 1) / kSubWin);
      // parse workgroups per K_subs block: about one block per CU (each block's
      // LDS tally is 128 KiB; more blocks = more flush atomics, fewer = fewer CUs)
      int64_t pairs = 0;
      for (int s = 0; s < p->S; ++s)
        pairs += ((p->ref_len[s] + kSubWin - 1) / kSubWin) * (int64_t)(pw_begin[s + 1] - pw_begin[s]);
      const int kc = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)kSubsWG, (pairs + 255) / 256,
                                                                   65535 / std::max<int64_t>(1, p->max_wg_reads)}));
      for (int s = 0; s < p->S; ++s)
        for (int w = 0; w * (int64_t)kSubWin < p->ref_len[s]; ++w) {
          const int b0 = (int)(p->work_sub.size() / 4);
          for (int c = pw_begin[s]; c < pw_begin[s + 1]; c += kc)
            p->work_sub.insert(p->work_sub.end(), {s, w, c, std::min(c + kc, pw_begin[s + 1])});
          const int b1 = (int)(p->work_sub.size() / 4);
          if (b1 > b0) p->work_subsum.insert(p->work_subsum.end(), {s, w, b0, b1});
          p->subsum_rows = std::max(p->subsum_rows, b1 - b0);
        }
    }
    // deferred placement: the per-wave queues after the parse LDS, when they fit
    p->defer_off = 0;
    if (MPC_DEFER_PLACE && p->parse_win == 2048 && p->in.neg_reads == 0 &&
        (p->tally_mode == 1 || (MPC_SUB1 && p->tally_mode == 3 && p->sub_wins == 1))) {
      const int off = (p->parse_lds + 15) & ~15;
      const int end = off + defer_bytes(p->parse_nw, MPC_DEFER_SUBEV && p->tally_mode == 3);
      if (end <= lds_cap && std::max(1, std::min(lds_cap / end, max_waves_cu / p->parse_nw)) == per_cu) {
        p->defer_off = off;
        p->parse_lds = end;
      }
    }
    for (int s = 0; s < p->S; ++s) {
      const int nb = (int)((p->ref_len[s] + 1 + kBW - 1) / kBW);
      if (pw_begin[s + 1] == pw_begin[s]) continue;  // no reads: nothing to tally
      for (int b = 0; b < nb; ++b)  // insertion buckets
        for (int c = pw_begin[s]; c < pw_begin[s + 1]; c += 256)
          p->work_bc.insert(p->work_bc.end(), {s, b, c, std::min(c + 256, pw_begin[s + 1])});
    }
    p->n_bc = (int64_t)(p->work_bc.size() / 4);
    // K_left blocks of 512 threads (units of 8 k events) when there are many
    // small insertion buckets: C5's 24 x 469 buckets of ~3 k events each are
    // ~22 units per block in turn, whose fixed per-unit cost dominated at 1024
    // threads (K_left 352 -> 287 us).  Few or large buckets (C1-C4) keep 1024
    // (measured 4-45 % slower at 512: one unit per block, latency-bound).  The
    // bucket size is estimated from the cs bytes per (sample, bucket)
    {
      int64_t nb_all = 0;
      for (int s = 0; s < p->S; ++s) nb_all += (p->ref_len[s] + 1 + kBW - 1) / kBW;
      p->left_ub = nb_all > 4 * 512 && in->cs_bytes / nb_all < (256 << 10) ? 512 : kUB;
    }
    // work units of left_ub * kEPT / 64 pages (parse_page_base bounds the pages)
    p->units_cap = (parse_page_base(in->cs_bytes, p->N, p->n_parse_wg, p->nbmax) + 1) / (p->left_ub * kEPT / kPgEv) +
                   p->n_bc + 1;
  }
  const int64_t N = p->N, Ng = p->Ng, G = p->G, R = p->row_cap, RU = p->runs_cap;
  const int64_t nbg = (G + kGB - 1) / kGB, nbk = (R + kKB - 1) / kKB;
  auto set = [&](int b, int64_t count, size_t elem) { p->cnt[b] = count; p->sz[b] = (size_t)std::max<int64_t>(count, 1) * elem; };
  set(mpc_plan::B_STATUS, MPC_ST_WORDS, 4);
  set(mpc_plan::B_NOF, p->S, 4);
  set(mpc_plan::B_GBASE, p->S + 1, 4);
  set(mpc_plan::B_IEND, N, 4);
  // insertion events in 64-event pages per (parse workgroup, bucket)
  // (parse_page_base: the last workgroup's region ends at this bound)
  p->pages_cap = parse_page_base(in->cs_bytes, N, p->n_parse_wg, p->nbmax) + 1;
  set(mpc_plan::B_PGOWN, p->pages_cap, 4);
  set(mpc_plan::B_PGLIST, p->pages_cap, 4);
  set(mpc_plan::B_INSSORT, p->pages_cap * kPgEv, 4);
  set(mpc_plan::B_BKCNT, (int64_t)p->n_parse_wg * p->nbmax, 4);
  set(mpc_plan::B_BKOFF, (int64_t)p->n_parse_wg * p->nbmax, 4);
  set(mpc_plan::B_RBASE, p->n_parse_wg, 8);
  set(mpc_plan::B_OVF, p->ovf_cap, sizeof(Ovf));
  set(mpc_plan::B_OVFCNT, 1, 4);
  set(mpc_plan::B_HASLEFT, (G + 31) / 32 + 1, 4);
  set(mpc_plan::B_MAXR, G, 4);
  const int64_t nrb = (N + kRS - 1) / kRS;
  set(mpc_plan::B_KIN, N, 4);
  set(mpc_plan::B_VIN, N, 4);
  set(mpc_plan::B_KOUT, N, 4);
  set(mpc_plan::B_VOUT, N, 4);
  set(mpc_plan::B_KTMP, N, 4);
  set(mpc_plan::B_VTMP, N, 4);
  set(mpc_plan::B_BCNT, nrb + 1, 4);
  set(mpc_plan::B_BPRE, nrb + 1, 4);
  // K_rsort's one workgroup gathers and sorts in time that grows with the read
  // blocks (C3, 977 blocks: 88 us): many reads take the multi-workgroup path
  p->rsort_multi = nrb > kRsortMultiBlocks;
  set(mpc_plan::B_GCNT, p->rsort_multi ? G + 1 : 0, 4);
  set(mpc_plan::B_KSLOT, p->rsort_multi ? nrb * (int64_t)kRS : 0, 4);
  set(mpc_plan::B_RSFLAG, p->rsort_multi ? 4 + 2 * ((G + 1 + kScanBlk - 1) / kScanBlk) : 0, 4);
  set(mpc_plan::B_RLEN, Ng, 4);
  set(mpc_plan::B_RPOS, N > 0 ? N : 1, 4);
  set(mpc_plan::B_RSTART, G + 1, 4);
  set(mpc_plan::B_RSLOC, G + 1, 4);
  set(mpc_plan::B_ROFF, G + 1, 4);
  set(mpc_plan::B_RCNT, G, 4);
  set(mpc_plan::B_RCNTALL, G * p->n_shards, 4);
  set(mpc_plan::B_DIFF, G, 4);
  set(mpc_plan::B_SUB, G * 4, 4);
  set(mpc_plan::B_M, RU, 4);
  set(mpc_plan::B_RUNR, RU, 4);
  set(mpc_plan::B_HIR, RU, 4);
  set(mpc_plan::B_LOR, RU, 4);
  set(mpc_plan::B_LOF, G, 4);
  set(mpc_plan::B_ROWCNT, G, 4);
  set(mpc_plan::B_ROWBASE, G, 4);
  set(mpc_plan::B_BSUM, 2 * nbg, 8);  // K_layout's look-back status words (rows, diff) per block
  set(mpc_plan::B_ROWS, R * 4, 4);
  set(mpc_plan::B_META, (R + 3) / 4 * 4, 1);
  set(mpc_plan::B_RES, R * 4, 4);
  set(mpc_plan::B_KEEP, nbk * 256, 4);
  set(mpc_plan::B_KSUM, nbk, 8);  // K_select's per-block look-back status words
  set(mpc_plan::B_CALLS, R * 4, 4);
  set(mpc_plan::B_NCALLS, p->S + 1, 4);
  set(mpc_plan::B_MAXD, p->S, 4);
  set(mpc_plan::B_SROW, p->S, 4);
  set(mpc_plan::B_WPARSE, (int64_t)p->work_parse.size(), 4);
  set(mpc_plan::B_WBC, (int64_t)p->work_bc.size(), 4);
  set(mpc_plan::B_UNITS, p->units_cap * 8, 4);  // 2 int4 per unit
  set(mpc_plan::B_RUNT, RU * 16, 4);            // per run: inline LEFT bases [bi from the 3' end][code]
  p->subev_cap = p->sub_wins ? in->cs_bytes / kSubEvBytes + 2 * N + 16 : 0;
  set(mpc_plan::B_SUBEV, p->subev_cap * p->sub_wins, 2);
  set(mpc_plan::B_SUBCNT, p->sub_wins ? (int64_t)p->n_parse_wg * kMaxCh * kMaxSubWins : 0, 4);
  set(mpc_plan::B_WSUB, (int64_t)p->work_sub.size(), 4);
  set(mpc_plan::B_BKCUR, p->tally_mode == 4 ? (int64_t)p->n_parse_wg * p->nbmax : 0, 4);
  set(mpc_plan::B_WWAVE, (int64_t)p->work_wave.size(), 4);
  set(mpc_plan::B_SUBSLAB, MPC_SUBS_SLAB ? (int64_t)(p->work_sub.size() / 4) * kSubWin * 2 : 0, 4);
  set(mpc_plan::B_WSUBSUM, (int64_t)p->work_subsum.size(), 4);
  set(mpc_plan::B_WOEV, p->wo_cap, sizeof(WoEv));
  set(mpc_plan::B_WOKEY, p->wo_cap ? p->wo_p2 : 0, 8);
  set(mpc_plan::B_WOIDX, p->wo_cap ? p->wo_p2 : 0, 4);
  set(mpc_plan::B_WOERUN, 2 * p->wo_cap, 4);  // run of every sorted string, then K_woprep's scratch
  set(mpc_plan::B_WOPOS, p->wo_cap, sizeof(WoPos));
  set(mpc_plan::B_WORUN, p->wo_cap ? 2 * p->wo_cap + 1 : 0, sizeof(WoRun));
  size_t o = 0;
  for (int b = 0; b < mpc_plan::B_COUNT; ++b) {
    o = (o + 255) & ~(size_t)255;
    p->off[b] = o;
    o += p->sz[b];
  }
  p->ws_bytes = (o + 255) & ~(size_t)255;
  p->in.h_cs_off = nullptr;  // host array only read while planning
  *out = p;
  return MPC_OK;
}

int mpc_plan_destroy(mpc_plan* p) { delete p; return MPC_OK; }

int mpc_plan_get_info(const mpc_plan* p, mpc_plan_info* info) {
  if (!p || !info) return fail(MPC_E_ARG, "null argument");
  info->tally_mode = p->tally_mode;
  info->parse_window = p->parse_win;
  info->parse_waves = p->parse_nw;
  info->parse_lds_bytes = p->parse_lds;
  info->deferred_placement = p->defer_off > 0 ? 1 : 0;
  info->reserved = 0;
  info->parse_workgroups = p->n_parse_wg;
  info->max_reads_per_workgroup = p->max_wg_reads;
  info->reads_per_workgroup_cap = wg_reads_cap(p->tally_mode);
  info->workspace_bytes = (int64_t)p->ws_bytes;
  info->overrides = p->overrides;
  return MPC_OK;
}

// host copies of the parse work tables (tests / tools): n_wg * 4 int32 records
// {sample, first read, end read, chunks} and n_wg * (MPC_PARSE_CHUNKS + 1)
// chunk boundaries; either pointer may be NULL; returns the workgroup count
int mpc_plan_parse_tables(const mpc_plan* p, int32_t* work, int32_t* chunks) {
  if (!p) return fail(MPC_E_ARG, "null argument");
  if (work) std::copy(p->work_parse.begin(), p->work_parse.end(), work);
  if (chunks) std::copy(p->work_wave.begin(), p->work_wave.end(), chunks);
  return p->n_parse_wg;
}

int mpc_plan_workspace_bytes(const mpc_plan* p, size_t* bytes) {
  if (!p || !bytes) return fail(MPC_E_ARG, "null argument");
  *bytes = p->ws_bytes;
  return MPC_OK;
}

int mpc_plan_set_input(mpc_plan* p, const mpc_input* in) {
  if (!p || !in) return fail(MPC_E_ARG, "null argument");
  if (in->n_reads != p->N || in->n_samples != p->S || in->cs_bytes > p->in.cs_bytes ||
      (in->neg_reads > 0) != (p->in.neg_reads > 0))  // (the K_parse the plan bound; the list capacity stays)
    return fail(MPC_E_ARG, "input shape differs from the plan");
  p->in = *in;
  p->in.h_cs_off = nullptr;  // the work split stays the one planned
  return MPC_OK;
}

int mpc_plan_bind(mpc_plan* p, void* ws, size_t bytes) {
  if (!p || !ws) return fail(MPC_E_ARG, "null argument");
  if (bytes < p->ws_bytes) return fail(MPC_E_WORKSPACE, "workspace too small");
  if (((uintptr_t)ws & 255) != 0) return fail(MPC_E_ARG, "workspace must be 256-byte aligned");
  if (((uintptr_t)p->in.cs & 15) != 0) return fail(MPC_E_ARG, "cs buffer must be 16-byte aligned");
  if (((uintptr_t)p->in.up & 3) != 0 || ((uintptr_t)p->in.down & 3) != 0)
    return fail(MPC_E_ARG, "flank buffers must be 4-byte aligned");
  p->ws = (uint8_t*)ws;
  HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_NOF), p->h_n.data(), 4 * p->S, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_GBASE), p->h_gbase.data(), 4 * (p->S + 1), hipMemcpyHostToDevice));
  if (!p->work_parse.empty())
    HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_WPARSE), p->work_parse.data(), 4 * p->work_parse.size(), hipMemcpyHostToDevice));
  if (!p->work_bc.empty())
    HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_WBC), p->work_bc.data(), 4 * p->work_bc.size(), hipMemcpyHostToDevice));
  if (!p->work_wave.empty())
    HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_WWAVE), p->work_wave.data(), 4 * p->work_wave.size(),
                     hipMemcpyHostToDevice));
  if (!p->work_sub.empty())
    HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_WSUB), p->work_sub.data(), 4 * p->work_sub.size(), hipMemcpyHostToDevice));
  if (!p->work_subsum.empty())
    HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_WSUBSUM), p->work_subsum.data(), 4 * p->work_subsum.size(),
                     hipMemcpyHostToDevice));
  HIPCHK(hipFuncSetAttribute(parse_kernel(p), hipFuncAttributeMaxDynamicSharedMemorySize,
                             p->parse_lds));
  p->bound = true;
  p->runt_dirty = true;
  return MPC_OK;
}

int mpc_plan_buffer(const mpc_plan* p, int which, size_t* off, int64_t* count) {
  if (!p || !off || !count) return fail(MPC_E_ARG, "null argument");
  int b;
  switch (which) {
    case MPC_BUF_STATUS: b = mpc_plan::B_STATUS; break;
    case MPC_BUF_CALLS: b = mpc_plan::B_CALLS; break;
    case MPC_BUF_NCALLS: b = mpc_plan::B_NCALLS; break;
    case MPC_BUF_MAXDEPTH: b = mpc_plan::B_MAXD; break;
    case MPC_BUF_ROWS: b = mpc_plan::B_ROWS; break;
    case MPC_BUF_ROWMETA: b = mpc_plan::B_META; break;
    case MPC_BUF_RIGHT_CNT: b = mpc_plan::B_RCNT; break;
    case MPC_BUF_RIGHT_CNT_ALL: b = mpc_plan::B_RCNTALL; break;
    case MPC_BUF_HASLEFT: b = mpc_plan::B_HASLEFT; break;
    case MPC_BUF_MAXR: b = mpc_plan::B_MAXR; break;
    case MPC_BUF_RUN_M: b = mpc_plan::B_M; break;
    case MPC_BUF_RUN_R: b = mpc_plan::B_RUNR; break;
    case MPC_BUF_DIFF: b = mpc_plan::B_DIFF; break;
    case MPC_BUF_SUB: b = mpc_plan::B_SUB; break;
    default: return fail(MPC_E_ARG, "unknown buffer");
  }
  *off = p->off[b];
  *count = p->cnt[b];
  return MPC_OK;
}

// the mixed RIGHT events sorted by (gap, read): the multi-workgroup chain when
// the plan has many reads (it falls back to K_rsort by itself), else K_rsort
static void launch_rsort(const mpc_plan* p, const Dev& d, hipStream_t st) {
  const int32_t nrb = (int32_t)((p->N + kRS - 1) / kRS);
  if (p->rsort_multi) {
    const int32_t ns = (int32_t)((p->G + 1 + kScanBlk - 1) / kScanBlk);
    hipLaunchKernelGGL(K_rscan1, dim3(ns), dim3(1024), 0, st, d);
    hipLaunchKernelGGL(K_rscan2, dim3(ns), dim3(1024), 0, st, d, ns);
    hipLaunchKernelGGL(K_rscatter, dim3(nrb), dim3(kRS), 0, st, d);
    hipLaunchKernelGGL(K_rsegsort, dim3((unsigned)((p->G + 1 + 3) / 4)), dim3(256), 0, st, d);
  }
  hipLaunchKernelGGL(K_rsort, dim3(1), dim3(kRS), 0, st, d, nrb, (int32_t)p->end_bit);
}

#define NEED_BOUND(p) do { if (!(p) || !(p)->bound) return fail(MPC_E_STATE, "plan not bound"); } while (0)

int mpc_parse(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  {
    ClearArgs c{};
    bool over = false;
    auto add = [&](void* ptr, int64_t words, uint32_t v) {
      if (c.n == 24) { over = true; return; }  // ClearArgs holds 24 ranges
      c.ptr[c.n] = reinterpret_cast<uint32_t*>(ptr); c.words[c.n] = words; c.value[c.n] = v; ++c.n;
    };
    add(d.status, MPC_ST_FIRST_READ, 0u);                // (disjoint ranges: no ordering between threads)
    add(d.status + MPC_ST_FIRST_READ, 1, 0xffffffffu);
    add(d.status + MPC_ST_FIRST_READ + 1, MPC_ST_WORDS - MPC_ST_FIRST_READ - 1, 0u);
    add(d.hasleft, (int64_t)(p->sz[mpc_plan::B_HASLEFT] / 4), 0u);
    add(d.ovf_cnt, 1, 0u);
    add(d.diff, p->G, 0u);
    add(d.sub, 4 * p->G, 0u);
    add(d.maxR, p->G, 0u);
    if (p->rsort_multi) add(d.gcnt, p->G + 1, 0u);
    if (p->tally_mode == 4) {  // the bucket page words and page counts of the HBM-state parse
      add(at<int32_t>(p, mpc_plan::B_BKCUR), (int64_t)p->n_parse_wg * p->nbmax, kPgInit);
      add(at<int32_t>(p, mpc_plan::B_BKCNT), (int64_t)p->n_parse_wg * p->nbmax, 0u);
    }
    add(d.maxdepth, p->S, 0u);
    add(d.ksum, 2 * p->cnt[mpc_plan::B_KSUM], 0u);  // look-back status words (epoch-tagged as well)
    add(d.bsum, 2 * p->cnt[mpc_plan::B_BSUM], 0u);
    add(d.M, p->runs_cap, 0u);
    add(d.runR, p->runs_cap, 0u);
    if (p->runt_dirty) add(d.runt, 16 * p->runs_cap, 0u);
    add(d.rows, 4 * p->row_cap, 0u);
    add(d.meta, (int64_t)(p->sz[mpc_plan::B_META] / 4), 0u);
    if (over) return fail(MPC_E_STATE, "K_clear range table overflow");
    const int64_t most = std::max<int64_t>(4 * p->row_cap, std::max<int64_t>(4 * p->G, (p->runt_dirty ? 16 : 1) * p->runs_cap));
    hipLaunchKernelGGL(K_clear, dim3(std::min<unsigned>(nblk(most, 256), 1024)), dim3(256), 0, st, c);
    HIPCHK(hipGetLastError());
    p->runt_dirty = false;  // only once the clear is enqueued
  }
  if (p->n_parse_wg > 0) {
    launch_parse(p, d, st);
    launch_subs(p, d, st);
  }
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_index(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  const int32_t nrb = (int32_t)((p->N + kRS - 1) / kRS);
  // the insertion work units need only the parse: cut in the RIGHT-split launch
  // (one stream: a second one's event fork/join cost more than the overlap, measured)
  const int32_t nub = (int32_t)((p->n_bc + kUnitEntriesPerBlock - 1) / kUnitEntriesPerBlock);  // unit-cutting blocks
  if (nrb + nub > 0) hipLaunchKernelGGL(K_rsplit_units, dim3(nrb + nub), dim3(kRS), 0, st, d, unit_args(p, d), nrb);
  launch_rsort(p, d, st);
  hipLaunchKernelGGL(K_rstart, dim3(nblk(std::max<int64_t>(p->G + 1, p->N))), dim3(256), 0, st, d);  // (M <= N)
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_runs(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  if (p->n_shards > 1) {
    hipLaunchKernelGGL(K_runs, dim3(nblk(p->G + 1, kRunsGB)), dim3(kRunsGB), 0, st, d, next_epoch());
    if (p->N > 0) hipLaunchKernelGGL(K_runR, dim3(std::min<unsigned>(nblk(p->N), 1024)), dim3(256), 0, st, d);
  }
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_tally(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  launch_left(p, d, st);  // (units: mpc_index)
  p->runt_dirty = true;  // until K_ins has mapped (and cleared) the run tallies
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_layout(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  if (p->wo_cap > 0) {  // negative starts: the wrapped odd positions first
    hipLaunchKernelGGL(K_woprep, dim3(1), dim3(1024), 0, st, d);
    if (p->N > 0) hipLaunchKernelGGL(K_wocover, dim3(nblk(p->N, 256)), dim3(256), 0, st, d);
    hipLaunchKernelGGL(K_layout<true>, dim3(nblk(p->G, kGB)), dim3(kGB), 0, st, d, next_epoch());
  } else {
    hipLaunchKernelGGL(K_layout<false>, dim3(nblk(p->G, kGB)), dim3(kGB), 0, st, d, next_epoch());
  }
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_rows(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  hipLaunchKernelGGL(K_ins, dim3(ins_grid(p)), dim3(kUB), 0, st, ins_args(p, d));
  HIPCHK(hipGetLastError());
  p->runt_dirty = false;  // K_ins (enqueued) zeroes every run tally it maps (all runs of all gaps)
  if (p->N > 0) launch_flank(p, d, st);
  if (p->wo_cap > 0) hipLaunchKernelGGL(K_worows, dim3(64), dim3(256), 0, st, d);
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_consensus(mpc_plan* p, double mdf, double gtf, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  d.mdf = mdf;
  d.gtf = gtf;
  const int64_t R = p->row_cap;
  if (nblk(R, 256) > kCallBlocksMax) hipLaunchKernelGGL(K_call<kCRBig>, dim3(nblk(R, 256 * kCRBig)), dim3(256), 0, st, d, R);
  else hipLaunchKernelGGL(K_call<1>, dim3(nblk(R, 256)), dim3(256), 0, st, d, R);
  hipLaunchKernelGGL(K_select, dim3(nblk(R, kKB)), dim3(256), 0, st, d, R, next_epoch());
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_profile_kernel(mpc_plan* p, int which, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  if (p->N == 0) return MPC_OK;
  switch (which) {
    case MPC_K_PARSE:  // re-adds the odd tallies: status/tallies are stale until the next mpc_run
      launch_parse(p, d, st);
      break;
    case MPC_K_LEFT:
      launch_left(p, d, st);
      p->runt_dirty = true;
      break;
    case MPC_K_INS:
      hipLaunchKernelGGL(K_ins, dim3(ins_grid(p)), dim3(kUB), 0, st, ins_args(p, d));
      break;
    case MPC_K_FLANK:
      launch_flank(p, d, st);
      break;
    case MPC_K_RSORT:
      launch_rsort(p, d, st);
      break;
    default:
      return fail(MPC_E_ARG, "unknown kernel");
  }
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

#if defined(MPC_STAMPS) || defined(MPC_STAMPS_LEFT)
// diagnostic build only: per-wave K_parse (K_left) segment cycle sums (kStampSeg per wave)
int mpc_debug_stamps(uint64_t* out, int64_t n_words) {
  const int64_t nw = std::min<int64_t>(n_words, (int64_t)kStampWaves * kStampSeg);
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), (size_t)nw * 8, 0, hipMemcpyDeviceToHost));
  return MPC_OK;
}
int mpc_debug_stamps_clear(void) {
  static std::vector<uint64_t> z((size_t)kStampWaves * kStampSeg, 0);
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z.data(), z.size() * 8, 0, hipMemcpyHostToDevice));
  return MPC_OK;
}
#endif

int mpc_run(mpc_plan* p, double mdf, double gtf, void* stream) {
  int rc;
  if ((rc = mpc_parse(p, stream))) return rc;
  if ((rc = mpc_index(p, stream))) return rc;
  if ((rc = mpc_runs(p, stream))) return rc;
  if ((rc = mpc_tally(p, stream))) return rc;
  if ((rc = mpc_layout(p, stream))) return rc;
  if ((rc = mpc_rows(p, stream))) return rc;
  return mpc_consensus(p, mdf, gtf, stream);
}

}  // extern "C"
