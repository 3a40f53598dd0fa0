// libmpc: MI355X (gfx950) pileup + consensus for the consensus rule of the
// MinION plasmid pipeline.  Hot path = Steps 4-6 of
// /root/reference/src/mapped_paf_read_parser.py (include/mpc.h maps every
// reference function to its replacement; DESIGN.md has layouts and rooflines).
//
// Pipeline (one stream, no host synchronization):
//   parse     K_parse       per workgroup: contiguous reads of one sample.  cs
//                           tokens -> substitution / deletion / span tallies
//                           (LDS), insertion events (bucket-sorted by gap),
//                           i_end, LEFT-event gap bitmap, data-error flags
//   index     K_rsplit      downstream (RIGHT) events: mixed gaps -> sort keys,
//                           RIGHT-only gaps -> longest flank
//             radix sort    stable (gap, read) order of mixed RIGHT events
//             K_rstart      per-gap ranges in the sorted list
//   tally     K_left        one workgroup per 16-gap bucket: insertion tallies F
//                           and max LEFT length M per run; upstream flank M
//   layout    K_seg*,K_replay  per-gap replay of the slot-layout state of
//                           processBaseString_* (:37-72), row offsets (scan)
//   rows      scan          depth = prefix(difference array)
//             K_assemble    odd rows + F -> rows (plain stores)
//             K_strings     flanks + long insertions -> rows (LDS hash)
//   consensus K_call        per-slot top/second/tie/N (:363-439), max depth
//             scan, K_emit  threshold test + ordered compaction of the calls
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mpc.h"
#include "mpc_device.h"

using namespace mpc;

namespace {

constexpr uint32_t DE_OP = MPC_DE_OP, DE_VALUE = MPC_DE_VALUE, DE_INDEX = MPC_DE_INDEX,
                   DE_KEY = MPC_DE_KEY, DE_CAP = MPC_DE_CAPACITY, DE_INTERNAL = MPC_DE_INTERNAL;

constexpr int kBlk = 1024;          // cs bytes staged per wave iteration (64 lanes x 16 B)
constexpr int kInsInline = 4;       // insertions up to this length travel as one event word
constexpr int kFSlots = 4;          // right-justified insertion slots tallied per run (== kInsInline)
constexpr int kMaxRefLen = (1 << 22) - 1;
constexpr int kAdvCap = 1 << 22;    // > any reference length: a clamped advance keeps i past the end
constexpr int kLaneCap = 1 << 24;   // saturation of one lane's advance sum (64 lanes stay < 2^31)
constexpr int kICap = 1 << 28;      // saturation of the running coordinate i
constexpr int kBW = 16;             // gaps per insertion bucket (K_left workgroup)
constexpr int kKMax = 8;            // runs per gap tallied in K_left's LDS (others go to HBM)
constexpr uint32_t kNullGap = 0x3fffffu;

struct Ovf {  // long insertion (len > kInsInline), tallied by K_strings
  int64_t off;  // absolute byte offset of the inserted bases in cs
  int32_t read;
  int32_t gap;  // local gap index (i), sample implied by read
  int32_t len;
  int32_t pad[3];
};

// insertion event: low word gap<<10 | (len-1)<<8 | bases (2 bits each, string
// order); high word = global read index
__device__ __forceinline__ uint64_t ins_event(int gap, int len, uint32_t bases, int64_t rg) {
  return ((uint64_t)(uint32_t)rg << 32) | ((uint32_t)gap << 10) | ((uint32_t)(len - 1) << 8) | bases;
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
  int32_t* rlen;                     // [Ng] downstream length by global read
  int32_t* right_start;              // [G+1]
  int32_t* diff;                     // [G]
  uint32_t* sub;                     // [G][4]
  int32_t* M;                        // [Ng+G] per run
  uint32_t* F;                       // [Ng+G][16]
  int32_t* hflag; int32_t* hscan; int32_t* segR; int32_t* seg_lo; int32_t* seg_hi; int32_t* seg_run;
  int32_t* lo_f; int32_t* rowcnt; int32_t* row_base;
  int32_t* depth;
  uint32_t* rows; uint8_t* meta; int64_t row_cap;
  uint32_t* res; int32_t* keep; int32_t* keep_scan; uint32_t* calls; int32_t* ncalls; uint32_t* maxdepth;
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

__device__ __forceinline__ int64_t readlane64(int64_t x, int j) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)x, j);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), j);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// ---------------------------------------------------------------------------
// K_parse: Step 4 of the reference (:285-323 tokenizer, :74-104 processOperation)
// ---------------------------------------------------------------------------
constexpr int kPW = 8;                 // waves per workgroup
constexpr int kRB = 256;               // cs bytes staged per row per block step (16 lanes x 16 B)
constexpr int kTPL = 4;                // tokens per lane per round (64 per row round; 4 rows <= kIB events)
constexpr int kIB = 256;               // staged insertion events per wave
constexpr int kRowBuf = kRB + 32;      // + room for 12-byte operand reads
constexpr int kRowTok = kRB + 4;
constexpr int kWaveLds = 4 * kRowBuf + 4 * 2 * kRowTok + 8 * kIB + 2 * 4 * 64 + 16;

struct ParseArgs {  // slim argument block (no SGPR spills)
  const uint8_t* cs; const int64_t* cs_off; const int32_t* tstart;
  const int64_t* up_off; const int64_t* down_off; const int32_t* n_of; const int32_t* gbase;
  const int4* work;  // per workgroup: {sample, first read, end read, 0}
  int64_t cs_base, ovf_cap, read_offset;
  int32_t fused, nbmax;
  int32_t* i_end; uint64_t* ins_raw; uint64_t* ins_sorted; int32_t* bk_cnt; int32_t* bk_off; int64_t* rbase;
  Ovf* ovf; uint32_t* ovf_cnt; uint32_t* hasleft; uint32_t* status;
  int32_t* diff; uint32_t* sub;
};

__host__ __device__ constexpr int parse_stage_bytes() { return kPW * kWaveLds + 16; }
__host__ __device__ inline int parse_hl_words(int n) { return (n + 1 + 31) / 32; }
__host__ __device__ inline int parse_lds_bytes(int n_max, bool fused, int nbmax) {
  const int tallies = fused ? 12 * (n_max + 1) : 0;
  const int buckets = 8 * nbmax;
  return parse_stage_bytes() + 4 * parse_hl_words(n_max) + (tallies > buckets ? tallies : buckets);
}

// DPP helpers on 16-lane rows
template <int N>
__device__ __forceinline__ int row_bcast(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x150 + N, 0xf, 0xf, false); }
__device__ __forceinline__ int row_scan(int x) {
  x += dpp_i32<0x111>(x);
  x += dpp_i32<0x112>(x);
  x += dpp_i32<0x114>(x);
  x += dpp_i32<0x118>(x);
  return x;
}

struct TokInfo { int adv; int kind; uint32_t pay; uint32_t err; };

// Semantics of one token that do not depend on its coordinate.  Operand bytes
// are read as aligned LDS words and decoded SWAR-style (8 digits, 4 bases);
// longer operands take a rare slow path.
__device__ __forceinline__ TokInfo analyze_token(const uint8_t* buf, int sx, int ex, bool is_last) {
  TokInfo r{0, 0, 0u, 0u};
  const int olen = ex - sx - 1;
  if (!(olen > 0 || is_last)) return r;  // empty operand: skipped unless last (:309, :320)
  const uint32_t op = buf[sx];
  const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
  const int a = sx + 1;
  const uint32_t q0 = b32[a >> 2], q1 = b32[(a >> 2) + 1];
  const uint32_t w0 = __builtin_amdgcn_alignbyte(q1, q0, (uint32_t)(a & 3));
  if (op == ':') {
    const uint32_t Tx = w0 ^ 0x30303030u;
    const uint32_t nd = (((Tx & 0x7F7F7F7Fu) + 0x76767676u) | Tx) & 0x80808080u;
    const uint32_t vm = olen >= 4 ? 0xffffffffu : ((1u << (8 * olen)) - 1u);
    if (olen >= 1 && olen <= 4 && (nd & vm) == 0) {
      // right-align up to 4 digits, then SWAR decimal conversion (pairs, quad)
      uint32_t X = (Tx & vm & 0x0F0F0F0Fu) << (8 * (4 - olen));
      X = (X * 2561u) >> 8;
      X = ((X & 0x00FF00FFu) * 6553601u) >> 16;
      r.adv = (int)(X & 0xffffu);
    } else {
      int64_t vv = 0;
      if (!py_int(buf + a, (int64_t)olen, &vv)) r.err |= DE_VALUE;
      else r.adv = vv <= 0 ? 0 : (vv < kAdvCap ? (int)vv : kAdvCap);
    }
    r.kind = r.adv > 0 ? 1 : 0;
  } else if (op == '*') {
    if (olen == 0) { r.err |= DE_INDEX; return r; }  // operand[-1] of '' (:96)
    const int cd = code_upper(buf[ex - 1]);
    if (cd < 0) r.err |= DE_KEY;
    r.pay = (uint32_t)(cd & 3);
    r.adv = 1;
    r.kind = 2;
  } else if (op == '+') {
    if (olen == 0) return r;
    uint32_t packed = 0;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cd = code_upper((w0 >> (8 * k)) & 0xffu);
      if (k < olen) { ok &= cd >= 0; packed |= (uint32_t)(cd & 3) << (2 * k); }
    }
    if (olen > 4)
      for (int k = 4; k < olen; ++k) ok &= code_upper(buf[a + k]) >= 0;
    if (!ok) r.err |= DE_KEY;
    r.pay = packed;
    r.kind = 3;
  } else if (op == '-') {
    r.adv = olen < kAdvCap ? olen : kAdvCap;
    r.kind = olen > 0 ? 4 : 0;
  } else if (op != 'Z') {
    r.err |= DE_OP;
  }
  return r;
}

// Long-token fallback (operand longer than a row block), executed by one row:
// the 16 lanes sweep HBM for the end of the operand.
struct LongTok { int adv; int kind; int code; int64_t olen; int64_t end; uint32_t err; };
__device__ LongTok long_token_row(const ParseArgs& a, int64_t pos, int64_t b1, int q, int rl) {
  const uint32_t op = a.cs[pos];
  const int64_t qq = pos + 1;
  int64_t e = b1;
  for (int64_t x = qq; x < b1; x += 16) {
    const int64_t idx = x + rl;
    const bool sp = idx < b1 && is_special(a.cs[idx]);
    const uint32_t bal = (uint32_t)(ballot(sp) >> (16 * q)) & 0xffffu;
    if (bal) { e = x + __ffs(bal) - 1; break; }
  }
  LongTok t{0, 0, 0, e - qq, e, 0u};
  const int64_t olen = e - qq;
  if (!(olen > 0 || e == b1)) return t;
  if (op == '+') {
    if (olen == 0) return t;
    bool bad = false;
    for (int64_t x = qq + rl; x < e; x += 16) bad |= code_upper(a.cs[x]) < 0;
    if ((ballot(bad) >> (16 * q)) & 0xffffu) t.err |= DE_KEY;
    t.kind = 3;
  } else if (op == ':') {
    int64_t vv = 0;
    const bool ok = py_int(a.cs + qq, olen, &vv);  // every lane of the row, same answer
    if (!ok) t.err |= DE_VALUE;
    else if (vv > 0) { t.adv = vv < kAdvCap ? (int)vv : kAdvCap; t.kind = 1; }
  } else if (op == '*') {
    if (olen == 0) t.err |= DE_INDEX;
    else {
      const int cd = code_upper(a.cs[e - 1]);
      if (cd < 0) t.err |= DE_KEY;
      t.code = cd & 3; t.adv = 1; t.kind = 2;
    }
  } else if (op == '-') {
    t.adv = olen < kAdvCap ? (int)olen : kAdvCap;
    t.kind = olen > 0 ? 4 : 0;
  } else if (op != 'Z') {
    t.err |= DE_OP;
  }
  return t;
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

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup = contiguous reads of ONE sample (host work table).  A wave takes
// batches of 64 consecutive reads (metadata loaded lane-parallel) and parses
// FOUR reads at a time, one per 16-lane row: each row stages its read's cs in
// 256-byte blocks, finds token starts with per-lane masks + a row DPP scan, and
// each lane executes up to kTPL consecutive tokens per round, so one row DPP
// scan of the lanes' advance sums gives every token its coordinate i.  No
// global store happens inside the read loop: substitutions, deletions and read
// spans are tallied in LDS (fused mode), insertion events are staged in a
// per-wave LDS ring and LEFT-event gaps in an LDS bitmap.  At the end the
// workgroup flushes its tallies and bucket-sorts its insertion events by gap.
__global__ __launch_bounds__(kPW * 64) void K_parse(ParseArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int l = lane();
  const int q = l >> 4, rl = l & 15;
  const int w = uniform_i32((int)(threadIdx.x >> 6));
  uint8_t* wl = lds + w * kWaveLds;
  uint8_t* buf = wl + q * kRowBuf;
  uint16_t* tok = reinterpret_cast<uint16_t*>(wl + 4 * kRowBuf) + q * kRowTok;
  uint64_t* ibuf = reinterpret_cast<uint64_t*>(wl + 4 * kRowBuf + 8 * kRowTok);
  int32_t* res_iend = reinterpret_cast<int32_t*>(wl + 4 * kRowBuf + 8 * kRowTok + 8 * kIB);
  uint32_t* res_err = reinterpret_cast<uint32_t*>(res_iend + 64);
  uint32_t* rowerr = res_err + 64;  // [4]
  uint32_t* misc = reinterpret_cast<uint32_t*>(lds + parse_stage_bytes() - 16);  // [0] WG event count
  const int4 wk = a.work[blockIdx.x];
  const int smp = wk.x;
  const int64_t r0 = wk.y, r1 = wk.z;
  const int n = a.n_of[smp];
  const int gb = a.gbase[smp];
  uint32_t* hl = reinterpret_cast<uint32_t*>(lds + parse_stage_bytes());       // LEFT gaps bitmap
  uint8_t* uni = lds + parse_stage_bytes() + 4 * parse_hl_words(n);
  uint32_t* sub_l = reinterpret_cast<uint32_t*>(uni);                          // [2*(n+1)] 4 x u16
  int32_t* diff_l = reinterpret_cast<int32_t*>(sub_l + 2 * (n + 1));           // [n+1]
  const bool fused = a.fused != 0;
  const int64_t rb_wg = (a.cs_off[r0] - a.cs_base) / 2 + r0;                   // insertion region
  const int64_t rb_cap = (a.cs_off[r1] - a.cs_base) / 2 + r1 - rb_wg;
  for (int k = threadIdx.x; k < parse_hl_words(n); k += blockDim.x) hl[k] = 0;
  if (fused)
    for (int k = threadIdx.x; k < 3 * (n + 1); k += blockDim.x) sub_l[k] = 0;
  if (threadIdx.x == 0) misc[0] = 0;
  __syncthreads();

  int nib = 0;  // staged insertion events of this wave (wave-uniform)
  auto flush_ibuf = [&]() {
    wave_sync_lds();
    int basepos = 0;
    if (l == 0) basepos = (int)atomicAdd(misc, (uint32_t)nib);
    basepos = __shfl(basepos, 0, 64);
    if (basepos + nib > rb_cap) {
      if (l == 0) atomicOr(&a.status[MPC_ST_FLAGS], DE_INTERNAL);
    } else {
      for (int k = l; k < nib; k += 64) a.ins_raw[rb_wg + basepos + k] = ibuf[k];
    }
    nib = 0;
  };
  auto odd_sub = [&](int pos, int code) {
    if (fused) atomicAdd(sub_l + 2 * pos + (code >> 1), 1u << (16 * (code & 1)));
    else atomicAdd(a.sub + (int64_t)(gb + pos) * 4 + code, 1u);
  };
  auto odd_diff = [&](int pos, int v) {
    if (fused) atomicAdd(diff_l + pos, v);
    else atomicAdd(a.diff + gb + pos, v);
  };

  for (int64_t base = r0 + 64 * w; base < r1; base += 64 * kPW) {
    const int nb = (int)(r1 - base < 64 ? r1 - base : 64);
    // ---- batch metadata, lane j = read base+j ----
    int64_t m_b0 = 0, m_b1 = 0;
    int m_ts = 0, m_up = 0, m_dn = 0;
    if (l < nb) {
      const int64_t r = base + l;
      m_b0 = a.cs_off[r]; m_b1 = a.cs_off[r + 1];
      m_ts = a.tstart[r];
      const int64_t u = a.up_off[r + 1] - a.up_off[r], dv = a.down_off[r + 1] - a.down_off[r];
      m_up = u > 0x7fffffff ? 0x7fffffff : (int)u;
      m_dn = dv > 0x7fffffff ? 0x7fffffff : (int)dv;
    }
    // ---- per-row read state (row-uniform values held by all 16 lanes) ----
    int nxt = q;           // next batch index this row takes: q, q+4, ...
    bool have = false;
    int cur = 0;           // batch index of the row's current read
    int64_t pos = 0, b1 = 0;
    int i = 0, dn = 0;
    uint32_t derr = 0;
    bool first = false;
    while (true) {
      // rows without a read take their next one
      // (the gather runs with the full exec mask: ds_bpermute returns 0 for
      // inactive source lanes)
      const bool take = !have && nxt < nb;
      const int src = take ? nxt : l;
      const int64_t g_b0 = __shfl(m_b0, src, 64);
      const int64_t g_b1 = __shfl(m_b1, src, 64);
      const int g_ts = __shfl(m_ts, src, 64);
      const int g_up = __shfl(m_up, src, 64);
      const int g_dn = __shfl(m_dn, src, 64);
      if (take) {
        cur = nxt;
        nxt += 4;
        const int64_t b0 = g_b0;
        b1 = g_b1;
        const int ts = g_ts;
        const int up = g_up;
        dn = g_dn;
        derr = 0;
        if (ts < 0) derr |= DE_INDEX;                   // deviation: no negative wrap
        if (up > 0 && ts > n) derr |= DE_INDEX;         // leftIndel(2*i) past the end
        if (up > 0 && ts >= 0 && ts <= n && rl == 0) atomicOr(hl + (ts >> 5), 1u << (ts & 31));
        if (b1 <= b0) derr |= DE_OP;                    // processOperation('', '')
        i = ts;
        pos = b0;
        first = true;
        have = true;
      }
      if (!ballot(have)) break;
      // ---- one 256-byte block step for every row with a read ----
      const bool live = have && derr == 0 && pos < b1;
      const int64_t apos = pos & ~(int64_t)15;
      const int prel = (int)(pos - apos);
      const int vend = live ? (int)((b1 < apos + kRB ? b1 : apos + kRB) - apos) : 0;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (live) v = *reinterpret_cast<const uint4*>(a.cs + apos + 16 * rl);
      *reinterpret_cast<uint4*>(buf + 16 * rl) = v;
      const uint32_t mask = live ? special_mask16(v, prel - 16 * rl, vend - 16 * rl) : 0u;
      const int cnt = __popc(mask);
      const int incl = row_scan(cnt);
      const int T = row_bcast<15>(incl);
      {
        int e = incl - cnt;
        uint32_t m = mask;
        while (m) {
          const int k = __ffs(m) - 1;
          m &= m - 1;
          tok[e++] = (uint16_t)(16 * rl + k);
        }
      }
      if (rl == 0) tok[T] = (uint16_t)vend;  // sentinel: end of the last token
      wave_sync_lds();
      const bool reaches_end = apos + kRB >= b1;
      bool go = live;
      if (go && first) {
        // the reference runs processOperation('', operand) if the cs does not
        // start with an operator -> sys.exit (:100-102)
        if (T == 0 || tok[0] != (uint16_t)prel) { derr |= DE_OP; go = false; }
        first = false;
      }
      const int Tproc = go ? (reaches_end ? T : T - 1) : 0;
      const bool longtok = go && Tproc <= 0;
      if (longtok) {
        // ---- long token: its operand runs past this row block (rare) ----
        const LongTok t = long_token_row(a, pos, b1, q, rl);
        const int itok = i;
        i = i + t.adv < kICap ? i + t.adv : kICap;
        uint32_t te = t.err;
        if (t.kind == 1 && (int64_t)itok + t.adv > n) te |= DE_INDEX;
        if (t.kind == 2 && itok >= n) te |= DE_INDEX;
        if (t.kind == 3 && itok > n) te |= DE_INDEX;
        if (te == 0 && rl == 0) {
          if (t.kind == 2) odd_sub(itok, t.code);
          if (t.kind == 4 && itok < n) {
            odd_diff(itok, -1);
            odd_diff((int64_t)itok + t.olen < n ? (int)(itok + t.olen) : n, 1);
          }
          if (t.kind == 3) {
            atomicOr(hl + (itok >> 5), 1u << (itok & 31));
            push_ovf(a, pos + 1, base + cur, itok, (int)t.olen);
          }
        }
        derr |= te;
        pos = t.end;
      }
      // ---- rounds: lanes execute up to kTPL consecutive tokens each ----
      const int64_t rg = a.read_offset + base + cur;
      for (int t0 = 0; ballot(t0 < Tproc); t0 += 16 * kTPL) {
        int Tr = Tproc - t0;
        Tr = Tr < 0 ? 0 : (Tr > 16 * kTPL ? 16 * kTPL : Tr);
        const int per = (Tr + 15) >> 4;
        const int ta = t0 + rl * per;
        int na = Tr - rl * per;
        na = na < 0 ? 0 : (na > per ? per : na);
        int pre[kTPL];
        uint32_t inf[kTPL];
        int lsum = 0, nins_l = 0;
        uint32_t err = 0;
#pragma unroll
        for (int k = 0; k < kTPL; ++k) {
          uint32_t info = 0;
          int adv = 0;
          if (k < na) {
            const int t = ta + k;
            const int sx = tok[t], ex = tok[t + 1];
            const TokInfo ti = analyze_token(buf, sx, ex, reaches_end && t == T - 1);
            const int olen = ex - sx - 1;
            adv = ti.adv;
            err |= ti.err;
            info = (uint32_t)ti.kind | (ti.pay << 3) | ((uint32_t)olen << 11) | ((uint32_t)sx << 21);
            nins_l += (ti.kind == 3 && olen <= kInsInline) ? 1 : 0;
          }
          pre[k] = lsum;
          inf[k] = info;
          lsum = lsum + adv < kLaneCap ? lsum + adv : kLaneCap;
        }
        const int rincl = row_scan(lsum);
        const int ibase = i + rincl - lsum;
        if (Tr > 0) {
          const int tot = row_bcast<15>(rincl);
          i = i + tot < kICap ? i + tot : kICap;
        }
        const int iin = wave_scan_i32(nins_l);
        const int itot = wave_last_i32(iin);
        if (nib + itot > kIB) flush_ibuf();
        int iw = nib + iin - nins_l;
        nib += itot;
#pragma unroll
        for (int k = 0; k < kTPL; ++k) {
          if (k < na) {
            const uint32_t info = inf[k];
            const int kind = (int)(info & 7u);
            const uint32_t pay = (info >> 3) & 0xffu;
            const int olen = (int)((info >> 11) & 0x3ffu);
            const int itok = ibase + pre[k];
            const int adv = (k + 1 < na ? pre[k + 1] : lsum) - pre[k];
            uint32_t te = 0;
            if (kind == 1 && itok + adv > n) te |= DE_INDEX;
            if (kind == 2 && itok >= n) te |= DE_INDEX;
            if (kind == 3 && itok > n) te |= DE_INDEX;
            err |= te;
            if (te == 0) {
              if (kind == 2) odd_sub(itok, (int)pay);
              if (kind == 4 && itok < n) {
                odd_diff(itok, -1);
                odd_diff(itok + olen < n ? itok + olen : n, 1);
              }
              if (kind == 3) {
                atomicOr(hl + (itok >> 5), 1u << (itok & 31));
                if (olen > kInsInline) push_ovf(a, apos + (info >> 21) + 1, base + cur, itok, olen);
              }
            }
            if (kind == 3 && olen <= kInsInline)
              ibuf[iw++] = te == 0 ? ins_event(itok, olen, pay, rg) : ins_event((int)kNullGap, 1, 0u, rg);
          }
        }
        if (ballot(err != 0)) {  // rare: fold the row's error bits together
          if (l < 4) rowerr[l] = 0;
          wave_sync_lds();
          if (err) atomicOr(rowerr + q, err);
          wave_sync_lds();
          derr |= rowerr[q];
        }
      }
      if (go && !longtok) pos = reaches_end ? b1 : apos + tok[T - 1];
      // ---- rows whose read is complete (or failed) finish it ----
      const bool done = have && (derr != 0 || pos >= b1);
      if (done) {
        if (derr == 0 && dn > 0 && i > n) derr |= DE_INDEX;  // rightIndel(2*i) past the end
        if (rl == 0) {
          res_iend[cur] = i < 0 ? 0 : (i > n ? n + 1 : i);
          res_err[cur] = derr;
        }
        have = false;
      }
    }
    wave_sync_lds();
    // ---- per-read results, lane-parallel ----
    int m_iend = 0;
    uint32_t m_err = 0;
    if (l < nb) {
      const int64_t r = base + l;
      m_iend = res_iend[l];
      m_err = res_err[l];
      a.i_end[r] = m_iend;
      if (m_err) {
        atomicOr(&a.status[MPC_ST_FLAGS], m_err);
        atomicMin(&a.status[MPC_ST_FIRST_READ], (uint32_t)r);
      }
    }
    // read span [tstart, min(i_end, n)) -> depth difference points
    const int e = m_iend > n ? n : m_iend;
    const bool span = l < nb && m_err == 0 && m_ts >= 0 && m_ts < e;
    if (fused) {
      if (span) { atomicAdd(diff_l + m_ts, 1); atomicAdd(diff_l + e, -1); }
    } else {
      peel_atomic_add(a.diff, (int64_t)gb + m_ts, 1, span);
      peel_atomic_add(a.diff, (int64_t)gb + e, -1, span);
    }
  }
  if (nib) flush_ibuf();
  __syncthreads();
  // ---- flush LDS tallies and the LEFT-gap bitmap ----
  if (fused) {
    for (int p = threadIdx.x; p <= n; p += blockDim.x) {
      const int32_t dv = diff_l[p];
      if (dv) atomicAdd(a.diff + gb + p, dv);
      const uint32_t w0 = sub_l[2 * p], w1 = sub_l[2 * p + 1];
      uint32_t* sg = a.sub + (int64_t)(gb + p) * 4;
      if (w0 & 0xffffu) atomicAdd(sg + 0, w0 & 0xffffu);
      if (w0 >> 16) atomicAdd(sg + 1, w0 >> 16);
      if (w1 & 0xffffu) atomicAdd(sg + 2, w1 & 0xffffu);
      if (w1 >> 16) atomicAdd(sg + 3, w1 >> 16);
    }
  }
  for (int k = threadIdx.x; k < parse_hl_words(n); k += blockDim.x) {
    const uint32_t v = hl[k];
    if (!v) continue;
    const int g0 = gb + 32 * k;  // global bit of local bit 0 of this word
    atomicOr(a.hasleft + (g0 >> 5), v << (g0 & 31));
    if (g0 & 31) atomicOr(a.hasleft + (g0 >> 5) + 1, v >> (32 - (g0 & 31)));
  }
  __syncthreads();
  // ---- bucket-sort this workgroup's insertion events by gap (counting sort) ----
  const int nbk = (n + 1 + kBW - 1) / kBW;
  uint32_t* bcnt = reinterpret_cast<uint32_t*>(uni);  // aliases the (flushed) tallies
  uint32_t* bcur = bcnt + nbk;
  const int E = (int)misc[0];
  for (int k = threadIdx.x; k < nbk; k += blockDim.x) bcnt[k] = 0;
  __syncthreads();
  for (int k = threadIdx.x; k < E; k += blockDim.x) {
    const uint32_t gap = (uint32_t)(a.ins_raw[rb_wg + k] >> 10) & kNullGap;
    if (gap <= (uint32_t)n) atomicAdd(bcnt + gap / kBW, 1u);
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan over buckets by one wave
    int carry = 0;
    for (int c0 = 0; c0 < nbk; c0 += 64) {
      const int k = c0 + l;
      const int v = k < nbk ? (int)bcnt[k] : 0;
      const int inc = wave_scan_i32(v);
      if (k < nbk) {
        bcur[k] = (uint32_t)(carry + inc - v);
        a.bk_cnt[(int64_t)blockIdx.x * a.nbmax + k] = v;
        a.bk_off[(int64_t)blockIdx.x * a.nbmax + k] = carry + inc - v;
      }
      carry += wave_last_i32(inc);
    }
  }
  if (threadIdx.x == 0) a.rbase[blockIdx.x] = rb_wg;
  __syncthreads();
  for (int k = threadIdx.x; k < E; k += blockDim.x) {
    const uint64_t ev = a.ins_raw[rb_wg + k];
    const uint32_t gap = (uint32_t)(ev >> 10) & kNullGap;
    if (gap <= (uint32_t)n) a.ins_sorted[rb_wg + atomicAdd(bcur + gap / kBW, 1u)] = ev;
  }
}

// ---------------------------------------------------------------------------
// Downstream (RIGHT) events.  A gap holding only RIGHT events needs only its
// longest downstream flank (slot bi = base bi, :64-72).  Gaps that also hold a
// LEFT event ("mixed") need the RIGHT events in read order -> sort keys.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool has_left(const uint32_t* bm, int64_t g) { return (bm[g >> 5] >> (g & 31)) & 1u; }

__global__ __launch_bounds__(256) void K_rsplit(Dev d, uint32_t sentinel) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = r < d.N;
  int64_t g = -1;
  int32_t len = 0;
  bool mixed = false;
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
    const int64_t rg = d.read_offset + r;
    d.keys_in[r] = mixed ? (uint32_t)g : sentinel;
    d.vals_in[r] = (int32_t)rg;
    d.rlen[rg] = len;
  }
  peel_atomic_max(d.maxR, g < 0 ? 0 : g, len, in && g >= 0 && !mixed);
}

// right_start[g] = #mixed RIGHT events with gap < g
__global__ __launch_bounds__(256) void K_rstart(Dev d) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t <= d.G) d.right_start[t] = (int32_t)lower_bound_u32(d.keys_out, 0, d.Ng, (uint32_t)t);
  if (t == 0) d.status[MPC_ST_MIXED] = (uint32_t)lower_bound_u32(d.keys_out, 0, d.Ng, (uint32_t)d.G);
}

__global__ __launch_bounds__(256) void K_zero_runs(Dev d) {
  const int64_t nruns = (int64_t)d.right_start[d.G] + d.G;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nruns; t += (int64_t)gridDim.x * blockDim.x) {
    d.M[t] = 0;
    const uint4 z = make_uint4(0, 0, 0, 0);
    uint4* f = reinterpret_cast<uint4*>(d.F + t * 16);
    f[0] = z; f[1] = z; f[2] = z; f[3] = z;
  }
}

// run index of a LEFT event of global read rg at global gap g: runs of gap g
// are [right_start[g] + g, right_start[g+1] + g + 1); run k follows the k-th
// mixed RIGHT event (the RIGHT event of read r comes after r's own LEFT events,
// :303-323).
__device__ __forceinline__ int64_t run_of2(const int32_t* right_start, const int32_t* vals_out, int64_t g, int64_t rg) {
  const int64_t lo = right_start[g], hi = right_start[g + 1];
  int64_t k = 0;
  if (hi > lo) k = lower_bound_i32(vals_out, lo, hi, (int32_t)rg) - lo;
  return lo + g + k;
}

// ---------------------------------------------------------------------------
// K_left: LEFT events -> per-run max length M and right-justified insertion
// tallies F.  One workgroup per (sample, 16-gap bucket): it reads the bucket's
// slice of every parse workgroup's bucket-sorted insertion events, so each gap
// is owned by exactly one workgroup and its (gap, run) counters live in LDS
// (runs k < kKMax; rarer runs go to HBM).  Upstream flank lengths and long
// insertions only update M (grid-stride tails, wave-aggregated atomics).
// ---------------------------------------------------------------------------
struct LeftArgs {
  const int64_t* up_off; const int32_t* tstart; const int32_t* sample;
  const int32_t* n_of; const int32_t* gbase; const int4* work;  // {sample, bucket, pw0, pw1}
  const uint64_t* ins_sorted; const int32_t* bk_cnt; const int32_t* bk_off; const int64_t* rbase;
  int64_t N, read_offset, ovf_cap;
  int32_t nbmax;
  const int32_t* right_start; const int32_t* vals_out;
  int32_t* M; uint32_t* F;
  const Ovf* ovf; const uint32_t* ovf_cnt;
};

__global__ __launch_bounds__(256) void K_left(LeftArgs a) {
  __shared__ uint32_t Fl[kBW][kKMax][16];
  __shared__ uint32_t Ml[kBW][kKMax];
  const int l = lane();
  const int w = uniform_i32((int)(threadIdx.x >> 6));
  const int4 wk = a.work[blockIdx.x];
  const int smp = wk.x, bk = wk.y, pw0 = wk.z, pw1 = wk.w;
  const int n = a.n_of[smp];
  const int gb = a.gbase[smp];
  const int g0 = bk * kBW;
  for (int k = threadIdx.x; k < kBW * kKMax * 16; k += blockDim.x) (&Fl[0][0][0])[k] = 0;
  for (int k = threadIdx.x; k < kBW * kKMax; k += blockDim.x) (&Ml[0][0])[k] = 0;
  __syncthreads();
  for (int pw = pw0 + w; pw < pw1; pw += 4) {
    const int64_t slot = (int64_t)pw * a.nbmax + bk;
    const int cnt = a.bk_cnt[slot];
    const int64_t src = a.rbase[pw] + a.bk_off[slot];
    for (int e = l; e < cnt; e += 64) {
      const uint64_t ev = a.ins_sorted[src + e];
      const int gap = (int)((ev >> 10) & kNullGap);
      if (gap > n || gap < g0 || gap >= g0 + kBW) continue;
      const int L = (int)((ev >> 8) & 3u) + 1;
      const int64_t rg = (int64_t)(ev >> 32);
      const int64_t g = (int64_t)gb + gap;
      const int64_t run = run_of2(a.right_start, a.vals_out, g, rg);
      const int64_t k = run - (a.right_start[g] + g);
      if (k < kKMax) {
        atomicMax(&Ml[gap - g0][k], (uint32_t)L);
        for (int bi = 0; bi < L; ++bi) {  // bi counts from the 3' end (:55-61)
          const int code = (int)((ev >> (2 * (L - 1 - bi))) & 3u);
          atomicAdd(&Fl[gap - g0][k][bi * 4 + code], 1u);
        }
      } else {
        atomicMax(a.M + run, L);
        for (int bi = 0; bi < L; ++bi) {
          const int code = (int)((ev >> (2 * (L - 1 - bi))) & 3u);
          atomicAdd(a.F + run * 16 + bi * 4 + code, 1u);
        }
      }
    }
  }
  // upstream flanks: LEFT event at gap tstart contributes its length to M
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < a.N; r0 += nthreads) {
    const int64_t r = r0 + threadIdx.x;
    bool act = false;
    int64_t run = 0;
    int32_t ul = 0;
    if (r < a.N) {
      const int s = a.sample[r];
      const int ts = a.tstart[r];
      const int64_t u = a.up_off[r + 1] - a.up_off[r];
      ul = u > 0x7fffffff ? 0x7fffffff : (int32_t)u;
      if (ul > 0 && ts >= 0 && ts <= a.n_of[s]) {
        act = true;
        run = run_of2(a.right_start, a.vals_out, (int64_t)a.gbase[s] + ts, a.read_offset + r);
      }
    }
    peel_atomic_max(a.M, run, ul, act);
  }
  // long insertions
  const int64_t nov = *a.ovf_cnt < (uint32_t)a.ovf_cap ? *a.ovf_cnt : a.ovf_cap;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nov; t += nthreads) {
    const Ovf o = a.ovf[t];
    const int64_t g = (int64_t)a.gbase[a.sample[o.read]] + o.gap;
    atomicMax(a.M + run_of2(a.right_start, a.vals_out, g, a.read_offset + o.read), o.len);
  }
  __syncthreads();
  // flush: lanes sweep (gap, run, field) so each 16-field row is contiguous
  for (int q = threadIdx.x; q < kBW * kKMax * 16; q += blockDim.x) {
    const int f = q & 15, k = (q >> 4) % kKMax, p = q / (16 * kKMax);
    const uint32_t m = Ml[p][k];
    if (!m) continue;
    const int64_t g = (int64_t)gb + g0 + p;
    const int64_t run = a.right_start[g] + g + k;
    if (f == 0) atomicMax(a.M + run, (int32_t)m);
    const uint32_t v = Fl[p][k][f];
    if (v) atomicAdd(a.F + run * 16 + f, v);
  }
}

// ---------------------------------------------------------------------------
// Layout: replay of processBaseString_leftIndel / _rightIndel slot creation.
// Per gap the list grows at the front (LEFT, right-justified) and at the back
// (RIGHT, left-justified).  State: lo = slots prepended, hi = slots appended.
//   LEFT  len L : base bi -> absolute hi-1-bi ; lo = max(lo, L-hi)
//   RIGHT len R : base bi -> absolute -lo+bi  ; hi = max(hi, R-lo)
// Within a run of LEFT events hi is constant and within a run of RIGHT events
// lo is constant, so only runs with a LEFT event (M>0) start a new segment.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void K_seg_flags(Dev d) {
  const int64_t nruns = (int64_t)d.right_start[d.G] + d.G;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nruns; t += (int64_t)gridDim.x * blockDim.x) {
    d.hflag[t] = d.M[t] > 0 ? 1 : 0;
    d.segR[t] = 0;
  }
}

// the first run of every gap is a segment head (separate launch: no race with K_seg_flags)
__global__ __launch_bounds__(256) void K_seg_heads(Dev d) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < d.G; g += (int64_t)gridDim.x * blockDim.x)
    d.hflag[d.right_start[g] + g] = 1;
}

__global__ __launch_bounds__(256) void K_seg_right(Dev d) {
  const int64_t nm = d.right_start[d.G];
  const int64_t nruns = nm + d.G;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nm; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = d.keys_out[t];
    const int64_t seg = d.hscan[t + g] - 1;  // segment of the run just before this RIGHT event
    atomicMax(d.segR + seg, d.rlen[d.vals_out[t]]);
  }
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nruns; t += (int64_t)gridDim.x * blockDim.x)
    if (d.hflag[t]) d.seg_run[d.hscan[t] - 1] = (int32_t)t;
}

__global__ __launch_bounds__(256) void K_replay(Dev d) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= d.G) return;
  const int64_t r0 = d.right_start[g] + g, r1 = d.right_start[g + 1] + g + 1;  // runs of gap g
  const int64_t s0 = d.hscan[r0] - 1, s1 = d.hscan[r1 - 1];                   // segments [s0, s1)
  int32_t lo = 0, hi = 0;
  for (int64_t sidx = s0; sidx < s1; ++sidx) {
    const int32_t m = d.M[d.seg_run[sidx]];
    d.seg_hi[sidx] = hi;                       // hi seen by this run's LEFT events
    if (m - hi > lo) lo = m - hi;
    d.seg_lo[sidx] = lo;                       // lo seen by the RIGHT events of the segment
    const int32_t R = d.segR[sidx];
    if (R - lo > hi) hi = R - lo;
  }
  if (d.seg_run[s0] != r0) atomicOr(&d.status[MPC_ST_FLAGS], DE_INTERNAL);
  // RIGHT-only gaps: their flanks were not sorted; slot bi = base bi
  const int32_t mr = d.maxR[g];
  if (mr - lo > hi) hi = mr - lo;
  d.lo_f[g] = lo;
  // rows of a gap = its slots + the odd position after it (if any)
  int s = 0;
  while (g >= d.gbase[s + 1]) ++s;
  const int64_t p = g - d.gbase[s];
  d.rowcnt[g] = lo + hi + (p < d.n_of[s] ? 1 : 0);
}

__global__ void K_rows_total(Dev d) {
  const int64_t tot = (int64_t)d.row_base[d.G - 1] + d.rowcnt[d.G - 1];
  d.status[MPC_ST_ROWS_NEEDED] = (uint32_t)tot;
  if (tot > d.row_cap) atomicOr(&d.status[MPC_ST_FLAGS], DE_CAP);
}

// ---------------------------------------------------------------------------
// Rows: one wave per gap writes the gap's slot rows (F contributions summed in
// LDS, plain stores) and the odd-position row that follows it.
// ---------------------------------------------------------------------------
constexpr int kAsmChunk = 128;  // rows per LDS chunk per wave

__global__ __launch_bounds__(256) void K_assemble(Dev d) {
  __shared__ uint32_t s_rows[4][kAsmChunk * 4];
  const int l = lane(), w = threadIdx.x >> 6;
  uint32_t* acc = s_rows[w];
  if (d.status[MPC_ST_FLAGS] & DE_CAP) return;
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t g = (int64_t)blockIdx.x * 4 + w; g < d.G; g += stride) {
    int s = 0;
    while (g >= d.gbase[s + 1]) ++s;
    const int64_t p = g - d.gbase[s];
    const int64_t n = d.n_of[s];
    const int64_t rb = d.row_base[g];
    const int32_t lo = d.lo_f[g];
    const int64_t nslots = (int64_t)d.rowcnt[g] - (p < n ? 1 : 0);
    const int64_t r0 = d.right_start[g] + g, r1 = d.right_start[g + 1] + g + 1;
    for (int64_t c0 = 0; c0 < nslots; c0 += kAsmChunk) {
      const int64_t cn = nslots - c0 < kAsmChunk ? nslots - c0 : kAsmChunk;
      for (int k = l; k < kAsmChunk * 4; k += 64) acc[k] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // F contributions: LEFT run with hi at its segment
      for (int64_t run = r0 + l; run < r1; run += 64) {
        const int32_t m = d.M[run];
        if (m <= 0) continue;
        const int32_t hi = d.seg_hi[d.hscan[run] - 1];
        const int bmax = m < kFSlots ? m : kFSlots;
        for (int bi = 0; bi < bmax; ++bi) {
          const int64_t slot = (int64_t)lo + hi - 1 - bi - c0;
          if (slot < 0 || slot >= cn) continue;
          for (int c = 0; c < 4; ++c) {
            const uint32_t v = d.F[run * 16 + bi * 4 + c];
            if (v) atomicAdd(acc + slot * 4 + c, v);
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int64_t k = l; k < cn; k += 64) {
        const uint4 v = make_uint4(acc[k * 4], acc[k * 4 + 1], acc[k * 4 + 2], acc[k * 4 + 3]);
        reinterpret_cast<uint4*>(d.rows)[rb + c0 + k] = v;
        d.meta[rb + c0 + k] = (c0 + k == 0) ? 2 : 0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (p < n && l == 0) {
      // odd position p: depth = reads covering p with a match or substitution
      const int64_t dep = d.depth[g];
      const uint32_t* sb = d.sub + g * 4;
      const uint32_t s0 = sb[0], s1 = sb[1], s2 = sb[2], s3 = sb[3];
      const int64_t match = dep - (int64_t)s0 - s1 - s2 - s3;
      uint32_t c[4] = {s0, s1, s2, s3};
      uint32_t fl = 0;
      if (match < 0) fl |= DE_INTERNAL;
      else if (match > 0) {
        const int rc = base_code_exact(d.ref[d.ref_off[s] + p]);
        if (rc < 0) fl |= DE_KEY;  // refarr base not in the dict (:61)
        else c[rc] += (uint32_t)match;
      }
      if (fl) atomicOr(&d.status[MPC_ST_FLAGS], fl);
      reinterpret_cast<uint4*>(d.rows)[rb + nslots] = make_uint4(c[0], c[1], c[2], c[3]);
      d.meta[rb + nslots] = 3;  // odd row, first (only) slot of its position
    }
  }
}

// Flank / long-insertion tallies.  Hot rows (every full-length read's upstream
// flank lands on gap 0, every downstream flank on gap n) are aggregated in an
// LDS open-addressed table keyed by row, then flushed with global atomics.
constexpr int kHash = 2048;
constexpr uint32_t kEmpty = 0xffffffffu;

__device__ __forceinline__ void hash_add(uint32_t* keys, uint32_t* vals, uint32_t* rows, uint32_t row, int code) {
  uint32_t h = (row * 2654435761u) & (kHash - 1);
#pragma unroll 1
  for (int probe = 0; probe < 32; ++probe) {
    const uint32_t k = keys[h];
    if (k == row) { atomicAdd(vals + h * 4 + code, 1u); return; }
    if (k == kEmpty) {
      const uint32_t prev = atomicCAS(keys + h, kEmpty, row);
      if (prev == kEmpty || prev == row) { atomicAdd(vals + h * 4 + code, 1u); return; }
    }
    h = (h + 1) & (kHash - 1);
  }
  atomicAdd(rows + (uint64_t)row * 4 + code, 1u);  // table full: go straight to HBM
}

struct StrArgs {
  uint32_t* status; const int32_t* sample; const int32_t* n_of; const int32_t* gbase;
  int64_t N, read_offset, ovf_cap;
  const int64_t* up_off; const uint8_t* up; const int32_t* tstart;
  const int64_t* down_off; const uint8_t* down; const int32_t* i_end;
  const int32_t* right_start; const int32_t* vals_out; const int32_t* row_base; const int32_t* lo_f;
  const int32_t* seg_hi; const int32_t* seg_lo; const int32_t* hscan;
  uint32_t* rows; const Ovf* ovf; const uint32_t* ovf_cnt; const uint8_t* cs;
};

// One wave takes 64 consecutive reads: lane j resolves read j's two flank
// anchors (row of base 0 and direction).  Because the reads are consecutive,
// their upstream (downstream) flanks form ONE contiguous byte range; the wave
// streams that range with coalesced 4-byte loads and maps each byte back to
// its read by a short search over the 64 offsets held in LDS.
__device__ __forceinline__ void strings_range(const StrArgs& d, const uint8_t* bytes, int64_t x0, int64_t x1,
                                              const int64_t* off, const int64_t* anc, bool left, int nb,
                                              uint32_t* keys, uint32_t* vals, uint32_t& lerr, int64_t& lread,
                                              int64_t base) {
  const int l = lane();
  const int64_t a0 = x0 & ~(int64_t)3;
  for (int64_t w0 = a0; w0 < x1; w0 += 256) {
    const int64_t wx = w0 + 4 * l;
    uint32_t word = 0;
    if (wx < x1) word = *reinterpret_cast<const uint32_t*>(bytes + wx);
    if (wx + 4 <= x0 || wx >= x1) continue;
    // read containing byte wx (or the first byte >= x0): last j with off[j] <= max(wx, x0)
    const int64_t first = wx < x0 ? x0 : wx;
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= first) lo = mid; else hi = mid - 1;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t x = wx + k;
      if (x < x0 || x >= x1) continue;
      while (lo + 1 < nb && off[lo + 1] <= x) ++lo;
      const int64_t ank = anc[lo];
      if (ank == INT64_MIN) continue;  // this read's flank is not placed (beyond the reference end)
      const int code = base_code_exact((word >> (8 * k)) & 0xffu);
      if (code < 0) { lerr |= DE_KEY; lread = base + lo; continue; }
      // LEFT: base bi counted from the 3' end sits at anchor - bi, bi = end-1-x ;
      // RIGHT: base bi = x - start sits at anchor + bi
      const int64_t row = left ? ank - (off[lo + 1] - 1 - x) : ank + (x - off[lo]);
      hash_add(keys, vals, d.rows, (uint32_t)row, code);
    }
  }
}

__global__ __launch_bounds__(256) void K_strings(StrArgs d) {
  __shared__ uint32_t s_keys[kHash];
  __shared__ uint32_t s_vals[kHash * 4];
  __shared__ int64_t s_uoff[4][65], s_doff[4][65], s_uanc[4][64], s_danc[4][64];
  if (d.status[MPC_ST_FLAGS] & DE_CAP) return;
  for (int k = threadIdx.x; k < kHash; k += blockDim.x) s_keys[k] = kEmpty;
  for (int k = threadIdx.x; k < kHash * 4; k += blockDim.x) s_vals[k] = 0;
  __syncthreads();
  const int l = lane();
  const int w = uniform_i32((int)(threadIdx.x >> 6));
  uint32_t lerr = 0;
  int64_t lread = -1;
  const int64_t nbatch = (d.N + 63) / 64;
  for (int64_t bt = (int64_t)blockIdx.x * 4 + w; bt < nbatch; bt += (int64_t)gridDim.x * 4) {
    const int64_t base = bt * 64;
    const int nb = (int)(d.N - base < 64 ? d.N - base : 64);
    int64_t uanc = INT64_MIN, danc = INT64_MIN;
    if (l < nb) {
      const int64_t r = base + l;
      const int s = d.sample[r];
      const int64_t n = d.n_of[s];
      const int64_t gb = d.gbase[s];
      const int64_t rg = d.read_offset + r;
      const int64_t ts = d.tstart[r];
      const int64_t ie = d.i_end[r];
      s_uoff[w][l] = d.up_off[r];
      s_doff[w][l] = d.down_off[r];
      if (l == nb - 1) { s_uoff[w][nb] = d.up_off[r + 1]; s_doff[w][nb] = d.down_off[r + 1]; }
      if (ts >= 0 && ts <= n) {            // LEFT at gap tstart: row = lo + hi_run - 1 - bi
        const int64_t g = gb + ts;
        const int64_t run = run_of2(d.right_start, d.vals_out, g, rg);
        uanc = (int64_t)d.row_base[g] + d.lo_f[g] + d.seg_hi[d.hscan[run] - 1] - 1;
      }
      if (ie <= n) {                       // RIGHT at gap i_end: row = lo - lo_at + bi
        const int64_t g = gb + ie;
        int64_t lo_at = 0;
        const int64_t a = d.right_start[g], b = d.right_start[g + 1];
        if (b > a) {                       // mixed gap: this read's RIGHT event
          const int64_t t = lower_bound_i32(d.vals_out, a, b, (int32_t)rg);
          lo_at = d.seg_lo[d.hscan[t + g] - 1];
        }
        danc = (int64_t)d.row_base[g] + d.lo_f[g] - lo_at;
      }
    }
    s_uanc[w][l] = uanc;
    s_danc[w][l] = danc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    strings_range(d, d.up, s_uoff[w][0], s_uoff[w][nb], s_uoff[w], s_uanc[w], true, nb, s_keys, s_vals, lerr,
                  lread, base);
    strings_range(d, d.down, s_doff[w][0], s_doff[w][nb], s_doff[w], s_danc[w], false, nb, s_keys, s_vals, lerr,
                  lread, base);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // long insertions (grid-stride, LEFT like the short ones)
  const int64_t nov = *d.ovf_cnt < (uint32_t)d.ovf_cap ? *d.ovf_cnt : d.ovf_cap;
  for (int64_t t = blockIdx.x * 4 + w; t < nov; t += (int64_t)gridDim.x * 4) {
    const Ovf o = d.ovf[t];
    const int64_t g = d.gbase[d.sample[o.read]] + o.gap;
    const int64_t run = run_of2(d.right_start, d.vals_out, g, d.read_offset + o.read);
    const int64_t rb = (int64_t)d.row_base[g] + d.lo_f[g] + d.seg_hi[d.hscan[run] - 1] - 1;
    for (int64_t bi = l; bi < o.len; bi += 64) {
      const int c = code_upper(d.cs[o.off + o.len - 1 - bi]);
      hash_add(s_keys, s_vals, d.rows, (uint32_t)(rb - bi), c < 0 ? 0 : c);
    }
  }
  if (lerr) {
    atomicOr(&d.status[MPC_ST_FLAGS], lerr);
    atomicMin(&d.status[MPC_ST_FIRST_READ], (uint32_t)lread);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < kHash; k += blockDim.x) {
    const uint32_t row = s_keys[k];
    if (row == kEmpty) continue;
    for (int c = 0; c < 4; ++c) {
      const uint32_t v = s_vals[k * 4 + c];
      if (v) atomicAdd(d.rows + (uint64_t)row * 4 + c, v);
    }
  }
}

// ---------------------------------------------------------------------------
// Consensus (Steps 5-6, :332-439)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int sample_of_row(const Dev& d, int64_t row) {
  int s = 0;
  while (s + 1 < d.S && row >= d.row_base[d.gbase[s + 1]]) ++s;
  return s;
}

__global__ __launch_bounds__(256) void K_call(Dev d, int64_t R) {
  const bool cap = (d.status[MPC_ST_FLAGS] & DE_CAP) != 0;
  const int64_t need = cap ? 0 : (int64_t)d.status[MPC_ST_ROWS_NEEDED];
  for (int64_t row0 = (int64_t)blockIdx.x * blockDim.x; row0 < R; row0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = row0 + threadIdx.x;
    uint4 out = make_uint4(0, 0, 0, 0);
    uint32_t slot0 = 0;
    int smp = -1;
    if (row < R && row < need) {
      const uint4 cv = reinterpret_cast<const uint4*>(d.rows)[row];
      const uint32_t c[4] = {cv.x, cv.y, cv.z, cv.w};  // A, T, C, G
      const uint8_t mt = d.meta[row];
      const uint32_t total = c[0] + c[1] + c[2] + c[3];
      if (total > 0) {
        // sorted(tuples in dict order, key=count)[::-1]: descending count, ties in
        // reverse dict order (stable sort then reverse, :371-374)
        int idx[4], m = 0;
        for (int k = 3; k >= 0; --k) if (c[k] > 0) idx[m++] = k;   // reverse dict order
        for (int a = 1; a < m; ++a) {                               // stable sort descending
          const int t = idx[a];
          int b = a - 1;
          while (b >= 0 && c[idx[b]] < c[t]) { idx[b + 1] = idx[b]; --b; }
          idx[b + 1] = t;
        }
        const char names[4] = {'A', 'T', 'C', 'G'};
        uint32_t base, base2, count, count2;
        if (m == 1 || c[idx[0]] > c[idx[1]]) { base = names[idx[0]]; count = c[idx[0]]; }
        else { base = 'N'; count = 0; for (int a = 0; a < m; ++a) if (c[idx[a]] == c[idx[0]]) count += c[idx[a]]; }
        if (m <= 1) { base2 = 'X'; count2 = 0; }
        else if (m == 2 || c[idx[1]] > c[idx[2]]) { base2 = names[idx[1]]; count2 = c[idx[1]]; }
        else { base2 = 'N'; count2 = 0; for (int a = 0; a < m; ++a) if (c[idx[a]] == c[idx[1]]) count2 += c[idx[a]]; }
        const uint32_t chrom1 = base;
        if ((double)count < d.gtf * (double)count2) base = 'N';   // :421
        out = make_uint4(base | (chrom1 << 8) | (base2 << 16) | (1u << 24), count, count2, total);
        if (mt & 2u) { slot0 = total; smp = sample_of_row(d, row); }  // slot 0 only (:336)
      }
    }
    if (row < R) reinterpret_cast<uint4*>(d.res)[row] = out;
    // max depth: one atomic per wave when the wave's slot-0 rows share a sample
    const uint64_t act = ballot(smp >= 0);
    if (act) {
      const int lead = __ffsll((unsigned long long)act) - 1;
      const int s0 = __shfl(smp, lead, 64);
      const bool same = (smp < 0) || smp == s0;
      if (ballot(!same)) {
        if (smp >= 0) atomicMax(d.maxdepth + smp, slot0);
      } else {
        const uint32_t mx = (uint32_t)wave_max((int)slot0);
        if (lane() == 0) atomicMax(d.maxdepth + s0, mx);
      }
    }
  }
}

__global__ __launch_bounds__(256) void K_keep(Dev d, int64_t R) {
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < R; row += (int64_t)gridDim.x * blockDim.x) {
    const uint4 v = reinterpret_cast<const uint4*>(d.res)[row];
    int k = 0;
    if (v.x >> 24) {
      const int s = sample_of_row(d, row);
      const double thr = (double)d.maxdepth[s] * d.mdf;   // :338
      k = (double)v.y > thr ? 1 : 0;                        // :428
    }
    d.keep[row] = k;
  }
}

__global__ __launch_bounds__(256) void K_emit(Dev d, int64_t R) {
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < R; row += (int64_t)gridDim.x * blockDim.x) {
    if (d.keep[row]) {
      const uint4 v = reinterpret_cast<const uint4*>(d.res)[row];
      reinterpret_cast<uint4*>(d.calls)[d.keep_scan[row]] = make_uint4(v.x & 0xffffffu, v.y, v.z, v.w);
    }
  }
  if (blockIdx.x == 0) {
    for (int s = threadIdx.x; s <= d.S; s += blockDim.x) {
      const int64_t rb = s < d.S ? (int64_t)d.row_base[d.gbase[s]] : R;
      d.ncalls[s] = rb < R ? d.keep_scan[rb] : (R > 0 ? d.keep_scan[R - 1] + d.keep[R - 1] : 0);
    }
  }
}

}  // namespace

// ===========================================================================
// Host side: plan, workspace layout, phases, C-ABI
// ===========================================================================
static thread_local std::string g_err;
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
  int64_t N = 0, Ng = 0, G = 0, row_cap = 0, runs_cap = 0, ins_cap = 0, ovf_cap = 0;
  int32_t S = 0;
  uint32_t sentinel = 0;
  int end_bit = 0;
  size_t ws_bytes = 0;
  uint8_t* ws = nullptr;
  size_t cub_tmp = 0;
  std::vector<int32_t> work_parse, work_left;  // int4 records
  int n_parse_wg = 0, n_left_wg = 0, parse_lds = 0, nbmax = 1;
  bool fused = false;
  enum {
    B_STATUS, B_NOF, B_GBASE, B_IEND, B_INSRAW, B_INSSORT, B_BKCNT, B_BKOFF, B_RBASE, B_OVF, B_OVFCNT,
    B_HASLEFT, B_MAXR, B_KIN, B_VIN, B_KOUT, B_VOUT, B_RLEN, B_RSTART, B_DIFF, B_SUB, B_M, B_F,
    B_HFLAG, B_HSCAN, B_SEGR, B_SEGLO, B_SEGHI, B_SEGRUN, B_LOF, B_ROWCNT, B_ROWBASE, B_DEPTH, B_ROWS,
    B_META, B_RES, B_KEEP, B_KEEPSCAN, B_CALLS, B_NCALLS, B_MAXD, B_WPARSE, B_WLEFT, B_CUB, B_COUNT
  };
  size_t off[B_COUNT];
  size_t sz[B_COUNT];
  int64_t cnt[B_COUNT];
  bool bound = false;
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
  d.rlen = at<int32_t>(this, B_RLEN); d.right_start = at<int32_t>(this, B_RSTART);
  d.diff = at<int32_t>(this, B_DIFF); d.sub = at<uint32_t>(this, B_SUB);
  d.M = at<int32_t>(this, B_M); d.F = at<uint32_t>(this, B_F);
  d.hflag = at<int32_t>(this, B_HFLAG); d.hscan = at<int32_t>(this, B_HSCAN);
  d.segR = at<int32_t>(this, B_SEGR); d.seg_lo = at<int32_t>(this, B_SEGLO); d.seg_hi = at<int32_t>(this, B_SEGHI);
  d.seg_run = at<int32_t>(this, B_SEGRUN);
  d.lo_f = at<int32_t>(this, B_LOF); d.rowcnt = at<int32_t>(this, B_ROWCNT); d.row_base = at<int32_t>(this, B_ROWBASE);
  d.depth = at<int32_t>(this, B_DEPTH); d.rows = at<uint32_t>(this, B_ROWS); d.meta = at<uint8_t>(this, B_META);
  d.row_cap = row_cap;
  d.res = at<uint32_t>(this, B_RES); d.keep = at<int32_t>(this, B_KEEP); d.keep_scan = at<int32_t>(this, B_KEEPSCAN);
  d.calls = at<uint32_t>(this, B_CALLS); d.ncalls = at<int32_t>(this, B_NCALLS); d.maxdepth = at<uint32_t>(this, B_MAXD);
  return d;
}

static ParseArgs parse_args(const mpc_plan* p, const Dev& d) {
  ParseArgs a;
  a.cs = d.cs; a.cs_off = d.cs_off; a.tstart = d.tstart; a.up_off = d.up_off; a.down_off = d.down_off;
  a.n_of = d.n_of; a.gbase = d.gbase;
  a.work = reinterpret_cast<const int4*>(p->ws + p->off[mpc_plan::B_WPARSE]);
  a.cs_base = d.cs_base; a.ovf_cap = d.ovf_cap; a.read_offset = d.read_offset;
  a.fused = p->fused ? 1 : 0; a.nbmax = p->nbmax;
  a.i_end = d.i_end;
  a.ins_raw = at<uint64_t>(p, mpc_plan::B_INSRAW); a.ins_sorted = at<uint64_t>(p, mpc_plan::B_INSSORT);
  a.bk_cnt = at<int32_t>(p, mpc_plan::B_BKCNT); a.bk_off = at<int32_t>(p, mpc_plan::B_BKOFF);
  a.rbase = at<int64_t>(p, mpc_plan::B_RBASE);
  a.ovf = d.ovf; a.ovf_cnt = d.ovf_cnt; a.hasleft = d.hasleft; a.status = d.status;
  a.diff = d.diff; a.sub = d.sub;
  return a;
}

static LeftArgs left_args(const mpc_plan* p, const Dev& d) {
  LeftArgs a;
  a.up_off = d.up_off; a.tstart = d.tstart; a.sample = d.sample; a.n_of = d.n_of; a.gbase = d.gbase;
  a.work = reinterpret_cast<const int4*>(p->ws + p->off[mpc_plan::B_WLEFT]);
  a.ins_sorted = at<uint64_t>(p, mpc_plan::B_INSSORT);
  a.bk_cnt = at<int32_t>(p, mpc_plan::B_BKCNT); a.bk_off = at<int32_t>(p, mpc_plan::B_BKOFF);
  a.rbase = at<int64_t>(p, mpc_plan::B_RBASE);
  a.N = d.N; a.read_offset = d.read_offset; a.ovf_cap = d.ovf_cap; a.nbmax = p->nbmax;
  a.right_start = d.right_start; a.vals_out = d.vals_out; a.M = d.M; a.F = d.F;
  a.ovf = d.ovf; a.ovf_cnt = d.ovf_cnt;
  return a;
}

static StrArgs str_args(const Dev& d) {
  StrArgs a;
  a.status = d.status; a.sample = d.sample; a.n_of = d.n_of; a.gbase = d.gbase; a.N = d.N;
  a.read_offset = d.read_offset; a.ovf_cap = d.ovf_cap; a.up_off = d.up_off; a.up = d.up; a.tstart = d.tstart;
  a.down_off = d.down_off; a.down = d.down; a.i_end = d.i_end; a.right_start = d.right_start;
  a.vals_out = d.vals_out; a.row_base = d.row_base; a.lo_f = d.lo_f; a.seg_hi = d.seg_hi; a.seg_lo = d.seg_lo;
  a.hscan = d.hscan; a.rows = d.rows; a.ovf = d.ovf; a.ovf_cnt = d.ovf_cnt; a.cs = d.cs;
  return a;
}

static inline unsigned nblk(int64_t n, int b = 256) {
  int64_t g = (n + b - 1) / b;
  if (g < 1) g = 1;
  if (g > 65535 * 16) g = 65535 * 16;
  return (unsigned)g;
}

static unsigned strings_grid(int64_t N) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((N + 255) / 256, 1024));
}

extern "C" {

int mpc_version(void) { return MPC_ABI_VERSION; }
const char* mpc_last_error(void) { return g_err.c_str(); }

int mpc_plan_create(const mpc_input* in, int64_t row_cap, mpc_plan** out) {
  if (!in || !out) return fail(MPC_E_ARG, "null argument");
  if (in->n_samples <= 0) return fail(MPC_E_ARG, "n_samples must be > 0");
  auto* p = new mpc_plan();
  p->in = *in;
  p->S = in->n_samples;
  p->N = in->n_reads;
  p->Ng = in->n_reads_global > 0 ? in->n_reads_global : in->n_reads;
  p->ref_len.assign(in->h_ref_len, in->h_ref_len + p->S);
  p->read_begin.assign(in->h_read_begin, in->h_read_begin + p->S + 1);
  p->h_n.resize(p->S);
  p->h_gbase.resize(p->S + 1);
  int64_t g = 0;
  for (int s = 0; s < p->S; ++s) {
    if (p->ref_len[s] < 0 || p->ref_len[s] > kMaxRefLen) { delete p; return fail(MPC_E_ARG, "reference length out of range (< 2^22)"); }
    p->h_n[s] = (int32_t)p->ref_len[s];
    p->h_gbase[s] = (int32_t)g;
    g += p->ref_len[s] + 1;
  }
  p->h_gbase[p->S] = (int32_t)g;
  p->G = g;
  if (p->G >= (1ll << 30)) { delete p; return fail(MPC_E_ARG, "too many positions"); }
  if (p->Ng >= (1ll << 31) - 1) { delete p; return fail(MPC_E_ARG, "too many reads"); }
  p->row_cap = row_cap > 0 ? row_cap : 1;
  p->runs_cap = p->Ng + p->G;
  p->ins_cap = in->cs_bytes / 2 + p->N + 16;
  p->ovf_cap = in->cs_bytes / 6 + 16;
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
    const int lds_cap = 160 * 1024;
    p->fused = parse_lds_bytes((int)n_max, true, p->nbmax) <= lds_cap;
    p->parse_lds = parse_lds_bytes((int)n_max, p->fused, p->nbmax);
    if (p->parse_lds > lds_cap) { delete p; return fail(MPC_E_ARG, "reference too long for the LDS budget"); }
    const int per_cu = std::max(1, std::min(4, lds_cap / p->parse_lds));
    const int64_t target = 256 * std::min(per_cu, 2);
    std::vector<int> pw_begin(p->S + 1, 0);
    for (int s = 0; s < p->S; ++s) {
      pw_begin[s] = (int)(p->work_parse.size() / 4);
      const int64_t a = p->read_begin[s], b = p->read_begin[s + 1], ns = b - a;
      if (ns <= 0) continue;
      int64_t ch = std::max<int64_t>(1, (target * ns + std::max<int64_t>(p->N, 1) - 1) / std::max<int64_t>(p->N, 1));
      ch = std::min<int64_t>(ch, (ns + 63) / 64);
      for (int64_t c = 0; c < ch; ++c) {
        const int64_t x = a + ns * c / ch, y = a + ns * (c + 1) / ch;
        if (y > x) p->work_parse.insert(p->work_parse.end(), {s, (int32_t)x, (int32_t)y, 0});
      }
    }
    pw_begin[p->S] = (int)(p->work_parse.size() / 4);
    p->n_parse_wg = pw_begin[p->S];
    for (int s = 0; s < p->S; ++s) {
      const int nb = (int)((p->ref_len[s] + 1 + kBW - 1) / kBW);
      if (pw_begin[s + 1] == pw_begin[s]) continue;  // no reads: nothing to tally
      for (int b = 0; b < nb; ++b) p->work_left.insert(p->work_left.end(), {s, b, pw_begin[s], pw_begin[s + 1]});
    }
    p->n_left_wg = (int)(p->work_left.size() / 4);
  }
  {
    size_t t = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                             (int32_t*)nullptr, (int)std::max<int64_t>(p->Ng, 1), 0, eb);
    size_t mx = t;
    t = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, t, (int32_t*)nullptr, (int32_t*)nullptr, (int)p->runs_cap);
    mx = std::max(mx, t);
    t = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, t, (int32_t*)nullptr, (int32_t*)nullptr, (int)p->G);
    mx = std::max(mx, t);
    t = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, (int32_t*)nullptr, (int32_t*)nullptr, (int)p->row_cap);
    p->cub_tmp = std::max(mx, t);
  }
  const int64_t N = p->N, Ng = p->Ng, G = p->G, R = p->row_cap, RU = p->runs_cap;
  auto set = [&](int b, int64_t count, size_t elem) { p->cnt[b] = count; p->sz[b] = (size_t)std::max<int64_t>(count, 1) * elem; };
  set(mpc_plan::B_STATUS, MPC_ST_WORDS, 4);
  set(mpc_plan::B_NOF, p->S, 4);
  set(mpc_plan::B_GBASE, p->S + 1, 4);
  set(mpc_plan::B_IEND, N, 4);
  set(mpc_plan::B_INSRAW, p->ins_cap, 8);
  set(mpc_plan::B_INSSORT, p->ins_cap, 8);
  set(mpc_plan::B_BKCNT, (int64_t)p->n_parse_wg * p->nbmax, 4);
  set(mpc_plan::B_BKOFF, (int64_t)p->n_parse_wg * p->nbmax, 4);
  set(mpc_plan::B_RBASE, p->n_parse_wg, 8);
  set(mpc_plan::B_OVF, p->ovf_cap, sizeof(Ovf));
  set(mpc_plan::B_OVFCNT, 1, 4);
  set(mpc_plan::B_HASLEFT, (G + 31) / 32 + 1, 4);
  set(mpc_plan::B_MAXR, G, 4);
  set(mpc_plan::B_KIN, Ng, 4);
  set(mpc_plan::B_VIN, Ng, 4);
  set(mpc_plan::B_KOUT, Ng, 4);
  set(mpc_plan::B_VOUT, Ng, 4);
  set(mpc_plan::B_RLEN, Ng, 4);
  set(mpc_plan::B_RSTART, G + 1, 4);
  set(mpc_plan::B_DIFF, G, 4);
  set(mpc_plan::B_SUB, G * 4, 4);
  set(mpc_plan::B_M, RU, 4);
  set(mpc_plan::B_F, RU * 16, 4);
  set(mpc_plan::B_HFLAG, RU, 4);
  set(mpc_plan::B_HSCAN, RU, 4);
  set(mpc_plan::B_SEGR, RU, 4);
  set(mpc_plan::B_SEGLO, RU, 4);
  set(mpc_plan::B_SEGHI, RU, 4);
  set(mpc_plan::B_SEGRUN, RU, 4);
  set(mpc_plan::B_LOF, G, 4);
  set(mpc_plan::B_ROWCNT, G, 4);
  set(mpc_plan::B_ROWBASE, G, 4);
  set(mpc_plan::B_DEPTH, G, 4);
  set(mpc_plan::B_ROWS, R * 4, 4);
  set(mpc_plan::B_META, R, 1);
  set(mpc_plan::B_RES, R * 4, 4);
  set(mpc_plan::B_KEEP, R, 4);
  set(mpc_plan::B_KEEPSCAN, R, 4);
  set(mpc_plan::B_CALLS, R * 4, 4);
  set(mpc_plan::B_NCALLS, p->S + 1, 4);
  set(mpc_plan::B_MAXD, p->S, 4);
  set(mpc_plan::B_WPARSE, (int64_t)p->work_parse.size(), 4);
  set(mpc_plan::B_WLEFT, (int64_t)p->work_left.size(), 4);
  set(mpc_plan::B_CUB, (int64_t)p->cub_tmp, 1);
  size_t o = 0;
  for (int b = 0; b < mpc_plan::B_COUNT; ++b) {
    o = (o + 255) & ~(size_t)255;
    p->off[b] = o;
    o += p->sz[b];
  }
  p->ws_bytes = (o + 255) & ~(size_t)255;
  *out = p;
  return MPC_OK;
}

int mpc_plan_destroy(mpc_plan* p) { delete p; return MPC_OK; }

int mpc_plan_workspace_bytes(const mpc_plan* p, size_t* bytes) {
  if (!p || !bytes) return fail(MPC_E_ARG, "null argument");
  *bytes = p->ws_bytes;
  return MPC_OK;
}

int mpc_plan_set_input(mpc_plan* p, const mpc_input* in) {
  if (!p || !in) return fail(MPC_E_ARG, "null argument");
  if (in->n_reads != p->N || in->n_samples != p->S || in->cs_bytes > p->in.cs_bytes)
    return fail(MPC_E_ARG, "input shape differs from the plan");
  p->in = *in;
  return MPC_OK;
}

int mpc_plan_bind(mpc_plan* p, void* ws, size_t bytes) {
  if (!p || !ws) return fail(MPC_E_ARG, "null argument");
  if (bytes < p->ws_bytes) return fail(MPC_E_WORKSPACE, "workspace too small");
  if (((uintptr_t)ws & 255) != 0) return fail(MPC_E_ARG, "workspace must be 256-byte aligned");
  if (((uintptr_t)p->in.cs & 15) != 0) return fail(MPC_E_ARG, "cs buffer must be 16-byte aligned");
  p->ws = (uint8_t*)ws;
  HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_NOF), p->h_n.data(), 4 * p->S, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_GBASE), p->h_gbase.data(), 4 * (p->S + 1), hipMemcpyHostToDevice));
  if (!p->work_parse.empty())
    HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_WPARSE), p->work_parse.data(), 4 * p->work_parse.size(), hipMemcpyHostToDevice));
  if (!p->work_left.empty())
    HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_WLEFT), p->work_left.data(), 4 * p->work_left.size(), hipMemcpyHostToDevice));
  HIPCHK(hipFuncSetAttribute((const void*)K_parse, hipFuncAttributeMaxDynamicSharedMemorySize, p->parse_lds));
  p->bound = true;
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
    case MPC_BUF_RIGHT_KEY: b = mpc_plan::B_KIN; break;
    case MPC_BUF_RIGHT_READ: b = mpc_plan::B_VIN; break;
    case MPC_BUF_HASLEFT: b = mpc_plan::B_HASLEFT; break;
    case MPC_BUF_MAXR: b = mpc_plan::B_MAXR; break;
    case MPC_BUF_RUN_M: b = mpc_plan::B_M; break;
    default: return fail(MPC_E_ARG, "unknown buffer");
  }
  *off = p->off[b];
  *count = p->cnt[b];
  return MPC_OK;
}

#define NEED_BOUND(p) do { if (!(p) || !(p)->bound) return fail(MPC_E_STATE, "plan not bound"); } while (0)

int mpc_parse(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  HIPCHK(hipMemsetAsync(d.status, 0, 4 * MPC_ST_WORDS, st));
  HIPCHK(hipMemsetAsync(d.status + MPC_ST_FIRST_READ, 0xff, 4, st));
  HIPCHK(hipMemsetAsync(d.hasleft, 0, p->sz[mpc_plan::B_HASLEFT], st));
  HIPCHK(hipMemsetAsync(d.ovf_cnt, 0, 4, st));
  HIPCHK(hipMemsetAsync(d.diff, 0, 4 * p->G, st));
  HIPCHK(hipMemsetAsync(d.sub, 0, 16 * p->G, st));
  if (p->n_parse_wg > 0)
    hipLaunchKernelGGL(K_parse, dim3(p->n_parse_wg), dim3(kPW * 64), p->parse_lds, st, parse_args(p, d));
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_index(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  HIPCHK(hipMemsetAsync(d.maxR, 0, 4 * p->G, st));
  if (p->N > 0) hipLaunchKernelGGL(K_rsplit, dim3(nblk(p->N)), dim3(256), 0, st, d, p->sentinel);
  if (p->Ng > 0) {
    size_t tb = p->cub_tmp;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(at<uint8_t>(p, mpc_plan::B_CUB), tb, d.keys_in, d.keys_out, d.vals_in,
                                              d.vals_out, (int)p->Ng, 0, p->end_bit, st));
  } else {
    HIPCHK(hipMemsetAsync(d.keys_out, 0xff, 4, st));
  }
  hipLaunchKernelGGL(K_rstart, dim3(nblk(p->G + 1)), dim3(256), 0, st, d);
  hipLaunchKernelGGL(K_zero_runs, dim3(nblk(p->runs_cap)), dim3(256), 0, st, d);
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_tally(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  if (p->n_left_wg > 0) hipLaunchKernelGGL(K_left, dim3(p->n_left_wg), dim3(256), 0, st, left_args(p, d));
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_layout(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  uint8_t* tmp = at<uint8_t>(p, mpc_plan::B_CUB);
  hipLaunchKernelGGL(K_seg_flags, dim3(nblk(p->runs_cap)), dim3(256), 0, st, d);
  hipLaunchKernelGGL(K_seg_heads, dim3(nblk(p->G)), dim3(256), 0, st, d);
  size_t tb = p->cub_tmp;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, d.hflag, d.hscan, (int)p->runs_cap, st));
  hipLaunchKernelGGL(K_seg_right, dim3(nblk(p->runs_cap)), dim3(256), 0, st, d);
  hipLaunchKernelGGL(K_replay, dim3(nblk(p->G)), dim3(256), 0, st, d);
  tb = p->cub_tmp;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, d.rowcnt, d.row_base, (int)p->G, st));
  hipLaunchKernelGGL(K_rows_total, dim3(1), dim3(1), 0, st, d);
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_rows(mpc_plan* p, void* stream) {
  NEED_BOUND(p);
  hipStream_t st = (hipStream_t)stream;
  Dev d = p->dev();
  uint8_t* tmp = at<uint8_t>(p, mpc_plan::B_CUB);
  size_t tb = p->cub_tmp;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, d.diff, d.depth, (int)p->G, st));
  hipLaunchKernelGGL(K_assemble, dim3(nblk(p->G, 4)), dim3(256), 0, st, d);
  hipLaunchKernelGGL(K_strings, dim3(strings_grid(p->N)), dim3(256), 0, st, str_args(d));
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
  HIPCHK(hipMemsetAsync(d.maxdepth, 0, 4 * p->S, st));
  hipLaunchKernelGGL(K_call, dim3(nblk(R)), dim3(256), 0, st, d, R);
  hipLaunchKernelGGL(K_keep, dim3(nblk(R)), dim3(256), 0, st, d, R);
  uint8_t* tmp = at<uint8_t>(p, mpc_plan::B_CUB);
  size_t tb = p->cub_tmp;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, d.keep, d.keep_scan, (int)R, st));
  hipLaunchKernelGGL(K_emit, dim3(nblk(R)), dim3(256), 0, st, d, R);
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
      hipLaunchKernelGGL(K_parse, dim3(p->n_parse_wg), dim3(kPW * 64), p->parse_lds, st, parse_args(p, d));
      break;
    case MPC_K_LEFT:
      hipLaunchKernelGGL(K_left, dim3(p->n_left_wg), dim3(256), 0, st, left_args(p, d));
      break;
    case MPC_K_STRINGS:
      hipLaunchKernelGGL(K_strings, dim3(strings_grid(p->N)), dim3(256), 0, st, str_args(d));
      break;
    default:
      return fail(MPC_E_ARG, "unknown kernel");
  }
  HIPCHK(hipGetLastError());
  return MPC_OK;
}

int mpc_run(mpc_plan* p, double mdf, double gtf, void* stream) {
  int rc;
  if ((rc = mpc_parse(p, stream))) return rc;
  if ((rc = mpc_index(p, stream))) return rc;
  if ((rc = mpc_tally(p, stream))) return rc;
  if ((rc = mpc_layout(p, stream))) return rc;
  if ((rc = mpc_rows(p, stream))) return rc;
  return mpc_consensus(p, mdf, gtf, stream);
}

}  // extern "C"
