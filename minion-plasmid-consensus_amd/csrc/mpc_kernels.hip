// libmpc: MI355X (gfx950) pileup + consensus for the consensus rule of the
// MinION plasmid pipeline.  Hot path = Steps 4-6 of
// /root/reference/src/mapped_paf_read_parser.py (see include/mpc.h for the
// function-by-function map and DESIGN.md for layouts and rooflines).
//
// Pipeline (one stream, no host synchronization):
//   parse    K_parse        one wave per read: cs tokens -> odd events, insertion
//                           events, i_end, LEFT marks, data-error flags
//   index    K_rsplit       downstream (RIGHT) events: mixed gaps -> sort keys,
//                           RIGHT-only gaps -> max length
//            radix sort     stable (gap, read) order of mixed RIGHT events
//            K_rstart       per-gap ranges in the sorted list; zero run tables
//   tally    K_spans        read spans -> depth difference array
//            K_odd          substitutions / deletions -> odd tallies
//            K_left         insertions + upstream flanks -> per-run max length M
//                           and right-justified insertion tallies F
//   layout   K_seg*         run segmentation + per-gap replay of the slot
//                           layout state (lo, hi) of processBaseString_* (:37-72)
//            scan           row offsets per gap
//   rows     scan           depth = prefix(diff)
//            K_assemble     odd rows + F -> rows (plain stores)
//            K_strings      flanks + long insertions -> rows (LDS hash, atomics)
//   consensus K_call        per-slot top/second/tie/N (:363-439), max depth
//            scan, K_emit   threshold test + ordered compaction of calls
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#include "mpc.h"
#include "mpc_device.h"

using namespace mpc;

namespace {

constexpr uint32_t DE_OP = MPC_DE_OP, DE_VALUE = MPC_DE_VALUE, DE_INDEX = MPC_DE_INDEX,
                   DE_KEY = MPC_DE_KEY, DE_CAP = MPC_DE_CAPACITY, DE_INTERNAL = MPC_DE_INTERNAL;

constexpr int kParseWaves = 4;     // waves per workgroup in K_parse
constexpr int kBlk = 1024;         // cs bytes staged per wave iteration (64 lanes x 16 B)
constexpr int kInsInline = 4;      // insertions up to this length are packed in one event word
constexpr int kFSlots = 4;         // right-justified insertion slots tallied per run (== kInsInline)
constexpr int kMaxRefLen = (1 << 22) - 1;

// odd event word: pos<<3 | kind<<2 | payload   (kind 0: SUB payload=base code;
// kind 1: deletion diff point, payload 0 = start (-1), 1 = end (+1))
__device__ __forceinline__ uint32_t ev_sub(int64_t pos, int code) { return (uint32_t)(pos << 3) | (uint32_t)code; }
__device__ __forceinline__ uint32_t ev_del(int64_t pos, int end) { return (uint32_t)(pos << 3) | 4u | (uint32_t)end; }
// insertion event word: gap<<10 | (len-1)<<8 | bases (2 bits each, string order)

struct Ovf {  // long insertion (len > kInsInline), tallied by K_strings
  int64_t off;  // absolute byte offset of the inserted bases in cs
  int32_t read;
  int32_t gap;  // local gap index (i), sample implied by read
  int32_t len;
  int32_t pad[3];
};

struct Dev {  // device-side views of the plan (passed by value)
  // inputs
  const uint8_t* ref; const int64_t* ref_off;
  const uint8_t* cs; const int64_t* cs_off;
  const int32_t* tstart;
  const uint8_t* up; const int64_t* up_off;
  const uint8_t* down; const int64_t* down_off;
  const int32_t* sample;
  int64_t N, Ng, read_offset, cs_base;
  int32_t S, G;
  // per sample tables (device)
  const int32_t* n_of; const int32_t* gbase; // gbase[S+1]
  // parse outputs
  uint32_t* status;
  int32_t* i_end;
  uint32_t* odd_ev; int32_t* odd_cnt;
  uint32_t* ins_ev; int32_t* ins_cnt;
  Ovf* ovf; uint32_t* ovf_cnt; int64_t ovf_cap;
  uint8_t* hasleft;
  // index
  int32_t* maxR;
  uint32_t* keys_in; int32_t* vals_in; uint32_t* keys_out; int32_t* vals_out;
  int32_t* rlen;         // [Ng] downstream length by global read (mixed only meaningful)
  int32_t* right_start;  // [G+1]
  // tally
  int32_t* diff;         // [G]
  uint32_t* sub;         // [G][4]
  int32_t* M;            // [Ng+G] per run
  uint32_t* F;           // [Ng+G][16]
  // layout
  int32_t* hflag;        // [Ng+G]
  int32_t* hscan;        // [Ng+G] inclusive scan of hflag
  int32_t* segR;         // [Ng+G]
  int32_t* seg_lo;       // [Ng+G]
  int32_t* seg_hi;       // [Ng+G]
  int32_t* seg_run;      // [Ng+G] head run of each segment
  int32_t* lo_f;         // [G]
  int32_t* rowcnt;       // [G]
  int32_t* row_base;     // [G] exclusive scan of rowcnt
  // rows
  int32_t* depth;        // [G] inclusive scan of diff
  uint32_t* rows;        // [R][4]
  uint8_t* meta;         // [R]
  int64_t row_cap;
  // consensus
  uint32_t* res;         // [R][4]
  int32_t* keep;         // [R]
  int32_t* keep_scan;    // [R]
  uint32_t* calls;       // [R][4]
  int32_t* ncalls;       // [S+1]
  uint32_t* maxdepth;    // [S]
  double mdf, gtf;
};

__device__ __forceinline__ void report(const Dev& d, uint32_t flags, int64_t read) {
  if (flags) {
    atomicOr(&d.status[MPC_ST_FLAGS], flags);
    if (read >= 0) atomicMin(&d.status[MPC_ST_FIRST_READ], (uint32_t)read);
  }
}

__device__ __forceinline__ int64_t ev_base(const Dev& d, int64_t r) {
  return (d.cs_off[r] - d.cs_base) + 2 * r;
}

// ---------------------------------------------------------------------------
// K_parse: Step 4 of the reference (:285-323 tokenizer, :74-104 processOperation)
// One wave per read; the read's cs is streamed through LDS in 1 KiB blocks
// (one 16-B load per lane), token starts are found with per-lane masks + a wave
// scan, then each lane executes one token; a wave scan of the per-token
// reference advance gives every token its coordinate i.
// ---------------------------------------------------------------------------
struct TokOut {
  int64_t adv;
  int kind;       // 0 none, 1 match, 2 sub, 3 ins, 4 del
  int code;       // sub base
  int64_t olen;
  uint32_t bases; // packed insertion bases (olen <= kInsInline)
  uint32_t err;
};

// Execute the semantics of one token that does NOT depend on i.
template <class P>
__device__ __forceinline__ TokOut token_semantics(uint32_t op, P operand, int64_t olen, bool is_last) {
  TokOut t{0, 0, 0, olen, 0u, 0u};
  if (!(olen > 0 || is_last)) return t;  // empty operand: skipped unless last (:309, :320)
  switch (op) {
    case ':': {
      int64_t v;
      if (!py_int(operand, olen, &v)) t.err |= DE_VALUE;
      else if (v > 0) { t.adv = v; t.kind = 1; }
      break;
    }
    case '*': {
      if (olen == 0) { t.err |= DE_INDEX; break; }  // operand[-1] of ''
      int c = base_code(operand[olen - 1]);
      if (c < 0) t.err |= DE_KEY;
      t.code = c < 0 ? 0 : c;
      t.adv = 1; t.kind = 2;
      break;
    }
    case '+': {
      if (olen == 0) break;
      uint32_t packed = 0;
      for (int64_t k = 0; k < olen; ++k) {
        int c = base_code(operand[k]);
        if (c < 0) { t.err |= DE_KEY; break; }
        if (k < kInsInline) packed |= (uint32_t)c << (2 * k);
      }
      t.bases = packed;
      t.kind = 3;
      break;
    }
    case '-':
      t.adv = olen; t.kind = olen > 0 ? 4 : 0;
      break;
    case 'Z':
      break;
    default:
      t.err |= DE_OP;
  }
  return t;
}

__global__ __launch_bounds__(256) void K_parse(Dev d) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[kParseWaves][kBlk + 16];
  __shared__ uint16_t s_tok[kParseWaves][kBlk + 1];
  const int l = lane(), w = threadIdx.x >> 6;
  uint8_t* buf = s_buf[w];
  uint16_t* tok = s_tok[w];
  const int64_t stride = (int64_t)gridDim.x * kParseWaves;
  for (int64_t r = (int64_t)blockIdx.x * kParseWaves + w; r < d.N; r += stride) {
    const int64_t b0 = d.cs_off[r], b1 = d.cs_off[r + 1];
    const int s = d.sample[r];
    const int64_t n = d.n_of[s];
    const int64_t gb = d.gbase[s];
    int64_t i = d.tstart[r];
    uint32_t derr = 0;
    const int64_t evb = ev_base(d, r);
    int64_t nodd = 0, nins = 0;
    const int64_t uplen = d.up_off[r + 1] - d.up_off[r];
    const int64_t dnlen = d.down_off[r + 1] - d.down_off[r];
    if (i < 0) derr |= DE_INDEX;                       // deviation: no negative wrap
    if (uplen > 0 && i > n) derr |= DE_INDEX;          // leftIndel(2*i) past the end
    if (uplen > 0 && i >= 0 && i <= n && l == 0) d.hasleft[gb + i] = 1;
    if (b1 <= b0) derr |= DE_OP;                       // processOperation('', '')
    int64_t pos = b0;
    bool first = true;
    while (pos < b1 && derr == 0) {
      const int64_t apos = pos & ~(int64_t)15;
      const int64_t vend = b1 < apos + kBlk ? b1 : apos + kBlk;
      const uint4 v = *reinterpret_cast<const uint4*>(d.cs + apos + 16 * l);
      *reinterpret_cast<uint4*>(buf + 16 * l) = v;
      uint32_t mask = 0;
      const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t c = (wv[k >> 2] >> (8 * (k & 3))) & 0xffu;
        const int64_t idx = apos + 16 * l + k;
        if (idx >= pos && idx < vend && is_special(c)) mask |= 1u << k;
      }
      const int cnt = __popc(mask);
      const int incl = wave_incl_scan(cnt);
      const int T = __shfl(incl, 63, 64);
      {
        int e = incl - cnt;
        uint32_t m = mask;
        while (m) {
          const int k = __ffs(m) - 1;
          m &= m - 1;
          tok[e++] = (uint16_t)(16 * l + k);
        }
      }
      asm volatile("" ::: "memory");
      const bool reaches_end = apos + kBlk >= b1;
      if (first) {
        // the reference runs processOperation('', operand) if the cs does not
        // start with an operator -> sys.exit (:100-102)
        if (T == 0 || tok[0] != (uint16_t)(pos - apos)) { derr |= DE_OP; break; }
        first = false;
      }
      const int Tproc = reaches_end ? T : T - 1;
      if (Tproc <= 0) {
        // ---- long token: its operand runs past this 1 KiB block ----
        const uint32_t op = d.cs[pos];
        const int64_t q = pos + 1;
        int64_t e = b1;
        for (int64_t x = q; x < b1; x += 64) {
          const int64_t idx = x + l;
          const bool sp = idx < b1 && is_special(d.cs[idx]);
          const uint64_t bal = ballot(sp);
          if (bal) { e = x + __ffsll((unsigned long long)bal) - 1; break; }
        }
        const int64_t olen = e - q;
        const bool is_last = e == b1;
        TokOut t{0, 0, 0, olen, 0u, 0u};
        if (op == '+' && olen > 0) {
          // validate in parallel, the bases are re-read by K_strings
          bool bad = false;
          for (int64_t x = q; x < e; x += 64) {
            const int64_t idx = x + l;
            if (idx < e && base_code(d.cs[idx]) < 0) bad = true;
          }
          if (ballot(bad)) t.err |= DE_KEY;
          t.kind = 3;
        } else if (op == ':' ) {
          int64_t vv = 0;
          bool ok = true;
          if (l == 0) ok = py_int(d.cs + q, olen, &vv);
          ok = __shfl((int)ok, 0, 64);
          vv = __shfl(vv, 0, 64);
          if (!ok) t.err |= DE_VALUE;
          else if (vv > 0) { t.adv = vv; t.kind = 1; }
        } else {
          t = token_semantics(op, d.cs + q, olen, is_last);
        }
        const int64_t itok = i;
        i += t.adv;
        if (t.kind == 1 && itok + t.adv > n) t.err |= DE_INDEX;
        if (t.kind == 2 && itok >= n) t.err |= DE_INDEX;
        if (t.kind == 3 && itok > n) t.err |= DE_INDEX;
        if (t.err == 0 && l == 0) {
          if (t.kind == 2) d.odd_ev[evb + nodd++] = ev_sub(itok, t.code);
          if (t.kind == 4 && itok < n) {
            d.odd_ev[evb + nodd++] = ev_del(itok, 0);
            d.odd_ev[evb + nodd++] = ev_del(itok + olen < n ? itok + olen : n, 1);
          }
          if (t.kind == 3) {
            d.hasleft[gb + itok] = 1;
            const uint32_t slot = atomicAdd(d.ovf_cnt, 1u);
            if ((int64_t)slot < d.ovf_cap) {
              Ovf o; o.off = q; o.read = (int32_t)r; o.gap = (int32_t)itok; o.len = (int32_t)olen;
              o.pad[0] = o.pad[1] = o.pad[2] = 0;
              d.ovf[slot] = o;
            } else {
              atomicOr(&d.status[MPC_ST_FLAGS], DE_INTERNAL);
            }
          }
        }
        nodd = __shfl(nodd, 0, 64);
        derr |= t.err;
        pos = e;
        continue;
      }
      // ---- lanes execute tokens 0 .. Tproc-1 of this block ----
      for (int t0 = 0; t0 < Tproc; t0 += 64) {
        const int t = t0 + l;
        const bool act = t < Tproc;
        TokOut tk{0, 0, 0, 0, 0u, 0u};
        int sx = 0;
        if (act) {
          sx = tok[t];
          const int ex = (t + 1 < T) ? (int)tok[t + 1] : (int)(vend - apos);
          const bool is_last = reaches_end && (t == T - 1);
          tk = token_semantics((uint32_t)buf[sx], buf + sx + 1, (int64_t)(ex - sx - 1), is_last);
        }
        const int64_t ai = wave_incl_scan(tk.adv);
        const int64_t itok = i + ai - tk.adv;
        i += __shfl(ai, 63, 64);
        if (tk.kind == 1 && itok + tk.adv > n) tk.err |= DE_INDEX;
        if (tk.kind == 2 && itok >= n) tk.err |= DE_INDEX;
        if (tk.kind == 3 && itok > n) tk.err |= DE_INDEX;
        int no = 0, ni = 0;
        bool ov = false;
        if (tk.err == 0) {
          if (tk.kind == 2) no = 1;
          if (tk.kind == 4 && itok < n) no = 2;
          if (tk.kind == 3) {
            if (tk.olen <= kInsInline) ni = 1; else ov = true;
          }
        }
        const int pk = no | (ni << 16);
        const int pi = wave_incl_scan(pk);
        const int pe = pi - pk;
        const int oo = pe & 0xffff, io = pe >> 16;
        if (no == 1) d.odd_ev[evb + nodd + oo] = ev_sub(itok, tk.code);
        if (no == 2) {
          d.odd_ev[evb + nodd + oo] = ev_del(itok, 0);
          d.odd_ev[evb + nodd + oo + 1] = ev_del(itok + tk.olen < n ? itok + tk.olen : n, 1);
        }
        if (ni) d.ins_ev[evb + nins + io] = (uint32_t)(itok << 10) | ((uint32_t)(tk.olen - 1) << 8) | tk.bases;
        if (tk.kind == 3 && tk.err == 0) d.hasleft[gb + itok] = 1;
        if (ov) {
          const uint32_t slot = atomicAdd(d.ovf_cnt, 1u);
          if ((int64_t)slot < d.ovf_cap) {
            Ovf o; o.off = apos + sx + 1; o.read = (int32_t)r; o.gap = (int32_t)itok; o.len = (int32_t)tk.olen;
            o.pad[0] = o.pad[1] = o.pad[2] = 0;
            d.ovf[slot] = o;
          } else {
            atomicOr(&d.status[MPC_ST_FLAGS], DE_INTERNAL);
          }
        }
        const int tot = __shfl(pi, 63, 64);
        nodd += tot & 0xffff;
        nins += tot >> 16;
        uint32_t e = tk.err;
        for (int dd = 32; dd >= 1; dd >>= 1) e |= __shfl_xor(e, dd, 64);
        derr |= e;
        if (derr) break;
      }
      pos = reaches_end ? b1 : apos + tok[T - 1];
    }
    if (derr == 0 && dnlen > 0 && i > n) derr |= DE_INDEX;  // rightIndel(2*i) past the end
    if (l == 0) {
      int64_t ie = i < 0 ? 0 : (i > n ? n + 1 : i);
      d.i_end[r] = (int32_t)ie;
      d.odd_cnt[r] = derr ? 0 : (int32_t)nodd;
      d.ins_cnt[r] = derr ? 0 : (int32_t)nins;
      report(d, derr, r);
    }
  }
}

// ---------------------------------------------------------------------------
// Downstream (RIGHT) events.  A gap holding only RIGHT events needs only its
// longest downstream flank (slot bi = base bi, :64-72).  Gaps that also hold a
// LEFT event ("mixed") need the RIGHT events in read order -> sort keys.
// ---------------------------------------------------------------------------
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
    len = (int32_t)(d.down_off[r + 1] - d.down_off[r]);
    if (len > 0 && ie <= n) {
      g = d.gbase[s] + ie;
      mixed = d.hasleft[g] != 0;
    }
    const int64_t rg = d.read_offset + r;
    d.keys_in[r] = mixed ? (uint32_t)g : sentinel;
    d.vals_in[r] = (int32_t)rg;
    d.rlen[rg] = len;
  }
  peel_atomic_max(d.maxR, g < 0 ? 0 : g, len, in && g >= 0 && !mixed);
}

// right_start[g] = #mixed RIGHT events with gap < g ; also zero the run tables.
__global__ __launch_bounds__(256) void K_rstart(Dev d) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t <= d.G) d.right_start[t] = (int32_t)lower_bound_u32(d.keys_out, 0, d.Ng, (uint32_t)t);
  if (t == 0) {
    const int64_t nm = lower_bound_u32(d.keys_out, 0, d.Ng, (uint32_t)d.G);
    d.status[MPC_ST_MIXED] = (uint32_t)nm;
  }
}

__global__ __launch_bounds__(256) void K_zero_runs(Dev d) {
  const int64_t nruns = (int64_t)d.right_start[d.G] + d.G;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nruns; t += (int64_t)gridDim.x * blockDim.x) {
    d.M[t] = 0;
    uint4 z = make_uint4(0, 0, 0, 0);
    uint4* f = reinterpret_cast<uint4*>(d.F + t * 16);
    f[0] = z; f[1] = z; f[2] = z; f[3] = z;
  }
}

// run index of a LEFT event of global read rg at global gap g: runs of gap g
// are [right_start[g] + g, right_start[g+1] + g + 1); run k follows the k-th
// mixed RIGHT event (RIGHT of read r comes after r's own LEFT events, :303-323).
__device__ __forceinline__ int64_t run_of(const Dev& d, int64_t g, int64_t rg) {
  const int64_t lo = d.right_start[g], hi = d.right_start[g + 1];
  int64_t k = 0;
  if (hi > lo) k = lower_bound_i32(d.vals_out, lo, hi, (int32_t)rg) - lo;
  return lo + g + k;
}

// ---------------------------------------------------------------------------
// Tallies
// ---------------------------------------------------------------------------
// Read spans [tstart, min(i_end, n)) -> depth difference array.
__global__ __launch_bounds__(256) void K_spans(Dev d) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool act = false;
  int64_t a = 0, b = 0;
  if (r < d.N) {
    const int s = d.sample[r];
    const int64_t n = d.n_of[s];
    const int64_t ts = d.tstart[r];
    int64_t e = d.i_end[r];
    e = e > n ? n : e;
    if (ts >= 0 && ts < e) { act = true; a = d.gbase[s] + ts; b = d.gbase[s] + e; }
  }
  peel_atomic_add(d.diff, a, 1, act);
  peel_atomic_add(d.diff, b, -1, act);
  // upstream flank lengths -> M of the run the flank belongs to (LEFT event)
  bool up = false;
  int64_t run = 0;
  int32_t ul = 0;
  if (r < d.N) {
    const int s = d.sample[r];
    const int64_t n = d.n_of[s];
    const int64_t ts = d.tstart[r];
    ul = (int32_t)(d.up_off[r + 1] - d.up_off[r]);
    if (ul > 0 && ts >= 0 && ts <= n) { up = true; run = run_of(d, d.gbase[s] + ts, d.read_offset + r); }
  }
  peel_atomic_max(d.M, run, ul, up);
}

// substitutions + deletion diff points (one wave per read, lanes over events)
__global__ __launch_bounds__(256) void K_odd(Dev d) {
  const int l = lane();
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < d.N; r += stride) {
    const int cnt = d.odd_cnt[r];
    if (cnt == 0) continue;
    const int64_t gb = d.gbase[d.sample[r]];
    const int64_t eb = ev_base(d, r);
    for (int e = l; e < cnt; e += 64) {
      const uint32_t ev = d.odd_ev[eb + e];
      const int64_t g = gb + (ev >> 3);
      if (ev & 4u) atomicAdd(d.diff + g, (ev & 1u) ? 1 : -1);
      else atomicAdd(d.sub + g * 4 + (ev & 3u), 1u);
    }
  }
}

// insertions (<= kInsInline bases) -> M and right-justified tallies F of their run
__global__ __launch_bounds__(256) void K_left(Dev d) {
  const int l = lane();
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < d.N; r += stride) {
    const int cnt = d.ins_cnt[r];
    if (cnt == 0) continue;
    const int64_t gb = d.gbase[d.sample[r]];
    const int64_t eb = ev_base(d, r);
    const int64_t rg = d.read_offset + r;
    for (int e = l; e < cnt; e += 64) {
      const uint32_t ev = d.ins_ev[eb + e];
      const int64_t g = gb + (ev >> 10);
      const int L = (int)((ev >> 8) & 3u) + 1;
      const int64_t run = run_of(d, g, rg);
      atomicMax(d.M + run, L);
      for (int bi = 0; bi < L; ++bi) {  // bi counts from the 3' end (:55-61)
        const int code = (int)((ev >> (2 * (L - 1 - bi))) & 3u);
        atomicAdd(d.F + run * 16 + bi * 4 + code, 1u);
      }
    }
  }
  // long insertions only contribute their length here
  const int64_t nov = *d.ovf_cnt < (uint32_t)d.ovf_cap ? *d.ovf_cnt : d.ovf_cap;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nov; t += (int64_t)gridDim.x * blockDim.x) {
    const Ovf o = d.ovf[t];
    const int64_t g = d.gbase[d.sample[o.read]] + o.gap;
    atomicMax(d.M + run_of(d, g, d.read_offset + o.read), o.len);
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
  int64_t sidx = s0;
  for (; sidx < s1; ++sidx) {
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
  // sample of gap g: rows of a gap = its slots + the odd position after it (if any)
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
      asm volatile("" ::: "memory");
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
      asm volatile("" ::: "memory");
      for (int64_t k = l; k < cn; k += 64) {
        uint4 v = make_uint4(acc[k * 4], acc[k * 4 + 1], acc[k * 4 + 2], acc[k * 4 + 3]);
        reinterpret_cast<uint4*>(d.rows)[rb + c0 + k] = v;
        d.meta[rb + c0 + k] = (c0 + k == 0) ? 2 : 0;
      }
      asm volatile("" ::: "memory");
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
  for (int probe = 0; probe < 32; ++probe) {
    uint32_t k = keys[h];
    if (k == row) { atomicAdd(vals + h * 4 + code, 1u); return; }
    if (k == kEmpty) {
      const uint32_t prev = atomicCAS(keys + h, kEmpty, row);
      if (prev == kEmpty || prev == row) { atomicAdd(vals + h * 4 + code, 1u); return; }
    }
    h = (h + 1) & (kHash - 1);
  }
  atomicAdd(rows + (uint64_t)row * 4 + code, 1u);  // table full: go straight to HBM
}

__global__ __launch_bounds__(256) void K_strings(Dev d) {
  __shared__ uint32_t s_keys[kHash];
  __shared__ uint32_t s_vals[kHash * 4];
  if (d.status[MPC_ST_FLAGS] & DE_CAP) return;
  for (int k = threadIdx.x; k < kHash; k += blockDim.x) s_keys[k] = kEmpty;
  for (int k = threadIdx.x; k < kHash * 4; k += blockDim.x) s_vals[k] = 0;
  __syncthreads();
  const int l = lane(), w = threadIdx.x >> 6;
  uint32_t lerr = 0;
  int64_t lread = -1;
  // reads of this block: contiguous chunk
  const int64_t per = (d.N + gridDim.x - 1) / gridDim.x;
  const int64_t ra = (int64_t)blockIdx.x * per, rz = ra + per < d.N ? ra + per : d.N;
  for (int64_t r = ra + w; r < rz; r += 4) {
    const int s = d.sample[r];
    const int64_t n = d.n_of[s];
    const int64_t gb = d.gbase[s];
    const int64_t rg = d.read_offset + r;
    // upstream: LEFT at gap tstart, run k, slot = lo + hi_run - 1 - bi
    const int64_t u0 = d.up_off[r], u1 = d.up_off[r + 1];
    const int64_t ts = d.tstart[r];
    if (u1 > u0 && ts >= 0 && ts <= n) {
      const int64_t g = gb + ts;
      const int64_t run = run_of(d, g, rg);
      const int64_t base = (int64_t)d.row_base[g] + d.lo_f[g] + d.seg_hi[d.hscan[run] - 1] - 1;
      const int64_t L = u1 - u0;
      for (int64_t bi = l; bi < L; bi += 64) {
        const int c = base_code_exact(d.up[u1 - 1 - bi]);
        if (c < 0) { lerr |= DE_KEY; lread = r; continue; }
        hash_add(s_keys, s_vals, d.rows, (uint32_t)(base - bi), c);
      }
    }
    // downstream: RIGHT at gap i_end, slot = lo_f - lo_at + bi
    const int64_t v0 = d.down_off[r], v1 = d.down_off[r + 1];
    const int64_t ie = d.i_end[r];
    if (v1 > v0 && ie <= n) {
      const int64_t g = gb + ie;
      int64_t lo_at = 0;
      const int64_t a = d.right_start[g], b = d.right_start[g + 1];
      if (b > a) {  // mixed gap: find this read's RIGHT event
        const int64_t t = lower_bound_i32(d.vals_out, a, b, (int32_t)rg);
        lo_at = d.seg_lo[d.hscan[t + g] - 1];
      }
      const int64_t base = (int64_t)d.row_base[g] + d.lo_f[g] - lo_at;
      const int64_t L = v1 - v0;
      for (int64_t bi = l; bi < L; bi += 64) {
        const int c = base_code_exact(d.down[v0 + bi]);
        if (c < 0) { lerr |= DE_KEY; lread = r; continue; }
        hash_add(s_keys, s_vals, d.rows, (uint32_t)(base + bi), c);
      }
    }
  }
  // long insertions (grid-stride, LEFT like the short ones)
  const int64_t nov = *d.ovf_cnt < (uint32_t)d.ovf_cap ? *d.ovf_cnt : d.ovf_cap;
  for (int64_t t = blockIdx.x * 4 + w; t < nov; t += (int64_t)gridDim.x * 4) {
    const Ovf o = d.ovf[t];
    const int64_t g = d.gbase[d.sample[o.read]] + o.gap;
    const int64_t run = run_of(d, g, d.read_offset + o.read);
    const int64_t base = (int64_t)d.row_base[g] + d.lo_f[g] + d.seg_hi[d.hscan[run] - 1] - 1;
    for (int64_t bi = l; bi < o.len; bi += 64) {
      const int c = base_code(d.cs[o.off + o.len - 1 - bi]);
      hash_add(s_keys, s_vals, d.rows, (uint32_t)(base - bi), c < 0 ? 0 : c);
    }
  }
  if (lerr) report(d, lerr, lread);
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
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < R; row += (int64_t)gridDim.x * blockDim.x) {
    if (row >= need) { reinterpret_cast<uint4*>(d.res)[row] = make_uint4(0, 0, 0, 0); continue; }
    const uint4 cv = reinterpret_cast<const uint4*>(d.rows)[row];
    const uint32_t c[4] = {cv.x, cv.y, cv.z, cv.w};  // A, T, C, G
    const uint8_t mt = d.meta[row];
    const uint32_t total = c[0] + c[1] + c[2] + c[3];
    uint4 out = make_uint4(0, 0, 0, 0);
    if (total > 0) {
      // sorted(tuples in dict order, key=count)[::-1]: descending count, ties in
      // reverse dict order (stable sort then reverse, :371-374)
      int idx[4], m = 0;
      for (int k = 3; k >= 0; --k) if (c[k] > 0) idx[m++] = k;   // reverse dict order
      for (int a = 1; a < m; ++a) {                               // stable sort descending
        int t = idx[a], b = a - 1;
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
      if (mt & 2u) atomicMax(d.maxdepth + sample_of_row(d, row), total);  // slot 0 only (:336)
    }
    reinterpret_cast<uint4*>(d.res)[row] = out;
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
  int64_t N = 0, Ng = 0, G = 0, row_cap = 0, runs_cap = 0, ev_cap = 0, ovf_cap = 0;
  int32_t S = 0;
  uint32_t sentinel = 0;
  int end_bit = 0;
  size_t ws_bytes = 0;
  uint8_t* ws = nullptr;
  size_t off[64];
  size_t cub_sort = 0, cub_scan_runs = 0, cub_scan_g = 0, cub_scan_rows = 0, cub_tmp = 0;
  // buffer offsets (bytes)
  enum {
    B_STATUS, B_NOF, B_GBASE, B_IEND, B_ODDEV, B_ODDCNT, B_INSEV, B_INSCNT, B_OVF, B_OVFCNT,
    B_HASLEFT, B_MAXR, B_KIN, B_VIN, B_KOUT, B_VOUT, B_RLEN, B_RSTART, B_DIFF, B_SUB, B_M, B_F,
    B_HFLAG, B_HSCAN, B_SEGR, B_SEGLO, B_SEGHI, B_SEGRUN, B_LOF, B_ROWCNT, B_ROWBASE, B_DEPTH, B_ROWS,
    B_META, B_RES, B_KEEP, B_KEEPSCAN, B_CALLS, B_NCALLS, B_MAXD, B_CUB, B_COUNT
  };
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
  d.odd_ev = at<uint32_t>(this, B_ODDEV); d.odd_cnt = at<int32_t>(this, B_ODDCNT);
  d.ins_ev = at<uint32_t>(this, B_INSEV); d.ins_cnt = at<int32_t>(this, B_INSCNT);
  d.ovf = at<Ovf>(this, B_OVF); d.ovf_cnt = at<uint32_t>(this, B_OVFCNT); d.ovf_cap = ovf_cap;
  d.hasleft = at<uint8_t>(this, B_HASLEFT); d.maxR = at<int32_t>(this, B_MAXR);
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

static inline unsigned nblk(int64_t n, int b = 256) {
  int64_t g = (n + b - 1) / b;
  if (g < 1) g = 1;
  if (g > 65535 * 16) g = 65535 * 16;
  return (unsigned)g;
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
  if (p->Ng >= (1ll << 31)) { delete p; return fail(MPC_E_ARG, "too many reads"); }
  p->row_cap = row_cap > 0 ? row_cap : 1;
  p->runs_cap = p->Ng + p->G;
  p->ev_cap = in->cs_bytes + 2 * p->N + 16;
  p->ovf_cap = in->cs_bytes / 6 + 16;
  int eb = 1;
  while ((1ll << eb) <= p->G + 1) ++eb;
  p->end_bit = eb;
  p->sentinel = (uint32_t)((1ull << eb) - 1);
  // hipcub temp sizes
  {
    size_t t = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                       (int32_t*)nullptr, (int)std::max<int64_t>(p->Ng, 1), 0, eb);
    p->cub_sort = t;
    t = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, t, (int32_t*)nullptr, (int32_t*)nullptr, (int)p->runs_cap);
    p->cub_scan_runs = t;
    t = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, t, (int32_t*)nullptr, (int32_t*)nullptr, (int)p->G);
    p->cub_scan_g = t;
    t = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, (int32_t*)nullptr, (int32_t*)nullptr, (int)p->row_cap);
    p->cub_scan_rows = t;
    p->cub_tmp = std::max(std::max(p->cub_sort, p->cub_scan_runs), std::max(p->cub_scan_g, p->cub_scan_rows));
  }
  const int64_t N = p->N, Ng = p->Ng, G = p->G, R = p->row_cap, RU = p->runs_cap;
  auto set = [&](int b, int64_t count, size_t elem) { p->cnt[b] = count; p->sz[b] = (size_t)std::max<int64_t>(count, 1) * elem; };
  set(mpc_plan::B_STATUS, MPC_ST_WORDS, 4);
  set(mpc_plan::B_NOF, p->S, 4);
  set(mpc_plan::B_GBASE, p->S + 1, 4);
  set(mpc_plan::B_IEND, N, 4);
  set(mpc_plan::B_ODDEV, p->ev_cap, 4);
  set(mpc_plan::B_ODDCNT, N, 4);
  set(mpc_plan::B_INSEV, p->ev_cap, 4);
  set(mpc_plan::B_INSCNT, N, 4);
  set(mpc_plan::B_OVF, p->ovf_cap, sizeof(Ovf));
  set(mpc_plan::B_OVFCNT, 1, 4);
  set(mpc_plan::B_HASLEFT, G, 1);
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
  p->ws = (uint8_t*)ws;
  HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_NOF), p->h_n.data(), 4 * p->S, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(at<int32_t>(p, mpc_plan::B_GBASE), p->h_gbase.data(), 4 * (p->S + 1), hipMemcpyHostToDevice));
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
  std::vector<uint32_t> st0(MPC_ST_WORDS, 0);
  st0[MPC_ST_FIRST_READ] = 0xffffffffu;
  HIPCHK(hipMemcpyAsync(d.status, st0.data(), 4 * MPC_ST_WORDS, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(d.hasleft, 0, p->G, st));
  HIPCHK(hipMemsetAsync(d.ovf_cnt, 0, 4, st));
  if (p->N > 0) {
    unsigned grid = (unsigned)std::min<int64_t>((p->N + kParseWaves - 1) / kParseWaves, 256 * 32);
    hipLaunchKernelGGL(K_parse, dim3(grid), dim3(256), 0, st, d);
  }
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
  HIPCHK(hipMemsetAsync(d.diff, 0, 4 * p->G, st));
  HIPCHK(hipMemsetAsync(d.sub, 0, 16 * p->G, st));
  if (p->N > 0) {
    hipLaunchKernelGGL(K_spans, dim3(nblk(p->N)), dim3(256), 0, st, d);
    unsigned grid = (unsigned)std::min<int64_t>((p->N + 3) / 4, 256 * 32);
    hipLaunchKernelGGL(K_odd, dim3(grid), dim3(256), 0, st, d);
    hipLaunchKernelGGL(K_left, dim3(grid), dim3(256), 0, st, d);
  }
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
  unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((p->N + 255) / 256, 1024));
  hipLaunchKernelGGL(K_strings, dim3(grid), dim3(256), 0, st, d);
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
  // rows beyond the needed count hold garbage: K_call works on row_cap rows but
  // the assemble kernel wrote only ROWS_NEEDED; clear the tail once per call.
  hipLaunchKernelGGL(K_call, dim3(nblk(R)), dim3(256), 0, st, d, R);
  hipLaunchKernelGGL(K_keep, dim3(nblk(R)), dim3(256), 0, st, d, R);
  uint8_t* tmp = at<uint8_t>(p, mpc_plan::B_CUB);
  size_t tb = p->cub_tmp;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, d.keep, d.keep_scan, (int)R, st));
  hipLaunchKernelGGL(K_emit, dim3(nblk(R)), dim3(256), 0, st, d, R);
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
