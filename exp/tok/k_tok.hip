// Prototype pass 1 of a split parse: a streaming cs tokenizer
// that writes the unit stream K_parse decodes in its rounds, as one 4-byte
// word per unit (format: exp/tok/tok_ref.c, its checker).  Experiment only:
// nothing in the package, the tests or bench.py loads it.
//
// One wave per contiguous byte range of S bytes (S a multiple of 1 KiB), in
// steps of 1 KiB (16 bytes per lane).  Per step: special-byte bits by v_perm
// lookups, read-start bits from one coalesced load of the read offsets, both
// in a per-wave LDS bit array with a 64-byte halo; then each lane walks the
// token starts it owns (count pass, wave scan, write pass).  Token ends /
// successors come from the bit array (or a global scan past the halo), the
// operand bytes from the step's bytes staged in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mpc_device.h"  // DPP wave scans of the product kernels

namespace {
constexpr int kStep = 1024;
constexpr int kWords = 34;  // 32-bit token-start words per step: 1 KiB + a 64-byte halo
constexpr int kWaves = 4;   // waves per block

using mpc::lane;
__device__ __forceinline__ uint32_t from_lane_below(uint32_t x) {  // lane l - 1's x (lane 0: 0), DPP wave_shr:1
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t bcast(uint32_t x, int src) { return (uint32_t)__builtin_amdgcn_readlane((int)x, src); }
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t hit_nibble(uint32_t z) {
  z >>= 7;
  z |= z >> 7;
  z |= z >> 14;
  return z & 0xfu;
}
// bit k: byte k of the 16 is special (':' 'Z' '*' '+' '-'), by two v_perm
// table lookups per word (lo nibble >= 8 selects the table row, the high
// nibble a bit of it)
__device__ __forceinline__ uint32_t special16(uint4 d) {
  const uint32_t w[4] = {d.x, d.y, d.z, d.w};
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t c = w[i];
    const uint32_t t1 = __builtin_amdgcn_perm(0x00000400u, 0x042C0000u, c & 0x07070707u);
    const uint32_t t2 = __builtin_amdgcn_perm(0x80402010u, 0x08040201u, (c >> 4) & 0x07070707u);
    const uint32_t y = t1 & t2;
    const uint32_t ok = (c << 4) & ~c;
    s |= hit_nibble((y + 0x7F7F7F7Fu) & ok & 0x80808080u) << (4 * i);
  }
  return s;
}
using mpc::is_special;
__device__ __forceinline__ uint32_t opcode(uint32_t c) {
  return c == ':' ? 0u : c == '*' ? 1u : c == '+' ? 2u : c == '-' ? 3u : c == 'Z' ? 4u : 5u;
}
// 8 bytes starting at cs + p (two aligned loads; cs is padded past its end)
__device__ __forceinline__ uint64_t load8(const uint8_t* cs, int64_t p) {
  const int64_t a = p & ~(int64_t)7;
  const uint64_t w0 = *reinterpret_cast<const uint64_t*>(cs + a);
  const uint64_t w1 = *reinterpret_cast<const uint64_t*>(cs + a + 8);
  const int sh = (int)(p & 7) * 8;
  return sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
}
// ':' operand (bytes (s, e), v = the 8 bytes after s) as a number, 16383 = escape
__device__ __forceinline__ uint32_t colon_value(uint64_t v, int64_t s, int64_t e) {
  const int64_t nd = e - s - 1;
  if (nd < 1 || nd > 8) return 16383u;
  uint32_t x = 0;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t c = (uint32_t)(v >> (8 * k)) & 0xffu;
    if (k < nd) {
      ok = ok && c - '0' <= 9u;
      x = x * 10u + (c - '0');
    }
  }
  return ok && x < 16383u ? x : 16383u;
}
__device__ __forceinline__ uint32_t op_fields(uint64_t v, int64_t s, int64_t e) {
  const int64_t ol = e - s - 1;
  uint32_t pay = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < ol) pay |= (uint32_t)((v >> (8 * k + 1)) & 3u) << (2 * k);
  return (uint32_t)(ol > 63 ? 63 : ol) << 4 | pay << 10;
}

// special byte by one 64-bit mask lookup (':' '+' '-' '*' < 64) or 'Z'
__device__ __forceinline__ bool special_lut(uint32_t c) {
  constexpr uint64_t kSp = (1ull << ':') | (1ull << '+') | (1ull << '-') | (1ull << '*');
  return c < 64 ? (kSp >> c) & 1ull : c == 'Z';
}
// ':' operand of nd bytes (v: its first 8) as a number, 16383 = escape: SWAR
// digit check and three multiply-add folds (pairs, quads, the 8 digits)
__device__ __forceinline__ uint32_t colon_swar(uint64_t v, int nd) {
  if (nd < 1 || nd > 8) return 16383u;
  const uint64_t m = nd == 8 ? ~0ull : (1ull << (8 * nd)) - 1ull;
  const uint64_t t = v ^ 0x3030303030303030ull;  // digit bytes -> 0..9
  if ((((t + 0x7676767676767676ull) | t) & 0x8080808080808080ull & m) != 0) return 16383u;
  uint64_t y = (t & m) << (8 * (8 - nd));  // right-aligned: leading zero digits
  y = (y * 10 + (y >> 8)) & 0x00FF00FF00FF00FFull;
  y = (y * 100 + (y >> 16)) & 0x0000FFFF0000FFFFull;
  y = (y * 10000 + (y >> 32)) & 0xFFFFFFFFull;
  return y < 16383u ? (uint32_t)y : 16383u;
}
__device__ __forceinline__ uint32_t op_fields_swar(uint64_t v, int ol) {
  const uint32_t p = ((uint32_t)v >> 1) & 0x03030303u;
  const uint32_t pay = (p | p >> 6 | p >> 12 | p >> 18) & (ol >= 4 ? 0xffu : (1u << (2 * (ol > 0 ? ol : 0))) - 1u);
  return (uint32_t)(ol > 63 ? 63 : ol) << 4 | pay << 10;
}

struct TokArgs {
  const uint8_t* cs; int64_t B;
  const int64_t* cs_off; int64_t N;
  const int64_t* wave_rn;  // per wave: first read with cs_off >= its first byte (host lower_bound)
  int64_t S, nwaves;
  uint32_t* units; uint32_t* wcount;
};

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// (v of the token before the step, for a ':' that the step's first unit absorbs)
struct Carry { uint32_t op, rs, val; int64_t pos; bool have_val; };

#ifndef TOK_WPE
#define TOK_WPE 4
#endif
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(TOK_WPE))) void K_tok(TokArgs a) {
  constexpr int kStaged = 32 * kWords;                 // staged bytes: the step + a 64-byte halo
  __shared__ uint32_t s_rs[kWaves][kWords];             // read-start bits of the staged bytes
  __shared__ uint64_t s_by[kWaves][(kStaged + 16) / 8];  // the staged bytes (+ load8 overrun)
  __shared__ uint16_t s_list[kWaves][kStaged];           // token starts (step offsets), ascending
  const int l = lane(), wi = (int)threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * kWaves + wi;
  if (w >= a.nwaves) return;
  uint32_t* rsb = s_rs[wi];
  uint8_t* by = reinterpret_cast<uint8_t*>(s_by[wi]);
  uint16_t* list = s_list[wi];
  const int64_t begin = w * a.S, end = begin + a.S < a.B ? begin + a.S : a.B;
  int64_t rn = a.wave_rn[w];
  // the token before `begin`: the last special byte within 32 bytes, or the
  // last read start if later (a longer token cannot be an absorbable ':')
  Carry c{0u, 0u, 0u, -1, true};
  {
    const int64_t p = begin - 1 - l;
    const uint64_t m = __ballot(l < 32 && p >= 0 && is_special(a.cs[p]));
    int64_t pq = m ? begin - 1 - __builtin_ctzll(m) : -1;
    const int64_t ro = rn > 0 ? a.cs_off[rn - 1] : -1;
    if (ro > pq) pq = ro;
    if (pq >= begin - 32 && pq >= 0) {
      c.pos = pq;
      c.op = a.cs[pq];
      c.rs = ro == pq;
      c.have_val = false;  // decoded from global memory by the first round
    }
  }
  uint32_t cnt = 0;
  uint32_t* out = a.units + w * a.S;
  // software pipeline: the next step's bytes and read offsets are loaded while
  // this step is tokenized
  uint4 dn = *reinterpret_cast<const uint4*>(a.cs + begin + 16 * l), dhn = make_uint4(0, 0, 0, 0);
  if (l < 5) dhn = *reinterpret_cast<const uint4*>(a.cs + begin + kStep + 16 * l);
  int64_t con = rn + l < a.N ? a.cs_off[rn + l] : INT64_MAX;
  for (int64_t A = begin; A < end; A += kStep) {
    // ---- stage the bytes; special-byte bits per 16-byte chunk (chunks 64..67: halo) ----
    const uint4 d = dn, dh = dhn;
    if (A + kStep < end) {
      dn = *reinterpret_cast<const uint4*>(a.cs + A + kStep + 16 * l);
      if (l < 5) dhn = *reinterpret_cast<const uint4*>(a.cs + A + 2 * kStep + 16 * l);
    }
    reinterpret_cast<uint4*>(by)[l] = d;
    uint32_t sp = special16(d);
    if (A + 16 * l + 16 > a.B) sp &= (A + 16 * l >= a.B) ? 0u : (1u << (a.B - A - 16 * l)) - 1u;
    uint32_t sph = 0;
    if (l < 5) {  // halo (lanes 0-3) and the overrun pad (lane 4)
      const int64_t h = A + kStep + 16 * l;
      reinterpret_cast<uint4*>(by)[64 + l] = dh;
      if (l < 4) {
        sph = special16(dh);
        if (h + 16 > a.B) sph &= (h >= a.B) ? 0u : (1u << (a.B - h)) - 1u;
      }
    }
    if (l < kWords) rsb[l] = 0;
    wave_sync_lds();
    for (bool first = true;; first = false) {  // read starts in the staged bytes, 64 offsets at a time
      const int64_t r = rn + l;
      const int64_t co = first ? con : r < a.N ? a.cs_off[r] : INT64_MAX;
      if (co < A + kStaged && co < a.B) {
        const int q = (int)(co - A);
        atomicOr(&rsb[q >> 5], 1u << (q & 31));
      }
      const int nb = __popcll(__ballot(co < A + kStep));
      rn += nb;
      if (nb < 64) break;
    }
    con = rn + l < a.N ? a.cs_off[rn + l] : INT64_MAX;  // the next step's first 64 offsets
    wave_sync_lds();
    const uint32_t tk = sp | ((rsb[l >> 1] >> (16 * (l & 1))) & 0xffffu);
    const uint32_t tkh = l < 4 ? sph | ((rsb[32 + (l >> 1)] >> (16 * (l & 1))) & 0xffffu) : 0u;
    // ---- token list: own chunks in lane order, then the halo chunks ----
    const uint32_t n_c = __popc(tk), n_h = __popc(tkh);
    const uint32_t inc = (uint32_t)mpc::wave_scan_i32((int)n_c), inch = (uint32_t)mpc::wave_scan_i32((int)n_h);
    const uint32_t n_step = bcast(inc, 63), n_list = n_step + bcast(inch, 3);
    {
      uint32_t k = inc - n_c;
      for (uint32_t m = tk; m; m &= m - 1) list[k++] = (uint16_t)(16 * l + __builtin_ctz(m));
      k = n_step + inch - n_h;
      for (uint32_t m = tkh; m; m &= m - 1) list[k++] = (uint16_t)(kStep + 16 * l + __builtin_ctz(m));
    }
    // owned tokens: starts below end
    const int64_t lim = end - A;  // > 0
    const uint32_t below_end = lim >= kStep ? n_c : __popc(tk & (16 * l >= lim ? 0u : 16 * l + 16 <= lim ? 0xffffu : (1u << (lim - 16 * l)) - 1u));
    const uint32_t n_own = bcast((uint32_t)mpc::wave_scan_i32((int)below_end), 63);
    wave_sync_lds();
    // ---- rounds: one token per lane ----
    uint32_t nout = 0;
    for (uint32_t j0 = 0; j0 < n_own; j0 += 64) {
      const uint32_t j = j0 + l;
      const bool valid = j < n_own;
      const int s = valid ? list[j] : 0;
      const bool has_nx = j + 1 < n_list;
      const int eq = has_nx ? (int)list[j + 1] : kStaged;  // successor, step offset
      const uint32_t op = by[s];
      const uint32_t rs = (rsb[s >> 5] >> (s & 31)) & 1u;
      uint32_t nx = has_nx ? (uint32_t)by[eq] : 0u;      // zero padding past B: not special
      uint32_t rs_e = has_nx ? (rsb[eq >> 5] >> (eq & 31)) & 1u : 0u;
      int len = eq - s - 1;                               // operand bytes
      if (__ballot(valid && !has_nx)) {  // rare, wave-uniform: no start in the rest of the staged bytes
        if (valid && !has_nx) {
          int64_t p = A + kStaged, rr = rn;
          while (rr < a.N && a.cs_off[rr] < p) ++rr;
          const int64_t nr = rr < a.N ? a.cs_off[rr] : INT64_MAX;
          while (p < a.B && p < nr && !is_special(a.cs[p])) ++p;
          const int64_t e = p < a.B ? p : a.B;
          const int64_t ol = e - (A + s) - 1;
          len = ol > 0x3fffffff ? 0x3fffffff : (int)ol;
          nx = e < a.B ? (uint32_t)a.cs[e] : 0u;
          rs_e = e < a.B && e == nr;
        }
      }
      const uint64_t v = load8(reinterpret_cast<const uint8_t*>(by), s + 1);  // the operand's first 8 bytes
      const bool colon = op == ':', spc = special_lut(op);
      const uint32_t v_self = colon ? colon_swar(v, len) : 0u;
      // the previous token: lane l - 1, else the carry
      uint32_t op_p = from_lane_below(op), rs_p = from_lane_below(rs), v_p = from_lane_below(v_self);
      if (l == 0) {
        if (!c.have_val && c.op == ':') c.val = colon_value(load8(a.cs, c.pos + 1), c.pos, A + s);
        c.have_val = true;
        op_p = c.op; rs_p = c.rs; v_p = c.val;
      }
      // branch-free unit word (tok_ref.c)
      const bool merged = !colon && spc && op_p == ':' && !rs;
      const bool absorbed = colon && special_lut(nx) && nx != ':' && !rs_e;
      const bool emit = valid && !absorbed;
      const uint32_t w_colon = rs << 3 | v_self << 18;
      const uint32_t w_op = opcode(op) | (merged ? rs_p : rs) << 3 | op_fields_swar(v, len) | (merged ? v_p : 0u) << 18;
      const uint32_t w_none = 5u | rs << 3 | (uint32_t)min(len + 1, 63) << 4;
      const uint32_t word = colon ? w_colon : spc ? w_op : w_none;
      const uint64_t em = __ballot(emit);
      if (emit) out[cnt + nout + lanes_below(em)] = word;  // contiguous across the round's lanes
      nout += __popcll(em);
      // carry to the next round / step: the round's last valid token
      const int lastl = (int)(n_own - 1 - j0 < 63 ? n_own - 1 - j0 : 63);
      c.op = bcast(op, lastl);
      c.rs = bcast(rs, lastl);
      c.val = bcast(v_self, lastl);
      c.have_val = true;
    }
    cnt += nout;
    wave_sync_lds();
  }
  if (l == 0) a.wcount[w] = cnt;
}
}  // namespace

extern "C" int tok_launch(const uint8_t* cs, int64_t B, const int64_t* cs_off, int64_t N, const int64_t* wave_rn,
                          int64_t S, int64_t nwaves, uint32_t* units, uint32_t* wcount, void* stream) {
  TokArgs t{cs, B, cs_off, N, wave_rn, S, nwaves, units, wcount};
  const int64_t blocks = (nwaves + kWaves - 1) / kWaves;
  hipLaunchKernelGGL(K_tok, dim3((unsigned)blocks), dim3(kWaves * 64), 0, (hipStream_t)stream, t);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
