// Device helpers shared by the gfx950 kernels (wave64 idioms, base codes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpc {

constexpr int kWave = 64;

__device__ __forceinline__ int lane() { return (int)(threadIdx.x & 63); }

// Dict order of the reference's slot dicts {'A','T','C','G'} (:59, :70): A0 T1 C2 G3.
__device__ __forceinline__ int base_code(uint32_t c) {
  switch (c) {
    case 'A': case 'a': return 0;
    case 'T': case 't': return 1;
    case 'C': case 'c': return 2;
    case 'G': case 'g': return 3;
  }
  return -1;
}
// Exact-case variant for strings the reference does NOT upper-case (flanks are
// upper-cased at ingest, :270; the reference base is upper-cased at :165).
__device__ __forceinline__ int base_code_exact(uint32_t c) {
  switch (c) {
    case 'A': return 0; case 'T': return 1; case 'C': return 2; case 'G': return 3;
  }
  return -1;
}

// SPECIAL_CHARS of the tokenizer (:290)
__device__ __forceinline__ bool is_special(uint32_t c) {
  return c == ':' || c == '*' || c == '+' || c == '-' || c == 'Z';
}

template <class T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int l = lane();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T t = __shfl_up(v, d, 64);
    if (l >= d) v += t;
  }
  return v;
}

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

template <class T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    T o = __shfl_xor(v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}

// ---- DPP wave64 scans (gfx9 row_shr / row_bcast; no LDS, no bpermute) ----
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, BANK_MASK, true);
}
// inclusive prefix sum over the 64 lanes (Kogge-Stone inside 16-lane rows, then
// row_bcast:15 / row_bcast:31 to carry row totals)
__device__ __forceinline__ int wave_scan_i32(int x) {
  x += dpp_i32<0x111>(x);        // row_shr:1
  x += dpp_i32<0x112>(x);        // row_shr:2
  x += dpp_i32<0x114>(x);        // row_shr:4
  x += dpp_i32<0x118>(x);        // row_shr:8
  x += dpp_i32<0x142, 0xa>(x);   // row_bcast:15 -> rows 1, 3
  x += dpp_i32<0x143, 0xc>(x);   // row_bcast:31 -> rows 2, 3
  return x;
}
// inclusive max-scan for x >= 0 (lanes outside a row / broadcast read 0)
__device__ __forceinline__ int wave_scan_max_i32(int x) {
  x = max(x, dpp_i32<0x111>(x));
  x = max(x, dpp_i32<0x112>(x));
  x = max(x, dpp_i32<0x114>(x));
  x = max(x, dpp_i32<0x118>(x));
  x = max(x, dpp_i32<0x142, 0xa>(x));
  x = max(x, dpp_i32<0x143, 0xc>(x));
  return x;
}
__device__ __forceinline__ int wave_last_i32(int x) { return __builtin_amdgcn_readlane(x, 63); }
__device__ __forceinline__ int uniform_i32(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t ballot(bool p) { return (uint64_t)__ballot(p ? 1 : 0); }

// Python str.strip() whitespace restricted to ASCII (the only bytes that can
// appear inside a tab-separated, rstrip()ed PAF field).
__device__ __forceinline__ bool py_space(uint32_t c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0b || c == 0x0c || (c >= 0x1c && c <= 0x1f);
}

// int(operand) of processOperation ':' (:77) in base 10 on ASCII bytes:
// optional surrounding whitespace, optional sign, digits with single '_'
// separators.  Saturates at 2^40 (any value that large hits IndexError first).
// Returns false on ValueError.
template <class P>
__device__ __forceinline__ bool py_int(P p, int64_t len, int64_t* out) {
  int64_t a = 0, b = len;
  // fast path: plain digits
  bool plain = len > 0 && len <= 12;
  int64_t v = 0;
  for (int64_t k = 0; plain && k < len; ++k) {
    uint32_t c = p[k];
    if (c >= '0' && c <= '9') v = v * 10 + (c - '0');
    else plain = false;
  }
  if (plain) { *out = v; return true; }
  while (a < b && py_space(p[a])) ++a;
  while (b > a && py_space(p[b - 1])) --b;
  bool neg = false;
  if (a < b && (p[a] == '+' || p[a] == '-')) { neg = p[a] == '-'; ++a; }
  if (a >= b) return false;
  v = 0;
  bool prev_digit = false;
  const int64_t cap = (int64_t)1 << 40;
  for (int64_t k = a; k < b; ++k) {
    uint32_t c = p[k];
    if (c >= '0' && c <= '9') {
      v = v < cap ? v * 10 + (c - '0') : cap;
      prev_digit = true;
    } else if (c == '_' && prev_digit && k + 1 < b && p[k + 1] >= '0' && p[k + 1] <= '9') {
      prev_digit = false;
    } else {
      return false;
    }
  }
  if (!prev_digit) return false;
  *out = neg ? -v : v;
  return true;
}

// Wave-aggregated atomicMax / atomicAdd for keys that repeat across lanes
// (hot gaps: every full-length read starts at gap 0 and ends at gap n).
__device__ __forceinline__ void peel_atomic_max(int32_t* base, int64_t key, int32_t val, bool active) {
  uint64_t act = ballot(active);
  while (act) {
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int64_t k = __shfl(key, leader, 64);
    const bool same = active && key == k;
    const uint64_t m = ballot(same);
    int32_t v = wave_max(same ? val : INT32_MIN);
    if (lane() == leader) atomicMax(base + k, v);
    if (same) active = false;
    act &= ~m;
  }
}

__device__ __forceinline__ void peel_atomic_add(int32_t* base, int64_t key, int32_t val, bool active) {
  uint64_t act = ballot(active);
  while (act) {
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int64_t k = __shfl(key, leader, 64);
    const bool same = active && key == k;
    const uint64_t m = ballot(same);
    int32_t v = wave_sum(same ? val : 0);
    if (lane() == leader && v != 0) atomicAdd(base + k, v);
    if (same) active = false;
    act &= ~m;
  }
}

// Block-aggregated atomicMax for keys that repeat across a whole block (hot
// gaps: thousands of reads start at gap 0 / end at gap n).  Same-address global
// atomics serialize at the memory side (~12 ns each), so the block's first
// thread's key is reduced in LDS and flushed with ONE atomic; other keys go
// through the wave-aggregated path.  Every thread of the block must call it.
__device__ __forceinline__ void block_atomic_max(int32_t* base, int64_t key, int32_t val, bool active,
                                                 int64_t* s_key, int32_t* s_val) {
  __syncthreads();
  if (threadIdx.x == 0) { *s_key = active ? key : -1; *s_val = INT32_MIN; }
  __syncthreads();
  const bool mine = active && key == *s_key;
  if (mine) atomicMax(s_val, val);
  peel_atomic_max(base, key, val, active && !mine);
  __syncthreads();
  if (threadIdx.x == 0 && *s_key >= 0 && *s_val != INT32_MIN) atomicMax(base + *s_key, *s_val);
}

// number of entries < x in sorted a[lo, hi)
__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* a, int64_t lo, int64_t hi, int32_t x) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int64_t lower_bound_u32(const uint32_t* a, int64_t lo, int64_t hi, uint32_t x) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

}  // namespace mpc
