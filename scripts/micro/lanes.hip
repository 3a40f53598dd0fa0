// Micro-benchmark: can one-lane-per-read token walking stream cs at HBM rates?
//   lanes [n_reads] [mean_len]
// Synthetic "cs" = reads of random length around mean_len, tokens of 2-9 bytes
// (special byte + digits).  Each kernel walks every read token by token and
// sums the token lengths (checksum = total bytes, verified).
//   K_direct   lane per read, one 16-B global load per token (serial chain)
//   K_ring     lane per read, LDS ring per lane filled at wave-uniform
//              maintenance points every R tokens (loads land one period later)
//   K_stream   coalesced wave streaming of the whole buffer (bandwidth roof)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t spec_bits(uint32_t w) {  // bit 7 of each byte: byte >= 0x80 ("special")
  return w & 0x80808080u;
}

__global__ __launch_bounds__(256) void K_direct(const uint8_t* cs, const int64_t* off, int64_t n, unsigned long long* out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t sum = 0;
  if (r < n) {
    int64_t p = off[r];
    const int64_t e = off[r + 1];
    while (p < e) {
      const int64_t A = p & ~3ll;
      const uint4 v = *reinterpret_cast<const uint4*>(cs + A);
      const uint32_t sh = (uint32_t)(p - A);
      const uint32_t x0 = __builtin_amdgcn_alignbyte(v.y, v.x, sh), x1 = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
      uint64_t m = ((uint64_t)spec_bits(x1) << 32 | spec_bits(x0)) & ~0x80ull;  // skip own op byte
      const int t = m ? (__builtin_ctzll(m) >> 3) : 8;
      const int len = (int)min<int64_t>(t, e - p);
      sum += len;
      p += len;
    }
  }
  atomicAdd(out, (unsigned long long)sum);
}

// ring: per lane 2 chunks of 32 B + 16 B mirror (20 dwords, stride 21)
template <int R>
__global__ __launch_bounds__(512) void K_ring(const uint8_t* cs, const int64_t* off, int64_t n, unsigned long long* out) {
  __shared__ uint32_t ring[8][64 * 21];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  uint32_t* rg = ring[w] + 21 * l;
  const int64_t r = (int64_t)blockIdx.x * 512 + threadIdx.x;
  uint64_t sum = 0;
  int64_t p = 0, e = 0, F = 0;  // F: absolute end of ring data (16-aligned)
  bool act = r < n;
  if (act) { p = off[r]; e = off[r + 1]; }
  int64_t base = p & ~15ll;  // ring holds [F - 64, F) mapped at (x - base) mod 64
  // initial fill: 64 B
  uint4 pend0 = make_uint4(0, 0, 0, 0), pend1 = pend0;
  if (act) {
    const uint4* s = reinterpret_cast<const uint4*>(cs + base);
    const uint4 a = s[0], b = s[1], c = s[2], d = s[3];
    uint32_t* q = rg;
    q[0] = a.x; q[1] = a.y; q[2] = a.z; q[3] = a.w; q[4] = b.x; q[5] = b.y; q[6] = b.z; q[7] = b.w;
    q[8] = c.x; q[9] = c.y; q[10] = c.z; q[11] = c.w; q[12] = d.x; q[13] = d.y; q[14] = d.z; q[15] = d.w;
    q[16] = a.x; q[17] = a.y; q[18] = a.z; q[19] = a.w;
    F = base + 64;
    pend0 = s[4]; pend1 = s[5];  // next 32 B in flight
  }
  bool pend_ok = act;
  while (__builtin_amdgcn_read_exec() && __ballot(act)) {
    for (int it = 0; it < R; ++it) {
      if (act && F - p >= 16) {
        const int64_t rel = p - base;            // ring offset of p: rel mod 64
        const int ro = (int)(rel & 63);
        const int dw = ro >> 2, sh = ro & 3;
        const uint32_t d0 = rg[dw], d1 = rg[dw + 1], d2 = rg[dw + 2];
        const uint32_t x0 = __builtin_amdgcn_alignbyte(d1, d0, sh), x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
        uint64_t m = ((uint64_t)spec_bits(x1) << 32 | spec_bits(x0)) & ~0x80ull;
        const int t = m ? (__builtin_ctzll(m) >> 3) : 8;
        const int len = (int)min<int64_t>(t, e - p);
        sum += len;
        p += len;
        if (p >= e) act = false;
      }
    }
    // maintenance: write the pending 32 B if the ring has room, then load the next 32 B
    if (pend_ok && F + 32 - p <= 64 + 0) {
      const int ro = (int)((F - base) & 63);  // 0 or 32
      uint32_t* q = rg + (ro >> 2);
      q[0] = pend0.x; q[1] = pend0.y; q[2] = pend0.z; q[3] = pend0.w;
      q[4] = pend1.x; q[5] = pend1.y; q[6] = pend1.z; q[7] = pend1.w;
      if (ro == 0) { rg[16] = pend0.x; rg[17] = pend0.y; rg[18] = pend0.z; rg[19] = pend0.w; }
      F += 32;
      pend_ok = F < e + 16;
      if (pend_ok) {
        const uint4* s = reinterpret_cast<const uint4*>(cs + F);
        pend0 = s[0]; pend1 = s[1];
      }
    }
  }
  atomicAdd(out, (unsigned long long)sum);
}

__global__ __launch_bounds__(256) void K_stream(const uint8_t* cs, int64_t bytes, unsigned long long* out) {
  uint64_t sum = 0;
  for (int64_t x = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 16; x < bytes; x += (int64_t)gridDim.x * 256 * 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(cs + x);
    sum += __popc(spec_bits(v.x)) + __popc(spec_bits(v.y)) + __popc(spec_bits(v.z)) + __popc(spec_bits(v.w));
  }
  atomicAdd(out, (unsigned long long)sum);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const int mean = argc > 2 ? atoi(argv[2]) : 1200;
  std::mt19937_64 g(1);
  std::vector<int64_t> off(n + 1, 0);
  for (int64_t r = 0; r < n; ++r) off[r + 1] = off[r] + mean / 2 + (int64_t)(g() % (uint64_t)mean);
  const int64_t bytes = off[n];
  std::vector<uint8_t> cs(bytes + 4096, 0x81);
  for (int64_t r = 0; r < n; ++r) {
    int64_t p = off[r];
    while (p < off[r + 1]) {
      cs[p] = 0x80 | (g() & 3);
      const int t = 2 + (int)(g() % 8);
      for (int k = 1; k < t && p + k < off[r + 1]; ++k) cs[p + k] = '0' + (g() % 10);
      p += t;
    }
  }
  uint8_t* dcs; int64_t* doff; unsigned long long* dout;
  CK(hipMalloc(&dcs, cs.size())); CK(hipMalloc(&doff, 8 * (n + 1))); CK(hipMalloc(&dout, 8));
  CK(hipMemcpy(dcs, cs.data(), cs.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(doff, off.data(), 8 * (n + 1), hipMemcpyHostToDevice));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch, bool check) {
    for (int k = 0; k < 2; ++k) launch();
    CK(hipMemset(dout, 0, 8));
    launch();
    unsigned long long s = 0; CK(hipMemcpy(&s, dout, 8, hipMemcpyDeviceToHost));
    CK(hipEventRecord(a)); for (int k = 0; k < 5; ++k) launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 5;
    printf("%-10s %9.1f us  %8.1f GB/s  %s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
           check ? (s == (unsigned long long)bytes ? "ok" : "CHECKSUM MISMATCH") : "");
  };
  printf("reads %lld mean %d bytes %lld\n", (long long)n, mean, (long long)bytes);
  run("direct", [&] { hipLaunchKernelGGL(K_direct, dim3((n + 255) / 256), dim3(256), 0, 0, dcs, doff, n, dout); }, true);
  run("ring R=1", [&] { hipLaunchKernelGGL(K_ring<1>, dim3((n + 511) / 512), dim3(512), 0, 0, dcs, doff, n, dout); }, true);
  run("ring R=2", [&] { hipLaunchKernelGGL(K_ring<2>, dim3((n + 511) / 512), dim3(512), 0, 0, dcs, doff, n, dout); }, true);
  run("ring R=3", [&] { hipLaunchKernelGGL(K_ring<3>, dim3((n + 511) / 512), dim3(512), 0, 0, dcs, doff, n, dout); }, true);
  run("stream", [&] { hipLaunchKernelGGL(K_stream, dim3(8192), dim3(256), 0, 0, dcs, bytes, dout); }, false);
  return 0;
}
