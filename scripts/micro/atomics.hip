// Micro-benchmark: cost of device-scope global atomics patterns on MI355X (design input for the
// flush / reduction strategy of the pileup kernels).  hipcc --offload-arch=gfx950 -O3 atomics.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void flush_same(uint32_t* dst, int n, int copies) {
  uint32_t* d = dst + (size_t)(blockIdx.x % copies) * n;
  for (int p = threadIdx.x; p < n; p += blockDim.x) atomicAdd(d + p, 1u + (p & 1));
}
__global__ void flush_store(uint32_t* dst, int n) {
  uint32_t* d = dst + (size_t)blockIdx.x * n;
  for (int p = threadIdx.x; p < n; p += blockDim.x) d[p] = 1u + (p & 1);
}
__global__ void reduce_cols(const uint32_t* src, uint32_t* dst, int n, int rows) {
  int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint32_t s = 0;
  for (int r = 0; r < rows; ++r) s += src[(size_t)r * n + p];
  dst[p] = s;
}
__global__ void spread(uint32_t* dst, int n, int per_thread, uint32_t seed) {
  uint32_t x = seed ^ (blockIdx.x * 977 + threadIdx.x * 131);
  for (int k = 0; k < per_thread; ++k) {
    x = x * 1664525u + 1013904223u;
    atomicAdd(dst + (x >> 8) % n, 1u);
  }
}
__global__ void one_addr(uint32_t* dst, int per_wave) {
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < per_wave; ++k) atomicMax(dst, blockIdx.x * 4 + (threadIdx.x >> 6) + k);
}
__global__ void lds_hot(uint32_t* dst, int iters, int naddr) {
  __shared__ uint32_t h[4096];
  for (int k = threadIdx.x; k < 4096; k += blockDim.x) h[k] = 0;
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u;
  for (int k = 0; k < iters; ++k) { x = x * 1664525u + 1013904223u; atomicAdd(h + (x >> 8) % naddr, 1u); }
  __syncthreads();
  if (threadIdx.x == 0) dst[blockIdx.x] = h[0];
}

template <class F>
float timeit(F f, int reps = 5) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  uint32_t* buf; hipMalloc(&buf, 256u << 20); hipMemset(buf, 0, 256u << 20);
  const int n = 2687 * 5;
  for (int blocks : {256, 512}) for (int copies : {1, 8, 32})
    printf("flush_same blocks=%d n=%d copies=%d: %.1f us\n", blocks, n, copies,
           timeit([&] { hipLaunchKernelGGL(flush_same, dim3(blocks), dim3(512), 0, 0, buf, n, copies); }));
  printf("flush_store 512 blocks: %.1f us\n", timeit([&] { hipLaunchKernelGGL(flush_store, dim3(512), dim3(512), 0, 0, buf, n); }));
  printf("reduce 512 rows: %.1f us\n", timeit([&] { hipLaunchKernelGGL(reduce_cols, dim3((n + 255) / 256), dim3(256), 0, 0, buf, buf + 512 * n, n, 512); }));
  for (int naddr : {43000, 1 << 20})
    printf("spread 5.4M atomics over %d addr: %.1f us\n", naddr,
           timeit([&] { hipLaunchKernelGGL(spread, dim3(2048), dim3(256), 0, 0, buf, naddr, 10, 7u); }));
  for (int waves : {400, 3200})
    printf("one_addr %d waves: %.1f us\n", waves, timeit([&] { hipLaunchKernelGGL(one_addr, dim3(waves / 4), dim3(256), 0, 0, buf, 1); }));
  printf("empty-ish (one_addr 4 waves): %.1f us\n", timeit([&] { hipLaunchKernelGGL(one_addr, dim3(1), dim3(256), 0, 0, buf, 1); }));
  for (int na : {160, 4096})
    printf("lds_hot 782 blocks x 256 thr x 80 atomics over %d: %.1f us\n", na,
           timeit([&] { hipLaunchKernelGGL(lds_hot, dim3(782), dim3(256), 0, 0, buf, 80, na); }));
  hipFree(buf);
  return 0;
}
