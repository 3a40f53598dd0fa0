// Micro-benchmark: VALU issue rate of one SIMD vs resident waves (design input
// for K_parse, whose SQ counters show a VALU instruction in ~80 % of a SIMD's
// quad-cycles at 4 waves/SIMD: is that the VALU pipe's ceiling, or could more
// ready waves issue more?).
//   hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate && ./valu_rate
// Each wave runs ITERS x 32 VALU instructions of one kind, in 8 independent
// chains (no dependency stall at 4 cycles per wave instruction), timed per wave
// with s_memtime; cycles per instruction per SIMD = wave cycles / (waves per
// SIMD x instructions per wave).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 4096;

#define OP8(ins)                                                                                  \
  ins " %0, %0, %8\n\t" ins " %1, %1, %8\n\t" ins " %2, %2, %8\n\t" ins " %3, %3, %8\n\t" ins " %4, %4, %8\n\t" \
      ins " %5, %5, %8\n\t" ins " %6, %6, %8\n\t" ins " %7, %7, %8\n\t"
#define OP8_3(ins)                                                                                        \
  ins " %0, %0, %8, %0\n\t" ins " %1, %1, %8, %1\n\t" ins " %2, %2, %8, %2\n\t" ins " %3, %3, %8, %3\n\t" \
      ins " %4, %4, %8, %4\n\t" ins " %5, %5, %8, %5\n\t" ins " %6, %6, %8, %6\n\t" ins " %7, %7, %8, %7\n\t"

template <int OP>
__global__ void K(uint32_t* out, unsigned long long* cyc) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const uint32_t c = blockIdx.x | 1u;
  unsigned long long t0, t1;
  __syncthreads();
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < ITERS; ++i) {
    if (OP == 0)  // 32-bit integer add (VOP2)
      asm volatile(OP8("v_add_u32") OP8("v_add_u32") OP8("v_add_u32") OP8("v_add_u32")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));
    else if (OP == 1)  // bit ops (VOP2)
      asm volatile(OP8("v_xor_b32") OP8("v_and_b32") OP8("v_or_b32") OP8("v_xor_b32")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));
    else if (OP == 2)  // three-operand integer (VOP3): v_lshl_add_u32 / v_bfe_u32-like shapes
      asm volatile(OP8_3("v_lshl_add_u32") OP8_3("v_add3_u32") OP8_3("v_lshl_add_u32") OP8_3("v_add3_u32")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));
    else if (OP == 3)  // f32 fma
      asm volatile(OP8_3("v_fma_f32") OP8_3("v_fma_f32") OP8_3("v_fma_f32") OP8_3("v_fma_f32")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));
    else  // compare + select (the parse's predicate pattern): v_cmp writes an SGPR pair
      asm volatile(
          "v_cmp_lt_u32 vcc, %0, %8\n\tv_cndmask_b32 %0, %1, %0, vcc\n\t"
          "v_cmp_lt_u32 vcc, %2, %8\n\tv_cndmask_b32 %2, %3, %2, vcc\n\t"
          "v_cmp_lt_u32 vcc, %4, %8\n\tv_cndmask_b32 %4, %5, %4, vcc\n\t"
          "v_cmp_lt_u32 vcc, %6, %8\n\tv_cndmask_b32 %6, %7, %6, vcc\n\t"
          "v_cmp_lt_u32 vcc, %1, %8\n\tv_cndmask_b32 %1, %0, %1, vcc\n\t"
          "v_cmp_lt_u32 vcc, %3, %8\n\tv_cndmask_b32 %3, %2, %3, vcc\n\t"
          "v_cmp_lt_u32 vcc, %5, %8\n\tv_cndmask_b32 %5, %4, %5, vcc\n\t"
          "v_cmp_lt_u32 vcc, %7, %8\n\tv_cndmask_b32 %7, %6, %7, vcc\n\t"
          "v_cmp_lt_u32 vcc, %0, %8\n\tv_cndmask_b32 %0, %1, %0, vcc\n\t"
          "v_cmp_lt_u32 vcc, %2, %8\n\tv_cndmask_b32 %2, %3, %2, vcc\n\t"
          "v_cmp_lt_u32 vcc, %4, %8\n\tv_cndmask_b32 %4, %5, %4, vcc\n\t"
          "v_cmp_lt_u32 vcc, %6, %8\n\tv_cndmask_b32 %6, %7, %6, vcc\n\t"
          "v_cmp_lt_u32 vcc, %1, %8\n\tv_cndmask_b32 %1, %0, %1, vcc\n\t"
          "v_cmp_lt_u32 vcc, %3, %8\n\tv_cndmask_b32 %3, %2, %3, vcc\n\t"
          "v_cmp_lt_u32 vcc, %5, %8\n\tv_cndmask_b32 %5, %4, %5, vcc\n\t"
          "v_cmp_lt_u32 vcc, %7, %8\n\tv_cndmask_b32 %7, %6, %7, vcc\n\t"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(c)
          : "vcc");
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
int run(const char* name, int cus) {
  printf("%-28s", name);
  for (int wps : {1, 2, 3, 4, 6, 8}) {  // waves per SIMD
    // one block of 4 * wps waves per CU (two blocks of 4 * wps / 2 beyond 16 waves)
    const int per_block = wps <= 4 ? 4 * wps : 2 * wps;
    const int blocks = wps <= 4 ? cus : 2 * cus;
    const int threads = per_block * 64;
    uint32_t* out;
    unsigned long long* cyc;
    CK(hipMalloc(&out, (size_t)blocks * threads * 4));
    CK(hipMalloc(&cyc, (size_t)blocks * per_block * 8));
    hipLaunchKernelGGL(K<OP>, dim3(blocks), dim3(threads), 0, 0, out, cyc);  // warm-up
    hipLaunchKernelGGL(K<OP>, dim3(blocks), dim3(threads), 0, 0, out, cyc);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)blocks * per_block);
    CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
    double mean = 0;
    for (auto v : h) mean += (double)v;
    mean /= (double)h.size();
    const double inst = (OP == 4 ? 32.0 : 32.0) * ITERS;  // instructions per wave
    // s_memtime ticks at the shader clock (MI355X_MICROARCH.md constants table)
    printf("  w%d %5.2f", wps, mean / (wps * inst));
    CK(hipFree(out));
    CK(hipFree(cyc));
  }
  printf("   (cycles per wave-instruction per SIMD)\n");
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  printf("%s, %d CUs; 8 independent chains per wave\n", p.gcnArchName, cus);
  run<0>("v_add_u32", cus);
  run<1>("v_xor/and/or_b32", cus);
  run<2>("v_lshl_add/add3_u32 (VOP3)", cus);
  run<3>("v_fma_f32", cus);
  run<4>("v_cmp + v_cndmask (vcc)", cus);
  return 0;
}
