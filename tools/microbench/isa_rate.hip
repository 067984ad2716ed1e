// Microbenchmark: issue cost of the integer instructions the NTT butterflies use, and whether the
// quarter-rate multiplies overlap with full-rate VALU work (inline asm, 8 independent chains).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;

#define MUL_LO(r) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r) : "v"(k));
#define MUL_HI(r) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(r) : "v"(k));
#define MAD64(r) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(r) : "v"(lo), "v"(k) : "s0", "s1");
#define ADD(r) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(k));
#define LSHLADD(r) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(r) : "v"(kk));
#define CMP64(r) asm volatile("v_cmp_le_u64 vcc, %0, %1" :: "v"(r), "v"(kk) : "vcc");

template <int MODE>
__global__ __launch_bounds__(256) void k(uint64_t* out, uint32_t s) {
  uint32_t k = threadIdx.x | 1u, lo = s ^ threadIdx.x;
  uint64_t kk = (uint64_t)k * 3;
  uint32_t a0 = 1, a1 = 2, a2 = 3, a3 = 4, a4 = 5, a5 = 6, a6 = 7, a7 = 8;
  uint32_t b0 = 1, b1 = 2, b2 = 3, b3 = 4, b4 = 5, b5 = 6, b6 = 7, b7 = 8;
  uint64_t c0 = 1, c1 = 2, c2 = 3, c3 = 4, c4 = 5, c5 = 6, c6 = 7, c7 = 8;
  for (int it = 0; it < ITERS; ++it) {
    if (MODE == 0) { ADD(a0) ADD(a1) ADD(a2) ADD(a3) ADD(a4) ADD(a5) ADD(a6) ADD(a7) }
    if (MODE == 1) { MUL_LO(a0) MUL_LO(a1) MUL_LO(a2) MUL_LO(a3) MUL_LO(a4) MUL_LO(a5) MUL_LO(a6) MUL_LO(a7) }
    if (MODE == 2) { MUL_HI(a0) MUL_HI(a1) MUL_HI(a2) MUL_HI(a3) MUL_HI(a4) MUL_HI(a5) MUL_HI(a6) MUL_HI(a7) }
    if (MODE == 3) { MAD64(c0) MAD64(c1) MAD64(c2) MAD64(c3) MAD64(c4) MAD64(c5) MAD64(c6) MAD64(c7) }
    if (MODE == 4) { LSHLADD(c0) LSHLADD(c1) LSHLADD(c2) LSHLADD(c3) LSHLADD(c4) LSHLADD(c5) LSHLADD(c6) LSHLADD(c7) }
    // 8 mul_lo + 8 adds interleaved: overlap test
    if (MODE == 5) { MUL_LO(a0) ADD(b0) MUL_LO(a1) ADD(b1) MUL_LO(a2) ADD(b2) MUL_LO(a3) ADD(b3)
                     MUL_LO(a4) ADD(b4) MUL_LO(a5) ADD(b5) MUL_LO(a6) ADD(b6) MUL_LO(a7) ADD(b7) }
    // 8 mad64 + 16 adds interleaved
    if (MODE == 6) { MAD64(c0) ADD(b0) ADD(a0) MAD64(c1) ADD(b1) ADD(a1) MAD64(c2) ADD(b2) ADD(a2) MAD64(c3) ADD(b3) ADD(a3)
                     MAD64(c4) ADD(b4) ADD(a4) MAD64(c5) ADD(b5) ADD(a5) MAD64(c6) ADD(b6) ADD(a6) MAD64(c7) ADD(b7) ADD(a7) }
    if (MODE == 7) { CMP64(c0) CMP64(c1) CMP64(c2) CMP64(c3) CMP64(c4) CMP64(c5) CMP64(c6) CMP64(c7) }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] =
      a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7 ^ c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}

template <int MODE>
static int run(const char* name, int instrs_per_iter, uint64_t* d) {
  dim3 grid(256 * 8), block(256);
  k<MODE><<<grid, block>>>(d, 1);
  CHK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) k<MODE><<<grid, block>>>(d, r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double wave_instr = 5.0 * grid.x * (block.x / 64) * (double)ITERS * instrs_per_iter;
  const double simd_cycles = 1024.0 * 2.4e9 * ms * 1e-3;  // at 2.4 GHz
  printf("%-28s %7.3f ms  %.2f SIMD-cycles per wave-instruction (at 2.4 GHz)\n", name, ms,
         simd_cycles / wave_instr);
  return 0;
}

int main() {
  uint64_t* d;
  CHK(hipMalloc(&d, 256 * 8 * 256 * 8));
  run<0>("v_add_u32", 8, d);
  run<1>("v_mul_lo_u32", 8, d);
  run<2>("v_mul_hi_u32", 8, d);
  run<3>("v_mad_u64_u32", 8, d);
  run<4>("v_lshl_add_u64", 8, d);
  run<7>("v_cmp_le_u64", 8, d);
  run<5>("8 mul_lo + 8 add", 16, d);
  run<6>("8 mad64 + 16 add", 24, d);
  return 0;
}
