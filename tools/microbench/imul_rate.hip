// Microbenchmark: throughput of the 32/64-bit integer multiply instructions the
// modular-arithmetic kernels are built from (v_mad_u64_u32, v_mul_lo_u32,
// v_mul_hi_u32) against a plain v_add_u32 baseline, on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr int ACC = 8;

__global__ void k_mad64(uint64_t* out, uint32_t s) {
  uint64_t acc[ACC]; uint32_t a = threadIdx.x ^ s;
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = i + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = (uint64_t)((uint32_t)acc[i]) * (a + i) + (acc[i] >> 32);
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mullo(uint64_t* out, uint32_t s) {
  uint32_t acc[ACC]; uint32_t a = threadIdx.x ^ s;
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = i + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = acc[i] * (a | 1u);
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mulhi(uint64_t* out, uint32_t s) {
  uint32_t acc[ACC]; uint32_t a = threadIdx.x ^ s;
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = i + threadIdx.x + 0x9e3779b9u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __umulhi(acc[i], a | 0x80000000u) ^ acc[i];
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_add(uint64_t* out, uint32_t s) {
  uint32_t acc[ACC]; uint32_t a = threadIdx.x ^ s;
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = i + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = (acc[i] + a) ^ (uint32_t)i;
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_add64(uint64_t* out, uint32_t s) {
  uint64_t acc[ACC]; uint64_t a = threadIdx.x ^ s;
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = i + threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = acc[i] + (a << 20);
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < ACC; ++i) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <typename K>
static int run(const char* name, K kern, int ops_per_inner, uint64_t* d) {
  hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  dim3 grid(256 * 8), block(256);
  kern<<<grid, block>>>(d, 1); CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) kern<<<grid, block>>>(d, r);
  CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
  float ms; CHK(hipEventElapsedTime(&ms, a, b));
  double lane_ops = 5.0 * grid.x * block.x * (double)ITERS * ACC * ops_per_inner;
  double peak = 256.0 * 4 * 32 * 2.4e9;  // lane-ops/s at one op per lane per cycle per SIMD32
  printf("%-8s %8.3f ms  %.2f Tops/s  (%.3f of 1-op/lane/clk)\n", name, ms, lane_ops / (ms * 1e-3) / 1e12,
         lane_ops / (ms * 1e-3) / peak);
  return 0;
}

int main() {
  uint64_t* d; CHK(hipMalloc(&d, 256 * 8 * 256 * 8));
  run("add32", k_add, 2, d);
  run("add64", k_add64, 1, d);
  run("mullo32", k_mullo, 1, d);
  run("mulhi32", k_mulhi, 2, d);
  run("mad64", k_mad64, 1, d);
  return 0;
}
