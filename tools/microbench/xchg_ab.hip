// A/B of the row pass's round exchange (dev microbenchmark, not libfhecore): north_star asks for
// "intra-wavefront __shfl for the small-radix stages".  A 2^8-point row lives in 16 lanes x 16
// registers; between its two radix-16 rounds the row is transposed (lane bits <-> register bits).
//   mode 0: through the LDS, as csrc/ntt.hip does (16 ds_write_b64 + wave fence + 16 ds_read_b64,
//           one pad word per 16), no VALU beyond addressing;
//   mode 1: in registers, a 4-step recursive transpose with cross-lane moves (DPP quad_perm for lane
//           distance 1 and 2, ds_swizzle for 4, DPP row_ror:8 for 8) and v_cndmask selects.
// Each iteration = round A (32 forward butterflies, the row kernels' arithmetic) + exchange +
// round B.  Prints butterflies/s per mode and checks that both exchanges produce the same
// transpose.  usage: xchg_ab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "../../gpu-fhe_amd/csrc/modarith.hpp"

using fhe::u32;
using fhe::u64;
constexpr int kE = 16, kT = 256;

__device__ __forceinline__ u32 xlane(u32 v, int d) {
  if (d == 1) return __builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  if (d == 2) return __builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  if (d == 4) return __builtin_amdgcn_ds_swizzle((int)v, 0x1F | (4 << 10));           // xor 4
  return __builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);             // row_ror:8
}

template <int K>
__device__ __forceinline__ void tstep(u64 (&x)[kE], u32 lane) {
  constexpr int d = 1 << K;
  // lanes with bit K set send x[j] and take the partner's x[jj] into x[j]; the others send x[jj]
  // and take the partner's x[j] into x[jj]: bit selects (v_bfi_b32), no divergence
  const u32 m32 = 0u - ((lane >> K) & 1u);
  const u64 m = ((u64)m32 << 32) | m32;
#pragma unroll
  for (int j = 0; j < kE; ++j) {
    if (j & d) continue;
    const int jj = j | d;
    const u64 send = (x[j] & m) | (x[jj] & ~m);
    const u64 recv = ((u64)xlane((u32)(send >> 32), d) << 32) | xlane((u32)send, d);
    x[j] = (recv & m) | (x[j] & ~m);
    x[jj] = (x[jj] & m) | (recv & ~m);
  }
}

__device__ __forceinline__ void reg_transpose(u64 (&x)[kE], u32 lane) {
  tstep<0>(x, lane);
  tstep<1>(x, lane);
  tstep<2>(x, lane);
  tstep<3>(x, lane);
}

// row r of the workgroup at lds + r * 272 (one pad word per 16, as LView<1, true>)
__device__ __forceinline__ void lds_transpose(u64 (&x)[kE], u64* row, u32 t) {
#pragma unroll
  for (int j = 0; j < kE; ++j) {
    const u32 p = t + 16 * j;
    row[p + (p >> 4)] = x[j];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int j = 0; j < kE; ++j) {
    const u32 p = 16 * t + j;
    x[j] = row[p + (p >> 4)];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ u64 csubk(u64 x, u64 m) {
  u64 nm = 0 - m;
  asm("" : "+s"(nm));
  return fhe::csub_fast(x, nm);
}

__device__ __forceinline__ void round4(u64 (&x)[kE], const ulonglong2 (&w)[8], u64 q, u64 q3) {
  const u64 nq = 0 - q;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      if (j & (1 << b)) continue;
      const int jj = j | (1 << b);
      const ulonglong2 t = w[(j + b) & 7];
      u64 u = (b & 1) ? csubk(x[j], 8 * q) : x[j];
      FHE_OPAQUE(u);
      u64 s = fhe::shoup_q3_add<true>(x[jj], t.x, t.y, nq, u);
      FHE_OPAQUE(s);
      x[j] = s;
      u64 t2 = (u << 1) + q3;
      FHE_OPAQUE(t2);
      x[jj] = t2 - s;
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(kT) void k_xchg(u64* __restrict__ out, const ulonglong2* __restrict__ tw,
                                           u64 q, u32 iters) {
  __shared__ u64 lds[16 * 272];
  const u32 gid = blockIdx.x * kT + threadIdx.x, t = threadIdx.x % 16, row = threadIdx.x / 16;
  u64 x[kE];
#pragma unroll
  for (int j = 0; j < kE; ++j) x[j] = (gid * 0x9e3779b97f4a7c15ull + j * 0x632be59bd9b4e019ull) % q;
  ulonglong2 w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = tw[(gid + k) & 63];
  u64 q3 = 3 * q;
  asm("" : "+s"(q3));
  for (u32 r = 0; r < iters; ++r) {
    round4(x, w, q, q3);
    if (MODE == 0) lds_transpose(x, lds + row * 272, t);
    else reg_transpose(x, threadIdx.x);
    round4(x, w, q, q3);
  }
  u64 acc = 0;
#pragma unroll
  for (int j = 0; j < kE; ++j) acc ^= x[j] * (j + 1);
  out[gid] = acc;
}

// one transpose of known data per mode (correctness)
template <int MODE>
__global__ void k_check(u64* out) {
  __shared__ u64 lds[16 * 272];
  const u32 t = threadIdx.x % 16, row = threadIdx.x / 16;
  u64 x[kE];
#pragma unroll
  for (int j = 0; j < kE; ++j) x[j] = (u64)row << 40 | (u64)t << 20 | j;
  if (MODE == 0) lds_transpose(x, lds + row * 272, t);
  else reg_transpose(x, threadIdx.x);
#pragma unroll
  for (int j = 0; j < kE; ++j) out[threadIdx.x * kE + j] = x[j];
}

int main() {
  const u64 q = 0xffffffffffc0001ull;
  ulonglong2 htw[64];
  for (int k = 0; k < 64; ++k) {
    const u64 wv = (0x1234567ull * (k + 1)) % q;
    htw[k] = ulonglong2{wv, (u64)(((unsigned __int128)wv << 64) / q)};
  }
  const int blocks = 8 * 256;
  const u32 iters = 40;
  u64 *d_out, *d_chk;
  ulonglong2* d_tw;
  if (hipMalloc(&d_out, (size_t)blocks * kT * 8) || hipMalloc(&d_tw, sizeof(htw)) ||
      hipMalloc(&d_chk, 2 * 256 * kE * 8))
    return 1;
  hipMemcpy(d_tw, htw, sizeof(htw), hipMemcpyHostToDevice);
  k_check<0><<<1, 256>>>(d_chk);
  k_check<1><<<1, 256>>>(d_chk + 256 * kE);
  static u64 h[2 * 256 * kE];
  hipMemcpy(h, d_chk, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256 * kE; ++i) bad += h[i] != h[256 * kE + i];
  printf("register transpose == LDS transpose: %s\n", bad ? "NO" : "yes");
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int mode = 0; mode < 2; ++mode) {
    auto launch = [&] {
      if (mode == 0) k_xchg<0><<<blocks, kT>>>(d_out, d_tw, q, iters);
      else k_xchg<1><<<blocks, kT>>>(d_out, d_tw, q, iters);
    };
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(a);
    for (int i = 0; i < 20; ++i) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double bfly = (double)blocks * kT * iters * 2 * 32 * 20;
    printf("mode %d (%s): %.3f ms/launch, %.3f Tbutterfly/s (incl. exchange)\n", mode,
           mode ? "registers: DPP + ds_swizzle" : "LDS", ms / 20, bfly / (ms * 1e-3) / 1e12);
  }
  return 0;
}
