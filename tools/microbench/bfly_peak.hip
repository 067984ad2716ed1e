// Integer-ALU ceiling for the NTT butterflies (measurement infrastructure for bench.py's
// `roofline_alu`; not part of libfhecore).
//
// Runs the exact butterfly instruction sequences of csrc/ntt.hip round_compute in the row passes
// (the lazy forms with the mad-chain remainder, shoup_q3<true>; headroom H = 16) on
// register-resident data at full occupancy, with no memory traffic:
//   forward  Cooley-Tukey, folded X-operand (shoup_q3_add), one top-bits reduction per 4-stage
//            round (the lz16 row passes' schedule: two per 8-stage pass), outputs s and (2u + 3q) - s;
//   inverse  Gentleman-Sande with lazy sums (round_compute's H = 16 form, gs_in ranges): sums
//            unreduced, a pair at 12q taken below 2q by top_bits first, (u - v + r q) w by
//            shoup_q3, and the round's end reductions back below 3q.
// Each thread holds kE = 16 values and runs 4-stage rounds on them exactly as a kernel round does
// (8 butterflies per stage), with 8 twiddle pairs in registers standing in for the round's
// gathered twiddles.  The result is the chip's butterflies/s ceiling for that arithmetic, measured
// on the same box and clock regime as the kernels it is compared with.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../gpu-fhe_amd/csrc/modarith.hpp"

namespace {

using fhe::u32;
using fhe::u64;
constexpr int kE = 16;
constexpr int kThreads = 256;

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// ntt.hip gs_red / gs_in (the static per-element ranges of a lazy GS round)
constexpr int gs_red(int r) { return r > 8 ? 2 : r; }
constexpr int gs_in(int j, int k) {
  int r = 3;
  for (int b = 0; b < k; ++b) r = ((j >> b) & 1) ? 3 : 2 * gs_red(r);
  return r;
}

// ntt.hip top_bits
__device__ __forceinline__ u64 top_bits(u64 x, u32 s, u64 nq) {
  return x + (u64)(u32)(x >> s) * nq;
}

__device__ __forceinline__ u64 csubk(u64 x, u64 m) {
  u64 nm = 0 - m;
  asm("" : "+s"(nm));
  return fhe::csub_fast(x, nm);
}

template <bool INV>
__global__ __launch_bounds__(kThreads) void k_bfly_peak(u64* __restrict__ out,
                                                        const ulonglong2* __restrict__ tw, u64 q,
                                                        u32 rounds) {
  const u32 gid = blockIdx.x * blockDim.x + threadIdx.x;
  u64 x[kE];
#pragma unroll
  for (int j = 0; j < kE; ++j) x[j] = (gid * 0x9e3779b97f4a7c15ull + j * 0x632be59bd9b4e019ull) % q;
  ulonglong2 w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = tw[(gid + k) & 63];
  const u64 nq = 0 - q;
  u64 q3 = 3 * q, q2 = 2 * q, q4 = 4 * q, q6 = 6 * q, q8 = 8 * q;
  asm("" : "+s"(q3));
  asm("" : "+s"(q2));
  asm("" : "+s"(q4));
  asm("" : "+s"(q6));
  asm("" : "+s"(q8));
  const u32 sb = 64 - __builtin_clzll(q);
  for (u32 r = 0; r < rounds; ++r) {
    if constexpr (INV) {
      static_for<0, 4>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        static_for<0, kE>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if constexpr (!(j & (1 << b))) {
            constexpr int jj = j | (1 << b);
            constexpr int ri = gs_in(j, b), rr = gs_red(ri);
            const ulonglong2 t = w[(j + b) & 7];
            u64 u = x[j], v = x[jj];
            if constexpr (rr != ri) {
              u = top_bits(u, sb, nq);
              v = top_bits(v, sb, nq);
            }
            const u64 off = rr == 2 ? q2 : rr == 3 ? q3 : rr == 4 ? q4 : rr == 6 ? q6 : q8;
            const u64 sum = u + v, dif = u - v + off;
            x[j] = sum;
            x[jj] = fhe::shoup_q3<true>(dif, t.x, t.y, nq);
          }
        });
      });
      static_for<0, kE>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (gs_in(j, 4) > 3) x[j] = top_bits(x[j], sb, nq);
      });
      continue;
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int j = 0; j < kE; ++j) {
        if (j & (1 << b)) continue;
        const int jj = j | (1 << b);
        const ulonglong2 t = w[(j + b) & 7];
        if constexpr (!INV) {
          u64 u = x[j];
          if (b == 1) u = top_bits(u, sb, nq);  // one per round, as in an lz16 row pass
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
  }
  u64 acc = 0;
#pragma unroll
  for (int j = 0; j < kE; ++j) acc ^= x[j];
  out[gid] = acc;
}

}  // namespace

extern "C" {

// Butterflies per second of the forward (inverse = 0) or inverse (1) arithmetic over `blocks`
// workgroups of 256 threads x `rounds` 4-stage rounds (32 butterflies per thread per round),
// timed over `reps` back-to-back launches after one warm-up launch.  Returns 0 on success.
int fhe_peak_bfly(int inverse, uint32_t blocks, uint32_t rounds, uint32_t reps,
                  double* bfly_per_s, double* ms_per_launch) {
  const u64 q = 0xffffffffffc0001ull;  // the configs[2] chain's first prime (60-bit)
  ulonglong2 htw[64];
  for (int k = 0; k < 64; ++k) {
    const u64 wv = (0x1234567ull * (k + 1)) % q;
    htw[k] = ulonglong2{wv, (u64)(((unsigned __int128)wv << 64) / q)};
  }
  u64* d_out = nullptr;
  ulonglong2* d_tw = nullptr;
  hipEvent_t e0, e1;
  if (hipMalloc(&d_out, (size_t)blocks * kThreads * 8) != hipSuccess) return -1;
  if (hipMalloc(&d_tw, sizeof(htw)) != hipSuccess) return -1;
  if (hipMemcpy(d_tw, htw, sizeof(htw), hipMemcpyHostToDevice) != hipSuccess) return -1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto launch = [&] {
    if (inverse)
      k_bfly_peak<true><<<blocks, kThreads>>>(d_out, d_tw, q, rounds);
    else
      k_bfly_peak<false><<<blocks, kThreads>>>(d_out, d_tw, q, rounds);
  };
  launch();
  (void)hipEventRecord(e0, nullptr);
  for (uint32_t r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(e1, nullptr);
  int rc = hipEventSynchronize(e1) == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -2;
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double per = (double)ms / reps;
  *ms_per_launch = per;
  *bfly_per_s = (double)blocks * kThreads * rounds * 4 * (kE / 2) / (per * 1e-3);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(d_out);
  (void)hipFree(d_tw);
  return rc;
}

}  // extern "C"
