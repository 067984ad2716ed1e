// Device-side modular arithmetic over 64-bit words for gfx950.
//
// Replaces the reference's numpy `%` (/root/reference/arithmetic.py:5,9,13) with exact
// word-level reductions.  gfx950 has no 64x64->128 multiply: a 64-bit product is built from
// v_mad_u64_u32 / v_mul_hi_u32 / v_mul_lo_u32, all ~quarter-rate (profiles/r01_imul_rate.txt),
// so every routine here is written to minimise the number of 32x32 partial products.
//
// Conventions (shared with oracle/fhe_oracle.c):
//  * moduli q < 2^61, so lazy values in [0, 4q) fit a word with room to spare;
//  * Shoup: w' = floor(w * 2^64 / q) precomputed for a constant operand w;
//  * Barrett (data x data): z < 4q^2, a = bitlen(q) - 1, b = 2 bitlen(q) + 2,
//    mu = floor(2^b / q); estimate floor(floor(z / 2^a) * mu / 2^(b - a)) is at most 2 low,
//    so r = z - est * q lies in [0, 3q).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhe {

using u64 = uint64_t;
using u32 = uint32_t;
using u128 = unsigned __int128;

// Per-modulus constants, one record per RNS limb (device and host share the layout).
struct ModParams {
  u64 q;
  u64 mu;    // Barrett: floor(2^(2 bitlen + 2) / q)
  u32 sh_a;  // bitlen - 1
  u32 sh_b;  // bitlen + 3  (= b - a)
};

__device__ __forceinline__ u64 mulhi64(u64 a, u64 b) { return (u64)(((u128)a * b) >> 64); }

__device__ __forceinline__ u64 csub(u64 x, u64 m) { return x >= m ? x - m : x; }

// x * w mod q up to one q: x < 2^64, result in [0, 2q).  (4 + 2 x 3 partial products.)
__device__ __forceinline__ u64 shoup_lazy(u64 x, u64 w, u64 ws, u64 q) {
  const u64 qh = mulhi64(x, ws);
  return x * w - qh * q;
}

// Barrett reduction of a 128-bit z < 4 q^2 into [0, q).
__device__ __forceinline__ u64 barrett_reduce(u128 z, const ModParams& m) {
  const u64 z1 = (u64)(z >> m.sh_a);
  const u64 est = (u64)(((u128)z1 * m.mu) >> m.sh_b);
  u64 r = (u64)z - est * m.q;
  r = csub(r, 2 * m.q);
  return csub(r, m.q);
}

__device__ __forceinline__ u64 mulmod_barrett(u64 a, u64 b, const ModParams& m) {
  return barrett_reduce((u128)a * b, m);
}

// Full reduction of any 64-bit x into [0, q), any q >= 2: Barrett for 2^31 <= q < 2^61
// (x < 2^64 <= 4 q^2 there), repeated subtraction above (x < 8q), hardware % below.
__device__ __forceinline__ u64 reduce_u64(u64 x, const ModParams& m) {
  if (m.mu == 0) {  // q >= 2^61: "wide" modulus, no Barrett constants
    while (x >= m.q) x -= m.q;
    return x;
  }
  if (m.q < (1ull << 31)) return x % m.q;
  return barrett_reduce((u128)x, m);
}

// Exact a * b mod q for a, b < q and any q < 2^64 (generic entry points only; the context
// kernels use Shoup/Barrett).  Wide moduli fall back to a 64-step double-and-add.
__device__ __forceinline__ u64 mulmod_any(u64 a, u64 b, const ModParams& m) {
  if (m.mu != 0) return barrett_reduce((u128)a * b, m);
  u64 r = 0;
  for (int i = 63; i >= 0; --i) {
    const u64 r2 = r >= m.q - r ? r - (m.q - r) : r + r;  // 2r mod q without overflow
    r = r2;
    if ((b >> i) & 1) r = r >= m.q - a ? r - (m.q - a) : r + a;
  }
  return r;
}

}  // namespace fhe
