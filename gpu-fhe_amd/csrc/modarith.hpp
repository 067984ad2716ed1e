// Device-side modular arithmetic over 64-bit words for gfx950.
//
// Replaces the reference's numpy `%` (/root/reference/arithmetic.py:5,9,13) with exact
// word-level reductions.  gfx950 has no 64x64->128 multiply: a 64-bit product is built from
// v_mad_u64_u32 / v_mul_hi_u32 / v_mul_lo_u32, ~1.8x the issue cost of a 32-bit add
// (tools/microbench/isa_rate.hip, profiles/r01_isa_rate.txt),
// so every routine here is written to minimise the number of 32x32 partial products.
//
// Conventions (shared with oracle/fhe_oracle.c):
//  * context moduli q < 2^63.  "Narrow" moduli (q < 2^61, Barrett constants present, mu != 0)
//    take the lazy butterflies and Montgomery / 128-bit-sum shortcuts; "wide" ones
//    (2^61 <= q < 2^63, mu == 0) the exact forms below (values kept below 2q < 2^64);
//  * Shoup: w' = floor(w * 2^64 / q) precomputed for a constant operand w;
//  * Barrett (data x data): z < 4q^2, a = bitlen(q) - 1, b = 2 bitlen(q) + 2,
//    mu = floor(2^b / q); estimate floor(floor(z / 2^a) * mu / 2^(b - a)) is at most 2 low,
//    so r = z - est * q lies in [0, 3q).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "modparams.hpp"

namespace fhe {

__device__ __forceinline__ u64 mulhi64(u64 a, u64 b) { return (u64)(((u128)a * b) >> 64); }

__device__ __forceinline__ u64 csub(u64 x, u64 m) { return x >= m ? x - m : x; }

// x * w mod q up to one q: x < 2^64, result in [0, 2q).  (4 + 2 x 3 partial products.)
__device__ __forceinline__ u64 shoup_lazy(u64 x, u64 w, u64 ws, u64 q) {
  const u64 qh = mulhi64(x, ws);
  return x * w - qh * q;
}

// ---- instruction-shaped forms for the butterflies -------------------------------------------
// Measured on gfx950 (tools/microbench/isa_rate.hip): v_mad_u64_u32, v_mul_lo/hi_u32 and every
// 64-bit VALU op (v_lshl_add_u64, v_cmp_*_u64) issue at half the rate of a 32-bit add.  Left
// alone, hipcc shrinks v_mad_u64_u32 chains whose high halves it can prove unused into
// v_mul_lo_u32 + v_add3 + borrow chains, and turns sign-mask selects into 64-bit compares +
// v_cndmask with VCC hazards (s_nop).  OPAQUE() is an empty asm that makes a value opaque to those
// rewrites without emitting an instruction (real inline-asm instructions would make the hazard
// recognizer pad every use).  tools/microbench/bfly_rate.hip: 44 vs 56 lane-cycles per butterfly.
#define FHE_OPAQUE(x) asm("" : "+v"(x))

__device__ __forceinline__ u64 mad_u64_u32(u32 a, u32 b, u64 c) { return (u64)a * b + c; }

// x >= m ? x - m : x for x, m < 2^63, given nm = -m mod 2^64: sign-mask select (v_bfi_b32).
__device__ __forceinline__ u64 csub_fast(u64 x, u64 nm) {
  const u64 d = x + nm;
  u32 m = (u32)((int32_t)(d >> 32) >> 31);
  FHE_OPAQUE(m);
  const u32 lo = ((u32)x & m) | ((u32)d & ~m);
  const u32 hi = ((u32)(x >> 32) & m) | ((u32)(d >> 32) & ~m);
  return ((u64)hi << 32) | lo;
}

// y * w mod q up to one q, y < 2^64, result in [0, 2q): Shoup with the exact quotient
// h = floor(y w' / 2^64) (1 mul_hi + 3 mads), then T = lo64(y w + h (-q)) by a chain of 6 mads
// (the low words through the chain's carries, the cross terms into the high word) -- no
// borrows, no compares.  nq = -q mod 2^64.
__device__ __forceinline__ u64 shoup_fast(u64 y, u64 w, u64 ws, u64 nq) {
  const u32 y0 = (u32)y, y1 = (u32)(y >> 32);
  const u32 s0 = (u32)ws, s1 = (u32)(ws >> 32);
  const u32 w0 = (u32)w, w1 = (u32)(w >> 32);
  const u32 n0 = (u32)nq, n1 = (u32)(nq >> 32);
  const u64 a = mad_u64_u32(y1, s0, __umulhi(y0, s0));
  const u64 b = mad_u64_u32(y0, s1, (u32)a);
  const u64 h = mad_u64_u32(y1, s1, a >> 32) + (b >> 32);
  const u32 h0 = (u32)h, h1 = (u32)(h >> 32);
  u64 t = mad_u64_u32(h0, n0, mad_u64_u32(y0, w0, 0));
  FHE_OPAQUE(t);
  u64 c = mad_u64_u32(y1, w0, t >> 32);
  FHE_OPAQUE(c);
  c = mad_u64_u32(y0, w1, c);
  FHE_OPAQUE(c);
  c = mad_u64_u32(h1, n0, c);
  FHE_OPAQUE(c);
  c = mad_u64_u32(h0, n1, c);
  FHE_OPAQUE(c);
  return ((u64)(u32)c << 32) | (u32)t;
}

// lo32(y1 w0 + y0 w1 + h1 n0 + h0 n1): the four cross terms of a remainder's high word as a chain
// of v_mad_u64_u32 whose low words carry the sum (the high words are never read), 4 instructions
// instead of 4 v_mul_lo_u32 + 2 v_add3_u32.  OPAQUE keeps the compiler from shrinking the chain
// back into mul_lo + add3 (it can see that only the low word is used).  The h terms come last:
// the chain starts before the quotient is ready.
__device__ __forceinline__ u32 cross_lo(u32 y0, u32 y1, u32 w0, u32 w1, u32 h0, u32 h1, u32 n0,
                                        u32 n1) {
  u64 c = mad_u64_u32(y1, w0, 0);
  FHE_OPAQUE(c);
  c = mad_u64_u32(y0, w1, c);
  FHE_OPAQUE(c);
  c = mad_u64_u32(h1, n0, c);
  FHE_OPAQUE(c);
  c = mad_u64_u32(h0, n1, c);
  FHE_OPAQUE(c);
  return (u32)c;
}

// High word of a remainder: hi32(t) + the cross terms.  CHAIN: the mad chain (one VALU fewer; the
// issue-bound row kernels); otherwise 4 v_mul_lo_u32 + 2 v_add3_u32, whose independent products
// carry no back-to-back 64-bit dependences (gfx950 pads each dependent v_mad_u64_u32 pair with a
// wait state, which costs the latency-bound column passes more than the saved instruction:
// HomMult column inverse +3 % with the chain).
template <bool CHAIN>
__device__ __forceinline__ u32 rem_hi(u64 t, u32 y0, u32 y1, u32 w0, u32 w1, u32 h0, u32 h1,
                                      u32 n0, u32 n1) {
  if constexpr (CHAIN) {
    u32 hi = (u32)(t >> 32) + cross_lo(y0, y1, w0, w1, h0, h1, n0, n1);
    FHE_OPAQUE(hi);  // one 32-bit add into the high word (not a 64-bit add of a shifted pair)
    return hi;
  } else {
    return (u32)(t >> 32) + y1 * w0 + y0 * w1 + h1 * n0 + h0 * n1;
  }
}

// y * w mod q up to two q, any y < 2^64, result in [0, 3q): Shoup with the quotient estimated
// from three of the four partial products of y * w'.  Dropping hi(y0 s0) (< 2^32 in the 2^32
// column) lowers h = floor(y w' / 2^64) by at most 1, so r = y w - h q grows by at most q; the
// 2^32-column sum y1 s0 + y0 s1 may carry into bit 64, which is added back into the high mad.
// Quotient: 3 mads + 1 select (vs 1 mul_hi + 3 mads + a 64-bit add for the exact one).
// Remainder: lo64(y w + h nq), nq = -q mod 2^64 (exact: the true value is < 3q).
template <bool CHAIN = false>
__device__ __forceinline__ u64 shoup_q3(u64 y, u64 w, u64 ws, u64 nq) {
  const u32 y0 = (u32)y, y1 = (u32)(y >> 32);
  const u32 s0 = (u32)ws, s1 = (u32)(ws >> 32);
  const u64 a = (u64)y1 * s0;
  u64 b;
  u64 cmask;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(b), "=s"(cmask) : "v"(y0), "v"(s1), "v"(a));
  u32 c;
  asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(c) : "s"(cmask));
  const u64 h = mad_u64_u32(y1, s1, ((u64)c << 32) | (u32)(b >> 32));
  // lo64(y w + h nq): the two low-word products as chained mads, the four cross terms only
  // contribute their low words to the high word (rem_hi: a 4-mad chain + 1 add with CHAIN, else
  // 4 mul_lo + 2 add3; no 64-bit add or borrow either way)
  const u32 w0 = (u32)w, w1 = (u32)(w >> 32), n0 = (u32)nq, n1 = (u32)(nq >> 32);
  const u32 h0 = (u32)h, h1 = (u32)(h >> 32);
  u64 t = mad_u64_u32(h0, n0, (u64)y0 * w0);
  FHE_OPAQUE(t);
  return ((u64)rem_hi<CHAIN>(t, y0, y1, w0, w1, h0, h1, n0, n1) << 32) | (u32)t;
}

// u + y * w mod q up to two q (the forward CT butterfly's sum output, shoup_q3 with the X-operand
// folded in): lo64(u + y w + h nq) -- the addend rides in the first mad of the remainder chain, so
// the sum costs no separate 64-bit add.  Exact as long as the true value u + (y w - h q) < 2^64.
template <bool CHAIN = false>
__device__ __forceinline__ u64 shoup_q3_add(u64 y, u64 w, u64 ws, u64 nq, u64 u) {
  const u32 y0 = (u32)y, y1 = (u32)(y >> 32);
  const u32 s0 = (u32)ws, s1 = (u32)(ws >> 32);
  const u64 a = (u64)y1 * s0;
  u64 b;
  u64 cmask;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(b), "=s"(cmask) : "v"(y0), "v"(s1), "v"(a));
  u32 c;
  asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(c) : "s"(cmask));
  const u64 h = mad_u64_u32(y1, s1, ((u64)c << 32) | (u32)(b >> 32));
  const u32 w0 = (u32)w, w1 = (u32)(w >> 32), n0 = (u32)nq, n1 = (u32)(nq >> 32);
  const u32 h0 = (u32)h, h1 = (u32)(h >> 32);
  u64 t = mad_u64_u32(h0, n0, mad_u64_u32(y0, w0, u));
  FHE_OPAQUE(t);
  return ((u64)rem_hi<CHAIN>(t, y0, y1, w0, w1, h0, h1, n0, n1) << 32) | (u32)t;
}

// a - b + k for a + k > b, with kp1 = k + 1: a + k + 1 + ~b, two 64-bit adds, no borrow chain.
__device__ __forceinline__ u64 sub_plus(u64 a, u64 b, u64 kp1) {
  u64 nb = ~b;
  FHE_OPAQUE(nb);
  return (a + kp1) + nb;
}

// Full reduction of a 128-bit z = (zhi, zlo) into [0, q) for a wide modulus 2^61 <= q < 2^63
// (also valid below): zhi 2^64 + zlo = zhi (2^64 mod q) + zlo, each term by an exact-quotient
// Shoup product into [0, 2q) (2q < 2^64), then three conditional subtractions.
__device__ __forceinline__ u64 reduce128_wide(u64 zlo, u64 zhi, const ModParams& m) {
  const u64 q = m.q;
  const u64 a = csub(shoup_lazy(zhi, m.r64, m.r64s, q), q);
  const u64 b = csub(shoup_lazy(zlo, 1, m.ones, q), q);
  return csub(a + b, q);
}

// Barrett reduction of a 128-bit z < 4 q^2 into [0, q) (wide moduli: reduce128_wide).
__device__ __forceinline__ u64 barrett_reduce(u128 z, const ModParams& m) {
  if (m.mu == 0) return reduce128_wide((u64)z, (u64)(z >> 64), m);
  const u64 z1 = (u64)(z >> m.sh_a);
  const u64 est = (u64)(((u128)z1 * m.mu) >> m.sh_b);
  u64 r = (u64)z - est * m.q;
  r = csub(r, 2 * m.q);
  return csub(r, m.q);
}

__device__ __forceinline__ u64 mulmod_barrett(u64 a, u64 b, const ModParams& m) {
  return barrett_reduce((u128)a * b, m);
}

// Montgomery reduction with R = 2^64 of t = (thi, tlo) < q 2^64: returns t R^-1 mod q up to one
// q, in [0, 2q).  m = tlo qinv (qinv = -q^-1) makes t + m q a multiple of 2^64, whose low word
// therefore carries out exactly when tlo != 0.  No shifts or compares on the modulus, unlike
// Barrett with its per-modulus shift counts.
__device__ __forceinline__ u64 mont_reduce_lazy(u64 tlo, u64 thi, u64 q, u64 qinv) {
  const u64 m = tlo * qinv;
  return thi + mulhi64(m, q) + (tlo != 0 ? 1 : 0);
}

// Subtractive Montgomery reduction (R = 2^64) of t = (thi, tlo) < q 2^64 with qi = q^-1 mod 2^64:
// m = tlo qi makes m q = t mod 2^64, so t - m q is an exact multiple of 2^64 (no carry term, unlike
// mont_reduce_lazy's t + m q) and (t - m q) / 2^64 = thi - hi64(m q) lies in (-q, q): returns
// thi + q - hi64(m q) in (0, 2q), congruent to t R^-1.
__device__ __forceinline__ u64 mont_redc(u64 tlo, u64 thi, u64 q, u64 qi) {
  const u64 m = tlo * qi;
  return (thi + q) - mulhi64(m, q);
}

// 128-bit products for the HomMult tensor, operands below 2^61 (forward outputs in [0, 2q), every
// modulus < 2^60: the lz16 contexts).  Written out as 32x32 partial products so the compiler does
// not lower a u128 multiply (11 VALU per product with its register-pair moves):
//   A B = a1 b1 2^64 + (a0 b1 + a1 b0) 2^32 + a0 b0, where a1, b1 < 2^29, so the middle column
//   (< 2^62; four of them < 2^63) never overflows and only the low column's carries need care.
__device__ __forceinline__ void mul_wide61(u64 A, u64 B, u64& tlo, u64& thi) {
  const u32 a0 = (u32)A, a1 = (u32)(A >> 32), b0 = (u32)B, b1 = (u32)(B >> 32);
  u64 p = mad_u64_u32(a0, b0, 0);
  FHE_OPAQUE(p);
  u64 m = mad_u64_u32(a0, b1, 0);
  FHE_OPAQUE(m);
  m = mad_u64_u32(a1, b0, m);
  FHE_OPAQUE(m);
  u32 c;
  const u32 th = __builtin_addc((u32)(p >> 32), (u32)m, 0u, &c);
  thi = mad_u64_u32(a1, b1, (u64)((u32)(m >> 32) + c));
  tlo = ((u64)th << 32) | (u32)p;
}

// A B + C D for operands below 2^61 (the tensor's d1): the two low-column products may carry out
// of 64 bits (captured from the second mad's carry-out), the four middle ones stay below 2^63.
__device__ __forceinline__ void mul2_wide61(u64 A, u64 B, u64 C, u64 D, u64& tlo, u64& thi) {
  const u32 a0 = (u32)A, a1 = (u32)(A >> 32), b0 = (u32)B, b1 = (u32)(B >> 32);
  const u32 c0 = (u32)C, c1 = (u32)(C >> 32), d0 = (u32)D, d1 = (u32)(D >> 32);
  u64 p = mad_u64_u32(a0, b0, 0);
  FHE_OPAQUE(p);
  u64 p2, cm;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(p2), "=s"(cm) : "v"(c0), "v"(d0), "v"(p));
  u64 m = mad_u64_u32(a0, b1, 0);
  FHE_OPAQUE(m);
  m = mad_u64_u32(a1, b0, m);
  FHE_OPAQUE(m);
  m = mad_u64_u32(c0, d1, m);
  FHE_OPAQUE(m);
  m = mad_u64_u32(c1, d0, m);
  FHE_OPAQUE(m);
  u32 cc;
  asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(cc) : "s"(cm));
  u32 c;
  const u32 th = __builtin_addc((u32)(p2 >> 32), (u32)m, 0u, &c);
  u64 h = mad_u64_u32(a1, b1, (u64)((u32)(m >> 32) + c + cc));  // < 2^31 + 2: no wrap
  FHE_OPAQUE(h);
  thi = mad_u64_u32(c1, d1, h);
  tlo = ((u64)th << 32) | (u32)p2;
}

// sum_d x_d k_d (D <= 4 terms) as a 128-bit (tlo, thi) for x_d, k_d < 2^61 with k_d < 2^60 (the
// key-switch inner product of an lz16 context: row-forward outputs reduced below 2q, key residues
// below q).  The middle column (2D products < 2^61 each) stays below 2^64, the high one far below;
// the low column's carries are counted straight from the mads' carry-outs (v_addc with the carry
// SGPR as carry-in).  24 VALU for D = 4 where the compiler's u128 lowering takes 55.
template <int D>
__device__ __forceinline__ void dot_wide61(const u64 (&x)[D], const u64 (&k)[D], u64& tlo,
                                           u64& thi) {
  u64 l = mad_u64_u32((u32)x[0], (u32)k[0], 0);
  FHE_OPAQUE(l);
  u32 carries = 0;
#pragma unroll
  for (int d = 1; d < D; ++d) {
    u64 nl, cm, dead;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(nl), "=s"(cm) : "v"((u32)x[d]), "v"((u32)k[d]), "v"(l));
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(carries), "=s"(dead) : "v"(carries), "s"(cm));
    l = nl;
  }
  u64 m = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    m = mad_u64_u32((u32)x[d], (u32)(k[d] >> 32), m);
    FHE_OPAQUE(m);
    m = mad_u64_u32((u32)(x[d] >> 32), (u32)k[d], m);
    FHE_OPAQUE(m);
  }
  u32 c;
  const u32 th = __builtin_addc((u32)(l >> 32), (u32)m, 0u, &c);
  u64 h = (u64)((u32)(m >> 32) + c + carries);  // m < 1.5 2^63: no 32-bit wrap
#pragma unroll
  for (int d = 0; d < D; ++d) {
    h = mad_u64_u32((u32)(x[d] >> 32), (u32)(k[d] >> 32), h);
    FHE_OPAQUE(h);
  }
  thi = h;
  tlo = ((u64)th << 32) | (u32)l;
}

// mont_redc with hi64(m q) written out (exactness matters here: an error in it shifts the result
// by integers, not by multiples of q): hi(m0 q0) + m1 q0 cannot overflow, the m0 q1 column's carry
// out of 64 bits is captured from the mad and added back into the high mad (6 VALU instead of the
// compiler's 9 with its register-pair moves).  t < q 2^64; result in (0, 2q).
__device__ __forceinline__ u64 mont_redc_x(u64 tlo, u64 thi, u64 q, u64 qi) {
  const u64 m = tlo * qi;
  const u32 m0 = (u32)m, m1 = (u32)(m >> 32), q0 = (u32)q, q1 = (u32)(q >> 32);
  const u64 a = mad_u64_u32(m1, q0, (u64)__umulhi(m0, q0));
  u64 b, cmask;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(b), "=s"(cmask) : "v"(m0), "v"(q1), "v"(a));
  u32 c;
  asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(c) : "s"(cmask));
  const u64 e = mad_u64_u32(m1, q1, ((u64)c << 32) | (u32)(b >> 32));
  return (thi + q) - e;
}

// Sum of up to four products y_k h_k with y_k, h_k < 2^61, from 30-bit pieces (lo = v & (2^30 - 1),
// hi = v >> 30 < 2^31): the partial products of each weight 1, 2^30, 2^60 sum in one 64-bit word
// (4 < 2^62, 8 < 2^64, 4 < 2^64) with no carries, so a term costs four v_mad_u64_u32 instead of a
// 128-bit product and add (the base conversions' inner loop).  mont() recombines the 128-bit sum
// once and Montgomery-reduces it: sum R^-1 mod q in [0, q), valid while sum < q 2^64.
constexpr u32 kLo30 = (1u << 30) - 1;
__device__ __forceinline__ u64 split30(u64 v) { return ((v >> 30) << 32) | (v & kLo30); }
struct Sum30 {
  u64 lo = 0, mid = 0, hi = 0;
  __device__ __forceinline__ void add(u32 yl, u32 yh, u32 hl, u32 hh) {
    lo = mad_u64_u32(yl, hl, lo);
    mid = mad_u64_u32(yl, hh, mid);
    mid = mad_u64_u32(yh, hl, mid);
    hi = mad_u64_u32(yh, hh, hi);
  }
  // h2 = split30(h): hl in the low word, hh in the high word
  __device__ __forceinline__ void add(u64 y2, u64 h2) {
    add((u32)y2, (u32)(y2 >> 32), (u32)h2, (u32)(h2 >> 32));
  }
  __device__ __forceinline__ u64 mont(u64 q, u64 qinv) const { return csub(mont_lazy(q, qinv), q); }
  // the same without the final subtraction: [0, 2q)
  __device__ __forceinline__ u64 mont_lazy(u64 q, u64 qinv) const {
    const u64 a = lo + (mid << 30);
    u64 h = (mid >> 34) + (a < lo ? 1 : 0);
    const u64 l = a + (hi << 60);
    h += (hi >> 4) + (l < a ? 1 : 0);
    return mont_reduce_lazy(l, h, q, qinv);
  }
};

// Full reduction of a 128-bit z = (zhi, zlo) with zhi < 2^64 (any value) into [0, q), q < 2^61:
// zhi 2^64 + zlo = zhi (2^64 mod q) + zlo, both terms by the 3-product Shoup (into [0, 3q) each),
// then three conditional subtractions.  The key-switch inner product accumulates up to 16
// products of residues (< 16 q^2 < 2^126) and reduces once.
__device__ __forceinline__ u64 reduce128(u64 zlo, u64 zhi, const ModParams& m) {
  const u64 nq = 0 - m.q;
  u64 r = shoup_q3(zhi, m.r64, m.r64s, nq) + shoup_q3(zlo, 1, m.ones, nq);
  r = csub(r, 4 * m.q);
  r = csub(r, 2 * m.q);
  return csub(r, m.q);
}

// reduce128 for any context modulus (wide ones by reduce128_wide; a wave-uniform branch when m is).
__device__ __forceinline__ u64 reduce128_any(u64 zlo, u64 zhi, const ModParams& m) {
  return m.mu == 0 ? reduce128_wide(zlo, zhi, m) : reduce128(zlo, zhi, m);
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

// t < 2^64 -> t mod q (Shoup by 1: [0, 3q), then two subtractions; wide moduli 2^61 <= q < 2^63:
// the exact quotient, [0, 2q), one subtraction)
__device__ __forceinline__ u64 reduce_word(u64 t, const ModParams& m) {
  if (m.mu == 0) return csub(shoup_lazy(t, 1, m.ones, m.q), m.q);
  u64 r = shoup_q3(t, 1, m.ones, 0 - m.q);
  r = csub(r, 2 * m.q);
  return csub(r, m.q);
}

// Exact a * b mod q for a, b < q and any q < 2^64 (generic entry points only; the context
// kernels use Shoup/Barrett).  q < 2^63: Barrett / reduce128_wide; above, a 64-step
// double-and-add.
__device__ __forceinline__ u64 mulmod_any(u64 a, u64 b, const ModParams& m) {
  if (m.q < (1ull << 63)) return barrett_reduce((u128)a * b, m);
  u64 r = 0;
  for (int i = 63; i >= 0; --i) {
    const u64 r2 = r >= m.q - r ? r - (m.q - r) : r + r;  // 2r mod q without overflow
    r = r2;
    if ((b >> i) & 1) r = r >= m.q - a ? r - (m.q - a) : r + a;
  }
  return r;
}

}  // namespace fhe
