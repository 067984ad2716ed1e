// Rescale (divide-and-round by the last modulus) and Galois automorphisms / rotation for gfx950:
// SURVEY.md §8(f) row 1, the first ciphertext operations after the north-star path.
//
// Not in the reference (its only ciphertext operation is poly_add, /root/reference/ polynomial.py:3-5);
// the definitions are the standard RNS-CKKS ones, restated in oracle/pyoracle.py
// (rescale_coeff / rescale_ntt, automorphism_coeff / automorphism_ntt, rotate):
//   rescale   out_i = (x_i - ((x_last + h) mod q_last - h)) q_last^-1 mod q_i,  h = q_last / 2
//             = floor((X + h) / q_last) mod q_i for the CRT value X (divide and round);
//   sigma_k   a(X) -> a(X^k), k odd: coefficient i -> i k mod 2N (negated past N); in the NTT
//             domain a gather, slot j <- slot brv(((2 brv(j) + 1) k mod 2N - 1) / 2);
//   rotate    (sigma_k c0 + KS0(sigma_k c1), KS1(sigma_k c1)) with the key for sigma_k(s) -> s.
// All HBM-bound elementwise / gather passes (the rotation's cost is its key-switch).
#include "internal.hpp"

namespace fhe {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ u32 brv(u32 x, u32 bits) { return __builtin_bitreverse32(x) >> (32 - bits); }

// Grid: x over coefficients, y = limb, z = poly.  in/out rows at stride N, polys at pin / pout.
__global__ __launch_bounds__(kThreads) void k_automorph(u64* __restrict__ out, u64 pout,
                                                        const u64* __restrict__ in, u64 pin,
                                                        u32 nlimbs, u32 limb0, u32 log_n, u32 k,
                                                        int ntt, const ModParams* __restrict__ mods) {
  const u64 n = 1ull << log_n;
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 l = blockIdx.y;
  const u64 p = blockIdx.z;
  const u64* row = in + p * pin + (u64)l * n;
  u64 v;
  if (ntt) {
    const u32 mask2 = (2u << log_n) - 1;
    const u32 e = ((2 * brv(c, log_n) + 1) * k) & mask2;  // k odd, e odd
    v = row[brv((e - 1) >> 1, log_n)];
  } else {
    const u32 mask2 = (2u << log_n) - 1;
    const u32 i = (c * k) & mask2;  // here k = kinv: the source of output coefficient c
    const u64 q = mods[limb0 + l].q;
    if (i < n) {
      v = row[i];
    } else {
      const u64 x = row[i - n];
      v = x ? q - x : 0;
    }
  }
  out[p * pout + (u64)l * n + c] = v;
}

// Rescale, coefficient form: in [polys][nl][N] -> out [polys][nl - 1][N].  Grid: x over
// coefficients, y = out limb i, z = poly.  tab[i] = {Shoup pair of q_last^-1 mod q_i}, half[i] =
// h mod q_i.
__global__ __launch_bounds__(kThreads) void k_rescale_coeff(u64* __restrict__ out,
                                                            const u64* __restrict__ in, u32 nl,
                                                            u32 log_n,
                                                            const ulonglong2* __restrict__ tab,
                                                            const u64* __restrict__ half,
                                                            const ModParams* __restrict__ mods) {
  const u64 n = 1ull << log_n;
  const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u32 i = blockIdx.y;
  const u64 p = blockIdx.z;
  const ModParams ml = mods[nl - 1], mi = mods[i];
  const u64 h = ml.q >> 1;
  const u64 t = csub(in[(p * nl + nl - 1) * n + c] + h, ml.q);
  const u64 tmp = csub(reduce_word(t, mi) + mi.q - half[i], mi.q);
  const u64 d = in[(p * nl + i) * n + c] + mi.q - tmp;
  const ulonglong2 w = tab[i];
  out[(p * (nl - 1) + i) * n + c] = csub(shoup_lazy(d, w.x, w.y, mi.q), mi.q);
}

// Rescale, NTT form, step 1: last [polys][N] (coefficient form of the last limb) ->
// tmp [polys][nl - 1][N] = ((last + h) mod q_last - h) mod q_i (to be NTT'd over limbs 0..nl-2).
__global__ __launch_bounds__(kThreads) void k_rescale_spread(u64* __restrict__ tmp,
                                                             const u64* __restrict__ last, u32 nl,
                                                             u32 log_n,
                                                             const u64* __restrict__ half,
                                                             const ModParams* __restrict__ mods) {
  const u64 n = 1ull << log_n;
  const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u32 i = blockIdx.y;
  const u64 p = blockIdx.z;
  const ModParams ml = mods[nl - 1], mi = mods[i];
  const u64 t = csub(last[p * n + c] + (ml.q >> 1), ml.q);
  tmp[(p * (nl - 1) + i) * n + c] = csub(reduce_word(t, mi) + mi.q - half[i], mi.q);
}

// Rescale, NTT form, step 2: out_i = (x_i - tmp_i) q_last^-1 mod q_i.
__global__ __launch_bounds__(kThreads) void k_rescale_finish(u64* __restrict__ out,
                                                             const u64* __restrict__ in,
                                                             const u64* __restrict__ tmp, u32 nl,
                                                             u32 log_n,
                                                             const ulonglong2* __restrict__ tab,
                                                             const ModParams* __restrict__ mods) {
  const u64 n = 1ull << log_n;
  const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u32 i = blockIdx.y;
  const u64 p = blockIdx.z;
  const u64 q = mods[i].q;
  const u64 d = in[(p * nl + i) * n + c] + q - tmp[(p * (nl - 1) + i) * n + c];
  const ulonglong2 w = tab[i];
  out[(p * (nl - 1) + i) * n + c] = csub(shoup_lazy(d, w.x, w.y, q), q);
}

inline u64 modinv_u64(u64 a, u64 q) { return powmod_u64(a % q, q - 2, q); }

// k^-1 mod 2^bits for odd k (Newton: each step doubles the correct low bits)
inline u32 modinv_odd_pow2(u32 k, u32 bits) {
  u32 inv = k;
  for (int i = 0; i < 5; ++i) inv *= 2 - k * inv;
  return inv & ((bits >= 32) ? 0xffffffffu : ((1u << bits) - 1));
}


// Double-hoisted rotation sum (launch_rotate_sum_hoisted): the per-rotation inner products of the
// hoisted rotations, each times its plaintext pt_r and summed in Q u P, so that one ModDown serves
// every term:  A_h = sum_r pt_r sum_j sigma_r(ext_j) evk_r,h[j],  C0 = sum_r pt_r sigma_r(c0),
// and for the unrotated term (gal 1, no key) C0 += pt c0, C1 += pt c1 (ModDown(P pt c1 + y) =
// pt c1 + ModDown(y) exactly, so pt c1 joins out_1 after ModDown instead).  Restated by
// oracle/pyoracle.py rotate_sum_hoisted.
// One thread = one position (row r of Q u P, coefficient i) for kRotSumBC ciphertexts, so each
// key word is loaded once for them; the kRotSumBC-ciphertext groups of one (row, 256 positions)
// are dealt to one XCD back to back (their key words then come from its L2).  The NTT-domain
// gather maps every aligned 64-slot block onto one aligned 64-slot block (brv(src) =
// brv(i) k + (k - 1) / 2 mod N: the top bits of brv(i) only reach the top bits of the product),
// so each wavefront's gathered loads stay within 512 contiguous bytes.
struct RotSumTerms {
  u32 count;
  u32 gal[kRotSumMax];
  const u64* kb[kRotSumMax];
  const u64* ka[kRotSumMax];
  const u64* pt[kRotSumMax];
  // per-term ciphertext and ModUp digits (rotate_sum_multi: every term its own); null: the
  // kernel's in / ext
  const u64* in[kRotSumMax];
  const u64* ext[kRotSumMax];
};
// 2 ciphertexts per thread: 110 VGPRs, 4 waves per SIMD for the gathers' latency; 4 took 182 (2
// waves): rot_sum 3.30 -> 2.48 ms per 32 x 8 terms, +18 % terms/s same-box
// (profiles/r06_rotsum_bc_ab.txt)
constexpr u32 kRotSumBC = 2;
// k_rot_sum flags: write the unrotated terms' c1 sum (cadd's second half)
constexpr int kRotSumC1 = 1;

// a + x y for the rotation sum's 128-bit accumulators: narrow moduli (q < 2^61) add exact
// products (at most 16 terms of q^2 < 2^122 each); wide ones reduce every product
template <bool WIDE>
__device__ __forceinline__ void rs_mac(u128& a, u64 x, u64 y, const ModParams& m) {
  const u128 p = (u128)x * y;
  if constexpr (WIDE) {
    a = csub((u64)a + reduce128_wide((u64)p, (u64)(p >> 64), m), m.q);
  } else {
    a += p;
  }
}
template <bool WIDE>
__device__ __forceinline__ u64 rs_fin(u128 a, const ModParams& m) {
  if constexpr (WIDE) return (u64)a;
  return reduce128((u64)a, (u64)(a >> 64), m);
}
// a + x y for x, y < 2^61 by the hand-written 61-bit product (mul_wide61: 4 mads where the
// compiler's u128 product takes 11 VALU with its register-pair moves)
__device__ __forceinline__ void rs_mac61(u128& a, u64 x, u64 y) {
  u64 lo, hi;
  mul_wide61(x, y, lo, hi);
  a += ((u128)hi << 64) | lo;
}

// FAST (every modulus < 2^60, the lz16 contexts, and dnum <= 4): each term's inner product is a
// 128-bit sum on 32-bit halves (dot_wide61) reduced by one Montgomery REDC to t R^-1 in (0, 2q);
// the term's plaintext word enters as p R mod q (one Shoup product by R per term and position,
// shared by the kRotSumBC ciphertexts), so (p R)(t R^-1) = p t adds into the 128-bit sums with
// one mul_wide61 (operands below 2q < 2^61; 16 terms of 4 q^2 stay below 2^126).  Against the u128
// form: 2 x 4 u128 products and 2 reduce128 per term and ciphertext become 2 dot_wide61 + 2 REDC.
template <int DNUM, bool WIDE, bool FAST = false>
__global__ __launch_bounds__(kThreads) void k_rot_sum(u64* __restrict__ acc, u64 acc_ws,
                                                      u64* __restrict__ cadd, int flags,
                                                      const u64* __restrict__ ext0,
                                                      const u64* __restrict__ in0,
                                                      const RotSumTerms tm, u32 rows, u32 L,
                                                      u32 alpha, u32 batch, u32 log_n,
                                                      const ModParams* __restrict__ mods) {
  const u64 n = 1ull << log_n, rn = (u64)rows * n, ln = (u64)L * n;
  const u32 per_row = (u32)(n / kThreads), nbc = (batch + kRotSumBC - 1) / kRotSumBC;
  const u32 xcd = blockIdx.x % 8, k8 = blockIdx.x / 8;
  const u32 bc = k8 % nbc, item = (k8 / nbc) * 8 + xcd;
  if (item >= rows * per_row) return;  // grid rounded up to whole groups of 8
  const u32 r = item / per_row;
  const u64 i = (u64)(item % per_row) * kThreads + threadIdx.x;
  const u64 e = (u64)r * n + i;
  const ModParams m = mods[r];  // rows = the context's L + K limbs in order
  const u32 own = r < L ? r / alpha : 0xffffffffu;
  const u32 b0 = bc * kRotSumBC, nb = min(kRotSumBC, batch - b0);
  u128 s0[kRotSumBC] = {}, s1[kRotSumBC] = {}, a0[kRotSumBC] = {}, a1[kRotSumBC] = {};
  const bool ident = (flags & kRotSumC1) != 0;
  const u32 sh = 32 - log_n, mask2 = (2u << log_n) - 1;
  for (u32 k = 0; k < tm.count; ++k) {
    const u32 g = tm.gal[k];
    const u64 p = tm.pt[k] ? tm.pt[k][e] : 1;  // no plaintext: the term itself (rotate_sum_multi)
    const u64* __restrict__ in = tm.in[k] ? tm.in[k] : in0;
    const u64* __restrict__ ext = tm.ext[k] ? tm.ext[k] : ext0;
    if (g == 1) {  // the unrotated term (workgroup-uniform)
      if (r < L) {
#pragma unroll
        for (u32 bb = 0; bb < kRotSumBC; ++bb) {
          if (bb >= nb) break;
          const u64* ct = in + (u64)(b0 + bb) * 2 * ln + e;
          if constexpr (FAST) {
            rs_mac61(a0[bb], p, ct[0]);
            rs_mac61(a1[bb], p, ct[ln]);
          } else {
            rs_mac<WIDE>(a0[bb], p, ct[0], m);
            rs_mac<WIDE>(a1[bb], p, ct[ln], m);
          }
        }
      }
      continue;
    }
    const u32 gi = ((2 * (__builtin_bitreverse32((u32)i) >> sh) + 1) * g) & mask2;
    const u64 si = __builtin_bitreverse32((gi - 1) >> 1) >> sh;
    const u64 es = (u64)r * n + si;
    u64 kb[DNUM], ka[DNUM];
#pragma unroll
    for (int j = 0; j < DNUM; ++j) {
      kb[j] = tm.kb[k][(u64)j * rn + e];
      ka[j] = tm.ka[k][(u64)j * rn + e];
    }
    if constexpr (FAST) {
      static_assert(!WIDE && DNUM <= 4, "FAST: narrow moduli, dot_wide61 of <= 4 terms");
      u64 pr = shoup_q3(p, m.r64, m.r64s, 0 - m.q);  // p R mod q in [0, 3q)
      pr = csub_fast(pr, 0 - 2 * m.q);                 // [0, 2q)
      const u64 qi = 0 - m.qinv;                       // q^-1 mod 2^64 (mont_redc_x)
#pragma unroll
      for (u32 bb = 0; bb < kRotSumBC; ++bb) {
        if (bb >= nb) break;
        const u32 b = b0 + bb;
        u64 x[DNUM];
#pragma unroll
        for (int j = 0; j < DNUM; ++j)
          x[j] = (u32)j == own ? in[(u64)b * 2 * ln + ln + es] : ext[((u64)j * batch + b) * rn + es];
        u64 lo, hi;
        dot_wide61<DNUM>(x, kb, lo, hi);
        rs_mac61(s0[bb], pr, mont_redc_x(lo, hi, m.q, qi));
        dot_wide61<DNUM>(x, ka, lo, hi);
        rs_mac61(s1[bb], pr, mont_redc_x(lo, hi, m.q, qi));
        if (r < L) rs_mac61(a0[bb], p, in[(u64)b * 2 * ln + es]);
      }
      continue;
    }
#pragma unroll
    for (u32 bb = 0; bb < kRotSumBC; ++bb) {
      if (bb >= nb) break;
      const u32 b = b0 + bb;
      u128 t0 = 0, t1 = 0;
#pragma unroll
      for (int j = 0; j < DNUM; ++j) {
        const u64 x = (u32)j == own ? in[(u64)b * 2 * ln + ln + es]
                                    : ext[((u64)j * batch + b) * rn + es];
        rs_mac<WIDE>(t0, x, kb[j], m);
        rs_mac<WIDE>(t1, x, ka[j], m);
      }
      rs_mac<WIDE>(s0[bb], p, rs_fin<WIDE>(t0, m), m);
      rs_mac<WIDE>(s1[bb], p, rs_fin<WIDE>(t1, m), m);
      if (r < L) rs_mac<WIDE>(a0[bb], p, in[(u64)b * 2 * ln + es], m);
    }
  }
#pragma unroll
  for (u32 bb = 0; bb < kRotSumBC; ++bb) {
    if (bb >= nb) break;
    const u32 b = b0 + bb;
    acc[(u64)b * rn + e] = rs_fin<WIDE>(s0[bb], m);
    acc[acc_ws + (u64)b * rn + e] = rs_fin<WIDE>(s1[bb], m);
    if (r < L) {
      cadd[(u64)b * ln + e] = rs_fin<WIDE>(a0[bb], m);
      if (ident) cadd[(u64)(batch + b) * ln + e] = rs_fin<WIDE>(a1[bb], m);
    }
  }
}
}  // namespace

int build_galois_tables(fhe_ctx* c) {
  // rescale tables for every last limb l in [1, L): entry [l][i], i < l
  const u32 L = c->L;
  std::vector<ulonglong2> tab((size_t)L * L, ulonglong2{0, 0});
  std::vector<u64> half((size_t)L * L, 0);
  for (u32 l = 1; l < L; ++l) {
    const u64 ql = c->moduli[l];
    for (u32 i = 0; i < l; ++i) {
      const u64 q = c->moduli[i];
      const u64 inv = modinv_u64(ql, q);
      tab[(size_t)l * L + i] = ulonglong2{inv, (u64)(((u128)inv << 64) / q)};
      half[(size_t)l * L + i] = (ql >> 1) % q;
    }
  }
  FHE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&c->d_rs_tab), tab.size() * sizeof(ulonglong2)));
  FHE_HIP_CHECK(hipMemcpy(c->d_rs_tab, tab.data(), tab.size() * sizeof(ulonglong2),
                          hipMemcpyHostToDevice));
  FHE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&c->d_rs_half), half.size() * sizeof(u64)));
  FHE_HIP_CHECK(hipMemcpy(c->d_rs_half, half.data(), half.size() * sizeof(u64), hipMemcpyHostToDevice));
  return kOk;
}

int launch_automorphism(const fhe_ctx* c, u64* out, u64 pout, const u64* in, u64 pin, u32 polys,
                        u32 limb0, u32 nlimbs, u32 galois_elt, bool ntt, hipStream_t s) {
  const u32 two_n = 2u << c->log_n;
  if ((galois_elt & 1) == 0 || galois_elt >= two_n) {
    set_error("automorphism: the Galois element must be odd and below 2N");
    return kInvalid;
  }
  if ((u64)polys * nlimbs == 0) return kOk;
  // coefficient form gathers through k^-1 mod 2N (odd elements form a group mod 2^(logN+1))
  u32 k = galois_elt;
  if (!ntt) k = (u32)modinv_odd_pow2(galois_elt, c->log_n + 1);
  if (int rc = check_grid(c->n / kThreads, kThreads, nlimbs, polys, "automorphism")) return rc;
  const dim3 g((u32)(c->n / kThreads), nlimbs, polys);
  k_automorph<<<g, kThreads, 0, s>>>(out, pout, in, pin, nlimbs, limb0, c->log_n, k, ntt ? 1 : 0,
                                     c->d_mods);
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

size_t rescale_workspace_bytes(const fhe_ctx* c, u32 polys, u32 nl) {
  return (size_t)polys * nl * c->n * sizeof(u64);
}

int launch_rescale(const fhe_ctx* c, u64* out, const u64* in, u32 polys, u32 nl, bool ntt,
                   void* ws, hipStream_t s) {
  if (nl < 2 || nl > c->L) {
    set_error("rescale: need 2 <= limbs <= L (the input spans Q-limbs 0 .. limbs-1)");
    return kInvalid;
  }
  if (polys == 0) return kOk;
  const u64 n = c->n;
  const ulonglong2* tab = c->d_rs_tab + (size_t)(nl - 1) * c->L;
  const u64* half = c->d_rs_half + (size_t)(nl - 1) * c->L;
  if (int rc = check_grid(n / kThreads, kThreads, nl - 1, polys, "rescale")) return rc;
  const dim3 g((u32)(n / kThreads), nl - 1, polys);
  if (!ntt) {
    k_rescale_coeff<<<g, kThreads, 0, s>>>(out, in, nl, c->log_n, tab, half, c->d_mods);
    FHE_HIP_CHECK(hipGetLastError());
    return kOk;
  }
  // NTT form: INTT of the last limb, spread it over the other limbs, NTT those, finish
  u64* last = static_cast<u64*>(ws);           // [polys][N]
  u64* tmp = last + (u64)polys * n;            // [polys][nl - 1][N]
  int rc;
  if ((rc = launch_ntt_strided(c, false, in + (u64)(nl - 1) * n, (u64)nl * n, last, n, polys,
                                nl - 1, 1, s)))
    return rc;
  if (!c->wide) {
    // the spread rides on the column-forward pass (k_rescale_col) and the finish on the row-forward
    // pass (k_moddown_row with one half and the q_last^-1 table): out_i = (x_i - NTT(tmp)_i)
    // q_last^-1 straight from registers; tmp exists only column-passed
    const u64 sn = (u64)(nl - 1) * n;
    if ((rc = launch_rescale_col(c, last, tmp, polys, nl - 1, half, s))) return rc;
    ModDownRowArgs da{tmp, out, out, in, 0, nl, nl - 1, 0, polys, KsEpilogue{}};
    da.ep.out_bs = sn;
    da.halves = 1;
    da.pinv = tab;
    return launch_moddown_row(c, da, s);
  }
  k_rescale_spread<<<g, kThreads, 0, s>>>(tmp, last, nl, c->log_n, half, c->d_mods);
  FHE_HIP_CHECK(hipGetLastError());
  if ((rc = launch_ntt(c, true, tmp, tmp, polys, (u64)(nl - 1) * n, 0, nl - 1, s))) return rc;
  k_rescale_finish<<<g, kThreads, 0, s>>>(out, in, tmp, nl, c->log_n, tab, c->d_mods);
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

size_t rotate_workspace_bytes(const fhe_ctx* c, u32 batch) {
  // sigma(c1) and sigma(c0) [batch][L][N], then the key-switch's own workspace
  return 2 * (size_t)batch * c->L * c->n * sizeof(u64) + keyswitch_workspace_bytes(c, c->L, batch);
}

int launch_rotate(const fhe_ctx* c, u64* out, const u64* in, u32 galois_elt, const u64* rot_b,
                  const u64* rot_a, u32 batch, void* ws, hipStream_t s) {
  if (c->K == 0) {
    set_error("rotate: context has no special primes (K = 0)");
    return kInvalid;
  }
  if (batch == 0) return kOk;
  const u32 L = c->L;
  const u64 n = c->n, ln = (u64)L * n;
  // Infinity-Cache-sized passes (ks_pass_batch), each in the front of the workspace
  if (const u32 pass = ks_pass_batch(c, batch); pass < batch) {
    for (u32 b0 = 0; b0 < batch; b0 += pass) {
      if (int rc = launch_rotate(c, out + b0 * 2 * ln, in + b0 * 2 * ln, galois_elt, rot_b, rot_a,
                                 std::min(pass, batch - b0), ws, s))
        return rc;
    }
    return kOk;
  }
  u64* sc1 = static_cast<u64*>(ws);  // [batch][L][N]
  u64* sc0 = sc1 + batch * ln;
  u64* kws = sc0 + batch * ln;
  int rc;
  // sigma(c0) is gathered by the ModDown finish itself where that is k_moddown_row
  const bool gather0 = ks_fused(c);
  if ((!gather0 &&
       (rc = launch_automorphism(c, sc0, ln, in, 2 * ln, batch, 0, L, galois_elt, true, s))) ||
      (rc = launch_automorphism(c, sc1, ln, in + ln, 2 * ln, batch, 0, L, galois_elt, true, s)))
    return rc;
  // key-switch sigma(c1): its coefficient form goes to the tail of the key-switch workspace
  const size_t kbytes = keyswitch_workspace_bytes(c, L, batch);
  u64* c_all = reinterpret_cast<u64*>(reinterpret_cast<char*>(kws) + kbytes) - batch * ln;
  const bool prep = ks_prepared(c);  // the INTT emits ModUp's scaled inputs
  if ((rc = launch_ntt_strided(c, false, sc1, ln, c_all, ln, batch, 0, L, s,
                               prep ? c->d_nfold_up : nullptr, prep && ks_split30(c))))
    return rc;
  CAll call = CAll::contiguous(c_all, L, n);
  call.scaled = prep;
  // out = (sigma(c0) + ks0, ks1) straight out of the key-switch's ModDown finish (KsEpilogue)
  KsEpilogue ep;
  ep.out_bs = 2 * ln;
  ep.add0 = gather0 ? in : sc0;
  ep.add_bs = gather0 ? 2 * ln : ln;
  ep.add_gal = gather0 ? galois_elt : 0;
  return launch_keyswitch_shard(c, out, out + ln, call, sc1, rot_b, rot_a, 0, L, batch, kws, s,
                                &ep);
}

size_t rotate_hoisted_workspace_bytes(const fhe_ctx* c, u32 batch) {
  // c1 (NTT form) and its coefficient form, sigma(c0) [batch][L][N], then the key-switch workspace
  // (its ext region holds the NTT-form digits across the rotations)
  // (+ [2 batch][K][N] for the fused ModDown's INTT output)
  return (3 * (size_t)c->L + 2 * (size_t)c->K) * batch * c->n * sizeof(u64) +
         keyswitch_workspace_bytes(c, c->L, batch);
}

// Hoisted rotations (Halevi-Shoup): the ModUp of c1 -- INTT, base conversion, NTT of every digit,
// the bulk of a key-switch -- runs once, and each rotation reads the NTT-form digits through its
// automorphism inside the inner product (sigma commutes with the digit decomposition up to the
// conversion's multiples of the digit modulus, which the key-switch tolerates either way).  Per
// rotation: the gathered inner product, then ModDown with sigma(c0) added in its finish (gathered
// there too on the fused ModDown; a separate sigma(c0) pass on the wide contexts).
// Restated by oracle/pyoracle.py rotate_hoisted; decrypts to sigma_k(m) like fhe_rotate, but is
// not bit-identical to it (ModUp of sigma(c1) vs sigma of ModUp(c1)).
int launch_rotate_hoisted(const fhe_ctx* c, u64* out, const u64* in, const u32* galois,
                          const u64* const* rot_b, const u64* const* rot_a, u32 count, u32 batch,
                          void* ws, hipStream_t s) {
  if (c->K == 0) {
    set_error("rotate_hoisted: context has no special primes (K = 0)");
    return kInvalid;
  }
  const u32 two_n = 2u << c->log_n;
  for (u32 r = 0; r < count; ++r)
    if ((galois[r] & 1) == 0 || galois[r] >= two_n) {
      set_error("rotate_hoisted: every Galois element must be odd and below 2N");
      return kInvalid;
    }
  if (batch == 0 || count == 0) return kOk;
  const u32 L = c->L;
  const u64 n = c->n, ln = (u64)L * n;
  u64* c1 = static_cast<u64*>(ws);  // [batch][L][N] NTT form
  u64* c_all = c1 + batch * ln;     // [batch][L][N] coefficient form
  u64* sc0 = c_all + batch * ln;    // [batch][L][N]
  u64* ydn = sc0 + batch * ln;      // [2 batch][K][N]
  u64* kws = ydn + 2 * batch * (u64)c->K * n;
  FHE_HIP_CHECK(hipMemcpy2DAsync(c1, ln * sizeof(u64), in + ln, 2 * ln * sizeof(u64),
                                 ln * sizeof(u64), batch, hipMemcpyDeviceToDevice, s));
  int rc;
  // prepared INTT (the ModUp digits' (D^_k)^-1 folded in) where the hoisted ModUp takes the fused
  // conversion pass (rns.hip hoist_up)
  const bool prep = ks_prepared(c);
  if ((rc = launch_ntt_strided(c, false, c1, ln, c_all, ln, batch, 0, L, s,
                               prep ? c->d_nfold_up : nullptr, prep && ks_split30(c))))
    return rc;
  CAll call = CAll::contiguous(c_all, L, n);
  call.scaled = prep;
  KsHoist up;
  up.modup_only = true;
  if ((rc = launch_keyswitch_shard(c, nullptr, nullptr, call, c1, nullptr, nullptr, 0, L, batch,
                                   kws, s, nullptr, &up)))
    return rc;
  for (u32 r = 0; r < count; ++r) {
    u64* o = out + (u64)r * batch * 2 * ln;
    KsHoist h;
    h.galois = galois[r];
    h.ydn = ydn;
    KsEpilogue ep;
    ep.out_bs = 2 * ln;
    if (ks_hoist_fused_down(c)) {  // the ModDown finish reads c0 through sigma itself
      ep.add0 = in;
      ep.add_bs = 2 * ln;
      ep.add_gal = galois[r];
    } else {
      if ((rc = launch_automorphism(c, sc0, ln, in, 2 * ln, batch, 0, L, galois[r], true, s)))
        return rc;
      ep.add0 = sc0;
      ep.add_bs = ln;
    }
    if ((rc = launch_keyswitch_shard(c, o, o + ln, call, c1, rot_b[r], rot_a[r], 0, L, batch, kws,
                                     s, &ep, &h)))
      return rc;
  }
  return kOk;
}

size_t rotate_sum_hoisted_workspace_bytes(const fhe_ctx* c, u32 batch) {
  // c1's coefficient form [batch][L][N], the c0 / c1 addends [2][batch][L][N], the fused ModDown's
  // INTT output [2 batch][K][N], then the key-switch workspace (ext digits, accumulators)
  return (3 * (size_t)c->L + 2 * (size_t)c->K) * batch * c->n * sizeof(u64) +
         keyswitch_workspace_bytes(c, c->L, batch);
}

namespace {
// The rotation sums' workspace regions (rotate_sum_hoisted_workspace_bytes)
struct RotSumWs {
  u64* c_all;  // [batch][L][N] coefficient form of the c1 being ModUp'ed
  u64* cadd;   // [2][batch][L][N]: the c0 sum, then the unrotated terms' c1 sum
  u64* ydn;    // [2 batch][K][N] the fused ModDown's INTT output
  u64* kws;    // key-switch workspace: ext [dnum][batch][L + K][N], then the accumulators
};
RotSumWs rotsum_ws(const fhe_ctx* c, void* ws, u32 batch) {
  const u64 ln = (u64)c->L * c->n;
  RotSumWs w;
  w.c_all = static_cast<u64*>(ws);
  w.cadd = w.c_all + batch * ln;
  w.ydn = w.cadd + 2 * batch * ln;
  w.kws = w.ydn + 2 * batch * (u64)c->K * c->n;
  return w;
}

int rotsum_check(const fhe_ctx* c, u32 count, const u32* galois, const char* who) {
  if (c->K == 0) {
    set_error(std::string(who) + ": context has no special primes (K = 0)");
    return kInvalid;
  }
  if (count > kRotSumMax) {
    set_error(std::string(who) + ": at most 16 terms per call");
    return kInvalid;
  }
  if (c->dnum > 8) {
    set_error(std::string(who) + ": dnum > 8");
    return kUnsupported;
  }
  const u32 two_n = 2u << c->log_n;
  for (u32 r = 0; r < count; ++r)
    if ((galois[r] & 1) == 0 || galois[r] >= two_n) {
      set_error(std::string(who) + ": every Galois element must be odd and below 2N");
      return kInvalid;
    }
  return kOk;
}

// ModUp of in's c1 ([batch][2][L][N], NTT form) into the ext region at kws (w.kws, or another
// region of ext_words(c, batch) words: a ModUp-only key-switch writes nothing past its digits):
// the prepared INTT (the fused hoisted ModUp's scaled inputs) and the hoisted ModUp (rns.hip,
// modup_only)
u64 ext_words(const fhe_ctx* c, u32 batch) {
  return (u64)c->dnum * batch * (c->L + c->K) * c->n;
}
int rotsum_modup(const fhe_ctx* c, const u64* in, u32 batch, const RotSumWs& w, hipStream_t s,
                 u64* kws = nullptr) {
  const u32 L = c->L;
  const u64 ln = (u64)L * c->n;
  const bool prep = ks_prepared(c);
  if (int rc = launch_ntt_strided(c, false, in + ln, 2 * ln, w.c_all, ln, batch, 0, L, s,
                                  prep ? c->d_nfold_up : nullptr, prep && ks_split30(c)))
    return rc;
  CAll call = CAll::contiguous(w.c_all, L, c->n);
  call.scaled = prep;
  KsHoist up;
  up.modup_only = true;
  return launch_keyswitch_shard(c, nullptr, nullptr, call, in + ln, nullptr, nullptr, 0, L, batch,
                                kws ? kws : w.kws, s, nullptr, &up);
}

// One k_rot_sum launch over the terms tm of ciphertexts in (whose ModUp is in the ext region when
// a term is rotated): the accumulators and cadd get the sums (flags: kRotSumC1)
int rotsum_pass(const fhe_ctx* c, const u64* in, const RotSumTerms& tm, int flags, u32 batch,
                const RotSumWs& w, hipStream_t s) {
  const u32 L = c->L, rows = L + c->K;
  const u64 n = c->n;
  const u64 blocks = (u64)rows * (n / kThreads);
  const u64 grid = (blocks + 7) / 8 * 8 * ((batch + kRotSumBC - 1) / kRotSumBC);
  if (int rc = check_grid(grid, kThreads, 1, 1, "rotate_sum")) return rc;
  u64* acc = ks_acc_region(c, w.kws, L, batch);
  const u64 acc_ws = (u64)batch * rows * n;
  const u64* ext = w.kws;
  switch (c->dnum) {
#define X(d)                                                                                      \
  case d:                                                                                         \
    if (c->wide)                                                                                  \
      k_rot_sum<d, true><<<dim3((u32)grid), kThreads, 0, s>>>(                                    \
          acc, acc_ws, w.cadd, flags, ext, in, tm, rows, L, c->alpha, batch, c->log_n, c->d_mods);\
    else if (c->lz16 && d <= 4)                                                                   \
      k_rot_sum<(d <= 4 ? d : 4), false, true><<<dim3((u32)grid), kThreads, 0, s>>>(              \
          acc, acc_ws, w.cadd, flags, ext, in, tm, rows, L, c->alpha, batch, c->log_n, c->d_mods);\
    else                                                                                          \
      k_rot_sum<d, false><<<dim3((u32)grid), kThreads, 0, s>>>(                                   \
          acc, acc_ws, w.cadd, flags, ext, in, tm, rows, L, c->alpha, batch, c->log_n, c->d_mods);\
    break;
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8)
#undef X
  }
  FHE_HIP_CHECK(hipGetLastError());
  prof_mark(s, "rot_sum");
  return kOk;
}

// ONE ModDown of both sums into out [batch][2][L][N]; out_0 += the c0 sum, out_1 += the unrotated
// terms' c1 sum (c1) in its finish
int rotsum_moddown(const fhe_ctx* c, u64* out, const u64* d2ref, bool c1, u32 batch,
                   const RotSumWs& w, hipStream_t s) {
  const u32 L = c->L;
  const u64 ln = (u64)L * c->n;
  KsHoist h;
  h.acc_ready = true;
  h.ydn = w.ydn;
  KsEpilogue ep;
  ep.out_bs = 2 * ln;
  ep.add0 = w.cadd;
  ep.add1 = c1 ? w.cadd + batch * ln : nullptr;
  ep.add_bs = ln;
  return launch_keyswitch_shard(c, out, out + ln, CAll::contiguous(w.c_all, L, c->n), d2ref,
                                nullptr, nullptr, 0, L, batch, w.kws, s, &ep, &h);
}
}  // namespace

// Double hoisting (the inner loop of a baby-step / giant-step linear transform): ModUp(c1) once
// (as launch_rotate_hoisted), one k_rot_sum pass that forms every rotation's inner product through
// its automorphism, multiplies it by pt_r and sums the terms in Q u P, then ONE ModDown per
// accumulator with the c0 (and unrotated c1) sums added in its finish.  Against count hoisted
// rotations + count plaintext products + a sum, it saves count - 1 ModDowns and every per-rotation
// output round trip.  Restated by oracle/pyoracle.py rotate_sum_hoisted.
int launch_rotate_sum_hoisted(const fhe_ctx* c, u64* out, const u64* in, const u32* galois,
                              const u64* const* rot_b, const u64* const* rot_a,
                              const u64* const* pt, u32 count, u32 batch, void* ws,
                              hipStream_t s) {
  if (int rc = rotsum_check(c, count, galois, "rotate_sum_hoisted")) return rc;
  RotSumTerms tm{};
  tm.count = count;
  bool ident = false, rotated = false;
  for (u32 r = 0; r < count; ++r) {
    tm.gal[r] = galois[r];
    tm.kb[r] = rot_b[r];
    tm.ka[r] = rot_a[r];
    tm.pt[r] = pt[r];
    ident = ident || galois[r] == 1;
    rotated = rotated || galois[r] != 1;
  }
  if (batch == 0) return kOk;
  const RotSumWs w = rotsum_ws(c, ws, batch);
  int rc;
  if (rotated && (rc = rotsum_modup(c, in, batch, w, s))) return rc;
  if ((rc = rotsum_pass(c, in, tm, ident ? kRotSumC1 : 0, batch, w, s))) return rc;
  return rotsum_moddown(c, out, in + (u64)c->L * c->n, ident, batch, w, s);
}

size_t rotate_sum_multi_workspace_bytes(const fhe_ctx* c, u32 count, u32 batch) {
  // the rotation sum's workspace, then the ModUp digits of every rotated term past the first
  return rotate_sum_hoisted_workspace_bytes(c, batch) +
         (size_t)(count > 1 ? count - 1 : 0) * ext_words(c, batch) * sizeof(u64);
}

namespace {
// The giant-step sum: every rotated term's ModUp into its own digit region (the first in w's ext
// region, the others in `extra`, ext_words each), then ONE k_rot_sum pass over all the terms (each
// with its own ciphertext and digits, no plaintext: the accumulators are written once) and ONE
// ModDown.
int rotsum_multi(const fhe_ctx* c, u64* out, const u64* const* cts, const u32* galois,
                 const u64* const* rot_b, const u64* const* rot_a, u32 count, u32 batch,
                 const RotSumWs& w, u64* extra, hipStream_t s) {
  RotSumTerms tm{};
  tm.count = count;
  u32 nrot = 0;
  for (u32 r = 0; r < count; ++r) {
    tm.gal[r] = galois[r];
    tm.kb[r] = rot_b ? rot_b[r] : nullptr;
    tm.ka[r] = rot_a ? rot_a[r] : nullptr;
    tm.pt[r] = nullptr;
    tm.in[r] = cts[r];
    if (galois[r] == 1) continue;
    u64* region = nrot == 0 ? w.kws : extra + (u64)(nrot - 1) * ext_words(c, batch);
    if (int rc = rotsum_modup(c, cts[r], batch, w, s, region)) return rc;
    tm.ext[r] = region;
    ++nrot;
  }
  int rc;
  if ((rc = rotsum_pass(c, cts[0], tm, kRotSumC1, batch, w, s))) return rc;
  return rotsum_moddown(c, out, cts[0] + (u64)c->L * c->n, true, batch, w, s);
}
}  // namespace

// sum_r rot_{galois[r]}(cts[r]) over count DIFFERENT ciphertexts with ONE ModDown (the giant-step
// sum of a baby-step / giant-step linear transform, Bossuat et al.'s second hoisting): a ModUp of
// each rotated term's own c1, one k_rot_sum pass over all the terms, then one ModDown of the summed
// accumulators with the sigma(c0) sum (and the unrotated terms' c0, c1) added in its finish.
// Restated by oracle/pyoracle.py rotate_sum_multi.
int launch_rotate_sum_multi(const fhe_ctx* c, u64* out, const u64* const* cts, const u32* galois,
                            const u64* const* rot_b, const u64* const* rot_a, u32 count,
                            u32 batch, void* ws, hipStream_t s) {
  if (int rc = rotsum_check(c, count, galois, "rotate_sum_multi")) return rc;
  if (batch == 0 || count == 0) return kOk;
  u64* extra = reinterpret_cast<u64*>(static_cast<char*>(ws) +
                                      rotate_sum_hoisted_workspace_bytes(c, batch));
  return rotsum_multi(c, out, cts, galois, rot_b, rot_a, count, batch, rotsum_ws(c, ws, batch),
                      extra, s);
}

size_t linear_transform_workspace_bytes(const fhe_ctx* c, u32 n2, u32 batch) {
  // the rotation sums' workspace, the n2 giant-step inputs [n2][batch][2][L][N], then the giant
  // steps' extra ModUp digit regions (rotate_sum_multi)
  return rotate_sum_multi_workspace_bytes(c, n2, batch) +
         (size_t)n2 * batch * 2 * c->L * c->n * sizeof(u64);
}

// Baby-step / giant-step linear transform with both hoistings (CKKS bootstrapping's CoeffToSlot /
// SlotToCoeff shape):  out = sum_g rot_{giant[g]}( sum_b pt[g n1 + b] rot_{baby[b]}(in) ).
// ONE ModUp of in's c1 serves every baby step of every giant step; each giant step's inner sum is
// one k_rot_sum pass + one ModDown (as launch_rotate_sum_hoisted, bit for bit); the giant sum is
// launch_rotate_sum_multi (one ModDown).  Restated by oracle/pyoracle.py linear_transform.
int launch_linear_transform(const fhe_ctx* c, u64* out, const u64* in, u32 n1, u32 n2,
                            const u32* baby, const u64* const* baby_b, const u64* const* baby_a,
                            const u32* giant, const u64* const* giant_b,
                            const u64* const* giant_a, const u64* const* pt, u32 batch, void* ws,
                            hipStream_t s) {
  if (n1 == 0 || n2 == 0 || n1 > kRotSumMax || n2 > kRotSumMax) {
    set_error("linear_transform: n1 and n2 must be 1..16");
    return kInvalid;
  }
  if (int rc = rotsum_check(c, n1, baby, "linear_transform")) return rc;
  if (int rc = rotsum_check(c, n2, giant, "linear_transform")) return rc;
  if (batch == 0) return kOk;
  const RotSumWs w = rotsum_ws(c, ws, batch);
  const u64 ct_words = (u64)batch * 2 * c->L * c->n;
  u64* inner = reinterpret_cast<u64*>(static_cast<char*>(ws) +
                                      rotate_sum_hoisted_workspace_bytes(c, batch));
  u64* extra = inner + (u64)n2 * ct_words;
  bool ident = false, rotated = false;
  for (u32 b = 0; b < n1; ++b) {
    ident = ident || baby[b] == 1;
    rotated = rotated || baby[b] != 1;
  }
  int rc;
  if (rotated && (rc = rotsum_modup(c, in, batch, w, s))) return rc;
  const u64* inner_ptr[kRotSumMax];
  for (u32 g = 0; g < n2; ++g) {
    RotSumTerms tm{};
    tm.count = n1;
    for (u32 b = 0; b < n1; ++b) {
      tm.gal[b] = baby[b];
      tm.kb[b] = baby_b ? baby_b[b] : nullptr;
      tm.ka[b] = baby_a ? baby_a[b] : nullptr;
      tm.pt[b] = pt[(u64)g * n1 + b];
    }
    u64* ig = inner + (u64)g * ct_words;
    if ((rc = rotsum_pass(c, in, tm, ident ? kRotSumC1 : 0, batch, w, s)) ||
        (rc = rotsum_moddown(c, ig, in + (u64)c->L * c->n, ident, batch, w, s)))
      return rc;
    inner_ptr[g] = ig;
  }
  return rotsum_multi(c, out, inner_ptr, giant, giant_b, giant_a, n2, batch, w, extra, s);
}

}  // namespace fhe
