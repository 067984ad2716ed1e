// RNS fast base conversion, ModUp / ModDown and the hybrid key-switch inner product (gfx950).
//
// None of this exists in the reference; the spec is SURVEY.md §8a':
//   baseconv   y_k = [x_k (S^_k)^-1]_{s_k};  out_t = sum_k y_k (S^_k mod t) mod t   (no correction)
//   ModUp      digit j (Q-limbs D_j) extended to every other limb of Q u P
//   key-switch acc{0,1} = sum_j NTT(ModUp_j(INTT d2)) (.) evk{b,a}_j  over Q u P
//   ModDown    out_i = (acc_i - NTT(baseconv_{P->Q}(INTT acc_P))_i) P^-1 mod q_i
// Restated bit-exactly by oracle/fhe_oracle.c (oracle_baseconv / oracle_keyswitch).
//
// Every constant multiplier is a Shoup pair, so a conversion costs S + S*T Shoup products per
// coefficient and no Barrett; partial sums stay in [0, 2t) by one conditional subtraction each.
#include <algorithm>
#include <vector>

#include "internal.hpp"

namespace fhe {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxSrc = 16;
// Word offsets of a conversion's S source rows within one ciphertext (kernel argument): rows need
// not be contiguous -- the rank-major all-gather output of the sharded key-switch puts a digit's
// limbs in different rank blocks (CAll).
struct KOff {
  u64 o[kMaxSrc];
};
inline KOff rows_contiguous(u32 S, u64 n) {
  KOff k{};
  for (u32 i = 0; i < S; ++i) k.o[i] = (u64)i * n;
  return k;
}

// out row r -> ctx limb: r < n0 ? base0 + r : base1 + (r - n0)
struct RowMap {
  u32 n0, base0, base1;
  __host__ __device__ u32 limb(u32 r) const { return r < n0 ? base0 + r : base1 + (r - n0); }
};

// in: S rows (stride N) over ctx limbs src0..src0+S-1; out: T rows (stride N), row r over
// ctx limb map.limb(r); rows whose limb lies in [skip_lo, skip_hi) are left untouched.
// inv[k] = (S^_k)^-1 mod s_k; hat[k * hs + limb] = S^_k mod limb.  Batch b = blockIdx.y reads
// in + b * in_bs and writes out + b * out_bs.
// The launch's conversion constants (S x T Shoup pairs' first words and each row's modulus) are
// staged in LDS once per workgroup, so the row loop reads broadcast LDS words instead of waiting
// on a scalar load per row; each output is a 128-bit sum of S full products y_k * (S^_k mod t)
// (< S t^2 < 2^126), reduced once (Montgomery for S < 8, else reduce128), instead of S Shoup
// products and S subtractions.
// WIDE (contexts with a modulus >= 2^61): the products' sum could pass 2^128, so each product
// y_k (S^_k mod t) is reduced on its own (reduce128_wide) and the sum kept below t.
constexpr int kMaxRows = 64;
template <int S, bool WIDE>
__global__ __launch_bounds__(kThreads) void k_baseconv(const u64* __restrict__ in, u64 in_bs,
                                                       KOff koff, u32 src0, u64* __restrict__ out,
                                                       u64 out_bs,
                                                       u32 T, RowMap map, u32 skip_lo, u32 skip_hi,
                                                       u64 n, const ulonglong2* __restrict__ inv,
                                                       const ulonglong2* __restrict__ hat, u32 hs,
                                                       const ModParams* __restrict__ mods) {
  // S < 8: y_k < 2^61 and S 2^61 < 2^64, so the sum stays below t 2^64 and one Montgomery
  // reduction (R = 2^64, folded into the table's second word) replaces reduce128
  constexpr bool kMont = !WIDE && S < 8;
  // S <= 4: the sums run on 30-bit pieces (Sum30), the LDS holding split30(hat)
  constexpr bool kSplit = !WIDE && S <= 4;
  __shared__ u64 s_hat[kMaxRows * S];
  __shared__ u32 s_limb[kMaxRows];
  for (u32 e = threadIdx.x; e < T * S; e += blockDim.x) {
    const u32 r = e / S, k = e % S;
    const ulonglong2 h = hat[(u64)k * hs + map.limb(r)];
    s_hat[e] = kSplit ? split30(h.y) : kMont ? h.y : h.x;
  }
  for (u32 r = threadIdx.x; r < T; r += blockDim.x) s_limb[r] = map.limb(r);
  __syncthreads();
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  in += (u64)blockIdx.y * in_bs;
  out += (u64)blockIdx.y * out_bs;
  u64 y[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const u64 qk = mods[src0 + k].q;
    const ulonglong2 w = inv[k];
    y[k] = csub(shoup_lazy(in[koff.o[k] + i], w.x, w.y, qk), qk);
    if constexpr (kSplit) y[k] = split30(y[k]);
  }
  for (u32 r = 0; r < T; ++r) {
    const u32 limb = s_limb[r];
    if (limb >= skip_lo && limb < skip_hi) continue;
    if constexpr (kSplit) {
      Sum30 acc;
#pragma unroll
      for (int k = 0; k < S; ++k) acc.add(y[k], s_hat[r * S + k]);
      const ModParams& m = mods[limb];
      out[(u64)r * n + i] = acc.mont(m.q, m.qinv);
      continue;
    }
    if constexpr (WIDE) {
      const ModParams& m = mods[limb];
      u64 sum = 0;
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const u128 p = (u128)y[k] * s_hat[r * S + k];
        sum = csub(sum + reduce128_wide((u64)p, (u64)(p >> 64), m), m.q);
      }
      out[(u64)r * n + i] = sum;
      continue;
    }
    u128 acc = 0;
#pragma unroll
    for (int k = 0; k < S; ++k) acc += (u128)y[k] * s_hat[r * S + k];
    if constexpr (kMont) {
      const ModParams& m = mods[limb];
      out[(u64)r * n + i] = csub(mont_reduce_lazy((u64)acc, (u64)(acc >> 64), m.q, m.qinv), m.q);
    } else {
      out[(u64)r * n + i] = reduce128((u64)acc, (u64)(acc >> 64), mods[limb]);
    }
  }
}

// acc{0,1}[b][r][i] = sum_j e_j[b][r][i] * evk{b,a}[j][r][i] mod t over own Q-limbs then P-limbs;
// e_j = d2_own row when row r's limb is in digit j, else ext[j][b] row (NTT form).  Grid: x over
// coefficients, y = row r (limb and modulus uniform per workgroup).  Each thread holds its
// 2 DNUM evaluation-key words in registers and walks the batch, so the key -- the dominant
// traffic of a key-switch -- is read once per batch; the DNUM products of a sum are accumulated
// as 128-bit integers (< 16 q^2) and reduced once (reduce128).
constexpr int kMaxDnum = 16;
template <int DNUM>
__global__ __launch_bounds__(kThreads) void k_ks_inner(u64* __restrict__ acc, u64 acc_ws,
                                                       const u64* __restrict__ ext,
                                                       const u64* __restrict__ d2_own,
                                                       const u64* __restrict__ evk_b,
                                                       const u64* __restrict__ evk_a, u32 rows,
                                                       u32 nq, RowMap map, u32 alpha, u32 L,
                                                       u32 batch, u32 log_n,
                                                       const ModParams* __restrict__ mods,
                                                       u32 gal) {
  const u32 r = blockIdx.y;
  const u64 n = 1ull << log_n, rn = (u64)rows * n;
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u64 e = (u64)r * n + i;
  // hoisted rotation (gal != 0): the digits and d2_own are read through sigma_gal's NTT-domain
  // gather (slot i <- slot brv(((2 brv(i) + 1) gal mod 2N - 1) / 2), galois.hip), the key at i
  u64 si = i;
  if (gal) {
    const u32 sh = 32 - log_n;
    const u32 g = ((2 * (__builtin_bitreverse32((u32)i) >> sh) + 1) * gal) & ((2u << log_n) - 1);
    si = __builtin_bitreverse32((g - 1) >> 1) >> sh;
  }
  const u64 es = (u64)r * n + si;
  const u32 limb = map.limb(r);
  const ModParams m = mods[limb];
  const u32 own = limb < L ? limb / alpha : 0xffffffffu;
  u64 kb[DNUM], ka[DNUM];
#pragma unroll
  for (int j = 0; j < DNUM; ++j) {
    kb[j] = evk_b[(u64)j * rn + e];
    ka[j] = evk_a[(u64)j * rn + e];
  }
  if (m.mu == 0) {  // wide modulus (uniform): DNUM products could pass 2^128, reduce each
    for (u32 b = 0; b < batch; ++b) {
      u64 s0 = 0, s1 = 0;
#pragma unroll
      for (int j = 0; j < DNUM; ++j) {
        const u64 x = (u32)j == own ? d2_own[((u64)b * nq + r) * n + si]
                                    : ext[((u64)j * batch + b) * rn + es];
        const u128 p0 = (u128)x * kb[j], p1 = (u128)x * ka[j];
        s0 = csub(s0 + reduce128_wide((u64)p0, (u64)(p0 >> 64), m), m.q);
        s1 = csub(s1 + reduce128_wide((u64)p1, (u64)(p1 >> 64), m), m.q);
      }
      acc[(u64)b * rn + e] = s0;
      acc[acc_ws + (u64)b * rn + e] = s1;
    }
    return;
  }
  for (u32 b = 0; b < batch; ++b) {
    u128 s0 = 0, s1 = 0;
#pragma unroll
    for (int j = 0; j < DNUM; ++j) {
      const u64 x = (u32)j == own ? d2_own[((u64)b * nq + r) * n + si]
                                  : ext[((u64)j * batch + b) * rn + es];
      s0 += (u128)x * kb[j];
      s1 += (u128)x * ka[j];
    }
    acc[(u64)b * rn + e] = reduce128((u64)s0, (u64)(s0 >> 64), m);
    acc[acc_ws + (u64)b * rn + e] = reduce128((u64)s1, (u64)(s1 >> 64), m);
  }
}

// out{0,1}[b][r][i] = (acc{0,1}[b][r][i] - conv{0,1}[b][r][i]) * P^-1 mod q over own Q-limbs.
// Grid: x over coefficients, y = own Q-limb r, z = batch entry b.
// (with the KsEpilogue: outputs at b * out_bs, plus add{0,1} when set)
__global__ __launch_bounds__(kThreads) void k_moddown_finish(u64* __restrict__ out0,
                                                             u64* __restrict__ out1,
                                                             const u64* __restrict__ acc,
                                                             u64 acc_ws, u32 rows,
                                                             const u64* __restrict__ conv,
                                                             u32 nq, u32 limb0, u32 log_n,
                                                             const ulonglong2* __restrict__ pinv,
                                                             const ModParams* __restrict__ mods,
                                                             KsEpilogue ep) {
  const u64 n = 1ull << log_n;
  const u32 r = blockIdx.y, b = blockIdx.z;
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u32 limb = limb0 + r;
  const u64 q = mods[limb].q;
  const ulonglong2 w = pinv[limb];
  const u64 total = (u64)gridDim.z * nq * n;
  const u64 e = ((u64)b * nq + r) * n + i;
  const u64 ai = ((u64)b * rows + r) * n + i;  // acc rows [0, nq) are the own Q-limbs
  const u64 c0 = conv[e], c1 = conv[total + e];
  u64 r0 = csub(shoup_lazy(acc[ai] + q - c0, w.x, w.y, q), q);
  u64 r1 = csub(shoup_lazy(acc[acc_ws + ai] + q - c1, w.x, w.y, q), q);
  const u64 ea = (u64)b * ep.add_bs + (u64)r * n + i;
  if (ep.add0) r0 = csub(r0 + ep.add0[ea], q);
  if (ep.add1) r1 = csub(r1 + ep.add1[ea], q);
  const u64 eo = (u64)b * ep.out_bs + (u64)r * n + i;
  out0[eo] = r0;
  out1[eo] = r1;
}

// Prologue of the fused conversion column pass (ntt.hip k_modup_col), ModUp and ModDown:
// y[b][k][i] = [x_k (D^_k)^-1]_{d_k} over S source rows at in + b in_bs + koff[k] (moduli
// mods[mod0 + k]).  Grid: x over coefficients, y = k, z = b.
__global__ __launch_bounds__(kThreads) void k_modup_scale(const u64* __restrict__ in, u64 in_bs,
                                                          KOff koff, u32 mod0,
                                                          u64* __restrict__ y, u32 S,
                                                          u32 log_n,
                                                          const ulonglong2* __restrict__ inv,
                                                          const ModParams* __restrict__ mods,
                                                          bool split) {
  const u64 n = 1ull << log_n;
  const u32 k = blockIdx.y, b = blockIdx.z;
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const u64 q = mods[mod0 + k].q;
  const ulonglong2 w = inv[k];
  // split30: k_modup_col reads its sources as Sum30 pieces on non-lz16 contexts (ks_split30)
  const u64 v = csub(shoup_lazy(in[(u64)b * in_bs + koff.o[k] + i], w.x, w.y, q), q);
  y[((u64)b * S + k) * n + i] = split ? split30(v) : v;
}

// host Shoup-pair table -> device ulonglong2 array (same 16-byte layout)
int upload(ulonglong2** dptr, const std::vector<Pair64>& v) {
  static_assert(sizeof(Pair64) == sizeof(ulonglong2), "table entry layout");
  if (v.empty()) return kOk;
  FHE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(dptr), v.size() * sizeof(Pair64)));
  FHE_HIP_CHECK(hipMemcpy(*dptr, v.data(), v.size() * sizeof(Pair64), hipMemcpyHostToDevice));
  return kOk;
}

// One base conversion launch over `batch` independent inputs (strides in_bs / out_bs words).
struct BcArgs {
  const u64* in;
  u64 in_bs;
  KOff koff;
  u32 src0;
  u64* out;
  u64 out_bs;
  u32 T;
  RowMap map;
  u32 skip_lo, skip_hi;
  u32 batch;
};

template <int S, bool WIDE>
void launch_bc(const BcArgs& a, u64 n, const ulonglong2* inv, const ulonglong2* hat, u32 hs,
               const ModParams* mods, hipStream_t s) {
  const dim3 g((u32)((n + kThreads - 1) / kThreads), a.batch);
  // the kernel stages at most kMaxRows target rows' constants: longer targets go in chunks
  for (u32 r0 = 0; r0 < a.T; r0 += kMaxRows) {
    const u32 t = std::min<u32>(kMaxRows, a.T - r0);
    RowMap m = a.map;
    if (r0 < m.n0) {
      m.n0 -= r0;
      m.base0 += r0;
    } else {
      m.base1 += r0 - m.n0;
      m.n0 = 0;
    }
    k_baseconv<S, WIDE><<<g, kThreads, 0, s>>>(a.in, a.in_bs, a.koff, a.src0, a.out + (u64)r0 * n,
                                               a.out_bs, t,
                                         m, a.skip_lo, a.skip_hi, n, inv, hat, hs, mods);
  }
}

int baseconv_any(u32 S, const BcArgs& a, u64 n, const ulonglong2* inv, const ulonglong2* hat,
                 u32 hs, const ModParams* mods, bool wide, hipStream_t s) {
  if (int rc = check_grid((n + kThreads - 1) / kThreads, kThreads, a.batch, 1, "baseconv"))
    return rc;
  switch (S) {
#define X(k)                                    \
  case k:                                       \
    if (wide)                                   \
      launch_bc<k, true>(a, n, inv, hat, hs, mods, s); \
    else                                        \
      launch_bc<k, false>(a, n, inv, hat, hs, mods, s); \
    break;
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)
#undef X
    default:
      set_error("baseconv: more than 16 source limbs");
      return kUnsupported;
  }
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

inline u32 grid_for(u64 work) {
  const u64 blocks = (work + kThreads - 1) / kThreads;
  return (u32)(blocks < 256 * 16 ? (blocks ? blocks : 1) : 256 * 16);
}

}  // namespace

int build_rns_tables(fhe_ctx* c) {
  if (c->K == 0) return kOk;
  const u32 L = c->L, K = c->K, M = L + K, alpha = c->alpha;
  if (alpha > (u32)kMaxSrc || K > (u32)kMaxSrc) {
    set_error("ctx_create: key-switch needs alpha <= 16 and K <= 16");
    return kUnsupported;
  }
  std::vector<Pair64> up_inv((size_t)c->dnum * alpha), up_hat((size_t)c->dnum * alpha * M);
  for (u32 j = 0; j < c->dnum; ++j) {
    const u32 lo = j * alpha, hi = std::min(L, lo + alpha);
    if (lo >= L) break;
    std::vector<Pair64> inv, hat;
    conv_tables(c->moduli, lo, hi - lo, inv, hat);
    std::copy(inv.begin(), inv.end(), up_inv.begin() + (size_t)j * alpha);
    std::copy(hat.begin(), hat.end(), up_hat.begin() + (size_t)j * alpha * M);
  }
  // Montgomery-scaled copy for the fused lz16 ModUp: .y = D^_k 2^128 mod t (host only: the
  // device tables built from it are d_modup_hat_rw / _rwp below)
  std::vector<Pair64> up_hat_r(up_hat);
  for (size_t i = 0; i < up_hat.size(); ++i) {
    const u64 t = c->moduli[i % M];
    up_hat_r[i].y = (u64)(((u128)up_hat[i].y << 64) % t);
  }
  std::vector<Pair64> dn_inv, dn_hat, pinv(L);
  conv_tables(c->moduli, L, K, dn_inv, dn_hat);
  for (u32 i = 0; i < L; ++i) {
    const u64 q = c->moduli[i];
    u64 pm = 1;
    for (u32 k = 0; k < K; ++k) pm = mulmod_u64(pm, c->moduli[L + k] % q, q);
    pinv[i] = shoup_pair(powmod_u64(pm, q - 2, q), q);
  }
  // The INTT of d2 ahead of a key-switch folds ModUp's (D^_k)^-1 into its last stage (N^-1 fold)
  std::vector<Pair64> nf_up((size_t)4 * M, Pair64{0, 0});
  for (u32 k = 0; k < L; ++k) {
    const u64 q = c->moduli[k];
    const u32 j = k / alpha;
    const u64 s = mulmod_u64(powmod_u64(c->n % q, q - 2, q), up_inv[(size_t)j * alpha + (k - j * alpha)].x, q);
    const u64 w = powmod_u64(powmod_u64(c->psi[k], q - 2, q), c->n / 2, q);  // psi^-N/2
    nf_up[4 * k] = shoup_pair(s, q);
    nf_up[4 * k + 1] = shoup_pair(mulmod_u64(w, s, q), q);
  }
  // ModDown's P-row INTT folds the conversion's (P^_k)^-1 into its last stage (N^-1 fold)
  std::vector<Pair64> nf_down((size_t)4 * M, Pair64{0, 0});
  for (u32 k = 0; k < K; ++k) {
    const u64 p = c->moduli[L + k];
    const u64 s = mulmod_u64(powmod_u64(c->n % p, p - 2, p), dn_inv[k].x, p);  // N^-1 (P^_k)^-1
    const u64 w = powmod_u64(powmod_u64(c->psi[L + k], p - 2, p), c->n / 2, p);  // psi^-N/2
    nf_down[4 * (L + k)] = shoup_pair(s, p);
    nf_down[4 * (L + k) + 1] = shoup_pair(mulmod_u64(w, s, p), p);
  }
  // {h, h w0} for the fused conversions (k_modup_col folds stage 0's twiddle w0 = psi^(N/2) into
  // the rows that stage multiplies)
  // (pscale: times P^-1 mod t as well for the Q limbs t < L)
  auto with_w0 = [&](const std::vector<Pair64>& hat, bool pscale) {
    std::vector<Pair64> out(hat.size());
    for (size_t i = 0; i < hat.size(); ++i) {
      const u32 t = (u32)(i % M);
      const u64 tm = c->moduli[t];
      const u64 w0 = powmod_u64(c->psi[t], c->n / 2, tm);
      const u64 h = pscale && t < L ? mulmod_u64(hat[i].y, pinv[t].x, tm) : hat[i].y;
      out[i] = Pair64{h, mulmod_u64(h, w0, tm)};
    }
    return out;
  };
  std::vector<Pair64> rpinv(L);
  for (u32 i = 0; i < L; ++i) {
    const u64 q = c->moduli[i];
    rpinv[i] = shoup_pair(mulmod_u64((u64)(((u128)1 << 64) % q), pinv[i].x, q), q);
  }
  int rc;
  if ((rc = upload(&c->d_modup_hat_w, with_w0(up_hat, false))) ||
      (rc = upload(&c->d_modup_hat_rw, with_w0(up_hat_r, false))) ||
      (rc = upload(&c->d_moddown_hat_w, with_w0(dn_hat, false))) ||
      (rc = upload(&c->d_modup_hat_rwp, with_w0(up_hat_r, true))) ||
      (rc = upload(&c->d_moddown_hat_wp, with_w0(dn_hat, true))) ||
      (rc = upload(&c->d_rpinv, rpinv)))
    return rc;
  if ((rc = upload(&c->d_modup_inv, up_inv)) || (rc = upload(&c->d_modup_hat, up_hat)) ||
      (rc = upload(&c->d_moddown_inv, dn_inv)) || (rc = upload(&c->d_moddown_hat, dn_hat)) ||
      (rc = upload(&c->d_pinv, pinv)) || (rc = upload(&c->d_nfold_down, nf_down)) ||
      (rc = upload(&c->d_nfold_up, nf_up)))
    return rc;
  return kOk;
}

size_t keyswitch_workspace_bytes(const fhe_ctx* c, u32 nlimbs, u32 batch) {
  const u64 rows = nlimbs + c->K;
  // ext [dnum][batch][rows][N] + acc [2][batch][rows][N] + conv [2][batch][nlimbs][N]
  // + y [batch][alpha][N] (fused ModUp) + c_all [batch][L][N] (single-device form, at the tail)
  return (u64)batch * ((u64)c->dnum * rows + 2 * rows + 2 * nlimbs + c->alpha + c->L) * c->n *
         sizeof(u64);
}

int launch_keyswitch_shard(const fhe_ctx* c, u64* ks0, u64* ks1, const u64* c_all,
                           const u64* d2_own, const u64* evk_b, const u64* evk_a, u32 limb0,
                           u32 nlimbs, u32 batch, void* ws, hipStream_t s) {
  return launch_keyswitch_shard(c, ks0, ks1, CAll::contiguous(c_all, c->L, c->n), d2_own, evk_b,
                                evk_a, limb0, nlimbs, batch, ws, s);
}

int launch_keyswitch_shard(const fhe_ctx* c, u64* ks0, u64* ks1, const CAll& call,
                           const u64* d2_own, const u64* evk_b, const u64* evk_a, u32 limb0,
                           u32 nlimbs, u32 batch, void* ws, hipStream_t s,
                           const KsEpilogue* epi, const KsHoist* hoist) {
  if (c->K == 0) {
    set_error("keyswitch: context has no special primes (K = 0)");
    return kInvalid;
  }
  if (c->dnum > (u32)kMaxDnum) {
    set_error("keyswitch: dnum > 16");
    return kUnsupported;
  }
  if (batch == 0) return kOk;
  // the coefficient-wise kernels put rows on y and (2 x) the batch on y / z
  if (int rc = check_grid(c->n / kThreads, kThreads, (u64)nlimbs + c->K, 2 * (u64)batch,
                          "keyswitch"))
    return rc;
  KsEpilogue ep = epi ? *epi : KsEpilogue{};
  if (ep.out_bs == 0) ep.out_bs = (u64)nlimbs * c->n;
  // Aliasing (fhecore.h): an output may be d2_own itself (in place: same start, the contiguous
  // [batch][nlimbs][N] layout) or lie wholly outside it.  k_ks_row_fin writes outputs while other
  // workgroups still read d2_own, but each thread reads the d2 words at exactly the positions it
  // later stores, so the in-place call is race-free there (and the other finishes run after the
  // last read of d2_own); any other overlap is refused here, before the first launch.
  if (!(hoist && hoist->modup_only)) {
    const u64 nw = (u64)nlimbs * c->n;
    if (int rc = ks_check_alias(ks0, ks1, d2_own, (u64)batch * nw,
                                (u64)(batch - 1) * ep.out_bs + nw, ep.out_bs == nw, "keyswitch"))
      return rc;
  }
  const u32 L = c->L, K = c->K, M = L + K, alpha = c->alpha, rows = nlimbs + K;
  const u64 n = c->n, rn = (u64)rows * n, B = batch;
  u64* ext = static_cast<u64*>(ws);          // [dnum][B][rows][N]
  u64* acc = ext + (u64)c->dnum * B * rn;    // [2][B][rows][N]
  u64* conv = acc + 2 * B * rn;              // [2][B][nlimbs][N]
  const u64 acc_ws = B * rn;
  const RowMap map{nlimbs, limb0, L};
  int rc;
  // Fused path: for dnum <= 4 the digits get only their column-forward pass here, and one fused
  // kernel (ntt.hip, k_ks_row_inner) runs every digit's row-forward pass and the inner product
  // (no NTT-form ext in HBM, no separate inner-product pass); otherwise full NTTs + k_ks_inner.
  // Wide contexts (a modulus >= 2^61) take the unfused kernels: the fused ones rely on lazy
  // ranges and 128-bit sums that need q < 2^61.
  // Hoisted rotations (KsHoist) take the unfused kernels: the digits must exist in NTT form in
  // HBM so that each rotation's inner product can gather them through its automorphism.
  const bool fused = !hoist && ks_fused(c);
  const u32 gal = hoist ? hoist->galois : 0;
  // The hoisted ModUp (modup_only) on the contexts the fused ModUp serves: the same conversion
  // column pass (plain table: the gathered inner products read plain residues), then one
  // row-forward pass per digit range (launch_ntt_row_fwd_r2), so the NTT-form digits land in HBM
  // for the gathers; in place of k_baseconv + a full NTT per range.
  const bool hoist_up = hoist && hoist->modup_only && ks_prepared(c);
  // Fused ModUp (with the fused row kernel, digits of <= 4 limbs): the base conversion runs
  // inside the column-forward pass (ntt.hip k_modup_col) after a one-pass prologue that scales the
  // digit's source rows; the extended rows are never written in coefficient form.
  const bool fused_up = (fused && alpha <= 4) || hoist_up;
  // lz16 fused ModUp: the extended rows come out times R = 2^64 (d_modup_hat_rw / _rwp), which the fused
  // row kernel's Montgomery inner product cancels (KsRowArgs::mont)
  const bool mont_ext = fused_up && !hoist_up && c->lz16;
  if (call.scaled && !fused_up && (!hoist || hoist->modup_only)) {
    set_error("keyswitch: a prepared (pre-scaled) input needs the fused ModUp (ks_prepared)");
    return kInvalid;
  }
  // ModDown's finish: k_moddown_row after the fused conversion (fused_down; a hoisted rotation's
  // inner step too, with its own scratch for the INTT output) or after k_baseconv (fused), else
  // the unfused k_moddown_finish
  const bool fused_down = K <= 4 && ((fused && (u64)c->dnum * rows >= 2 * (u64)K) ||
                                     (hoist && hoist->ydn && ks_hoist_fused_down(c)));
  // ModDown's P^-1 folded into the accumulators' Q rows (the ModUp conversion tables of the Q
  // targets and the own digit's R factor carry P^-1) and into the P -> Q conversion table, so
  // k_moddown_row's finish is a subtraction: the lz16 fused ModUp with the fused ModDown
  const bool pscale = mont_ext && fused_down;
  // k_moddown_finish adds its addend rows un-permuted: a sigma-gathered addend
  // (KsEpilogue::add_gal, which only k_moddown_row implements) reaching it would give a wrong
  // ciphertext with no error, so a caller whose path predicate (ks_fused / ks_hoist_fused_down)
  // drifts from this selection is refused before anything is launched
  if (ep.add_gal && !fused_down && !fused) {
    set_error("keyswitch: a sigma-gathered epilogue addend needs a k_moddown_row finish");
    return kInvalid;
  }
  if (!hoist || hoist->modup_only) {  // ModUp (a hoisted rotation's inner step skips it)
  u64* yws = conv + 2 * B * (u64)nlimbs * n;  // [B][alpha][N]
  auto ntt_fwd = [&](u64* p, u32 l0, u32 nl) {
    return fused ? launch_ntt_col_fwd(c, p, rn, p, rn, batch, l0, nl, s)
                 : launch_ntt(c, true, p, p, batch, rn, l0, nl, s);
  };
  // ModUp + NTT, per digit, for every row outside the digit itself.  Prepared inputs (no
  // per-digit scaling pass into the shared yws) put every digit's conversion pass in one launch.
  ModUpColArgs pend[4];
  u32 npend = 0;
  for (u32 j = 0; j < c->dnum; ++j) {
    const u32 lo = j * alpha, hi = std::min(L, lo + alpha);
    u64* e = ext + (u64)j * B * rn;
    KOff ko{};  // the digit's source rows in c_all
    for (u32 k = 0; k < hi - lo; ++k) ko.o[k] = call.off(lo + k, n);
    if (fused_up) {
      const u32 S = hi - lo;
      // the conversion's inputs y_k = [x_k (D^_k)^-1]: already in c_all when it is prepared (its
      // INTT folded the factor in), else one scaling pass into yws
      const u64* ysrc = call.ptr;
      u64 ybs = call.bs, yoff[4] = {};
      for (u32 k = 0; k < S; ++k) yoff[k] = ko.o[k];
      if (!call.scaled) {
        k_modup_scale<<<dim3((u32)(n / kThreads), S, batch), kThreads, 0, s>>>(
            call.ptr, call.bs, ko, lo, yws, S, c->log_n, c->d_modup_inv + (size_t)j * alpha,
            c->d_mods, ks_split30(c));
        FHE_HIP_CHECK(hipGetLastError());
        ysrc = yws;
        ybs = (u64)S * n;
        for (u32 k = 0; k < S; ++k) yoff[k] = (u64)k * n;
      }
      // this rank's own rows of digit j are skipped: ks_row_inner takes them from d2_own
      const u32 own_lo = std::max(lo, limb0), own_hi = std::min(hi, limb0 + nlimbs);
      const u32 skip_len = own_hi > own_lo ? own_hi - own_lo : 0;
      const u32 skip_at = skip_len ? own_lo - limb0 : rows;
      const ModUpColArgs ma{ysrc, ybs, {yoff[0], yoff[1], yoff[2], yoff[3]}, e, rn, S,
                            rows - skip_len, skip_at, skip_len, nlimbs, limb0, L, batch,
                            (pscale     ? c->d_modup_hat_rwp
                             : mont_ext ? c->d_modup_hat_rw
                                        : c->d_modup_hat_w) +
                                (size_t)j * alpha * M,
                            M};
      if (call.scaled && npend < 4) {
        pend[npend++] = ma;
        continue;
      }
      if ((rc = launch_modup_col(c, ma, s))) return rc;
      continue;
    }
    const BcArgs up{call.ptr, call.bs, ko, lo, e, rn, rows, map, lo, hi, batch};
    if ((rc = baseconv_any(hi - lo, up, n, c->d_modup_inv + (size_t)j * alpha,
                           c->d_modup_hat + (size_t)j * alpha * M, M, c->d_mods, c->wide, s)))
      return rc;
    // own Q-limbs outside [lo, hi): up to two ranges, then the P-limbs
    const u32 a0 = limb0, a1 = std::min(limb0 + nlimbs, lo);
    if (a1 > a0 && (rc = ntt_fwd(e, a0, a1 - a0))) return rc;
    const u32 b0 = std::max(limb0, hi), b1 = limb0 + nlimbs;
    if (b1 > b0 && (rc = ntt_fwd(e + (u64)(b0 - limb0) * n, b0, b1 - b0))) return rc;
    if ((rc = ntt_fwd(e + (u64)nlimbs * n, L, K))) return rc;
  }
  if (npend && (rc = launch_modup_cols(c, pend, npend, s))) return rc;
  if (hoist_up) {
    // the row-forward passes of every digit's extended rows: [0, lo) and [hi, rows), whose limbs
    // are [limb0, limb0 + lo) and (the own Q-limbs past the digit, then P) [hi, L + K) when this
    // is the single-device form (limb0 = 0, nlimbs = L)
    for (u32 j = 0; j < c->dnum; ++j) {
      const u32 lo = j * alpha, hi = std::min(L, lo + alpha);
      u64* e = ext + (u64)j * B * rn;
      if (limb0 != 0 || nlimbs != L) {
        set_error("keyswitch: the hoisted ModUp is single-device (all Q-limbs)");
        return kInvalid;
      }
      if ((rc = launch_ntt_row_fwd_r2(c, e, rn, e, rn, batch, 0, lo, s)) ||
          (rc = launch_ntt_row_fwd_r2(c, e + (u64)hi * n, rn, e + (u64)hi * n, rn, batch, hi,
                                      rows - hi, s)))
        return rc;
    }
  }
  prof_mark(s, "ks_modup");
  if (hoist) return kOk;  // modup_only: the NTT-form digits stay in the workspace's ext region
  }
  // the fused row kernel also runs the first (row) pass of ModDown's INTT on the special rows
  const bool row_pinv = fused && fused_down;
  // With P^-1 in the constants the Q rows wait for ModDown's conversion and finish in the same
  // workgroup (k_ks_row_fin): the row kernel covers only the special rows first, their column
  // inverse runs in place in the accumulators (the ext region stays intact for the Q rows), and
  // neither the accumulators' Q rows nor k_moddown_row's pass over them touch HBM.
  // (outputs are d2_own itself or disjoint from it: ks_check_alias above)
  const bool qfin = pscale && row_pinv;
  if (fused) {
    KsRowArgs ka{acc, acc_ws, ext, B * rn, d2_own, evk_b, evk_a, rows, nlimbs, limb0, L,
                 alpha, L, batch, mont_ext};
    ka.pinv = row_pinv ? 1u : 0u;
    ka.rscale = pscale ? c->d_rpinv : nullptr;
    if (qfin) {
      ka.row0 = nlimbs;
      ka.nrows = K;
    }
    if ((rc = launch_ks_row_inner(c, ka, s))) return rc;
  }
  const dim3 gi((u32)(n / kThreads), rows);
  if (!fused && !(hoist && hoist->acc_ready)) switch (c->dnum) {
#define X(k)                                                                                     \
  case k:                                                                                        \
    k_ks_inner<k><<<gi, kThreads, 0, s>>>(acc, acc_ws, ext, d2_own, evk_b, evk_a, rows, nlimbs, \
                                          map, alpha, L, batch, c->log_n, c->d_mods, gal);      \
    break;
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)
#undef X
  }
  FHE_HIP_CHECK(hipGetLastError());
  prof_mark(s, "ks_inner");
  // ModDown: INTT the P rows of both accumulators, convert P -> own Q-limbs, NTT, finish
  u64* accp = acc + (u64)nlimbs * n;
  // Fused ModDown (fused path, K <= 4): the P -> Q conversion runs inside the column-forward
  // pass of the conversion NTT (k_modup_col, as ModUp), on the P rows the INTT has already scaled
  // into the ext region (free once the inner product has run): conv is never written in
  // coefficient form.
  if (fused_down) {
    // the INTT writes y = [x_k (P^_k)^-1]_{p_k} straight into [2 batch][K][N] (its last stage
    // folds N^-1 (P^_k)^-1, c->d_nfold_down): no separate scaling pass
    u64* ydn = qfin ? accp : hoist ? hoist->ydn : ext;
    const u64 yps = qfin ? rn : (u64)K * n;  // poly stride of the scaled P rows
    if ((rc = row_pinv ? launch_ntt_col_inv(c, accp, rn, ydn, yps, 2 * batch, L, K, s,
                                            c->d_nfold_down, ks_split30(c))
                       : launch_ntt_strided(c, false, accp, rn, ydn, yps, 2 * batch, L, K,
                                            s, c->d_nfold_down, ks_split30(c))))
      return rc;
    prof_mark(s, "ks_moddown_conv");
    const ModUpColArgs md{ydn, yps, {0, n, 2 * n, 3 * n}, conv, (u64)nlimbs * n, K, nlimbs,
                          nlimbs, 0, nlimbs, limb0, 0, 2 * batch,
                          pscale ? c->d_moddown_hat_wp : c->d_moddown_hat_w, M};
    if ((rc = launch_modup_col(c, md, s))) return rc;
    prof_mark(s, "ks_moddown_col");
    if (qfin) {
      const KsFinArgs fa{ext, B * rn, d2_own, evk_b, evk_a, rows, nlimbs, limb0, alpha, L, batch,
                         c->d_rpinv, conv, ks0, ks1, ep};
      if ((rc = launch_ks_row_fin(c, fa, s))) return rc;
      prof_mark(s, "ks_row_fin");
      return kOk;
    }
    const ModDownRowArgs da{conv, ks0, ks1, acc, acc_ws, rows, nlimbs, limb0, batch, ep};
    if ((rc = launch_moddown_row(c, da, s))) return rc;
    prof_mark(s, "moddown_row_finish");
    return kOk;
  }
  if ((rc = launch_ntt(c, false, accp, accp, 2 * batch, rn, L, K, s))) return rc;
  const BcArgs down{accp, rn, rows_contiguous(K, n), L, conv, (u64)nlimbs * n, nlimbs,
                    RowMap{nlimbs, limb0, 0}, 0, 0, 2 * batch};
  if ((rc = baseconv_any(K, down, n, c->d_moddown_inv, c->d_moddown_hat, M, c->d_mods, c->wide, s)))
    return rc;
  prof_mark(s, "ks_moddown_conv");
  if (fused) {  // conversion NTT's row pass finishes ModDown in its epilogue
    if ((rc = launch_ntt_col_fwd(c, conv, (u64)nlimbs * n, conv, (u64)nlimbs * n, 2 * batch, limb0,
                                 nlimbs, s)))
      return rc;
    prof_mark(s, "ks_moddown_col");
    const ModDownRowArgs da{conv, ks0, ks1, acc, acc_ws, rows, nlimbs, limb0, batch, ep};
    if ((rc = launch_moddown_row(c, da, s))) return rc;
    prof_mark(s, "moddown_row_finish");
    return kOk;
  }
  if ((rc = launch_ntt(c, true, conv, conv, 2 * batch, (u64)nlimbs * n, limb0, nlimbs, s)))
    return rc;
  k_moddown_finish<<<dim3((u32)(n / kThreads), nlimbs, batch), kThreads, 0, s>>>(
      ks0, ks1, acc, acc_ws, rows, conv, nlimbs, limb0, c->log_n, c->d_pinv, c->d_mods, ep);
  FHE_HIP_CHECK(hipGetLastError());
  prof_mark(s, "moddown_finish");
  return kOk;
}

int launch_baseconv(const fhe_ctx* c, u64* out, const u64* in, u32 s0, u32 S, u32 t0, u32 T,
                    hipStream_t s) {
  const u32 M = c->L + c->K;
  if (S == 0 || T == 0 || s0 + S > M || t0 + T > M || (s0 < t0 + T && t0 < s0 + S)) {
    set_error("baseconv: limb ranges out of bounds or overlapping");
    return kInvalid;
  }
  // the (s0, S) tables, cached on the context: built, uploaded and synchronised once
  ulonglong2* d_tab = nullptr;
  {
    auto* cc = const_cast<fhe_ctx*>(c);
    std::lock_guard<std::mutex> lock(cc->bc_mutex);
    const uint64_t key = ((uint64_t)s0 << 32) | S;
    for (auto& t : cc->bc_tables)
      if (t.first == key) d_tab = t.second;
    if (!d_tab) {
      std::vector<Pair64> inv, hat;
      conv_tables(c->moduli, s0, S, inv, hat);
      FHE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d_tab), (inv.size() + hat.size()) * 16));
      hipError_t e = hipMemcpyAsync(d_tab, inv.data(), inv.size() * 16, hipMemcpyHostToDevice, s);
      if (e == hipSuccess)
        e = hipMemcpyAsync(d_tab + S, hat.data(), hat.size() * 16, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);  // the host vectors outlive the copies
      if (e != hipSuccess) {
        // never cache a table whose upload did not complete: a later call would read garbage
        (void)hipFree(d_tab);
        set_error(std::string("baseconv: table upload: ") + hipGetErrorString(e));
        return kDevice;
      }
      cc->bc_tables.emplace_back(key, d_tab);  // registered only once it is complete
    }
  }
  const BcArgs a{in, 0, rows_contiguous(S, c->n), s0, out, 0, T, RowMap{T, t0, 0}, 0, 0, 1};
  return baseconv_any(S, a, c->n, d_tab, d_tab + S, M, c->d_mods, c->wide, s);
}

}  // namespace fhe
