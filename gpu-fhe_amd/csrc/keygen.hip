// Sampling, key generation, encryption and decryption: the operations
// that turn HomMult / key-switch / rotation into end-to-end checks with real keys.  Not in the
// reference; restated by oracle/pyoracle.py (philox, sample_*, keygen_*, encrypt_*, decrypt).
//
// Randomness is counter-based (Philox4x32-10, the Random123 construction), so every sample is a
// pure function of (seed, stream tag, poly, limb, coefficient): GPU and oracle agree bit for bit
// and no generator state lives on the device.
//   uniform mod q   floor(r q / 2^128) of a 128-bit draw (bias < 2^-67 for q < 2^61)
//   ternary         (r mod 3) - 1 of a 32-bit draw, the same integer on every limb
//   error           centred binomial, eta = 21 (sd ~3.2): popcount of 21 bits minus 21 bits
// Keys and ciphertexts are NTT form over their limbs (the layout of the rest of the library).
#include "../../include/fhecore.h"
#include "internal.hpp"

namespace fhe {
namespace {

constexpr int kThreads = 256;

struct P4 {
  u32 x, y, z, w;
};

__host__ __device__ inline P4 philox4x32_10(P4 c, u32 k0, u32 k1) {
  constexpr u32 M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  for (int r = 0; r < 10; ++r) {
    const u64 p0 = (u64)M0 * c.x, p1 = (u64)M1 * c.z;
    c = P4{(u32)(p1 >> 32) ^ c.y ^ k0, (u32)p1, (u32)(p0 >> 32) ^ c.w ^ k1, (u32)p0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

enum Kind : int { kUniform = 0, kTernary = 1, kError = 2 };

// out rows [poly][limb][N] (poly stride pstride) over ctx limbs limb0 + l.  Grid: x over
// coefficients, y = limb, z = poly.  The draw for (poly, coefficient) of a small distribution does
// not depend on the limb, so every limb holds the same integer.
__global__ __launch_bounds__(kThreads) void k_sample(u64* __restrict__ out, u64 pstride,
                                                     u32 limb0, u32 log_n, int kind, u32 seed_lo,
                                                     u32 seed_hi, u32 tag,
                                                     const ModParams* __restrict__ mods) {
  const u64 n = 1ull << log_n;
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 l = blockIdx.y, p = blockIdx.z;
  const u32 limb = limb0 + l;
  const u64 q = mods[limb].q;
  u64 v;
  if (kind == kUniform) {
    const P4 r = philox4x32_10(P4{c, limb, p, tag}, seed_lo, seed_hi);
    const u64 lo = ((u64)r.y << 32) | r.x, hi = ((u64)r.w << 32) | r.z;
    const u128 t = (u128)hi * q + (u64)(((u128)lo * q) >> 64);
    v = (u64)(t >> 64);
  } else {
    const P4 r = philox4x32_10(P4{c, 0xffffffffu, p, tag}, seed_lo, seed_hi);
    int64_t s;
    if (kind == kTernary) {
      s = (int64_t)(r.x % 3u) - 1;
    } else {
      const u64 bits = ((u64)r.y << 32) | r.x;
      s = (int64_t)__popcll(bits & 0x1fffffull) - (int64_t)__popcll((bits >> 21) & 0x1fffffull);
    }
    v = s >= 0 ? (u64)s : q - (u64)(-s);
  }
  out[(u64)p * pstride + (u64)l * n + c] = v;
}

// out = x + y * s over [polys][nlimbs][N] rows, NTT form: c0 + c1 s (decryption) and friends.
// s has one row per limb (broadcast over polys).  Grid: x over coefficients, y = limb, z = poly.
__global__ __launch_bounds__(kThreads) void k_mac_s(u64* __restrict__ out, u64 pout,
                                                    const u64* __restrict__ x, u64 px,
                                                    const u64* __restrict__ y, u64 py,
                                                    const u64* __restrict__ s, u32 limb0,
                                                    u32 log_n, int negate,
                                                    const ModParams* __restrict__ mods) {
  const u64 n = 1ull << log_n;
  const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 l = blockIdx.y;
  const u64 p = blockIdx.z;
  const ModParams m = mods[limb0 + l];
  const u64 off = (u64)l * n + c;
  u64 t = mulmod_barrett(y[p * py + off], s[off], m);
  if (negate) t = t ? m.q - t : 0;
  out[p * pout + off] = csub((x ? x[p * px + off] : 0) + t, m.q);
}

// row[c] = (row[c] + k y[c]) mod q for one limb; k a constant with its Shoup companion.
__global__ __launch_bounds__(kThreads) void k_axpy_const(u64* __restrict__ row,
                                                         const u64* __restrict__ y, u64 k, u64 ks,
                                                         u64 q) {
  const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  row[c] = csub(row[c] + csub(shoup_lazy(y[c], k, ks, q), q), q);
}

int sample(const fhe_ctx* c, u64* out, u64 pstride, u32 polys, u32 limb0, u32 nlimbs, int kind,
           u64 seed, u32 tag, hipStream_t s) {
  if ((u64)polys * nlimbs == 0) return kOk;
  if (int rc = check_grid(c->n / kThreads, kThreads, nlimbs, polys, "sample")) return rc;
  k_sample<<<dim3((u32)(c->n / kThreads), nlimbs, polys), kThreads, 0, s>>>(
      out, pstride, limb0, c->log_n, kind, (u32)seed, (u32)(seed >> 32), tag, c->d_mods);
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

int mac_s(const fhe_ctx* c, u64* out, u64 pout, const u64* x, u64 px, const u64* y, u64 py,
          const u64* sk, u32 polys, u32 limb0, u32 nlimbs, bool negate, hipStream_t s) {
  if ((u64)polys * nlimbs == 0) return kOk;
  if (int rc = check_grid(c->n / kThreads, kThreads, nlimbs, polys, "mac_s")) return rc;
  k_mac_s<<<dim3((u32)(c->n / kThreads), nlimbs, polys), kThreads, 0, s>>>(
      out, pout, x, px, y, py, sk, limb0, c->log_n, negate ? 1 : 0, c->d_mods);
  FHE_HIP_CHECK(hipGetLastError());
  return kOk;
}

// stream tags: which draw a sample belongs to (same seed, disjoint counters)
enum Tag : u32 { kTagSecret = 1, kTagPkA = 2, kTagPkE = 3, kTagKsA = 0x100, kTagKsE = 0x101,
                 kTagEncU = 32, kTagEncE0 = 33, kTagEncE1 = 34, kTagEncA = 35, kTagEncE = 36 };

}  // namespace
}  // namespace fhe

using namespace fhe;

extern "C" {

int fhe_sample(const fhe_ctx* c, uint64_t* out, uint32_t polys, uint32_t limb0, uint32_t nlimbs,
               int kind, uint64_t seed, uint32_t tag, fhe_stream_t s) {
  if (!c || (uint64_t)limb0 + nlimbs > c->moduli.size() || kind < 0 || kind > 2) {
    set_error("fhe_sample: null context, limb window out of range or unknown kind");
    return kInvalid;
  }
  return sample(c, out, (u64)nlimbs * c->n, polys, limb0, nlimbs, kind, seed, tag,
                static_cast<hipStream_t>(s));
}

int fhe_keygen_secret(const fhe_ctx* c, uint64_t* sk, uint64_t seed, fhe_stream_t st) {
  if (!c) return (set_error("fhe_keygen_secret: null context"), kInvalid);
  const hipStream_t s = static_cast<hipStream_t>(st);
  const u32 M = (u32)c->moduli.size();
  int rc;
  if ((rc = sample(c, sk, (u64)M * c->n, 1, 0, M, kTernary, seed, kTagSecret, s))) return rc;
  return launch_ntt(c, true, sk, sk, 1, (u64)M * c->n, 0, M, s);
}

int fhe_keygen_public(const fhe_ctx* c, uint64_t* pk, const uint64_t* sk, uint64_t seed,
                      fhe_stream_t st) {
  if (!c) return (set_error("fhe_keygen_public: null context"), kInvalid);
  const hipStream_t s = static_cast<hipStream_t>(st);
  const u32 L = c->L;
  const u64 ln = (u64)L * c->n;
  u64* b = pk;       // b = -a s + e
  u64* a = pk + ln;  // uniform, NTT form
  int rc;
  if ((rc = sample(c, a, ln, 1, 0, L, kUniform, seed, kTagPkA, s)) ||
      (rc = sample(c, b, ln, 1, 0, L, kError, seed, kTagPkE, s)) ||
      (rc = launch_ntt(c, true, b, b, 1, ln, 0, L, s)))
    return rc;
  return mac_s(c, b, ln, b, ln, a, ln, sk, 1, 0, L, true, s);
}

// evk_j = (-a_j s + e_j + P g_j s_from, a_j) over Q u P, NTT form; key [2][dnum][L + K][N]
// (b part then a part).  g_j = 1 mod the primes of digit j, 0 mod the other Q-primes; P g_j
// is 0 mod every P-prime, so the P rows carry only -a_j s + e_j.
int fhe_keygen_switch(const fhe_ctx* c, uint64_t* key, const uint64_t* sk, const uint64_t* s_from,
                      uint64_t seed, fhe_stream_t st) {
  if (!c || c->K == 0) return (set_error("fhe_keygen_switch: needs a context with K > 0"), kInvalid);
  const hipStream_t s = static_cast<hipStream_t>(st);
  const u32 L = c->L, M = L + c->K, dnum = c->dnum, alpha = c->alpha;
  const u64 mn = (u64)M * c->n;
  u64* kb = key;
  u64* ka = key + (u64)dnum * mn;
  int rc;
  for (u32 j = 0; j < dnum; ++j) {
    u64* b = kb + j * mn;
    u64* a = ka + j * mn;
    if ((rc = sample(c, a, mn, 1, 0, M, kUniform, seed, kTagKsA + 2 * j, s)) ||
        (rc = sample(c, b, mn, 1, 0, M, kError, seed, kTagKsE + 2 * j, s)) ||
        (rc = launch_ntt(c, true, b, b, 1, mn, 0, M, s)) ||
        (rc = mac_s(c, b, mn, b, mn, a, mn, sk, 1, 0, M, true, s)))
      return rc;
    // + P g_j s_from on the Q-limbs of digit j: P g_j = P mod q_i there, 0 on the other Q-limbs
    const u32 lo = j * alpha, hi = std::min(L, lo + alpha);
    for (u32 i = lo; i < hi; ++i) {
      const u64 q = c->moduli[i];
      u64 pm = 1;
      for (u32 k = 0; k < c->K; ++k) pm = mulmod_u64(pm, c->moduli[L + k] % q, q);
      k_axpy_const<<<(u32)(c->n / kThreads), kThreads, 0, s>>>(
          b + (u64)i * c->n, s_from + (u64)i * c->n, pm, (u64)(((u128)pm << 64) / q), q);
      FHE_HIP_CHECK(hipGetLastError());
    }
  }
  return kOk;
}

// Public-key encryption of an NTT-form plaintext pt [L][N]: c0 = b u + e0 + pt, c1 = a u + e1.
int fhe_encrypt(const fhe_ctx* c, uint64_t* ct, const uint64_t* pt, const uint64_t* pk,
                uint64_t seed, void* ws, fhe_stream_t st) {
  if (!c) return (set_error("fhe_encrypt: null context"), kInvalid);
  const hipStream_t s = static_cast<hipStream_t>(st);
  const u32 L = c->L;
  const u64 ln = (u64)L * c->n;
  int rc0 = ensure_ws(c, ln * sizeof(u64), &ws, s);
  if (rc0) return rc0;
  u64* u = static_cast<u64*>(ws);  // [L][N]
  u64* c0 = ct;
  u64* c1 = ct + ln;
  int rc;
  if ((rc = sample(c, u, ln, 1, 0, L, kTernary, seed, kTagEncU, s)) ||
      (rc = launch_ntt(c, true, u, u, 1, ln, 0, L, s)) ||
      (rc = sample(c, c0, ln, 1, 0, L, kError, seed, kTagEncE0, s)) ||
      (rc = sample(c, c1, ln, 1, 0, L, kError, seed, kTagEncE1, s)) ||
      (rc = launch_ntt(c, true, c0, c0, 2, ln, 0, L, s)) ||
      (rc = mac_s(c, c0, ln, c0, ln, pk, ln, u, 1, 0, L, false, s)) ||        // + b u
      (rc = mac_s(c, c1, ln, c1, ln, pk + ln, ln, u, 1, 0, L, false, s)) ||   // + a u
      (rc = launch_vec_ctx(c, kAdd, c0, c0, pt, 1, 0, L, s)))
    return rc;
  return kOk;
}

// Secret-key encryption: c1 = a (uniform), c0 = -a s + e + pt.
int fhe_encrypt_sk(const fhe_ctx* c, uint64_t* ct, const uint64_t* pt, const uint64_t* sk,
                   uint64_t seed, fhe_stream_t st) {
  if (!c) return (set_error("fhe_encrypt_sk: null context"), kInvalid);
  const hipStream_t s = static_cast<hipStream_t>(st);
  const u32 L = c->L;
  const u64 ln = (u64)L * c->n;
  int rc;
  if ((rc = sample(c, ct + ln, ln, 1, 0, L, kUniform, seed, kTagEncA, s)) ||
      (rc = sample(c, ct, ln, 1, 0, L, kError, seed, kTagEncE, s)) ||
      (rc = launch_ntt(c, true, ct, ct, 1, ln, 0, L, s)) ||
      (rc = mac_s(c, ct, ln, ct, ln, ct + ln, ln, sk, 1, 0, L, true, s)) ||
      (rc = launch_vec_ctx(c, kAdd, ct, ct, pt, 1, 0, L, s)))
    return rc;
  return kOk;
}

// pt = c0 + c1 s over the first nlimbs Q-limbs (a ciphertext at any level), NTT form; batch
// ciphertexts [batch][2][nlimbs][N] -> [batch][nlimbs][N].
int fhe_decrypt(const fhe_ctx* c, uint64_t* pt, const uint64_t* ct, const uint64_t* sk,
                uint32_t batch, uint32_t nlimbs, fhe_stream_t st) {
  if (!c || nlimbs == 0 || nlimbs > c->L)
    return (set_error("fhe_decrypt: null context or nlimbs outside [1, L]"), kInvalid);
  const u64 ln = (u64)nlimbs * c->n;
  return mac_s(c, pt, ln, ct, 2 * ln, ct + ln, 2 * ln, sk, batch, 0, nlimbs, false,
               static_cast<hipStream_t>(st));
}

}  // extern "C"
