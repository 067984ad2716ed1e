// Host side of fhe_ctx: parameter validation and the device-resident tables (twiddles with Shoup
// companions, Barrett constants, base-conversion constants), built by host_tables.cpp.
//
// The reference has no context -- MOD is passed on every call (/root/reference/arithmetic.py:3,7,11)
// and NTT takes no parameters at all (arithmetic.py:15).  The context here owns everything the
// kernels need per modulus so that the hot calls take only device pointers and sizes.
// Conventions follow SURVEY.md §8a' (psi = g^((q-1)/2N), g the smallest primitive root).
#include <string>

#include "internal.hpp"

namespace fhe {
namespace {

template <class T>
int upload(T** dptr, const T* src, size_t count) {
  FHE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(dptr), count * sizeof(T)));
  FHE_HIP_CHECK(hipMemcpy(*dptr, src, count * sizeof(T), hipMemcpyHostToDevice));
  return kOk;
}

}  // namespace

int gen_moduli(u32 log_n, u32 count, u32 bits, u32 skip, u64* out) {
  std::string err;
  if (!gen_moduli_host(log_n, count, bits, skip, out, err)) {
    set_error(err);
    return kInvalid;
  }
  return kOk;
}

int ctx_create(fhe_ctx** out, u32 log_n, const u64* q, u32 L, const u64* p, u32 K, u32 dnum,
               int device) {
  if (!out) {
    set_error("ctx_create: null out pointer");
    return kInvalid;
  }
  *out = nullptr;
  if (log_n < 10 || log_n > 17) {
    set_error("ctx_create: log_n must be in [10, 17]");
    return kUnsupported;
  }
  if (L == 0 || L > 64 || K > 16 || (K > 0 && (dnum == 0 || dnum > L))) {
    set_error("ctx_create: need 1 <= L <= 64, K <= 16, 1 <= dnum <= L when K > 0");
    return kInvalid;
  }
  const u64 n = 1ull << log_n;
  std::vector<u64> mods(q, q + L);
  if (K) mods.insert(mods.end(), p, p + K);
  for (size_t i = 0; i < mods.size(); ++i) {
    const u64 m = mods[i];
    if (m >= (1ull << 63) || m % (2 * n) != 1 || !is_prime_u64(m)) {
      set_error("ctx_create: modulus #" + std::to_string(i) + " = " + std::to_string(m) +
                " is not a prime < 2^63 with q = 1 mod 2N");
      return kInvalid;
    }
    for (size_t j = 0; j < i; ++j)
      if (mods[j] == m) {
        set_error("ctx_create: duplicate modulus " + std::to_string(m));
        return kInvalid;
      }
  }
  int ndev = 0;
  FHE_HIP_CHECK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_error("ctx_create: device index out of range");
    return kInvalid;
  }
  FHE_HIP_CHECK(hipSetDevice(device));

  int cus = 0;
  FHE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  auto* c = new fhe_ctx();
  c->device = device;
  c->num_cus = cus;
  c->lz16 = true;
  c->wide = false;
  for (u64 m : mods) {
    // lz16: 2^32 < m < 2^60 and m >= 2^s - 2^(s-4), s = bitlength(m) (the top-bits reductions,
    // ntt.hip top_bits, work on the 32-bit halves); the largest primes below a power of two all
    // qualify
    const u64 pw = 1ull << (63 - __builtin_clzll(m));  // 2^(s-1)
    c->lz16 = c->lz16 && m < (1ull << 60) && m > (1ull << 32) && m >= 2 * pw - pw / 8;
    c->wide = c->wide || m >= (1ull << 61);
  }
  c->log_n = log_n;
  c->n = n;
  c->L = L;
  c->K = K;
  c->dnum = K ? dnum : 0;
  c->alpha = K ? (L + dnum - 1) / dnum : 0;
  c->moduli = mods;
  const size_t M = mods.size();
  std::vector<Pair64> twf(M * n), twi(M * n), nfold(4 * M);
  // the HomMult's 9 + 7-stage forward (ntt.hip k_hm_col9) needs its own row layout of the forward
  // table: narrow contexts at N = 2^16 (Q limbs only: HomMult never runs on P limbs)
  const bool split9 = log_n == 16 && !c->wide;
  std::vector<Pair64> twf9(split9 ? L * n : 0);
  c->psi.resize(M);
  c->mods_host.resize(M);
  for (size_t i = 0; i < M; ++i) {
    c->mods_host[i] = make_mod_params(mods[i]);
    c->psi[i] = ntt_tables(mods[i], log_n, &twf[i * n], &twi[i * n], &nfold[4 * i],
                           split9 && i < L ? &twf9[i * n] : nullptr);
  }
  int rc = kOk;
  if ((rc = upload(&c->d_mods, c->mods_host.data(), M)) ||
      (rc = upload(&c->d_tw_fwd, reinterpret_cast<const ulonglong2*>(twf.data()), M * n)) ||
      (rc = upload(&c->d_tw_inv, reinterpret_cast<const ulonglong2*>(twi.data()), M * n)) ||
      (rc = upload(&c->d_nfold, reinterpret_cast<const ulonglong2*>(nfold.data()), 4 * M)) ||
      (split9 && (rc = upload(&c->d_tw_fwd9, reinterpret_cast<const ulonglong2*>(twf9.data()),
                              (size_t)L * n))) ||
      (rc = build_rns_tables(c)) ||
      (rc = build_galois_tables(c))) {
    ctx_destroy(c);
    return rc;
  }
  *out = c;
  return kOk;
}

int ctx_destroy(fhe_ctx* c) {
  if (!c) return kOk;
  (void)hipSetDevice(c->device);
  for (auto& t : c->bc_tables) (void)hipFree(t.second);
  for (void* ptr : {(void*)c->d_mods, (void*)c->d_tw_fwd, (void*)c->d_tw_fwd9, (void*)c->d_tw_inv, (void*)c->d_nfold, (void*)c->d_nfold_down, (void*)c->d_nfold_up,
                    (void*)c->d_modup_inv, (void*)c->d_modup_hat, (void*)c->d_moddown_inv,
                    (void*)c->d_moddown_hat, (void*)c->d_modup_hat_w, (void*)c->d_modup_hat_rw,
                    (void*)c->d_moddown_hat_w, (void*)c->d_modup_hat_rwp,
                    (void*)c->d_moddown_hat_wp, (void*)c->d_rpinv, (void*)c->d_pinv, (void*)c->d_rs_tab,
                    (void*)c->d_rs_half, c->workspace})
    if (ptr) (void)hipFree(ptr);
  delete c;
  return kOk;
}

}  // namespace fhe
