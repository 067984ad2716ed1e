// fhecore.hpp -- header-only C++ Context / Ciphertext / Evaluator over the libfhecore C ABI.
//
// north_star asks for a C++ ciphertext/context/evaluator API in front of the NTT/modmul hot path.
// The reference has none (it is module-level Python, /root/reference/arithmetic.py:3-19), so this
// layer is build-defined: RAII ownership of the context and of device buffers, ciphertexts as
// [components][limbs][N] uint64 device arrays, and an Evaluator whose methods map 1:1 to the
// C entry points (include/fhecore.h).  Errors become fhe::Error exceptions carrying
// fhe_last_error().  Requires the HIP runtime (hipMalloc/hipMemcpy) and -lfhecore.
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "fhecore.h"

namespace fhe {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc, const char* what) {
  if (rc != FHE_OK) throw Error(rc, std::string(what) + ": " + fhe_last_error());
}

inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(FHE_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// Owning device array of uint64 words.
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t words) : n_(words) {
    if (n_) check_hip(hipMalloc(reinterpret_cast<void**>(&p_), n_ * 8), "hipMalloc");
  }
  ~DeviceBuffer() {
    if (p_) (void)hipFree(p_);
  }
  DeviceBuffer(DeviceBuffer&& o) noexcept : p_(std::exchange(o.p_, nullptr)), n_(std::exchange(o.n_, 0)) {}
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    std::swap(p_, o.p_);
    std::swap(n_, o.n_);
    return *this;
  }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;

  uint64_t* data() const { return p_; }
  size_t size() const { return n_; }
  void upload(const std::vector<uint64_t>& h) {
    if (h.size() != n_) throw Error(FHE_EINVAL, "upload: size mismatch");
    check_hip(hipMemcpy(p_, h.data(), n_ * 8, hipMemcpyHostToDevice), "hipMemcpy H2D");
  }
  std::vector<uint64_t> download() const {
    std::vector<uint64_t> h(n_);
    check_hip(hipMemcpy(h.data(), p_, n_ * 8, hipMemcpyDeviceToHost), "hipMemcpy D2H");
    return h;
  }

 private:
  uint64_t* p_ = nullptr;
  size_t n_ = 0;
};

// RNS parameters + device tables (fhe_ctx).  Immutable once built.
class Context {
 public:
  Context(uint32_t log_n, const std::vector<uint64_t>& q, const std::vector<uint64_t>& p = {},
          uint32_t dnum = 1, int device = 0)
      : log_n_(log_n), L_((uint32_t)q.size()), K_((uint32_t)p.size()), dnum_(p.empty() ? 0 : dnum) {
    check(fhe_ctx_create(&c_, log_n, q.data(), L_, p.empty() ? nullptr : p.data(), K_,
                         K_ ? dnum : 0, device),
          "fhe_ctx_create");
  }
  // The SURVEY.md §8a' chain: L + K largest 60-bit NTT primes for N = 2^log_n.
  static Context standard(uint32_t log_n, uint32_t L, uint32_t K = 0, uint32_t dnum = 1,
                          int device = 0) {
    std::vector<uint64_t> m(L + K);
    check(fhe_gen_moduli(log_n, L + K, 60, 0, m.data()), "fhe_gen_moduli");
    return Context(log_n, std::vector<uint64_t>(m.begin(), m.begin() + L),
                   std::vector<uint64_t>(m.begin() + L, m.end()), dnum, device);
  }
  ~Context() {
    if (c_) fhe_ctx_destroy(c_);
  }
  Context(Context&& o) noexcept
      : c_(std::exchange(o.c_, nullptr)), log_n_(o.log_n_), L_(o.L_), K_(o.K_), dnum_(o.dnum_) {}
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;

  const fhe_ctx* get() const { return c_; }
  uint32_t log_n() const { return log_n_; }
  uint64_t n() const { return 1ull << log_n_; }
  uint32_t L() const { return L_; }
  uint32_t K() const { return K_; }
  uint32_t dnum() const { return dnum_; }

 private:
  fhe_ctx* c_ = nullptr;
  uint32_t log_n_, L_, K_, dnum_;
};

// Keys, NTT form: secret [L+K][N], public [2][L][N], switch
// [2][dnum][L+K][N] = (b part, a part) -- the (evk_b, evk_a) of keyswitch / rotate / mul_relin.
struct SecretKey {
  DeviceBuffer s;
};
struct PublicKey {
  DeviceBuffer pk;
};
struct SwitchKey {
  DeviceBuffer key;
  size_t half = 0;  // words of the b part
  const uint64_t* b() const { return key.data(); }
  const uint64_t* a() const { return key.data() + half; }
};

// Counter-based (Philox4x32-10) key generation: every key is a function of (context, seeds).
// Each seed is a nonce: never reuse one per secret key (see the SECURITY note in fhecore.h).
class KeyGenerator {
 public:
  KeyGenerator(const Context& ctx, uint64_t seed, hipStream_t stream = nullptr)
      : ctx_(ctx), s_(stream) {
    sk_.s = DeviceBuffer((size_t)(ctx.L() + ctx.K()) * ctx.n());
    check(fhe_keygen_secret(ctx.get(), sk_.s.data(), seed, s_), "fhe_keygen_secret");
  }
  const SecretKey& secret() const { return sk_; }
  PublicKey public_key(uint64_t seed) const {
    PublicKey p{DeviceBuffer((size_t)2 * ctx_.L() * ctx_.n())};
    check(fhe_keygen_public(ctx_.get(), p.pk.data(), sk_.s.data(), seed, s_), "fhe_keygen_public");
    return p;
  }
  // switches s^2 to s
  SwitchKey relin_key(uint64_t seed) const {
    DeviceBuffer s2((size_t)(ctx_.L() + ctx_.K()) * ctx_.n());
    check(fhe_vec_mul(ctx_.get(), s2.data(), sk_.s.data(), sk_.s.data(), 1, 0, ctx_.L() + ctx_.K(), s_),
          "fhe_vec_mul");
    return switch_key(s2, seed);
  }
  // switches sigma_k(s) to s
  SwitchKey rotation_key(uint32_t galois_elt, uint64_t seed) const {
    DeviceBuffer sk((size_t)(ctx_.L() + ctx_.K()) * ctx_.n());
    check(fhe_automorphism(ctx_.get(), sk.data(), sk_.s.data(), 1, 0, ctx_.L() + ctx_.K(), galois_elt,
                           1, s_),
          "fhe_automorphism");
    return switch_key(sk, seed);
  }

 private:
  SwitchKey switch_key(const DeviceBuffer& s_from, uint64_t seed) const {
    SwitchKey k;
    k.half = (size_t)ctx_.dnum() * (ctx_.L() + ctx_.K()) * ctx_.n();
    k.key = DeviceBuffer(2 * k.half);
    check(fhe_keygen_switch(ctx_.get(), k.key.data(), sk_.s.data(), s_from.data(), seed, s_),
          "fhe_keygen_switch");
    return k;
  }
  const Context& ctx_;
  hipStream_t s_;
  SecretKey sk_;
};

// A ciphertext (or plain polynomial when components == 1): [components][limbs][N] residues.
struct Ciphertext {
  uint32_t components = 0, limbs = 0;
  uint64_t n = 0;
  bool ntt_form = false;
  DeviceBuffer buf;
  Ciphertext() = default;
  Ciphertext(const Context& ctx, uint32_t comps, uint32_t nlimbs, bool ntt = false)
      : components(comps), limbs(nlimbs), n(ctx.n()), ntt_form(ntt), buf((size_t)comps * nlimbs * ctx.n()) {}
  uint64_t* data() const { return buf.data(); }
};

// One rank of a limb-sharded job: libfhecore's RCCL communicator.  Rank 0 calls
// Comm::unique_id() and sends the bytes to the other ranks (MPI, sockets, torch.distributed...);
// every rank then constructs its Comm on its own GPU.  shard(ctx) = the Q-limbs this rank owns.
class Comm {
 public:
  using Id = std::array<uint8_t, FHE_COMM_ID_BYTES>;
  static Id unique_id() {
    Id id{};
    check(fhe_comm_get_unique_id(id.data()), "fhe_comm_get_unique_id");
    return id;
  }
  Comm(const Id& id, int nranks, int rank, int device = 0) {
    check(fhe_comm_create(&c_, id.data(), nranks, rank, device), "fhe_comm_create");
  }
  ~Comm() {
    if (c_) fhe_comm_destroy(c_);
  }
  Comm(Comm&& o) noexcept : c_(std::exchange(o.c_, nullptr)) {}
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;
  fhe_comm_t get() const { return c_; }
  std::pair<uint32_t, uint32_t> shard(const Context& ctx) const {  // (limb0, nlimbs)
    uint32_t lo = 0, nl = 0;
    check(fhe_comm_shard(ctx.get(), c_, &lo, &nl), "fhe_comm_shard");
    return {lo, nl};
  }

 private:
  fhe_comm_t c_ = nullptr;
};

// The hybrid partition of a key-switch batch (fhe_dist_hybrid_make): `groups` ciphertext groups of
// ranks / groups limb shards.  Rank `rank` builds its group's Comm with
// Comm(group_id, plan.g, plan.shard, device) and key-switches plan.batch ciphertexts from plan.batch0.
inline fhe_dist_hybrid hybrid_plan(uint32_t L, uint32_t log_n, uint32_t ranks, uint32_t groups,
                                   uint32_t rank, uint32_t batch, uint32_t chunks = 0) {
  fhe_dist_hybrid h{};
  check(fhe_dist_hybrid_make(&h, L, log_n, ranks, groups, rank, batch, chunks),
        "fhe_dist_hybrid_make");
  return h;
}

// Homomorphic operations on one stream.
class Evaluator {
 public:
  explicit Evaluator(const Context& ctx, hipStream_t stream = nullptr) : ctx_(ctx), s_(stream) {}

  void ntt(Ciphertext& x) const {
    check(fhe_ntt_fwd(ctx_.get(), x.data(), x.components, 0, x.limbs, s_), "fhe_ntt_fwd");
    x.ntt_form = true;
  }
  void intt(Ciphertext& x) const {
    check(fhe_ntt_inv(ctx_.get(), x.data(), x.components, 0, x.limbs, s_), "fhe_ntt_inv");
    x.ntt_form = false;
  }
  void add(Ciphertext& out, const Ciphertext& a, const Ciphertext& b) const {
    same(a, b, "add");
    check(fhe_vec_add(ctx_.get(), out.data(), a.data(), b.data(), a.components, 0, a.limbs, s_),
          "fhe_vec_add");
  }
  void sub(Ciphertext& out, const Ciphertext& a, const Ciphertext& b) const {
    same(a, b, "sub");
    check(fhe_vec_sub(ctx_.get(), out.data(), a.data(), b.data(), a.components, 0, a.limbs, s_),
          "fhe_vec_sub");
  }
  // coefficient-wise product (= polynomial product when both are in NTT form)
  void mul_pointwise(Ciphertext& out, const Ciphertext& a, const Ciphertext& b) const {
    same(a, b, "mul_pointwise");
    check(fhe_vec_mul(ctx_.get(), out.data(), a.data(), b.data(), a.components, 0, a.limbs, s_),
          "fhe_vec_mul");
  }
  // ct x ct tensor: (a0, a1) x (b0, b1) -> (d0, d1, d2), coefficient form in and out.
  Ciphertext multiply(const Ciphertext& a, const Ciphertext& b) const {
    same(a, b, "multiply");
    if (a.components != 2 || a.ntt_form) throw Error(FHE_EINVAL, "multiply: need 2-component, coefficient form");
    Ciphertext d(ctx_, 3, a.limbs);
    if (ws_.size() * 8 < fhe_hommult_workspace(ctx_.get(), 1, a.limbs))
      ws_ = DeviceBuffer((fhe_hommult_workspace(ctx_.get(), 1, a.limbs) + 7) / 8);
    check(fhe_hommult(ctx_.get(), d.data(), a.data(), b.data(), 1, 0, a.limbs, ws_.data(), s_),
          "fhe_hommult");
    return d;
  }
  // Hybrid key-switch of d2 (NTT form, L limbs) with the key (evk_b, evk_a), NTT form [dnum][L+K][N].
  std::pair<Ciphertext, Ciphertext> keyswitch(const Ciphertext& d2, const DeviceBuffer& evk_b,
                                              const DeviceBuffer& evk_a) const {
    Ciphertext k0(ctx_, 1, d2.limbs, true), k1(ctx_, 1, d2.limbs, true);
    const size_t need = fhe_keyswitch_workspace(ctx_.get(), ctx_.L(), 1);
    if (ws_.size() * 8 < need) ws_ = DeviceBuffer((need + 7) / 8);
    check(fhe_keyswitch(ctx_.get(), k0.data(), k1.data(), d2.data(), evk_b.data(), evk_a.data(), 1,
                        ws_.data(), s_),
          "fhe_keyswitch");
    return {std::move(k0), std::move(k1)};
  }
  // The limb-sharded key-switch (fhe_keyswitch_dist): d2_own = this rank's limbs of d2 (NTT
  // form, comm.shard(ctx) limbs), evk_*_own [dnum][nlimbs + K][N] (own Q-limbs then all P-limbs).
  // Every rank calls it together; the ranks' outputs concatenate to keyswitch()'s.
  std::pair<Ciphertext, Ciphertext> keyswitch_dist(const Comm& comm, const Ciphertext& d2_own,
                                                   const DeviceBuffer& evk_b_own,
                                                   const DeviceBuffer& evk_a_own,
                                                   uint32_t chunks = 0) const {
    if (d2_own.limbs != comm.shard(ctx_).second)
      throw Error(FHE_EINVAL, "keyswitch_dist: d2_own must hold this rank's limbs");
    Ciphertext k0(ctx_, d2_own.components, d2_own.limbs, true);
    Ciphertext k1(ctx_, d2_own.components, d2_own.limbs, true);
    const size_t need = fhe_keyswitch_dist_workspace(ctx_.get(), comm.get(), d2_own.components, chunks);
    if (ws_.size() * 8 < need) ws_ = DeviceBuffer((need + 7) / 8);
    check(fhe_keyswitch_dist(ctx_.get(), comm.get(), k0.data(), k1.data(), d2_own.data(),
                             evk_b_own.data(), evk_a_own.data(), d2_own.components, chunks,
                             ws_.data(), s_),
          "fhe_keyswitch_dist");
    return {std::move(k0), std::move(k1)};
  }
  // Public-key encryption of an NTT-form plaintext (1 component, L limbs) -> [2][L][N] NTT form.
  Ciphertext encrypt(const Ciphertext& pt, const PublicKey& pk, uint64_t seed) const {
    if (pt.components != 1 || pt.limbs != ctx_.L() || !pt.ntt_form)
      throw Error(FHE_EINVAL, "encrypt: need a 1-component NTT-form plaintext over L limbs");
    Ciphertext ct(ctx_, 2, ctx_.L(), true);
    check(fhe_encrypt(ctx_.get(), ct.data(), pt.data(), pk.pk.data(), seed, nullptr, s_), "fhe_encrypt");
    return ct;
  }
  // c0 + c1 s over the ciphertext's limbs -> 1-component NTT-form plaintext.
  Ciphertext decrypt(const Ciphertext& ct, const SecretKey& sk) const {
    if (ct.components != 2 || !ct.ntt_form) throw Error(FHE_EINVAL, "decrypt: need an NTT-form ciphertext");
    Ciphertext pt(ctx_, 1, ct.limbs, true);
    check(fhe_decrypt(ctx_.get(), pt.data(), ct.data(), sk.s.data(), 1, ct.limbs, s_), "fhe_decrypt");
    return pt;
  }
  // Relin(a x b), optionally rescaled; NTT form over L limbs in.
  Ciphertext mul_relin(const Ciphertext& a, const Ciphertext& b, const SwitchKey& rk, bool rescale) const {
    same(a, b, "mul_relin");
    if (a.components != 2 || !a.ntt_form || a.limbs != ctx_.L())
      throw Error(FHE_EINVAL, "mul_relin: need 2-component NTT-form ciphertexts over L limbs");
    Ciphertext out(ctx_, 2, ctx_.L() - (rescale ? 1 : 0), true);
    const size_t need = fhe_mul_relin_workspace(ctx_.get(), 1);
    if (ws_.size() * 8 < need) ws_ = DeviceBuffer((need + 7) / 8);
    check(fhe_mul_relin(ctx_.get(), out.data(), a.data(), b.data(), rk.b(), rk.a(), 1, rescale ? 1 : 0,
                        ws_.data(), s_),
          "fhe_mul_relin");
    return out;
  }
  // Divide-and-round by the last modulus: drops one limb, keeps the form.
  Ciphertext rescale(const Ciphertext& x) const {
    if (x.limbs < 2) throw Error(FHE_EINVAL, "rescale: need at least 2 limbs");
    Ciphertext out(ctx_, x.components, x.limbs - 1, x.ntt_form);
    const size_t need = fhe_rescale_workspace(ctx_.get(), x.components, x.limbs);
    if (x.ntt_form && ws_.size() * 8 < need) ws_ = DeviceBuffer((need + 7) / 8);
    check(fhe_rescale(ctx_.get(), out.data(), x.data(), x.components, x.limbs, x.ntt_form ? 1 : 0,
                      x.ntt_form ? ws_.data() : nullptr, s_),
          "fhe_rescale");
    return out;
  }
  // Galois element of a slot rotation by `step` (5^step mod 2N).
  uint32_t galois_elt(int step) const {
    const uint64_t two_n = 2 * ctx_.n();
    uint64_t g = 1, b = 5;
    uint64_t e = step >= 0 ? (uint64_t)step : (uint64_t)(-(int64_t)step) * (two_n / 2 - 1);
    for (; e; e >>= 1, b = b * b % two_n)
      if (e & 1) g = g * b % two_n;
    return (uint32_t)g;
  }
  // Rotation of a 2-component NTT-form ciphertext over all L limbs by Galois element k, with the
  // key-switch key from sigma_k(s) to s (NTT form [dnum][L+K][N]).
  Ciphertext rotate(const Ciphertext& ct, uint32_t galois_elt, const DeviceBuffer& rot_b,
                    const DeviceBuffer& rot_a) const {
    if (ct.components != 2 || !ct.ntt_form || ct.limbs != ctx_.L())
      throw Error(FHE_EINVAL, "rotate: need a 2-component NTT-form ciphertext over L limbs");
    Ciphertext out(ctx_, 2, ct.limbs, true);
    const size_t need = fhe_rotate_workspace(ctx_.get(), 1);
    if (ws_.size() * 8 < need) ws_ = DeviceBuffer((need + 7) / 8);
    check(fhe_rotate(ctx_.get(), out.data(), ct.data(), galois_elt, rot_b.data(), rot_a.data(), 1,
                     ws_.data(), s_),
          "fhe_rotate");
    return out;
  }
  Ciphertext rotate(const Ciphertext& ct, uint32_t galois_elt, const SwitchKey& key) const {
    if (ct.components != 2 || !ct.ntt_form || ct.limbs != ctx_.L())
      throw Error(FHE_EINVAL, "rotate: need a 2-component NTT-form ciphertext over L limbs");
    Ciphertext out(ctx_, 2, ct.limbs, true);
    const size_t need = fhe_rotate_workspace(ctx_.get(), 1);
    if (ws_.size() * 8 < need) ws_ = DeviceBuffer((need + 7) / 8);
    check(fhe_rotate(ctx_.get(), out.data(), ct.data(), galois_elt, key.b(), key.a(), 1, ws_.data(), s_),
          "fhe_rotate");
    return out;
  }
  // Several rotations of one ciphertext sharing a single ModUp (fhe_rotate_hoisted); output r
  // decrypts to sigma_{galois_elts[r]}(m).
  std::vector<Ciphertext> rotate_hoisted(const Ciphertext& ct, const std::vector<uint32_t>& galois_elts,
                                         const std::vector<const SwitchKey*>& keys) const {
    if (ct.components != 2 || !ct.ntt_form || ct.limbs != ctx_.L())
      throw Error(FHE_EINVAL, "rotate_hoisted: need a 2-component NTT-form ciphertext over L limbs");
    if (keys.size() != galois_elts.size())
      throw Error(FHE_EINVAL, "rotate_hoisted: one key per Galois element");
    const size_t words = (size_t)2 * ct.limbs * ctx_.n(), count = galois_elts.size();
    DeviceBuffer all(words * (count ? count : 1));
    std::vector<const uint64_t*> kb(count), ka(count);
    for (size_t r = 0; r < count; ++r) {
      kb[r] = keys[r]->b();
      ka[r] = keys[r]->a();
    }
    const size_t need = fhe_rotate_hoisted_workspace(ctx_.get(), 1);
    if (ws_.size() * 8 < need) ws_ = DeviceBuffer((need + 7) / 8);
    check(fhe_rotate_hoisted(ctx_.get(), all.data(), ct.data(), galois_elts.data(), kb.data(),
                             ka.data(), (uint32_t)count, 1, ws_.data(), s_),
          "fhe_rotate_hoisted");
    std::vector<Ciphertext> out;
    for (size_t r = 0; r < count; ++r) {
      out.emplace_back(ctx_, 2, ct.limbs, true);
      if (hipMemcpyAsync(out.back().data(), all.data() + r * words, words * 8,
                         hipMemcpyDeviceToDevice, s_) != hipSuccess)
        throw Error(FHE_EDEVICE, "rotate_hoisted: copy");
    }
    if (hipStreamSynchronize(s_) != hipSuccess) throw Error(FHE_EDEVICE, "rotate_hoisted: sync");
    return out;
  }
  // sum_r pts[r] * rot_{galois_elts[r]}(ct) with one ModUp and one ModDown (fhe_rotate_sum_hoisted,
  // double hoisting: the inner loop of a baby-step / giant-step linear transform).  keys[r] may be
  // null for galois_elts[r] == 1 (the unrotated term); pts[r] [L + K][N] NTT form over Q u P.
  Ciphertext rotate_sum(const Ciphertext& ct, const std::vector<uint32_t>& galois_elts,
                        const std::vector<const SwitchKey*>& keys,
                        const std::vector<const DeviceBuffer*>& pts) const {
    if (ct.components != 2 || !ct.ntt_form || ct.limbs != ctx_.L())
      throw Error(FHE_EINVAL, "rotate_sum: need a 2-component NTT-form ciphertext over L limbs");
    const size_t count = galois_elts.size();
    if (keys.size() != count || pts.size() != count)
      throw Error(FHE_EINVAL, "rotate_sum: one key (or null) and one plaintext per term");
    std::vector<const uint64_t*> kb(count ? count : 1), ka(count ? count : 1),
        pp(count ? count : 1);
    for (size_t r = 0; r < count; ++r) {
      kb[r] = keys[r] ? keys[r]->b() : nullptr;
      ka[r] = keys[r] ? keys[r]->a() : nullptr;
      if (!pts[r] || pts[r]->size() != (size_t)(ctx_.L() + ctx_.K()) * ctx_.n())
        throw Error(FHE_EINVAL, "rotate_sum: plaintexts are [L + K][N]");
      pp[r] = pts[r]->data();
    }
    Ciphertext out(ctx_, 2, ct.limbs, true);
    const size_t need = fhe_rotate_sum_hoisted_workspace(ctx_.get(), 1);
    if (ws_.size() * 8 < need) ws_ = DeviceBuffer((need + 7) / 8);
    check(fhe_rotate_sum_hoisted(ctx_.get(), out.data(), ct.data(), galois_elts.data(), kb.data(),
                                 ka.data(), pp.data(), (uint32_t)count, 1, ws_.data(), s_),
          "fhe_rotate_sum_hoisted");
    return out;
  }

 private:
  static void same(const Ciphertext& a, const Ciphertext& b, const char* who) {
    if (a.components != b.components || a.limbs != b.limbs || a.n != b.n)
      throw Error(FHE_EINVAL, std::string(who) + ": shape mismatch");
  }
  const Context& ctx_;
  hipStream_t s_;
  mutable DeviceBuffer ws_;
};

}  // namespace fhe
