// C++ API smoke/parity test (run by tests/test_cpp_api.py on a GPU box): Context / Evaluator from
// include/fhecore.hpp against a schoolbook negacyclic product computed here with __int128.
#include <cstdio>
#include <random>

#include "fhecore.hpp"

using u64 = uint64_t;
using u128 = unsigned __int128;

static std::vector<u64> negacyclic(const std::vector<u64>& a, const std::vector<u64>& b, u64 q) {
  const size_t n = a.size();
  std::vector<u128> acc(n, 0);
  std::vector<u64> out(n);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) {
      const u64 p = (u64)((u128)a[i] * b[j] % q);
      const size_t k = i + j;
      if (k < n) acc[k] = (acc[k] + p) % q;
      else acc[k - n] = (acc[k - n] + q - p) % q;
    }
  for (size_t i = 0; i < n; ++i) out[i] = (u64)acc[i];
  return out;
}

int main() {
  try {
    const uint32_t log_n = 10, L = 2;
    const u64 n = 1ull << log_n;
    fhe::Context ctx = fhe::Context::standard(log_n, L);
    std::vector<u64> q(L);
    fhe::check(fhe_ctx_moduli(ctx.get(), q.data(), nullptr), "moduli");
    std::mt19937_64 rng(7);
    std::vector<u64> ha(2 * L * n), hb(2 * L * n);
    for (uint32_t c = 0; c < 2; ++c)
      for (uint32_t l = 0; l < L; ++l)
        for (u64 i = 0; i < n; ++i) {
          ha[(c * L + l) * n + i] = rng() % q[l];
          hb[(c * L + l) * n + i] = rng() % q[l];
        }
    fhe::Ciphertext a(ctx, 2, L), b(ctx, 2, L);
    a.buf.upload(ha);
    b.buf.upload(hb);
    fhe::Evaluator ev(ctx);
    fhe::Ciphertext d = ev.multiply(a, b);
    const std::vector<u64> hd = d.buf.download();
    for (uint32_t l = 0; l < L; ++l) {
      auto sl = [&](const std::vector<u64>& v, uint32_t c) {
        return std::vector<u64>(v.begin() + (c * L + l) * n, v.begin() + (c * L + l + 1) * n);
      };
      const auto d0 = negacyclic(sl(ha, 0), sl(hb, 0), q[l]);
      const auto d2 = negacyclic(sl(ha, 1), sl(hb, 1), q[l]);
      for (u64 i = 0; i < n; ++i) {
        if (hd[(0 * L + l) * n + i] != d0[i] || hd[(2 * L + l) * n + i] != d2[i]) {
          std::printf("FAIL limb %u coeff %llu\n", l, (unsigned long long)i);
          return 1;
        }
      }
    }
    // NTT round trip through the Evaluator
    ev.ntt(a);
    ev.intt(a);
    if (a.buf.download() != ha) {
      std::printf("FAIL ntt round trip\n");
      return 1;
    }
    // rescale (coefficient form) of d = (d0, d1, d2) over 2 limbs: X = CRT(x0, x1) < q0 q1 < 2^122,
    // out = floor((X + q1 / 2) / q1) mod q0
    {
      fhe::Ciphertext dc = ev.rescale(d);
      if (dc.limbs != 1) {
        std::printf("FAIL rescale shape\n");
        return 1;
      }
      const std::vector<u64> hr = dc.buf.download();
      const u64 q0 = q[0], q1 = q[1];
      const u64 q0inv_mod_q1 = [&] {  // q0^-1 mod q1 by Fermat
        u128 r = 1, b = q0 % q1;
        for (u64 e = q1 - 2; e; e >>= 1, b = b * b % q1)
          if (e & 1) r = r * b % q1;
        return (u64)r;
      }();
      for (uint32_t c = 0; c < 3; ++c)
        for (u64 i = 0; i < n; ++i) {
          const u64 x0 = hd[(c * L + 0) * n + i], x1 = hd[(c * L + 1) * n + i];
          // X = x0 + q0 * ((x1 - x0) q0^-1 mod q1)
          const u64 t = (u64)((u128)((x1 + q1 - x0 % q1) % q1) * q0inv_mod_q1 % q1);
          const u128 X = (u128)x0 + (u128)q0 * t;
          const u64 want = (u64)(((X + q1 / 2) / q1) % q0);
          if (hr[c * n + i] != want) {
            std::printf("FAIL rescale comp %u coeff %llu\n", c, (unsigned long long)i);
            return 1;
          }
        }
    }
    // keys, encryption, rotation and mult+relin+rescale through the C++ layer (§8f): an integer
    // plaintext m (small coefficients) must decrypt back to m + small noise, and a rotation by
    // Galois element k to sigma_k(m)
    {
      fhe::Context kc = fhe::Context::standard(10, 3, 2, 3);
      fhe::KeyGenerator kg(kc, 42);
      const fhe::PublicKey pk = kg.public_key(43);
      fhe::Evaluator kev(kc);
      const u64 kn = kc.n();
      std::vector<u64> kq(5);
      fhe::check(fhe_ctx_moduli(kc.get(), kq.data(), nullptr), "moduli");
      std::vector<int64_t> m(kn);
      for (u64 i = 0; i < kn; ++i) m[i] = (int64_t)(rng() % 2001) - 1000;
      std::vector<u64> hp(3 * kn);
      for (uint32_t l = 0; l < 3; ++l)
        for (u64 i = 0; i < kn; ++i) hp[l * kn + i] = m[i] >= 0 ? (u64)m[i] : kq[l] - (u64)(-m[i]);
      fhe::Ciphertext pt(kc, 1, 3, false);
      pt.buf.upload(hp);
      kev.ntt(pt);
      const fhe::Ciphertext ct = kev.encrypt(pt, pk, 44);
      auto decrypt_limb0 = [&](const fhe::Ciphertext& c) {
        fhe::Ciphertext d = kev.decrypt(c, kg.secret());
        kev.intt(d);
        const std::vector<u64> hd = d.buf.download();
        std::vector<int64_t> r(kn);
        for (u64 i = 0; i < kn; ++i) {
          const u64 v = hd[i];  // limb 0
          r[i] = v > kq[0] / 2 ? -(int64_t)(kq[0] - v) : (int64_t)v;
        }
        return r;
      };
      const std::vector<int64_t> back = decrypt_limb0(ct);
      for (u64 i = 0; i < kn; ++i)
        if (std::llabs(back[i] - m[i]) > 1000) {
          std::printf("FAIL encrypt/decrypt coeff %llu\n", (unsigned long long)i);
          return 1;
        }
      const uint32_t k = kev.galois_elt(1);
      const fhe::SwitchKey rk = kg.rotation_key(k, 45);
      const std::vector<int64_t> r2 = decrypt_limb0(kev.rotate(ct, k, rk));
      for (u64 i = 0; i < kn; ++i) {
        const u64 t = i * k % (2 * kn);  // sigma_k moves coefficient i to i k mod 2N (negated past N)
        const int64_t want = t < kn ? m[i] : -m[i];
        if (std::llabs(r2[t % kn] - want) > 1000) {
          std::printf("FAIL rotation coeff %llu\n", (unsigned long long)i);
          return 1;
        }
      }
      // hoisted: the same rotation and the conjugation from one ModUp
      const uint32_t kconj = 2 * (uint32_t)kn - 1;
      const fhe::SwitchKey ck = kg.rotation_key(kconj, 47);
      const std::vector<fhe::Ciphertext> hs = kev.rotate_hoisted(ct, {k, kconj}, {&rk, &ck});
      for (int h = 0; h < 2; ++h) {
        const uint32_t g = h ? kconj : k;
        const std::vector<int64_t> rh = decrypt_limb0(hs[h]);
        for (u64 i = 0; i < kn; ++i) {
          const u64 t = i * g % (2 * kn);
          const int64_t want = t < kn ? m[i] : -m[i];
          if (std::llabs(rh[t % kn] - want) > 1000) {
            std::printf("FAIL hoisted rotation %d coeff %llu\n", h, (unsigned long long)i);
            return 1;
          }
        }
      }
      // double-hoisted rotation sum with all-ones plaintexts (NTT of the constant 1): decrypts to
      // sigma_k(m) + sigma_conj(m)
      {
        fhe::DeviceBuffer ones((size_t)(kc.L() + kc.K()) * kn);
        ones.upload(std::vector<u64>((size_t)(kc.L() + kc.K()) * kn, 1));
        const std::vector<int64_t> rs = decrypt_limb0(kev.rotate_sum(ct, {k, kconj}, {&rk, &ck},
                                                                     {&ones, &ones}));
        std::vector<int64_t> want(kn, 0);
        for (uint32_t g : {k, kconj})
          for (u64 i = 0; i < kn; ++i) {
            const u64 t = i * g % (2 * kn);
            want[t % kn] += t < kn ? m[i] : -m[i];
          }
        for (u64 i = 0; i < kn; ++i)
          if (std::llabs(rs[i] - want[i]) > 2000) {
            std::printf("FAIL rotation sum coeff %llu\n", (unsigned long long)i);
            return 1;
          }
      }
      const fhe::SwitchKey rl = kg.relin_key(46);
      const fhe::Ciphertext sq = kev.mul_relin(ct, ct, rl, false);
      if (sq.limbs != 3) {
        std::printf("FAIL mul_relin shape\n");
        return 1;
      }
    }
    {  // the limb-sharded key-switch over a one-rank RCCL communicator == fhe_keyswitch
      fhe::Context kc = fhe::Context::standard(log_n, 4, 2, 2);
      const fhe::Comm comm(fhe::Comm::unique_id(), 1, 0, 0);
      const auto sh = comm.shard(kc);
      std::vector<u64> mq(6);
      fhe::check(fhe_ctx_moduli(kc.get(), mq.data(), nullptr), "moduli");
      const uint32_t B = 3;
      fhe::Ciphertext d2(kc, B, 4, true);
      std::vector<u64> hd2((size_t)B * 4 * n);
      for (size_t i = 0; i < hd2.size(); ++i) hd2[i] = rng() % mq[(i / n) % 4];
      d2.buf.upload(hd2);
      fhe::DeviceBuffer eb((size_t)2 * 6 * n), ea((size_t)2 * 6 * n);
      std::vector<u64> he(2 * 6 * n), ha2(2 * 6 * n);
      for (size_t i = 0; i < he.size(); ++i) {
        he[i] = rng() % mq[(i / n) % 6];
        ha2[i] = rng() % mq[(i / n) % 6];
      }
      eb.upload(he);
      ea.upload(ha2);
      fhe::Evaluator kev(kc);
      const auto dist = kev.keyswitch_dist(comm, d2, eb, ea, 2);
      const auto r0 = dist.first.buf.download(), r1 = dist.second.buf.download();
      for (uint32_t b = 0; b < B; ++b) {
        fhe::Ciphertext one(kc, 1, 4, true);
        one.buf.upload(std::vector<u64>(hd2.begin() + (size_t)b * 4 * n, hd2.begin() + (size_t)(b + 1) * 4 * n));
        const auto ref = kev.keyswitch(one, eb, ea);
        const auto f0 = ref.first.buf.download(), f1 = ref.second.buf.download();
        for (u64 i = 0; i < 4 * n; ++i)
          if (r0[b * 4 * n + i] != f0[i] || r1[b * 4 * n + i] != f1[i]) {
            std::printf("FAIL keyswitch_dist ct %u word %llu\n", b, (unsigned long long)i);
            return 1;
          }
      }
      if (sh.first != 0 || sh.second != 4) {
        std::printf("FAIL comm shard\n");
        return 1;
      }
      // hybrid partition helper: 8 ranks as 4 ciphertext groups x 2 limb shards of 33 ciphertexts
      const fhe_dist_hybrid h = fhe::hybrid_plan(4, 12, 8, 4, 5, 33);
      if (h.g != 2 || h.group != 2 || h.shard != 1 || h.batch0 != 18 || h.batch != 9 ||
          h.plan.limb0 != 2 || h.plan.nlimbs != 2) {
        std::printf("FAIL hybrid plan\n");
        return 1;
      }
    }
    std::printf("cpp api ok\n");
    return 0;
  } catch (const fhe::Error& e) {
    std::printf("fhe::Error %d: %s\n", e.code, e.what());
    return 2;
  }
}
