// Host-code sanitizer run (ASan/UBSan on the host side): the pure-host parts of
// libfhecore -- number theory and table construction (csrc/host_tables.cpp), the FHEC wire
// parser (csrc/wire.cpp) -- and the C oracle (oracle/fhe_oracle.c, test infrastructure), built
// with -fsanitize=address,undefined by tests/cpp/Makefile and exercised here with checks of their
// own.  GPU code is out of scope (no device sanitizers on this pool).  tests/test_sanitizers.py
// builds and runs it; it prints "host_sanitize OK" and exits 0 when every check holds.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../gpu-fhe_amd/csrc/host_tables.hpp"
#include "../../gpu-fhe_amd/csrc/wire.hpp"

extern "C" {
int oracle_gen_moduli(uint32_t log_n, uint32_t count, uint32_t bits, uint32_t skip, uint64_t* out);
void oracle_ntt_fwd(uint64_t* data, uint64_t polys, uint32_t log_n, const uint64_t* moduli,
                    uint32_t L);
void oracle_ntt_inv(uint64_t* data, uint64_t polys, uint32_t log_n, const uint64_t* moduli,
                    uint32_t L);
void oracle_vec_op(int op, uint64_t* out, const uint64_t* a, const uint64_t* b, uint64_t rows,
                   uint64_t cols, const uint64_t* mods, uint64_t mod_stride);
void oracle_hommult(uint64_t* d, const uint64_t* a, const uint64_t* b, uint64_t batch,
                    uint32_t log_n, const uint64_t* moduli, uint32_t L);
void oracle_baseconv(uint64_t* out, const uint64_t* x, uint64_t n, const uint64_t* src, uint32_t S,
                     const uint64_t* dst, uint32_t T);
void oracle_keyswitch(uint64_t* ks0, uint64_t* ks1, const uint64_t* d2, const uint64_t* evk_b,
                      const uint64_t* evk_a, uint32_t log_n, const uint64_t* qs, uint32_t L,
                      const uint64_t* ps, uint32_t K, uint32_t dnum);
}

using namespace fhe;

static int g_fail = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                            \
    }                                                                      \
  } while (0)

static std::mt19937_64 rng(12345);

static std::vector<u64> uniform(const std::vector<u64>& mods, size_t per) {
  std::vector<u64> v(mods.size() * per);
  for (size_t l = 0; l < mods.size(); ++l)
    for (size_t i = 0; i < per; ++i) v[l * per + i] = rng() % mods[l];
  return v;
}

static void test_moduli_and_tables() {
  for (u32 log_n = 10; log_n <= 17; ++log_n)
    for (u32 bits : {40u, 50u, 55u, 60u, 61u, 62u, 63u}) {
      u64 q[4], qo[4];
      std::string err;
      CHECK(gen_moduli_host(log_n, 4, bits, 1, q, err));
      CHECK(oracle_gen_moduli(log_n, 4, bits, 1, qo) == 0);
      for (int i = 0; i < 4; ++i) {
        CHECK(q[i] == qo[i]);
        CHECK(is_prime_u64(q[i]) && q[i] % (2ull << log_n) == 1 && q[i] < (1ull << bits));
        if (i) CHECK(q[i] < q[i - 1]);
      }
      if (log_n > 12) continue;  // full tables: a few sizes suffice
      const u64 n = 1ull << log_n;
      std::vector<Pair64> twf(n), twi(n), nf(4);
      const u64 psi = ntt_tables(q[0], log_n, twf.data(), twi.data(), nf.data());
      CHECK(powmod_u64(psi, n, q[0]) == q[0] - 1);  // primitive 2N-th root
      std::vector<u64> fw, iw;
      for (u64 k = 0; k < n; ++k) {
        CHECK(twf[k].x < q[0] && twf[k].y == (u64)(((u128)twf[k].x << 64) / q[0]));
        CHECK(twi[k].x < q[0] && twi[k].y == (u64)(((u128)twi[k].x << 64) / q[0]));
        fw.push_back(twf[k].x);
        iw.push_back(mulmod_u64(twf[k].x, twi[k].x, q[0]));  // lane-major keeps pairs aligned
      }
      for (u64 v : iw) CHECK(v == 1);
      CHECK(mulmod_u64(nf[0].x, n % q[0], q[0]) == 1);
      const ModParams m = make_mod_params(q[0]);
      CHECK((m.mu == 0) == (q[0] >= (1ull << 61)));
      CHECK(m.q * (0 - m.qinv) == 1);  // qinv = -q^-1 mod 2^64
    }
  std::string err;
  u64 q;
  CHECK(!gen_moduli_host(10, 1, 64, 0, &q, err) && !err.empty());
  CHECK(!gen_moduli_host(16, 1, 12, 0, &q, err));
}

static void test_lane_major_permutation() {
  for (u32 log_n : {10u, 13u, 16u}) {
    const u64 n = 1ull << log_n;
    std::vector<Pair64> t(2 * n);
    for (u64 i = 0; i < 2 * n; ++i) t[i] = Pair64{i, ~i};
    lane_major_rows(t.data(), t.size(), log_n, 4);
    std::vector<char> seen(2 * n, 0);
    for (u64 i = 0; i < 2 * n; ++i) {
      CHECK(t[i].y == ~t[i].x && t[i].x < 2 * n && i / n == t[i].x / n);
      seen[t[i].x] = 1;
    }
    for (char s : seen) CHECK(s);
  }
}

static void test_conv_tables() {
  std::vector<u64> mods(10);
  std::string err;
  CHECK(gen_moduli_host(12, 10, 60, 0, mods.data(), err));
  for (u32 s0 : {0u, 3u}) {
    const u32 S = 4;
    std::vector<Pair64> inv, hat;
    conv_tables(mods, s0, S, inv, hat);
    CHECK(inv.size() == S && hat.size() == S * mods.size());
    for (u32 k = 0; k < S; ++k) {
      const u64 sk = mods[s0 + k];
      u64 h = 1;
      for (u32 i = 0; i < S; ++i)
        if (i != k) h = mulmod_u64(h, mods[s0 + i] % sk, sk);
      CHECK(mulmod_u64(h, inv[k].x, sk) == 1);
      for (size_t t = 0; t < mods.size(); ++t) {
        u64 hm = 1;
        for (u32 i = 0; i < S; ++i)
          if (i != k) hm = mulmod_u64(hm, mods[s0 + i] % mods[t], mods[t]);
        CHECK(hat[k * mods.size() + t].x == hm);
      }
    }
  }
}

static void test_wire() {
  const u32 log_n = 10;
  const u64 n = 1ull << log_n;
  std::vector<u64> mods(5);
  std::string err;
  CHECK(gen_moduli_host(log_n, 5, 60, 0, mods.data(), err));
  const u32 polys = 2, limb0 = 1, nl = 3;
  size_t size = 0;
  CHECK(wire_size(log_n, polys, nl, &size));
  std::vector<unsigned char> blob(size);
  wire_header(blob.data(), log_n, polys, limb0, nl, 1, mods.data() + limb0);
  std::vector<u64> body;
  for (u32 p = 0; p < polys; ++p) {
    auto r = uniform(std::vector<u64>(mods.begin() + limb0, mods.begin() + limb0 + nl), n);
    body.insert(body.end(), r.begin(), r.end());
  }
  std::memcpy(blob.data() + 24 + 8 * nl, body.data(), body.size() * 8);
  wire_seal(blob.data(), size);
  WireInfo info{};
  CHECK(wire_parse(blob.data(), size, log_n, mods.data(), mods.size(), info, err));
  CHECK(info.polys == polys && info.limb0 == limb0 && info.nlimbs == nl && info.ntt_form == 1);
  CHECK(info.words == body.size() &&
        std::memcmp(blob.data() + info.body, body.data(), body.size() * 8) == 0);
  // every single-byte corruption is caught, and nothing reads outside the buffer
  for (int trial = 0; trial < 400; ++trial) {
    std::vector<unsigned char> bad(blob);
    bad[rng() % bad.size()] ^= (unsigned char)(1 + rng() % 255);
    CHECK(!wire_parse(bad.data(), bad.size(), log_n, mods.data(), mods.size(), info, err));
  }
  // truncations and hostile headers (sizes that overflow, windows past the context)
  for (size_t cut : {(size_t)0, (size_t)7, (size_t)24, size / 2, size - 1})
    CHECK(!wire_parse(blob.data(), cut, log_n, mods.data(), mods.size(), info, err));
  for (u32 hp : {0xffffffffu, 0x40000000u})
    for (u32 hl : {0xffffffffu, 3u}) {
      std::vector<unsigned char> bad(blob);
      std::memcpy(bad.data() + 12, &hp, 4);
      std::memcpy(bad.data() + 20, &hl, 4);
      CHECK(!wire_parse(bad.data(), bad.size(), log_n, mods.data(), mods.size(), info, err));
    }
  size_t huge = 0;
  CHECK(!wire_size(17, 0xffffffffull, 0xffffffffull, &huge) || huge > size);
  // a residue >= q with a valid checksum is still refused
  std::vector<unsigned char> bad(blob);
  const u64 q = mods[limb0];
  std::memcpy(bad.data() + 24 + 8 * nl, &q, 8);
  wire_seal(bad.data(), bad.size());
  CHECK(!wire_parse(bad.data(), bad.size(), log_n, mods.data(), mods.size(), info, err));
}

// negacyclic schoolbook product, exact
static std::vector<u64> negacyclic(const u64* a, const u64* b, u64 n, u64 q) {
  std::vector<u64> c(n, 0);
  for (u64 i = 0; i < n; ++i)
    for (u64 j = 0; j < n; ++j) {
      const u64 p = mulmod_u64(a[i], b[j], q);
      const u64 k = (i + j) % n;
      c[k] = (i + j < n) ? (c[k] + p) % q : (c[k] + q - p) % q;
    }
  return c;
}

static void test_oracle() {
  const u32 log_n = 10, L = 3;
  const u64 n = 1ull << log_n;
  for (u32 bits : {55u, 60u, 63u}) {
    std::vector<u64> mods(L);
    std::string err;
    CHECK(gen_moduli_host(log_n, L, bits, 0, mods.data(), err));
    auto x = uniform(mods, n);
    auto y = x;
    oracle_ntt_fwd(y.data(), 1, log_n, mods.data(), L);
    oracle_ntt_inv(y.data(), 1, log_n, mods.data(), L);
    CHECK(y == x);
    // HomMult against the schoolbook product, one ciphertext pair
    std::vector<u64> a, b;
    for (int p = 0; p < 2; ++p) {
      auto r = uniform(mods, n), s = uniform(mods, n);
      a.insert(a.end(), r.begin(), r.end());
      b.insert(b.end(), s.begin(), s.end());
    }
    std::vector<u64> d(3 * L * n);
    oracle_hommult(d.data(), a.data(), b.data(), 1, log_n, mods.data(), L);
    for (u32 l = 0; l < L; ++l) {
      const u64 q = mods[l];
      const u64 *a0 = &a[l * n], *a1 = &a[(L + l) * n], *b0 = &b[l * n], *b1 = &b[(L + l) * n];
      CHECK(std::memcmp(&d[l * n], negacyclic(a0, b0, n, q).data(), n * 8) == 0);
      auto t1 = negacyclic(a0, b1, n, q), t2 = negacyclic(a1, b0, n, q);
      for (u64 i = 0; i < n; ++i) CHECK(d[(L + l) * n + i] == (t1[i] + t2[i]) % q);
      CHECK(std::memcmp(&d[(2 * L + l) * n], negacyclic(a1, b1, n, q).data(), n * 8) == 0);
    }
    std::vector<u64> o(L * n);
    oracle_vec_op(2, o.data(), a.data(), b.data(), L, n, mods.data(), 1);
    for (u64 i = 0; i < L * n; ++i) CHECK(o[i] == mulmod_u64(a[i], b[i], mods[i / n]));
  }
  // base conversion: a small CRT value converts exactly
  std::vector<u64> mods(7);
  std::string err;
  CHECK(gen_moduli_host(log_n, 7, 60, 0, mods.data(), err));
  std::vector<u64> xs(3 * n), out(4 * n);
  for (u64 i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) xs[k * n + i] = i * 7919 % mods[k];
  oracle_baseconv(out.data(), xs.data(), n, mods.data(), 3, mods.data() + 3, 4);
  for (u64 i = 0; i < n; ++i)
    for (int t = 0; t < 4; ++t) {
      // fast base conversion: X + e Q for some 0 <= e < 3
      const u64 want = i * 7919 % mods[3 + t];
      bool ok = false;
      u64 qprod = 1;
      for (int k = 0; k < 3; ++k) qprod = mulmod_u64(qprod, mods[k] % mods[3 + t], mods[3 + t]);
      for (u64 e = 0; e < 3; ++e)
        ok = ok || out[t * n + i] == (want + mulmod_u64(e, qprod, mods[3 + t])) % mods[3 + t];
      CHECK(ok);
    }
  // key-switch runs clean (shapes, ragged digit) -- values are checked on the GPU side
  const u32 Lq = 3, K = 2, dnum = 2;
  std::vector<u64> qs(mods.begin(), mods.begin() + Lq), ps(mods.begin() + Lq, mods.begin() + Lq + K);
  std::vector<u64> allm(qs);
  allm.insert(allm.end(), ps.begin(), ps.end());
  auto d2 = uniform(qs, n);
  std::vector<u64> eb, ea;
  for (u32 j = 0; j < dnum; ++j) {
    auto r = uniform(allm, n), s = uniform(allm, n);
    eb.insert(eb.end(), r.begin(), r.end());
    ea.insert(ea.end(), s.begin(), s.end());
  }
  std::vector<u64> k0(Lq * n), k1(Lq * n);
  oracle_keyswitch(k0.data(), k1.data(), d2.data(), eb.data(), ea.data(), log_n, qs.data(), Lq,
                   ps.data(), K, dnum);
  for (u64 i = 0; i < Lq * n; ++i) CHECK(k0[i] < qs[i / n] && k1[i] < qs[i / n]);
}

int main() {
  test_moduli_and_tables();
  test_lane_major_permutation();
  test_conv_tables();
  test_wire();
  test_oracle();
  if (g_fail) {
    std::fprintf(stderr, "host_sanitize: %d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_sanitize OK\n");
  return 0;
}
