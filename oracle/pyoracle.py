"""CPU math oracle for the FHE polynomial-arithmetic hot path (TEST INFRASTRUCTURE ONLY).

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  The shipped path lives in
``gpu-fhe_amd/`` and runs hand-written HIP kernels; it never routes through this file.

What it restates
----------------
* ``vec_add`` / ``vec_sub`` / ``vec_mul``: the reference's coefficient-wise modular ops,
  ``/root/reference/arithmetic.py:3-13`` (``(a op b) % MOD``), with EXACT semantics -- the
  values the reference produces on ``dtype=object`` inputs.  Pinned by the golden vectors in
  ``tests/golden/`` that ``tests/golden/make_golden.py`` captured by importing the reference.
* ``NTT`` / ``iNTT``: the reference's are identities (``arithmetic.py:15-19``), so their
  parity is UNPINNED BY THE REFERENCE.  The build-defined spec (SURVEY.md §8a') is restated
  here twice -- as the O(N^2) defining sum and as the Cooley-Tukey / Gentleman-Sande loops --
  and the two are checked against each other and against a schoolbook negacyclic product.
* HomMult, RNS fast base conversion, ModUp / ModDown and the hybrid key-switch:
  absent from the reference; restated from SURVEY.md §8a'.

Everything is exact Python-int arithmetic; numpy object arrays vectorise the small cases.
"""
from __future__ import annotations

import math
import random
from functools import lru_cache

import numpy as np

# --------------------------------------------------------------------------------------
# number theory
# --------------------------------------------------------------------------------------

_MR_BASES = (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37)


def is_prime(n: int) -> bool:
    """Deterministic Miller-Rabin for n < 3.3e24 (covers every 64-bit modulus)."""
    if n < 2:
        return False
    for p in _MR_BASES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in _MR_BASES:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _pollard_rho(n: int) -> int:
    if n % 2 == 0:
        return 2
    rng = random.Random(n)
    while True:
        c = rng.randrange(1, n)
        x = y = rng.randrange(2, n)
        d = 1
        while d == 1:
            x = (x * x + c) % n
            y = (y * y + c) % n
            y = (y * y + c) % n
            d = math.gcd(abs(x - y), n)
        if d != n:
            return d


def factorize(n: int) -> dict:
    """Prime factorisation {p: e} (Pollard rho + Miller-Rabin)."""
    out: dict = {}
    stack = [n]
    while stack:
        m = stack.pop()
        if m == 1:
            continue
        if is_prime(m):
            out[m] = out.get(m, 0) + 1
            continue
        for p in (2, 3, 5, 7, 11, 13):
            if m % p == 0:
                stack += [p, m // p]
                break
        else:
            d = _pollard_rho(m)
            stack += [d, m // d]
    return out


@lru_cache(maxsize=None)
def primitive_root(q: int) -> int:
    """Smallest generator of (Z/qZ)^* (SURVEY.md §8a': g = smallest primitive root)."""
    fs = list(factorize(q - 1))
    g = 2
    while True:
        if all(pow(g, (q - 1) // f, q) != 1 for f in fs):
            return g
        g += 1


@lru_cache(maxsize=None)
def psi_for(q: int, n: int) -> int:
    """psi = g^((q-1)/2N) mod q: a primitive 2N-th root of unity (SURVEY.md §8a')."""
    assert (q - 1) % (2 * n) == 0, "q must be 1 mod 2N"
    psi = pow(primitive_root(q), (q - 1) // (2 * n), q)
    assert pow(psi, n, q) == q - 1
    return psi


def gen_moduli(log_n: int, count: int, bits: int = 60, skip: int = 0) -> list:
    """The ``count`` largest primes q < 2^bits with q = 1 (mod 2N), descending, after skipping
    the first ``skip`` (SURVEY.md §8a': "the largest primes below 2^60, in descending order";
    special primes P continue the same list)."""
    step = 2 << log_n
    q = ((1 << bits) - 1) // step * step + 1
    if q >= (1 << bits):
        q -= step
    out = []
    while len(out) < count + skip:
        if is_prime(q):
            out.append(q)
        q -= step
        assert q > step, "ran out of NTT primes"
    return out[skip:]


def bitrev(x: int, bits: int) -> int:
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


@lru_cache(maxsize=None)
def twiddles(q: int, log_n: int):
    """(psi_brv, psi_inv_brv, n_inv): psi_brv[k] = psi^brv(k), psi_inv_brv[k] = psi^-brv(k)."""
    n = 1 << log_n
    psi = psi_for(q, n)
    psi_inv = pow(psi, q - 2, q)
    pw = [1] * n
    pwi = [1] * n
    for i in range(1, n):
        pw[i] = pw[i - 1] * psi % q
        pwi[i] = pwi[i - 1] * psi_inv % q
    brv = [bitrev(k, log_n) for k in range(n)]
    return [pw[b] for b in brv], [pwi[b] for b in brv], pow(n, q - 2, q)


# --------------------------------------------------------------------------------------
# reference operators, exact semantics (arithmetic.py:3-13, ' polynomial.py':3-5)
# --------------------------------------------------------------------------------------

def _obj(x):
    return np.asarray(x).astype(object)


def vec_add(a, b, mod):
    """(a + b) % MOD, exact -- arithmetic.py:3-5 on dtype=object."""
    assert np.shape(a) == np.shape(b)
    return (_obj(a) + _obj(b)) % _obj(mod)


def vec_sub(a, b, mod):
    """(a - b) % MOD, exact (Python floor-mod: result in [0, MOD)) -- arithmetic.py:7-9."""
    assert np.shape(a) == np.shape(b)
    return (_obj(a) - _obj(b)) % _obj(mod)


def vec_mul(a, b, mod):
    """(a * b) % MOD, exact -- arithmetic.py:11-13 (= poly_mul_pointwise in the NTT domain)."""
    assert np.shape(a) == np.shape(b)
    return (_obj(a) * _obj(b)) % _obj(mod)


def poly_add(a, b, mod):
    """Intended result of ' polynomial.py':3-5 (the reference discards it and returns None)."""
    return vec_add(a[0], b[0], mod), vec_add(a[1], b[1], mod)


# --------------------------------------------------------------------------------------
# negacyclic NTT (SURVEY.md §8a')
# --------------------------------------------------------------------------------------

def ntt_naive(a, q: int):
    """Defining sum: NTT(a)[k] = sum_i a_i psi^((2 brv(k) + 1) i) mod q. O(N^2)."""
    n = len(a)
    log_n = n.bit_length() - 1
    psi = psi_for(q, n)
    a = [int(v) for v in a]
    out = []
    for k in range(n):
        root = pow(psi, 2 * bitrev(k, log_n) + 1, q)
        acc, w = 0, 1
        for ai in a:
            acc += ai * w
            w = w * root % q
        out.append(acc % q)
    return out


def ntt_fwd(a, q: int):
    """Cooley-Tukey, natural in -> bit-reversed out (SEAL / Longa-Naehrig loop)."""
    a = [int(v) for v in a]
    n = len(a)
    tw, _, _ = twiddles(q, n.bit_length() - 1)
    t, m = n, 1
    while m < n:
        t //= 2
        for i in range(m):
            s = tw[m + i]
            j1 = 2 * i * t
            for j in range(j1, j1 + t):
                u, v = a[j], a[j + t] * s % q
                a[j], a[j + t] = (u + v) % q, (u - v) % q
        m *= 2
    return a


def ntt_inv(a, q: int):
    """Gentleman-Sande, bit-reversed in -> natural out, times N^-1."""
    a = [int(v) for v in a]
    n = len(a)
    _, twi, n_inv = twiddles(q, n.bit_length() - 1)
    t, m = 1, n
    while m > 1:
        h = m // 2
        j1 = 0
        for i in range(h):
            s = twi[h + i]
            for j in range(j1, j1 + t):
                u, v = a[j], a[j + t]
                a[j], a[j + t] = (u + v) % q, (u - v) * s % q
            j1 += 2 * t
        t *= 2
        m = h
    return [x * n_inv % q for x in a]


def ntt_fwd_np(a, q: int):
    """Vectorised (numpy object) form of ntt_fwd: same butterflies, stage at a time."""
    n = len(a)
    log_n = n.bit_length() - 1
    tw = np.array(twiddles(q, log_n)[0], dtype=object)
    x = np.array([int(v) for v in a], dtype=object)
    for s in range(log_n):
        m, t = 1 << s, n >> (s + 1)
        x = x.reshape(m, 2, t)
        w = tw[m:2 * m].reshape(m, 1)
        u, v = x[:, 0, :], x[:, 1, :] * w % q
        x = np.stack([(u + v) % q, (u - v) % q], axis=1)
    return x.reshape(n)


def ntt_inv_np(a, q: int):
    n = len(a)
    log_n = n.bit_length() - 1
    _, twi, n_inv = twiddles(q, log_n)
    twi = np.array(twi, dtype=object)
    x = np.array([int(v) for v in a], dtype=object)
    for s in range(log_n - 1, -1, -1):
        m, t = 1 << s, n >> (s + 1)
        x = x.reshape(m, 2, t)
        w = twi[m:2 * m].reshape(m, 1)
        u, v = x[:, 0, :], x[:, 1, :]
        x = np.stack([(u + v) % q, (u - v) * w % q], axis=1)
    return x.reshape(n) * n_inv % q


def negacyclic_mul(a, b, q: int):
    """Schoolbook product in Z_q[X]/(X^N + 1)."""
    n = len(a)
    a = np.array([int(v) for v in a], dtype=object)
    b = [int(v) for v in b]
    out = np.zeros(n, dtype=object)
    for j, bj in enumerate(b):
        if bj == 0:
            continue
        rolled = np.concatenate([-a[n - j:], a[:n - j]]) if j else a
        out = out + rolled * bj
    return out % q


# --------------------------------------------------------------------------------------
# RNS polynomials: arrays shaped [..., limb, N] (limb-major, SURVEY.md §2 kernel inventory)
# --------------------------------------------------------------------------------------

def rns_ntt_fwd(x, moduli):
    x = np.asarray(x)
    out = np.empty(x.shape, dtype=object)
    for idx in np.ndindex(*x.shape[:-1]):
        out[idx] = ntt_fwd_np(x[idx], moduli[idx[-1]])
    return out


def rns_ntt_inv(x, moduli):
    x = np.asarray(x)
    out = np.empty(x.shape, dtype=object)
    for idx in np.ndindex(*x.shape[:-1]):
        out[idx] = ntt_inv_np(x[idx], moduli[idx[-1]])
    return out


def _mods_col(moduli):
    return np.array([int(q) for q in moduli], dtype=object).reshape(-1, 1)


def hommult(a, b, moduli):
    """ct x ct tensor (SURVEY.md §8a'): a, b = (2, L, N) coefficient form -> (3, L, N).
    d0 = A0 B0, d1 = A0 B1 + A1 B0, d2 = A1 B1 (NTT domain, per limb), then INTT."""
    qs = _mods_col(moduli)
    A = rns_ntt_fwd(a, moduli)
    B = rns_ntt_fwd(b, moduli)
    d0 = A[0] * B[0] % qs
    d1 = (A[0] * B[1] + A[1] * B[0]) % qs
    d2 = A[1] * B[1] % qs
    return rns_ntt_inv(np.stack([d0, d1, d2]), moduli)


def baseconv(x, src, dst):
    """Fast basis extension without correction (SURVEY.md §8a'), coefficient domain.
    x: (len(src), N). y_i = [x_i * (S/s_i)^-1]_{s_i}; out_t = sum_i y_i * ((S/s_i) mod t) mod t."""
    src = [int(s) for s in src]
    S = math.prod(src)
    x = np.asarray(x).astype(object)
    ys = []
    for i, s in enumerate(src):
        hat = S // s
        ys.append(x[i] * pow(hat % s, -1, s) % s)
    out = []
    for t in dst:
        t = int(t)
        acc = np.zeros(x.shape[-1], dtype=object)
        for i, s in enumerate(src):
            acc = acc + ys[i] * ((S // s) % t)
        out.append(acc % t)
    return np.stack(out)


def digit_ranges(L: int, dnum: int):
    """Limb ranges of the dnum gadget digits: alpha = ceil(L / dnum) limbs each (last may be short)."""
    alpha = -(-L // dnum)
    return [(j * alpha, min(L, (j + 1) * alpha)) for j in range(dnum) if j * alpha < L]


def modup(c, qs, ps, dnum):
    """c: (L, N) coefficient form over Q. Returns [dnum] arrays of shape (L + K, N): digit j
    extended from its limbs D_j to every limb of Q u P (own limbs copied)."""
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    allm = qs + ps
    out = []
    for lo, hi in digit_ranges(len(qs), dnum):
        dj = qs[lo:hi]
        others = [i for i in range(len(allm)) if not lo <= i < hi]
        conv = baseconv(c[lo:hi], dj, [allm[i] for i in others])
        ext = np.empty((len(allm), c.shape[-1]), dtype=object)
        ext[lo:hi] = np.asarray(c[lo:hi]).astype(object)
        for k, i in enumerate(others):
            ext[i] = conv[k]
        out.append(ext)
    return out


def moddown_ntt(acc, qs, ps):
    """acc: (L + K, N) NTT form over Q u P -> (L, N) NTT form over Q:
    out = (acc_Q - NTT(conv_{P->Q}(INTT(acc_P)))) * P^-1 mod q_i."""
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    L = len(qs)
    xp = rns_ntt_inv(np.asarray(acc[L:]), ps)
    conv = baseconv(xp, ps, qs)
    convn = rns_ntt_fwd(conv, qs)
    P = math.prod(ps)
    out = []
    for i, q in enumerate(qs):
        out.append((acc[i] - convn[i]) * pow(P % q, -1, q) % q)
    return np.stack(out)


def keyswitch(d2_ntt, evk_b, evk_a, qs, ps, dnum):
    """Hybrid key-switch (SURVEY.md §8a'): d2 (L, N) NTT form over Q; evk_b/evk_a (dnum, L+K, N)
    NTT form over Q u P.  Returns (ks0, ks1), each (L, N) NTT form over Q."""
    allm = list(qs) + list(ps)
    c = rns_ntt_inv(d2_ntt, qs)
    ext = modup(c, qs, ps, dnum)
    mods = _mods_col(allm)
    acc0 = np.zeros((len(allm), c.shape[-1]), dtype=object)
    acc1 = np.zeros_like(acc0)
    for j, e in enumerate(ext):
        en = rns_ntt_fwd(e, allm)
        acc0 = (acc0 + en * np.asarray(evk_b[j]).astype(object)) % mods
        acc1 = (acc1 + en * np.asarray(evk_a[j]).astype(object)) % mods
    return moddown_ntt(acc0, qs, ps), moddown_ntt(acc1, qs, ps)


# --------------------------------------------------------------------------------------
# small-N key material for the decrypt check (not on the hot path)
# --------------------------------------------------------------------------------------

def _to_rns(poly, mods):
    return np.stack([np.array([int(v) % m for v in poly], dtype=object) for m in mods])


def gen_relin_key(s, qs, ps, dnum, rng):
    """evk_j = (-a_j s + e_j + P g_j s^2, a_j) over Q u P, NTT form; g_j = CRT gadget of digit j
    (g_j = 1 mod the primes of D_j, 0 mod the other primes of Q)."""
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    allm = qs + ps
    n = len(s)
    Q, P = math.prod(qs), math.prod(ps)
    s_rns = _to_rns(s, allm)
    s_n = rns_ntt_fwd(s_rns, allm)
    mods = _mods_col(allm)
    s2_n = s_n * s_n % mods
    evk_b, evk_a = [], []
    for lo, hi in digit_ranges(len(qs), dnum):
        Dj = math.prod(qs[lo:hi])
        Qhat = Q // Dj
        g = Qhat * pow(Qhat % Dj, -1, Dj)
        a = np.stack([np.array([rng.randrange(m) for _ in range(n)], dtype=object) for m in allm])
        e = [rng.randrange(-3, 4) for _ in range(n)]
        e_n = rns_ntt_fwd(_to_rns(e, allm), allm)
        pg = np.array([(P * g) % m for m in allm], dtype=object).reshape(-1, 1)
        b = (-a * s_n + e_n + pg * s2_n) % mods
        evk_b.append(b)
        evk_a.append(a)
    return np.stack(evk_b), np.stack(evk_a)


def crt_centered(x_rns, qs):
    """CRT-reconstruct (L, N) residues to centred integers in (-Q/2, Q/2]."""
    qs = [int(q) for q in qs]
    Q = math.prod(qs)
    acc = 0
    for i, q in enumerate(qs):
        hat = Q // q
        acc = acc + np.asarray(x_rns[i]).astype(object) * (hat * pow(hat % q, -1, q))
    acc = acc % Q
    return np.where(acc > Q // 2, acc - Q, acc)


def keyswitch_shard(c_all, d2_own, evk_b_own, evk_a_own, qs, ps, dnum, lo, hi):
    """One rank's part of the limb-sharded key-switch, restated on the CPU.

    c_all: (L, N) coefficient form of all of d2 (after the all-gather); d2_own: (hi - lo, N) NTT
    form of Q-limbs [lo, hi); evk_*_own: (dnum, hi - lo + K, N) rows = own Q-limbs then P-limbs.
    Uses nothing but these inputs; returns (ks0, ks1) for limbs [lo, hi), NTT form."""
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    L, K = len(qs), len(ps)
    rows = list(range(lo, hi)) + list(range(L, L + K))
    allm = qs + ps
    rmods = [allm[t] for t in rows]
    n = np.asarray(c_all).shape[-1]
    c_all = np.asarray(c_all).astype(object)
    acc0 = np.zeros((len(rows), n), dtype=object)
    acc1 = np.zeros_like(acc0)
    col = _mods_col(rmods)
    for j, (dlo, dhi) in enumerate(digit_ranges(L, dnum)):
        others = [t for t in rows if not dlo <= t < dhi]
        conv = baseconv(c_all[dlo:dhi], qs[dlo:dhi], [allm[t] for t in others]) if others else []
        convn = rns_ntt_fwd(conv, [allm[t] for t in others]) if others else []
        ext = np.empty((len(rows), n), dtype=object)
        k = 0
        for r, t in enumerate(rows):
            if dlo <= t < dhi:
                ext[r] = np.asarray(d2_own[r]).astype(object)
            else:
                ext[r] = convn[k]
                k += 1
        acc0 = (acc0 + ext * np.asarray(evk_b_own[j]).astype(object)) % col
        acc1 = (acc1 + ext * np.asarray(evk_a_own[j]).astype(object)) % col
    nq = hi - lo
    P = math.prod(ps)
    outs = []
    for acc in (acc0, acc1):
        xp = rns_ntt_inv(acc[nq:], ps)
        conv = rns_ntt_fwd(baseconv(xp, ps, qs[lo:hi]), qs[lo:hi])
        outs.append(np.stack([(acc[i] - conv[i]) * pow(P % q, -1, q) % q
                              for i, q in enumerate(qs[lo:hi])]))
    return outs[0], outs[1]


# ---- rescale and rotation (Galois automorphisms) ------------------------
# Not in the reference (its repo has no ciphertext operations beyond poly_add); restated from the
# standard RNS-CKKS definitions (SEAL's divide_and_round_q_last / apply_galois, OpenFHE's
# ModReduce / Automorphism), on this repo's layout and NTT convention (SURVEY.md §8a').


def galois_elt(step: int, n: int) -> int:
    """Galois element of a rotation by `step` slots: 5^step mod 2N (step < 0: 5^-|step|)."""
    return pow(5, step, 2 * n) if step >= 0 else pow(pow(5, -step, 2 * n), -1, 2 * n)


def automorphism_coeff(x, k: int, moduli):
    """sigma_k(a)(X) = a(X^k), k odd, coefficient form (L, N): coefficient i moves to i k mod 2N,
    negated when that lands in [N, 2N)."""
    x = np.asarray(x, dtype=object)
    n = x.shape[-1]
    out = np.zeros_like(x)
    for l, q in enumerate(moduli):
        q = int(q)
        for i in range(n):
            m = i * k % (2 * n)
            v = int(x[l][i])
            if m < n:
                out[l][m] = v
            else:
                out[l][m - n] = (q - v) % q
    return out


def automorphism_ntt_index(k: int, log_n: int):
    """NTT-domain automorphism as a gather: out[j] = in[src[j]].  Slot j holds the evaluation at
    psi^(2 brv(j) + 1); sigma_k maps it to the evaluation at psi^((2 brv(j) + 1) k)."""
    n = 1 << log_n
    src = []
    for j in range(n):
        e = (2 * bitrev(j, log_n) + 1) * k % (2 * n)
        src.append(bitrev((e - 1) // 2, log_n))
    return src


def automorphism_ntt(x, k: int, log_n: int):
    idx = automorphism_ntt_index(k, log_n)
    x = np.asarray(x, dtype=object)
    return x[..., idx]


def gen_switch_key(s, s_from_ntt, qs, ps, dnum, rng):
    """Key-switch key from s_from (given in NTT form over Q u P) to s: the gen_relin_key
    construction with s^2 replaced by s_from (evk_j = (-a_j s + e_j + P g_j s_from, a_j))."""
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    allm = qs + ps
    n = len(s)
    Q, P = math.prod(qs), math.prod(ps)
    s_n = rns_ntt_fwd(_to_rns(s, allm), allm)
    mods = _mods_col(allm)
    evk_b, evk_a = [], []
    for lo, hi in digit_ranges(len(qs), dnum):
        Dj = math.prod(qs[lo:hi])
        Qhat = Q // Dj
        g = Qhat * pow(Qhat % Dj, -1, Dj)
        a = np.stack([np.array([rng.randrange(m) for _ in range(n)], dtype=object) for m in allm])
        e = [rng.randrange(-3, 4) for _ in range(n)]
        e_n = rns_ntt_fwd(_to_rns(e, allm), allm)
        pg = np.array([(P * g) % m for m in allm], dtype=object).reshape(-1, 1)
        b = (-a * s_n + e_n + pg * np.asarray(s_from_ntt, dtype=object)) % mods
        evk_b.append(b)
        evk_a.append(a)
    return np.stack(evk_b), np.stack(evk_a)


def gen_rot_key(s, k: int, qs, ps, dnum, rng):
    """Rotation key for Galois element k: switches sigma_k(s) back to s."""
    allm = [int(m) for m in list(qs) + list(ps)]
    sk = automorphism_coeff(_to_rns(s, allm), k, allm)
    return gen_switch_key(s, rns_ntt_fwd(sk, allm), qs, ps, dnum, rng)


def rotate(ct_ntt, k: int, rot_b, rot_a, qs, ps, dnum, log_n: int):
    """ct = (c0, c1) in NTT form over Q: (sigma_k c0 + KS0(sigma_k c1), KS1(sigma_k c1)).
    Decrypts to sigma_k(m) under s."""
    c0 = automorphism_ntt(ct_ntt[0], k, log_n)
    c1 = automorphism_ntt(ct_ntt[1], k, log_n)
    ks0, ks1 = keyswitch(c1, rot_b, rot_a, qs, ps, dnum)
    col = _mods_col(qs)
    return np.stack([(c0 + ks0) % col, ks1 % col])


def rotate_hoisted(ct_ntt, ks, keys, qs, ps, dnum, log_n: int):
    """Hoisted rotations (Halevi-Shoup), restated for gpu-fhe_amd/csrc/galois.hip
    launch_rotate_hoisted: ModUp(c1) once -- INTT, digit base conversion, NTT of every extended
    digit -- then per Galois element k with key (rot_b, rot_a): the digits gathered through
    sigma_k in the NTT domain, the inner product with the key, ModDown, plus sigma_k(c0).
    Not bit-identical to rotate() (ModUp(sigma c1) differs from sigma ModUp(c1) by multiples of
    the digit moduli), but decrypts to sigma_k(m) the same way.  Returns [len(ks), 2, L, N]."""
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    allm = qs + ps
    c1 = np.asarray(ct_ntt[1]).astype(object)
    ext = [rns_ntt_fwd(e, allm) for e in modup(rns_ntt_inv(c1, qs), qs, ps, dnum)]
    # the digit's own rows are c1 itself (NTT(INTT(c1)) = c1)
    for (lo, hi), e in zip(digit_ranges(len(qs), dnum), ext):
        e[lo:hi] = c1[lo:hi]
    mods = _mods_col(allm)
    col = _mods_col(qs)
    out = []
    for k, (rot_b, rot_a) in zip(ks, keys):
        idx = automorphism_ntt_index(k, log_n)
        acc0 = np.zeros((len(allm), c1.shape[-1]), dtype=object)
        acc1 = np.zeros_like(acc0)
        for j, e in enumerate(ext):
            g = e[..., idx]
            acc0 = (acc0 + g * np.asarray(rot_b[j]).astype(object)) % mods
            acc1 = (acc1 + g * np.asarray(rot_a[j]).astype(object)) % mods
        c0 = automorphism_ntt(ct_ntt[0], k, log_n)
        out.append(np.stack([(c0 + moddown_ntt(acc0, qs, ps)) % col, moddown_ntt(acc1, qs, ps)]))
    return np.stack(out)


def rotate_sum_hoisted(ct_ntt, ks, keys, pts, qs, ps, dnum, log_n: int):
    """sum_r pt_r * rot_{k_r}(ct) with one ModUp and one ModDown (double hoisting, the inner
    loop of a baby-step / giant-step linear transform), restated for gpu-fhe_amd/csrc/galois.hip
    launch_rotate_sum_hoisted.  pts[r]: (L + K, N) NTT form over Q u P.  Per rotation the
    key-switch accumulators of rotate_hoisted are multiplied by pt_r and summed in Q u P;
    sigma_k(c0) times pt_r is summed over Q; ModDown runs once on each summed accumulator:
      out = (sum_r pt_r sigma_r(c0) + ModDown(A0), ModDown(A1)),
      A_h = sum_r pt_r acc_h^(r).
    k_r = 1 is the unrotated term (no key; keys[r] may be None): pt_r c0 joins the c0 sum and
    pt_r (P mod q_i) c1 joins A1's Q rows, so that ModDown returns pt_r c1 exactly
    (ModDown(P x + y) = x + ModDown(y)).  Decrypts to sum_r pt_r sigma_r(m) up to one ModDown's
    rounding, not to the sum of separate rotate_hoisted outputs bit for bit.  (L, N) x 2 out."""
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    allm = qs + ps
    L = len(qs)
    P = math.prod(ps)
    c0 = np.asarray(ct_ntt[0]).astype(object)
    c1 = np.asarray(ct_ntt[1]).astype(object)
    n = c1.shape[-1]
    mods = _mods_col(allm)
    col = _mods_col(qs)
    ext = None
    if any(int(k) != 1 for k in ks):
        ext = [rns_ntt_fwd(e, allm) for e in modup(rns_ntt_inv(c1, qs), qs, ps, dnum)]
        for (lo, hi), e in zip(digit_ranges(L, dnum), ext):
            e[lo:hi] = c1[lo:hi]
    a0 = np.zeros((len(allm), n), dtype=object)
    a1 = np.zeros_like(a0)
    s0 = np.zeros((L, n), dtype=object)
    pcol = np.array([P % q for q in qs], dtype=object).reshape(-1, 1)
    for k, key, pt in zip(ks, keys, pts):
        k = int(k)
        pt = np.asarray(pt).astype(object)
        if k == 1:
            s0 = (s0 + pt[:L] * c0) % col
            a1[:L] = (a1[:L] + pt[:L] * (pcol * c1 % col)) % col
            continue
        rot_b, rot_a = key
        idx = automorphism_ntt_index(k, log_n)
        acc0 = np.zeros((len(allm), n), dtype=object)
        acc1 = np.zeros_like(acc0)
        for j, e in enumerate(ext):
            g = e[..., idx]
            acc0 = (acc0 + g * np.asarray(rot_b[j]).astype(object)) % mods
            acc1 = (acc1 + g * np.asarray(rot_a[j]).astype(object)) % mods
        a0 = (a0 + pt * acc0) % mods
        a1 = (a1 + pt * acc1) % mods
        s0 = (s0 + pt[:L] * c0[..., idx]) % col
    return np.stack([(s0 + moddown_ntt(a0, qs, ps)) % col, moddown_ntt(a1, qs, ps)])


def rotate_sum_multi(cts, ks, keys, qs, ps, dnum, log_n: int):
    """sum_r rot_{k_r}(cts[r]) over different ciphertexts with ONE ModDown (the giant-step sum of a
    baby-step / giant-step linear transform), restated for gpu-fhe_amd/csrc/galois.hip
    launch_rotate_sum_multi.  Per rotated term: ModUp of its own c1, the gathered inner product
    with its key added into the Q u P sums A_h, sigma_k(c0) into the c0 sum; an unrotated term
    (k = 1, no key) adds c0 and c1 themselves (exactly: ModDown(P x + y) = x + ModDown(y)).
      out = (C0 + ModDown(A0), C1 + ModDown(A1)).  (L, N) x 2 out."""
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    allm = qs + ps
    L = len(qs)
    mods = _mods_col(allm)
    col = _mods_col(qs)
    n = np.asarray(cts[0]).shape[-1]
    a0 = np.zeros((len(allm), n), dtype=object)
    a1 = np.zeros_like(a0)
    s0 = np.zeros((L, n), dtype=object)
    s1 = np.zeros_like(s0)
    for ct, k, key in zip(cts, ks, keys):
        k = int(k)
        c0 = np.asarray(ct[0]).astype(object)
        c1 = np.asarray(ct[1]).astype(object)
        if k == 1:
            s0 = (s0 + c0) % col
            s1 = (s1 + c1) % col
            continue
        ext = [rns_ntt_fwd(e, allm) for e in modup(rns_ntt_inv(c1, qs), qs, ps, dnum)]
        for (lo, hi), e in zip(digit_ranges(L, dnum), ext):
            e[lo:hi] = c1[lo:hi]
        rot_b, rot_a = key
        idx = automorphism_ntt_index(k, log_n)
        for j, e in enumerate(ext):
            g = e[..., idx]
            a0 = (a0 + g * np.asarray(rot_b[j]).astype(object)) % mods
            a1 = (a1 + g * np.asarray(rot_a[j]).astype(object)) % mods
        s0 = (s0 + c0[..., idx]) % col
    return np.stack([(s0 + moddown_ntt(a0, qs, ps)) % col, (s1 + moddown_ntt(a1, qs, ps)) % col])


def linear_transform(ct_ntt, baby, baby_keys, giant, giant_keys, pts, qs, ps, dnum, log_n: int):
    """Baby-step / giant-step plaintext-matrix product with both hoistings, restated for
    gpu-fhe_amd/csrc/galois.hip launch_linear_transform:
      out = sum_g rot_{giant[g]}( sum_b pts[g][b] rot_{baby[b]}(ct) ),
    each giant step's inner sum exactly rotate_sum_hoisted (one ModUp of ct shared by all of them on
    the device, one ModDown each), the outer sum exactly rotate_sum_multi (one ModDown)."""
    inner = [rotate_sum_hoisted(ct_ntt, baby, baby_keys, row, qs, ps, dnum, log_n) for row in pts]
    return rotate_sum_multi(inner, giant, giant_keys, qs, ps, dnum, log_n)


def rescale_coeff(x, moduli):
    """Divide-and-round by the last modulus: x (l, N) coefficient form over q_0..q_{l-1} ->
    (l - 1, N) with out_i = floor((X + q_last // 2) / q_last) mod q_i, X the CRT value in
    [0, Q).  RNS form: (x_i - ((x_last + h) mod q_last - h)) q_last^-1 mod q_i, h = q_last // 2."""
    moduli = [int(q) for q in moduli]
    x = np.asarray(x, dtype=object)
    ql = moduli[-1]
    h = ql // 2
    t = (x[-1] + h) % ql
    out = []
    for i, q in enumerate(moduli[:-1]):
        tmp = (t - h) % q
        out.append((x[i] - tmp) * pow(ql % q, -1, q) % q)
    return np.stack(out)


def rescale_exact(x, moduli):
    """The same through CRT big integers (test cross-check of rescale_coeff)."""
    moduli = [int(q) for q in moduli]
    Q = math.prod(moduli)
    x = np.asarray(x, dtype=object)
    X = 0
    for i, q in enumerate(moduli):
        hat = Q // q
        X = X + x[i] * (hat * pow(hat % q, -1, q))
    X = X % Q
    ql = moduli[-1]
    Y = (X + ql // 2) // ql
    return np.stack([Y % q for q in moduli[:-1]])


def rescale_ntt(x, moduli):
    """Rescale of an NTT-form (l, N) input: INTT, divide-and-round, NTT over the l - 1 limbs."""
    c = rns_ntt_inv(x, moduli)
    return rns_ntt_fwd(rescale_coeff(c, moduli), moduli[:-1])


# ---- the fused multiply -> relinearise -> rescale pipeline ----------------

def tensor_ntt(a, b, moduli):
    """a, b (2, L, N) NTT form -> (3, L, N): (a0 b0, a0 b1 + a1 b0, a1 b1) mod q per limb."""
    qs = _mods_col(moduli)
    a = np.asarray(a, dtype=object)
    b = np.asarray(b, dtype=object)
    return np.stack([a[0] * b[0] % qs, (a[0] * b[1] + a[1] * b[0]) % qs, a[1] * b[1] % qs])


def mul_relin(a, b, evk_b, evk_a, qs, ps, dnum, rescale: bool):
    """Relin(a x b) = (d0 + KS0(d2), d1 + KS1(d2)), NTT form; then optionally rescale_ntt."""
    d = tensor_ntt(a, b, qs)
    ks0, ks1 = keyswitch(d[2], evk_b, evk_a, qs, ps, dnum)
    col = _mods_col(qs)
    out = np.stack([(d[0] + ks0) % col, (d[1] + ks1) % col])
    if rescale:
        out = np.stack([rescale_ntt(out[0], qs), rescale_ntt(out[1], qs)])
    return out


# ---- sampling, keys, encryption (restating csrc/keygen.hip) -------------
# Counter-based Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
# SC'11 -- the Random123 construction), so each sample is a function of its coordinates.

_M32 = 0xFFFFFFFF
TAG = {"secret": 1, "pk_a": 2, "pk_e": 3, "ks_a": 0x100, "ks_e": 0x101, "enc_u": 32,
       "enc_e0": 33, "enc_e1": 34, "enc_a": 35, "enc_e": 36}


def philox4x32_10(c, k0, k1):
    x, y, z, w = c
    for _ in range(10):
        p0, p1 = 0xD2511F53 * x, 0xCD9E8D57 * z
        x, y, z, w = ((p1 >> 32) ^ y ^ k0) & _M32, p1 & _M32, ((p0 >> 32) ^ w ^ k1) & _M32, p0 & _M32
        k0, k1 = (k0 + 0x9E3779B9) & _M32, (k1 + 0xBB67AE85) & _M32
    return x, y, z, w


def sample(kind: str, seed: int, tag: int, poly: int, limbs, n: int):
    """(len(limbs), n) residues; limbs = [(ctx limb index, q)].  kind: uniform / ternary / error.
    Small distributions draw one integer per coefficient, shared by every limb."""
    k0, k1 = seed & _M32, (seed >> 32) & _M32
    out = np.zeros((len(limbs), n), dtype=object)
    if kind == "uniform":
        for r, (li, q) in enumerate(limbs):
            for c in range(n):
                x, y, z, w = philox4x32_10((c, li, poly, tag), k0, k1)
                lo, hi = (y << 32) | x, (w << 32) | z
                out[r, c] = (hi * q + ((lo * q) >> 64)) >> 64
        return out
    vals = []
    for c in range(n):
        x, y, _, _ = philox4x32_10((c, _M32, poly, tag), k0, k1)
        if kind == "ternary":
            vals.append(x % 3 - 1)
        else:
            bits = (y << 32) | x
            vals.append(bin(bits & 0x1FFFFF).count("1") - bin((bits >> 21) & 0x1FFFFF).count("1"))
    for r, (_, q) in enumerate(limbs):
        out[r] = [v % q for v in vals]
    return out


def keygen_secret(seed, allm, log_n):
    n = 1 << log_n
    s = sample("ternary", seed, TAG["secret"], 0, list(enumerate(allm)), n)
    return rns_ntt_fwd(s, allm)


def keygen_public(seed, sk_ntt, qs, log_n):
    n = 1 << log_n
    lim = list(enumerate(qs))
    a = sample("uniform", seed, TAG["pk_a"], 0, lim, n)
    e = rns_ntt_fwd(sample("error", seed, TAG["pk_e"], 0, lim, n), qs)
    col = _mods_col(qs)
    return np.stack([(e - a * np.asarray(sk_ntt)[:len(qs)]) % col, a])


def keygen_switch(seed, sk_ntt, s_from_ntt, qs, ps, dnum, log_n):
    """[2][dnum][L + K][N]: evk_j = (-a_j s + e_j + P g_j s_from, a_j) (same gadget as gen_relin_key)."""
    n = 1 << log_n
    qs = [int(q) for q in qs]
    ps = [int(p) for p in ps]
    allm = qs + ps
    lim = list(enumerate(allm))
    col = _mods_col(allm)
    P = math.prod(ps)
    kb, ka = [], []
    for j, (lo, hi) in enumerate(digit_ranges(len(qs), dnum)):
        a = sample("uniform", seed, TAG["ks_a"] + 2 * j, 0, lim, n)
        e = rns_ntt_fwd(sample("error", seed, TAG["ks_e"] + 2 * j, 0, lim, n), allm)
        b = (e - a * np.asarray(sk_ntt)) % col
        for i in range(lo, hi):
            b[i] = (b[i] + (P % qs[i]) * np.asarray(s_from_ntt)[i]) % qs[i]
        kb.append(b)
        ka.append(a)
    return np.stack([np.stack(kb), np.stack(ka)])


def encrypt(seed, pt_ntt, pk, qs, log_n):
    n = 1 << log_n
    lim = list(enumerate(qs))
    col = _mods_col(qs)
    u = rns_ntt_fwd(sample("ternary", seed, TAG["enc_u"], 0, lim, n), qs)
    e0 = rns_ntt_fwd(sample("error", seed, TAG["enc_e0"], 0, lim, n), qs)
    e1 = rns_ntt_fwd(sample("error", seed, TAG["enc_e1"], 0, lim, n), qs)
    pk = np.asarray(pk, dtype=object)
    return np.stack([(e0 + pk[0] * u + np.asarray(pt_ntt, dtype=object)) % col,
                     (e1 + pk[1] * u) % col])


def encrypt_sk(seed, pt_ntt, sk_ntt, qs, log_n):
    n = 1 << log_n
    lim = list(enumerate(qs))
    col = _mods_col(qs)
    a = sample("uniform", seed, TAG["enc_a"], 0, lim, n)
    e = rns_ntt_fwd(sample("error", seed, TAG["enc_e"], 0, lim, n), qs)
    return np.stack([(e - a * np.asarray(sk_ntt)[:len(qs)] + np.asarray(pt_ntt, dtype=object)) % col,
                     a])


def decrypt(ct, sk_ntt, qs):
    col = _mods_col(qs)
    ct = np.asarray(ct, dtype=object)
    return (ct[0] + ct[1] * np.asarray(sk_ntt, dtype=object)[:len(qs)]) % col
