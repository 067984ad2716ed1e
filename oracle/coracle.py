"""ctypes binding of oracle/_build/liboracle.so, the exact C restatement (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
Arrays are numpy uint64, C-contiguous, layout [poly][limb][N].
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_u64p = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32, u64, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.oracle_gen_moduli.argtypes = [u32, u32, u32, u32, _u64p]
        L.oracle_gen_moduli.restype = i32
        L.oracle_psi.argtypes = [u64, u32]
        L.oracle_psi.restype = u64
        L.oracle_primitive_root.argtypes = [u64]
        L.oracle_primitive_root.restype = u64
        for f in (L.oracle_ntt_fwd, L.oracle_ntt_inv):
            f.argtypes = [_u64p, u64, u32, _u64p, u32]
            f.restype = None
        L.oracle_vec_op.argtypes = [i32, _u64p, _u64p, _u64p, u64, u64, _u64p, u64]
        L.oracle_vec_op.restype = None
        L.oracle_hommult.argtypes = [_u64p, _u64p, _u64p, u64, u32, _u64p, u32]
        L.oracle_hommult.restype = None
        L.oracle_baseconv.argtypes = [_u64p, _u64p, u64, _u64p, u32, _u64p, u32]
        L.oracle_baseconv.restype = None
        L.oracle_keyswitch.argtypes = [_u64p, _u64p, _u64p, _u64p, _u64p, u32, _u64p, u32, _u64p,
                                       u32, u32]
        L.oracle_keyswitch.restype = None
        _u32p = ctypes.POINTER(ctypes.c_uint32)
        L.oracle_rotate_sum_hoisted.argtypes = [_u64p, _u64p, _u32p, u32, _u64p, _u64p, _u64p, u32,
                                                _u64p, u32, _u64p, u32, u32]
        L.oracle_rotate_sum_hoisted.restype = None
        for f in (L.port_ntt_fwd, L.port_ntt_inv):
            f.argtypes = [_u64p, u64, u32, _u64p, u32]
            f.restype = None
        L.port_hommult.argtypes = [_u64p, _u64p, _u64p, u64, u32, _u64p, u32]
        L.port_hommult.restype = None
        L.port_keyswitch.argtypes = [_u64p, _u64p, _u64p, _u64p, _u64p, u64, u32, _u64p, u32,
                                     _u64p, u32, u32]
        L.port_keyswitch.restype = None
        L.port_vec_op.argtypes = [i32, _u64p, _u64p, _u64p, u64, u64, _u64p]
        L.port_vec_op.restype = None
        _lib = L
    return _lib


def _p(x: np.ndarray):
    assert x.dtype == np.uint64 and x.flags.c_contiguous
    return x.ctypes.data_as(_u64p)


def _u64(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint64))


def gen_moduli(log_n: int, count: int, bits: int = 60, skip: int = 0) -> np.ndarray:
    out = np.zeros(count, dtype=np.uint64)
    if lib().oracle_gen_moduli(log_n, count, bits, skip, _p(out)) != 0:
        raise ValueError("not enough NTT primes")
    return out


def psi(q: int, log_n: int) -> int:
    return int(lib().oracle_psi(int(q), log_n))


def ntt_fwd(x, moduli) -> np.ndarray:
    """x: [..., L, N] -> new array, forward negacyclic NTT per limb."""
    x = _u64(x).copy()
    m = _u64(moduli)
    L, n = x.shape[-2], x.shape[-1]
    assert m.size == L
    lib().oracle_ntt_fwd(_p(x), x.size // (L * n), n.bit_length() - 1, _p(m), L)
    return x


def ntt_inv(x, moduli) -> np.ndarray:
    x = _u64(x).copy()
    m = _u64(moduli)
    L, n = x.shape[-2], x.shape[-1]
    assert m.size == L
    lib().oracle_ntt_inv(_p(x), x.size // (L * n), n.bit_length() - 1, _p(m), L)
    return x


def vec_op(op: str, a, b, mods_per_row) -> np.ndarray:
    """Exact (a op b) mod q on a 2-D view; q = mods_per_row[row] (length 1 = scalar)."""
    a = _u64(a)
    b = _u64(b)
    assert a.shape == b.shape
    a2 = a.reshape(-1, a.shape[-1]) if a.ndim > 1 else a.reshape(1, -1)
    b2 = b.reshape(a2.shape)
    m = _u64(mods_per_row).reshape(-1)
    out = np.empty_like(a2)
    stride = 0 if m.size == 1 else 1
    assert stride == 0 or m.size == a2.shape[0]
    lib().oracle_vec_op({"add": 0, "sub": 1, "mul": 2}[op], _p(out), _p(a2), _p(b2), a2.shape[0],
                        a2.shape[1], _p(m), stride)
    return out.reshape(a.shape)


def hommult(a, b, moduli) -> np.ndarray:
    """a, b: [batch, 2, L, N] (or [2, L, N]) coefficient form -> [batch, 3, L, N]."""
    a = _u64(a)
    b = _u64(b)
    squeeze = a.ndim == 3
    if squeeze:
        a, b = a[None], b[None]
    B, _, L, n = a.shape
    d = np.empty((B, 3, L, n), dtype=np.uint64)
    m = _u64(moduli)
    lib().oracle_hommult(_p(d), _p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), B,
                         n.bit_length() - 1, _p(m), L)
    return d[0] if squeeze else d


# -- the tuned CPU port (oracle/fhe_cpu_port.c): bench.py's cpu_baseline, checked against the
# exact functions above by tests/test_oracle.py

def port_ntt(x, moduli, forward=True) -> np.ndarray:
    """In-place style on a copy: the port's lazy Harvey NTT (forward) or GS inverse."""
    x = _u64(x).copy()
    m = _u64(moduli)
    L, n = x.shape[-2], x.shape[-1]
    assert m.size == L
    fn = lib().port_ntt_fwd if forward else lib().port_ntt_inv
    fn(_p(x), x.size // (L * n), n.bit_length() - 1, _p(m), L)
    return x


def port_vec_op(op: str, a, b, mods_per_row, out=None) -> np.ndarray:
    """The tuned port's vec_add / vec_sub / vec_mul on canonical [rows, cols] residues, row r
    modulo mods_per_row[r] (bench.py --workload vec cpu_baseline)."""
    a2 = np.ascontiguousarray(_u64(a).reshape(-1, a.shape[-1]))
    b2 = np.ascontiguousarray(_u64(b).reshape(a2.shape))
    m = np.ascontiguousarray(_u64(mods_per_row).reshape(-1))
    assert m.size == a2.shape[0]
    o = np.empty_like(a2) if out is None else out.reshape(a2.shape)
    lib().port_vec_op({"add": 0, "sub": 1, "mul": 2}[op], _p(o), _p(a2), _p(b2), a2.shape[0],
                      a2.shape[1], _p(m))
    return o.reshape(a.shape)


def port_hommult_into(d, a, b, moduli) -> None:
    """d[B, 3, L, N] = HomMult(a, b) by the tuned port; no allocation (the timed call)."""
    B, _, L, n = a.shape
    lib().port_hommult(_p(d), _p(a), _p(b), B, n.bit_length() - 1, _p(_u64(moduli)), L)


def port_hommult(a, b, moduli) -> np.ndarray:
    a = _u64(a)
    b = _u64(b)
    squeeze = a.ndim == 3
    if squeeze:
        a, b = a[None], b[None]
    d = np.empty((a.shape[0], 3) + a.shape[2:], dtype=np.uint64)
    port_hommult_into(d, np.ascontiguousarray(a), np.ascontiguousarray(b), moduli)
    return d[0] if squeeze else d


def baseconv(x, src, dst) -> np.ndarray:
    x = _u64(x)
    src = _u64(src)
    dst = _u64(dst)
    n = x.shape[-1]
    out = np.empty((dst.size, n), dtype=np.uint64)
    lib().oracle_baseconv(_p(out), _p(x), n, _p(src), src.size, _p(dst), dst.size)
    return out


def port_keyswitch(d2, evk_b, evk_a, qs, ps, dnum):
    """The tuned CPU port's key-switch (oracle/fhe_cpu_port.c): d2 [batch][L][N] -> (ks0, ks1)."""
    d2 = _u64(d2)
    B, L, n = d2.shape
    qs = _u64(qs)
    ps = _u64(ps)
    ks0 = np.empty((B, L, n), dtype=np.uint64)
    ks1 = np.empty((B, L, n), dtype=np.uint64)
    lib().port_keyswitch(_p(ks0), _p(ks1), _p(d2), _p(_u64(evk_b)), _p(_u64(evk_a)), B,
                         n.bit_length() - 1, _p(qs), qs.size, _p(ps), ps.size, dnum)
    return ks0, ks1


def keyswitch(d2, evk_b, evk_a, qs, ps, dnum):
    d2 = _u64(d2)
    L, n = d2.shape
    qs = _u64(qs)
    ps = _u64(ps)
    ks0 = np.empty((L, n), dtype=np.uint64)
    ks1 = np.empty((L, n), dtype=np.uint64)
    lib().oracle_keyswitch(_p(ks0), _p(ks1), _p(d2), _p(_u64(evk_b)), _p(_u64(evk_a)),
                           n.bit_length() - 1, _p(qs), qs.size, _p(ps), ps.size, dnum)
    return ks0, ks1


def rotate_sum_hoisted(ct, galois, keys_b, keys_a, pts, qs, ps, dnum):
    """sum_r pts[r] * rot_{galois[r]}(ct), one ModUp and one ModDown (double hoisting; restates
    pyoracle.rotate_sum_hoisted).  ct [2][L][N] NTT form; keys_* [count][dnum][L+K][N] (any
    values where galois[r] == 1); pts [count][L+K][N].  Returns [2][L][N]."""
    ct = _u64(ct)
    _, L, n = ct.shape
    g = np.ascontiguousarray(np.asarray(galois, dtype=np.uint32))
    qs = _u64(qs)
    ps = _u64(ps)
    out = np.empty((2, L, n), dtype=np.uint64)
    lib().oracle_rotate_sum_hoisted(_p(out), _p(ct), g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                    g.size, _p(_u64(keys_b)), _p(_u64(keys_a)), _p(_u64(pts)),
                                    n.bit_length() - 1, _p(qs), qs.size, _p(ps), ps.size, dnum)
    return out
