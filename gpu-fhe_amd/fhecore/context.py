"""Context / Ciphertext / Evaluator: the host-side API over libfhecore.

SURVEY.md §8b asks for a Context/Ciphertext/Evaluator layer above the C ABI (the reference has
no such layer: it passes ``MOD`` per call, /root/reference/arithmetic.py:3-13).  Device memory,
streams and multi-GPU collectives are PyTorch-ROCm plumbing; every arithmetic operation is a
libfhecore call into hand-written gfx950 kernels.  Tensors are int64 views of the uint64
residues, layout [..., limb, N], on a HIP device.
"""
from __future__ import annotations

import ctypes
import secrets
import threading
from functools import lru_cache

import numpy as np

from . import _capi
from ._capi import check, load

try:  # torch is the device-memory / stream provider
    import torch
except ImportError:  # pragma: no cover - the image always has torch
    torch = None


# ----------------------------------------------------------------------------- parameters

@lru_cache(maxsize=None)
def _gen_moduli_cached(log_n: int, count: int, bits: int, skip: int) -> tuple:
    out = (ctypes.c_uint64 * count)()
    check(load().fhe_gen_moduli(log_n, count, bits, skip, out), "fhe_gen_moduli")
    return tuple(int(v) for v in out)


def gen_moduli(log_n: int, count: int, bits: int = 60, skip: int = 0) -> list:
    """SURVEY.md §8a' modulus chain: the largest primes < 2^bits, q = 1 mod 2N, descending."""
    return list(_gen_moduli_cached(log_n, count, bits, skip))


def default_params(log_n: int, L: int, K: int = 0):
    """(Q-moduli, P-moduli): L + K consecutive primes of the §8a' chain."""
    m = gen_moduli(log_n, L + K)
    return m[:L], m[L:]


# ----------------------------------------------------------------------------- device helpers

def _nonce(seed):
    """The Philox seed of one keygen/encryption call: a fresh CSPRNG draw unless given."""
    return secrets.randbits(64) if seed is None else int(seed)


def _require_device():
    if torch is None or not torch.cuda.is_available():
        raise _capi.FheError("fhecore needs a HIP device (torch.cuda.is_available() is False); "
                             "there is no CPU fallback")


def to_device(x, device=None):
    """numpy uint64/int64 (or any integer array with values in [0, 2^64)) -> int64 device tensor."""
    _require_device()
    if isinstance(x, torch.Tensor):
        return x.to(device or "cuda").contiguous()
    a = np.ascontiguousarray(np.asarray(x, dtype=np.uint64))
    if not a.flags.writeable:
        a = a.copy()
    return torch.from_numpy(a.view(np.int64)).to(device or "cuda")


def to_host(t) -> np.ndarray:
    """int64 device tensor -> numpy uint64 array."""
    return t.detach().to("cpu").contiguous().numpy().view(np.uint64)


def _ptr(t) -> int:
    return ctypes.c_void_p(t.data_ptr() if t is not None else None)


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check_tensor(t, what, shape_tail=None):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{what}: expected a HIP device tensor")
    if t.dtype not in (torch.int64, torch.uint64):
        raise TypeError(f"{what}: expected int64/uint64 residues, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")
    if shape_tail is not None and tuple(t.shape[-len(shape_tail):]) != tuple(shape_tail):
        raise ValueError(f"{what}: trailing shape {tuple(t.shape)} != (..., {shape_tail})")


def _check_out(out, ref, shape, what):
    """A caller-supplied output: its raw pointer goes straight to a kernel, so it must be a
    contiguous int64/uint64 HIP tensor of exactly `shape` on the device of `ref` (a CPU tensor or
    one on another GPU would be written through an invalid device address)."""
    _check_tensor(out, what)
    if out.device != ref.device:
        raise ValueError(f"{what}: on {out.device}, the inputs are on {ref.device}")
    if tuple(out.shape) != tuple(shape):
        raise ValueError(f"{what}: shape {tuple(out.shape)} != {tuple(shape)}")
    return out


# ----------------------------------------------------------------------------- context

# Tensors allocated by this module while a Graph is capturing: the captured kernels keep their
# addresses, so the Graph holds a reference to each (else the caching allocator would hand their
# memory to other tensors while replays still write it).
_CAPTURE = threading.local()


def _keep(t):
    keep = getattr(_CAPTURE, "keep", None)
    if keep is not None:
        keep.append(t)
    return t


def _empty(*args, **kw):
    return _keep(torch.empty(*args, **kw))


def _empty_like(*args, **kw):
    return _keep(torch.empty_like(*args, **kw))


class Context:
    """RNS-CKKS-style parameter context on one HIP device (wraps ``fhe_ctx``).

    moduli: Q-primes (L of them); special: P-primes (K, for key-switching); dnum gadget digits.
    Defaults follow SURVEY.md §8a' (``default_params``).
    """

    def __init__(self, log_n: int, moduli=None, special=None, dnum: int = 1, L: int = None,
                 K: int = 0, device: int = None):
        _require_device()
        lib = load()
        if moduli is None:
            if L is None:
                raise ValueError("give moduli or L")
            moduli, dflt_special = default_params(log_n, L, K)
            if special is None:
                special = dflt_special
        special = list(special or [])
        moduli = [int(q) for q in moduli]
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.log_n = int(log_n)
        self.n = 1 << self.log_n
        self.L, self.K = len(moduli), len(special)
        self.dnum = int(dnum) if self.K else 0
        self.alpha = -(-self.L // self.dnum) if self.K else 0
        self._ptr = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.fhe_ctx_create(ctypes.byref(self._ptr), self.log_n, _capi.u64_array(moduli),
                                     self.L, _capi.u64_array(special) if special else None,
                                     self.K, self.dnum, self.device), "fhe_ctx_create")
        mods = (ctypes.c_uint64 * (self.L + self.K))()
        psi = (ctypes.c_uint64 * (self.L + self.K))()
        check(lib.fhe_ctx_moduli(self._ptr, mods, psi), "fhe_ctx_moduli")
        self.moduli = [int(v) for v in mods][: self.L]
        self.special = [int(v) for v in mods][self.L:]
        self.psi = [int(v) for v in psi]

    # -- lifetime
    def close(self):
        if getattr(self, "_ptr", None) and self._ptr.value:
            load().fhe_ctx_destroy(self._ptr)
            self._ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._ptr

    @property
    def all_moduli(self):
        return self.moduli + self.special

    def _dev(self):
        return torch.device("cuda", self.device)

    def empty(self, *shape):
        return _empty(shape, dtype=torch.int64, device=self._dev())

    def workspace(self, nbytes: int):
        return _empty((max(int(nbytes), 8) + 7) // 8, dtype=torch.int64, device=self._dev())

    # -- NTT (replaces NTT / iNTT, arithmetic.py:15-19)
    def ntt_(self, t, limb0: int = 0):
        """In-place forward NTT of a [..., nlimbs, N] tensor (limb l uses modulus limb0 + l)."""
        return self._ntt(t, limb0, True)

    def intt_(self, t, limb0: int = 0):
        return self._ntt(t, limb0, False)

    def ntt(self, t, out=None, limb0: int = 0):
        """Out-of-place forward NTT: returns out = NTT(t) (a new tensor unless `out` is given);
        t is left untouched and nothing is copied (the first pass reads t, writes out)."""
        return self._ntt_to(t, out, limb0, True)

    def intt(self, t, out=None, limb0: int = 0):
        return self._ntt_to(t, out, limb0, False)

    def _ntt_to(self, t, out, limb0, fwd):
        _check_tensor(t, "ntt", (self.n,))
        if out is None:
            out = _empty_like(t)
        else:
            _check_out(out, t, t.shape, "ntt: out")
        nl = t.shape[-2] if t.dim() >= 2 else 1
        polys = t.numel() // (nl * self.n)
        fn = load().fhe_ntt_fwd_to if fwd else load().fhe_ntt_inv_to
        with torch.cuda.device(self.device):
            check(fn(self._ptr, _ptr(out), _ptr(t), polys, limb0, nl, _stream(t)), fn.__name__)
        return out

    def _ntt(self, t, limb0, fwd):
        _check_tensor(t, "ntt", (self.n,))
        nl = t.shape[-2] if t.dim() >= 2 else 1
        polys = t.numel() // (nl * self.n)
        fn = load().fhe_ntt_fwd if fwd else load().fhe_ntt_inv
        with torch.cuda.device(self.device):
            check(fn(self._ptr, _ptr(t), polys, limb0, nl, _stream(t)), fn.__name__)
        return t

    # -- coefficient-wise ops (replace vec_add / vec_sub / vec_mul, arithmetic.py:3-13)
    def vec(self, op: str, a, b, out=None, limb0: int = 0):
        _check_tensor(a, op, (self.n,))
        _check_tensor(b, op, (self.n,))
        if a.shape != b.shape:
            raise AssertionError("a.shape != b.shape")  # the reference asserts (arithmetic.py:4)
        out = _empty_like(a) if out is None else _check_out(out, a, a.shape, op + ": out")
        nl = a.shape[-2] if a.dim() >= 2 else 1
        polys = a.numel() // (nl * self.n)
        fn = {"add": load().fhe_vec_add, "sub": load().fhe_vec_sub, "mul": load().fhe_vec_mul}[op]
        with torch.cuda.device(self.device):
            check(fn(self._ptr, _ptr(out), _ptr(a), _ptr(b), polys, limb0, nl, _stream(a)),
                  fn.__name__)
        return out

    # -- HomMult (SURVEY.md §8a')
    def hommult(self, a, b, out=None, limb0: int = 0, workspace=None):
        """a, b: [batch, 2, nlimbs, N] (or [2, nlimbs, N]) coefficient form -> [batch, 3, nlimbs, N]."""
        _check_tensor(a, "hommult", (self.n,))
        _check_tensor(b, "hommult", (self.n,))
        if a.shape != b.shape or a.shape[-3] != 2:
            raise ValueError("hommult: a, b must both be [batch, 2, nlimbs, N]")
        squeeze = a.dim() == 3
        batch = 1 if squeeze else a.shape[0]
        nl = a.shape[-2]
        shape = (3, nl, self.n) if squeeze else (batch, 3, nl, self.n)
        out = self.empty(*shape) if out is None else _check_out(out, a, shape, "hommult: out")
        lib = load()
        ws = workspace
        if ws is None:
            ws = self.workspace(lib.fhe_hommult_workspace(self._ptr, batch, nl))
        with torch.cuda.device(self.device):
            check(lib.fhe_hommult(self._ptr, _ptr(out), _ptr(a), _ptr(b), batch, limb0, nl,
                                  _ptr(ws), _stream(a)), "fhe_hommult")
        return out

    # -- base conversion / key-switch (SURVEY.md §8a')
    def baseconv(self, x, s0: int, t0: int, T: int):
        _check_tensor(x, "baseconv", (self.n,))
        S = x.shape[-2]
        out = self.empty(T, self.n)
        with torch.cuda.device(self.device):
            check(load().fhe_baseconv(self._ptr, _ptr(out), _ptr(x), s0, S, t0, T, _stream(x)),
                  "fhe_baseconv")
        return out

    def keyswitch(self, d2, evk_b, evk_a, workspace=None, out=None):
        """d2 [L, N] or [batch, L, N] NTT form; evk_b/evk_a [dnum, L + K, N] NTT form (one key for the
        whole batch) -> (ks0, ks1) shaped like d2, NTT form.
        out = (ks0, ks1): caller-provided outputs shaped like d2 (either may be d2 itself, in place;
        any other overlap with d2 or between them raises FheError, fhecore.h)."""
        for t, nm in ((d2, "d2"), (evk_b, "evk_b"), (evk_a, "evk_a")):
            _check_tensor(t, nm, (self.n,))
        if tuple(evk_b.shape) != (self.dnum, self.L + self.K, self.n) or evk_a.shape != evk_b.shape:
            raise ValueError("keyswitch: evk must be [dnum, L + K, N]")
        if d2.shape[-2] != self.L:
            raise ValueError("keyswitch: d2 must be [..., L, N]")
        batch = d2.numel() // (self.L * self.n)
        if out is None:
            ks0, ks1 = _empty_like(d2), _empty_like(d2)
        else:
            ks0 = _check_out(out[0], d2, d2.shape, "keyswitch: ks0")
            ks1 = _check_out(out[1], d2, d2.shape, "keyswitch: ks1")
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_keyswitch_workspace(self._ptr, self.L,
                                        lib.fhe_keyswitch_pass_batch(self._ptr, batch)))
        with torch.cuda.device(self.device):
            check(lib.fhe_keyswitch(self._ptr, _ptr(ks0), _ptr(ks1), _ptr(d2), _ptr(evk_b),
                                    _ptr(evk_a), batch, _ptr(ws), _stream(d2)), "fhe_keyswitch")
        return ks0, ks1

    # ---- rescale and rotation -------------------------------------
    def galois_elt(self, step: int) -> int:
        """Galois element of a slot rotation by `step` (5^step mod 2N; negative steps invert)."""
        two_n = 2 * self.n
        return pow(5, step, two_n) if step >= 0 else pow(pow(5, -step, two_n), -1, two_n)

    def rescale(self, x, ntt_form: bool = True, workspace=None):
        """Divide-and-round by the last modulus: x [..., l, N] over Q-limbs 0..l-1 (2 <= l <= L)
        -> [..., l - 1, N], same form (oracle: pyoracle.rescale_ntt/_coeff)."""
        _check_tensor(x, "x", (self.n,))
        nl = x.shape[-2]
        polys = x.numel() // (nl * self.n)
        out = _empty(*x.shape[:-2], nl - 1, self.n, dtype=x.dtype, device=x.device)
        lib = load()
        ws = None
        if ntt_form:
            ws = workspace if workspace is not None else self.workspace(
                lib.fhe_rescale_workspace(self._ptr, polys, nl))
        with torch.cuda.device(self.device):
            check(lib.fhe_rescale(self._ptr, _ptr(out), _ptr(x), polys, nl, int(ntt_form),
                                  _ptr(ws), _stream(x)), "fhe_rescale")
        return out

    def automorphism(self, x, galois_elt: int, ntt_form: bool = True, limb0: int = 0):
        """sigma_k(a)(X) = a(X^k) on x [..., nlimbs, N] over limbs [limb0, limb0 + nlimbs)."""
        _check_tensor(x, "x", (self.n,))
        nl = x.shape[-2]
        polys = x.numel() // (nl * self.n)
        out = _empty_like(x)
        with torch.cuda.device(self.device):
            check(load().fhe_automorphism(self._ptr, _ptr(out), _ptr(x), polys, limb0, nl,
                                          galois_elt, int(ntt_form), _stream(x)), "fhe_automorphism")
        return out

    def rotate(self, ct, galois_elt: int, rot_b, rot_a, workspace=None, out=None):
        """ct [..., 2, L, N] NTT form -> (sigma c0 + KS0(sigma c1), KS1(sigma c1)) with the
        key-switch key rot_b/rot_a [dnum, L + K, N] from sigma_k(s) to s.  out: a caller-provided
        output shaped like ct, which must not overlap ct (FheError otherwise, fhecore.h)."""
        _check_tensor(ct, "ct", (2, self.L, self.n))
        if tuple(rot_b.shape) != (self.dnum, self.L + self.K, self.n) or rot_a.shape != rot_b.shape:
            raise ValueError("rotate: key must be [dnum, L + K, N]")
        batch = ct.numel() // (2 * self.L * self.n)
        out = _empty_like(ct) if out is None else _check_out(out, ct, ct.shape, "rotate: out")
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_rotate_workspace(self._ptr, lib.fhe_keyswitch_pass_batch(self._ptr, batch)))
        with torch.cuda.device(self.device):
            check(lib.fhe_rotate(self._ptr, _ptr(out), _ptr(ct), galois_elt, _ptr(rot_b),
                                 _ptr(rot_a), batch, _ptr(ws), _stream(ct)), "fhe_rotate")
        return out

    def rotate_hoisted(self, ct, galois_elts, rot_keys, workspace=None, out=None):
        """Several rotations of the same ct [..., 2, L, N] (NTT form) sharing one ModUp
        (fhe_rotate_hoisted): galois_elts[r] with rot_keys[r] = (rot_b, rot_a), each
        [dnum, L + K, N].  Returns [count, ..., 2, L, N]; output r decrypts to sigma_r(m)."""
        _check_tensor(ct, "ct", (2, self.L, self.n))
        elts = [int(g) for g in galois_elts]
        if len(rot_keys) != len(elts):
            raise ValueError("rotate_hoisted: one key per Galois element")
        for kb, ka in rot_keys:
            if tuple(kb.shape) != (self.dnum, self.L + self.K, self.n) or ka.shape != kb.shape:
                raise ValueError("rotate_hoisted: keys must be [dnum, L + K, N]")
            if kb.device != ct.device or ka.device != ct.device or not (
                    kb.is_contiguous() and ka.is_contiguous()):
                raise ValueError("rotate_hoisted: keys must be contiguous on the ct's device")
        batch = ct.numel() // (2 * self.L * self.n)
        count = len(elts)
        if out is None:
            out = _empty(count, *ct.shape, dtype=ct.dtype, device=ct.device)
        else:
            _check_out(out, ct, (count, *ct.shape), "rotate_hoisted: out")
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_rotate_hoisted_workspace(self._ptr, batch))
        g_arr = (ctypes.c_uint32 * max(count, 1))(*elts)
        b_arr = (ctypes.c_void_p * max(count, 1))(*[kb.data_ptr() for kb, _ in rot_keys])
        a_arr = (ctypes.c_void_p * max(count, 1))(*[ka.data_ptr() for _, ka in rot_keys])
        with torch.cuda.device(self.device):
            check(lib.fhe_rotate_hoisted(self._ptr, _ptr(out), _ptr(ct), g_arr, b_arr, a_arr,
                                         count, batch, _ptr(ws), _stream(ct)),
                  "fhe_rotate_hoisted")
        return out

    def rotate_sum_hoisted(self, ct, galois_elts, rot_keys, pts, workspace=None, out=None):
        """sum_r pts[r] * rot_{galois_elts[r]}(ct) for ct [..., 2, L, N] (NTT form) with one ModUp
        and one ModDown (fhe_rotate_sum_hoisted, double hoisting): rot_keys[r] = (rot_b, rot_a)
        [dnum, L + K, N], or None for the unrotated term (Galois element 1); pts[r] [L + K, N]
        NTT form over Q u P.  Returns [..., 2, L, N]."""
        _check_tensor(ct, "ct", (2, self.L, self.n))
        elts = [int(g) for g in galois_elts]
        count = len(elts)
        if len(rot_keys) != count or len(pts) != count:
            raise ValueError("rotate_sum_hoisted: one key (or None) and one plaintext per term")
        for g, key, pt in zip(elts, rot_keys, pts):
            if tuple(pt.shape) != (self.L + self.K, self.n) or pt.device != ct.device or not \
                    pt.is_contiguous():
                raise ValueError("rotate_sum_hoisted: plaintexts must be contiguous [L + K, N] "
                                 "on the ct's device")
            if key is None:
                if g != 1:
                    raise ValueError("rotate_sum_hoisted: only Galois element 1 takes no key")
                continue
            kb, ka = key
            if tuple(kb.shape) != (self.dnum, self.L + self.K, self.n) or ka.shape != kb.shape:
                raise ValueError("rotate_sum_hoisted: keys must be [dnum, L + K, N]")
            if kb.device != ct.device or ka.device != ct.device or not (
                    kb.is_contiguous() and ka.is_contiguous()):
                raise ValueError("rotate_sum_hoisted: keys must be contiguous on the ct's device")
        batch = ct.numel() // (2 * self.L * self.n)
        if out is None:
            out = _empty(*ct.shape, dtype=ct.dtype, device=ct.device)
        else:
            _check_out(out, ct, tuple(ct.shape), "rotate_sum_hoisted: out")
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_rotate_sum_hoisted_workspace(self._ptr, batch))
        n_arr = max(count, 1)
        g_arr = (ctypes.c_uint32 * n_arr)(*elts)
        b_arr = (ctypes.c_void_p * n_arr)(*[k[0].data_ptr() if k else None for k in rot_keys])
        a_arr = (ctypes.c_void_p * n_arr)(*[k[1].data_ptr() if k else None for k in rot_keys])
        p_arr = (ctypes.c_void_p * n_arr)(*[p.data_ptr() for p in pts])
        with torch.cuda.device(self.device):
            check(lib.fhe_rotate_sum_hoisted(self._ptr, _ptr(out), _ptr(ct), g_arr, b_arr, a_arr,
                                             p_arr, count, batch, _ptr(ws), _stream(ct)),
                  "fhe_rotate_sum_hoisted")
        return out

    def _rot_keys(self, elts, rot_keys, ct, who):
        """Host arrays of key pointers (None for the unrotated element 1), shapes checked."""
        if len(rot_keys) != len(elts):
            raise ValueError(f"{who}: one key (or None) per Galois element")
        for g, key in zip(elts, rot_keys):
            if key is None:
                if g != 1:
                    raise ValueError(f"{who}: only Galois element 1 takes no key")
                continue
            kb, ka = key
            if tuple(kb.shape) != (self.dnum, self.L + self.K, self.n) or ka.shape != kb.shape:
                raise ValueError(f"{who}: keys must be [dnum, L + K, N]")
            if kb.device != ct.device or ka.device != ct.device or not (
                    kb.is_contiguous() and ka.is_contiguous()):
                raise ValueError(f"{who}: keys must be contiguous on the ct's device")
        k = max(len(elts), 1)
        return ((ctypes.c_uint32 * k)(*elts),
                (ctypes.c_void_p * k)(*[kk[0].data_ptr() if kk else None for kk in rot_keys]),
                (ctypes.c_void_p * k)(*[kk[1].data_ptr() if kk else None for kk in rot_keys]))

    def _pts(self, pts, ct, who):
        for pt in pts:
            if tuple(pt.shape) != (self.L + self.K, self.n) or pt.device != ct.device or not \
                    pt.is_contiguous():
                raise ValueError(f"{who}: plaintexts must be contiguous [L + K, N] on the ct's "
                                 "device")
        return (ctypes.c_void_p * max(len(pts), 1))(*[p.data_ptr() for p in pts])

    def rotate_sum_multi(self, cts, galois_elts, rot_keys, workspace=None, out=None):
        """sum_r rot_{galois_elts[r]}(cts[r]) over different ciphertexts (each [..., 2, L, N], NTT
        form, one shape) with one ModDown (fhe_rotate_sum_multi, the giant-step sum of a BSGS
        linear transform); rot_keys[r] = (rot_b, rot_a) or None for Galois element 1."""
        if not cts:
            raise ValueError("rotate_sum_multi: at least one ciphertext")
        ct = cts[0]
        _check_tensor(ct, "ct", (2, self.L, self.n))
        for c in cts:
            if c.shape != ct.shape or c.device != ct.device or not c.is_contiguous():
                raise ValueError("rotate_sum_multi: ciphertexts of one shape, contiguous, on one "
                                 "device")
        elts = [int(g) for g in galois_elts]
        if len(cts) != len(elts):
            raise ValueError("rotate_sum_multi: one Galois element per ciphertext")
        g_arr, b_arr, a_arr = self._rot_keys(elts, rot_keys, ct, "rotate_sum_multi")
        batch = ct.numel() // (2 * self.L * self.n)
        if out is None:
            out = _empty(*ct.shape, dtype=ct.dtype, device=ct.device)
        else:
            _check_out(out, ct, tuple(ct.shape), "rotate_sum_multi: out")
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_rotate_sum_multi_workspace(self._ptr, len(cts), batch))
        c_arr = (ctypes.c_void_p * len(cts))(*[c.data_ptr() for c in cts])
        with torch.cuda.device(self.device):
            check(lib.fhe_rotate_sum_multi(self._ptr, _ptr(out), c_arr, g_arr, b_arr, a_arr,
                                           len(elts), batch, _ptr(ws), _stream(ct)),
                  "fhe_rotate_sum_multi")
        return out

    def linear_transform(self, ct, baby_elts, baby_keys, giant_elts, giant_keys, pts,
                         workspace=None, out=None):
        """Baby-step / giant-step plaintext-matrix product with both hoistings
        (fhe_linear_transform): sum_g rot_{giant[g]}(sum_b pts[g][b] rot_{baby[b]}(ct)) for
        ct [..., 2, L, N] NTT form; pts[g][b] [L + K, N] NTT form over Q u P."""
        _check_tensor(ct, "ct", (2, self.L, self.n))
        baby = [int(g) for g in baby_elts]
        giant = [int(g) for g in giant_elts]
        n1, n2 = len(baby), len(giant)
        if len(pts) != n2 or any(len(row) != n1 for row in pts):
            raise ValueError("linear_transform: pts must be n2 lists of n1 plaintexts")
        bg, bb, ba = self._rot_keys(baby, baby_keys, ct, "linear_transform")
        gg, gb, ga = self._rot_keys(giant, giant_keys, ct, "linear_transform")
        p_arr = self._pts([p for row in pts for p in row], ct, "linear_transform")
        batch = ct.numel() // (2 * self.L * self.n)
        if out is None:
            out = _empty(*ct.shape, dtype=ct.dtype, device=ct.device)
        else:
            _check_out(out, ct, tuple(ct.shape), "linear_transform: out")
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_linear_transform_workspace(self._ptr, n2, batch))
        with torch.cuda.device(self.device):
            check(lib.fhe_linear_transform(self._ptr, _ptr(out), _ptr(ct), n1, n2, bg, bb, ba, gg,
                                           gb, ga, p_arr, batch, _ptr(ws), _stream(ct)),
                  "fhe_linear_transform")
        return out

    # ---- sampling, keys, encryption --------------------------------
    # seed=None draws a fresh 64-bit nonce from the OS CSPRNG.  An explicit seed is for
    # reproducible tests: never reuse one per secret key (fhecore.h SECURITY note).
    KIND = {"uniform": 0, "ternary": 1, "error": 2}

    def sample(self, kind: str, polys: int, seed: int, tag: int, limb0: int = 0, nlimbs=None):
        """[polys, nlimbs, N] residues of a Philox4x32-10 draw (oracle: pyoracle.sample)."""
        nl = (self.L + self.K - limb0) if nlimbs is None else nlimbs
        out = _empty(polys, nl, self.n, dtype=torch.int64, device=self._dev())
        with torch.cuda.device(self.device):
            check(load().fhe_sample(self._ptr, _ptr(out), polys, limb0, nl, self.KIND[kind],
                                    seed, tag, _stream(out)), "fhe_sample")
        return out

    def keygen_secret(self, seed=None):
        """Ternary secret, NTT form over all L + K limbs: [L + K, N]."""
        seed = _nonce(seed)
        sk = _empty(self.L + self.K, self.n, dtype=torch.int64, device=self._dev())
        with torch.cuda.device(self.device):
            check(load().fhe_keygen_secret(self._ptr, _ptr(sk), seed, _stream(sk)), "fhe_keygen_secret")
        return sk

    def keygen_public(self, sk, seed=None):
        seed = _nonce(seed)
        pk = _empty(2, self.L, self.n, dtype=torch.int64, device=self._dev())
        with torch.cuda.device(self.device):
            check(load().fhe_keygen_public(self._ptr, _ptr(pk), _ptr(sk), seed, _stream(pk)),
                  "fhe_keygen_public")
        return pk

    def keygen_switch(self, sk, s_from, seed=None):
        """Key-switch key from s_from ([L + K, N] NTT form) to sk: (evk_b, evk_a), each
        [dnum, L + K, N] -- the operands of keyswitch / rotate / mul_relin."""
        seed = _nonce(seed)
        key = _empty(2, self.dnum, self.L + self.K, self.n, dtype=torch.int64, device=self._dev())
        with torch.cuda.device(self.device):
            check(load().fhe_keygen_switch(self._ptr, _ptr(key), _ptr(sk), _ptr(s_from), seed,
                                           _stream(key)), "fhe_keygen_switch")
        return key[0], key[1]

    def keygen_relin(self, sk, seed=None):
        """Relinearisation key: switches s^2 to s."""
        s2 = _empty_like(sk)
        lib = load()
        with torch.cuda.device(self.device):
            check(lib.fhe_vec_mul(self._ptr, _ptr(s2), _ptr(sk), _ptr(sk), 1, 0, self.L + self.K,
                                  _stream(sk)), "fhe_vec_mul")
        return self.keygen_switch(sk, s2, seed)

    def keygen_rotation(self, sk, galois_elt: int, seed=None):
        """Rotation key for Galois element k: switches sigma_k(s) to s."""
        return self.keygen_switch(sk, self.automorphism(sk, galois_elt, ntt_form=True), seed)

    def encrypt(self, pt, pk, seed=None):
        """Public-key encryption of an NTT-form plaintext [L, N] -> ciphertext [2, L, N]."""
        seed = _nonce(seed)
        ct = _empty(2, self.L, self.n, dtype=torch.int64, device=self._dev())
        with torch.cuda.device(self.device):
            ws = self.workspace(self.L * self.n * 8)  # a Graph keeps it (no internal workspace)
            check(load().fhe_encrypt(self._ptr, _ptr(ct), _ptr(pt), _ptr(pk), seed, _ptr(ws),
                                     _stream(ct)), "fhe_encrypt")
        return ct

    def encrypt_sk(self, pt, sk, seed=None):
        seed = _nonce(seed)
        ct = _empty(2, self.L, self.n, dtype=torch.int64, device=self._dev())
        with torch.cuda.device(self.device):
            check(load().fhe_encrypt_sk(self._ptr, _ptr(ct), _ptr(pt), _ptr(sk), seed, _stream(ct)),
                  "fhe_encrypt_sk")
        return ct

    def decrypt(self, ct, sk):
        """ct [..., 2, l, N] (any level l <= L) -> plaintext c0 + c1 s [..., l, N], NTT form."""
        _check_tensor(ct, "ct", (self.n,))
        nl = ct.shape[-2]
        batch = ct.numel() // (2 * nl * self.n)
        pt = _empty(*ct.shape[:-3], nl, self.n, dtype=ct.dtype, device=ct.device)
        with torch.cuda.device(self.device):
            check(load().fhe_decrypt(self._ptr, _ptr(pt), _ptr(ct), _ptr(sk), batch, nl, _stream(ct)),
                  "fhe_decrypt")
        return pt

    # ---- fused multiply -> relinearise -> rescale ------------------
    def mul_relin(self, a, b, evk_b, evk_a, rescale: bool = True, workspace=None, out=None):
        """a, b [..., 2, L, N] NTT form -> Relin(a x b) [..., 2, L, N] (rescale: [..., 2, L-1, N]),
        NTT form (oracle: pyoracle.mul_relin)."""
        _check_tensor(a, "a", (2, self.L, self.n))
        _check_tensor(b, "b", (2, self.L, self.n))
        if a.shape != b.shape:
            raise ValueError("mul_relin: a and b must have the same shape")
        if tuple(evk_b.shape) != (self.dnum, self.L + self.K, self.n) or evk_a.shape != evk_b.shape:
            raise ValueError("mul_relin: key must be [dnum, L + K, N]")
        batch = a.numel() // (2 * self.L * self.n)
        shape = (*a.shape[:-2], self.L - (1 if rescale else 0), self.n)
        if out is None:
            out = _empty(shape, dtype=a.dtype, device=a.device)
        else:
            _check_out(out, a, shape, "mul_relin: out")
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_mul_relin_workspace(self._ptr, lib.fhe_keyswitch_pass_batch(self._ptr, batch)))
        with torch.cuda.device(self.device):
            check(lib.fhe_mul_relin(self._ptr, _ptr(out), _ptr(a), _ptr(b), _ptr(evk_b),
                                    _ptr(evk_a), batch, int(rescale), _ptr(ws), _stream(a)),
                  "fhe_mul_relin")
        return out

    # ---- wire format ----------------------------------------------
    def serialize(self, x, ntt_form: bool, limb0: int = 0) -> bytes:
        """x [..., nlimbs, N] over limbs [limb0, limb0 + nlimbs) -> an FHEC v1 blob."""
        _check_tensor(x, "x", (self.n,))
        nl = x.shape[-2]
        polys = x.numel() // (nl * self.n)
        lib = load()
        size = lib.fhe_serialized_size(self._ptr, polys, nl)
        buf = ctypes.create_string_buffer(size)
        with torch.cuda.device(self.device):
            check(lib.fhe_serialize(self._ptr, _ptr(x), polys, limb0, nl, int(ntt_form), buf, size,
                                    _stream(x)), "fhe_serialize")
        return buf.raw

    def deserialize(self, blob: bytes):
        """FHEC v1 blob -> (tensor [polys, nlimbs, N] on this context's device, limb0, ntt_form).
        Rejects blobs for another N / other moduli, corrupted or out-of-range data."""
        lib = load()
        polys, limb0, nl, ntt = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
        check(lib.fhe_deserialize(self._ptr, blob, len(blob), None, 0, ctypes.byref(polys),
                                  ctypes.byref(limb0), ctypes.byref(nl), ctypes.byref(ntt), None),
              "fhe_deserialize")
        out = _empty(polys.value, nl.value, self.n, dtype=torch.int64, device=self._dev())
        with torch.cuda.device(self.device):
            check(lib.fhe_deserialize(self._ptr, blob, len(blob), _ptr(out), out.numel(), None, None,
                                      None, None, _stream(out)), "fhe_deserialize")
        return out, limb0.value, bool(ntt.value)

    def keyswitch_shard(self, c_all, d2_own, evk_b, evk_a, limb0: int, workspace=None,
                        ranks: int = None):
        """One rank's key-switch given the all-gathered coefficient-form d2.

        c_all: [batch, L, N] (ranks=None), or the rank-major all-gather output
        [ranks, batch, c, N], c = ceil(L / ranks) (fhecore.dist.gather_ranked: no reorder copy);
        d2_own [batch, nlimbs, N] NTT form of limbs [limb0, limb0 + nlimbs); evk_* [dnum,
        nlimbs + K, N].  Returns (ks0, ks1) shaped like d2_own."""
        for t, nm in ((c_all, "c_all"), (d2_own, "d2_own"), (evk_b, "evk_b"), (evk_a, "evk_a")):
            _check_tensor(t, nm, (self.n,))
        nl = d2_own.shape[-2]
        batch = d2_own.numel() // (nl * self.n)
        width = self.L if ranks is None else -(-self.L // ranks)
        if c_all.numel() != (ranks or 1) * batch * width * self.n:
            raise ValueError("keyswitch_shard: c_all must be [batch, L, N] or "
                             "[ranks, batch, ceil(L / ranks), N]")
        if tuple(evk_b.shape) != (self.dnum, nl + self.K, self.n) or evk_a.shape != evk_b.shape:
            raise ValueError("keyswitch_shard: evk slices must be [dnum, nlimbs + K, N]")
        ks0, ks1 = _empty_like(d2_own), _empty_like(d2_own)
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_keyswitch_workspace(self._ptr, nl, batch))
        with torch.cuda.device(self.device):
            if ranks is None:
                check(lib.fhe_keyswitch_shard(self._ptr, _ptr(ks0), _ptr(ks1), _ptr(c_all),
                                              _ptr(d2_own), _ptr(evk_b), _ptr(evk_a), limb0, nl,
                                              batch, _ptr(ws), _stream(d2_own)),
                      "fhe_keyswitch_shard")
            else:
                check(lib.fhe_keyswitch_shard_ranked(self._ptr, _ptr(ks0), _ptr(ks1), _ptr(c_all),
                                                     ranks, _ptr(d2_own), _ptr(evk_b), _ptr(evk_a),
                                                     limb0, nl, batch, _ptr(ws), _stream(d2_own)),
                      "fhe_keyswitch_shard_ranked")
        return ks0, ks1

    def keyswitch_dist(self, comm, d2_own, evk_b, evk_a, chunks: int = 0, workspace=None):
        """Limb-sharded key-switch over an RCCL communicator, all in libfhecore
        (fhe_keyswitch_dist): INTT of this rank's limbs, one ncclAllGather per chunk of the batch
        overlapping the previous chunk's work, then the local key-switch.  comm:
        fhecore.dist.RcclComm; d2_own [batch, nlimbs, N] NTT form of comm.shard(L)'s limbs;
        evk_* [dnum, nlimbs + K, N].  Returns (ks0, ks1) shaped like d2_own."""
        for t, nm in ((d2_own, "d2_own"), (evk_b, "evk_b"), (evk_a, "evk_a")):
            _check_tensor(t, nm, (self.n,))
            if t.device != self._dev():
                raise ValueError(f"keyswitch_dist: {nm} is on {t.device}, the context on "
                                 f"{self._dev()}")
        shard = comm.shard(self.L)
        nl = d2_own.shape[-2]
        if nl != shard.nlimbs:
            raise ValueError(f"keyswitch_dist: d2_own has {nl} limbs, this rank owns "
                             f"{shard.nlimbs}")
        batch = d2_own.numel() // (nl * self.n) if nl else d2_own.shape[0]
        if tuple(evk_b.shape) != (self.dnum, nl + self.K, self.n) or evk_a.shape != evk_b.shape:
            raise ValueError("keyswitch_dist: evk slices must be [dnum, nlimbs + K, N]")
        ks0, ks1 = _empty_like(d2_own), _empty_like(d2_own)
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_keyswitch_dist_workspace(self._ptr, comm.handle, batch, chunks))
        with torch.cuda.device(self.device):
            check(lib.fhe_keyswitch_dist(self._ptr, comm.handle, _ptr(ks0), _ptr(ks1),
                                         _ptr(d2_own), _ptr(evk_b), _ptr(evk_a), batch, chunks,
                                         _ptr(ws), _stream(d2_own)), "fhe_keyswitch_dist")
        return ks0, ks1

    def keyswitch_dist_loopback(self, d2_parts, evk_b_parts, evk_a_parts, chunks: int = 0,
                                workspace=None):
        """fhe_keyswitch_dist's G-rank plan run on this one device (fhe_keyswitch_dist_loopback):
        per-rank lists (rank r: d2 [batch, nlimbs_r, N] NTT form of LimbShard(L, G, r)'s limbs,
        evk slices [dnum, nlimbs_r + K, N]; None for ranks owning no limb).  Returns the per-rank
        (ks0, ks1) lists -- concatenated over the ranks they equal keyswitch()."""
        G = len(d2_parts)
        if not G or len(evk_b_parts) != G or len(evk_a_parts) != G:
            raise ValueError("keyswitch_dist_loopback: one entry per rank in every list")
        from .dist import LimbShard

        batch = None
        ks0, ks1 = [None] * G, [None] * G
        for r in range(G):
            sh = LimbShard(self.L, G, r)
            if sh.nlimbs == 0:
                continue
            d2 = d2_parts[r]
            _check_tensor(d2, f"d2[{r}]", (sh.nlimbs, self.n))
            for t, nm in ((d2, "d2"), (evk_b_parts[r], "evk_b"), (evk_a_parts[r], "evk_a")):
                if nm != "d2":
                    _check_tensor(t, f"{nm}[{r}]", (self.dnum, sh.nlimbs + self.K, self.n))
                # the C side launches on the context's device with these raw pointers
                if t.device != self._dev():
                    raise ValueError(f"keyswitch_dist_loopback: {nm}[{r}] is on {t.device}, "
                                     f"the context on {self._dev()}")
            b = d2.numel() // (sh.nlimbs * self.n)
            if batch is not None and b != batch:
                raise ValueError("keyswitch_dist_loopback: every rank needs the same batch")
            batch = b
            ks0[r], ks1[r] = _empty_like(d2), _empty_like(d2)
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_keyswitch_dist_loopback_workspace(self._ptr, G, batch, chunks))
        arr = lambda ts: (ctypes.c_void_p * G)(*[t.data_ptr() if t is not None else None  # noqa: E731
                                                  for t in ts])
        ref = next(t for t in d2_parts if t is not None)
        with torch.cuda.device(self.device):
            check(lib.fhe_keyswitch_dist_loopback(self._ptr, G, arr(ks0), arr(ks1), arr(d2_parts),
                                                  arr(evk_b_parts), arr(evk_a_parts), batch,
                                                  chunks, _ptr(ws), _stream(ref)),
                  "fhe_keyswitch_dist_loopback")
        return ks0, ks1


    def keyswitch_dist_hybrid_loopback(self, groups: int, d2_parts, evk_b_parts, evk_a_parts,
                                       chunks: int = 0, workspace=None):
        """The hybrid partition (fhe_dist_hybrid: `groups` ciphertext groups x g limb shards, G =
        len(d2_parts) ranks) run on this one device (fhe_keyswitch_dist_hybrid_loopback).  Rank r
        (group r // g, shard r % g): d2 [group batch, nlimbs, N] NTT form of its group's
        ciphertexts and LimbShard(L, g, r % g)'s limbs (None if it owns none), evk slices
        [dnum, nlimbs + K, N].  Returns the per-rank (ks0, ks1) lists."""
        G = len(d2_parts)
        if not G or groups < 1 or G % groups or len(evk_b_parts) != G or len(evk_a_parts) != G:
            raise ValueError("keyswitch_dist_hybrid_loopback: one entry per rank, groups | ranks")
        from .dist import LimbShard

        g = G // groups
        ks0, ks1 = [None] * G, [None] * G
        job = 0
        for r in range(G):
            sh = LimbShard(self.L, g, r % g)
            d2 = d2_parts[r]
            if sh.nlimbs == 0 or d2 is None:
                continue
            _check_tensor(d2, f"d2[{r}]", (sh.nlimbs, self.n))
            for t, nm in ((evk_b_parts[r], "evk_b"), (evk_a_parts[r], "evk_a")):
                _check_tensor(t, f"{nm}[{r}]", (self.dnum, sh.nlimbs + self.K, self.n))
            for t, nm in ((d2, "d2"), (evk_b_parts[r], "evk_b"), (evk_a_parts[r], "evk_a")):
                if t.device != self._dev():
                    raise ValueError(f"keyswitch_dist_hybrid_loopback: {nm}[{r}] is on "
                                     f"{t.device}, the context on {self._dev()}")
            if r % g == 0:
                job += d2.numel() // (sh.nlimbs * self.n)
            ks0[r], ks1[r] = _empty_like(d2), _empty_like(d2)
        lib = load()
        ws = workspace if workspace is not None else self.workspace(
            lib.fhe_keyswitch_dist_hybrid_loopback_workspace(self._ptr, G, groups, job, chunks))
        arr = lambda ts: (ctypes.c_void_p * G)(*[t.data_ptr() if t is not None else None  # noqa: E731
                                                  for t in ts])
        ref = next(t for t in d2_parts if t is not None)
        with torch.cuda.device(self.device):
            check(lib.fhe_keyswitch_dist_hybrid_loopback(
                self._ptr, G, groups, arr(ks0), arr(ks1), arr(d2_parts), arr(evk_b_parts),
                arr(evk_a_parts), job, chunks, _ptr(ws), _stream(ref)),
                "fhe_keyswitch_dist_hybrid_loopback")
        return ks0, ks1


class Graph:
    """Capture libfhecore calls issued on the current stream into a HIP graph and replay them
    (fhe_graph_*).  The tensors a captured call reads and writes are baked into the graph:
    outputs and workspaces that the Context methods allocate inside the block are kept alive by
    the Graph (``Graph.tensors``; read results from there or pass ``out=``), and caller-owned
    tensors must outlive it.  Every call is given a workspace -- the one passed in, or one this
    module allocates and the Graph keeps -- since the context's internal one is refused while
    capturing (include/fhecore.h)::

        with fhecore.Graph() as g:
            ctx.mul_relin(a, b, kb, ka, workspace=ws, out=out)
        g.launch()
    """

    def __init__(self):
        self._g = None
        self.tensors = []

    def __enter__(self):
        self._stream = torch.cuda.current_stream()
        check(load().fhe_graph_begin(ctypes.c_void_p(self._stream.cuda_stream)), "fhe_graph_begin")
        _CAPTURE.keep = self.tensors
        return self

    def __exit__(self, exc_type, exc, tb):
        _CAPTURE.keep = None
        g = ctypes.c_void_p()
        rc = load().fhe_graph_end(ctypes.c_void_p(self._stream.cuda_stream), ctypes.byref(g))
        if exc_type is None:
            check(rc, "fhe_graph_end")
            self._g = g
        return False

    def launch(self):
        check(load().fhe_graph_launch(self._g, ctypes.c_void_p(self._stream.cuda_stream)),
              "fhe_graph_launch")

    def __del__(self):
        if getattr(self, "_g", None):
            try:
                load().fhe_graph_destroy(self._g)
            except Exception:  # interpreter shutdown
                pass
