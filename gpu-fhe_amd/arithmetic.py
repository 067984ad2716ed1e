"""Drop-in for the reference's ``arithmetic`` module, computed by libfhecore on a HIP device.

Put ``gpu-fhe_amd/`` on ``sys.path`` where the reference directory used to be and
``from arithmetic import *`` keeps working (the reference star-imports this module from
``primitive.py:1``).  Same names, argument order and meaning as
/root/reference/arithmetic.py:3-19:

* ``vec_add(a, b, MOD)`` / ``vec_sub`` / ``vec_mul`` -- ``(a op b) % MOD`` elementwise.  Shape
  mismatch raises ``AssertionError`` exactly like ``arithmetic.py:4,8,12``.  Results are the
  EXACT Python-int values (what the reference yields on dtype=object input); the reference's own
  uint64 path wraps mod 2^64 for sub/mul and is not reproduced.  ``MOD`` is a
  scalar or any array that broadcasts against the operands (e.g. a per-limb ``(L, 1)`` column).
* ``NTT(x, MOD=None)`` / ``iNTT(x, MOD=None)`` -- the negacyclic transform of SURVEY.md §8a'
  (the reference's are identity stubs, arithmetic.py:15-19).  ``x`` is ``(N,)`` or
  ``(..., L, N)`` with residues in [0, q_l); ``MOD`` defaults to the §8a' modulus chain for
  (N, L) and may be a scalar or a length-L sequence.  A NEW array is returned (the reference
  returns its argument).

numpy inputs are copied to the device and back; int64/uint64 HIP tensors stay on the device.
There is no CPU fallback: without a HIP device or without lib/libfhecore.so these raise.
"""
import ctypes as _ctypes

import numpy as np

from fhecore import _capi as _capi
from fhecore import context as _context

_OPS = {"add": 0, "sub": 1, "mul": 2}
_U64_MAX = (1 << 64) - 1


def _torch():
    import torch

    return torch


def _is_tensor(x):
    try:
        return isinstance(x, _torch().Tensor)
    except ImportError:  # pragma: no cover
        return False


def _as_words(x):
    """numpy integer/object array -> (uint64 or int64 array, was_object, is_signed)."""
    arr = np.asarray(x)
    if arr.dtype == object:
        flat = [int(v) for v in arr.reshape(-1)]
        lo = min(flat, default=0)
        hi = max(flat, default=0)
        if lo < -(1 << 63) or hi > _U64_MAX:
            raise ValueError("libfhecore operands must fit a 64-bit word")
        if lo < 0:
            if hi >= (1 << 63):
                raise ValueError("mixed negative and >= 2^63 operands do not fit one word type")
            return np.array(flat, dtype=np.int64).reshape(arr.shape), True, True
        return np.array(flat, dtype=np.uint64).reshape(arr.shape), True, False
    if arr.dtype.kind == "u":
        return arr.astype(np.uint64), False, False
    if arr.dtype.kind == "i":
        if arr.size and arr.min() < 0:
            return arr.astype(np.int64), False, True
        return arr.astype(np.uint64), False, False
    if arr.dtype.kind == "b":
        return arr.astype(np.uint64), False, False
    raise TypeError(f"unsupported operand dtype {arr.dtype}")


def _moduli_layout(shape, mod):
    """-> (rows, cols, mods list, mod_stride) for a C-contiguous array of `shape`."""
    m = np.asarray(mod, dtype=object)
    size = int(np.prod(shape)) if shape else 1
    if m.ndim == 0:
        return 1, size, [int(m)], 0
    mb = np.broadcast_to(m, shape)
    if len(shape) >= 1 and shape[-1] > 0:
        cols = shape[-1]
        rows = size // cols if cols else 0
        first = mb[..., :1]
        if np.all(mb == first):
            return rows, cols, [int(v) for v in first.reshape(-1)], 1
    return size, 1, [int(v) for v in mb.reshape(-1)], 1


def _vec_tensor(op, a, b, mod):
    torch = _torch()
    if a.dtype not in (torch.int64, torch.uint64) or b.dtype != a.dtype:
        raise TypeError("device operands must both be int64 or uint64 tensors")
    a = a.contiguous()
    b = b.contiguous()
    rows, cols, mods, stride = _moduli_layout(tuple(a.shape), mod)
    out = torch.empty_like(a)
    _vec_launch(op, out, a, b, rows, cols, mods, stride, signed=False)
    return out


def _vec_launch(op, out, a, b, rows, cols, mods, stride, signed):
    for q in mods:
        if not 2 <= q <= _U64_MAX:
            raise ValueError(f"MOD must be an integer in [2, 2^64), got {q}")
    lib = _capi.load()
    marr = _capi.u64_array(mods)
    dev = out.device.index if out.device.index is not None else 0
    torch = _torch()
    stream = _ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)
    with torch.cuda.device(dev):
        _capi.check(lib.fhe_vec_op_mod(_OPS[op], out.data_ptr(), a.data_ptr(), b.data_ptr(), rows,
                                       cols, marr, stride, int(signed), dev, stream),
                    "fhe_vec_op_mod")


def _vec(op, a, b, mod):
    assert a.shape == b.shape  # arithmetic.py:4,8,12
    if _is_tensor(a) or _is_tensor(b):
        return _vec_tensor(op, a, b, mod)
    _context._require_device()
    wa, obj_a, sa = _as_words(a)
    wb, obj_b, sb = _as_words(b)
    signed = sa or sb
    if signed:
        if (wa.dtype == np.uint64 and wa.size and wa.max() >= (1 << 63)) or (
                wb.dtype == np.uint64 and wb.size and wb.max() >= (1 << 63)):
            raise ValueError("mixed negative and >= 2^63 operands do not fit one word type")
        wa, wb = wa.astype(np.int64), wb.astype(np.int64)
    shape = np.broadcast_shapes(wa.shape, np.shape(mod))
    wa = np.ascontiguousarray(np.broadcast_to(wa, shape))
    wb = np.ascontiguousarray(np.broadcast_to(wb, shape))
    rows, cols, mods, stride = _moduli_layout(shape, mod)
    torch = _torch()
    ta = _context.to_device(wa.view(np.uint64))
    tb = _context.to_device(wb.view(np.uint64))
    out = torch.empty_like(ta)
    if ta.numel():
        _vec_launch(op, out, ta, tb, rows, cols, mods, stride, signed)
    res = _context.to_host(out).reshape(shape)
    if obj_a or obj_b:
        return res.astype(object)
    kinds = {np.asarray(a).dtype.kind, np.asarray(b).dtype.kind}
    if "i" in kinds and max(mods) <= (1 << 63):
        return res.astype(np.int64)
    return res


def vec_add(a, b, MOD):
    """(a + b) % MOD, exact (arithmetic.py:3-5)."""
    return _vec("add", a, b, MOD)


def vec_sub(a, b, MOD):
    """(a - b) % MOD, exact, result in [0, MOD) (arithmetic.py:7-9)."""
    return _vec("sub", a, b, MOD)


def vec_mul(a, b, MOD):
    """(a * b) % MOD, exact (arithmetic.py:11-13); in the NTT domain = poly_mul_pointwise."""
    return _vec("mul", a, b, MOD)


# --------------------------------------------------------------------------------------- NTT

_CTX_CACHE = {}


def _ctx_for(log_n, moduli, device):
    key = (log_n, tuple(moduli), device)
    ctx = _CTX_CACHE.get(key)
    if ctx is None:
        ctx = _context.Context(log_n, moduli=list(moduli), device=device)
        _CTX_CACHE[key] = ctx
    return ctx


def _ntt(x, mod, forward):
    is_t = _is_tensor(x)
    shape = tuple(x.shape)
    if len(shape) == 0:
        raise ValueError("NTT needs at least one dimension")
    n = shape[-1]
    log_n = n.bit_length() - 1
    if n < 2 or (1 << log_n) != n:
        raise ValueError(f"NTT length must be a power of two, got {n}")
    if mod is None:
        L = shape[-2] if len(shape) >= 2 else 1
        moduli = _context.gen_moduli(log_n, L)
        view = (-1, L, n)
    else:
        m = [int(v) for v in np.asarray(mod, dtype=object).reshape(-1)]
        if len(m) == 1:
            moduli, view = m, (-1, 1, n)
        else:
            if len(shape) < 2 or shape[-2] != len(m):
                raise ValueError(f"MOD has {len(m)} moduli but x has shape {shape}")
            moduli, view = m, (-1, len(m), n)
    torch = _torch()
    if is_t:
        t = x.reshape(view).clone()
        dev = t.device.index or 0
    else:
        _context._require_device()
        w = np.asarray(x)
        if w.dtype == object:
            w = np.array([int(v) for v in w.reshape(-1)], dtype=object).reshape(w.shape)
        w = w.astype(np.uint64).reshape(view)
        qcol = np.array(moduli, dtype=np.uint64).reshape(1, -1, 1)
        if np.any(np.asarray(x).astype(object).reshape(view) < 0) or np.any(w >= qcol):
            raise ValueError("NTT input must hold residues in [0, q) for every limb")
        dev = torch.cuda.current_device()
        t = _context.to_device(w, device=torch.device("cuda", dev))
    ctx = _ctx_for(log_n, moduli, dev)
    (ctx.ntt_ if forward else ctx.intt_)(t)
    if is_t:
        return t.reshape(shape)
    out = _context.to_host(t).reshape(shape)
    return out.astype(object) if np.asarray(x).dtype == object else out


def NTT(x, MOD=None):
    """Forward negacyclic NTT per limb, natural -> bit-reversed (SURVEY.md §8a')."""
    return _ntt(x, MOD, True)


def iNTT(x, MOD=None):
    """Inverse of NTT (bit-reversed -> natural, N^-1 included)."""
    return _ntt(x, MOD, False)
