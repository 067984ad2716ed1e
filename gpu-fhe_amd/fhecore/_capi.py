"""ctypes binding of libfhecore (include/fhecore.h).

The library is built in-tree by ``make -C gpu-fhe_amd`` (``__graft_entry__.build()``) into
``gpu-fhe_amd/lib/libfhecore.so``.  There is no fallback: if the shared object is missing or
fails to load, every entry point raises -- the product path never silently computes on the CPU.
"""
from __future__ import annotations

import ctypes
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FHECORE_LIB overrides the in-tree library (A/B builds of the same sources in tools/).
LIB_PATH = os.environ.get("FHECORE_LIB") or os.path.join(_PKG_ROOT, "lib", "libfhecore.so")

FHE_OK = 0
_ERRNAMES = {-1: "FHE_EINVAL", -2: "FHE_ENOMEM", -3: "FHE_EDEVICE", -4: "FHE_EUNSUPPORTED"}

_u32, _u64, _i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
_vp = ctypes.c_void_p
_u64p = ctypes.POINTER(ctypes.c_uint64)
_sz = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/fhecore.h one to one
SIGNATURES = {
    "fhe_last_error": (ctypes.c_char_p, []),
    "fhe_version": (ctypes.c_char_p, []),
    "fhe_gen_moduli": (_i32, [_u32, _u32, _u32, _u32, _u64p]),
    "fhe_ctx_create": (_i32, [ctypes.POINTER(_vp), _u32, _u64p, _u32, _u64p, _u32, _u32, _i32]),
    "fhe_ctx_destroy": (_i32, [_vp]),
    "fhe_ctx_moduli": (_i32, [_vp, _u64p, _u64p]),
    "fhe_ctx_shape": (_i32, [_vp, ctypes.POINTER(_u32), ctypes.POINTER(_u32),
                             ctypes.POINTER(_u32), ctypes.POINTER(_u32), ctypes.POINTER(_i32)]),
    "fhe_ctx_reserve": (_i32, [_vp, _sz]),
    "fhe_vec_add": (_i32, [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp]),
    "fhe_vec_sub": (_i32, [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp]),
    "fhe_vec_mul": (_i32, [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp]),
    "fhe_vec_op_mod": (_i32, [_i32, _vp, _vp, _vp, _u64, _u64, _u64p, _u64, _i32, _i32, _vp]),
    "fhe_ntt_fwd": (_i32, [_vp, _vp, _u32, _u32, _u32, _vp]),
    "fhe_ntt_inv": (_i32, [_vp, _vp, _u32, _u32, _u32, _vp]),
    "fhe_ntt_fwd_to": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32, _vp]),
    "fhe_ntt_inv_to": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32, _vp]),
    "fhe_hommult_workspace": (_sz, [_vp, _u32, _u32]),
    "fhe_hommult": (_i32, [_vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp]),
    "fhe_baseconv": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32, _u32, _vp]),
    "fhe_keyswitch_workspace": (_sz, [_vp, _u32, _u32]),
    "fhe_keyswitch_pass_batch": (_u32, [_vp, _u32]),
    "fhe_keyswitch": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp]),
    "fhe_keyswitch_shard": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp,
                                   _vp]),
    "fhe_comm_get_unique_id": (_i32, [ctypes.c_char_p]),
    "fhe_comm_create": (_i32, [ctypes.POINTER(_vp), ctypes.c_char_p, _i32, _i32, _i32]),
    "fhe_comm_destroy": (_i32, [_vp]),
    "fhe_comm_shard": (_i32, [_vp, _vp, ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "fhe_keyswitch_dist_workspace": (_sz, [_vp, _vp, _u32, _u32]),
    "fhe_keyswitch_dist": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp]),
    "fhe_keyswitch_shard_ranked": (_i32, [_vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _u32, _u32,
                                          _u32, _vp, _vp]),
    "fhe_comm_gather_ms": (_i32, [_vp, ctypes.POINTER(ctypes.c_float), _u32,
                                  ctypes.POINTER(_u32)]),
    "fhe_dist_plan_make": (_i32, [_vp, _u32, _u32, _u32, _u32, _u32, _u32]),
    "fhe_dist_plan_chunk": (_i32, [_vp, _u32, ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "fhe_dist_plan_send_word": (_u64, [_vp, _u32, _u32]),
    "fhe_dist_plan_read_word": (_u64, [_vp, _u32, _u32]),
    "fhe_keyswitch_dist_loopback_workspace": (_sz, [_vp, _u32, _u32, _u32]),
    "fhe_keyswitch_dist_loopback": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _vp,
                                           _vp]),
    "fhe_dist_hybrid_make": (_i32, [_vp, _u32, _u32, _u32, _u32, _u32, _u32, _u32]),
    "fhe_keyswitch_dist_hybrid_loopback_workspace": (_sz, [_vp, _u32, _u32, _u32, _u32]),
    "fhe_keyswitch_dist_hybrid_loopback": (_i32, [_vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _u32,
                                                  _u32, _vp, _vp]),
    "fhe_rescale_workspace": (_sz, [_vp, _u32, _u32]),
    "fhe_rescale": (_i32, [_vp, _vp, _vp, _u32, _u32, _i32, _vp, _vp]),
    "fhe_automorphism": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32, _u32, _i32, _vp]),
    "fhe_rotate_workspace": (_sz, [_vp, _u32]),
    "fhe_rotate": (_i32, [_vp, _vp, _vp, _u32, _vp, _vp, _u32, _vp, _vp]),
    "fhe_rotate_hoisted_workspace": (_sz, [_vp, _u32]),
    "fhe_rotate_hoisted": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp]),
    "fhe_rotate_sum_hoisted_workspace": (_sz, [_vp, _u32]),
    "fhe_rotate_sum_hoisted": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp]),
    "fhe_rotate_sum_multi_workspace": (_sz, [_vp, _u32, _u32]),
    "fhe_rotate_sum_multi": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp]),
    "fhe_linear_transform_workspace": (_sz, [_vp, _u32, _u32]),
    "fhe_linear_transform": (_i32, [_vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _u32, _vp, _vp]),
    "fhe_serialized_size": (_sz, [_vp, _u32, _u32]),
    "fhe_serialize": (_i32, [_vp, _vp, _u32, _u32, _u32, _i32, _vp, _sz, _vp]),
    "fhe_deserialize": (_i32, [_vp, _vp, _sz, _vp, _sz, ctypes.POINTER(_u32), ctypes.POINTER(_u32),
                               ctypes.POINTER(_u32), ctypes.POINTER(_i32), _vp]),
    "fhe_mul_relin_workspace": (_sz, [_vp, _u32]),
    "fhe_mul_relin": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _u32, _i32, _vp, _vp]),
    "fhe_graph_begin": (_i32, [_vp]),
    "fhe_graph_end": (_i32, [_vp, ctypes.POINTER(_vp)]),
    "fhe_graph_launch": (_i32, [_vp, _vp]),
    "fhe_graph_destroy": (_i32, [_vp]),
    "fhe_sample": (_i32, [_vp, _vp, _u32, _u32, _u32, _i32, _u64, _u32, _vp]),
    "fhe_keygen_secret": (_i32, [_vp, _vp, _u64, _vp]),
    "fhe_keygen_public": (_i32, [_vp, _vp, _vp, _u64, _vp]),
    "fhe_keygen_switch": (_i32, [_vp, _vp, _vp, _vp, _u64, _vp]),
    "fhe_encrypt": (_i32, [_vp, _vp, _vp, _vp, _u64, _vp, _vp]),
    "fhe_encrypt_sk": (_i32, [_vp, _vp, _vp, _vp, _u64, _vp]),
    "fhe_decrypt": (_i32, [_vp, _vp, _vp, _vp, _u32, _u32, _vp]),
    "fhe_prof_begin": (_i32, [_u32, _vp]),
    "fhe_prof_end": (_i32, [ctypes.POINTER(ctypes.c_float), _u32, ctypes.POINTER(_u32),
                            ctypes.c_char_p, _sz]),
}

_lib = None


class FheError(RuntimeError):
    """A libfhecore entry point returned a negative status."""


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FheError(f"libfhecore not built: {LIB_PATH} is missing "
                           "(run `make -C gpu-fhe_amd` or __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            # an A/B variant built from an older commit (FHECORE_LIB, tools/build_variant.sh) may
            # lack entry points added since; the in-tree library must export every one
            if os.environ.get("FHECORE_LIB") and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str) -> None:
    if rc != FHE_OK:
        msg = load().fhe_last_error().decode(errors="replace")
        raise FheError(f"{what} failed: {_ERRNAMES.get(rc, rc)}: {msg}")


def u64_array(values):
    arr = (ctypes.c_uint64 * len(values))(*[int(v) for v in values])
    return arr


class DistPlan(ctypes.Structure):
    """fhe_dist_plan (include/fhecore.h): where fhe_keyswitch_dist puts and reads every row."""

    _fields_ = [(f, _u32) for f in ("L", "log_n", "ranks", "rank", "batch", "limb0", "nlimbs",
                                    "width", "chunks", "chunk_batch")] + \
               [("block_words", _u64), ("gather_words", _u64)]



class DistHybrid(ctypes.Structure):
    """fhe_dist_hybrid (include/fhecore.h): `groups` ciphertext groups x g limb shards."""

    _fields_ = [(f, _u32) for f in ("ranks", "groups", "g", "group", "shard", "batch0", "batch")] + \
               [("plan", DistPlan)]
