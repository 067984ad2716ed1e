"""HomMult kernel times on CU-masked streams (dev tool): how much of each kernel's speed survives
on a fraction of the CUs, to judge whether the HBM-bound column passes and the VALU-bound row
kernel could run side by side on disjoint CU sets.
usage: python tools/cumask_probe.py [pair]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))

import torch  # noqa: E402

import fhecore as fc  # noqa: E402
from fhecore._capi import check, load  # noqa: E402
from bench import uniform_limbs  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]


def masked_stream(bits):
    words = (ctypes.c_uint32 * 8)()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, words)
    assert rc == 0, rc
    return s


def run(ctx, lib, a, b, d, ws, B, s, reps=60):
    for _ in range(20):
        check(lib.fhe_hommult(ctx.handle, d.data_ptr(), a.data_ptr(), b.data_ptr(), B, 0, 8,
                              ws.data_ptr(), s), "hommult")
    hip.hipStreamSynchronize(s)
    check(lib.fhe_prof_begin(4 * reps + 4, s), "prof")
    for _ in range(reps):
        check(lib.fhe_hommult(ctx.handle, d.data_ptr(), a.data_ptr(), b.data_ptr(), B, 0, 8,
                              ws.data_ptr(), s), "hommult")
    hip.hipStreamSynchronize(s)
    ms = (ctypes.c_float * (4 * reps + 4))()
    cnt = ctypes.c_uint32()
    names = ctypes.create_string_buffer(64 * reps + 256)
    check(lib.fhe_prof_end(ms, 4 * reps + 4, ctypes.byref(cnt), names, 64 * reps + 256), "end")
    per = {}
    for nm, v in zip(names.value.decode().split("\n"), ms[:cnt.value]):
        per.setdefault(nm, []).append(v)
    return {k: round(sum(v) / len(v), 4) for k, v in per.items()}


def main():
    torch.cuda.set_device(0)
    lib = load()
    ctx = fc.Context(16, L=8)
    n = 1 << 16
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    B = 64
    a = uniform_limbs(gen, ctx.moduli, (B, 2), n)
    b = uniform_limbs(gen, ctx.moduli, (B, 2), n)
    d = torch.empty(B, 3, 8, n, dtype=torch.int64, device="cuda")
    ws = ctx.workspace(lib.fhe_hommult_workspace(ctx.handle, B, 8))
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    out = {"cus": ncu}
    masks = {"all": range(ncu), "low_half": range(ncu // 2), "even": range(0, ncu, 2),
             "3_of_4": [c for c in range(ncu) if c % 4 != 3], "1_of_4": range(0, ncu, 4),
             "low_quarter": range(ncu // 4)}
    for name, bits in masks.items():
        s = masked_stream(list(bits))
        out[name] = run(ctx, lib, a, b, d, ws, B, s)
        hip.hipStreamDestroy(s)
    print(json.dumps(out, indent=1))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def concurrent(split=128, reps=100):
    """Two HomMult pipelines of 32 ciphertexts on disjoint CU sets (bits [0, split) and
    [split, 256)), issued alternately, vs one pipeline of 64 on all CUs: whole-job HomMult/s."""
    import time
    torch.cuda.set_device(0)
    lib = load()
    ctx = fc.Context(16, L=8)
    n = 1 << 16
    gen = torch.Generator(device="cuda")
    gen.manual_seed(4)
    bufs = []
    for B in (32, 32, 64):
        a = uniform_limbs(gen, ctx.moduli, (B, 2), n)
        b = uniform_limbs(gen, ctx.moduli, (B, 2), n)
        d = torch.empty(B, 3, 8, n, dtype=torch.int64, device="cuda")
        ws = ctx.workspace(lib.fhe_hommult_workspace(ctx.handle, B, 8))
        bufs.append((a, b, d, ws, B))
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    sa, sb = masked_stream(range(split)), masked_stream(range(split, ncu))
    sall = masked_stream(range(ncu))

    def hm(buf, s):
        a, b, d, ws, B = buf
        check(lib.fhe_hommult(ctx.handle, d.data_ptr(), a.data_ptr(), b.data_ptr(), B, 0, 8,
                              ws.data_ptr(), s), "hommult")

    res = {}
    for name in ("single64", "pair32", "single64_again", "pair32_again"):
        for _ in range(20):
            if name.startswith("single"):
                hm(bufs[2], sall)
            else:
                hm(bufs[0], sa)
                hm(bufs[1], sb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if name.startswith("single"):
                hm(bufs[2], sall)
            else:
                hm(bufs[0], sa)
                hm(bufs[1], sb)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[name] = round(64 * reps / dt, 1)
    return res


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pair":
    print(json.dumps({f"split{sp}": concurrent(sp) for sp in (128, 96, 160)}, indent=1))
