"""A/B of the single-launch NTT (ntt.hip k_ntt_fused, experimental entry fhe_x_ntt_fused) against
the two-pass NTT (fhe_ntt_fwd / fhe_ntt_inv) on the GPU: XCD census of a persistent grid, bit-exact
check of both directions, then kernel times (HIP events) for several lags and grid sizes.
Dev / measurement tool.  usage: python tools/time_ntt_fused.py [polys] [log_n] [L]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))

import torch  # noqa: E402

import fhecore as fc  # noqa: E402
from fhecore._capi import load  # noqa: E402

lib = load()
lib.fhe_x_xcc_census.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                  ctypes.POINTER(ctypes.c_uint32)]
lib.fhe_x_ntt_fused.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]

polys = int(sys.argv[1]) if len(sys.argv) > 1 else 64
log_n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
L = int(sys.argv[3]) if len(sys.argv) > 3 else 8
n = 1 << log_n
out = {"polys": polys, "log_n": log_n, "L": L}

hist = (ctypes.c_uint32 * 16)()
bmap = (ctypes.c_uint32 * 4096)()
assert lib.fhe_x_xcc_census(0, 4096, hist, bmap) == 0
out["census_4096_blocks"] = list(hist)
out["xcc_raw_first_24_blocks"] = [hex(v) for v in bmap[:24]]
out["blocks_b_and_b8_same_xcc"] = sum(bmap[b] == bmap[b + 8] for b in range(4088)) / 4088
print(json.dumps(out), flush=True)

ctx = fc.Context(log_n, L=L)
gen = torch.Generator(device="cuda")
gen.manual_seed(3)
x = torch.stack([torch.randint(0, q, (polys, n), generator=gen, dtype=torch.int64, device="cuda")
                 for q in ctx.moduli], 1).contiguous()
P = polys * L
ctr = torch.zeros(8 + P + 1, dtype=torch.int32, device="cuda")
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
cus = torch.cuda.get_device_properties(0).multi_processor_count


def fused(t, fwd, lag, wgs):
    rc = lib.fhe_x_ntt_fused(ctx.handle, int(fwd), t.data_ptr(), polys, 0, L, lag, wgs, 8,
                             ctr.data_ptr(), stream)
    assert rc == 0, lib.fhe_last_error()


# correctness: both directions against the two-pass path
ref = ctx.ntt(x)
y = x.clone()
fused(y, True, 4, 4 * cus)
torch.cuda.synchronize()
out["error_flag_fwd"] = int(ctr[8 + P].item())
out["heads_after_fwd"] = ctr[:8].tolist()
out["done_counts_fwd_first16"] = ctr[8:24].tolist()
out["fwd_words_wrong"] = int((y != ref).sum().item())
out["fwd_bit_exact"] = bool(torch.equal(y, ref))
fused(y, False, 4, 4 * cus)
torch.cuda.synchronize()
out["error_flag_inv"] = int(ctr[8 + P].item())
out["inv_round_trip_exact"] = bool(torch.equal(y, x))
print(json.dumps(out), flush=True)
if not (out["fwd_bit_exact"] and out["inv_round_trip_exact"]):
    sys.exit(1)


def time_it(fn, reps=100):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


if os.environ.get("FUSED_QUICK"):  # the PMC passes: 20 launches of each, nothing else
    for _ in range(20):
        ctx.ntt_(y)
    for _ in range(20):
        fused(y, True, 8, 4 * cus)
    torch.cuda.synchronize()
    sys.exit(0)
res = {}
# sustained clock first
t0 = time.time()
while time.time() - t0 < 0.5:
    ctx.ntt_(y)
    ctx.intt_(y)
torch.cuda.synchronize()
res["two_pass_fwd_ms"] = time_it(lambda: ctx.ntt_(y))
res["two_pass_inv_ms"] = time_it(lambda: ctx.intt_(y))
for wmul in (4, 8):
    for lag in (2, 4, 6, 8, 12):
        res[f"fused_fwd_lag{lag}_wg{wmul}x_ms"] = time_it(lambda: fused(y, True, lag, wmul * cus))
        res[f"fused_inv_lag{lag}_wg{wmul}x_ms"] = time_it(lambda: fused(y, False, lag, wmul * cus))
res["two_pass_fwd_ms_again"] = time_it(lambda: ctx.ntt_(y))
res["error_flag"] = int(ctr[8 + P].item())
bytes_pass = polys * L * n * 16
res = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}
res["alg_bytes_per_transform_batch"] = bytes_pass
print(json.dumps(res), flush=True)
