"""Per-GPU HomMult throughput at the per-rank shapes bench.py runs for N = 1, 2, 4, 8 GPUs
(L = 8 limbs sharded over the ranks, global batch 64 N, the last rank's limb window), timed on one GPU (dev tool: predicts the
driver's scaling runs, which shard with no collective).  usage: python tools/shape_scan.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-fhe_amd"))
import torch  # noqa: E402

import fhecore as fc  # noqa: E402
from fhecore import dist as fdist  # noqa: E402
from fhecore._capi import load  # noqa: E402

L, n = 8, 1 << 16
ctx = fc.Context(16, L=L)
for world in (1, 2, 4, 8):
    shard = fdist.LimbShard(L, world, world - 1)
    B = 64 * world
    mods = ctx.moduli[shard.lo:shard.hi]
    a = torch.stack([torch.randint(0, q, (B, 2, n), dtype=torch.int64, device="cuda") for q in mods], 2)
    b = torch.stack([torch.randint(0, q, (B, 2, n), dtype=torch.int64, device="cuda") for q in mods], 2)
    d = ctx.empty(B, 3, shard.nlimbs, n)
    ws = ctx.workspace(load().fhe_hommult_workspace(ctx.handle, B, shard.nlimbs))
    step = lambda: fdist.sharded_hommult(ctx, a, b, shard, out=d, workspace=ws)  # noqa: E731
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    import ctypes
    lib = load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    lib.fhe_prof_begin(200, st)
    t0 = time.perf_counter()
    for _ in range(100):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 100
    ms = (ctypes.c_float * 200)(); cnt = ctypes.c_uint32(); names = ctypes.create_string_buffer(8192)
    lib.fhe_prof_end(ms, 200, ctypes.byref(cnt), names, 8192)
    per = {}
    for nm, v in zip(names.value.decode().split("\n"), ms[:cnt.value]):
        per.setdefault(nm, []).append(v)
    print("   ", " ".join(f"{k}={sum(v)/len(v)*1000:.1f}us" for k, v in per.items()))
    print(f"world={world}: per-rank {shard.nlimbs} limbs x {B} ct: {dt*1e3:.3f} ms/step -> "
          f"job {B / dt:.0f} HomMult/s if every rank matches", flush=True)
