import os, sys, time, ctypes
sys.path.insert(0, "gpu-fhe_amd")
import torch
import fhecore as fc
from fhecore import dist as fdist
from fhecore._capi import load
from fhecore.context import _ptr, _stream
L, n = 8, 1 << 16
ctx = fc.Context(16, L=L)
lib = load()
for world in (1, 8, 1):
    shard = fdist.LimbShard(L, world, 0)
    B = 16 * world
    mods = ctx.moduli[shard.lo:shard.hi]
    a = torch.stack([torch.randint(0, q, (B, 2, n), dtype=torch.int64, device="cuda") for q in mods], 2)
    b = torch.stack([torch.randint(0, q, (B, 2, n), dtype=torch.int64, device="cuda") for q in mods], 2)
    d = ctx.empty(B, 3, shard.nlimbs, n)
    ws = ctx.workspace(lib.fhe_hommult_workspace(ctx.handle, B, shard.nlimbs))
    st = _stream(a)
    raw = lambda: lib.fhe_hommult(ctx.handle, _ptr(d), _ptr(a), _ptr(b), B, shard.lo, shard.nlimbs, _ptr(ws), st)
    py = lambda: fdist.sharded_hommult(ctx, a, b, shard, out=d, workspace=ws)
    for name, f in (("raw", raw), ("py", py)):
        for _ in range(5): f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(100): f()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"world={world} {name}: host enqueue {(t1-t0)/100*1e6:.1f} us/step, total {(t2-t0)/100*1e6:.1f} us/step", flush=True)
