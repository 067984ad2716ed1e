"""Step-by-step probe of the single-launch NTT experiment (dev tool): small shapes first, every
launch synchronised and reported before the next, so a hang names its configuration."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))
import torch  # noqa: E402

import fhecore as fc  # noqa: E402
from fhecore._capi import load  # noqa: E402

lib = load()
lib.fhe_x_ntt_fused.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
ctx = fc.Context(16, L=8)
for polys, wgs, lag in [(1, 8, 8), (1, 8, 1), (2, 16, 1), (8, 64, 2), (64, 1024, 4)]:
    P = polys * 8
    x = torch.stack([torch.randint(0, q, (polys, 1 << 16), dtype=torch.int64, device="cuda")
                     for q in ctx.moduli], 1).contiguous()
    ref = ctx.ntt(x)
    y = x.clone()
    ctr = torch.zeros(8 + P + 1, dtype=torch.int32, device="cuda")
    print(f"launch polys={polys} wgs={wgs} lag={lag}", flush=True)
    t0 = time.time()
    rc = lib.fhe_x_ntt_fused(ctx.handle, 1, y.data_ptr(), polys, 0, 8, lag, wgs, 8, ctr.data_ptr(),
                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    print(f"  rc={rc} {time.time() - t0:.3f}s heads={ctr[:8].tolist()} err={int(ctr[8 + P])} "
          f"done={ctr[8:8 + min(P, 16)].tolist()} wrong={int((y != ref).sum())}", flush=True)
