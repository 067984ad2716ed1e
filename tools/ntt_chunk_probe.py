"""Chunking probe (dev tool): forward + inverse NTT of 64 polys x 8 limbs at N = 2^16 issued as one
call, or as calls of `chunk` polys each (each chunk's column and row passes back to back, so a
chunk's intermediate can stay in the 256 MB Infinity Cache between the passes).  Prints NTT/s per
chunk size, sustained (warmup, then timed with HIP events).  Also HomMult at batch 64 vs chunks,
on one stream or dealt round-robin over several (each stream with its own workspace), so that
chunk tails overlap while each chunk's intermediate stays cache-sized.
usage: python tools/ntt_chunk_probe.py [hm]   (hm: the HomMult part only)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-fhe_amd"))
import torch
import fhecore as fc

log_n, L, P = 16, 8, 64
n = 1 << log_n
ctx = fc.Context(log_n, L=L)
x = torch.randint(0, 2**59, (P, L, n), dtype=torch.int64, device="cuda")
a = torch.randint(0, 2**59, (P, 2, L, n), dtype=torch.int64, device="cuda")
b = torch.randint(0, 2**59, (P, 2, L, n), dtype=torch.int64, device="cuda")
d = torch.empty(P, 3, L, n, dtype=torch.int64, device="cuda")


def run_ntt(chunk):
    for c0 in range(0, P, chunk):
        ctx.ntt_(x[c0:c0 + chunk])
    for c0 in range(0, P, chunk):
        ctx.intt_(x[c0:c0 + chunk])


def run_hm(chunk):
    for c0 in range(0, P, chunk):
        ctx.hommult(a[c0:c0 + chunk], b[c0:c0 + chunk], out=d[c0:c0 + chunk])


_STREAMS = {}


def run_hm_streams(chunk, ns):
    if ns not in _STREAMS:
        _STREAMS[ns] = [(torch.cuda.Stream(), ctx.workspace(fc.load().fhe_hommult_workspace(ctx.handle, chunk, L)))
                        for _ in range(ns)]
    main = torch.cuda.current_stream()
    ss = _STREAMS[ns]
    for s, _ in ss:
        s.wait_stream(main)
    for i, c0 in enumerate(range(0, P, chunk)):
        s, ws = ss[i % ns]
        with torch.cuda.stream(s):
            ctx.hommult(a[c0:c0 + chunk], b[c0:c0 + chunk], out=d[c0:c0 + chunk], workspace=ws)
    for s, _ in ss:
        main.wait_stream(s)


def timeit(f, steps=200, warm=100):
    for _ in range(warm):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


HM_ONLY = sys.argv[1:] == ["hm"]
for rep in range(2):
    for chunk in (() if HM_ONLY else (64, 32, 16, 8)):
        ms = timeit(lambda: run_ntt(chunk))
        print(f"ntt chunk {chunk:3d}: {ms * 1e3:8.1f} us per fwd+inv of {P}x{L} -> "
              f"{2 * P * L / ms * 1e3 / 1e6:.3f} M NTT/s", flush=True)
    for chunk in (64, 32, 16, 8):
        ms = timeit(lambda: run_hm(chunk), steps=100, warm=50)
        print(f"hommult chunk {chunk:3d}: {ms * 1e3:8.1f} us per {P} -> {P / ms * 1e3:.0f} HomMult/s",
              flush=True)
    for chunk, ns in ((16, 2), (8, 2), (8, 4)):
        ms = timeit(lambda: run_hm_streams(chunk, ns), steps=100, warm=50)
        print(f"hommult chunk {chunk:3d} on {ns} streams: {ms * 1e3:8.1f} us per {P} -> "
              f"{P / ms * 1e3:.0f} HomMult/s", flush=True)
