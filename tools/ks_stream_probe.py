"""Key-switch throughput with the batch split over concurrent HIP streams (dev probe): whether the
latency-bound key-switch kernels (k_ks_row_inner, k_moddown_row at 0.52-0.53 of the VALU issue
ceiling) gain from running beside another batch's VALU-heavier kernels (k_modup_col at 0.70).
Configs[3] shape (N = 2^16, L = 16, K = 4, dnum = 4), one key, fhe_keyswitch per stream with its
own workspace.  usage: python tools/ks_stream_probe.py [--reps R]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))

import torch  # noqa: E402

import fhecore as fc  # noqa: E402
from fhecore._capi import load  # noqa: E402
from bench import uniform_limbs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    log_n, L, K, dnum = 16, 16, 4, 4
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    kb = uniform_limbs(gen, ctx.all_moduli, (dnum,), n)
    ka = uniform_limbs(gen, ctx.all_moduli, (dnum,), n)
    lib = load()
    out = {}
    for total, nstreams in ((32, 1), (32, 2), (64, 1), (64, 2), (64, 4)):
        per = total // nstreams
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        d2 = [uniform_limbs(gen, ctx.moduli, (per,), n) for _ in range(nstreams)]
        ws = [ctx.workspace(lib.fhe_keyswitch_workspace(ctx.handle, L, per)) for _ in range(nstreams)]
        torch.cuda.synchronize()

        def step():
            for s, d, w in zip(streams, d2, ws):
                with torch.cuda.stream(s):
                    ctx.keyswitch(d, kb, ka, workspace=w)

        for _ in range(10):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        out[f"batch {total} over {nstreams} stream(s)"] = {
            "ms_per_step": round(dt * 1e3, 4), "keyswitch_per_s": round(total / dt, 1)}
        del d2, ws
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
