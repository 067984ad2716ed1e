"""Per-GPU rate of the default bench line at each rank shape of an N-GPU run, on one GPU (dev tool).

The driver's N-GPU runs give every rank L/N limbs of N times the ciphertexts (weak scaling), and
the key-switch leg 1/N of the limbs of one fixed batch (strong scaling).  This times rank 0's
share of each leg for N = 1, 2, 4, 8 in one process, with no collective, so the per-GPU kernel
efficiency at the N = 8 shapes can be read before an 8-GPU node runs them.
usage: python tools/shard_shape.py [--steps K] [--warmup W]"""
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
from fhecore import dist as fdist  # noqa: E402
from fhecore._capi import load  # noqa: E402
from bench import uniform_limbs  # noqa: E402


def rate(fn, warmup, steps):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--ks-batch", type=int, default=32, help="the key-switch leg's batch (bench.py)")
    args = ap.parse_args()
    log_n, n, L = 16, 1 << 16, 8
    ctx = fc.Context(log_n, L=L)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    out = {}
    for G in (1, 2, 4, 8):
        sh = fdist.LimbShard(L, G, 0)
        gb = 64 * G
        mods = ctx.moduli[sh.lo:sh.hi]
        a = uniform_limbs(gen, mods, (gb, 2), n)
        b = uniform_limbs(gen, mods, (gb, 2), n)
        d = ctx.empty(gb, 3, sh.nlimbs, n)
        ws = ctx.workspace(load().fhe_hommult_workspace(ctx.handle, gb, sh.nlimbs))
        dt = rate(lambda: fdist.sharded_hommult(ctx, a, b, sh, out=d, workspace=ws),
                  args.warmup, args.steps)
        npolys = 64 * L // sh.nlimbs
        x = uniform_limbs(gen, mods, (npolys,), n)

        def pair():
            ctx.ntt_(x, limb0=sh.lo)
            ctx.intt_(x, limb0=sh.lo)

        dn = rate(pair, args.warmup, args.steps)
        out[f"N={G}"] = {"limbs_per_gpu": sh.nlimbs, "ciphertexts_per_gpu": gb,
                         "hommult_ms_per_step": round(dt * 1e3, 4),
                         "job_hommult_per_s_if_linear": round(gb * G / dt, 1),
                         "per_gpu_poly_limb_hommults_per_s": round(gb * sh.nlimbs / dt, 1),
                         "ntt_pair_ms": round(dn * 1e3, 4),
                         "per_gpu_ntt_per_s": round(2 * npolys * sh.nlimbs / dn, 1)}
        del a, b, d, ws, x
        torch.cuda.empty_cache()
    # key-switch leg, rank 0 of N: its limb shard of the leg's batch over a ranked gather region
    # filled with residues (timing only: the per-rank kernels of fhe_keyswitch_dist after its
    # gather)
    Lk, K, dnum, B = 16, 4, 4, args.ks_batch
    kctx = fc.Context(log_n, L=Lk, K=K, dnum=dnum)
    lib = load()
    for G in (1, 2, 4, 8):
        sh = fdist.LimbShard(Lk, G, 0)
        rows = sh.evk_rows(K)
        allm = kctx.all_moduli
        eb = uniform_limbs(gen, [allm[r] for r in rows], (dnum,), n)
        ea = uniform_limbs(gen, [allm[r] for r in rows], (dnum,), n)
        d2 = uniform_limbs(gen, kctx.moduli[sh.lo:sh.hi], (B,), n)
        gat = torch.zeros(G * B * sh.width * n, dtype=torch.int64, device="cuda")
        ks0 = kctx.empty(B, sh.nlimbs, n)
        ks1 = kctx.empty(B, sh.nlimbs, n)
        ws = kctx.workspace(lib.fhe_keyswitch_workspace(kctx.handle, sh.nlimbs, B))

        def ks():
            rc = lib.fhe_keyswitch_shard_ranked(kctx.handle, ks0.data_ptr(), ks1.data_ptr(),
                                                gat.data_ptr(), G, d2.data_ptr(), eb.data_ptr(),
                                                ea.data_ptr(), sh.lo, sh.nlimbs, B,
                                                ws.data_ptr(),
                                                torch.cuda.current_stream().cuda_stream)
            assert rc == 0, lib.fhe_last_error()

        dk = rate(ks, 20, 50)
        out[f"ks N={G}"] = {"limbs_per_gpu": sh.nlimbs, "batch": B, "ms_per_batch": round(dk * 1e3, 4),
                            "speedup_vs_N1_if_gather_hidden": None}
    base = out["ks N=1"]["ms_per_batch"]
    for G in (1, 2, 4, 8):
        out[f"ks N={G}"]["speedup_vs_N1_if_gather_hidden"] = round(
            base / out[f"ks N={G}"]["ms_per_batch"], 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
