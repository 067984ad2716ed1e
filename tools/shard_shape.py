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


# xGMI on MI355X: 7 GPU-GPU links per GPU at 153.6 GB/s each, bidirectional (1075 GB/s aggregate),
# so 76.8 GB/s per link and direction; a fully connected 8-GPU node gives every pair its own link.
LINK_GBPS_DIR = 76.8


def ks_partition_model(out, L, K, B, n):
    """Per-rank time of one key-switch batch at N GPUs for the shipped partition (one all-gather of
    the coefficient-form d2) and the P-sharded one (the same gather, plus an all-gather of the INTT'd
    special-limb part of both accumulators, 2 K limbs per ciphertext, before ModDown), from the
    measured rank-shape compute above and the bytes each rank receives.  N GPUs of one node reach
    each other over N - 1 links (one per pair).  Two link models: 'direct' (every peer's block on
    its own link at the per-direction peak: the floor) and 'ring' (RCCL's ring all-gather at a bus
    bandwidth of 0.7 of the N - 1 links' aggregate).  Step time = max(compute, comm) with the
    chunked overlap, and compute + comm without it."""
    res = {"assumptions": {
        "link_GBps_per_direction": LINK_GBPS_DIR,
        "links_between_N_gpus": "N - 1 per GPU (fully connected node, one link per pair)",
        "ring_bus_bandwidth": "0.7 x (N - 1) x link_GBps_per_direction",
        "batch": B, "bytes_per_limb_row": n * 8}}
    row = n * 8
    for G in (2, 4, 8):
        c = -(-L // G)
        d2_peer = B * c * row  # one peer's block of the d2 gather
        kp = -(-K // G)        # special limbs a P-owning rank holds
        owners = min(K, G)
        p_peer = 2 * B * kp * row
        variants = {
            "replicated P (shipped)": (out[f"ks N={G}"]["ms_per_batch"],
                                       [(G - 1, d2_peer)]),
            "P-sharded": (out[f"ks N={G} P-sharded proxy"]["ms_per_batch"],
                          [(G - 1, d2_peer), (owners - 1, p_peer)]),
        }
        for name, (comp, gathers) in variants.items():
            recv = sum(k * b for k, b in gathers)
            direct = sum(b for k, b in gathers if k) / (LINK_GBPS_DIR * 1e9) * 1e3
            ring = recv / (0.7 * (G - 1) * LINK_GBPS_DIR * 1e9) * 1e3  # received / bus bandwidth
            res[f"N={G} {name}"] = {
                "compute_ms": comp, "recv_MB": round(recv / 1e6, 1),
                "comm_ms_direct": round(direct, 4), "comm_ms_ring": round(ring, 4),
                "step_ms_overlapped_direct": round(max(comp, direct), 4),
                "step_ms_overlapped_ring": round(max(comp, ring), 4),
                "step_ms_serial_ring": round(comp + ring, 4),
                "keyswitch_per_s_overlapped_direct": round(B / max(comp, direct) * 1e3, 1),
                "keyswitch_per_s_overlapped_ring": round(B / max(comp, ring) * 1e3, 1)}
    return res


def hybrid_shapes(gen, B, warmup=20, steps=50):
    """Per-rank compute of the hybrid partition's key-switch leg (fhe_dist_hybrid: G / g ciphertext
    groups x g limb shards) at G = 2, 4, 8 for every divisor g, timed on this GPU, plus the xGMI
    model of the group's all-gather.  Rank 0 of group 0 (the fullest group: ceil(B g / G)
    ciphertexts, the widest shard) runs its chunked local step exactly as fhe_keyswitch_dist does
    after each gather: 4 chunks when g > 1, one call and no gather when g = 1."""
    Lk, K, dnum, log_n = 16, 4, 4, 16
    n = 1 << log_n
    lib = load()
    ctx = fc.Context(log_n, L=Lk, K=K, dnum=dnum)
    res = {"assumptions": {"link_GBps_per_direction": LINK_GBPS_DIR, "batch": B,
                           "comm": "each rank receives (g - 1) peer blocks of its group's chunk; "
                                   "direct: one link per peer at the per-direction peak; ring: "
                                   "0.7 x (g - 1) links' aggregate",
                           "step": "first chunk's gather exposed + max(compute, the other chunks' "
                                   "gathers), the chunked overlap of fhe_keyswitch_dist"}}
    for G in (1, 2, 4, 8):
        for g in [d for d in (1, 2, 4, 8) if d <= G and G % d == 0]:
            groups = G // g
            sh = fdist.LimbShard(Lk, g, 0)
            gb = -(-B // groups)  # group 0's ciphertexts
            c = 1 if g == 1 else min(4, gb)
            cb = -(-gb // c)
            rows = sh.evk_rows(K)
            allm = ctx.all_moduli
            eb = uniform_limbs(gen, [allm[r] for r in rows], (dnum,), n)
            ea = uniform_limbs(gen, [allm[r] for r in rows], (dnum,), n)
            d2 = uniform_limbs(gen, ctx.moduli[sh.lo:sh.hi], (cb,), n)
            gat = torch.zeros(g * cb * sh.width * n, dtype=torch.int64, device="cuda")
            ks0 = ctx.empty(cb, sh.nlimbs, n)
            ks1 = ctx.empty(cb, sh.nlimbs, n)
            ws = ctx.workspace(lib.fhe_keyswitch_workspace(ctx.handle, sh.nlimbs, cb))

            def chunked():
                for _ in range(c):
                    ctx.intt(d2, limb0=sh.lo)
                    rc = lib.fhe_keyswitch_shard_ranked(
                        ctx.handle, ks0.data_ptr(), ks1.data_ptr(), gat.data_ptr(), g,
                        d2.data_ptr(), eb.data_ptr(), ea.data_ptr(), sh.lo, sh.nlimbs, cb,
                        ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
                    assert rc == 0, lib.fhe_last_error()

            comp = rate(chunked, warmup, steps) * 1e3
            peer = gb * sh.width * n * 8  # one peer's block of the group's whole gather
            recv = (g - 1) * peer
            direct = peer / (LINK_GBPS_DIR * 1e9) * 1e3 if g > 1 else 0.0
            ring = recv / (0.7 * (g - 1) * LINK_GBPS_DIR * 1e9) * 1e3 if g > 1 else 0.0
            ent = {"groups": groups, "limb_shards_g": g, "limbs_per_gpu": sh.nlimbs,
                   "ciphertexts_per_group": gb, "chunks": c, "compute_ms": round(comp, 4),
                   "recv_MB": round(recv / 1e6, 1)}
            for tag, cm in (("direct", direct), ("ring", ring)):
                step = cm / c + max(comp, cm * (c - 1) / c)
                ent[f"step_ms_{tag}"] = round(step, 4)
                ent[f"keyswitch_per_s_{tag}"] = round(B / step * 1e3, 1)
            res[f"G={G} g={g}"] = ent
            del eb, ea, d2, gat, ks0, ks1, ws
            torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--ks-batch", type=int, default=32, help="the key-switch leg's batch (bench.py)")
    ap.add_argument("--hybrid", action="store_true",
                    help="only the hybrid partition's rank shapes and model (fhe_dist_hybrid)")
    args = ap.parse_args()
    if args.hybrid:
        gen = torch.Generator(device="cuda")
        gen.manual_seed(6)
        print(json.dumps({"ks hybrid partition": hybrid_shapes(gen, args.ks_batch)}, indent=1))
        return
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
                         # each rank covers its limbs of all gb ciphertexts (bench.py hm_per_s)
                         "job_hommult_per_s_if_linear": round(gb / dt, 1),
                         "per_gpu_poly_limb_hommults_per_s": round(gb * sh.nlimbs / dt, 1),
                         "ntt_pair_ms": round(dn * 1e3, 4),
                         "per_gpu_ntt_per_s": round(2 * npolys * sh.nlimbs / dn, 1)}
        del a, b, d, ws, x
        torch.cuda.empty_cache()
    # key-switch leg, rank 0 of N: its limb shard of the leg's batch over a ranked gather region
    # filled with residues (timing only: the per-rank kernels of fhe_keyswitch_dist after its
    # gather).  "replicated P": the shipped partition (every rank extends into all K special
    # limbs); "P-sharded proxy": the same shard on a context with ceil(K / N) special primes, the
    # most loaded rank of a partition that deals the K special limbs out over the ranks (its
    # ModDown conversion reads 1 P row instead of K: a slight under-estimate of that rank's work).
    Lk, K, dnum, B = 16, 4, 4, args.ks_batch
    lib = load()
    kctxs = {}
    for G in (1, 2, 4, 8):
        for tag, kk in (("", K), (" P-sharded proxy", -(-K // G))):
            kctx = kctxs.get(kk) or kctxs.setdefault(kk, fc.Context(log_n, L=Lk, K=kk, dnum=dnum))
            sh = fdist.LimbShard(Lk, G, 0)
            rows = sh.evk_rows(kk)
            allm = kctx.all_moduli
            eb = uniform_limbs(gen, [allm[r] for r in rows], (dnum,), n)
            ea = uniform_limbs(gen, [allm[r] for r in rows], (dnum,), n)
            d2 = uniform_limbs(gen, kctx.moduli[sh.lo:sh.hi], (B,), n)
            gat = torch.zeros(G * B * sh.width * n, dtype=torch.int64, device="cuda")
            ks0 = kctx.empty(B, sh.nlimbs, n)
            ks1 = kctx.empty(B, sh.nlimbs, n)
            ws = kctx.workspace(lib.fhe_keyswitch_workspace(kctx.handle, sh.nlimbs, B))

            def ks():
                kctx.intt(d2, limb0=sh.lo)  # the rank's INTT of its own limbs ahead of the gather
                rc = lib.fhe_keyswitch_shard_ranked(kctx.handle, ks0.data_ptr(), ks1.data_ptr(),
                                                    gat.data_ptr(), G, d2.data_ptr(),
                                                    eb.data_ptr(), ea.data_ptr(), sh.lo,
                                                    sh.nlimbs, B, ws.data_ptr(),
                                                    torch.cuda.current_stream().cuda_stream)
                assert rc == 0, lib.fhe_last_error()

            dk = rate(ks, 20, 50)
            out[f"ks N={G}{tag}"] = {"limbs_per_gpu": sh.nlimbs, "special_limbs_per_gpu": kk,
                                     "batch": B, "ms_per_batch": round(dk * 1e3, 4)}
            del eb, ea, d2, gat, ks0, ks1, ws
    # the leg's chunking at N > 1 (fhe_keyswitch_dist: one call per chunk of the batch): rank 0's
    # share of the whole batch issued as chunks of B / c ciphertexts, c = 1, 2, 4 -- the launch
    # tails that more, smaller chunks cost against the gather time they let overlap
    kctx = kctxs[K]
    for G in (2, 4, 8):
        sh = fdist.LimbShard(Lk, G, 0)
        rows = sh.evk_rows(K)
        allm = kctx.all_moduli
        eb = uniform_limbs(gen, [allm[r] for r in rows], (dnum,), n)
        ea = uniform_limbs(gen, [allm[r] for r in rows], (dnum,), n)
        for c in (1, 2, 4):
            cb = B // c
            d2 = uniform_limbs(gen, kctx.moduli[sh.lo:sh.hi], (cb,), n)
            gat = torch.zeros(G * cb * sh.width * n, dtype=torch.int64, device="cuda")
            ks0 = kctx.empty(cb, sh.nlimbs, n)
            ks1 = kctx.empty(cb, sh.nlimbs, n)
            ws = kctx.workspace(lib.fhe_keyswitch_workspace(kctx.handle, sh.nlimbs, cb))

            def chunked():
                for _ in range(c):
                    kctx.intt(d2, limb0=sh.lo)
                    rc = lib.fhe_keyswitch_shard_ranked(
                        kctx.handle, ks0.data_ptr(), ks1.data_ptr(), gat.data_ptr(), G,
                        d2.data_ptr(), eb.data_ptr(), ea.data_ptr(), sh.lo, sh.nlimbs, cb,
                        ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
                    assert rc == 0, lib.fhe_last_error()

            out.setdefault(f"ks N={G} chunked", {})[f"{c} chunk(s) of {cb}"] = round(
                rate(chunked, 20, 50) * 1e3, 4)
            del d2, gat, ks0, ks1, ws
    base = out["ks N=1"]["ms_per_batch"]
    for G in (1, 2, 4, 8):
        for tag in ("", " P-sharded proxy"):
            out[f"ks N={G}{tag}"]["speedup_vs_N1_if_gather_hidden"] = round(
                base / out[f"ks N={G}{tag}"]["ms_per_batch"], 3)
    out["ks partition model"] = ks_partition_model(out, Lk, K, B, n)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--remodel":
        # recompute the model from a saved run's measured rank shapes (no GPU)
        with open(sys.argv[2]) as f:
            saved = json.load(f)
        saved["ks partition model"] = ks_partition_model(saved, 16, 4, saved["ks N=1"]["batch"],
                                                         1 << 16)
        print(json.dumps(saved, indent=1))
    else:
        main()
