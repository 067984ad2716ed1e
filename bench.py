#!/usr/bin/env python3
"""bench.py -- HomMult / NTT throughput of libfhecore on MI355X (BASELINE.json configs[2]).

Workload (one "step"): ct x ct HomMult (NTT -> tensor -> INTT, SURVEY.md §8a') at N = 2^16 with
8 RNS limbs over a batch of `--batch` ciphertext pairs per GPU, inputs resident in HBM.
Multi-GPU: one process per GPU (torch.distributed over RCCL); RNS limbs are sharded -- rank r owns
limbs [r L/G, (r+1) L/G) of every ciphertext of a global batch of batch*G pairs, so per-GPU work
is fixed ("scaling": "weak") and the data path has no collective.

Prints ONE JSON line (rank 0).  `value` = HomMult/s of the whole job; the NTT throughput
(forward length-2^16 single-limb transforms per second) and pipeline HBM figures ride along.
`roofline` is for the dominant kernel (hm_row_tensor: 4 row-forward passes + tensor + 3 row-inverse
passes, which reads 4 and writes 3 polynomials = the HomMult's algorithmic traffic), timed per
launch with HIP events recorded by libfhecore on the launch stream.  `cpu_baseline` is the exact C
restatement in oracle/ (OpenMP), run on rank 0 at N = 1 over a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fhecore as fc  # noqa: E402
from fhecore._capi import load  # noqa: E402

LOG_N, LIMBS = 16, 8
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, HBM3E peak)
METRIC = "NTTs/sec + HomMult/sec at N=2^16, 8 RNS limbs; achieved HBM GB/s vs peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="ct pairs per GPU per step")
    ap.add_argument("--ntt-polys", type=int, default=64, help="polys per NTT-throughput call")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def uniform_limbs(gen, moduli, lead):
    """Uniform residues in [0, q_l) per limb, int64 device tensor [*lead, len(moduli), N]."""
    n = 1 << LOG_N
    parts = []
    for q in moduli:
        # q < 2^61: draw 64-bit words and reduce on device (rejection-free, tiny bias is irrelevant
        # for throughput); exact uniformity is only needed by the parity tests, which use numpy.
        r = torch.randint(0, 2**62, (*lead, 1, n), generator=gen, dtype=torch.int64, device="cuda")
        parts.append(torch.remainder(r, q))
    return torch.cat(parts, dim=len(lead)).contiguous()


def prof_collect(max_marks=64):
    lib = load()
    ms = (ctypes.c_float * max_marks)()
    cnt = ctypes.c_uint32()
    names = ctypes.create_string_buffer(4096)
    fc._capi.check(lib.fhe_prof_end(ms, max_marks, ctypes.byref(cnt), names, 4096), "fhe_prof_end")
    nm = names.value.decode().split("\n")[: cnt.value]
    return list(zip(nm, [ms[i] for i in range(cnt.value)]))


def cpu_baseline(moduli, budget_s):
    """Exact C restatement (oracle/, test infrastructure) timed on this host: HomMult/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    rng = np.random.default_rng(0)
    n = 1 << LOG_N
    B = 2
    a = np.stack([np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in moduli])
                  for _ in range(2 * B)]).reshape(B, 2, LIMBS, n)
    b = a[::-1].copy()
    coracle.hommult(a[:1], b[:1], moduli)  # tables
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s:
        coracle.hommult(a, b, moduli)
        done += B
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "HomMult/s", "cores": threads, "kind": "port",
            "sample": f"{done} HomMults (N=2^16, L=8, exact C restatement oracle/fhe_oracle.c, "
                      f"OpenMP {threads} threads) in {dt:.1f} s"}


def traffic_from_profile(batch_local, nlimbs):
    """HBM bytes per hm_row_tensor launch from the committed PMC summary, when it was measured on
    this exact per-GPU shape (else null)."""
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    k = rec.get("hm_row_tensor")
    if not k or k.get("batch") != batch_local or k.get("nlimbs") != nlimbs:
        return None
    return k.get("bytes_per_launch")


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    if LIMBS % world:
        raise SystemExit("limbs must divide evenly across GPUs")
    nl = LIMBS // world
    limb0 = rank * nl
    n = 1 << LOG_N
    ctx = fc.Context(LOG_N, L=LIMBS)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234 + rank)
    gbatch = args.batch * world                      # ciphertext pairs per step, whole job
    mods = ctx.moduli[limb0:limb0 + nl]
    a = uniform_limbs(gen, mods, (gbatch, 2))
    b = uniform_limbs(gen, mods, (gbatch, 2))
    d = ctx.empty(gbatch, 3, nl, n)
    lib = load()
    ws = ctx.workspace(lib.fhe_hommult_workspace(ctx.handle, gbatch, nl))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    for _ in range(args.warmup):
        ctx.hommult(a, b, out=d, limb0=limb0, workspace=ws)
    barrier(world)
    fc._capi.check(lib.fhe_prof_begin(8 * args.steps + 8, stream), "fhe_prof_begin")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.hommult(a, b, out=d, limb0=limb0, workspace=ws)
    barrier(world)
    dt = time.perf_counter() - t0
    marks = prof_collect(8 * args.steps + 8)
    dt_max = max_over_ranks(dt, world)

    # per-kernel averages over the timed region
    per = {}
    for name, ms in marks:
        per.setdefault(name, []).append(ms)
    kavg = {k: sum(v) / len(v) for k, v in per.items()}
    dom = "hm_row_tensor"
    dom_ms = kavg.get(dom, float("nan"))
    # algorithmic bytes per launch of the dominant kernel: read 4 + write 3 polys of this rank's limbs
    alg_bytes = gbatch * 7 * nl * n * 8
    achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
    step_ms = dt_max / args.steps * 1e3
    hommult_per_s = gbatch * args.steps / dt_max  # every rank covers its limbs of all gbatch pairs
    # pipeline-level: whole HomMult algorithmic bytes (all 8 limbs) per second, per GPU
    pipe_gbps = hommult_per_s * 7 * LIMBS * n * 8 / 1e9 / world

    # NTT throughput: forward NTTs over this rank's limbs, batched
    x = uniform_limbs(gen, mods, (args.ntt_polys,))
    for _ in range(3):
        ctx.ntt_(x, limb0=limb0)
    barrier(world)
    t1 = time.perf_counter()
    nsteps = max(args.steps, 10)
    for _ in range(nsteps):
        ctx.ntt_(x, limb0=limb0)
    barrier(world)
    ntt_dt = max_over_ranks(time.perf_counter() - t1, world)
    ntt_per_s = args.ntt_polys * nl * world * nsteps / ntt_dt

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(ctx.moduli, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(hommult_per_s, 2),
            "unit": "HomMult/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (uniform residues per limb, seeded)",
            "config": {"workload": "hommult ct x ct (NTT -> tensor -> INTT), BASELINE configs[2]",
                       "log_n": LOG_N, "limbs": LIMBS, "batch_per_gpu": args.batch,
                       "global_batch": gbatch * 1, "parallelism": f"rns-limb-shard x{world}"},
            "ntt_per_sec": round(ntt_per_s, 1),
            "ntt_config": {"log_n": LOG_N, "polys": args.ntt_polys, "limbs_per_gpu": nl},
            "hommult_pipeline_hbm_gbps_per_gpu": round(pipe_gbps, 1),
            "hommult_pipeline_frac_of_peak": round(pipe_gbps / HBM_PEAK_GBPS, 4),
            "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic_from_profile(gbatch, nl),
                         "kernel": dom, "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
