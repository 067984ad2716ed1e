#!/usr/bin/env python3
"""bench.py -- HomMult / NTT / key-switch throughput of libfhecore on MI355X.

Default workload (BASELINE.json configs[2], what `value` reports): ct x ct HomMult
(NTT -> tensor -> INTT, SURVEY.md §8a') at N = 2^16 with 8 RNS limbs over a batch of `--batch`
ciphertext pairs per GPU, inputs resident in HBM.  One "step" = one HomMult pass over the batch.
Multi-GPU: one process per GPU (torch.distributed over RCCL); RNS limbs are sharded -- rank r owns
limbs [r L/G, (r+1) L/G) of every ciphertext of a global batch of batch*G pairs, so per-GPU work
is fixed ("scaling": "weak") and the HomMult data path has no collective.

Other workloads (`--workload`): `ntt` (forward + inverse negacyclic NTT, N = 2^16, 8 limbs) and
`keyswitch` (BASELINE configs[3]: N = 2^16, L = 16, K = 4, dnum = 4, limbs sharded across the
ranks with one RCCL all-gather of INTT(d2) per key-switch).

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel of the workload, timed per
launch with HIP events that libfhecore records on the launch stream (fhe_prof_begin/end);
`achieved` = its algorithmic bytes per launch / its mean launch time.  `cpu_baseline` is the exact
C restatement in oracle/ (OpenMP), run on rank 0 at N = 1 over a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fhecore as fc  # noqa: E402
from fhecore import dist as fdist  # noqa: E402
from fhecore._capi import check, load  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "NTTs/sec + HomMult/sec at N=2^16, 8 RNS limbs; achieved HBM GB/s vs peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the chip ramps its clock up over the first ~50 ms of sustained load: short warmups measure the
    # ramp (W=5, K=20 reads ~15 % low at N=2^16, L=8); the defaults time the sustained rate
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--workload", choices=["hommult", "ntt", "keyswitch", "mulrelin", "ntt-batch",
                                           "vec", "rotate", "rotsum", "lintrans"],
                    default="hommult")
    ap.add_argument("--batch", type=int, default=None,
                    help="ciphertexts per GPU per step (default 64 for hommult -- the throughput "
                         "batch: +3.5 %% over 16, fewer launch tails --, 32 for mulrelin and rotate "
                         "-- the key-switch's best batch -- and 16 for the others)")
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--bits", type=int, default=60, choices=[60, 61, 62, 63],
                    help="hommult: modulus chain of the largest primes below 2^bits (62, 63: the "
                         "exact wide-modulus butterflies)")
    ap.add_argument("--ks-chunks", type=int, default=0,
                    help="keyswitch: all-gather chunks per batch (0 = 1 at N = 1, 4 above)")
    ap.add_argument("--ks-groups", type=int, default=1,
                    help="keyswitch: ciphertext groups of the hybrid partition (fhe_dist_hybrid): "
                         "the ranks form this many groups of N / groups limb shards, each group "
                         "key-switches its share of the batch with the all-gather inside the group "
                         "(1 = the limb-only partition, north_star's; N = whole ciphertexts per GPU)")
    ap.add_argument("--ks-batch", type=int, default=32,
                    help="keyswitch (and the default line's key-switch leg): ciphertexts per "
                         "call, the whole job's (limbs sharded: strong scaling)")
    ap.add_argument("--inverse", action="store_true",
                    help="ntt-batch: time the inverse transform (configs[4]'s round trip back) "
                         "instead of the forward")
    ap.add_argument("--no-keyswitch-leg", action="store_true",
                    help="hommult: skip the key-switch ride-along leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dist-check", action="store_true",
                    help="skip the closing dist_check (profiling runs: its small launches would "
                         "mix into the per-kernel averages)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="hommult: skip the live rocprofv3 traffic passes (roofline.traffic then "
                         "falls back to the committed profiles/hbm_traffic.json)")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # FHE_BENCH_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU (the
    # driver's runs use RCCL, one rank per GPU)
    backend = os.environ.get("FHE_BENCH_BACKEND", "nccl")
    dev = local % torch.cuda.device_count() if backend != "nccl" else local
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            torch.distributed.init_process_group(backend)
    return world, rank


def barrier(world):
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    nccl = torch.distributed.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if nccl else "cpu")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def uniform_limbs(gen, moduli, lead, n):
    """Residues in [0, q_l) per limb: int64 device tensor [*lead, len(moduli), n]."""
    parts = []
    for q in moduli:
        r = torch.randint(0, 2**62, (*lead, 1, n), generator=gen, dtype=torch.int64, device="cuda")
        parts.append(torch.remainder(r, q))
    return torch.cat(parts, dim=len(lead)).contiguous()


def timed(fn, args, world, max_marks):
    """Warmup, then exactly `steps` calls between barrier+sync brackets with nothing else on the
    stream; then the same `steps` calls again with a HIP-event mark after each launch group, whose
    averages are the per-kernel durations (kernel_ms, roofline.achieved).  The marks stay out of
    the timed window: each record costs ~4 us of idle GPU between kernels (rocprofv3 trace,
    DESIGN.md §6)."""
    for _ in range(args.warmup):
        fn()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fn()
    barrier(world)
    dt = time.perf_counter() - t0
    lib = load()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    check(lib.fhe_prof_begin(max_marks, stream), "fhe_prof_begin")
    for _ in range(args.steps):
        fn()
    barrier(world)
    ms = (ctypes.c_float * max_marks)()
    cnt = ctypes.c_uint32()
    names = ctypes.create_string_buffer(32 * max_marks + 64)
    check(lib.fhe_prof_end(ms, max_marks, ctypes.byref(cnt), names, 32 * max_marks + 64),
          "fhe_prof_end")
    per = {}
    for nm, v in zip(names.value.decode().split("\n"), ms[: cnt.value]):
        per.setdefault(nm, []).append(v)
    return max_over_ranks(dt, world), {k: sum(v) / len(v) for k, v in per.items()}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """OpenMP threads the baseline runs with: OMP_NUM_THREADS (the GPU box allots 16 host CPUs per
    GPU and sets it), else every CPU this process may run on."""
    return int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))


def cpu_host():
    """What the cpu_baseline ran on: the model, the threads used, the CPUs this process may use
    (sched_getaffinity) and the machine's total (os.cpu_count: the whole box, shared)."""
    omp = os.environ.get("OMP_NUM_THREADS")
    why = (f"OMP_NUM_THREADS={omp} is set by the GPU box, which allots that many host CPUs to "
           "each GPU; the affinity mask and cpu_count show the whole shared machine, so using them "
           "would time CPUs allotted to other jobs" if omp else
           "OMP_NUM_THREADS unset: every CPU of the affinity mask")
    return {"cpu_model": cpu_model(), "threads": cpu_threads(),
            "affinity_cpus": len(os.sched_getaffinity(0)), "host_cpus": os.cpu_count(),
            "threads_why": why}


def cpu_baseline_hommult(moduli, log_n, budget_s):
    """The tuned CPU port (oracle/fhe_cpu_port.c: lazy Harvey NTTs with Shoup twiddles,
    Montgomery tensor, no 128-bit division, no per-limb allocation; OpenMP over (ciphertext,
    limb)), bit-exact with the checker (tests/test_oracle.py), timed on this host: HomMult/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402

    threads = cpu_threads()
    rng = np.random.default_rng(0)
    n, L, B = 1 << log_n, len(moduli), max(4, threads // 2)
    a = np.stack([np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in moduli])
                  for _ in range(2 * B)]).reshape(B, 2, L, n)
    b = a[::-1].copy()
    d = np.empty((B, 3, L, n), dtype=np.uint64)
    coracle.port_hommult_into(d[:1], a[:1], b[:1], moduli)  # twiddle tables outside the sample
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s:
        coracle.port_hommult_into(d, a, b, moduli)
        done += B
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 2), "unit": "HomMult/s", "cores": threads, "kind": "port",
            **cpu_host(),
            "sample": f"{done} HomMults (N=2^{log_n}, L={L}, batches of {B}) by the tuned C port "
                      f"oracle/fhe_cpu_port.c (bit-exact with the checker), OpenMP {threads} "
                      f"threads, in {dt:.1f} s"}


def traffic_from_profile(kernel, shape):
    """HBM bytes per launch of `kernel` from profiles/hbm_traffic.json when it was measured on
    this exact per-GPU shape (FETCH_SIZE/WRITE_SIZE passes, corrected as MI355X_MICROARCH.md
    §HBM prescribes); otherwise null.  Returns (bytes, source)."""
    path = os.path.join("profiles", "hbm_traffic.json")
    try:
        with open(os.path.join(ROOT, path)) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None, None
    rec = tab.get(kernel)
    if not rec or rec.get("shape") != shape or rec.get("bytes_per_launch") is None:
        return None, None
    return rec["bytes_per_launch"], (f"committed, not measured in this run: {path} = "
                                     f"{tab.get('_source', 'rocprofv3 PMC passes')}, same kernel "
                                     "and per-GPU shape")


def profiled_parent(environ=None):
    """Why this process runs under a profiler, or None.  rocprofv3 starts its target with the
    rocprofiler-sdk tool library in LD_PRELOAD and its settings in ROCPROF* / ROCP_* variables;
    that library initialises the GPU before the target's first line runs.  A nested rocprofv3
    started from such a process inherits the preload, so its own launcher has initialised the GPU
    when it execs the probe -- an exec the GPU box refuses (round 4: tools/kspmc.sh profiled
    bench.py, whose live PMC passes then exited 126)."""
    env = os.environ if environ is None else environ
    # only the preload is the hazard (a nested launcher inherits it); ROCPROF* / ROCP_* settings
    # alone -- e.g. left in a login environment -- start nothing and must not switch off the live
    # passes (advisor r5)
    if "rocprof" in env.get("LD_PRELOAD", ""):
        return "LD_PRELOAD names the rocprofiler tool library"
    return None


def rocprof_pmc(counters, probe, probe_args, timeout_s=150):
    """One `rocprofv3 --pmc <counters>` pass (no tracing) over a child process running
    tools/<probe> with `probe_args`: the child is started with Popen in its own session and killed
    with its group on timeout.  rocprofv3's launcher then execs the probe's interpreter, which is
    only safe while nothing in that launcher has touched the GPU: when this process itself runs
    under a profiler (profiled_parent), the launcher would inherit the profiler's preload, so the
    pass is skipped without starting anything.  Returns (rows, stdout, None) -- rows of (kernel
    name, counter, value) per dispatch -- or (None, None, reason)."""
    import csv
    import glob
    import shutil
    import signal
    import subprocess
    import tempfile
    nested = profiled_parent()
    if nested:
        return None, None, f"skipped: this process runs under a profiler ({nested}); a nested " \
                           "rocprofv3 would exec its target after the GPU was initialised"
    prof = shutil.which("rocprofv3") or (
        "/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if not prof:
        return None, None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="fhe_pmc_", dir="/tmp")
    try:
        cmd = [prof, "--pmc", *counters, "-d", tmp, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.join(ROOT, "tools", probe), *probe_args]
        env = dict(os.environ, TMPDIR="/tmp")
        proc = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE,
                                stderr=subprocess.DEVNULL, start_new_session=True, text=True)
        try:
            out, _ = proc.communicate(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait()
            return None, None, f"rocprofv3 --pmc {' '.join(counters)} timed out after {timeout_s} s"
        if proc.returncode != 0:
            return None, None, f"rocprofv3 --pmc {' '.join(counters)} exited with {proc.returncode}"
        rows = []
        for f in glob.glob(os.path.join(tmp, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    rows.append((r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])))
        return rows, out, None
    except (OSError, ValueError, KeyError) as e:
        return None, None, f"PMC pass failed: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def measure_traffic_live(kernel_match, probe_args, timeout_s=150):
    """HBM bytes per launch of the kernel whose name contains `kernel_match`, measured in this run:
    two rocprofv3 passes (--pmc FETCH_SIZE, then --pmc WRITE_SIZE, one counter group each, no
    tracing) over a child process that repeats the launch at the bench shape
    (tools/hm_traffic_probe.py), corrected as MI355X_MICROARCH.md's HBM section prescribes and as
    tools/pmc_traffic.sh calibrated on the column pass: read = 2 x FETCH_SIZE KiB, write =
    WRITE_SIZE KiB.  Returns (bytes, None) or (None, reason)."""
    per = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        rows, _, why = rocprof_pmc([counter], "hm_traffic_probe.py", probe_args, timeout_s)
        if rows is None:
            return None, why
        vals = [v for k, c, v in rows if kernel_match in k and c == counter]
        if not vals:
            return None, f"no {kernel_match} dispatch in the {counter} pass"
        per[counter] = sum(vals) / len(vals)
    return int(2 * 1024 * per["FETCH_SIZE"] + 1024 * per["WRITE_SIZE"]), None


def measure_hommult_valu_live(log_n, limbs, batch, kernel_ms, timeout_s=150):
    """VALU issue of k_hommult_row measured in this run: one `rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES
    GRBM_GUI_ACTIVE` pass over tools/hm_traffic_probe.py --peak (the HomMult at the bench shape, then
    the butterfly ceiling kernels in the same process).  VALU instructions per launch over this
    run's HIP-event time give the achieved rate; the ceiling is the faster of the two ceiling
    kernels; GRBM_GUI_ACTIVE per dispatch / 8 XCDs / duration gives each kernel's clock, so
    `frac_per_cycle` = frac x ceiling clock / kernel clock separates issue efficiency from clock.
    Returns (dict, None) or (None, reason)."""
    rows, out, why = rocprof_pmc(["SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE"],
                                 "hm_traffic_probe.py",
                                 ["--log-n", str(log_n), "--limbs", str(limbs), "--batch",
                                  str(batch), "--peak"], timeout_s)
    if rows is None:
        return None, why
    try:
        meta = json.loads(out.strip().splitlines()[-1])
        peak_ms = meta["peak_ms_per_launch"]
    except (ValueError, IndexError, KeyError):
        return None, "hm_traffic_probe printed no result line"
    per = {}
    for k, c, v in rows:
        key = ("hm" if "k_hommult_row" in k else "inverse" if "k_bfly_peak<true>" in k
               else "forward" if "k_bfly_peak<false>" in k else None)
        if key:
            per.setdefault(key, {}).setdefault(c, []).append(v)
    mean = lambda key, c: sum(per[key][c]) / len(per[key][c])  # noqa: E731
    try:
        hm_valu, hm_grbm = mean("hm", "SQ_INSTS_VALU"), mean("hm", "GRBM_GUI_ACTIVE")
        ceil = {k: (mean(k, "SQ_INSTS_VALU") / (peak_ms[k] * 1e-3) / 1e9,
                    mean(k, "GRBM_GUI_ACTIVE") / 8 / (peak_ms[k] * 1e-3) / 1e9)
                for k in ("forward", "inverse")}
    except (KeyError, ZeroDivisionError):
        return None, "no k_hommult_row or ceiling dispatches in the VALU pass"
    ceil_rate, ceil_clock = max(ceil.values())
    achieved = hm_valu / (kernel_ms * 1e-3) / 1e9
    clock = hm_grbm / 8 / (kernel_ms * 1e-3) / 1e9
    frac = achieved / ceil_rate
    return {"bound": "valu", "achieved": round(achieved, 1), "peak": round(ceil_rate, 1),
            "unit": "G VALU wave-instructions/s", "frac": round(frac, 4),
            "kernel": "hm_row_tensor (k_hommult_row)", "valu_instr_per_launch": round(hm_valu),
            "clock_ghz": round(clock, 3), "peak_clock_ghz": round(ceil_clock, 3),
            "frac_per_cycle": round(frac * ceil_clock / clock, 4) if clock else None,
            "valu_source": "measured in this run: rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES "
                           "GRBM_GUI_ACTIVE over tools/hm_traffic_probe.py --peak (same shape; "
                           "ceiling = k_bfly_peak in that process); time from this run's HIP "
                           "events"}, None


def measure_keyswitch_valu_live(log_n, batch, chunks=1, timeout_s=150):
    """SQ_INSTS_VALU of one key-switch call at the leg's shape and chunking, measured in this run: one
    `rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES` pass over tools/ks_valu_probe.py, which makes a few
    fhe_keyswitch_dist calls and then runs the butterfly ceiling kernels (bfly_peak.hip) in the same
    process.  Returns ({per-kernel VALU per call}, ceiling G VALU wave-instructions/s, None) or
    (None, None, reason)."""
    rows, out, why = rocprof_pmc(["SQ_INSTS_VALU", "SQ_WAVES"], "ks_valu_probe.py",
                                 ["--log-n", str(log_n), "--batch", str(batch),
                                  "--chunks", str(chunks)], timeout_s)
    if rows is None:
        return None, None, why
    try:
        meta = json.loads(out.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return None, None, "ks_valu_probe printed no result line"
    short = lambda k: k.replace("void fhe::(anonymous namespace)::", "").replace(  # noqa: E731
        "void (anonymous namespace)::", "").split("(")[0]
    tot, cnt = {}, {}
    for k, c, v in rows:
        if c != "SQ_INSTS_VALU":
            continue
        tot[short(k)] = tot.get(short(k), 0.0) + v
        cnt[short(k)] = cnt.get(short(k), 0) + 1
    ks = {k: v / meta["calls"] for k, v in tot.items()
          if "fhe::" in k or (k.startswith("k_") and "bfly_peak" not in k)}
    ceil = 0.0
    for k, v in tot.items():
        if k.startswith("k_bfly_peak"):
            ms = meta["peak_ms_per_launch"]["inverse" if "<true>" in k else "forward"]
            ceil = max(ceil, v / cnt[k] / (ms * 1e-3) / 1e9)
    if not ks or not ceil:
        return None, None, "no key-switch or ceiling dispatches in the PMC pass"
    return ks, ceil, None


def measure_keyswitch_traffic_live(log_n, batch, chunks=1, timeout_s=150):
    """HBM bytes of one key-switch call (every kernel it launches) at the leg's shape, measured in
    this run: a --pmc FETCH_SIZE pass and a --pmc WRITE_SIZE pass (separate: the two do not fit
    one pass) over tools/ks_valu_probe.py --no-peak, summed over the calls' dispatches and divided
    by the calls; read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB (the gfx950 correction, as
    measure_traffic_live).  Returns ({kernel: bytes per call}, total bytes per call, None) or
    (None, None, reason)."""
    short = lambda k: k.replace("void fhe::(anonymous namespace)::", "").replace(  # noqa: E731
        "void fhe::", "").split("(")[0]
    per, calls = {}, None
    for counter, scale in (("FETCH_SIZE", 2048), ("WRITE_SIZE", 1024)):
        rows, out, why = rocprof_pmc([counter], "ks_valu_probe.py",
                                     ["--log-n", str(log_n), "--batch", str(batch),
                                      "--chunks", str(chunks), "--no-peak"], timeout_s)
        if rows is None:
            return None, None, why
        try:
            calls = json.loads(out.strip().splitlines()[-1])["calls"]
        except (ValueError, IndexError, KeyError):
            return None, None, "ks_valu_probe printed no result line"
        for k, c, v in rows:
            if c == counter and "fhe::" in k and "bfly_peak" not in k:
                per[short(k)] = per.get(short(k), 0.0) + v * scale
    if not per or not calls:
        return None, None, "no key-switch dispatches in the traffic passes"
    per = {k: v / calls for k, v in per.items()}
    return per, int(sum(per.values())), None


def roofline(kernel, alg_bytes, ms, shape):
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    traffic, src = traffic_from_profile(kernel, shape)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
            "traffic_source": src, "kernel": kernel, "alg_bytes_per_launch": alg_bytes,
            "kernel_ms": round(ms, 4)}


def transform_roofline(kavg, alg_bytes, shape):
    """HBM roofline of whole NTTs (2 x 8 x N algorithmic bytes per transform)
    against the summed mean time of every pass launch of one step (column + row, and both
    directions when the step runs both): what the transform achieves, not one pass of it."""
    ms = sum(kavg.values())
    out = roofline(" + ".join(kavg) + " (whole transform)", alg_bytes, ms, shape)
    out["passes"] = sorted(kavg)
    return out


_PEAKS = {}


def alu_peaks():
    """Butterflies/s ceilings of the NTT arithmetic on this GPU (tools/microbench/bfly_peak.hip:
    the kernels' exact forward CT / inverse GS instruction sequences, register-resident, full
    occupancy, no memory traffic), measured once per process on the warmed-up chip."""
    if not _PEAKS:
        lib = ctypes.CDLL(os.environ.get("FHE_PEAK_LIB") or
                          os.path.join(ROOT, "tools", "microbench", "libbflypeak.so"))
        lib.fhe_peak_bfly.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double)]
        blocks = 8 * torch.cuda.get_device_properties(0).multi_processor_count
        for inv in (0, 1):
            rate, ms = ctypes.c_double(), ctypes.c_double()
            if lib.fhe_peak_bfly(inv, blocks, 256, 20, ctypes.byref(rate), ctypes.byref(ms)):
                raise RuntimeError("fhe_peak_bfly failed")
            _PEAKS["inv" if inv else "fwd"] = rate.value
    return _PEAKS


def row_bflies(log_n):
    """Butterflies in one row pass of one poly-limb (the last log R2 stages of N = R1 x R2)."""
    return (1 << log_n) // 2 * (log_n - log_n // 2)


def roofline_alu(kernel, fwd_bflies, inv_bflies, ms, valu_per_bfly=None):
    """Integer-ALU roofline of a launch that runs `fwd_bflies` forward and `inv_bflies` inverse
    butterflies in `ms`: the ceiling time at the measured butterfly rates vs the measured time."""
    pk = alu_peaks()
    t_ceil = fwd_bflies / pk["fwd"] + inv_bflies / pk["inv"]
    total = fwd_bflies + inv_bflies
    achieved = total / (ms * 1e-3) / 1e12
    peak = total / t_ceil / 1e12
    out = {"bound": "valu", "achieved": round(achieved, 4), "peak": round(peak, 4),
           "unit": "Tbutterfly/s", "frac": round(achieved / peak, 4), "kernel": kernel,
           "butterflies_per_launch": {"forward": fwd_bflies, "inverse": inv_bflies},
           "peak_source": "tools/microbench/bfly_peak.hip, measured in this run "
                          f"(forward {pk['fwd'] / 1e12:.3f}, inverse {pk['inv'] / 1e12:.3f} "
                          "Tbutterfly/s)"}
    if valu_per_bfly:
        out["valu_instr_per_butterfly"] = valu_per_bfly
    return out


def run_hommult(args, world, rank):
    """The headline line (BASELINE configs[2]) with two ride-along legs that share its process:
    the NTTs/sec half of the metric (forward + inverse NTTs, N = 2^16, 8 limbs) and the configs[3]
    key-switch through the native RCCL path (fhe_keyswitch_dist: limbs sharded over the ranks, one
    all-gather per chunk), so that the driver's 1 -> 8 GPU runs also measure the only collective.
    Order: everything is allocated first; the NTT leg runs first (it also brings the chip to its
    sustained clock, which the driver's short --warmup would otherwise leave inside the timed
    region: DESIGN.md §8 "Warmup matters"), then the HomMult leg (W warmup + exactly K timed
    steps), then the key-switch leg."""
    L = 8
    shard = fdist.LimbShard(L, world, rank)
    n = 1 << args.log_n
    mods = fc.gen_moduli(args.log_n, L, bits=args.bits) if args.bits != 60 else None
    ctx = fc.Context(args.log_n, moduli=mods) if mods else fc.Context(args.log_n, L=L)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234 + rank)
    gbatch = args.batch * world  # ciphertext pairs per step, whole job
    mods = ctx.moduli[shard.lo:shard.hi]
    a = uniform_limbs(gen, mods, (gbatch, 2), n)
    b = uniform_limbs(gen, mods, (gbatch, 2), n)
    d = ctx.empty(gbatch, 3, shard.nlimbs, n)
    ws = ctx.workspace(load().fhe_hommult_workspace(ctx.handle, gbatch, shard.nlimbs))
    step = lambda: fdist.sharded_hommult(ctx, a, b, shard, out=d, workspace=ws)  # noqa: E731
    # NTT throughput rides along (BASELINE metric "NTTs/sec"): forward + inverse NTTs of 512
    # poly-limbs per GPU (64 polys x 8 limbs at N = 1; the same count of this rank's limbs above, so
    # per-GPU work stays fixed like the HomMult leg's), sustained, every NTT counted
    npolys = 64 * L // max(shard.nlimbs, 1)
    x = uniform_limbs(gen, mods, (npolys,), n)

    def ntt_pair():
        ctx.ntt_(x, limb0=shard.lo)
        ctx.intt_(x, limb0=shard.lo)

    nargs = argparse.Namespace(warmup=100, steps=200)
    ntt_dt, ntt_k = timed(ntt_pair, nargs, world, 8 * nargs.steps + 8)
    ntt_per_s = 2 * npolys * shard.nlimbs * world * nargs.steps / ntt_dt

    dt, kavg = timed(step, args, world, 8 * args.steps + 8)
    hm_per_s = gbatch * args.steps / dt  # each rank covers its limbs of all gbatch pairs
    shape = {"log_n": args.log_n, "batch": gbatch, "nlimbs": shard.nlimbs}
    # dominant kernel: reads 4 and writes 3 polynomials of this rank's limbs = algorithmic traffic
    dom = "hm_row_tensor"
    alg = gbatch * 7 * shard.nlimbs * n * 8
    pipe_gbps = hm_per_s * 7 * L * n * 8 / 1e9 / world
    out = {
        "metric": METRIC, "value": round(hm_per_s, 2), "unit": "HomMult/s",
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "config": {"workload": "hommult ct x ct (NTT -> tensor -> INTT), BASELINE configs[2]",
                   "log_n": args.log_n, "limbs": L, "batch_per_gpu": args.batch,
                   "global_batch": gbatch, "parallelism": f"rns-limb-shard x{world}"},
        "ntt_per_sec": round(ntt_per_s, 1),
        "ntt_config": {"log_n": args.log_n, "direction": "forward+inverse", "polys_per_gpu": npolys,
                       "limbs_per_gpu": shard.nlimbs, "warmup": nargs.warmup,
                       "steps": nargs.steps, "order": "run before the HomMult leg"},
        "ntt_kernel_ms": {k: round(v, 4) for k, v in ntt_k.items()},
        "hommult_pipeline_hbm_gbps_per_gpu": round(pipe_gbps, 1),
        "hommult_pipeline_frac_of_peak": round(pipe_gbps / HBM_PEAK_GBPS, 4),
        "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
        "roofline": roofline(dom, alg, kavg.get(dom, float("nan")), shape),
    }
    # algorithmic bytes exclude the twiddles (cache-resident), reported separately:
    # the forward and inverse row tables of this rank's limbs, (w, w') pairs of 16 B, N per limb
    tw = 2 * shard.nlimbs * n * 16
    rf = out["roofline"]
    rf["twiddle_bytes_per_launch"] = tw
    rf["achieved_with_twiddles"] = round((alg + tw) / (rf["kernel_ms"] * 1e-3) / 1e9, 1)
    rf["frac_with_twiddles"] = round(rf["achieved_with_twiddles"] / HBM_PEAK_GBPS, 4)
    # the fused row kernel is limited by VALU issue: its integer-ALU roofline, and
    # the same for the whole pipeline (7 full NTTs per ct x ct limb)
    units = gbatch * shard.nlimbs
    rb = row_bflies(args.log_n)
    if not args.bits > 60:  # the ceiling kernel runs the lazy (q < 2^61) arithmetic
        out["roofline_alu"] = roofline_alu(dom, 4 * rb * units, 3 * rb * units,
                                           kavg.get(dom, float("nan")),
                                           {"forward": 16.25, "inverse": 18.2})  # lz16 row passes, round averages (bfly_peak.hip)
        full = (n // 2) * args.log_n
        out["hommult_pipeline_alu"] = roofline_alu("hm_col_fwd + hm_row_tensor + hm_col_inv",
                                                   4 * full * units, 3 * full * units,
                                                   sum(kavg.values()))
    out["limiter"] = "valu" if out.get("roofline_alu", {}).get("frac", 0) > \
        out["roofline"]["frac"] else "hbm"
    if args.bits != 60:
        out["config"]["modulus_bits"] = args.bits
    # HBM traffic of the dominant kernel measured in this run (rank 0 of a one-GPU job only: the
    # profiled child shares the GPU); the committed figure stays beside it for comparison
    if rank == 0 and world == 1 and not args.no_pmc and args.bits == 60:
        live, why = measure_traffic_live("k_hommult_row", [
            "--log-n", str(args.log_n), "--limbs", str(L), "--batch", str(gbatch)])
        if live is not None:
            rf["traffic_committed"], rf["traffic"] = rf["traffic"], live
            rf["traffic_source"] = (
                "measured in this run: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes "
                "(separate) over tools/hm_traffic_probe.py at this shape, k_hommult_row mean per "
                "dispatch; read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB (gfx950 correction)")
            rf["traffic_over_alg"] = round(live / alg, 4)
            rf["traffic_over_alg_with_twiddles"] = round(live / (alg + tw), 4)
        else:
            rf["traffic_live_error"] = why
        valu, why = measure_hommult_valu_live(args.log_n, L, gbatch, rf["kernel_ms"])
        out["roofline_valu"] = valu if valu is not None else {"valu_live_error": why,
                                                               "frac": None}
    legs = {}
    if not (args.no_keyswitch_leg or args.bits != 60):
        def ks_leg():
            legs["ks"] = KeyswitchLeg(args, world, rank)
            return legs["ks"].run(argparse.Namespace(warmup=20, steps=50))

        out["keyswitch_leg"] = guarded_leg(ks_leg, out, rank, "keyswitch_leg")
        # the profiled child pass runs outside the watchdog: it has its own time limit, after
        # which it is killed and the committed profile stands in
        if "ks" in legs and "error" not in out["keyswitch_leg"] and world == 1:
            try:
                out["keyswitch_leg"]["roofline_valu"] = legs["ks"].valu_roofline()
            except Exception as e:  # noqa: BLE001 -- a measurement, never a reason to fail the line
                out["keyswitch_leg"]["roofline_valu"] = {"valu_live_error": repr(e), "frac": None}
            try:
                legs["ks"].traffic(out["keyswitch_leg"])
            except Exception as e:  # noqa: BLE001 -- as above
                out["keyswitch_leg"]["roofline"]["traffic_live_error"] = repr(e)
    # after every timed leg: the sharded paths against each rank's single-device result
    if not args.no_dist_check:
        out["dist_check"] = guarded_leg(lambda: dist_check(world, rank, hm_ctx=ctx,
                                                           ks_leg=legs.get("ks")),
                                        out, rank, "dist_check")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_hommult(ctx.moduli, args.log_n, args.cpu_seconds)
    return out, cpu


def run_vec(args, world, rank):
    """The reference's own operators (vec_add / vec_sub / vec_mul, /root/reference/arithmetic.py:3-13,
    = poly_mul_pointwise in the NTT domain) through the context kernel k_vec_ctx: one step = one
    add, one sub and one mul over `batch` polynomials x 8 limbs x N = 2^16 on this rank's limbs.
    HBM-bound: 24 B per coefficient per op (two reads, one write)."""
    L = 8
    shard = fdist.LimbShard(L, world, rank)
    n = 1 << args.log_n
    ctx = fc.Context(args.log_n, L=L)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5 + rank)
    mods = ctx.moduli[shard.lo:shard.hi]
    polys = 2 * args.batch
    # one (a, b, out) set per operator, 384 MiB each at the default shape: an operator's inputs
    # were last touched two operators (768 MiB) earlier, so they stream from HBM rather than from
    # the 256 MB Infinity Cache
    sets = []
    for _ in range(3):
        a = uniform_limbs(gen, mods, (polys,), n)
        sets.append((a, uniform_limbs(gen, mods, (polys,), n), torch.empty_like(a)))
    lib = load()

    def step():
        for fn, (a, b, out) in zip((lib.fhe_vec_add, lib.fhe_vec_sub, lib.fhe_vec_mul), sets):
            check(fn(ctx.handle, out.data_ptr(), a.data_ptr(), b.data_ptr(), polys, shard.lo,
                     shard.nlimbs, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
                  "fhe_vec")

    dt, kavg = timed(step, args, world, 8 * args.steps + 8)
    coeffs = polys * shard.nlimbs * n
    per_op = coeffs * 24
    ops_per_s = 3 * coeffs * world * args.steps / dt
    out_line = {"metric": "vec_add/vec_sub/vec_mul coefficients/sec at N=2^16, 8 RNS limbs (HBM-bound)",
                "value": round(ops_per_s, 1), "unit": "coeff-op/s",
                "ms_per_step": round(dt / args.steps * 1e3, 4),
                "config": {"workload": "reference vec_add + vec_sub + vec_mul (k_vec_ctx)",
                           "log_n": args.log_n, "limbs": L, "polys_per_gpu": polys,
                           "parallelism": f"rns-limb-shard x{world}"},
                "kernel_ms": {k: round(v, 4) for k, v in kavg.items()}}
    for k, v in kavg.items():
        out_line["roofline_" + k] = roofline(k, per_op, v, {"log_n": args.log_n, "polys": polys})
    dom = max(kavg, key=kavg.get)
    out_line["roofline"] = roofline(dom, per_op, kavg[dom], {"log_n": args.log_n, "polys": polys})
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_vec(ctx.moduli, args.log_n, args.cpu_seconds)
    return out_line, cpu


def cpu_baseline_vec(moduli, log_n, budget_s):
    """The reference's vec_add / vec_sub / vec_mul (/root/reference/arithmetic.py:3-13) on this
    host: the tuned C port (oracle/fhe_cpu_port.c port_vec_op: exact, OpenMP over rows, no `%`;
    bit-exact with the checker, tests/test_oracle.py) over 64 polys x 8 limbs x N, one add + one
    sub + one mul per step like the GPU leg: coefficient-ops/s.  Beside it, the reference's own
    numpy expression `(a op b) % MOD` on uint64 (single thread, what arithmetic.py executes; wrong
    for sub when a < b and for every 60-bit mul), timed on a smaller sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402

    rng = np.random.default_rng(5)
    n, L, P = 1 << log_n, len(moduli), 64
    a = np.stack([rng.integers(0, q, (P, n), dtype=np.uint64) for q in moduli], axis=1)
    b = np.stack([rng.integers(0, q, (P, n), dtype=np.uint64) for q in moduli], axis=1)
    a2, b2 = a.reshape(P * L, n), b.reshape(P * L, n)
    rowm = np.tile(np.asarray(moduli, dtype=np.uint64), P)
    out = np.empty_like(a2)
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s:
        for op in ("add", "sub", "mul"):
            coracle.port_vec_op(op, a2, b2, rowm, out=out)
        done += 3 * a2.size
    dt = time.perf_counter() - t0
    # the reference's numpy expression, single-threaded, on 8 polys x 8 limbs
    qa, qb = a[:8], b[:8]
    qm = np.asarray(moduli, dtype=np.uint64)[None, :, None]
    t1 = time.perf_counter()
    ref_done = 0
    while time.perf_counter() - t1 < min(2.0, budget_s):
        np.remainder(np.add(qa, qb), qm)
        np.remainder(np.subtract(qa, qb), qm)
        np.remainder(np.multiply(qa, qb), qm)
        ref_done += 3 * qa.size
    rdt = time.perf_counter() - t1
    return {"value": round(done / dt, 1), "unit": "coeff-op/s", "cores": cpu_threads(),
            "kind": "port", **cpu_host(),
            "sample": f"{done / 3 / a2.size:.0f} steps of add + sub + mul over {P} polys x {L} limbs "
                      f"x N=2^{log_n} by the tuned C port (port_vec_op, exact), OpenMP "
                      f"{cpu_threads()} threads, in {dt:.1f} s",
            "reference_numpy_uint64": {
                "value": round(ref_done / rdt, 1), "unit": "coeff-op/s", "cores": 1,
                "note": "the reference's own expression (a op b) % MOD with numpy uint64 "
                        "(/root/reference/arithmetic.py:3-13), 8 polys x 8 limbs, "
                        f"{rdt:.1f} s; inexact for sub (a < b) and 60-bit mul"}}


def run_ntt(args, world, rank):
    L = 8
    shard = fdist.LimbShard(L, world, rank)
    n = 1 << args.log_n
    ctx = fc.Context(args.log_n, L=L)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(99 + rank)
    polys = 4 * args.batch
    x = uniform_limbs(gen, ctx.moduli[shard.lo:shard.hi], (polys,), n)

    def step():
        ctx.ntt_(x, limb0=shard.lo)
        ctx.intt_(x, limb0=shard.lo)

    dt, kavg = timed(step, args, world, 8 * args.steps + 8)
    ntts = 2 * polys * shard.nlimbs * world * args.steps
    dom = max(kavg, key=kavg.get)
    shape = {"log_n": args.log_n, "polys": polys, "nlimbs": shard.nlimbs}
    out = {"metric": METRIC, "value": round(ntts / dt, 1), "unit": "NTT/s",
           "ms_per_step": round(dt / args.steps * 1e3, 4),
           "config": {"workload": "forward+inverse NTT, single-limb transforms", "log_n": args.log_n,
                      "limbs": L, "polys_per_gpu": polys, "parallelism": f"rns-limb-shard x{world}"},
           "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
           # the whole transform: one NTT reads and writes each coefficient once (16 B per
           # coefficient per direction), over the summed time of its column and row passes
           "roofline": transform_roofline(kavg, 2 * polys * shard.nlimbs * n * 16, shape),
           # each pass alone (every pass moves the data once more)
           "roofline_passes": {k: roofline(k, polys * shard.nlimbs * n * 16, v, shape)
                               for k, v in kavg.items()}}
    # butterflies of the dominant pass: row passes run the last log R2 stages, column passes the
    # first log R1
    pb = polys * shard.nlimbs * (row_bflies(args.log_n) if "row" in dom
                                 else (n // 2) * (args.log_n // 2))
    fwd = "fwd" in dom
    out["roofline_alu"] = roofline_alu(dom, pb if fwd else 0, 0 if fwd else pb, kavg[dom])
    out["limiter"] = "valu" if out["roofline_alu"]["frac"] > out["roofline"]["frac"] else "hbm"
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_ntt(ctx.moduli, args.log_n, args.cpu_seconds)
    return out, cpu


def cpu_baseline_ntt(moduli, log_n, budget_s):
    """The tuned CPU port (oracle/fhe_cpu_port.c) timed on this host: forward + inverse NTT/s over
    single-limb transforms (OpenMP across poly-limbs), the GPU leg's unit of work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402

    threads = cpu_threads()
    rng = np.random.default_rng(0)
    n, P = 1 << log_n, max(4, threads // 2)
    mods = list(moduli)
    x = np.stack([np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in mods]) for _ in range(P)])
    m = np.asarray(mods, dtype=np.uint64)
    lib = coracle.lib()
    p = coracle._p(x)
    lib.port_ntt_fwd(coracle._p(x[:1].copy()), 1, log_n, coracle._p(m), len(mods))  # tables
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s:
        lib.port_ntt_fwd(p, P, log_n, coracle._p(m), len(mods))
        lib.port_ntt_inv(p, P, log_n, coracle._p(m), len(mods))
        done += 2 * P * len(mods)
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 1), "unit": "NTT/s", "cores": threads, "kind": "port",
            **cpu_host(),
            "sample": f"{done} forward+inverse NTTs (N=2^{log_n}, {len(mods)} limbs x {P} polys per "
                      f"call) by the tuned C port oracle/fhe_cpu_port.c, OpenMP {threads} threads, "
                      f"in {dt:.1f} s"}


def cpu_baseline_keyswitch(moduli, special, log_n, dnum, budget_s):
    """The tuned CPU port's key-switch (oracle/fhe_cpu_port.c port_keyswitch; test/measurement
    infrastructure, bit-exact with the checker) timed on this host: key-switches/s over batches of
    2 ciphertexts sharing the key (OpenMP across limbs), after one untimed call builds its tables."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402

    threads = cpu_threads()
    rng = np.random.default_rng(2)
    n = 1 << log_n
    allm = list(moduli) + list(special)
    B = 2
    d2 = np.stack([rng.integers(0, q, (B, n), dtype=np.uint64) for q in moduli], axis=1)
    evk = [np.stack([rng.integers(0, q, (dnum, n), dtype=np.uint64) for q in allm], axis=1)
           for _ in range(2)]
    coracle.port_keyswitch(d2[:1], evk[0], evk[1], moduli, special, dnum)  # tables
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s:
        coracle.port_keyswitch(d2, evk[0], evk[1], moduli, special, dnum)
        done += B
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 2), "unit": "keyswitch/s", "cores": threads, "kind": "port",
            **cpu_host(),
            "sample": f"{done} key-switches (N=2^{log_n}, L={len(moduli)}, K={len(special)}, "
                      f"dnum={dnum}, batches of {B}) by the tuned C port oracle/fhe_cpu_port.c "
                      f"(bit-exact with the checker), OpenMP {threads} threads, in {dt:.1f} s"}


def run_ntt_batch(args, world, rank):
    """BASELINE configs[4]: 1024 concurrent forward NTTs at N = 2^17 with 32 RNS limbs (one job of
    32,768 single-limb transforms), the polynomials sharded across the ranks (no collective; total
    work fixed -> strong scaling).  Every pass reads and writes each coefficient once: 2 x 8 x N
    bytes per NTT per pass."""
    log_n, L, P = 17, 32, 1024
    if P % world:
        raise SystemExit(f"ntt-batch: {P} polys do not split over {world} ranks")
    mine = P // world
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(4242 + rank)
    x = torch.empty(mine, L, n, dtype=torch.int64, device="cuda")
    for l, q in enumerate(ctx.moduli):  # uniform residues, one limb at a time (bounded temporaries)
        r = torch.randint(0, 2**62, (mine, n), generator=gen, dtype=torch.int64, device="cuda")
        x[:, l, :] = torch.remainder(r, q)
        del r
    # in place: canonical in, canonical out (the inverse is a bijection of canonical residues, so
    # timing it on uniform inputs is the round trip's second half)
    inv = bool(getattr(args, "inverse", False))
    step = (lambda: ctx.intt_(x)) if inv else (lambda: ctx.ntt_(x))  # noqa: E731
    dt, kavg = timed(step, args, world, 4 * args.steps + 4)
    ntts = P * L * args.steps
    shape = {"log_n": log_n, "polys": mine, "nlimbs": L}
    per_pass = mine * L * n * 16
    d = "inverse" if inv else "forward"
    out = {"metric": f"NTTs/sec, 1024 x N=2^17 x 32 RNS limbs ({d}, batched); achieved HBM GB/s vs peak",
           "value": round(ntts / dt, 1), "unit": "NTT/s",
           "ms_per_step": round(dt / args.steps * 1e3, 4), "scaling": "strong",
           "config": {"workload": f"batched {d} NTT, BASELINE configs[4]", "log_n": log_n,
                      "limbs": L, "polys": P, "polys_per_gpu": mine,
                      "parallelism": f"poly-shard x{world}"},
           # whole transform: read + write every coefficient once (two passes move it twice)
           "ntt_alg_hbm_gbps_per_gpu": round(ntts / world / dt * n * 16 / 1e9, 1),
           "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
           "roofline": transform_roofline(kavg, per_pass, shape),
           "roofline_passes": {k: roofline(k, per_pass, v, shape) for k, v in kavg.items()}}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_ntt(ctx.moduli[:8], log_n, args.cpu_seconds)
    return out, cpu


def valu_profile():
    """The newest profiles/rNN_keyswitch_pmc.json: per-kernel SQ_INSTS_VALU per launch of the
    key-switch at the bench shape (rocprofv3 --pmc pass, tools/valu_roofline.py), with its file
    name, or (None, None)."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_keyswitch_pmc.json")))
    for path in reversed(paths):
        try:
            with open(path) as f:
                return json.load(f), os.path.relpath(path, ROOT)
        except (OSError, ValueError):
            continue
    return None, None


def ks_design_min_bytes(B, nl, L, K, dnum, n):
    """HBM bytes one fused key-switch call (lz16 path, B ciphertexts, nl own Q-limbs of L, K
    special limbs, dnum digits) must move with this kernel sequence: every kernel reads its inputs
    and writes its outputs once, the keys once per batch.  Per kernel: the INTT of
    d2 (2 passes), ModUp (the gathered sources in, the extended rows out), the P rows' inner
    product (their extended rows and keys in, both accumulators' P rows out), the P rows' column
    inverse, ModDown's conversion (P rows in, conv out), the Q rows' inner product + finish
    (extended rows of the other digits, conv, d2, keys in; both outputs out)."""
    row = n * 8
    rows = nl + K
    intt = 4 * B * nl * row
    modup = B * (dnum * rows - nl) * row + B * L * row
    p_inner = B * dnum * K * row + dnum * 2 * K * row + 2 * B * K * row
    p_colinv = 2 * 2 * B * K * row
    moddown = 2 * B * K * row + 2 * B * nl * row
    q_fin = B * nl * (dnum - 1) * row + 2 * B * nl * row + B * nl * row + dnum * 2 * nl * row + \
        2 * B * nl * row
    return intt + modup + p_inner + p_colinv + moddown + q_fin


class KeyswitchLeg:
    """BASELINE configs[3] through the native multi-GPU path: N = 2^16, L = 16, K = 4, dnum = 4,
    a global batch of `--ks-batch` ciphertexts (one key), limbs sharded over the ranks, INTT +
    one ncclAllGather per chunk + the local key-switch inside libfhecore (fhe_keyswitch_dist on
    its own RCCL communicator; one chunk at N = 1, 4 above so transfers overlap compute).  The
    batch is the whole job's: strong scaling.  Allocates on construction, times in run()."""

    L, K, DNUM = 16, 4, 4

    def __init__(self, args, world, rank):
        self.world, self.rank = world, rank
        # hybrid partition (fhe_dist_hybrid): `groups` ciphertext groups of g limb shards; groups = 1
        # is the limb-only partition (every rank one limb shard of the whole batch)
        self.groups = max(1, getattr(args, "ks_groups", 1) or 1)
        if world % self.groups:
            raise SystemExit(f"--ks-groups {self.groups} does not divide {world} ranks")
        self.g = world // self.groups
        self.shard = fdist.LimbShard(self.L, self.g, rank % self.g)
        self.log_n = args.log_n
        n = 1 << args.log_n
        self.ctx = ctx = fc.Context(args.log_n, L=self.L, K=self.K, dnum=self.DNUM)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(7 + rank)
        rows = self.shard.evk_rows(self.K)
        allm = ctx.all_moduli
        self.evk_b = uniform_limbs(gen, [allm[r] for r in rows], (self.DNUM,), n)
        self.evk_a = uniform_limbs(gen, [allm[r] for r in rows], (self.DNUM,), n)
        self.B = args.ks_batch
        self.chunks = args.ks_chunks or (1 if self.g == 1 else 4)
        self.hybrid = fdist.hybrid_plan(self.L, self.log_n, world, self.groups, rank, self.B,
                                        self.chunks)
        self.my_batch = self.hybrid.batch  # this rank's group's ciphertexts
        self.d2 = uniform_limbs(gen, ctx.moduli[self.shard.lo:self.shard.hi], (self.my_batch,), n)
        self.live_pmc = world == 1 and rank == 0 and not args.no_pmc
        # the group's torch.distributed sub-group (every rank creates all of them, in order);
        # None: the group is the world (groups = 1) or one rank (g = 1)
        self.group = fdist.hybrid_groups(world, self.groups) if 1 < self.groups < world else None
        # the native path needs one GPU per rank (RCCL refuses two ranks on one device); the
        # gloo rehearsal of several ranks on one GPU takes the torch.distributed form instead
        # (fhecore.dist.sharded_keyswitch: INTT, one all_gather through the host, local step)
        self.native = world == 1 or torch.distributed.get_backend() == "nccl"
        if self.native:
            self.comm = fdist.RcclComm(group=self.group, local=self.g == 1)
            self.ws = ctx.workspace(load().fhe_keyswitch_dist_workspace(
                ctx.handle, self.comm.handle, max(self.my_batch, 1), self.chunks))

    def step(self):
        if self.native:
            self.ctx.keyswitch_dist(self.comm, self.d2, self.evk_b, self.evk_a,
                                    chunks=self.chunks, workspace=self.ws)
        else:
            fdist.sharded_keyswitch(self.ctx, self.d2, self.evk_b, self.evk_a, self.shard,
                                    group=self.group)

    def run(self, targs, valu=False):
        L, K, dnum, B, world = self.L, self.K, self.DNUM, self.B, self.world
        n = 1 << self.log_n
        dt, kavg = timed(self.step, targs, world, 64 * targs.steps + 64)
        gather = self.comm.gather_ms() if self.native else []  # the last call's chunks
        ks_per_s = B * targs.steps / dt
        ms_per_ks = dt / (B * targs.steps) * 1e3
        # d2 in + evk (dnum * 2 * (L + K) limbs) + 2 L limbs out per key-switch; the
        # key is shared by the batch, so per batch: B (d2 + out) + one key, unsharded
        alg = (B * 3 * L + dnum * 2 * (L + K)) * n * 8 // B
        res = {"value": round(ks_per_s, 2), "unit": "keyswitch/s",
               "ms_per_step": round(dt / targs.steps * 1e3, 4),
               "config": {"workload": "hybrid key-switch, BASELINE configs[3] (fhe_keyswitch_dist)",
                          "log_n": self.log_n, "L": L, "K": K, "dnum": dnum, "batch": B,
                          "chunks": self.chunks if self.native else 1, "scaling": "strong",
                          "ks_groups": self.groups,
                          "parallelism": (f"rns-limb-shard x{world}, " if self.groups == 1 else
                                          f"hybrid: {self.groups} ciphertext groups x "
                                          f"rns-limb-shard x{self.g}, ") + (
                              "RCCL all-gather in libfhecore (fhe_keyswitch_dist)" if self.native
                              else "torch.distributed all_gather (gloo, host-staged; "
                                   "fhecore.dist.sharded_keyswitch)")},
               "warmup": targs.warmup, "steps": targs.steps,
               "gather_ms_per_chunk": [round(v, 4) for v in gather],
               "keyswitch_alg_hbm_gbps_per_gpu": round(ks_per_s * alg / 1e9 / world, 1),
               "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
               "roofline": roofline("keyswitch (whole, per GPU)", alg // world, ms_per_ks,
                                    {"log_n": self.log_n, "L": L, "world": world})}
        plan = fdist.hybrid_plan(L, self.log_n, world, self.groups, self.rank, B,
                                 self.chunks if self.native else 1).plan
        # what each rank ends up with (its group's g blocks; nothing is gathered at g = 1)
        res["gather_bytes_per_chunk"] = plan.block_words * 8 * self.g if self.g > 1 else 0
        # integer-ALU roofline of one key-switch on this rank, butterflies only: INTT of the own
        # d2 limbs; ModUp: every digit's extended rows = dnum (nl + K) - nl forward NTTs; ModDown:
        # INTT of the 2 K special rows, forward NTT of the 2 nl converted rows
        # (per job key-switch: this rank processes my_batch of the job's B ciphertexts)
        nl, full = self.shard.nlimbs, (n // 2) * self.log_n
        share = self.my_batch / B
        res["roofline_alu"] = roofline_alu(
            "keyswitch (whole, per GPU; NTT butterflies only)",
            round((dnum * (nl + K) + nl) * full * share), round((nl + 2 * K) * full * share),
            ms_per_ks)
        # ... and by VALU instruction issue, which counts everything the kernels execute (base
        # conversion products, inner products, reductions, addressing): SQ_INSTS_VALU of each
        # key-switch kernel at this shape from a rocprofv3 --pmc pass over a child process
        # (tools/ks_valu_probe.py), over this run's time, against the issue rate of the butterfly
        # ceiling kernel in that profiled process.  Without the pass (--no-pmc, or it failed) the
        # committed profile of the same shape stands in, and says so.
        self.step_s = dt / targs.steps
        if world == 1 and valu:
            res["roofline_valu"] = self.valu_roofline()
            self.traffic(res)
        return res

    def traffic(self, res):
        """roofline.traffic of the key-switch line: the HBM bytes every kernel of one call moves,
        from this run's FETCH_SIZE / WRITE_SIZE passes, per key-switch like `achieved`; null and
        the reason when the passes are off (--no-pmc) or fail."""
        rf = res["roofline"]
        if not self.live_pmc:
            rf["traffic_live_error"] = "--no-pmc"
            return
        per, total, why = measure_keyswitch_traffic_live(self.log_n, self.B, self.chunks)
        if total is None:
            rf["traffic_live_error"] = why
            return
        alg = rf["alg_bytes_per_launch"]
        rf["traffic"] = total // self.B
        rf["traffic_over_alg"] = round(total / self.B / alg, 3)
        # against the bytes this kernel sequence must move (each kernel's inputs and outputs once:
        # the extended basis, the accumulators' P rows, conv, the keys once per batch) -- how much
        # of traffic_over_alg is the two-pass design and how much is waste
        dmin = ks_design_min_bytes(self.B, self.shard.nlimbs, self.L, self.K, self.DNUM,
                                   1 << self.log_n)
        rf["traffic_design_min"] = dmin // self.B
        rf["traffic_over_design_min"] = round(total / dmin, 3)
        rf["traffic_per_call_by_kernel"] = {k: int(v) for k, v in sorted(per.items())}
        rf["traffic_source"] = (
            "measured in this run: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes "
            f"(separate) over tools/ks_valu_probe.py --no-peak (batch {self.B}, {self.chunks} "
            "chunk(s)), every key-switch kernel's dispatches summed per call, per key-switch; "
            "read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB (gfx950 correction)")

    def valu_roofline(self):
        step_s = self.step_s
        why = "--no-pmc"
        if self.live_pmc:
            ks, ceil, why = measure_keyswitch_valu_live(self.log_n, self.B, self.chunks)
            if ks is not None:
                per_step = sum(ks.values())
                ach = per_step / step_s / 1e9
                return {"bound": "valu", "achieved": round(ach, 1), "peak": round(ceil, 2),
                        "unit": "G VALU wave-instructions/s", "frac": round(ach / ceil, 4),
                        "valu_instr_per_step": per_step,
                        "valu_source": "measured in this run: rocprofv3 --pmc SQ_INSTS_VALU over "
                                       "tools/ks_valu_probe.py (same shape; ceiling = "
                                       "k_bfly_peak in that process); time from this run",
                        "valu_instr_per_kernel": {k: round(v) for k, v in ks.items()}}
        prof, prof_path = valu_profile()
        shape = (prof or {}).get("shape", {})
        if not prof or self.B != shape.get("batch") or self.chunks != shape.get("chunks", 1):
            return {"valu_live_error": why, "frac": None}
        try:
            per_step = sum(v["valu_instr_per_launch"] * v["launches_per_step"]
                           for k, v in prof["kernels"].items() if k.startswith("k_") and
                           "bfly_peak" not in k)
        except (KeyError, TypeError):
            return {"valu_live_error": f"{why}; {prof_path} lacks per-step counts", "frac": None}
        ach = per_step / step_s / 1e9
        return {"bound": "valu", "achieved": round(ach, 1), "peak": prof["ceiling_valu_g_per_s"],
                "unit": "G VALU wave-instructions/s",
                "frac": round(ach / prof["ceiling_valu_g_per_s"], 4),
                "valu_instr_per_step": per_step, "valu_live_error": why,
                "valu_source": f"committed, not measured in this run: {prof_path} "
                               "(SQ_INSTS_VALU of every key-switch kernel, same shape); time from this run"}


def run_keyswitch(args, world, rank):
    leg = KeyswitchLeg(args, world, rank)
    out = leg.run(args, valu=True)
    out["metric"] = ("key-switches/sec at N=2^16, L=16, K=4, dnum=4 (RNS limbs sharded, RCCL "
                     "all-gather)")
    out.pop("warmup")
    out.pop("steps")
    out["scaling"] = out["config"].pop("scaling")
    if not args.no_dist_check:
        out["dist_check"] = guarded_leg(lambda: dist_check(world, rank, ks_leg=leg), out, rank,
                                        "dist_check")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_keyswitch(leg.ctx.moduli, leg.ctx.special, args.log_n, leg.DNUM,
                                     args.cpu_seconds)
    return out, cpu


def run_mulrelin(args, world, rank):
    """ct x ct multiply -> relinearise -> rescale, NTT form, at the key-switch
    configuration (N = 2^16, L = 16, K = 4, dnum = 4), captured once in a HIP graph and replayed.
    Single-device per rank (replicas: no collective; the sharded key-switch is --workload
    keyswitch)."""
    L, K, dnum = 16, 4, 4
    n = 1 << args.log_n
    ctx = fc.Context(args.log_n, L=L, K=K, dnum=dnum)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11 + rank)
    B = args.batch
    a = uniform_limbs(gen, ctx.moduli, (B, 2), n)
    b = uniform_limbs(gen, ctx.moduli, (B, 2), n)
    kb = uniform_limbs(gen, ctx.all_moduli, (dnum,), n)
    ka = uniform_limbs(gen, ctx.all_moduli, (dnum,), n)
    ws = ctx.workspace(load().fhe_mul_relin_workspace(ctx.handle, B))
    out = torch.empty(B, 2, L - 1, n, dtype=torch.int64, device="cuda")
    side = torch.cuda.Stream()  # the legacy default stream cannot be captured
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        ctx.mul_relin(a, b, kb, ka, rescale=True, workspace=ws, out=out)  # eager once
        with fc.Graph() as g:
            ctx.mul_relin(a, b, kb, ka, rescale=True, workspace=ws, out=out)
        dt, kavg = timed(g.launch, args, world, 4)
    per_s = B * args.steps * world / dt
    # per multiply: read 2 cts (4 L limbs), the key once per batch, write 2 (L-1) limbs
    alg = (B * (4 * L + 2 * (L - 1)) + dnum * 2 * (L + K)) * n * 8 // B
    out_line = {"metric": "mult+relin+rescale/sec at N=2^16, L=16, K=4, dnum=4 (NTT form, HIP graph)",
                "value": round(per_s, 2), "unit": "mul_relin/s",
                "ms_per_step": round(dt / args.steps * 1e3, 4),
                "config": {"workload": "ct x ct multiply + relinearise + rescale (SURVEY §8f row 4)",
                           "log_n": args.log_n, "L": L, "K": K, "dnum": dnum, "batch": B,
                           "parallelism": f"replicas x{world}"},
                "roofline": roofline("mul_relin (whole pipeline)", alg, dt / (B * args.steps) * 1e3 * world,
                                     {"log_n": args.log_n, "L": L})}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_mulrelin(ctx.moduli, ctx.special, args.log_n, dnum, args.cpu_seconds)
    return out_line, cpu


def cpu_baseline_mulrelin(moduli, special, log_n, dnum, budget_s):
    """mult + relinearise on this host from the tuned C port's pieces (oracle/fhe_cpu_port.c):
    the NTT-form tensor by port_vec_op (d0 = a0 b0, d1 = a0 b1 + a1 b0, d2 = a1 b1), the
    key-switch of d2 by port_keyswitch, the combine by port_vec_op adds.  The rescale the GPU
    pipeline also runs is NOT included (one INTT + L - 1 NTTs + elementwise per ciphertext
    polynomial), so this baseline is lighter than the GPU leg."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402

    rng = np.random.default_rng(11)
    n, L = 1 << log_n, len(moduli)
    allm = list(moduli) + list(special)
    B = 2
    ct = [np.stack([rng.integers(0, q, (B, n), dtype=np.uint64) for q in moduli], axis=1)
          for _ in range(4)]  # a0, a1, b0, b1 [B][L][N]
    evk = [np.stack([rng.integers(0, q, (dnum, n), dtype=np.uint64) for q in allm], axis=1)
           for _ in range(2)]
    rowm = np.tile(np.asarray(moduli, dtype=np.uint64), B)
    flat = lambda x: x.reshape(B * L, n)  # noqa: E731

    def one():
        a0, a1, b0, b1 = (flat(x) for x in ct)
        d0 = coracle.port_vec_op("mul", a0, b0, rowm)
        d1 = coracle.port_vec_op("add", coracle.port_vec_op("mul", a0, b1, rowm),
                                 coracle.port_vec_op("mul", a1, b0, rowm), rowm)
        d2 = coracle.port_vec_op("mul", a1, b1, rowm).reshape(B, L, n)
        k0, k1 = coracle.port_keyswitch(d2, evk[0], evk[1], moduli, special, dnum)
        coracle.port_vec_op("add", d0, flat(k0), rowm)
        coracle.port_vec_op("add", d1, flat(k1), rowm)

    one()  # tables
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s:
        one()
        done += B
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 2), "unit": "mul_relin/s", "cores": cpu_threads(),
            "kind": "port", **cpu_host(),
            "sample": f"{done} mult + relinearise (N=2^{log_n}, L={L}, K={len(special)}, "
                      f"dnum={dnum}, batches of {B}; rescale not included) composed from the tuned "
                      f"C port (port_vec_op, port_keyswitch), OpenMP {cpu_threads()} threads, "
                      f"in {dt:.1f} s"}


def run_rotate(args, world, rank):
    """Hoisted rotations (fhe_rotate_hoisted, a widening beyond SURVEY §8f row 1): R Galois
    elements of the same ciphertexts sharing one ModUp, at the key-switch configuration
    (N = 2^16, L = 16, K = 4, dnum = 4), batch B per call.  `value` counts rotations (B R per
    step); the same R rotations through R fhe_rotate calls are timed beside it."""
    L, K, dnum, R = 16, 4, 4, 8
    n = 1 << args.log_n
    ctx = fc.Context(args.log_n, L=L, K=K, dnum=dnum)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(13 + rank)
    B = args.batch
    ct = uniform_limbs(gen, ctx.moduli, (B, 2), n)
    keys = [(uniform_limbs(gen, ctx.all_moduli, (dnum,), n),
             uniform_limbs(gen, ctx.all_moduli, (dnum,), n)) for _ in range(R)]
    elts = [ctx.galois_elt(r) for r in range(1, R + 1)]
    lib = load()
    ws = ctx.workspace(max(lib.fhe_rotate_hoisted_workspace(ctx.handle, B),
                           lib.fhe_rotate_workspace(ctx.handle, B)))
    out = torch.empty(R, B, 2, L, n, dtype=torch.int64, device="cuda")
    hoisted = lambda: ctx.rotate_hoisted(ct, elts, keys, workspace=ws, out=out)  # noqa: E731

    def plain():
        for r in range(R):
            ctx.rotate(ct, elts[r], keys[r][0], keys[r][1], workspace=ws)

    dt, kavg = timed(hoisted, args, world, 64)
    dt_plain, _ = timed(plain, args, world, 1)
    per_s = B * R * args.steps * world / dt
    return {"metric": "hoisted rotations/sec at N=2^16, L=16, K=4, dnum=4 (8 Galois elements per ModUp)",
            "value": round(per_s, 2), "unit": "rotations/s",
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "config": {"workload": "hoisted rotations (fhe_rotate_hoisted)", "log_n": args.log_n,
                       "L": L, "K": K, "dnum": dnum, "rotations_per_modup": R, "batch": B,
                       "parallelism": f"replicas x{world}"},
            "unhoisted_rotations_per_sec": round(B * R * args.steps * world / dt_plain, 2),
            "hoisting_speedup": round(dt_plain / dt, 3),
            "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
            # per rotation: read the ct (2 L limbs), write the rotated ct (2 L), each element's key
            # (dnum * 2 * (L + K) limbs) once per batch -- algorithmic, as SURVEY §8d counts the
            # key-switch; the dominant kernel is the gathered inner product (k_ks_inner)
            "roofline": roofline("hoisted rotation (whole, per GPU)",
                                 (B * 4 * L + dnum * 2 * (L + K)) * n * 8 // B,
                                 dt / (B * R * args.steps) * 1e3,
                                 {"log_n": args.log_n, "L": L, "R": R}),
            "roofline_inner_product": roofline(
                "ks_inner (gathered inner product, per launch)",
                (dnum * B * (L + K) + 2 * dnum * (L + K) + 2 * B * (L + K)) * n * 8,
                kavg.get("ks_inner", float("nan")), {"log_n": args.log_n, "L": L, "B": B})}, (
        cpu_baseline_rotate(ctx.moduli, ctx.special, args.log_n, dnum, args.cpu_seconds)
        if rank == 0 and world == 1 and not args.no_cpu_baseline else None)


def cpu_baseline_rotate(moduli, special, log_n, dnum, budget_s):
    """Rotations on this host: sigma_k of both ciphertext polys (an NTT-domain slot permutation,
    numpy fancy indexing) + the tuned port's key-switch of sigma(c1) (port_keyswitch) + the
    combine (port_vec_op) -- unhoisted, one key-switch per rotation, as a CPU library runs it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle  # noqa: E402

    rng = np.random.default_rng(13)
    n, L = 1 << log_n, len(moduli)
    allm = list(moduli) + list(special)
    B = 2
    c0 = np.stack([rng.integers(0, q, (B, n), dtype=np.uint64) for q in moduli], axis=1)
    c1 = np.stack([rng.integers(0, q, (B, n), dtype=np.uint64) for q in moduli], axis=1)
    evk = [np.stack([rng.integers(0, q, (dnum, n), dtype=np.uint64) for q in allm], axis=1)
           for _ in range(2)]
    k = pow(5, 1, 2 * n)
    # NTT-domain automorphism: slot i <- brv(((2 brv(i) + 1) k mod 2N - 1) / 2)
    idx = np.arange(n)
    brv = np.array([int(f"{i:0{log_n}b}"[::-1], 2) for i in range(n)])
    perm = brv[(((2 * brv[idx] + 1) * k) % (2 * n) - 1) // 2]
    rowm = np.tile(np.asarray(moduli, dtype=np.uint64), B)

    def one():
        s0 = np.ascontiguousarray(c0[..., perm])
        s1 = np.ascontiguousarray(c1[..., perm])
        k0, _ = coracle.port_keyswitch(s1, evk[0], evk[1], moduli, special, dnum)
        coracle.port_vec_op("add", s0.reshape(B * L, n), k0.reshape(B * L, n), rowm)

    one()
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s:
        one()
        done += B
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 2), "unit": "rotations/s", "cores": cpu_threads(),
            "kind": "port", **cpu_host(),
            "sample": f"{done} rotations (N=2^{log_n}, L={L}, K={len(special)}, dnum={dnum}, "
                      f"batches of {B}, unhoisted) by numpy permutations + the tuned C port's "
                      f"key-switch, OpenMP {cpu_threads()} threads, in {dt:.1f} s"}


def run_rotsum(args, world, rank):
    """Double-hoisted rotation sum (fhe_rotate_sum_hoisted, the inner loop of a baby-step /
    giant-step linear transform, a widening beyond SURVEY §8f rows 1 and 4): out = sum_r pt_r
    rot_r(ct) over R = 8 terms (the unrotated one and 7 rotations) with one ModUp and one ModDown,
    at the key-switch configuration (N = 2^16, L = 16, K = 4, dnum = 4), batch B per call.
    `value` counts terms (B R per step).  The same sum through the single-hoisted API
    (fhe_rotate_hoisted of the 7 rotations, then a plaintext product per term and the adds,
    fhe_vec_mul / fhe_vec_add) is timed beside it."""
    L, K, dnum, R = 16, 4, 4, 8
    n = 1 << args.log_n
    ctx = fc.Context(args.log_n, L=L, K=K, dnum=dnum)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(17 + rank)
    B = args.batch
    ct = uniform_limbs(gen, ctx.moduli, (B, 2), n)
    elts = [1] + [ctx.galois_elt(r) for r in range(1, R)]
    keys = [None] + [(uniform_limbs(gen, ctx.all_moduli, (dnum,), n),
                      uniform_limbs(gen, ctx.all_moduli, (dnum,), n)) for _ in range(R - 1)]
    pts = [uniform_limbs(gen, ctx.all_moduli, (), n) for _ in range(R)]
    lib = load()
    ws = ctx.workspace(max(lib.fhe_rotate_sum_hoisted_workspace(ctx.handle, B),
                           lib.fhe_rotate_hoisted_workspace(ctx.handle, B)))
    out = torch.empty(B, 2, L, n, dtype=torch.int64, device="cuda")
    fused = lambda: ctx.rotate_sum_hoisted(ct, elts, keys, pts, workspace=ws, out=out)  # noqa: E731
    # the single-hoisted composition: the plaintexts broadcast over the batch (Q rows only)
    rot = torch.empty(R - 1, B, 2, L, n, dtype=torch.int64, device="cuda")
    ptq = [p[:L].expand(B, 2, L, n).contiguous() for p in pts]
    prod = torch.empty(B, 2, L, n, dtype=torch.int64, device="cuda")
    acc = torch.empty(B, 2, L, n, dtype=torch.int64, device="cuda")

    def single():
        ctx.rotate_hoisted(ct, elts[1:], keys[1:], workspace=ws, out=rot)
        ctx.vec("mul", ct, ptq[0], out=acc)
        for r in range(1, R):
            ctx.vec("mul", rot[r - 1], ptq[r], out=prod)
            ctx.vec("add", acc, prod, out=acc)

    dt, kavg = timed(fused, args, world, 64)
    dt_single, _ = timed(single, args, world, 1)
    del rot, ptq, prod, acc
    per_s = B * R * args.steps * world / dt
    # per call: read the batch's cts (2 L limbs each) and write the sums (2 L), every key
    # ((R - 1) dnum 2 (L + K) limbs) and plaintext (R (L + K)) once per batch
    alg_call = (B * 4 * L + (R - 1) * dnum * 2 * (L + K) + R * (L + K)) * n * 8
    return {"metric": "rotation-sum terms/sec at N=2^16, L=16, K=4, dnum=4 (8 terms per ModUp "
                      "and per ModDown, double hoisting)",
            "value": round(per_s, 2), "unit": "terms/s",
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "config": {"workload": "double-hoisted rotation sum (fhe_rotate_sum_hoisted)",
                       "log_n": args.log_n, "L": L, "K": K, "dnum": dnum, "terms": R,
                       "rotations": R - 1, "batch": B, "parallelism": f"replicas x{world}"},
            "rotsums_per_sec": round(B * args.steps * world / dt, 2),
            "single_hoisted_terms_per_sec": round(B * R * args.steps * world / dt_single, 2),
            "double_hoisting_speedup": round(dt_single / dt, 3),
            "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
            "roofline": roofline("rotation sum (whole call, per GPU)", alg_call,
                                 dt / (args.steps) * 1e3, {"log_n": args.log_n, "L": L, "R": R,
                                                           "B": B}),
            # the gathered inner product x plaintext: reads the ModUp digits ((dnum - 1) B (L + K)
            # rows) and the ct (2 L rows per ciphertext) once per term through the automorphism,
            # each term's keys and plaintext once, writes the two accumulators and the c0 sums
            "roofline_rot_sum": roofline(
                "rot_sum (gathered inner products x plaintexts, per launch)",
                (R * ((dnum - 1) * B * (L + K) + B * 2 * L + 2 * dnum * (L + K) + (L + K)) +
                 2 * B * (L + K) + 2 * B * L) * n * 8,
                kavg.get("rot_sum", float("nan")), {"log_n": args.log_n, "L": L, "B": B})}, None


def run_lintrans(args, world, rank):
    """Baby-step / giant-step linear transform with both hoistings (fhe_linear_transform: CKKS
    bootstrapping's CoeffToSlot / SlotToCoeff shape, a widening beyond SURVEY §8f rows 1 and 4):
    n1 = 4 baby x n2 = 4 giant steps = 16 diagonals per ciphertext, at the key-switch configuration
    (N = 2^16, L = 16, K = 4, dnum = 4), batch B per call.  `value` counts transforms (B per step).
    The same 16-diagonal product by the hoisted diagonal method (fhe_rotate_hoisted of the 15
    rotations, then a plaintext product per diagonal and the adds) is timed beside it."""
    L, K, dnum, n1, n2 = 16, 4, 4, 4, 4
    n = 1 << args.log_n
    ctx = fc.Context(args.log_n, L=L, K=K, dnum=dnum)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(19 + rank)
    B = args.batch
    ct = uniform_limbs(gen, ctx.moduli, (B, 2), n)
    key = lambda: (uniform_limbs(gen, ctx.all_moduli, (dnum,), n),  # noqa: E731
                   uniform_limbs(gen, ctx.all_moduli, (dnum,), n))
    baby = [1] + [ctx.galois_elt(b) for b in range(1, n1)]
    giant = [1] + [ctx.galois_elt(g * n1) for g in range(1, n2)]
    bkeys = [None] + [key() for _ in range(1, n1)]
    gkeys = [None] + [key() for _ in range(1, n2)]
    pts = [[uniform_limbs(gen, ctx.all_moduli, (), n) for _ in range(n1)] for _ in range(n2)]
    lib = load()
    ws = ctx.workspace(max(lib.fhe_linear_transform_workspace(ctx.handle, n2, B),
                           lib.fhe_rotate_hoisted_workspace(ctx.handle, B)))
    out = torch.empty(B, 2, L, n, dtype=torch.int64, device="cuda")
    fused = lambda: ctx.linear_transform(ct, baby, bkeys, giant, gkeys, pts, workspace=ws,  # noqa: E731
                                         out=out)
    dt, kavg = timed(fused, args, world, 128)
    # the hoisted diagonal method: sum_i diag_i rot_i(ct), i < n1 n2, one ModUp for the rotations
    D = n1 * n2
    elts = [ctx.galois_elt(i) for i in range(1, D)]
    keys = [key() for _ in range(1, D)]
    rot = torch.empty(D - 1, B, 2, L, n, dtype=torch.int64, device="cuda")
    diag = [uniform_limbs(gen, ctx.moduli, (), n).expand(B, 2, L, n).contiguous()
            for _ in range(D)]
    prod = torch.empty(B, 2, L, n, dtype=torch.int64, device="cuda")
    acc = torch.empty(B, 2, L, n, dtype=torch.int64, device="cuda")

    def diagonal():
        ctx.rotate_hoisted(ct, elts, keys, workspace=ws, out=rot)
        ctx.vec("mul", ct, diag[0], out=acc)
        for i in range(1, D):
            ctx.vec("mul", rot[i - 1], diag[i], out=prod)
            ctx.vec("add", acc, prod, out=acc)

    dt_diag, _ = timed(diagonal, args, world, 1)
    del rot, diag, prod, acc
    per_s = B * args.steps * world / dt
    # per call: read the cts (2 L limbs each), write the results (2 L); every key ((n1 - 1) +
    # (n2 - 1) rotation keys of dnum 2 (L + K) limbs) and diagonal (n1 n2 (L + K)) once per batch
    alg_call = (B * 4 * L + (n1 + n2 - 2) * dnum * 2 * (L + K) + D * (L + K)) * n * 8
    return {"metric": "BSGS linear transforms/sec at N=2^16, L=16, K=4, dnum=4 (16 diagonals: "
                      "4 baby x 4 giant steps, double hoisting)",
            "value": round(per_s, 2), "unit": "transforms/s",
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "config": {"workload": "BSGS linear transform (fhe_linear_transform)",
                       "log_n": args.log_n, "L": L, "K": K, "dnum": dnum, "n1": n1, "n2": n2,
                       "diagonals": D, "batch": B, "parallelism": f"replicas x{world}"},
            "diagonals_per_sec": round(D * per_s, 2),
            "hoisted_diagonal_method_per_sec": round(B * args.steps * world / dt_diag, 2),
            "bsgs_speedup": round(dt_diag / dt, 3),
            "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
            "roofline": roofline("linear transform (whole call, per GPU)", alg_call,
                                 dt / args.steps * 1e3, {"log_n": args.log_n, "L": L, "B": B})}, None


def shard_mismatches(got, ref_full, shard) -> int:
    """Words of this rank's limb slice `got` [..., nlimbs, N] that differ from its limbs of the
    single-device result `ref_full` [..., L, N]."""
    if shard.nlimbs == 0:
        return 0
    return int((got != shard.own(ref_full)).sum().item())


def check_keyswitch_shard(engine, shard, K, d2, evk_b, evk_a, dist_fn) -> int:
    """One rank's bitwise check of the limb-sharded key-switch (G ranks must equal
    G = 1 bit for bit).  Every rank holds the same full seeded d2 [B, L, N] and key [dnum, L + K,
    N]; it runs the distributed path on its own slices (dist_fn(d2_own, evk_b_own, evk_a_own) ->
    (ks0_own, ks1_own), a collective every rank enters) and the single-device key-switch of the
    whole input on its own device, and counts the mismatched words of its own limbs."""
    rows = shard.evk_rows(K)
    k0, k1 = dist_fn(shard.own(d2).contiguous(), evk_b[:, rows].contiguous(),
                     evk_a[:, rows].contiguous())
    r0, r1 = engine.keyswitch(d2, evk_b, evk_a)
    return shard_mismatches(k0, r0, shard) + shard_mismatches(k1, r1, shard)


def check_hommult_shard(engine, shard, a, b) -> int:
    """The same for the limb-sharded HomMult: a, b [B, 2, L, N] full on every rank."""
    got = fdist.sharded_hommult(engine, shard.own(a).contiguous(), shard.own(b).contiguous(), shard)
    return shard_mismatches(got, engine.hommult(a, b), shard)


def sum_over_ranks(x: int, world: int) -> int:
    if world == 1:
        return x
    nccl = torch.distributed.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.int64, device="cuda" if nccl else "cpu")
    torch.distributed.all_reduce(t)
    return int(t.item())


def dist_check(world, rank, hm_ctx=None, ks_leg=None, seed=4321):
    """Bitwise check of the multi-GPU paths this process timed, outside every timed window: the
    native RCCL key-switch (fhe_keyswitch_dist, chunked like the leg) and one limb-sharded HomMult
    batch against each rank's single-device result (fhe_keyswitch / fhe_hommult of the full
    input).  The inputs come from one seed shared by all ranks, so every rank can rebuild the whole
    ciphertext.  Returns "bit-exact" or {"mismatched_words": n, ...} summed over the ranks."""
    gen = torch.Generator(device="cuda")
    gen.manual_seed(seed)
    parts, bad = [], 0
    if hm_ctx is not None:
        shard = fdist.LimbShard(hm_ctx.L, world, rank)
        a = uniform_limbs(gen, hm_ctx.moduli, (2, 2), hm_ctx.n)
        b = uniform_limbs(gen, hm_ctx.moduli, (2, 2), hm_ctx.n)
        bad += check_hommult_shard(hm_ctx, shard, a, b)
        parts.append(f"sharded HomMult (2 ciphertexts, L={hm_ctx.L})")
        del a, b
    if ks_leg is not None:
        ctx, shard = ks_leg.ctx, ks_leg.shard
        # a batch of 2 per chunk per ciphertext group so that the chunked own-stream path
        # (chunks > 1) runs as timed; each rank checks its group's ciphertexts
        B = 2 * ks_leg.chunks * ks_leg.groups
        h = fdist.hybrid_plan(ctx.L, ctx.log_n, world, ks_leg.groups, rank, B, ks_leg.chunks)
        mine = slice(h.batch0, h.batch0 + h.batch)
        d2 = uniform_limbs(gen, ctx.moduli, (B,), ctx.n)
        kb = uniform_limbs(gen, ctx.all_moduli, (ks_leg.DNUM,), ctx.n)
        ka = uniform_limbs(gen, ctx.all_moduli, (ks_leg.DNUM,), ctx.n)
        if ks_leg.native:
            fn = lambda d, eb, ea: ctx.keyswitch_dist(ks_leg.comm, d, eb, ea,  # noqa: E731
                                                      chunks=ks_leg.chunks)
            how = f"fhe_keyswitch_dist over RCCL, {ks_leg.chunks} chunk(s)"
        else:
            fn = lambda d, eb, ea: fdist.sharded_keyswitch(ctx, d, eb, ea, shard,  # noqa: E731
                                                           group=ks_leg.group)
            how = "torch.distributed all_gather form (gloo)"
        if ks_leg.groups > 1:
            how += f", hybrid: {ks_leg.groups} ciphertext groups x {ks_leg.g} limb shards"
        bad += check_keyswitch_shard(ctx, shard, ks_leg.K, d2[mine].contiguous(), kb, ka, fn)
        parts.append(f"key-switch ({how}, batch {B}, L={ctx.L}, K={ctx.K})")
        del d2, kb, ka
    torch.cuda.synchronize()
    bad = sum_over_ranks(bad, world)
    what = f"{world} rank(s) vs each rank's single-device fhe_keyswitch / fhe_hommult: " + \
        "; ".join(parts)
    if bad == 0:
        return {"result": "bit-exact", "checked": what}
    return {"result": "MISMATCH", "mismatched_words": bad, "checked": what}


_EMIT = {"failed": []}  # json_fd, args, world (set by main); failed: reasons for a non-zero exit
_EMIT_LOCK = threading.Lock()  # the main thread and a leg's watchdog may both try to print


def failure_reasons(out):
    """Why this run must exit non-zero although its line was printed: a ride-along leg that raised
    or never finished, or a dist_check that found mismatched words."""
    why = list(_EMIT.get("failed", []))
    for k, v in out.items():
        if isinstance(v, dict) and "error" in v:
            why.append(f"{k}: {v['error']}")
    dc = out.get("dist_check")
    if isinstance(dc, dict) and dc.get("result") != "bit-exact":
        why.append(f"dist_check: {dc}")
    return why


def emit_line(out, cpu):
    """Rank 0's one JSON line on the saved stdout -- at most once per process, whichever thread
    (the main one or a leg's watchdog) gets there first."""
    with _EMIT_LOCK:
        if _EMIT.get("emitted"):
            return False
        _EMIT["emitted"] = True
    args, world = _EMIT["args"], _EMIT["world"]
    out = dict(out)
    line = {"metric": out.pop("metric"), "value": out.pop("value"), "unit": out.pop("unit"),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": out.pop("ms_per_step"), "higher_is_better": True,
            "scaling": out.pop("scaling", "weak"),
            "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (uniform residues per RNS limb, seeded)",
            "config": out.pop("config")}
    line.update(out)
    # why the live rocprofv3 passes did not run, at the top level of the line (the per-roofline
    # *_live_error fields say it again where the committed profiles stand in)
    skip = "--no-pmc" if getattr(args, "no_pmc", False) else profiled_parent()
    if skip:
        line["pmc_skipped"] = skip
    line["cpu_baseline"] = cpu
    sys.stdout.flush()
    os.write(_EMIT["json_fd"], (json.dumps(line) + "\n").encode())
    return True


EXIT_LEG_FAILED = 3  # the line was printed, but a leg failed, hung or a dist_check mismatched


def guarded_leg(fn, out, rank, name, timeout_s=180.0):
    """Runs a ride-along leg (or the dist_check) after the headline is measured, so that nothing
    it does can cost the headline line -- but neither can it pass for a success: an exception
    becomes {"error": ...} in the line and the process exits EXIT_LEG_FAILED after printing it
    (main / conclude), and a leg still running after `timeout_s` (e.g. a collective that never
    completes on some node) makes rank 0 print the line without it and every rank exit
    EXIT_LEG_FAILED at once."""

    def fire():
        if rank == 0:
            o = dict(out)
            o[name] = {"error": f"did not finish within {timeout_s:.0f} s; line emitted without it"}
            emit_line(o, None)
        sys.stderr.write(f"bench.py: {name} did not finish within {timeout_s:.0f} s\n")
        sys.stderr.flush()
        os._exit(EXIT_LEG_FAILED)

    timer = threading.Timer(timeout_s, fire)
    timer.daemon = True
    timer.start()
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 -- reported in the line, then a non-zero exit
        _EMIT.setdefault("failed", []).append(f"{name}: {type(e).__name__}")
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        timer.cancel()


def conclude(out, cpu, rank):
    """Print rank 0's line, then the exit status of this rank: 0, or EXIT_LEG_FAILED when a leg
    raised or hung, or the dist_check found mismatched words (every rank sees the summed count,
    so every rank exits non-zero together)."""
    if rank == 0:
        emit_line(out, cpu)
    why = failure_reasons(out)
    if why:
        sys.stderr.write("bench.py: exiting %d: %s\n" % (EXIT_LEG_FAILED, "; ".join(why)))
        return EXIT_LEG_FAILED
    return 0


def main():
    # stdout carries exactly one JSON line: anything else the libraries print there (RCCL prints
    # its version banner to stdout when a communicator comes up) is sent to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    args = parse()
    if args.workload == "keyswitch" and args.batch is not None:
        args.ks_batch = args.batch
    if args.batch is None:
        # mul-relin and rotate at the key-switch's best batch (32: profiles/r04_ks_batch_sweep.txt,
        # r04_mulrelin_rotate_batch_ab.txt: +2 % / +4 % over 16)
        args.batch = {"hommult": 64, "mulrelin": 32, "rotate": 32, "rotsum": 32,
                      "lintrans": 32}.get(
            args.workload, 16)
    world, rank = dist_setup(args)
    _EMIT.update(json_fd=json_fd, args=args, world=world)
    run = {"hommult": run_hommult, "ntt": run_ntt, "keyswitch": run_keyswitch, "vec": run_vec,
           "mulrelin": run_mulrelin, "ntt-batch": run_ntt_batch, "rotate": run_rotate,
           "rotsum": run_rotsum, "lintrans": run_lintrans}[args.workload]
    out, cpu = run(args, world, rank)
    rc = conclude(out, cpu, rank)
    if world > 1:
        torch.distributed.destroy_process_group()
    if rc:
        sys.exit(rc)


if __name__ == "__main__":
    main()
