"""CPU checks of bench.py's guards (no GPU).

* A ride-along leg that raises is reported inside the line, and the run then exits non-zero.
* A leg that never finishes makes rank 0 print the line without it, and every rank exits non-zero.
* The multi-rank dist_check (every rank's shard of the sharded key-switch / HomMult against its
  single-device result) is exact on an honest gloo world-2 run, and a forced mismatch turns into a
  non-zero exit after the line is printed.

The driver's scaling runs therefore always get the headline line, and never read a hang, an error
or a wrong answer as a success."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from fhecore.dist import LimbShard, sharded_keyswitch  # noqa: E402


def _fresh():
    bench._EMIT.clear()
    bench._EMIT["failed"] = []


def test_guarded_leg_reports_exceptions():
    _fresh()

    def boom():
        raise RuntimeError("no communicator")

    res = bench.guarded_leg(boom, {"metric": "m"}, 0, "keyswitch_leg", timeout_s=30)
    assert res == {"error": "RuntimeError: no communicator"}
    assert bench._EMIT["failed"] == ["keyswitch_leg: RuntimeError"]
    _fresh()
    assert bench.guarded_leg(lambda: {"value": 1}, {}, 0, "x", timeout_s=30) == {"value": 1}
    assert bench.failure_reasons({"x": {"value": 1}}) == []


_LINE = """
import argparse, os, sys, time
sys.path.insert(0, {root!r})
import bench
bench._EMIT.update(json_fd=os.dup(1), args=argparse.Namespace(steps=3, warmup=1), world=1)
out = {{"metric": "m", "value": 42.0, "unit": "HomMult/s", "ms_per_step": 1.0,
        "config": {{"workload": "w"}}}}
"""


def _run(body):
    code = _LINE.format(root=ROOT) + body
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=100)
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    return r, lines


def test_guarded_leg_timeout_emits_the_line_and_fails():
    r, lines = _run("""
bench.guarded_leg(lambda: time.sleep(60), out, 0, "keyswitch_leg", timeout_s=1.0)
print("not reached")
""")
    assert r.returncode == bench.EXIT_LEG_FAILED
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["value"] == 42.0 and "did not finish" in line["keyswitch_leg"]["error"]
    assert "not reached" not in r.stdout


def test_leg_error_prints_the_line_then_exits_nonzero():
    r, lines = _run("""
def boom():
    raise RuntimeError("ncclAllGather failed")
out["keyswitch_leg"] = bench.guarded_leg(boom, out, 0, "keyswitch_leg", timeout_s=30)
sys.exit(bench.conclude(out, None, 0))
""")
    assert r.returncode == bench.EXIT_LEG_FAILED
    line = json.loads(lines[0])
    assert line["value"] == 42.0 and "ncclAllGather failed" in line["keyswitch_leg"]["error"]
    assert "exiting 3" in r.stderr


def test_dist_check_mismatch_prints_the_line_then_exits_nonzero():
    r, lines = _run("""
out["dist_check"] = {"result": "MISMATCH", "mismatched_words": 7, "checked": "x"}
sys.exit(bench.conclude(out, None, 0))
""")
    assert r.returncode == bench.EXIT_LEG_FAILED
    assert json.loads(lines[0])["dist_check"]["mismatched_words"] == 7


def test_clean_run_exits_zero_and_emits_once():
    r, lines = _run("""
out["dist_check"] = {"result": "bit-exact", "checked": "x"}
rc = bench.conclude(out, None, 0)
assert not bench.emit_line(out, None)  # a second emit (e.g. a late watchdog) prints nothing
sys.exit(rc)
""")
    assert r.returncode == 0, r.stderr
    assert len(lines) == 1


# ---- the dist_check itself at gloo world 2, against the CPU restatement of the engine ---------

def _dist_worker(rank, world, port, corrupt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from test_dist_cpu import K, L, CpuEngine, _data, _t

        qs, ps, d2, eb, ea, a, b = _data(3)
        eng = CpuEngine(qs, ps)
        shard = LimbShard(L, world, rank)

        def dist_fn(d, kb, ka):
            k0, k1 = sharded_keyswitch(eng, d, kb, ka, shard)
            if corrupt and rank == world - 1:
                k0 = k0.clone()
                k0.view(-1)[5] ^= 1
            return k0, k1

        bad = bench.check_keyswitch_shard(eng, shard, K, _t(d2), _t(eb), _t(ea), dist_fn)
        bad += bench.check_hommult_shard(eng, shard, _t(a), _t(b))
        t = torch.tensor([bad], dtype=torch.int64)
        dist.all_reduce(t)
        q.put((rank, int(t.item())))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("corrupt", [False, True])
def test_dist_check_gloo_world2(corrupt):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, corrupt, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = dict(q.get() for _ in range(world))
    # every rank sees the same summed count: all exit non-zero together on a mismatch
    assert got == {0: (1 if corrupt else 0), 1: (1 if corrupt else 0)}


def test_shard_mismatches_counts_only_own_limbs():
    full = torch.arange(2 * 4 * 8, dtype=torch.int64).reshape(2, 4, 8)
    sh = LimbShard(4, 2, 1)
    got = full[:, 2:4].clone()
    assert bench.shard_mismatches(got, full, sh) == 0
    got[1, 0, 3] += 1
    got[0, 1, 0] -= 1
    assert bench.shard_mismatches(got, full, sh) == 2
    assert bench.shard_mismatches(torch.empty(2, 0, 8), full, LimbShard(4, 8, 7)) == 0


def test_keyswitch_valu_live_parsing(monkeypatch):
    """The live VALU pass: per-call VALU of the key-switch kernels (torch's own and the ceiling
    kernel's excluded), and the ceiling = VALU per ceiling launch / that launch's own time."""
    ns = "void fhe::(anonymous namespace)::"
    rows = [(ns + "k_modup_col<16, 16, 4>(unsigned long*)", "SQ_INSTS_VALU", 100.0),
            (ns + "k_modup_col<16, 16, 4>(unsigned long*)", "SQ_INSTS_VALU", 100.0),
            (ns + "k_moddown_row<16, 16>(unsigned long*)", "SQ_INSTS_VALU", 50.0),
            (ns + "k_moddown_row<16, 16>(unsigned long*)", "SQ_WAVES", 7.0),
            ("void at::native::vectorized_elementwise_kernel<4>(int)", "SQ_INSTS_VALU", 1e9),
            ("void (anonymous namespace)::k_bfly_peak<false>(unsigned long*)", "SQ_INSTS_VALU", 6e8),
            ("void (anonymous namespace)::k_bfly_peak<false>(unsigned long*)", "SQ_INSTS_VALU", 6e8),
            ("void (anonymous namespace)::k_bfly_peak<true>(unsigned long*)", "SQ_INSTS_VALU", 5e8)]
    out = "noise\n" + json.dumps({"calls": 2, "batch": 32,
                                  "peak_ms_per_launch": {"forward": 1.0, "inverse": 1.0}})
    seen = {}

    def fake(counters, probe, args, timeout_s=150):
        seen.update(counters=counters, probe=probe, args=args)
        return rows, out, None

    monkeypatch.setattr(bench, "rocprof_pmc", fake)
    ks, ceil, why = bench.measure_keyswitch_valu_live(16, 32)
    assert why is None and seen["probe"] == "ks_valu_probe.py"
    assert seen["args"] == ["--log-n", "16", "--batch", "32", "--chunks", "1"]
    assert ks == {"k_modup_col<16, 16, 4>": 100.0, "k_moddown_row<16, 16>": 25.0}
    assert ceil == pytest.approx(600.0)  # 6e8 per 1 ms launch = 600 G/s
    monkeypatch.setattr(bench, "rocprof_pmc", lambda *a, **k: (None, None, "timed out"))
    assert bench.measure_keyswitch_valu_live(16, 32) == (None, None, "timed out")


def test_keyswitch_valu_fallback_reads_committed_profile(monkeypatch):
    """Without the live pass (--no-pmc) the key-switch VALU roofline comes from the newest committed
    profiles/rNN_keyswitch_pmc.json, which must carry per-step counts for the leg's batch; a failed
    live pass falls back the same way and says why."""
    from types import SimpleNamespace

    leg = SimpleNamespace(live_pmc=False, B=32, chunks=1, step_s=2.0e-3, log_n=16)
    r = bench.KeyswitchLeg.valu_roofline(leg)
    assert r["frac"] is not None and 0.2 < r["frac"] < 1.5, r
    assert r["valu_source"].startswith("committed") and r["valu_live_error"] == "--no-pmc"
    monkeypatch.setattr(bench, "measure_keyswitch_valu_live", lambda *a: (None, None, "timed out"))
    leg.live_pmc = True
    r = bench.KeyswitchLeg.valu_roofline(leg)
    assert r["valu_live_error"] == "timed out" and r["frac"] is not None
    leg.B = 7  # no committed profile of that batch
    assert bench.KeyswitchLeg.valu_roofline(leg)["frac"] is None
    leg.B, leg.chunks = 32, 4  # nor of that launch layout
    assert bench.KeyswitchLeg.valu_roofline(leg)["frac"] is None


def test_rocprof_pmc_skips_under_a_profiler(monkeypatch):
    """Under a profiler (the rocprofiler tool library in LD_PRELOAD) a nested rocprofv3 would exec
    its target after its launcher initialised the GPU -- refused on the GPU box (round 4,
    tools/kspmc.sh).  rocprof_pmc must then return the reason without starting any process.
    ROCPROF* / ROCP_* settings without the preload start nothing and switch nothing off."""
    import subprocess

    def no_popen(*a, **k):
        raise AssertionError("rocprof_pmc started a process under a profiler")

    monkeypatch.setattr(subprocess, "Popen", no_popen)
    for var, val in (("LD_PRELOAD", "/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so"),):
        for k in [k for k in os.environ if k.startswith(("ROCPROF", "ROCP_"))]:
            monkeypatch.delenv(k)
        monkeypatch.delenv("LD_PRELOAD", raising=False)
        monkeypatch.setenv(var, val)
        assert bench.profiled_parent() is not None
        rows, out, why = bench.rocprof_pmc(["SQ_WAVES"], "ks_valu_probe.py", [])
        assert rows is None and out is None and why.startswith("skipped: this process runs under")
        # and the live measurements built on it report the skip instead of a number
        ks, ceil, why2 = bench.measure_keyswitch_valu_live(16, 32)
        assert ks is None and why2 == why
        live, why3 = bench.measure_traffic_live("k_hommult_row", [])
        assert live is None and why3 == why
    assert bench.profiled_parent({"LD_PRELOAD": "/usr/lib/libother.so", "PATH": "/bin"}) is None
    for stray in ({"ROCPROF_OUTPUT_PATH": "/tmp/x"}, {"ROCP_TOOL_LIBRARIES": "x.so"}):
        assert bench.profiled_parent(stray) is None


def test_keyswitch_traffic_live_sums_kernels(monkeypatch):
    """The key-switch line's roofline.traffic: FETCH_SIZE and WRITE_SIZE passes (separate) over
    ks_valu_probe.py --no-peak at the leg's batch and chunks; every fhe:: kernel's dispatches summed
    per call, read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB; other kernels ignored."""
    seen = []

    def fake(counters, probe, args, timeout_s=150):
        seen.append((counters, probe, args))
        c = counters[0]
        rows = [("void fhe::(anonymous namespace)::k_modup_col<16, 16, 4>(args)", c, 100.0),
                ("void fhe::(anonymous namespace)::k_modup_col<16, 16, 4>(args)", c, 100.0),
                ("void fhe::(anonymous namespace)::k_ks_row_inner<16, 16, 4, true>(x)", c, 50.0),
                ("ncclDevKernel_AllGather(x)", c, 1e9), ("other", "SQ_WAVES", 5.0)]
        return rows, '{"calls": 2, "batch": 32, "chunks": 1}\n', None

    monkeypatch.setattr(bench, "rocprof_pmc", fake)
    per, total, why = bench.measure_keyswitch_traffic_live(16, 32, 1)
    assert why is None and [s[0] for s in seen] == [["FETCH_SIZE"], ["WRITE_SIZE"]]
    assert all(s[1] == "ks_valu_probe.py" and "--no-peak" in s[2] and
               s[2][s[2].index("--chunks") + 1] == "1" for s in seen)
    # per call: modup 200 KiB fetched x 2 + 200 KiB written over 2 calls
    assert per["k_modup_col<16, 16, 4>"] == (200 * 2048 + 200 * 1024) / 2
    assert per["k_ks_row_inner<16, 16, 4, true>"] == (50 * 2048 + 50 * 1024) / 2
    assert total == int(sum(per.values()))
    monkeypatch.setattr(bench, "rocprof_pmc", lambda *a, **k: (None, None, "skipped: x"))
    assert bench.measure_keyswitch_traffic_live(16, 32) == (None, None, "skipped: x")


def test_hommult_valu_live_rates_and_clocks(monkeypatch):
    """The HomMult line's roofline_valu: one SQ_INSTS_VALU / SQ_WAVES / GRBM_GUI_ACTIVE pass over
    hm_traffic_probe.py --peak; achieved = VALU per k_hommult_row launch over the run's kernel
    time, ceiling = the faster k_bfly_peak, clocks from GRBM_GUI_ACTIVE / 8 XCDs / duration."""
    seen = {}

    def fake(counters, probe, args, timeout_s=150):
        seen.update(counters=counters, probe=probe, args=args)
        rows = []
        for k, valu, grbm in (("void fhe::(anonymous namespace)::k_hommult_row<16, 16>(x)", 4e8, 8 * 2e6),
                              ("void (anonymous namespace)::k_bfly_peak<false>(x)", 6e8, 8 * 2.4e6),
                              ("void (anonymous namespace)::k_bfly_peak<true>(x)", 5e8, 8 * 2.4e6)):
            rows += [(k, "SQ_INSTS_VALU", valu), (k, "GRBM_GUI_ACTIVE", grbm), (k, "SQ_WAVES", 1.0)]
        meta = '{"calls": 4, "batch": 64, "peak_ms_per_launch": {"forward": 1.0, "inverse": 1.0}}\n'
        return rows, meta, None

    monkeypatch.setattr(bench, "rocprof_pmc", fake)
    r, why = bench.measure_hommult_valu_live(16, 8, 64, 1.0)
    assert why is None and seen["probe"] == "hm_traffic_probe.py" and "--peak" in seen["args"]
    assert seen["counters"] == ["SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE"]
    assert r["achieved"] == pytest.approx(400.0) and r["peak"] == pytest.approx(600.0)
    assert r["frac"] == pytest.approx(400 / 600, abs=1e-4)
    assert r["clock_ghz"] == pytest.approx(2.0) and r["peak_clock_ghz"] == pytest.approx(2.4)
    assert r["frac_per_cycle"] == pytest.approx(400 / 600 * 2.4 / 2.0, abs=1e-3)
    monkeypatch.setattr(bench, "rocprof_pmc", lambda *a, **k: (None, None, "skipped: x"))
    assert bench.measure_hommult_valu_live(16, 8, 64, 1.0) == (None, "skipped: x")


def test_keyswitch_design_minimum_bytes():
    """bench.ks_design_min_bytes: the bytes the fused key-switch's kernel sequence must move
    (DESIGN.md §3).  At the bench shape (B 32, L 16, K 4, dnum 4, N 2^16) 5.989 GB per call, which
    profiles/r06_bench_keyswitch.json's measured 6.046 GB matches to 1 %; a limb shard moves less."""
    b = bench.ks_design_min_bytes(32, 16, 16, 4, 4, 1 << 16)
    assert b == 5989466112
    assert 6046000000 / b < 1.01
    assert bench.ks_design_min_bytes(32, 2, 16, 4, 4, 1 << 16) < b / 3
