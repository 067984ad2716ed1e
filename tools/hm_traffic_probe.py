"""The profiled command of bench.py's live HBM-traffic measurement (measurement infrastructure, not
product): a few HomMult calls at the bench shape on cuda:0 through the C ABI, so that a
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` pass over this process sees the same
k_hommult_row launches as the timed run.  With --peak it then runs the butterfly ceiling kernels of
tools/microbench/bfly_peak.hip in the same process (the VALU pass: SQ_INSTS_VALU and
GRBM_GUI_ACTIVE of both) and prints their HIP-event times as one JSON line.  bench.py runs it as a
child process (Popen; never exec).
usage: python tools/hm_traffic_probe.py --log-n 16 --limbs 8 --batch 64 [--calls 4] [--peak]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))

import torch  # noqa: E402

import fhecore as fc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--limbs", type=int, default=8)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--peak", action="store_true")
    a = ap.parse_args()
    n = 1 << a.log_n
    ctx = fc.Context(a.log_n, L=a.limbs)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234)
    x = torch.stack([torch.randint(0, q, (a.batch, 2, n), generator=gen, dtype=torch.int64,
                                   device="cuda") for q in ctx.moduli], 2)
    y = torch.stack([torch.randint(0, q, (a.batch, 2, n), generator=gen, dtype=torch.int64,
                                   device="cuda") for q in ctx.moduli], 2)
    d = ctx.empty(a.batch, 3, a.limbs, n)
    for _ in range(a.calls):
        ctx.hommult(x, y, out=d)
    torch.cuda.synchronize()
    out = {"calls": a.calls, "batch": a.batch}
    if a.peak:
        lib = ctypes.CDLL(os.environ.get("FHE_PEAK_LIB") or
                          os.path.join(ROOT, "tools", "microbench", "libbflypeak.so"))
        lib.fhe_peak_bfly.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double)]
        blocks = 8 * torch.cuda.get_device_properties(0).multi_processor_count
        ms = {}
        for inv in (0, 1):
            rate, t = ctypes.c_double(), ctypes.c_double()
            if lib.fhe_peak_bfly(inv, blocks, 256, 20, ctypes.byref(rate), ctypes.byref(t)):
                raise RuntimeError("fhe_peak_bfly failed")
            ms["inverse" if inv else "forward"] = t.value
        out["peak_ms_per_launch"] = ms
    print(json.dumps(out))


if __name__ == "__main__":
    main()
