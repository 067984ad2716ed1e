"""The profiled command of bench.py's live key-switch VALU measurement (measurement
infrastructure, not product): a few fhe_keyswitch_dist calls at the key-switch leg's shape (N = 2^16,
L = 16, K = 4, dnum = 4, one-rank RCCL communicator, the leg's chunks) on cuda:0, then the butterfly
ceiling kernels of tools/microbench/bfly_peak.hip, so that one `rocprofv3 --pmc SQ_INSTS_VALU
SQ_WAVES` pass over this process counts the VALU instructions of every key-switch kernel and of the
ceiling kernel.  Prints one JSON line: the calls made and the ceiling kernels' own HIP-event times.
bench.py runs it as a child process (never exec).
usage: python tools/ks_valu_probe.py --log-n 16 --batch 32 [--chunks 1] [--calls 4]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))

import torch  # noqa: E402

import fhecore as fc  # noqa: E402
from fhecore.dist import RcclComm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--no-peak", action="store_true",
                    help="skip the ceiling kernels (bench.py's HBM-traffic passes count only the "
                         "key-switch)")
    a = ap.parse_args()
    L, K, dnum = 16, 4, 4
    n = 1 << a.log_n
    ctx = fc.Context(a.log_n, L=L, K=K, dnum=dnum)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)

    def rows(mods, lead):
        return torch.stack([torch.randint(0, q, lead + (n,), generator=gen, dtype=torch.int64,
                                          device="cuda") for q in mods], len(lead))

    d2 = rows(ctx.moduli, (a.batch,))
    eb, ea = rows(ctx.all_moduli, (dnum,)), rows(ctx.all_moduli, (dnum,))
    comm = RcclComm()
    ws = ctx.workspace(fc.load().fhe_keyswitch_dist_workspace(ctx.handle, comm.handle, a.batch, a.chunks))
    for _ in range(a.calls):
        ctx.keyswitch_dist(comm, d2, eb, ea, chunks=a.chunks, workspace=ws)
    torch.cuda.synchronize()
    if a.no_peak:
        comm.close()
        print(json.dumps({"calls": a.calls, "batch": a.batch, "chunks": a.chunks}))
        return
    lib = ctypes.CDLL(os.environ.get("FHE_PEAK_LIB") or
                      os.path.join(ROOT, "tools", "microbench", "libbflypeak.so"))
    lib.fhe_peak_bfly.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    blocks = 8 * torch.cuda.get_device_properties(0).multi_processor_count
    ms = {}
    for inv in (0, 1):
        rate, t = ctypes.c_double(), ctypes.c_double()
        if lib.fhe_peak_bfly(inv, blocks, 256, 20, ctypes.byref(rate), ctypes.byref(t)):
            raise RuntimeError("fhe_peak_bfly failed")
        ms["inverse" if inv else "forward"] = t.value
    comm.close()
    print(json.dumps({"calls": a.calls, "batch": a.batch, "chunks": a.chunks,
                      "peak_ms_per_launch": ms}))


if __name__ == "__main__":
    main()
