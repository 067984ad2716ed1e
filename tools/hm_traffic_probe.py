"""The profiled command of bench.py's live HBM-traffic measurement (measurement infrastructure, not
product): a few HomMult calls at the bench shape on cuda:0 through the C ABI, so that a
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` pass over this process sees the same
k_hommult_row launches as the timed run.  bench.py runs it as a child process (never exec).
usage: python tools/hm_traffic_probe.py --log-n 16 --limbs 8 --batch 64 [--calls 4]"""
import argparse
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


if __name__ == "__main__":
    main()
