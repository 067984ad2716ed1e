"""Single-device key-switch throughput against the batch size (dev probe): fhe_keyswitch at N = 2^16,
L = 16, K = 4, dnum = 4 for each batch given, HIP-event timed on the current stream.  FHECORE_LIB
picks an A/B build.  usage: python tools/ks_batch_probe.py 32 48 64"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-fhe_amd"))

import torch  # noqa: E402

import fhecore as fc  # noqa: E402


def main():
    L, K, dnum, n = 16, 4, 4, 1 << 16
    ctx = fc.Context(16, L=L, K=K, dnum=dnum)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)

    def rows(mods, lead):
        return torch.stack([torch.randint(0, q, lead + (n,), generator=gen, dtype=torch.int64,
                                          device="cuda") for q in mods], len(lead))

    eb, ea = rows(ctx.all_moduli, (dnum,)), rows(ctx.all_moduli, (dnum,))
    out = {}
    for B in (int(a) for a in sys.argv[1:]):
        d2 = rows(ctx.moduli, (B,))
        for _ in range(5):
            ctx.keyswitch(d2, eb, ea)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(4, 640 // B)
        e0.record()
        for _ in range(reps):
            ctx.keyswitch(d2, eb, ea)
        e1.record()
        e1.synchronize()
        out[B] = round(B * reps / (e0.elapsed_time(e1) * 1e-3), 1)
        del d2
    print(json.dumps({"keyswitch_per_s": out, "lib": os.environ.get("FHECORE_LIB", "in-tree")}))


if __name__ == "__main__":
    main()
