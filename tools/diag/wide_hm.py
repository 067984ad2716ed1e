"""Diagnostic: the wide-modulus HomMult at N = 2^16, 8 limbs against the C oracle, repeated."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "gpu-fhe_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import numpy as np
import fhecore as fc
import coracle

def rand(mods, log_n, lead=(), seed=0):
    rng = np.random.default_rng(seed)
    n = 1 << log_n
    return np.stack([rng.integers(0, q, size=lead + (n,), dtype=np.uint64) for q in mods], axis=len(lead))

for bits in (62, 63, 61):
    mods = fc.gen_moduli(16, 8, bits=bits)
    ctx = fc.Context(16, moduli=mods)
    a = rand(mods, 16, (1, 2), seed=bits)
    b = rand(mods, 16, (1, 2), seed=bits + 1)
    want = coracle.hommult(a[0], b[0], mods)
    for rep in range(3):
        d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))[0]
        bad = np.argwhere(d != want)
        print(bits, rep, "mismatches", len(bad), "wide", ctx.moduli[0] >= 2**61, flush=True)
        if len(bad):
            polys = np.unique(bad[:, 0]); limbs = np.unique(bad[:, 1])
            print("  polys", polys, "limbs", limbs, "first", bad[:5].tolist(),
                  "got", [int(d[tuple(x)]) for x in bad[:3]], "want", [int(want[tuple(x)]) for x in bad[:3]],
                  "q", [int(mods[x[1]]) for x in bad[:3]], flush=True)
