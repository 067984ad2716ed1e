"""Quick GPU parity probe (dev tool): NTT / HomMult / keyswitch vs the C oracle."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gpu-fhe_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import fhecore as fc
import coracle as co
rng = np.random.default_rng(0)
def rand(mods, *lead):
    n = 1 << ln
    return np.stack([rng.integers(0, q, size=lead + (n,), dtype=np.uint64) for q in mods], axis=len(lead))
for ln, L in [(12, 1), (14, 4), (16, 8), (17, 2), (10, 3), (11, 2), (13, 2), (15, 2)]:
    ctx = fc.Context(ln, L=L)
    x = rand(ctx.moduli, 2)
    t = fc.to_device(x)
    ctx.ntt_(t)
    X = fc.to_host(t)
    ref = co.ntt_fwd(x, ctx.moduli)
    ok_f = (X == ref).all()
    ctx.intt_(t)
    ok_i = (fc.to_host(t) == x).all()
    print(f"logN={ln} L={L} fwd {ok_f} inv-roundtrip {ok_i}", flush=True)
    if not ok_f:
        bad = np.argwhere(X != ref); print("  first bad", bad[:5], X[tuple(bad[0])], ref[tuple(bad[0])])
ln, L = 16, 8
ctx = fc.Context(ln, L=L)
a = rand(ctx.moduli, 2, 2); b = rand(ctx.moduli, 2, 2)
d = fc.to_host(ctx.hommult(fc.to_device(a), fc.to_device(b)))
print("hommult", (d == co.hommult(a, b, ctx.moduli)).all(), flush=True)
# keyswitch L=16 K=4 dnum=4 (uniform evk, bit-exact vs oracle)
ln = 16; L = 16; K = 4; dnum = 4
ctx = fc.Context(ln, L=L, K=K, dnum=dnum)
allm = ctx.all_moduli
d2 = rand(ctx.moduli)
eb = rand(allm, dnum); ea = rand(allm, dnum)
ks0, ks1 = ctx.keyswitch(fc.to_device(d2), fc.to_device(eb), fc.to_device(ea))
r0, r1 = co.keyswitch(d2, eb, ea, ctx.moduli, ctx.special, dnum)
print("keyswitch", (fc.to_host(ks0) == r0).all(), (fc.to_host(ks1) == r1).all(), flush=True)
