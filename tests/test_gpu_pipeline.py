"""GPU parity for the fused multiply -> relinearise -> rescale pipeline and HIP-graph replay
(gpu-fhe_amd/csrc/pipeline.hip) against oracle/pyoracle.py mul_relin, plus a
real-key decryption check.  Not in the reference (parity unpinned by the reference)."""
import random

import numpy as np
import pytest

import coracle
import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fc():
    import fhecore

    return fhecore


def rand(mods, log_n, lead=(), seed=0):
    rng = np.random.default_rng(seed)
    n = 1 << log_n
    return np.stack([rng.integers(0, q, size=lead + (n,), dtype=np.uint64) for q in mods],
                    axis=len(lead))


def _oracle(ct_a, ct_b, kb, ka, ctx, rescale):
    qs, ps = ctx.moduli, ctx.all_moduli[ctx.L:]
    d = pyoracle.tensor_ntt(ct_a, ct_b, qs)
    ks0, ks1 = coracle.keyswitch(np.asarray(d[2], dtype=np.uint64), kb, ka, qs, ps, ctx.dnum)
    col = pyoracle._mods_col(qs)
    out = np.stack([(d[0] + ks0.astype(object)) % col, (d[1] + ks1.astype(object)) % col])
    if rescale:
        out = np.stack([coracle.ntt_fwd(np.asarray(pyoracle.rescale_coeff(
            coracle.ntt_inv(np.asarray(o, dtype=np.uint64), qs).astype(object), qs),
            dtype=np.uint64), qs[:-1]).astype(object) for o in out])
    return out


@pytest.mark.parametrize("log_n,L,K,dnum,batch", [(10, 3, 2, 3, 1), (12, 4, 2, 2, 2)])
@pytest.mark.parametrize("rescale", [False, True])
def test_mul_relin_matches_oracle(fc, log_n, L, K, dnum, batch, rescale):
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    a = rand(ctx.moduli, log_n, (batch, 2), seed=1)
    b = rand(ctx.moduli, log_n, (batch, 2), seed=2)
    kb = rand(ctx.all_moduli, log_n, (dnum,), seed=3)
    ka = rand(ctx.all_moduli, log_n, (dnum,), seed=4)
    d = fc.to_device
    got = fc.to_host(ctx.mul_relin(d(a), d(b), d(kb), d(ka), rescale=rescale))
    for i in range(batch):
        want = _oracle(a[i].astype(object), b[i].astype(object), kb, ka, ctx, rescale)
        assert (got[i].astype(object) == want).all()


def test_mul_relin_rescale_decrypts_to_product(fc):
    """Encrypt m1, m2 at scale delta, multiply + relinearise with a real key, rescale: decrypts to
    round(m1 * m2 * delta^2 / q_last) (negacyclic product), up to noise."""
    log_n, L, K, dnum = 10, 3, 2, 3
    n = 1 << log_n
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    qs, ps = ctx.moduli, ctx.all_moduli[L:]
    rng = random.Random(8)
    s = [rng.randrange(-1, 2) for _ in range(n)]
    evk_b, evk_a = pyoracle.gen_relin_key(s, qs, ps, dnum, rng)
    col = pyoracle._mods_col(qs)
    s_n = coracle.ntt_fwd(np.asarray(pyoracle._to_rns(s, qs), dtype=np.uint64), qs).astype(object)
    delta = 1 << 40

    def enc(m):
        a = np.stack([np.array([rng.randrange(q) for _ in range(n)], dtype=object) for q in qs])
        e = pyoracle._to_rns([rng.randrange(-3, 4) for _ in range(n)], qs)
        mm = pyoracle._to_rns([v * delta for v in m], qs)
        body = coracle.ntt_fwd(np.asarray((mm + e) % col, dtype=np.uint64), qs).astype(object)
        return np.stack([(body - a * s_n) % col, a]).astype(np.uint64)

    m1 = [rng.randrange(-8, 9) for _ in range(n)]
    m2 = [rng.randrange(-8, 9) for _ in range(n)]
    d = fc.to_device
    out = fc.to_host(ctx.mul_relin(d(enc(m1)), d(enc(m2)), d(evk_b.astype(np.uint64)),
                                   d(evk_a.astype(np.uint64)), rescale=True))
    q2 = qs[:-1]
    col2 = pyoracle._mods_col(q2)
    dec_n = (out[0].astype(object) + out[1].astype(object) * s_n[:-1]) % col2
    dec = pyoracle.crt_centered(coracle.ntt_inv(np.asarray(dec_n, dtype=np.uint64), q2)
                                .astype(object), q2)
    prod = pyoracle.negacyclic_mul([v % qs[0] for v in m1], [v % qs[0] for v in m2], qs[0])
    prod = [int(v) - qs[0] if int(v) > qs[0] // 2 else int(v) for v in prod]
    scale = delta * delta / qs[-1]
    err = max(abs(int(x) - p * scale) for x, p in zip(dec, prod))
    assert err < scale * 1e-3, err


def test_graph_replay_matches_eager(fc):
    import torch

    log_n, L, K, dnum = 12, 4, 2, 2
    ctx = fc.Context(log_n, L=L, K=K, dnum=dnum)
    d = fc.to_device
    a, b = d(rand(ctx.moduli, log_n, (2, 2), seed=5)), d(rand(ctx.moduli, log_n, (2, 2), seed=6))
    kb, ka = d(rand(ctx.all_moduli, log_n, (dnum,), seed=7)), d(rand(ctx.all_moduli, log_n, (dnum,), seed=8))
    eager = fc.to_host(ctx.mul_relin(a, b, kb, ka, rescale=True))
    ws = ctx.workspace(fc.load().fhe_mul_relin_workspace(ctx.handle, 2))
    out = torch.empty(2, 2, L - 1, 1 << log_n, dtype=torch.int64, device=a.device)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        with fc.Graph() as g:
            ctx.mul_relin(a, b, kb, ka, rescale=True, workspace=ws, out=out)
        out.zero_()
        g.launch()
        g.launch()
    stream.synchronize()
    assert (fc.to_host(out) == eager).all()
