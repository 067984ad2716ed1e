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


def test_graph_keeps_its_allocations_and_refuses_internal_workspace(fc):
    """a graph captured without workspace=/out= must not reference memory that is
    freed and reused after capture.  The Context's own allocations inside the block are kept by
    the Graph; replays after heavy allocation churn still reproduce the eager result.  At the C
    ABI a NULL workspace is refused while capturing (the internal workspace could be regrown)."""
    import ctypes

    import torch
    from fhecore.context import _ptr

    log_n, L = 12, 3
    ctx = fc.Context(log_n, L=L)
    d = fc.to_device
    a, b = d(rand(ctx.moduli, log_n, (2, 2), seed=15)), d(rand(ctx.moduli, log_n, (2, 2), seed=16))
    eager = fc.to_host(ctx.hommult(a, b))
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        with fc.Graph() as g:
            out = ctx.hommult(a, b)  # output and workspace allocated inside the capture
        assert any(t.data_ptr() == out.data_ptr() for t in g.tensors) and len(g.tensors) >= 2
        del out
        junk = [torch.full((1 << 20,), -1, dtype=torch.int64, device=a.device) for _ in range(8)]
        g.launch()
        g.launch()
    stream.synchronize()
    assert all((j == -1).all() for j in junk)  # replays wrote only the graph's own buffers
    assert (fc.to_host(g.tensors[0]) == eager).all()
    # the C ABI: workspace == NULL during capture -> FHE_EINVAL, and the capture still ends cleanly
    lib = fc.load()
    dst = ctx.empty(2, 3, L, 1 << log_n)
    with torch.cuda.stream(stream):
        sp = ctypes.c_void_p(stream.cuda_stream)
        assert lib.fhe_graph_begin(sp) == 0
        rc = lib.fhe_hommult(ctx.handle, _ptr(dst), _ptr(a), _ptr(b), 2, 0, L, None, sp)
        gr = ctypes.c_void_p()
        lib.fhe_graph_end(sp, ctypes.byref(gr))
        if gr.value:
            lib.fhe_graph_destroy(gr)
    assert rc != 0 and "capturing" in lib.fhe_last_error().decode()
