"""Per-kernel numerics on the MI355X vs plain PyTorch fp32 references of the same op."""
import math

import numpy as np
import pytest
import torch

from tests.parity_util import rel

pytestmark = pytest.mark.gpu


def _attn_ref(qkv, B, T, H, Dh, causal, keep=None, rate=0.0):
    D = H * Dh
    q, k, v = (qkv[:, i * D:(i + 1) * D].float().reshape(B, T, H, Dh) for i in range(3))
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(Dh)
    if causal:
        m = torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril()
        s = s.masked_fill(~m, float("-inf"))
    p = torch.softmax(s, -1)
    if keep is not None:
        p = torch.where(keep, p / (1 - rate), torch.zeros((), device=p.device))
    return torch.einsum("bhqk,bkhd->bqhd", p, v).reshape(B * T, D)


def _unpack_attn_mask(words, T):
    """Decode pcv_attn_drop_mask's packed layout (attention.hip drop_word) into a [T,T] bool mask."""
    n64 = 2 * ((T + 127) // 128)
    q = np.arange(T)[:, None]
    k = np.arange(T)[None, :]
    w = ((((q >> 4) * n64 + (k >> 6)) * 4 + ((q & 15) >> 2)) * 16 + ((k & 15) >> 2) * 4 + ((k & 63) >> 4))
    bit = (q & 3) * 4 + (k & 3)
    return ((words.astype(np.int64)[w] >> bit) & 1).astype(bool)


@pytest.mark.parametrize("T,rate", [(257, 0.1), (100, 0.5), (1030, 0.2)])
def test_attn_drop_mask_bits(dev, T, rate):
    from oracle import rng
    from plaincv_amd import kernels as K
    seed = torch.tensor([4321], dtype=torch.int32, device=dev)
    W = K.attn_mask_words(T)
    mask = torch.zeros(3 * W, dtype=torch.int16, device=dev)
    K.attn_drop_mask(seed, 20, T, rate, mask, layers=3, site_stride=4)
    words = mask.cpu().numpy().view(np.uint16)
    for layer in range(3):
        got = _unpack_attn_mask(words[layer * W:(layer + 1) * W], T)
        assert np.array_equal(got, rng.keep_mask(4321, 20 + 4 * layer, (T, T), rate))


@pytest.mark.parametrize("B,T,H,Dh,causal,rate", [(2, 257, 4, 32, False, 0.0), (2, 100, 2, 64, True, 0.0),
                                                  (1, 1024, 2, 64, True, 0.0), (2, 257, 4, 32, False, 0.1),
                                                  (3, 70, 3, 32, True, 0.0), (2, 100, 2, 64, True, 0.2),
                                                  (1, 300, 2, 32, False, 0.3),
                                                  (1, 2048, 2, 64, True, 0.0)])   # C5: T = 2048, Dh = 64
def test_attention_fwd_bwd(dev, B, T, H, Dh, causal, rate):
    from oracle import rng
    from plaincv_amd import kernels as K
    torch.manual_seed(0)
    D = H * Dh
    qkv = torch.randn(B * T, 3 * D, device=dev).to(torch.bfloat16)
    out = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev)
    seed = torch.tensor([1234], dtype=torch.int32, device=dev)
    mask = None
    if rate > 0:
        mask = torch.zeros(2 * K.attn_mask_words(T), dtype=torch.int16, device=dev)
        K.attn_drop_mask(seed, 3, T, rate, mask, layers=2, site_stride=4)   # layer 1 -> site 7
        mask = mask[K.attn_mask_words(T):]
    K.attn_fwd(qkv, out, lse, B, T, H, Dh, causal, drop_rate=rate, mask=mask)
    keep = None
    if rate > 0:
        keep = torch.from_numpy(rng.keep_mask(1234, 7, (T, T), rate)).to(dev)
    qf = qkv.float().requires_grad_(True)
    ref = _attn_ref(qf, B, T, H, Dh, causal, keep, rate)
    assert (out.float() - ref).abs().max().item() < 2e-2
    do = torch.randn(B * T, D, device=dev).to(torch.bfloat16)
    ref.backward(do.float())
    dqkv = torch.zeros(B * T, 3 * D, device=dev, dtype=torch.bfloat16)
    delta = torch.empty(B * H * T, device=dev)
    K.attn_bwd(qkv, out, do, lse, delta, dqkv, B, T, H, Dh, causal, drop_rate=rate, mask=mask)
    g = qf.grad
    err = (dqkv.float() - g).abs().max().item()
    scale = g.abs().max().item()
    assert err < 3e-2 * max(1.0, scale), (err, scale)


@pytest.mark.parametrize("B,T,H,rate,delta_ready", [(2, 257, 4, 0.1, False), (3, 17, 2, 0.0, False),
                                                     (1, 320, 3, 0.2, True), (2, 1, 2, 0.0, False),
                                                     (2, 64, 4, 0.1, True), (4, 257, 4, 0.0, True),
                                                     (3, 50, 4, 0.1, False), (2, 256, 4, 0.1, False),
                                                     (2, 33, 2, 0.1, False), (2, 241, 4, 0.0, False)])
def test_attention_short_path(dev, B, T, H, rate, delta_ready):
    """One-workgroup-per-(batch, head) kernels for Dh = 32, T <= 320, non-causal (the ViT): against
    the fp32 reference, and against themselves (bit-identical reruns: dQ is summed in a fixed order).
    T = 16 n + 1 (257, 33, 17): the single tail key / query row is handled outside the MFMA blocks.
    B = 64 (the benchmarked batch, XCD placement of the (b, h) workgroups on) is
    test_attention_short_path_c2_batch."""
    _short_path_case(dev, B, T, H, rate, delta_ready)


@pytest.mark.parametrize("rate", [0.0, 0.1])
def test_attention_short_path_c2_batch(dev, rate):
    """The benchmarked shape: B 64, T 257, 4 heads of 32 -- B % 8 == 0, so the (batch, head) workgroups
    are placed on the XCD whose L2 holds batch b's rows."""
    _short_path_case(dev, 64, 257, 4, rate, False)


def _short_path_case(dev, B, T, H, rate, delta_ready):
    from oracle import rng
    from plaincv_amd import kernels as K
    Dh = 32
    D = H * Dh
    g = torch.Generator(device=dev).manual_seed(T + B)
    qkv = torch.randn(B * T, 3 * D, device=dev, generator=g).to(torch.bfloat16)
    do = torch.randn(B * T, D, device=dev, generator=g).to(torch.bfloat16)
    seed = torch.tensor([99], dtype=torch.int32, device=dev)
    mask = None
    if rate > 0:
        mask = torch.zeros(K.attn_mask_words(T), dtype=torch.int16, device=dev)
        K.attn_drop_mask(seed, 5, T, rate, mask)
    res = []
    for _ in range(2):
        out = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(B * H * T, device=dev)
        K.attn_fwd(qkv, out, lse, B, T, H, Dh, False, drop_rate=rate, mask=mask)
        delta = torch.empty(B * H * T, device=dev)
        if delta_ready:
            o4, d4 = out.float().reshape(B, T, H, Dh), do.float().reshape(B, T, H, Dh)
            delta.copy_((o4 * d4).sum(-1).permute(0, 2, 1).reshape(-1))
        dqkv = torch.zeros(B * T, 3 * D, device=dev, dtype=torch.bfloat16)
        K.attn_bwd(qkv, out, do, lse, delta, dqkv, B, T, H, Dh, False, drop_rate=rate, mask=mask,
                   delta_ready=delta_ready)
        torch.cuda.synchronize()
        res.append((out.float(), lse.clone(), dqkv.float(), delta.clone()))
    for x, y in zip(res[0], res[1]):
        assert torch.equal(x, y)
    keep = torch.from_numpy(rng.keep_mask(99, 5, (T, T), rate)).to(dev) if rate > 0 else None
    qf = qkv.float().requires_grad_(True)
    ref = _attn_ref(qf, B, T, H, Dh, False, keep, rate)
    ref.backward(do.float())
    out, lse, dqkv, delta = res[0]
    assert (out - ref).abs().max().item() < 2e-2
    err, scale = (dqkv - qf.grad).abs().max().item(), qf.grad.abs().max().item()
    assert err < 3e-2 * max(1.0, scale), (err, scale)


def test_layernorm_rmsnorm(dev):
    from plaincv_amd import kernels as K
    torch.manual_seed(1)
    R, D = 1000, 128
    x = torch.randn(R, D, device=dev) * 3 + 1
    sc, bi = torch.randn(D, device=dev), torch.randn(D, device=dev)
    y = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(R, device=dev), torch.empty(R, device=dev)
    K.layernorm_fwd(x, sc, bi, y, mean, rstd)
    xr = x.clone().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xr, (D,), sc, bi, eps=1e-6)
    assert torch.allclose(y.float(), ref, atol=3e-2, rtol=1e-2)
    dy = torch.randn(R, D, device=dev)
    ref.backward(dy)
    dres = torch.randn(R, D, device=dev)
    dx = torch.empty(R, D, device=dev)
    dxb = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    ds, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    K.layernorm_bwd(dy, x, sc, mean, rstd, dres, dx, dxb, ds, db)
    assert torch.allclose(dx, xr.grad + dres, atol=1e-3, rtol=1e-3)
    xh = (x - x.mean(-1, keepdim=True)) / torch.sqrt(x.var(-1, unbiased=False, keepdim=True) + 1e-6)
    assert torch.allclose(ds, (dy * xh).sum(0), atol=1e-2, rtol=1e-3)
    assert torch.allclose(db, dy.sum(0), atol=1e-2, rtol=1e-3)
    # RMSNorm (bf16 stream)
    D = 768
    x = (torch.randn(R, D, device=dev) * 2).to(torch.bfloat16)
    sc = torch.rand(D, device=dev) + 0.5
    y = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    rs = torch.empty(R, device=dev)
    K.rmsnorm_fwd(x, sc, y, rs)
    xf = x.float().requires_grad_(True)
    ref = xf * torch.rsqrt((xf * xf).mean(-1, keepdim=True) + 1e-6) * sc
    assert torch.allclose(y.float(), ref, atol=3e-2, rtol=1e-2)
    dy = torch.randn(R, D, device=dev).to(torch.bfloat16)
    ref.backward(dy.float())
    dx = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    ds = torch.zeros(D, device=dev)
    K.rmsnorm_bwd(dy, x, sc, rs, None, dx, ds)
    assert torch.allclose(dx.float(), xf.grad, atol=3e-2, rtol=2e-2)
    gs = (dy.float() * xf.detach() * torch.rsqrt((xf.detach() ** 2).mean(-1, keepdim=True) + 1e-6)).sum(0)
    assert torch.allclose(ds, gs, atol=5e-1, rtol=1e-2)


def test_rope_swiglu_xent_embed(dev):
    from oracle.lm import apply_rotary, precompute_freqs_cis
    from plaincv_amd import kernels as K
    torch.manual_seed(2)
    B, T, H, Dh = 2, 64, 3, 64
    D = H * Dh
    cos, sin = precompute_freqs_cis(Dh, T, 500000.0)
    qkv = torch.randn(B * T, 3 * D, device=dev).to(torch.bfloat16)
    ref_q = apply_rotary(qkv[:, :D].float().cpu().reshape(B, T, H, Dh).to(torch.bfloat16), cos, sin)
    ref_k = apply_rotary(qkv[:, D:2 * D].float().cpu().reshape(B, T, H, Dh).to(torch.bfloat16), cos, sin)
    x = qkv.clone()
    K.rope(x, T, Dh, cos.to(dev), sin.to(dev), ncols=2 * D)
    assert torch.allclose(x[:, :D].float().cpu(), ref_q.reshape(B * T, D).float(), atol=1e-2)
    assert torch.allclose(x[:, D:2 * D].float().cpu(), ref_k.reshape(B * T, D).float(), atol=1e-2)
    assert torch.equal(x[:, 2 * D:], qkv[:, 2 * D:])
    K.rope(x, T, Dh, cos.to(dev), sin.to(dev), backward=True, ncols=2 * D)
    assert (x.float() - qkv.float()).abs().max().item() < 5e-2
    # swiglu
    R, F = 300, 2048
    gu = torch.randn(R, 2 * F, device=dev).to(torch.bfloat16)
    h = torch.empty(R, F, device=dev, dtype=torch.bfloat16)
    K.swiglu_fwd(gu, h)
    g, u = gu[:, :F].float().requires_grad_(True), gu[:, F:].float().requires_grad_(True)
    ref = torch.nn.functional.silu(g) * u
    assert torch.allclose(h.float(), ref, atol=2e-2, rtol=1e-2)
    dh = torch.randn(R, F, device=dev).to(torch.bfloat16)
    ref.backward(dh.float())
    dgu = torch.empty(R, 2 * F, device=dev, dtype=torch.bfloat16)
    K.swiglu_bwd(dh, gu, dgu)
    assert torch.allclose(dgu[:, :F].float(), g.grad, atol=3e-2, rtol=2e-2)
    assert torch.allclose(dgu[:, F:].float(), u.grad, atol=3e-2, rtol=2e-2)
    # xent (bf16 logits, ragged V)
    R, V = 64, 50257
    buf = torch.randn(R, 50264, device=dev).to(torch.bfloat16)
    lg = buf[:, :V]
    lab = torch.randint(0, V, (R,), device=dev, dtype=torch.int32)
    rl, rc = torch.empty(R, device=dev), torch.empty(R, device=dev)
    lcopy = lg.float().clone()
    K.xent(lg, lab, rl, rc, lg, grad_scale=1.0 / R)     # in place: logits -> dlogits
    lr_ = lcopy.requires_grad_(True)
    lref = torch.nn.functional.cross_entropy(lr_, lab.long(), reduction="none")
    assert torch.allclose(rl, lref.detach(), atol=1e-3, rtol=1e-4)
    lref.mean().backward()
    assert torch.allclose(lg.float(), lr_.grad, atol=1e-4)
    assert torch.equal(rc, (lcopy.argmax(-1) == lab.long()).float())
    torch.manual_seed(2)
    # reference on fresh data
    buf2 = torch.randn(R, 50264, device=dev).to(torch.bfloat16)
    lg2 = buf2[:, :V].clone()
    rl2, rc2 = torch.empty(R, device=dev), torch.empty(R, device=dev)
    d2 = torch.empty_like(lg2)
    K.xent(lg2, lab, rl2, rc2, d2, grad_scale=1.0 / R)
    lf = lg2.float().requires_grad_(True)
    loss = torch.nn.functional.cross_entropy(lf, lab.long(), reduction="none")
    assert torch.allclose(rl2, loss.detach(), atol=1e-3, rtol=1e-4)
    loss.mean().backward()
    assert torch.allclose(d2.float(), lf.grad, atol=1e-4)
    assert torch.equal(rc2, (lf.argmax(-1) == lab.long()).float())
    # planted ties: accuracy counts the FIRST maximal index (torch.argmax / jnp.argmax)
    buf3 = torch.randn(R, 50264, device=dev).to(torch.bfloat16)
    lg3 = buf3[:, :V]
    j1 = torch.randint(0, V // 2, (R,), device=dev)
    j2 = j1 + torch.randint(1, V // 2, (R,), device=dev)
    rows = torch.arange(R, device=dev)
    lg3[rows, j1] = 8.0
    lg3[rows, j2] = 8.0
    lab3 = torch.where(rows % 2 == 0, j1, j2).to(torch.int32)
    rl3, rc3 = torch.empty(R, device=dev), torch.empty(R, device=dev)
    K.xent(lg3, lab3, rl3, rc3, None, grad_scale=1.0)
    assert torch.equal(rc3, (rows % 2 == 0).float())
    assert torch.allclose(rl3, torch.nn.functional.cross_entropy(lg3.float(), lab3.long(), reduction="none"),
                          atol=1e-3, rtol=1e-4)
    # ties inside one 16-B chunk (the kernel recovers the first index from the winning chunk)
    buf4 = torch.randn(R, 50264, device=dev).to(torch.bfloat16)
    lg4 = buf4[:, :V]
    k8 = torch.randint(0, V // 8 - 1, (R,), device=dev) * 8
    lg4[rows, k8 + 2] = 9.0
    lg4[rows, k8 + 5] = 9.0
    lab4 = torch.where(rows % 2 == 0, k8 + 2, k8 + 5).to(torch.int32)
    rl4, rc4 = torch.empty(R, device=dev), torch.empty(R, device=dev)
    K.xent(lg4, lab4, rl4, rc4, None, grad_scale=1.0)
    assert torch.equal(rc4, (rows % 2 == 0).float())
    # embedding
    Vv, Dd = 1000, 64
    tab = torch.randn(Vv, Dd, device=dev).to(torch.bfloat16)
    ids = torch.randint(0, Vv, (500,), device=dev, dtype=torch.int32)
    out = torch.empty(500, Dd, device=dev, dtype=torch.bfloat16)
    K.embed_fwd(ids, tab, out)
    assert torch.equal(out, tab[ids.long()])
    dx = torch.randn(500, Dd, device=dev).to(torch.bfloat16)
    dt = torch.zeros(Vv, Dd, device=dev)
    K.embed_bwd(ids, dx, dt)
    ref = torch.zeros(Vv, Dd, device=dev).index_add_(0, ids.long(), dx.float())
    assert torch.allclose(dt, ref, atol=1e-4)


def test_gemm_dropout_matches_oracle_hash(dev):
    from oracle import rng
    from plaincv_amd import kernels as K
    M, N, Kd = 100, 256, 64
    a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    w = torch.randn(Kd, N, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev)
    seed = torch.tensor([99], dtype=torch.int32, device=dev)
    K.gemm(a, w, out, drop_rate=0.25, seed=seed, site=3)
    keep = torch.from_numpy(rng.keep_mask(99, 3, (M, N), 0.25)).to(dev)
    ref = torch.where(keep, (a.float() @ w.float()) / 0.75, torch.zeros((), device=dev))
    assert torch.allclose(out, ref, atol=1e-2, rtol=1e-3)
    frac = keep.float().mean().item()
    assert abs(frac - 0.75) < 0.02


@pytest.mark.parametrize("shapes", [[(128, 256), (256, 128), (128, 200), (48, 100), (128, 128)],
                                    [(96, 256), (7, 33), (200, 64)]])
def test_muon_fused_matches_batched_chain(dev, shapes):
    """pcv_muon_fused (one workgroup per matrix, NS in LDS) vs the batched-GEMM NS chain:
    same momentum, same bf16 NS numerics (up to A'A' vs A'A'^T on a symmetric A'), so the
    updates agree to bf16 rounding of the orthogonalised direction (|du| <= 2e-2 * lr)."""
    from plaincv_amd.optim.muon import Muon
    from plaincv_amd.params import Layout, ParamStore
    lay = Layout()
    for i, s in enumerate(shapes):
        lay.add(f"Dense_{i}/kernel", s)
    lay.add("Dense_0/bias", (shapes[0][1],))
    g = torch.Generator().manual_seed(7)
    init = {k: torch.randn(*l.shape, generator=g) * 0.1 for k, l in lay.leaves.items()}
    grads = [{k: torch.randn(*l.shape, generator=g) for k, l in lay.leaves.items()} for _ in range(3)]
    ups = []
    for fused in (True, False):
        store = ParamStore(lay, dev)
        store.load(init)
        tx = Muon(1e-3, weight_decay=0.1, fused=fused)
        st = tx.init(store)
        assert (st.n_fused > 0) == fused
        for gr in grads:
            store.zero_grad()
            for k, v in gr.items():
                store.grads[k].copy_(v.to(dev))
            tx.step_(store, st)
        torch.cuda.synchronize()
        ups.append({k: (store.params[k].cpu() - init[k]) for k in init})
    for k in init:
        d = (ups[0][k] - ups[1][k]).abs().max().item()
        assert d <= 3 * 2e-2 * 1e-3, (k, d)


@pytest.mark.parametrize("M,N,K,rate", [(1000, 128, 256, 0.0), (777, 128, 128, 0.1), (300, 96, 64, 0.0)])
def test_gemm_ln_forward(dev, M, N, K, rate):
    """pcv_gemm_ln mode 1 (GEMM + bias + dropout + residual, then LayerNorm of each row) vs fp32 torch."""
    from oracle import rng
    from plaincv_amd import kernels as K_
    torch.manual_seed(3)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = (torch.randn(K, N, device=dev) * 0.1).to(torch.bfloat16)
    bias, res = torch.randn(N, device=dev), torch.randn(M, N, device=dev)
    sc, sh = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    seed = torch.tensor([21], dtype=torch.int32, device=dev)
    K_.gemm_ln(a, b, out, ln_mode=1, res=res, ln_scale=sc, ln_bias=sh, ln_y=y, ln_mean=mean, ln_rstd=rstd,
               bias=bias, drop_rate=rate, seed=seed, site=9)
    v = a.float() @ b.float() + bias
    if rate > 0:
        keep = torch.from_numpy(rng.keep_mask(21, 9, (M, N), rate)).to(dev)
        v = torch.where(keep, v / (1 - rate), torch.zeros((), device=dev))
    x1 = v + res
    assert torch.allclose(out, x1, atol=2e-3, rtol=1e-3)
    ref = torch.nn.functional.layer_norm(x1, (N,), sc, sh, eps=1e-6)
    assert (y.float() - ref).abs().max().item() < 3e-2
    assert torch.allclose(mean, x1.mean(-1), atol=1e-4)
    assert torch.allclose(rstd, 1 / torch.sqrt(x1.var(-1, unbiased=False) + 1e-6), rtol=1e-3)


@pytest.mark.parametrize("M,N,K,rate,reps", [(1000, 128, 256, 0.0, 1), (513, 64, 128, 0.0, 1), (700, 128, 384, 0.1, 1),
                                             (1000, 128, 256, 0.1, 32), (1000, 128, 256, 0.1, -1), (16448, 128, 256, 0.1, -1)])
def test_gemm_ln_backward(dev, M, N, K, rate, reps):
    """pcv_gemm_ln mode 2 (dgrad GEMM, LayerNorm backward, residual add, parameter grads, and the
    dropout-backward bf16 copy + column sum consumed by the sublayer below)."""
    from oracle import rng
    from plaincv_amd import kernels as K_
    torch.manual_seed(4)
    dh = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)     # dy = dh @ w^T  (tb=True)
    x = torch.randn(M, N, device=dev) * 2 + 0.5
    sc = torch.rand(N, device=dev) + 0.5
    mean = x.mean(-1)
    rstd = 1 / torch.sqrt(x.var(-1, unbiased=False) + 1e-6)
    dres = torch.randn(M, N, device=dev)
    dx = torch.empty(M, N, device=dev)
    dxb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ds, db, cs = (torch.full((N,), 0.5, device=dev) for _ in range(3))
    seed = torch.tensor([5], dtype=torch.int32, device=dev)
    if reps < 0:   # one plain-stored row per output row tile, summed by a column-sum job
        wss = [torch.full((K_.col_rows(M, reps), N), 9.0, device=dev) for _ in range(3)]
        assert wss[0].shape[0] == -(-M // 64)
        K_.gemm_ln(dh, w, dx, tb=True, ln_mode=2, res=dres, ln_scale=sc, ln_y=dxb, ln_mean=mean, ln_rstd=rstd,
                   ln_x=x, ln_dscale=wss[0], ln_dbias=wss[1], colsum=wss[2], col_reps=reps, drop_rate=rate,
                   seed=seed, site=11)
        snap = [ws_.clone() for ws_ in wss]
        K_.GroupedWGrad([("colsum", ws_, t) for ws_, t in zip(wss, (ds, db, cs))], dev)()
        torch.cuda.synchronize()
        assert all(torch.equal(a_, b_) for a_, b_ in zip(snap, wss))   # plain column sums leave the rows
        assert all((ws_[: -(-M // 64)] != 9.0).all() for ws_ in wss)      # every row of the buffer was stored
    elif reps > 1:   # replica rows [reps, N], folded afterwards
        wss = [torch.zeros(reps, N, device=dev) for _ in range(3)]
        K_.gemm_ln(dh, w, dx, tb=True, ln_mode=2, res=dres, ln_scale=sc, ln_y=dxb, ln_mean=mean, ln_rstd=rstd,
                   ln_x=x, ln_dscale=wss[0], ln_dbias=wss[1], colsum=wss[2], col_reps=reps, drop_rate=rate,
                   seed=seed, site=11)
        K_.GroupedWGrad([("fold", ws, t) for ws, t in zip(wss, (ds, db, cs))], dev)()
        torch.cuda.synchronize()
        assert all(ws.abs().max().item() == 0.0 for ws in wss)   # fold resets the replicas
    else:
        K_.gemm_ln(dh, w, dx, tb=True, ln_mode=2, res=dres, ln_scale=sc, ln_y=dxb, ln_mean=mean, ln_rstd=rstd,
                   ln_x=x, ln_dscale=ds, ln_dbias=db, colsum=cs, drop_rate=rate, seed=seed, site=11)
    dy = dh.float() @ w.float().t()
    xr = x.clone().requires_grad_(True)
    scr = sc.clone().requires_grad_(True)
    shr = torch.zeros(N, device=dev, requires_grad=True)
    torch.nn.functional.layer_norm(xr, (N,), scr, shr, eps=1e-6).backward(dy)
    ref = xr.grad + dres
    assert torch.allclose(dx, ref, atol=2e-3, rtol=2e-3), (dx - ref).abs().max().item()
    yref = ref
    if rate > 0:
        keep = torch.from_numpy(rng.keep_mask(5, 11, (M, N), rate)).to(dev)
        yref = torch.where(keep, ref / (1 - rate), torch.zeros((), device=dev))
    assert (dxb.float() - yref).abs().max().item() < 3e-2
    assert torch.allclose(ds - 0.5, scr.grad, atol=5e-2, rtol=2e-3)
    assert torch.allclose(db - 0.5, shr.grad, atol=5e-2, rtol=2e-3)
    assert torch.allclose(cs - 0.5, yref.sum(0), atol=5e-2, rtol=2e-3)


@pytest.mark.parametrize("M,N,K", [(1000, 256, 128), (777, 200, 64)])
def test_gemm_colsum_epilogue(dev, M, N, K):
    """Generic GEMM epilogue column sum (bias gradient of the layer that produced the output)."""
    from plaincv_amd import kernels as K_
    torch.manual_seed(6)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)
    aux = torch.randn(M, N, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.ones(N, device=dev)
    K_.gemm(a, w, out, tb=True, aux=aux, act=K_.EPI_GELU_BWD, colsum=cs)
    xa = aux.float().requires_grad_(True)
    gl = torch.nn.functional.gelu(xa, approximate="tanh")
    (gd,) = torch.autograd.grad(gl, xa, torch.ones_like(gl))
    ref = (a.float() @ w.float().t()) * gd
    assert (out.float() - ref).abs().max().item() < 5e-2
    assert torch.allclose(cs - 1.0, ref.sum(0), atol=5e-2, rtol=1e-2)


@pytest.mark.parametrize("tile", [64, 128])
def test_grouped_wgrad(dev, tile):
    """One grouped launch of weight-gradient GEMMs == separate fp32 A^T B accumulations, split-K partials
    and the row slices of the column sums through the workspace + fold launch: a repeat from the same
    C / column accumulators is bit-identical."""
    from plaincv_amd import kernels as K_
    torch.manual_seed(9)
    shapes = [(16640, 128, 384), (16640, 128, 128), (16640, 128, 512), (16640, 512, 128), (300, 72, 40),
              (64, 8, 8)]
    items, refs = [], []
    for Kd, M, N in shapes:
        a = torch.randn(Kd, M, device=dev).to(torch.bfloat16)
        b = torch.randn(Kd, N, device=dev).to(torch.bfloat16)
        c = torch.randn(M, N, device=dev)
        refs.append(c + 0.5 * (a.float().t() @ b.float()))
        items.append((a, b, c, 0.5))
    # column-sum jobs in the same launch (bf16 and fp32 inputs, ragged row counts, strided rows)
    xs = [torch.randn(16640, 392, device=dev)[:, :384].to(torch.bfloat16), torch.randn(1001, 136, device=dev)[:, :128],
          torch.randn(7, 8, device=dev).to(torch.bfloat16)]
    outs = [torch.randn(x.shape[1], device=dev) for x in xs]
    cref = [o + x.float().sum(0) for x, o in zip(xs, outs)]
    g = K_.GroupedWGrad(items + [("colsum", x, o) for x, o in zip(xs, outs)], dev, tile=tile)
    assert g.fold_blocks > 0 and g.ws is not None
    c0 = [c.clone() for _, _, c, _ in items]
    o0 = [o.clone() for o in outs]
    g()
    torch.cuda.synchronize()
    first = [c.clone() for _, _, c, _ in items] + [o.clone() for o in outs]
    for (_, _, c, _), c_ in zip(items, c0):
        c.copy_(c_)
    for o, o_ in zip(outs, o0):
        o.copy_(o_)
    g()
    torch.cuda.synchronize()
    for t, f in zip([c for _, _, c, _ in items] + outs, first):
        assert torch.equal(t, f)
    for o, r in zip(outs, cref):
        assert torch.allclose(o, r, atol=2e-2, rtol=1e-4), (o - r).abs().max().item()
    for (a, b, c, _), ref in zip(items, refs):
        err = (c - ref).abs().max().item()
        assert err < 2e-3 * max(1.0, ref.abs().max().item()), err
    # a second run accumulates again (beta = 1 semantics)
    for (a, b, c, _), ref in zip(items, refs):
        c.copy_(ref)
    for o, r in zip(outs, cref):
        o.copy_(r)
    g()
    torch.cuda.synchronize()
    for (a, b, c, _), ref in zip(items, refs):
        ref2 = ref + 0.5 * (a.float().t() @ b.float())
        assert (c - ref2).abs().max().item() < 2e-3 * max(1.0, ref2.abs().max().item())


@pytest.mark.parametrize("B,T,H,Dh", [(4, 257, 4, 32), (2, 128, 12, 64), (16, 1024, 12, 64), (8, 2048, 16, 64)])
def test_gemm_attn_delta_epilogue(dev, B, T, H, Dh):
    """dO GEMM epilogue computing the attention-backward delta = rowsum per head of dO * O (the last two:
    the LM bench shapes, on the 256-wide kernel's form of the epilogue)."""
    from plaincv_amd import kernels as K_
    torch.manual_seed(12)
    R, D = B * T, H * Dh
    dy = torch.randn(R, D, device=dev).to(torch.bfloat16)
    w = (torch.randn(D, D, device=dev) * 0.1).to(torch.bfloat16)
    o = torch.randn(R, D, device=dev).to(torch.bfloat16)
    do = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    delta = torch.full((B * H * T,), 7.0, device=dev)
    K_.gemm(dy, w, do, tb=True, attn_delta=(o, delta, T, H))
    ref_do = (dy.float() @ w.float().t())
    assert (do.float() - ref_do).abs().max().item() < 5e-2 * max(1.0, ref_do.abs().max().item())
    ref = (do.float() * o.float()).reshape(B, T, H, Dh).sum(-1).permute(0, 2, 1).reshape(-1)
    assert torch.allclose(delta, ref, atol=1e-3, rtol=1e-3), (delta - ref).abs().max().item()


def test_transpose_batch(dev):
    from plaincv_amd import kernels as K_
    torch.manual_seed(8)
    shapes = [(768, 2304), (100, 37), (64, 64), (130, 1000)]
    pairs, srcs = [], []
    for r, c in shapes:
        base = torch.randn(r, (c + 7) // 8 * 8, device=dev).to(torch.bfloat16)
        src = base[:, :c]
        dst = torch.zeros(c, (r + 7) // 8 * 8, device=dev, dtype=torch.bfloat16)[:, :r]
        pairs.append((src, dst))
        srcs.append(src)
    K_.TransposeBatch(pairs, dev)()
    for src, dst in pairs:
        assert torch.equal(dst, src.t())


@pytest.mark.parametrize("split", [True, False, "defer"])
@pytest.mark.parametrize("B,D,Kc,rate", [(64, 128, 200, 0.1), (4, 64, 10, 0.0), (33, 96, 256, 0.3), (1, 32, 1, 0.0)])
def test_vit_head_fused(dev, B, D, Kc, rate, split):
    """csrc/vit_head.hip vs torch fp32 on the same bf16-rounded GEMM operands: LayerNorm of strided cls
    rows, logits, CE metrics, dlogits, the head bias / LN parameter gradients, dx and the dropout-VJP
    bf16 rows (dropout bits from oracle.rng at the flat index (b * T) * D + c).  split: one
    workgroup per 16 rows with the last-workgroup reduction; a second launch on the same workspace
    (ticket reset by the kernel) reproduces the first bit for bit.  defer: the workgroups leave their
    partial rows for a later fold (done here row by row, as the grouped launch's fold jobs)."""
    from oracle import rng
    from plaincv_amd import kernels as K
    T = 5
    g = torch.Generator().manual_seed(B + D + Kc)
    X = torch.randn(B * T, D, generator=g).to(dev)
    x = X.view(B, T * D)[:, :D]
    s, c = (torch.rand(D, generator=g) + 0.5).to(dev), (0.1 * torch.randn(D, generator=g)).to(dev)
    Kp = (Kc + 7) // 8 * 8
    Wfull = torch.zeros(D, Kp, dtype=torch.bfloat16, device=dev)
    Wfull[:, :Kc] = (0.1 * torch.randn(D, Kc, generator=g)).to(torch.bfloat16).to(dev)
    W = Wfull[:, :Kc]
    bias = (0.1 * torch.randn(Kc, generator=g)).to(dev)
    labels = torch.randint(0, Kc, (B,), generator=g, dtype=torch.int32).to(dev)
    yf = torch.empty(B, D, dtype=torch.bfloat16, device=dev)
    logits = torch.empty(B, Kp, device=dev)[:, :Kc]
    bad_defer = split == "defer" and not (B > 16 and Kc % 8 == 0 and D % 8 == 0)
    met = torch.empty(8 if split == "defer" else 2, device=dev)
    dl = torch.empty(B, Kp, device=dev)[:, :Kc]
    dlb = torch.zeros(B, Kp, dtype=torch.bfloat16, device=dev)[:, :Kc]
    DX = torch.zeros(B * T, D, device=dev)
    DYM = torch.zeros(B * T, D, dtype=torch.bfloat16, device=dev)
    gs, gc, gb = torch.full((D,), 0.5, device=dev), torch.full((D,), -0.25, device=dev), torch.full((Kc,), 1.0, device=dev)
    seed = torch.tensor([99], dtype=torch.int32, device=dev)
    work = K.vit_head_work(B, D, Kc, dev) if split else None

    def run():
        K.vit_head(x, s, c, W, bias, labels, yf, logits, met, grad_scale=1.0 / B, dlogits=dl, dlogits_b=dlb,
                   dx=DX.view(B, T * D)[:, :D], dscale=gs, dbias=gc, dym=DYM.view(B, T * D)[:, :D], drop_rate=rate,
                   seed=seed, site=13, row_stride=T, dhead_bias=gb, work=work, defer=split == "defer")
        if split == "defer":
            v = K.vit_head_fold_views(work, B, D, Kc)
            assert float(met.abs().sum()) == 0.0            # zeroed by the head, for the fold to add into
            for key, out in (("metrics", met), ("dhead_bias", gb), ("dscale", gs), ("dbias", gc)):
                for j in range(v[key].shape[0]):
                    out += v[key][j]
    if bad_defer:   # deferred head sums need B > 16 and K, D multiples of 8: refused before any launch
        with pytest.raises((RuntimeError, ValueError)):
            run()
        return
    run()
    if split:
        first = [t.clone() for t in (met, gs, gc, gb, DX, DYM, dl)]
        gs.fill_(0.5), gc.fill_(-0.25), gb.fill_(1.0)
        run()
        for a, b in zip(first, (met, gs, gc, gb, DX, DYM, dl)):
            assert torch.equal(a, b)
    torch.cuda.synchronize()
    # torch reference with the same bf16 operand rounding
    xr = x.clone().requires_grad_(True)
    sr, cr = s.clone().requires_grad_(True), c.clone().requires_grad_(True)
    mu = xr.mean(-1, keepdim=True)
    var = ((xr * xr).mean(-1, keepdim=True) - mu * mu).clamp(min=0)
    y = (xr - mu) * torch.rsqrt(var + 1e-6) * sr + cr
    yb = y.to(torch.bfloat16).float()
    z = yb @ W.float() + bias
    assert rel(logits, z.detach()) < 1e-5
    assert rel(yf.float(), y.detach()) < 4e-3                # bf16 rounding of the LN output
    lse = torch.logsumexp(z, -1)
    loss = (lse - z.gather(1, labels.long()[:, None])[:, 0]).mean()
    acc = (z.argmax(-1) == labels.long()).float().mean()
    assert abs(met[0].item() - loss.item()) < 1e-5 and abs(met[1].item() - acc.item()) < 1e-6
    d_ref = (torch.softmax(z, -1) - torch.nn.functional.one_hot(labels.long(), Kc).float()) / B
    assert rel(dl, d_ref.detach()) < 1e-5
    assert rel(gb - 1.0, d_ref.detach().sum(0)) < 1e-5
    dy = dlb.float() @ W.float().t()                         # the bf16 dlogits operand, as the GEMM
    gx, gsr, gcr = torch.autograd.grad(y, (xr, sr, cr), dy)
    got_dx = DX.view(B, T * D)[:, :D]
    assert rel(got_dx, gx) < 1e-4
    assert rel(gs - 0.5, gsr) < 1e-4 and rel(gc + 0.25, gcr) < 1e-4
    keep = torch.ones(B, D, dtype=torch.bool)
    if rate > 0:
        km = rng.keep_mask(99, 13, (B * T, D), rate)
        keep = torch.from_numpy(km).view(B, T * D)[:, :D]
    want = torch.where(keep.to(dev), gx / (1 - rate), torch.zeros((), device=dev)).to(torch.bfloat16).float()
    assert rel(DYM.view(B, T * D)[:, :D].float(), want) < 4e-3
    others = DYM.view(B, T, D)[:, 1:]
    assert (others == 0).all()


@pytest.mark.parametrize("rate", [0.0, 0.1])
def test_vit_embed_ln_fused(dev, rate):
    """pcv_vit_embed_ln_fwd == pcv_vit_embed_fwd + pcv_layernorm_fwd, bit for bit (x, y, mean, rstd)."""
    from plaincv_amd import kernels as K_
    B, T, D = 64, 257, 128
    g = torch.Generator(device=dev).manual_seed(1)
    patch = torch.randn(B * (T - 1), D, device=dev, generator=g)
    cls, pos = torch.randn(D, device=dev, generator=g), torch.randn(T, D, device=dev, generator=g)
    sc, bi = torch.randn(D, device=dev, generator=g), torch.randn(D, device=dev, generator=g)
    seed = torch.tensor([11], dtype=torch.int32, device=dev)
    outs = []
    for fused in (True, False):
        x = torch.empty(B * T, D, device=dev)
        y = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
        mean, rstd = torch.empty(B * T, device=dev), torch.empty(B * T, device=dev)
        if fused:
            K_.vit_embed_ln_fwd(patch, cls, pos, x, B, T, D, sc, bi, y, mean, rstd, rate=rate, seed=seed, site=1)
        else:
            K_.vit_embed_fwd(patch, cls, pos, x, None, B, T, D, rate, seed, 1)
            K_.layernorm_fwd(x, sc, bi, y, mean, rstd)
        torch.cuda.synchronize()
        outs.append((x, y, mean, rstd))
    for name, a, b in zip(("x", "y", "mean", "rstd"), *outs):
        bad = (a != b).nonzero()
        assert bad.numel() == 0, (name, bad.shape[0], bad[:4].tolist(), (a.float() - b.float()).abs().max().item(),
                                  a.flatten()[:4].tolist(), b.flatten()[:4].tolist())


def test_gemm_gelu_saved_derivative(dev):
    """EPI_GELU_D (forward: out = gelu(h), aux = bf16(gelu'(h))) + EPI_MUL_AUX (backward: out *= aux)
    against EPI_GELU / EPI_GELU_BWD on the same operands: the forward outputs are bit-identical (the
    same sigmoid form); aux is gelu' at the fp32 pre-activation within bf16 rounding of the exact
    torch derivative; the backward product within bf16 rounding of dY * gelu'(h)."""
    from plaincv_amd import kernels as K_
    M, N, Kd = 16448, 256, 128
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
    w = (0.2 * torch.randn(Kd, N, device=dev, generator=g)).to(torch.bfloat16)
    bias = torch.randn(N, device=dev, generator=g)
    o1, o2 = (torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2))
    h, d = (torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2))
    K_.gemm(x, w, o1, bias=bias, aux=h, act=K_.EPI_GELU)
    K_.gemm(x, w, o2, bias=bias, aux=d, act=K_.EPI_GELU_D)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    pre = (x.float() @ w.float() + bias).requires_grad_(True)
    torch.nn.functional.gelu(pre, approximate="tanh").sum().backward()
    exact = pre.grad
    assert ((d.float() - exact).abs() <= 2 ** -8 * exact.abs() + 1e-3).all()
    dy = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
    wt = (0.2 * torch.randn(N, Kd, device=dev, generator=g)).to(torch.bfloat16)
    b1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K_.gemm(dy, wt, b1, tb=True, aux=d, act=K_.EPI_MUL_AUX)
    torch.cuda.synchronize()
    ref = (dy.float() @ wt.float().t()) * d.float()
    assert ((b1.float() - ref).abs() <= 2 ** -7 * ref.abs() + 1e-2).all()


@pytest.mark.parametrize("B,T,H", [(2, 1024, 12), (1, 2048, 16)])   # 124M (C3) / 420M (C5) head geometry
def test_attention_lm_geometry(dev, B, T, H):
    """The LM's causal flash attention at the benchmarked head counts (12 heads at T 1024, 16 at T 2048,
    Dh 64) against the fp32 reference, with bounds relative to the reference's own magnitude: the output
    to 1e-2 of max |O| (bf16 output rounding is 2^-9), dq | dk | dv to 1e-2 of max |grad| (bf16 P and dS
    operands); measured values printed (LMATTN)."""
    from plaincv_amd import kernels as K
    torch.manual_seed(1)
    Dh = 64
    D = H * Dh
    qkv = torch.randn(B * T, 3 * D, device=dev).to(torch.bfloat16)
    out = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev)
    K.attn_fwd(qkv, out, lse, B, T, H, Dh, True)
    qf = qkv.float().requires_grad_(True)
    ref = _attn_ref(qf, B, T, H, Dh, True, None, 0.0)
    fwd_rel = ((out.float() - ref).abs().max() / ref.abs().max()).item()
    do = torch.randn(B * T, D, device=dev).to(torch.bfloat16)
    ref.backward(do.float())
    dqkv = torch.zeros(B * T, 3 * D, device=dev, dtype=torch.bfloat16)
    delta = torch.empty(B * H * T, device=dev)
    K.attn_bwd(qkv, out, do, lse, delta, dqkv, B, T, H, Dh, True)
    g = qf.grad
    rel = [((dqkv.float()[:, k * D:(k + 1) * D] - g[:, k * D:(k + 1) * D]).abs().max() /
            g[:, k * D:(k + 1) * D].abs().max()).item() for k in range(3)]
    print(f"LMATTN B={B} T={T} H={H}: fwd rel {fwd_rel:.2e}  dq / dk / dv rel {rel[0]:.2e} {rel[1]:.2e} {rel[2]:.2e}")
    assert fwd_rel <= 1e-2, fwd_rel
    assert max(rel) <= 1e-2, rel


@pytest.mark.parametrize("M,N,Kd,T,Dh", [(16384, 2304, 768, 1024, 64), (16384, 3072, 1024, 2048, 64),
                                         (2048, 384, 256, 128, 32)])
def test_gemm_rope_fused_matches_two_launches(dev, M, N, Kd, T, Dh):
    """pcv_gemm_rope (RoPE in the 256-wide GEMM's epilogue; the last case takes the two-launch fallback)
    against gemm + rope: the rotation runs on the same bf16-rounded product, so the values agree."""
    from plaincv_amd import kernels as K
    from plaincv_amd.models.LM.transformer import precompute_freqs_cis
    torch.manual_seed(3)
    a = (torch.randn(M, Kd, device=dev) * 0.5).to(torch.bfloat16)
    b = (torch.randn(N, Kd, device=dev) * 0.05).to(torch.bfloat16)
    cos, sin = precompute_freqs_cis(Dh, T, 500000.0)
    cos, sin = cos.to(dev), sin.to(dev)
    rc = 2 * (N // 3)
    ref = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(a, b, ref, tb=True)
    K.rope(ref, T, Dh, cos, sin, ncols=rc)
    out = torch.empty_like(ref)
    K.gemm_rope(a, b, out, T, Dh, cos, sin, rc)
    torch.cuda.synchronize()
    diff = (out.float() - ref.float()).abs()
    print(f"GEMMROPE M={M} N={N}: max diff {diff.max().item():.3g}, differing {(diff > 0).float().mean().item():.2e}")
    assert (diff > 0).float().mean().item() < 1e-4 and diff.max().item() <= 2e-2 * ref.float().abs().max().item()
    assert torch.equal(out[:, rc:], ref[:, rc:])


@pytest.mark.parametrize("B,T,H,Dh,doc", [(2, 1024, 4, 64, False), (1, 300, 2, 64, False), (2, 512, 2, 64, True),
                                          (2, 257, 2, 32, False)])
def test_attn_bwd_rope_fused_matches_two_launches(dev, B, T, H, Dh, doc):
    """attn_bwd(..., rope=(cos, sin)) (inverse RoPE in the dq / dk stores) against attn_bwd + rope backward."""
    from plaincv_amd import kernels as K
    from plaincv_amd.models.LM.transformer import precompute_freqs_cis
    torch.manual_seed(5)
    D = H * Dh
    qkv = torch.randn(B * T, 3 * D, device=dev).to(torch.bfloat16)
    out = torch.empty(B * T, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev)
    dd = None
    if doc:
        starts = torch.tensor([0, 100, 333], dtype=torch.int32)
        pos = torch.arange(T)
        st = starts[(pos[:, None] >= starts[None, :]).sum(1) - 1]
        en = torch.cat([starts[1:], torch.tensor([T], dtype=torch.int32)])[(pos[:, None] >= starts[None, :]).sum(1) - 1]
        dd = (st.repeat(B, 1).to(torch.int32).contiguous().to(dev), en.repeat(B, 1).to(torch.int32).contiguous().to(dev))
    K.attn_fwd(qkv, out, lse, B, T, H, Dh, True, doc=dd)
    do = torch.randn(B * T, D, device=dev).to(torch.bfloat16)
    cos, sin = precompute_freqs_cis(Dh, T, 10000.0)
    cos, sin = cos.to(dev), sin.to(dev)
    delta = torch.empty(B * H * T, device=dev)
    ref = torch.zeros(B * T, 3 * D, device=dev, dtype=torch.bfloat16)
    K.attn_bwd(qkv, out, do, lse, delta, ref, B, T, H, Dh, True, doc=dd)
    K.rope(ref, T, Dh, cos, sin, backward=True, ncols=2 * D)
    got = torch.zeros_like(ref)
    K.attn_bwd(qkv, out, do, lse, delta, got, B, T, H, Dh, True, doc=dd, rope=(cos, sin))
    torch.cuda.synchronize()
    diff = (got.float() - ref.float()).abs()
    print(f"ATTNROPE B={B} T={T}: max diff {diff.max().item():.3g}, differing {(diff > 0).float().mean().item():.2e}")
    assert (diff > 0).float().mean().item() < 1e-4 and diff.max().item() <= 2e-2 * ref.float().abs().max().item()
    assert torch.equal(got[:, 2 * D:], ref[:, 2 * D:])


@pytest.mark.parametrize("R,F,Kd", [(16384, 2048, 768), (16384, 2730, 1024), (1000, 300, 128)])
def test_gemm_swiglu_bwd_fused_matches_two_launches(dev, R, F, Kd):
    """pcv_gemm_swiglu_bwd (the GLU VJP in the 256-wide GEMM's epilogue, dh never stored; the last case
    takes the two-launch fallback) against gemm into dh + swiglu_bwd, pad columns included."""
    from plaincv_amd import kernels as K
    torch.manual_seed(9)
    Fp = (F + 7) // 8 * 8
    dx = torch.randn(R, Kd, device=dev).to(torch.bfloat16)
    w2 = (torch.randn(F, Kd, device=dev) * 0.05).to(torch.bfloat16)
    gu = torch.randn(R, 2 * Fp, device=dev).to(torch.bfloat16)
    dh = torch.empty(R, Fp, device=dev, dtype=torch.bfloat16)[:, :F]
    ref = torch.full((R, 2 * Fp), 7.0, device=dev, dtype=torch.bfloat16)
    K.gemm(dx, w2, dh, tb=True)
    K.swiglu_bwd(dh, gu, ref, F=F)
    got = torch.full_like(ref, 7.0)
    K.gemm_swiglu_bwd(dx, w2, gu, got, torch.empty(R, Fp, device=dev, dtype=torch.bfloat16)[:, :F], F)
    torch.cuda.synchronize()
    diff = (got.float() - ref.float()).abs()
    print(f"GEMMSWIGLU R={R} F={F}: max diff {diff.max().item():.3g}, differing {(diff > 0).float().mean().item():.2e}")
    assert (diff > 0).float().mean().item() < 1e-4 and diff.max().item() <= 2e-2 * ref.float().abs().max().item()
    assert torch.equal(got[:, F:Fp], torch.zeros_like(got[:, F:Fp]))


@pytest.mark.parametrize("R,F,Kd", [(16384, 2048, 768), (16384, 2730, 1024)])
def test_gemm_swiglu_fwd_fused_matches_two_launches(dev, R, F, Kd):
    """pcv_gemm_swiglu_fwd (interleaved [gate | up] weight rows, GLU in the 256-wide GEMM's epilogue)
    against gemm on the plain layout + swiglu_fwd: gu and h, pad columns included."""
    from plaincv_amd import kernels as K
    torch.manual_seed(11)
    Fp = (F + 7) // 8 * 8
    y = torch.randn(R, Kd, device=dev).to(torch.bfloat16)
    wt = torch.zeros(2 * Fp, Kd, device=dev, dtype=torch.bfloat16)   # plain [gate | up] rows, pads 0
    wt[:F] = (torch.randn(F, Kd, device=dev) * 0.05).to(torch.bfloat16)
    wt[Fp:Fp + F] = (torch.randn(F, Kd, device=dev) * 0.05).to(torch.bfloat16)
    wi = torch.zeros(K.swiglu_interleaved_rows(F), Kd, device=dev, dtype=torch.bfloat16)
    for j in range(0, Fp, 128):
        n = min(128, Fp - j)
        wi[2 * j:2 * j + n] = wt[j:j + n]
        wi[2 * j + 128:2 * j + 128 + n] = wt[Fp + j:Fp + j + n]
    assert K.gemm_swiglu_fwd_ok(y, wi, F)
    gu_ref = torch.empty(R, 2 * Fp, device=dev, dtype=torch.bfloat16)
    h_ref = torch.full((R, Fp), 5.0, device=dev, dtype=torch.bfloat16)
    K.gemm(y, wt, gu_ref, tb=True)
    K.swiglu_fwd(gu_ref, h_ref, F=F)
    gu = torch.full_like(gu_ref, 5.0)
    h = torch.full_like(h_ref, 5.0)
    K.gemm_swiglu_fwd(y, wi, gu, h, F)
    torch.cuda.synchronize()
    for name, a, b in (("gu", gu, gu_ref), ("h", h, h_ref)):
        diff = (a.float() - b.float()).abs()
        print(f"GEMMSWIGLUFWD R={R} F={F} {name}: max diff {diff.max().item():.3g}, "
              f"differing {(diff > 0).float().mean().item():.2e}")
        assert (diff > 0).float().mean().item() < 1e-4 and diff.max().item() <= 2e-2 * b.float().abs().max().item()
    assert torch.equal(h[:, F:], torch.zeros_like(h[:, F:]))
