"""GEMM kernel vs a torch fp32 reference on bf16-rounded operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _padded(rows, cols, dev, g):
    """bf16 [rows, cols] view of a buffer whose leading dimension is padded to 8."""
    ld = (cols + 7) // 8 * 8
    return torch.randn(rows, ld, device=dev, generator=g).to(torch.bfloat16)[:, :cols]


def _ref(a, b, ta, tb):
    A = a.float().t() if ta else a.float()
    B = b.float().t() if tb else b.float()
    return A @ B


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (257, 200, 48), (1000, 384, 128), (64, 50257 % 1000, 130),
                                   (16448, 128, 256), (33, 2730, 1024), (512, 512, 4096)])
def test_gemm_layouts(dev, ta, tb, M, N, K):
    from plaincv_amd import kernels as k
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + K)
    a = _padded(*((K, M) if ta else (M, K)), dev, g)
    b = _padded(*((N, K) if tb else (K, N)), dev, g)
    out = torch.empty(M, N, device=dev, dtype=torch.float32)
    k.gemm(a, b, out, ta=ta, tb=tb)
    ref = _ref(a, b, ta, tb)
    err = (out - ref).abs().max().item()
    assert err <= 1e-3 * (K ** 0.5) * 4, err


def test_gemm_padded_ld_and_bf16_out(dev):
    from plaincv_amd import kernels as k
    M, N, K = 300, 2730, 768
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    wbuf = torch.randn(K, 2736, device=dev).to(torch.bfloat16)
    w = wbuf[:, :N]
    obuf = torch.zeros(M, 2736, device=dev, dtype=torch.bfloat16)
    out = obuf[:, :N]
    k.gemm(a, w, out)
    ref = a.float() @ w.float()
    assert torch.allclose(out.float(), ref, rtol=2e-2, atol=2e-1)
    assert obuf[:, N:].abs().max().item() == 0.0


def test_gemm_epilogues(dev):
    from plaincv_amd import kernels as k
    M, N, K = 513, 256, 128
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (0.1 * torch.randn(K, N, device=dev)).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.float32)
    k.gemm(a, w, out, bias=bias, aux=aux, act=k.EPI_GELU, res=res)
    h = a.float() @ w.float() + bias
    ref = torch.nn.functional.gelu(h, approximate="tanh") + res
    assert torch.allclose(aux.float(), h, rtol=1e-2, atol=1e-2)
    assert torch.allclose(out, ref, rtol=1e-3, atol=1e-3)
    # accumulate (beta=1) and split-K
    c = torch.randn(128, 384, device=dev)
    c0 = c.clone()
    x = torch.randn(16448, 128, device=dev).to(torch.bfloat16)
    dy = torch.randn(16448, 384, device=dev).to(torch.bfloat16)
    k.gemm(x, dy, c, ta=True, beta=1.0)
    ref = c0 + x.float().t() @ dy.float()
    assert torch.allclose(c, ref, rtol=1e-3, atol=5e-2), (c - ref).abs().max()


@pytest.mark.parametrize("M,N,K", [(768, 50257, 16384), (4100, 4100, 16384), (1024, 50280, 4096), (50257, 1000, 544),
                                   (50257, 768, 16384)])
def test_gemm_big_wgrad(dev, M, N, K):
    """Split-K / fp32-atomic weight-gradient form of the 256x256 kernel (C += alpha X^T dY, both operands
    K-major) through pcv_gemm_bf16's dispatch: ragged M/N (clamped DMA columns, masked atomics), padded
    row strides, K not a multiple of the split; compared with the 128x128 path (big kernel disabled)."""
    from plaincv_amd import hip
    from plaincv_amd import kernels as k
    lib = hip.load()
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + K)
    a = _padded(K, M, dev, g)
    b = _padded(K, N, dev, g)
    assert lib.pcv_gemm_big_wgrad_ok(M, N, K, hip.ptr(a), a.stride(0), hip.ptr(b), b.stride(0)) == 1
    c0 = torch.randn(M, N, device=dev, generator=g)
    outs = []
    for on in (1, 0):
        prev = lib.pcv_gemm_big_enable(on)
        try:
            c = c0.clone()
            k.gemm(a, b, c, ta=True, alpha=0.25, beta=1.0)
            torch.cuda.synchronize()
        finally:
            lib.pcv_gemm_big_enable(prev)
        outs.append(c)
    ref = c0 + 0.25 * (a.float().t() @ b.float())
    tol = 2e-5 * K + 1e-4 * ref.abs().max().item()   # fp32 accumulation-order differences only
    for out in outs:
        assert (out - ref).abs().max().item() <= tol
    assert (outs[0] - outs[1]).abs().max().item() <= tol


def test_gemm_batched(dev):
    from plaincv_amd import kernels as k
    B, M, N, K = 5, 128, 256, 256
    a = torch.randn(B, M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(B, N, K, device=dev).to(torch.bfloat16)
    out = torch.empty(B, M, N, device=dev)
    k.gemm(a, b, out, tb=True)
    ref = a.float() @ b.float().transpose(1, 2)
    assert torch.allclose(out, ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("M,N,K,res", [(16384, 50257, 768, False), (8192, 4096, 1000, True), (16384, 2304, 128, False),
                                       (6000, 5472, 2736, True), (4100, 8200, 200, False),
                                       (16384, 768, 2304, True), (16384, 768, 4100, False), (16384, 1024, 1024, True)])
def test_gemm_big_kernel(dev, M, N, K, res):
    """256x256 / 256x192 8-wave ping-pong kernel (gemm_big.hip) through pcv_gemm_bf16's dispatch (both operands
    K-contiguous, bf16 out, >= 512 tiles): ragged M/N (clamped DMA rows), ragged K (register tail),
    padded row strides, residual epilogue; and the same call with the big path disabled."""
    from plaincv_amd import hip
    from plaincv_amd import kernels as k
    lib = hip.load()
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    a = _padded(M, K, dev, g)
    b = _padded(N, K, dev, g)
    r = _padded(M, N, dev, g) if res else None
    assert lib.pcv_gemm_big_ok(M, N, K, hip.ptr(a), a.stride(0), hip.ptr(b), b.stride(0)) == 1
    outs = []
    prev_stream = lib.pcv_gemm_stream_enable(0)   # (pcv_gemm_bf16 prefers the persistent kernel)
    try:
        for on in (1, 0):
            prev = lib.pcv_gemm_big_enable(on)
            try:
                out = torch.empty(M, (N + 7) // 8 * 8, device=dev, dtype=torch.bfloat16)[:, :N]
                k.gemm(a, b, out, tb=True, alpha=0.5, res=r)
                torch.cuda.synchronize()
            finally:
                lib.pcv_gemm_big_enable(prev)
            outs.append(out.float())
    finally:
        lib.pcv_gemm_stream_enable(prev_stream)
    ref = 0.5 * (a.float() @ b.float().t())
    if res:
        ref = ref + r.float()
    tol = 1e-3 * (K ** 0.5) * 4 + 1e-2 * ref.abs().max().item()   # bf16 output rounding
    for out in outs:
        assert (out - ref).abs().max().item() <= tol
    assert (outs[0] - outs[1]).abs().max().item() <= tol


@pytest.mark.parametrize("M,N,K,res", [(16384, 50257, 768, False), (16384, 768, 50257, False), (8192, 4096, 1024, True),
                                       (16384, 2304, 192, False), (6000, 5472, 2736, True), (4100, 8200, 200, False),
                                       (16384, 768, 2304, True), (16384, 768, 4100, False), (16384, 1024, 1024, True),
                                       (16384, 2048, 768, False), (8000, 1000, 200, True), (16384, 5472, 1024, False),
                                       (16384, 50280, 1024, False), (20000, 30000, 256, True)])
def test_gemm_stream_kernel(dev, M, N, K, res):
    """Persistent continuous-ring kernel (gemm_stream.hip), called through its own entry point: many tiles
    per workgroup (the lm_head: 49-50 per CU, the shapes pcv_gemm_bf16 dispatches to it), one tile per
    workgroup (N = 768, 256 x 192), ragged M / N (masked tiles), ragged K (the masked last ring step: K % 32 =
    17, 8, 4, 16), the residual epilogue and padded row strides.  Against an fp32 product of the same bf16
    operands, against gemm_big and the 128x128 family on the same product, and bitwise run-to-run."""
    from plaincv_amd import hip
    from plaincv_amd import kernels as k
    lib = hip.load()
    g = torch.Generator(device=dev).manual_seed(M + 3 * N + K)
    a = _padded(M, K, dev, g)
    b = _padded(N, K, dev, g)
    r = _padded(M, N, dev, g) if res else None
    dispatched = lib.pcv_gemm_stream_ok(M, N, K, hip.ptr(a), a.stride(0), hip.ptr(b), b.stride(0)) == 1
    print(f"GEMMSTREAM M={M} N={N} K={K}: pcv_gemm_bf16 dispatches it: {dispatched}")

    def run(stream_on, big_on):
        ps, pb = lib.pcv_gemm_stream_enable(stream_on), lib.pcv_gemm_big_enable(big_on)
        try:
            out = torch.full((M, (N + 7) // 8 * 8), 7.0, device=dev, dtype=torch.bfloat16)
            if stream_on:   # the kernel itself, whatever pcv_gemm_bf16's dispatch rule picks
                hip.call("pcv_gemm_stream", hip.ptr(a), hip.ptr(b), hip.ptr(out), M, N, K, a.stride(0), b.stride(0),
                         out.stride(0), 0.5, hip.ptr(r), r.stride(0) if r is not None else 0, 1.0, hip.stream_ptr())
            else:
                k.gemm(a, b, out[:, :N], tb=True, alpha=0.5, res=r)
            torch.cuda.synchronize()
        finally:
            lib.pcv_gemm_stream_enable(ps)
            lib.pcv_gemm_big_enable(pb)
        return out

    o1, o2 = run(1, 1), run(1, 1)
    assert torch.equal(o1, o2), "persistent GEMM not run-to-run identical"
    assert bool((o1[:, N:] == 7.0).all()), "wrote into the row padding past N"
    ref = 0.5 * (a.float() @ b.float().t())
    if res:
        ref = ref + r.float()
    tol = 1e-3 * (K ** 0.5) * 4 + 1e-2 * ref.abs().max().item()   # bf16 output rounding
    err = (o1[:, :N].float() - ref).abs().max().item()
    print(f"GEMMSTREAM M={M} N={N} K={K} res={res} max|err| {err:.3g} tol {tol:.3g}")
    assert err <= tol
    del ref
    for other in ((0, 1), (0, 0)):   # pcv_gemm_bf16 with the stream path off: gemm_big, then the 128 x 128 family
        if other == (0, 1) and not lib.pcv_gemm_big_ok(M, N, K, hip.ptr(a), a.stride(0), hip.ptr(b), b.stride(0)):
            continue
        o = run(*other)
        assert (o[:, :N].float() - o1[:, :N].float()).abs().max().item() <= tol, other


@pytest.mark.parametrize("case", ["layer124", "layer420", "lm_head124", "ragged", "beta0"])
def test_gemm_wgrad_grouped(dev, case):
    """Grouped deterministic split-K weight gradients (gemm_wgrad.hip): C_j = beta C_j + alpha A_j^T B_j for
    the four matrices of an LM layer in one launch (124M / 420M widths at the bench's 16 384 token rows),
    the vocabulary-wide lm_head alone, ragged M / N (not multiples of 256), beta 0 and explicit splits.
    Against an fp32 product of the same bf16 operands, and bitwise run-to-run (the splits' partial slabs
    are summed in split order by whichever split finishes last)."""
    from plaincv_amd import kernels as k
    g = torch.Generator(device=dev).manual_seed(hash(case) % 1000)
    R = 16384
    shapes = {"layer124": [(2048, 768), (768, 4096), (768, 768), (768, 2304)],
              "layer420": [(2730, 1024), (1024, 5472), (1024, 1024), (1024, 3072)],
              "lm_head124": [(768, 50257)],
              "ragged": [(300, 1000), (777, 130)],
              "beta0": [(768, 2304)]}[case]
    Kr = 4096 if case == "ragged" else R
    jobs = []
    for M, N in shapes:
        a = _padded(Kr, M, dev, g)
        b = _padded(Kr, N, dev, g)
        b.mul_(0.1)   # (in place: keeps the padded row stride)
        c = torch.randn(M, N, device=dev, generator=g)
        jobs.append((a, b, c))
    beta = 0.0 if case == "beta0" else 1.0
    splits = {"ragged": 3, "beta0": 2}.get(case, 0)
    c0 = [c.clone() for _, _, c in jobs]
    grp = k.WGradGroup(jobs, dev, splits=splits)
    grp(alpha=0.5, beta=beta)
    torch.cuda.synchronize()
    first = [c.clone() for _, _, c in jobs]
    for (_, _, c), init in zip(jobs, c0):
        c.copy_(init)
    grp(alpha=0.5, beta=beta)
    torch.cuda.synchronize()
    for (a, b, c), init, f in zip(jobs, c0, first):
        assert torch.equal(c, f), "grouped weight gradient not run-to-run identical"
        ref = beta * init + 0.5 * (a.float().t() @ b.float())
        err = (c - ref).abs().max().item()
        tol = 2e-5 * (a.float().abs().t() @ b.float().abs()).max().item() + 1e-5
        print(f"WGRAD {case} M={a.shape[1]} N={b.shape[1]} K={a.shape[0]} splits={splits} max|err| {err:.3g} tol {tol:.3g}")
        assert err <= tol


def test_gemm_wgrad_groups_share_workspace(dev):
    """Groups of different tile counts built on ONE shared workspace (the LM builds the 4-matrix layer groups
    and the lm_head group on the device's workspace) and launched interleaved: each group's slabs must
    never overwrite another group's tile tickets (a per-group ticket region sized by its own tile count
    did, and the lm_head weight gradient came out 0.6 off)."""
    from plaincv_amd import kernels as k
    g = torch.Generator(device=dev).manual_seed(5)
    Kr = 2048
    big = [(_padded(Kr, 768, dev, g), _padded(Kr, 20000, dev, g), torch.zeros(768, 20000, device=dev))]
    small = [(_padded(Kr, 512, dev, g), _padded(Kr, 512, dev, g), torch.zeros(512, 512, device=dev)),
             (_padded(Kr, 256, dev, g), _padded(Kr, 768, dev, g), torch.zeros(256, 768, device=dev))]
    gb = k.WGradGroup(big, dev, splits=2)
    gs = k.WGradGroup(small, dev, splits=4)
    assert gb.ws.data_ptr() == gs.ws.data_ptr() and gb.ws_bytes > 0 and gs.ws_bytes > 0
    for _ in range(3):
        gs(beta=1.0)
        gb(beta=1.0)
    torch.cuda.synchronize()
    for a, b, c in big + small:
        ref = 3.0 * (a.float().t() @ b.float())
        err = (c - ref).abs().max().item()
        assert err <= 1e-4 * ref.abs().max().item(), err
