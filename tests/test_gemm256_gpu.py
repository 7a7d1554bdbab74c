"""256x256 bf16 LDS-DMA GEMM (csrc/kernels/gemm_bf16_256.hip): K-contiguous and row-contiguous
(transposed-read) operands, batched, split-K, ragged M/N edges, against an fp32 PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def C():
    import ringdp

    c = ringdp._C
    c.set_bf16_tile_mode(256)
    yield c
    c.set_bf16_tile_mode(0)
    c.set_gemm256_phased(1)


def _operand(rows, K, row, batch, g):
    """logical [batch][rows][K]; storage K-contiguous ([rows][K]) or row-contiguous ([K][rows])."""
    x = (torch.randn(batch, rows, K, generator=g) * 0.5).bfloat16()
    store = x.transpose(1, 2).contiguous() if row else x.contiguous()
    return x.float(), store.cuda()


@pytest.mark.parametrize("phased", [1, 0])
@pytest.mark.parametrize("a_row,b_row", [(False, False), (True, True), (True, False), (False, True)])
@pytest.mark.parametrize("M,N,K,batch", [(520, 264, 640, 2), (256, 512, 128, 1), (8, 8, 64, 3), (304, 696, 64, 1)])
def test_gemm256_layouts(C, a_row, b_row, M, N, K, batch, phased):
    C.set_gemm256_phased(phased)  # K-contiguous operands: the phased pipeline or the older kernel
    g = torch.Generator().manual_seed(M + N + K)
    a, ad = _operand(M, K, a_row, batch, g)
    b, bd = _operand(N, K, b_row, batch, g)
    lda = M if a_row else K
    ldb = N if b_row else K
    bias = torch.randn(N, generator=g).cuda()
    out = C.gemm(ad, bd, M, N, K, lda, ldb, a_row, b_row, batch, M * K, N * K, False, bias)
    ref = torch.bmm(a, b.transpose(1, 2)) + bias.cpu()
    err = (out.cpu().view(batch, M, N) - ref).abs().max() / ref.abs().max()
    assert err < 2e-3, float(err)


@pytest.mark.parametrize("M,N", [(768, 768), (2304, 768), (776, 3072)])
def test_gemm256_wgrad_splitk(C, M, N):
    """dW = dz^T x over 4096 token rows, both operands row-contiguous (the ViT weight gradient)."""
    T = 4096
    g = torch.Generator().manual_seed(M * 7 + N)
    dz = (torch.randn(T, M, generator=g) * 0.5).bfloat16()
    x = (torch.randn(T, N, generator=g) * 0.5).bfloat16()
    out = torch.empty(M, N, device="cuda")
    C.gemm_splitk_f32(dz.cuda(), x.cuda(), M, N, T, M, N, True, True, 8, out)
    ref = dz.float().t() @ x.float()
    err = (out.cpu() - ref).abs().max() / ref.abs().max()
    assert err < 1e-4, float(err)


def _gelu_grad(x):
    return 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * 0.3989422804014327 * torch.exp(-0.5 * x * x)


def _select(C, kern):
    C.set_gemm256_persist(1 if kern == "persist" else 0)
    C.set_gemm_two_wg(1 if kern == "2wg" else 0)


@pytest.mark.parametrize("kern", ["persist", "1wg", "2wg"])
@pytest.mark.parametrize("epi", ["bf16_bias", "gelu_preact", "residual", "gelu_bwd", "f32_plain"])
@pytest.mark.parametrize("M,N,K,batch", [(4200, 4104, 128, 1), (1000, 776, 192, 3), (264, 256, 64, 1)])
def test_gemm256_persistent_epilogues(C, kern, epi, M, N, K, batch):
    """The persistent phased kernel (several tiles per workgroup once tiles > CUs, next tile's first k-tile
    landing during the epilogue, exact-count edge stores into a sink) against fp32 references, for every
    epilogue kind it serves; 1wg is the one-workgroup-per-tile kernel on the same inputs, 2wg the
    two-workgroups-per-CU 256x128 kernel (gemm_bf16_256n: 3-stage DMA ring, register double-buffered
    fragments; K = 64 and 192 give it 2 and 6 stages)."""
    _select(C, kern)
    try:
        g = torch.Generator().manual_seed(M * 3 + N + K + batch)
        a, ad = _operand(M, K, False, batch, g)
        b, bd = _operand(N, K, False, batch, g)
        ref = torch.bmm(a, b.transpose(1, 2))
        bias = torch.randn(N, generator=g)
        side = (torch.randn(batch, M, N, generator=g)).bfloat16()
        if epi == "f32_plain":
            out = C.gemm(ad, bd, M, N, K, K, K, False, False, batch, M * K, N * K, False)
            want = ref
        elif epi == "bf16_bias":
            out = C.gemm(ad, bd, M, N, K, K, K, False, False, batch, M * K, N * K, True, bias.cuda())
            want = ref + bias
        elif epi == "gelu_preact":
            pre = torch.empty(batch * M * N, device="cuda", dtype=torch.bfloat16)
            out = C.gemm(ad, bd, M, N, K, K, K, False, False, batch, M * K, N * K, True, bias.cuda(), 2, None, pre)
            z = ref + bias
            want = torch.nn.functional.gelu(z)
            perr = (pre.cpu().float().view(batch, M, N) - z).abs().max() / z.abs().max()
            assert perr < 8e-3, float(perr)
        elif epi == "residual":
            out = C.gemm(ad, bd, M, N, K, K, K, False, False, batch, M * K, N * K, True, bias.cuda(), 0, side.cuda())
            want = ref + bias + side.float()
        else:  # GELU backward: C = (A B^T) * GELU'(preact)
            out = C.gemm(ad, bd, M, N, K, K, K, False, False, batch, M * K, N * K, True, None, 3, None, side.cuda())
            want = ref * _gelu_grad(side.float())
        got = out.cpu().float().view(batch, M, N)
        err = (got - want).abs().max() / want.abs().max()
        assert err < (2e-3 if epi == "f32_plain" else 8e-3), float(err)
    finally:
        _select(C, "1wg")


@pytest.mark.parametrize("kern", ["persist", "1wg", "2wg"])
def test_gemm256_persistent_splitk(C, kern):
    """K-contiguous split-K through the persistent kernel (work items = tiles x splits) and the 2-WG kernel."""
    _select(C, kern)
    try:
        M, N, K = 1032, 1288, 4096
        g = torch.Generator().manual_seed(11)
        a = (torch.randn(M, K, generator=g) * 0.5).bfloat16()
        b = (torch.randn(N, K, generator=g) * 0.5).bfloat16()
        out = torch.empty(M, N, device="cuda")
        C.gemm_splitk_f32(a.cuda(), b.cuda(), M, N, K, K, K, False, False, 8, out)
        ref = a.float() @ b.float().t()
        err = (out.cpu() - ref).abs().max() / ref.abs().max()
        assert err < 1e-4, float(err)
    finally:
        _select(C, "1wg")


@pytest.mark.parametrize("M,N,K", [(520, 264, 640), (304, 696, 64), (8, 8, 64), (256, 128, 96 * 2)])
def test_gemm256_two_wg_shapes(C, M, N, K):
    """2-WG kernel on ragged edges (M, N not multiples of 256 / 128) and stage counts 1, 2, 6, 10, 20."""
    _select(C, "2wg")
    try:
        g = torch.Generator().manual_seed(M + 3 * N + K)
        a, ad = _operand(M, K, False, 1, g)
        b, bd = _operand(N, K, False, 1, g)
        out = C.gemm(ad, bd, M, N, K, K, K, False, False, 1, M * K, N * K, False)
        ref = a[0] @ b[0].t()
        err = (out.cpu().view(M, N) - ref).abs().max() / ref.abs().max()
        assert err < 2e-3, float(err)
    finally:
        _select(C, "1wg")
