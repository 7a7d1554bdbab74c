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
