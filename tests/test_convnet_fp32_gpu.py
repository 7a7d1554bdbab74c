"""The ConvNet at the reference's fp32 precision (VERDICT r1 missing #3; ref/launch_dist.py:50-59).

* every fp32 kernel (conv fwd / dgrad / wgrad+bias, fused ReLU+max-pool fwd/bwd) against the ATen
  fp32 oracle at the ConvNet's shapes;
* the whole model, forward + backward, against the ATen fp32 model;
* convergence: 200 SGD steps on fixed synthetic batches; the fp32 loss trajectory must stay within
  1e-3 of the ATen fp32 model's at every step, the bf16 fast path within a stated band.
"""
import pytest
import torch
import torch.nn.functional as F

from ringdp._native import C

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(a, b, rtol=1e-5, atol=1e-5):
    err = float((a - b).abs().max())
    assert err <= atol + rtol * float(b.abs().max()), err


@pytest.mark.parametrize("B,Cin,H,K,R,pad", [(3, 1, 28, 32, 5, 1), (5, 32, 13, 64, 3, 0), (4, 64, 10, 128, 3, 0),
                                             (7, 2048, 1, 10, 1, 0), (2, 3, 9, 5, 3, 1)])
def test_conv_f32_kernels(B, Cin, H, K, R, pad):
    g = torch.Generator(device=DEV).manual_seed(B * 100 + K)
    x = torch.randn(B, Cin, H, H, device=DEV, generator=g)
    w = torch.randn(K, Cin, R, R, device=DEV, generator=g) * 0.1
    b = torch.randn(K, device=DEV, generator=g)
    z = C.f32_conv_fwd(x, w, b, pad)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=pad).float()
    _close(z, ref)
    dz = torch.randn_like(z)
    dx = C.f32_conv_dgrad(dz, w, H, H, pad)
    xr = x.double().requires_grad_()
    wr = w.double().requires_grad_()
    br = b.double().requires_grad_()
    F.conv2d(xr, wr, br, padding=pad).backward(dz.double())
    _close(dx, xr.grad.float())
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    C.f32_conv_wgrad(dz, x, pad, 0.0, 1.0, dw, db)
    _close(dw, wr.grad.float(), rtol=2e-5)
    _close(db, br.grad.float(), rtol=2e-5)


def _conv_roundtrip(B, Cin, H, K, R, pad, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(B, Cin, H, H, device=DEV, generator=g)
    w = torch.randn(K, Cin, R, R, device=DEV, generator=g) * 0.1
    b = torch.randn(K, device=DEV, generator=g)
    z = C.f32_conv_fwd(x, w, b, pad)
    dz = torch.randn_like(z)
    dx = C.f32_conv_dgrad(dz, w, H, H, pad)
    dw, db = torch.empty_like(w), torch.empty_like(b)
    C.f32_conv_wgrad(dz, x, pad, 0.0, 1.0, dw, db)
    xr, wr, br = (t.double().requires_grad_() for t in (x, w, b))
    ref = F.conv2d(xr, wr, br, padding=pad)
    ref.backward(dz.double())
    return (z, dx, dw, db), (ref.detach().float(), xr.grad.float(), wr.grad.float(), br.grad.float())


@pytest.mark.parametrize("B,Cin,H,K,R,pad", [(40, 32, 13, 64, 3, 0), (33, 64, 10, 128, 3, 0), (70, 1, 28, 32, 5, 1),
                                             (300, 2048, 1, 10, 1, 0)])
def test_conv_f32_many_tiles_and_slices(B, Cin, H, K, R, pad):
    """Batches that give ragged m tiles, several split-K weight-gradient slices and the 128x32 / 32x128
    tile layouts."""
    got, ref = _conv_roundtrip(B, Cin, H, K, R, pad, B + K)
    for a, r, tol in zip(got, ref, (1e-5, 1e-5, 3e-5, 3e-5)):
        _close(a, r, rtol=tol)


@pytest.mark.parametrize("slices", ["1", "3", "8", ""])
@pytest.mark.parametrize("B,Cin,H,K,R,pad", [(100, 64, 10, 128, 3, 0), (100, 32, 13, 64, 3, 0), (6, 3, 9, 5, 3, 1),
                                             (700, 64, 10, 128, 3, 0)])
def test_conv_f32_dgrad_split_k(monkeypatch, slices, B, Cin, H, K, R, pad):
    """Small-batch data gradients split K into slices whose partial dx planes are summed in order
    (conv_f32_dgrad_slices: the reference's B=100 conv3 / conv2 shapes take 8 / 5); forced counts, the
    unsplit path (1) and the automatic choice ("": B=700 conv3 has enough tiles to stay unsplit)."""
    if slices:
        monkeypatch.setenv("RINGDP_F32_DGRAD_SLICES", slices)
    else:
        monkeypatch.delenv("RINGDP_F32_DGRAD_SLICES", raising=False)
    g = torch.Generator(device=DEV).manual_seed(B + Cin)
    w = torch.randn(K, Cin, R, R, device=DEV, generator=g) * 0.1
    OH = H + 2 * pad - R + 1
    dz = torch.randn(B, K, OH, OH, device=DEV, generator=g)
    dx = C.f32_conv_dgrad(dz, w, H, H, pad)
    ref = torch.nn.grad.conv2d_input((B, Cin, H, H), w.double(), dz.double(), padding=pad).float()
    _close(dx, ref)


@pytest.mark.parametrize("slices", ["1", "2", "5", ""])
@pytest.mark.parametrize("B,Cin,H,K,st", [(100, 64, 10, 128, 2), (100, 32, 13, 64, 1), (3, 16, 6, 24, 2), (900, 64, 10, 128, 2)])
def test_conv_f32_pool_split_k(monkeypatch, slices, B, Cin, H, K, st):
    """Small-batch valid conv + ReLU + 2x2 pool by split K (conv_f32_fwd_slices: B=100 conv3 / conv2 take 5 / 3
    slices; B=900 conv3 stays one fused launch) against fp64, and against conv-then-pool."""
    if slices:
        monkeypatch.setenv("RINGDP_F32_FWD_SLICES", slices)
    else:
        monkeypatch.delenv("RINGDP_F32_FWD_SLICES", raising=False)
    g = torch.Generator(device=DEV).manual_seed(B + K + st)
    x = torch.randn(B, Cin, H, H, device=DEV, generator=g)
    w = torch.randn(K, Cin, 3, 3, device=DEV, generator=g) * 0.2
    b = torch.randn(K, device=DEV, generator=g) * 0.1
    a, code = C.f32_conv_pool_fwd(x, w, b, 0, 0.0, 1.0, st)
    ref = F.max_pool2d(F.relu(F.conv2d(x.double(), w.double(), b.double())), 2, st).float()
    _close(a, ref, rtol=1e-5, atol=1e-5)
    a2, code2 = C.f32_pool_relu_fwd(C.f32_conv_fwd(x, w, b, 0, 0.0, 1.0), 2, st)
    # another fp32 summation order than the unsplit conv (K = 576 products of magnitude ~5): a few ulp
    torch.testing.assert_close(a, a2, rtol=1e-5, atol=1e-5)
    assert float((code == code2).float().mean()) > 0.995
    assert bool(((code == 255) == (a == 0)).all())


def test_conv_f32_batch_chunks(monkeypatch):
    """The host launchers split the batch so every index stays 32-bit; a lowered limit runs that path
    (conv2 shape: 7744 output elements per image, limit 3 images -> chunks of 3, 3, 2)."""
    monkeypatch.setenv("RINGDP_F32_CHUNK_LIMIT", str(3 * 7744))
    got, ref = _conv_roundtrip(8, 32, 13, 64, 3, 0, 5)
    for a, r in zip(got, ref):
        _close(a, r, rtol=3e-5)
    z = torch.randn(8, 64, 11, 11, device=DEV)
    a, code = C.f32_pool_relu_fwd(z, 2, 1)
    assert torch.equal(a, F.max_pool2d(F.relu(z), 2, 1))


@pytest.mark.parametrize("B,Cin,H,K,R,pad,u8,st", [(5, 1, 28, 32, 5, 1, True, 2), (9, 64, 10, 128, 3, 0, False, 2),
                                                   (3, 3, 8, 8, 3, 1, False, 2), (7, 32, 13, 64, 3, 0, False, 1),
                                                   (4, 5, 9, 80, 3, 1, False, 1)])
def test_conv_f32_pool_fused(B, Cin, H, K, R, pad, u8, st):
    """conv + bias + ReLU + 2x2/s2 max-pool in one launch == conv kernel then the pool kernel, and == ATen.
    Bit-exact where both launches use the same tile layout; at small batches the plain conv may take the
    32x32 tiles with the k-range split over 4 waves (another fp32 summation order): then equal to a few
    ulp, and the argmax codes equal except at near-ties."""
    g = torch.Generator(device=DEV).manual_seed(B * 7 + K)
    if u8:
        x = torch.randint(0, 256, (B, Cin, H, H), dtype=torch.uint8, device=DEV, generator=g)
        mean, std = 0.1307, 0.3081
        xf = (x.float() / 255.0 - mean) / std
    else:
        x = torch.randn(B, Cin, H, H, device=DEV, generator=g)
        mean, std = 0.0, 1.0
        xf = x
    w = torch.randn(K, Cin, R, R, device=DEV, generator=g) * 0.2
    b = torch.randn(K, device=DEV, generator=g) * 0.1
    a, code = C.f32_conv_pool_fwd(x, w, b, pad, mean, std, st)
    z = C.f32_conv_fwd(x, w, b, pad, mean, std)
    a2, code2 = C.f32_pool_relu_fwd(z, 2, st)
    if not torch.equal(a, a2):
        torch.testing.assert_close(a, a2, rtol=4e-6, atol=4e-6)
        assert float((code == code2).float().mean()) > 0.995
    else:
        assert torch.equal(code, code2)
    ref = F.max_pool2d(F.relu(F.conv2d(xf.double(), w.double(), b.double(), padding=pad)), 2, st).float()
    _close(a, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("u8", [True, False])
@pytest.mark.parametrize("B", [1, 7, 37])
def test_conv1_f32_dedicated(B, u8):
    """conv1 + ReLU + pool1 (one wave per image) == the generic conv+pool kernels bit-exactly, and its
    weight/bias gradient from the pooled gradient == pool backward + generic wgrad (fp32 rounding)."""
    g = torch.Generator(device=DEV).manual_seed(B + 11 * u8)
    if u8:
        x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=DEV, generator=g)
        mean, std = 0.1307, 0.3081
    else:
        x = torch.randn(B, 1, 28, 28, device=DEV, generator=g)
        mean, std = 0.0, 1.0
    w = torch.randn(32, 1, 5, 5, device=DEV, generator=g) * 0.2
    b = torch.randn(32, device=DEV, generator=g) * 0.1
    a, code = C.f32_conv1_pool_fwd(x, w, b, mean, std)
    a_ref, code_ref = C.f32_conv_pool_fwd(x, w, b, 1, mean, std)
    _close(a, a_ref, rtol=1e-6, atol=1e-6)
    assert float((code != code_ref).float().mean()) < 1e-3  # ties only
    da = torch.randn(B, 32, 13, 13, device=DEV, generator=g)
    dw, db = torch.empty_like(w), torch.empty_like(b)
    C.f32_conv1_wgrad(x, da, code, mean, std, dw, db)
    dz = C.f32_pool_relu_bwd(da, code, 26, 26, 2, 2)
    dw_ref, db_ref = torch.empty_like(w), torch.empty_like(b)
    C.f32_conv_wgrad(dz, x, 1, mean, std, dw_ref, db_ref)
    _close(dw, dw_ref, rtol=2e-5, atol=1e-5)
    _close(db, db_ref, rtol=2e-5, atol=1e-5)


def test_conv_f32_uint8_input_fuses_normalize():
    g = torch.Generator(device=DEV).manual_seed(3)
    xu8 = torch.randint(0, 256, (6, 1, 28, 28), dtype=torch.uint8, device=DEV, generator=g)
    w = torch.randn(32, 1, 5, 5, device=DEV, generator=g) * 0.2
    b = torch.randn(32, device=DEV, generator=g)
    xn = (xu8.float() / 255.0 - 0.1307) / 0.3081
    _close(C.f32_conv_fwd(xu8, w, b, 1, 0.1307, 0.3081), F.conv2d(xn, w, b, padding=1), rtol=1e-5, atol=1e-4)
    dz = torch.randn(6, 32, 26, 26, device=DEV, generator=g)
    dw, db = torch.empty_like(w), torch.empty_like(b)
    C.f32_conv_wgrad(dz, xu8, 1, 0.1307, 0.3081, dw, db)
    wr = w.double().requires_grad_()
    F.conv2d(xn.double(), wr, b.double(), padding=1).backward(dz.double())
    _close(dw, wr.grad.float(), rtol=2e-5, atol=1e-3)


@pytest.mark.parametrize("H,k,st", [(26, 2, 2), (11, 2, 1), (8, 2, 2), (9, 2, 2), (10, 3, 2)])
def test_pool_relu_f32(H, k, st):
    g = torch.Generator(device=DEV).manual_seed(H)
    z = torch.randn(4, 16, H, H, device=DEV, generator=g)
    z[0, 0, :2, :2] = 0.5  # ties: the first maximum wins, as in max_pool2d
    a, code = C.f32_pool_relu_fwd(z, k, st)
    zr = z.clone().requires_grad_()
    ref = F.max_pool2d(F.relu(zr), k, st)
    assert torch.equal(a, ref)
    da = torch.randn_like(a)
    ref.backward(da)
    dz = C.f32_pool_relu_bwd(da, code, H, H, k, st)
    _close(dz, zr.grad, rtol=0, atol=1e-6)


def _models(seed=0):
    from ringdp.models import ConvNet

    torch.manual_seed(seed)
    m32 = ConvNet(precision="fp32").to(DEV)
    ref = ConvNet().to(DEV)
    ref.load_state_dict(m32.state_dict())
    return m32, ref


@pytest.mark.parametrize("B", [64, 2048])
def test_fp32_convnet_matches_aten(B):
    """Forward + gradients of the fp32 model against ATen fp32.  B=2048 runs the large-batch kernels of
    csrc/kernels/conv_f32.hip in the model (scatter data gradients, dedicated weight gradients, the conv2 / conv3
    + pool forwards, the tiled pool2 backward); B=64 the small-batch split-K path."""
    m32, ref = _models()
    x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=DEV)
    y = torch.randint(0, 10, (B,), device=DEV)
    out = m32(x)
    rout = ref.reference_forward(x)
    _close(out.detach(), rout.detach(), rtol=1e-4, atol=1e-5)
    F.cross_entropy(out, y).backward()
    F.cross_entropy(rout, y).backward()
    for (n, p), q in zip(m32.named_parameters(), ref.parameters()):
        if B <= 64:
            _close(p.grad, q.grad, rtol=1e-4, atol=1e-6)
        else:
            # tens of millions of pooling windows: a few near-ties (top-2 gap below the ~1e-7 summation-order
            # difference) pick the other argmax than ATen and route one element's gradient elsewhere, so the
            # per-element bound does not hold; the relative L2 error stays ~1e-3 or below (measured: conv1.weight
            # 1.6e-3, the rest <= 5e-4, conv3.bias / fc1 ~2e-7 - the same with every large-batch kernel switched
            # off, i.e. the generic implicit GEMMs: tools/scratch/fp32_diag.py)
            rel = float((p.grad - q.grad).norm() / q.grad.norm())
            assert rel < 5e-3, (n, rel)


@pytest.mark.parametrize("B", [100, 700])
def test_fp32_net_node_matches_per_layer_backward(B):
    """ringdp's cross entropy on the fp32 model at a small batch is ONE node over the whole network (one
    weight-gradient reduction launch; cross entropy + fc1 data gradient + pool3 backward fused).  The loss and fc1's
    gradients (same logits gradient, same GEMM, same fixed-order reduction) equal the per-layer backward's bit for
    bit; the conv layers' to fp32 rounding (fc1's data gradient is an fmaf chain instead of the GEMM's MFMAs)."""
    from ringdp.ops.loss import _CrossEntropy, cross_entropy

    m_a, _ = _models(3)
    m_b, _ = _models(3)
    x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=DEV)
    y = torch.randint(0, 10, (B,), device=DEV)
    y[1] = -100
    la = cross_entropy(m_a(x), y, label_smoothing=0.05)
    assert type(la.grad_fn).__name__ == "_NetCEF32Backward", la.grad_fn
    # the same cross-entropy kernels without the fusion hook: the per-layer nodes
    lb = _CrossEntropy.apply(m_b(x), y, -100, 0.05, "mean")
    la.backward()
    lb.backward()
    assert torch.equal(la.detach(), lb.detach())
    for (n, p), q in zip(m_a.named_parameters(), m_b.parameters()):
        if n.startswith("fc1"):
            assert torch.equal(p.grad, q.grad), n
        else:
            rel = float((p.grad - q.grad).norm() / q.grad.norm())
            assert rel < 1e-5, (n, rel)
    # another use of the logits keeps the per-layer path (gradients through both are summed by autograd)
    m_c, _ = _models(3)
    out = m_c(x)
    (cross_entropy(out, y) + out.square().mean()).backward()
    assert all(p.grad is not None for p in m_c.parameters())


@pytest.mark.parametrize("B", [100, 64, 37])
def test_conv_dgrad_pool2s1_fused_matches_two_ops(B):
    """conv3's data gradient with pool2's 2x2/s1 backward summing the split-K planes as it stages them == the
    data gradient (planes summed by slab_sum) followed by the pool backward, bit for bit (B=37: B*C not a multiple
    of the pool tile -> the two-op fallback)."""
    g = torch.Generator(device=DEV).manual_seed(B)
    w = torch.randn(128, 64, 3, 3, device=DEV, generator=g) * 0.1
    dz = torch.randn(B, 128, 8, 8, device=DEV, generator=g)
    code = torch.randint(0, 4, (B, 64, 10, 10), dtype=torch.uint8, device=DEV, generator=g)
    code[torch.rand(code.shape, device=DEV, generator=g) < 0.3] = 255
    fused = C.f32_conv_dgrad_pool2s1_bwd(dz, w, code)
    ref = C.f32_pool_relu_bwd(C.f32_conv_dgrad(dz, w, 10, 10, 0), code, 11, 11, 2, 1)
    assert torch.equal(fused, ref)


def _trajectory(model, forward, steps, xs, ys, lr):
    from ringdp.optim import SGD

    opt = SGD(model.parameters(), lr=lr)
    out = []
    for i in range(steps):
        loss = F.cross_entropy(forward(xs[i % len(xs)]), ys[i % len(ys)])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        out.append(float(loss))
    return torch.tensor(out)


@pytest.mark.parametrize("B", [128, 2048])
def test_convergence_200_steps_fp32_and_bf16(B):
    """200 SGD steps of the fp32 and bf16 models against ATen fp32; B=2048 takes the large-batch fp32 kernels."""
    from ringdp.models import ConvNet

    g = torch.Generator(device=DEV).manual_seed(7)
    xs = [torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=DEV, generator=g) for _ in range(8)]
    # learnable labels: a fixed random linear map of the pixels, so the loss really falls
    proj = torch.randn(784, 10, device=DEV, generator=g)
    ys = [(x.float().view(B, -1) @ proj).argmax(1) for x in xs]
    lr, steps = 0.01, 200
    m32, ref = _models(1)
    l_ref = _trajectory(ref, ref.reference_forward, steps, xs, ys, lr)
    l_32 = _trajectory(m32, m32, steps, xs, ys, lr)
    torch.manual_seed(1)
    m16 = ConvNet().to(DEV)
    l_16 = _trajectory(m16, m16, steps, xs, ys, lr)
    assert l_ref[-20:].mean() < l_ref[:8].mean() - 0.3, l_ref  # it actually trains
    d32 = float((l_32 - l_ref).abs().max())
    d16 = float((l_16 - l_ref).abs().max())
    print(f"max |loss - aten fp32| over {steps} steps: fp32 {d32:.2e}, bf16 {d16:.2e}")
    assert d32 < 1e-3, d32  # measured 1.9e-4
    assert d16 < 5e-3, d16  # bf16 activations/weights, fp32 accumulation and masters (measured 3.7e-4)


@pytest.mark.parametrize("B", [600, 1024])
@pytest.mark.parametrize("Cin,H,K", [(64, 10, 128), (32, 13, 64)])
def test_conv_dgrad_f32_scatter(B, Cin, H, K):
    """conv3's and conv2's data gradients over the live taps only (scatter form, csrc/kernels/conv_f32.hip
    conv3_dgrad_f32_kernel / conv2_dgrad_f32_kernel: batches of at least 2 images per CU) against fp64,
    against the implicit-GEMM path that 100-image batches take (same values up to summation order), and
    bit-identical across runs."""
    g = torch.Generator(device=DEV).manual_seed(B + K)
    w = torch.randn(K, Cin, 3, 3, device=DEV, generator=g) * 0.1
    dz = torch.randn(B, K, H - 2, H - 2, device=DEV, generator=g)
    dx = C.f32_conv_dgrad(dz, w, H, H, 0)
    ref = torch.nn.grad.conv2d_input((B, Cin, H, H), w.double(), dz.double()).float()
    _close(dx, ref)
    assert torch.equal(dx, C.f32_conv_dgrad(dz, w, H, H, 0))
    small = C.f32_conv_dgrad(dz[:100].contiguous(), w, H, H, 0)  # the split-K implicit GEMM
    _close(small, dx[:100], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B", [1024, 1500])
@pytest.mark.parametrize("Cin,H,K", [(64, 10, 128), (32, 13, 64)])
def test_conv_wgrad_f32_dedicated(B, Cin, H, K):
    """conv3's and conv2's weight + bias gradients on the dedicated kernels (csrc/kernels/conv_f32.hip
    conv3_wgrad_f32_kernel / conv2_wgrad_f32_kernel: 128 image slices x the 16-channel tiles, slab + fixed-order
    reduction) against fp64 and bit-identical across runs."""
    g = torch.Generator(device=DEV).manual_seed(B + K)
    x = torch.randn(B, Cin, H, H, device=DEV, generator=g)
    w = torch.randn(K, Cin, 3, 3, device=DEV, generator=g) * 0.1
    dz = torch.randn(B, K, H - 2, H - 2, device=DEV, generator=g)
    dw, db = torch.empty_like(w), torch.empty(K, device=DEV)
    C.f32_conv_wgrad(dz, x, 0, 0.0, 1.0, dw, db)
    xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
    br = torch.zeros(K, device=DEV, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wr, br).backward(dz.double())
    _close(dw, wr.grad.float(), rtol=2e-5)
    _close(db, br.grad.float(), rtol=2e-5)
    dw2, db2 = torch.empty_like(w), torch.empty(K, device=DEV)
    C.f32_conv_wgrad(dz, x, 0, 0.0, 1.0, dw2, db2)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("B", [1024, 1100])
def test_conv2_pool_f32_dedicated(B):
    """conv2 + bias + ReLU + overlapping 2x2/s1 max-pool on the dedicated forward kernel
    (csrc/kernels/conv_f32.hip conv2_pool_f32_kernel: batches of >= 4 images per CU) against fp64: pooled
    values, and the argmax codes wherever the window's maximum is not a near-tie."""
    g = torch.Generator(device=DEV).manual_seed(B + 5)
    x = torch.randn(B, 32, 13, 13, device=DEV, generator=g)
    w = torch.randn(64, 32, 3, 3, device=DEV, generator=g) * 0.1
    b = torch.randn(64, device=DEV, generator=g) * 0.1
    a, code = C.f32_conv_pool_fwd(x, w, b, 0, 0.0, 1.0, 1)
    z = F.conv2d(x.double(), w.double(), b.double())  # [B, 64, 11, 11]
    win = torch.stack([z[..., :-1, :-1], z[..., :-1, 1:], z[..., 1:, :-1], z[..., 1:, 1:]], -1)
    best, arg = win.max(-1)
    ref = best.clamp_min(0).float()
    _close(a, ref, rtol=1e-5, atol=1e-5)
    top2 = win.topk(2, -1).values
    clear = ((top2[..., 0] - top2[..., 1]) > 1e-4 * (1 + top2[..., 0].abs())) & (best > 1e-4)
    want = torch.where(best > 0, arg, torch.full_like(arg, 255)).to(torch.uint8)
    assert torch.equal(code[clear], want[clear])
    assert torch.equal(code[best < -1e-4], want[best < -1e-4])  # dead windows: 255
    a2, code2 = C.f32_conv_pool_fwd(x, w, b, 0, 0.0, 1.0, 1)
    assert torch.equal(a, a2) and torch.equal(code, code2)


@pytest.mark.parametrize("B", [1024, 1100])
def test_conv3_pool_f32_dedicated(B):
    """conv3 + bias + ReLU + 2x2/s2 max-pool on the dedicated forward kernel (csrc/kernels/conv_f32.hip
    conv3_pool_f32_kernel: weights resident in 8 waves' registers, window-major m-tiles pooled in registers)
    against fp64: pooled values, argmax codes wherever the window maximum is not a near-tie, dead windows 255,
    and against the implicit-GEMM path at a batch below the dedicated kernel's threshold."""
    g = torch.Generator(device=DEV).manual_seed(B + 7)
    x = torch.randn(B, 64, 10, 10, device=DEV, generator=g)
    w = torch.randn(128, 64, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(128, device=DEV, generator=g) * 0.1
    a, code = C.f32_conv_pool_fwd(x, w, b, 0, 0.0, 1.0, 2)
    z = F.conv2d(x.double(), w.double(), b.double())  # [B, 128, 8, 8]
    win = torch.stack([z[..., 0::2, 0::2], z[..., 0::2, 1::2], z[..., 1::2, 0::2], z[..., 1::2, 1::2]], -1)
    best, arg = win.max(-1)
    _close(a, best.clamp_min(0).float(), rtol=1e-5, atol=1e-5)
    top2 = win.topk(2, -1).values
    clear = ((top2[..., 0] - top2[..., 1]) > 1e-4 * (1 + top2[..., 0].abs())) & (best > 1e-4)
    want = torch.where(best > 0, arg, torch.full_like(arg, 255)).to(torch.uint8)
    assert torch.equal(code[clear], want[clear])
    assert torch.equal(code[best < -1e-4], want[best < -1e-4])
    a2, code2 = C.f32_conv_pool_fwd(x, w, b, 0, 0.0, 1.0, 2)
    assert torch.equal(a, a2) and torch.equal(code, code2)
    small, _ = C.f32_conv_pool_fwd(x[:100].contiguous(), w, b, 0, 0.0, 1.0, 2)  # the GEMM path
    _close(small, a[:100], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("planes,H", [((64, 64), 11), ((4, 8), 9), ((3, 5), 11)])
def test_pool2s1_bwd_tile_matches_elementwise(planes, H):
    """The LDS-tiled overlapping-pool backward (csrc/kernels/conv_f32.hip pool2s1_bwd_tile_kernel, 16 planes per
    tile) against autograd through max_pool2d: (64, 64) planes take the tiled path with the compile-time 10 x 10
    window grid, 9 x 9 inputs its runtime-size variant, (3, 5) = 15 planes the per-element kernel."""
    n, c = planes
    g = torch.Generator(device=DEV).manual_seed(n + c)
    z = torch.randn(n, c, H, H, device=DEV, generator=g)
    a, code = C.f32_pool_relu_fwd(z, 2, 1)
    zr = z.clone().requires_grad_()
    ref = F.max_pool2d(F.relu(zr), 2, 1)
    da = torch.randn_like(a)
    ref.backward(da)
    dz = C.f32_pool_relu_bwd(da, code, H, H, 2, 1)
    _close(dz, zr.grad, rtol=0, atol=1e-6)
