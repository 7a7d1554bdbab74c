"""Numerics of ringdp's ConvNet HIP kernels against plain PyTorch fp32 references (same ops,
inputs rounded to bf16 the way the kernels consume them)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GEO = {2: dict(cin=32, cout=64, ih=13, ps=1, oh=11, ph=10), 3: dict(cin=64, cout=128, ih=10, ps=2, oh=8, ph=4)}


def C():
    import ringdp

    return ringdp._C


def bf(t):
    return t.bfloat16().float()


def unpool(dout, idx, pooled, ps, oh):
    """d(conv) [B, OH, OH, C] from d(pooled), argmax (dy*2+dx) and the ReLU mask (pooled > 0)."""
    B, PH, _, Cc = dout.shape
    dev = dout.device
    g = dout.float() * (pooled.float() > 0)
    i = idx.long()
    py = torch.arange(PH, device=dev).view(1, PH, 1, 1)
    px = torch.arange(PH, device=dev).view(1, 1, PH, 1)
    y = py * ps + i // 2
    x = px * ps + i % 2
    n = torch.arange(B, device=dev).view(B, 1, 1, 1)
    c = torch.arange(Cc, device=dev).view(1, 1, 1, Cc)
    lin = ((n * oh + y) * oh + x) * Cc + c
    out = torch.zeros(B * oh * oh * Cc, device=dev)
    out.index_add_(0, lin.reshape(-1), g.reshape(-1))
    return out.view(B, oh, oh, Cc)


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12))


@pytest.mark.parametrize("B", [1, 7, 100])
@pytest.mark.parametrize("u8", [True, False])
def test_conv1_forward(B, u8):
    torch.manual_seed(B)
    dev = torch.device("cuda")
    w = torch.randn(32, 1, 5, 5, device=dev) * 0.2
    b = torch.randn(32, device=dev) * 0.1
    if u8:
        x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=dev)
        xn = (x.float() / 255.0 - 0.1307) / 0.3081
        a1, idx = C().convnet_conv1_fwd(x, w, b, 0.1307, 0.3081, 1.0 / 255.0)
    else:
        xn = torch.randn(B, 1, 28, 28, device=dev)
        a1, idx = C().convnet_conv1_fwd(xn, w, b, 0.0, 1.0, 1.0)
    y = F.conv2d(xn, w, b, padding=1)
    ref = F.max_pool2d(F.relu(y), 2, 2).permute(0, 2, 3, 1)
    assert a1.shape == (B, 13, 13, 32) and a1.dtype == torch.bfloat16
    assert rel_err(a1, ref) < 1e-2
    # argmax must point at a maximal element of its window
    yw = y.permute(0, 2, 3, 1).reshape(B, 13, 2, 13, 2, 32).permute(0, 1, 3, 5, 2, 4).reshape(B, 13, 13, 32, 4)
    picked = torch.gather(yw, 4, idx.long().unsqueeze(-1)).squeeze(-1)
    assert torch.all((yw.max(-1).values - picked) <= 1e-4 * (1 + yw.abs().max(-1).values))


@pytest.mark.parametrize("layer", [2, 3])
@pytest.mark.parametrize("B", [1, 5, 100, 600])
def test_conv_forward(layer, B):
    g = GEO[layer]
    torch.manual_seed(layer * 1000 + B)
    dev = torch.device("cuda")
    inp = torch.randn(B, g["ih"], g["ih"], g["cin"], device=dev).bfloat16()
    w = torch.randn(g["cout"], g["cin"], 3, 3, device=dev) * 0.1
    b = torch.randn(g["cout"], device=dev) * 0.1
    out, idx = C().convnet_conv_fwd(layer, inp, w, b)
    y = F.conv2d(inp.permute(0, 3, 1, 2).float(), bf(w), b)
    ref = F.max_pool2d(F.relu(y), 2, g["ps"]).permute(0, 2, 3, 1)
    assert out.shape == (B, g["ph"], g["ph"], g["cout"])
    assert rel_err(out, ref) < 1e-2
    assert int(idx.max()) <= 3


@pytest.mark.parametrize("layer", [2, 3])
@pytest.mark.parametrize("B", [1, 3, 64, 257])
def test_conv_backward(layer, B):
    g = GEO[layer]
    torch.manual_seed(7 * layer + B)
    dev = torch.device("cuda")
    inp = torch.randn(B, g["ih"], g["ih"], g["cin"], device=dev).bfloat16()
    w = torch.randn(g["cout"], g["cin"], 3, 3, device=dev) * 0.1
    b = torch.randn(g["cout"], device=dev) * 0.1
    out, idx = C().convnet_conv_fwd(layer, inp, w, b)
    dout = torch.randn(B, g["ph"], g["ph"], g["cout"], device=dev).bfloat16()
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    din = C().convnet_conv_bwd(layer, inp, w, dout, idx, out, True, dw, db)
    dconv = bf(unpool(dout, idx, out, g["ps"], g["oh"])).permute(0, 3, 1, 2)
    x = inp.permute(0, 3, 1, 2).float().requires_grad_()
    wq = bf(w).requires_grad_()
    bq = b.clone().requires_grad_()
    F.conv2d(x, wq, bq).backward(dconv)
    assert rel_err(din.permute(0, 3, 1, 2), x.grad) < 1.5e-2
    assert rel_err(dw, wq.grad) < 5e-3
    assert rel_err(db, bq.grad) < 5e-3


@pytest.mark.parametrize("B", [1, 9, 100, 300])
@pytest.mark.parametrize("u8", [True, False])
def test_conv1_wgrad(B, u8):
    torch.manual_seed(11 + B)
    dev = torch.device("cuda")
    w = torch.randn(32, 1, 5, 5, device=dev) * 0.2
    b = torch.randn(32, device=dev) * 0.1
    if u8:
        x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=dev)
        xn = (x.float() / 255.0 - 0.1307) / 0.3081
        norm = (0.1307, 0.3081, 1.0 / 255.0)
    else:
        x = torch.randn(B, 1, 28, 28, device=dev)
        xn = x
        norm = (0.0, 1.0, 1.0)
    a1, idx = C().convnet_conv1_fwd(x, w, b, *norm)
    da1 = torch.randn(B, 13, 13, 32, device=dev).bfloat16()
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    C().convnet_conv1_wgrad(x, da1, idx, a1, dw, db, *norm)
    dconv = bf(unpool(da1, idx, a1, 2, 26)).permute(0, 3, 1, 2)
    wq = w.clone().requires_grad_()
    bq = b.clone().requires_grad_()
    F.conv2d(bf(xn), wq, bq, padding=1).backward(dconv)
    assert rel_err(dw, wq.grad) < 5e-3
    assert rel_err(db, bq.grad) < 5e-3


@pytest.mark.parametrize("B", [1, 6, 100, 1000])
def test_fc_forward_backward(B):
    torch.manual_seed(B)
    dev = torch.device("cuda")
    a3 = torch.randn(B, 4, 4, 128, device=dev).bfloat16()
    w = torch.randn(10, 2048, device=dev) * 0.05
    b = torch.randn(10, device=dev)
    logits = C().convnet_fc_fwd(a3, w, b)
    xflat = a3.float().permute(0, 3, 1, 2).reshape(B, 2048)  # CHW flatten, as view(-1, 2048)
    ref = F.linear(xflat, w, b)
    assert rel_err(logits, ref) < 1e-4
    dl = torch.randn(B, 10, device=dev)
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    da3 = C().convnet_fc_bwd(a3, w, dl, dw, db)
    da_ref = (dl @ w).view(B, 128, 4, 4).permute(0, 2, 3, 1)
    assert rel_err(da3, da_ref) < 1e-2
    assert rel_err(dw, dl.t() @ xflat) < 1e-4
    assert rel_err(db, dl.sum(0)) < 1e-5


@pytest.mark.parametrize("B,Cn", [(1, 10), (100, 10), (4097, 10), (33, 1000)])
@pytest.mark.parametrize("smooth", [0.0, 0.1])
@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_cross_entropy(B, Cn, smooth, reduction):
    from ringdp.nn import CrossEntropyLoss

    torch.manual_seed(B + Cn)
    dev = torch.device("cuda")
    logits = (torch.randn(B, Cn, device=dev) * 3).requires_grad_()
    y = torch.randint(0, Cn, (B,), device=dev)
    if B > 3:
        y[1] = -100
    loss = CrossEntropyLoss(reduction=reduction, label_smoothing=smooth)(logits, y)
    ref_logits = logits.detach().clone().requires_grad_()
    ref = F.cross_entropy(ref_logits, y, reduction=reduction, label_smoothing=smooth)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    gout = torch.randn_like(ref) if reduction == "none" else torch.tensor(1.7, device=dev)
    loss.backward(gout)
    ref.backward(gout)
    torch.testing.assert_close(logits.grad, ref_logits.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("momentum,nesterov,wd,damp", [(0.0, False, 0.0, 0.0), (0.9, True, 1e-4, 0.0),
                                                       (0.9, False, 1e-2, 0.1)])
@pytest.mark.parametrize("flat", [True, False])
def test_sgd_matches_torch(momentum, nesterov, wd, damp, flat):
    import ringdp

    torch.manual_seed(3)
    dev = torch.device("cuda")
    shapes = [(10, 2048), (10,), (128, 64, 3, 3), (33,)]
    ps = [torch.randn(s, device=dev) for s in shapes]
    ref_ps = [p.clone().requires_grad_() for p in ps]
    my_ps = [p.clone().requires_grad_() for p in ps]
    if flat:
        # emulate DDP flattening: params + grads as views of aligned flat buffers
        offs, tot = [], 0
        for p in my_ps:
            offs.append(tot)
            tot += (p.numel() + 15) // 16 * 16
        fp = torch.zeros(tot, device=dev)
        fg = torch.zeros(tot, device=dev)
        for p, o in zip(my_ps, offs):
            v = fp[o:o + p.numel()].view_as(p)
            v.copy_(p.data)
            p.data = v
            p._ringdp_flat = (fp, fg, o, len(my_ps))
    ref_opt = torch.optim.SGD(ref_ps, lr=0.05, momentum=momentum, nesterov=nesterov, weight_decay=wd, dampening=damp)
    my_opt = ringdp.optim.SGD(my_ps, lr=0.05, momentum=momentum, nesterov=nesterov, weight_decay=wd, dampening=damp)
    for step in range(4):
        grads = [torch.randn(s, device=dev) for s in shapes]
        for p, g in zip(ref_ps, grads):
            p.grad = g.clone()
        for i, (p, g) in enumerate(zip(my_ps, grads)):
            if flat:
                view = fg[offs[i]:offs[i] + p.numel()].view_as(p)
                view.copy_(g)
                p.grad = view
            else:
                p.grad = g.clone()
        ref_opt.step()
        my_opt.step()
        for a, r in zip(my_ps, ref_ps):
            torch.testing.assert_close(a.detach(), r.detach(), rtol=1e-5, atol=1e-6)


def test_cast_kernels():
    dev = torch.device("cuda")
    x = torch.randn(12345, device=dev)
    y = torch.empty(12345, dtype=torch.bfloat16, device=dev)
    C().cast_copy(y, x)
    torch.testing.assert_close(y, x.bfloat16(), rtol=0, atol=0)
    z = torch.empty(12345, device=dev)
    C().cast_copy(z, y)
    torch.testing.assert_close(z, y.float(), rtol=0, atol=0)
    h = torch.empty(12345, dtype=torch.float16, device=dev)
    C().cast_copy(h, x)
    torch.testing.assert_close(h, x.half(), rtol=0, atol=0)


def test_synth_images_deterministic():
    dev = torch.device("cuda")
    a = C().synth_u8_images(64, 28, 28, 10, 5, dev)
    b = C().synth_u8_images(64, 28, 28, 10, 5, dev)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert a[0].shape == (64, 1, 28, 28) and int(a[1].max()) < 10
