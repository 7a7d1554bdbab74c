"""Numerics of ringdp's ConvNet HIP kernels against plain PyTorch fp32 references (same ops,
inputs rounded to bf16 the way the kernels consume them).

Blocks under test (csrc/kernels/convnet.hip): F1 conv1+relu+pool1, F2 conv2+relu+pool2 (with pool2
codes), F3 conv3+relu+pool3+fc1, their backward kernels and the weight packer."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

NORM_U8 = (0.1307, 0.3081, 1.0 / 255.0)
NORM_F32 = (0.0, 1.0, 1.0)


def C():
    import ringdp

    return ringdp._C


def bf(t):
    return t.bfloat16().float()


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12))


def weights(dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    w1 = (torch.randn(32, 1, 5, 5, generator=g) * 0.2).to(dev)
    b1 = (torch.randn(32, generator=g) * 0.1).to(dev)
    w2 = (torch.randn(64, 32, 3, 3, generator=g) * 0.1).to(dev)
    b2 = (torch.randn(64, generator=g) * 0.1).to(dev)
    w3 = (torch.randn(128, 64, 3, 3, generator=g) * 0.1).to(dev)
    b3 = (torch.randn(128, generator=g) * 0.1).to(dev)
    wf = (torch.randn(10, 2048, generator=g) * 0.05).to(dev)
    bfc = torch.randn(10, generator=g).to(dev)
    return w1, b1, w2, b2, w3, b3, wf, bfc


def packed(ws):
    w1, _, w2, _, w3, _, wf, _ = ws
    return C().cn_pack_weights(w1, w2, w3, wf)


def unpool2x2(dout, idx, pooled, oh):
    """d(conv) [B, OH, OH, C] from d(pooled) [B, PH, PH, C] of a 2x2/s2 pool, argmax (dy*2+dx)
    and the ReLU mask (pooled > 0)."""
    B, PH, _, Cc = dout.shape
    dev = dout.device
    g = dout.float() * (pooled.float() > 0)
    i = idx.long()
    py = torch.arange(PH, device=dev).view(1, PH, 1, 1)
    px = torch.arange(PH, device=dev).view(1, 1, PH, 1)
    y = py * 2 + i // 2
    x = px * 2 + i % 2
    n = torch.arange(B, device=dev).view(B, 1, 1, 1)
    c = torch.arange(Cc, device=dev).view(1, 1, 1, Cc)
    lin = ((n * oh + y) * oh + x) * Cc + c
    out = torch.zeros(B * oh * oh * Cc, device=dev)
    out.index_add_(0, lin.reshape(-1), g.reshape(-1))
    return out.view(B, oh, oh, Cc)


def conv1_codes(idx):
    """pool1 code rows [B,13 py,16 co/2,16 px] bytes of two nibbles (low: even co, high: odd co; px 13..15
    zero) -> [B,13,13,32] (NHWC, like a1)."""
    assert idx.dim() == 4 and idx.shape[1:] == (13, 16, 16)
    assert not idx[:, :, :, 13:].any()
    nib = torch.stack([idx & 15, idx >> 4], -1)  # [B, 13, 16, 16, 2]
    h = nib[:, :, :, :13].permute(0, 1, 3, 2, 4).reshape(idx.shape[0], 13, 13, 32)
    # one-hot destination (1 << argmax, 0 if the ReLU is off) -> argmax | 4 * relu
    assert torch.all((h == 0) | (h == 1) | (h == 2) | (h == 4) | (h == 8))
    arg = (h == 2).to(torch.uint8) + 2 * (h == 4).to(torch.uint8) + 3 * (h == 8).to(torch.uint8)
    return torch.where(h != 0, arg | 4, torch.zeros_like(h))


def input_batch(B, u8, dev):
    if u8:
        x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device=dev)
        return x, (x.float() / 255.0 - 0.1307) / 0.3081, NORM_U8
    x = torch.randn(B, 1, 28, 28, device=dev)
    return x, x, NORM_F32


def test_pack_layout_roundtrip():
    """Packed fragments hold exactly the bf16-rounded weights (spot-check via a 1-image forward)."""
    dev = torch.device("cuda")
    ws = weights(dev)
    p = packed(ws)
    assert p.dtype == torch.bfloat16 and p.dim() == 1
    # every weight value must appear (fwd fragments alone cover all of w2 / w3)
    w2 = ws[2]
    vals = set(bf(w2).flatten().tolist())
    assert vals <= set(p.float().tolist())


@pytest.mark.parametrize("B", [1, 7, 100, 1100])
@pytest.mark.parametrize("u8", [True, False])
def test_conv1_forward(B, u8):
    torch.manual_seed(B)
    dev = torch.device("cuda")
    ws = weights(dev, B)
    w1, b1 = ws[0], ws[1]
    x, xn, norm = input_batch(B, u8, dev)
    a1, idx = C().cn_conv1_fwd(x, packed(ws), b1, *norm)
    idx = conv1_codes(idx)
    y = F.conv2d(bf(xn), bf(w1), b1, padding=1)
    ref = F.max_pool2d(F.relu(y), 2, 2).permute(0, 2, 3, 1)
    assert a1.shape == (B, 13, 13, 32) and a1.dtype == torch.bfloat16
    assert rel_err(a1, ref) < 1e-2
    yw = y.permute(0, 2, 3, 1).reshape(B, 13, 2, 13, 2, 32).permute(0, 1, 3, 5, 2, 4).reshape(B, 13, 13, 32, 4)
    picked = torch.gather(yw, 4, (idx.long() & 3).unsqueeze(-1)).squeeze(-1)
    ok = (yw.max(-1).values - picked) <= 1e-3 * (1 + yw.abs().max(-1).values)
    # the argmax only matters (and is only defined) where the pooled value passes the ReLU
    assert torch.all(ok | ((idx & 4) == 0))
    # bit 2 of the argmax byte is the ReLU mask of the pooled value
    assert torch.equal((idx & 4) != 0, a1.float() > 0)


def pool2_ref(z2):
    """relu + 2x2/s1 max pool of a bf16 z2 [B,11,11,64] with the kernel's code byte: one-hot bit
    dy*2+dx of the first maximum in (0,0),(0,1),(1,0),(1,1) order, 0 where the pooled value is 0."""
    z = z2.float()
    v = torch.stack([z[:, :-1, :-1], z[:, :-1, 1:], z[:, 1:, :-1], z[:, 1:, 1:]], -1)
    m = v.max(-1).values.clamp_min(0)
    first = torch.argmax((v == m.unsqueeze(-1)).to(torch.int8), -1)
    code = torch.where(m > 0, 1 << first, torch.zeros_like(first)).to(torch.uint8)
    return m.bfloat16(), code


@pytest.mark.parametrize("B", [1, 5, 100, 600])
def test_conv2_forward(B):
    torch.manual_seed(B)
    dev = torch.device("cuda")
    ws = weights(dev, B + 1)
    a1 = torch.relu(torch.randn(B, 13, 13, 32, device=dev)).bfloat16()
    a2, idx2 = C().cn_conv2_fwd(a1, packed(ws), ws[3])
    z = F.conv2d(a1.permute(0, 3, 1, 2).float(), bf(ws[2]), ws[3]).permute(0, 2, 3, 1)
    ref = F.max_pool2d(F.relu(z.permute(0, 3, 1, 2)), 2, 1).permute(0, 2, 3, 1)
    assert a2.shape == (B, 10, 10, 64) and a2.dtype == torch.bfloat16 and idx2.dtype == torch.uint8
    assert rel_err(a2, ref) < 1e-2
    # codes: one-hot (a single bit of 0..3) where the pooled value is > 0, else 0; the named position
    # holds the window maximum
    live = idx2 != 0
    assert torch.equal(live, a2.float() != 0)
    assert torch.all((idx2 & (idx2 - 1)) == 0) and int(idx2.max()) <= 8
    v = torch.stack([z[:, :-1, :-1], z[:, :-1, 1:], z[:, 1:, :-1], z[:, 1:, 1:]], -1)
    arg = torch.log2(idx2.clamp_min(1).float()).long()
    picked = torch.gather(v, 4, arg.unsqueeze(-1)).squeeze(-1)
    tol = 1e-2 * (1 + v.abs().amax(-1))
    assert torch.all(((v.amax(-1) - picked) <= tol)[live])
    # on bf16-exact inputs the codes are exactly torch's first-max argmax
    za, zc = pool2_ref(z.bfloat16())
    assert float((zc == idx2).float().mean()) > 0.99


def f3_reference(a2, ws):
    w3, b3, wf, bfc = ws[4], ws[5], ws[6], ws[7]
    y = F.conv2d(a2.permute(0, 3, 1, 2).float(), bf(w3), b3)
    a3 = F.max_pool2d(F.relu(y), 2, 2)
    return y, a3, F.linear(a3.reshape(-1, 2048), bf(wf), bfc)


@pytest.mark.parametrize("B", [1, 3, 100, 700])
def test_conv3_fc_forward(B):
    torch.manual_seed(B)
    dev = torch.device("cuda")
    ws = weights(dev, B + 2)
    a2 = torch.relu(torch.randn(B, 10, 10, 64, device=dev)).bfloat16()
    logits, a3, idx3 = C().cn_conv3_fc_fwd(a2, packed(ws), ws[5], ws[7])
    y, a3_ref, logits_ref = f3_reference(a2, ws)
    assert a3.shape == (B, 16, 128) and idx3.shape == (B, 16, 128)
    a3_nchw = a3.view(B, 4, 4, 128).permute(0, 3, 1, 2)
    assert rel_err(a3_nchw, a3_ref) < 1e-2
    assert rel_err(logits, logits_ref) < 1.5e-2
    assert int(idx3.max()) <= 3


# 3000 / 9000: above fc_in_c3_max_batch, the 8-wave conv3 backward (dgrad and wgrad workgroups, the wgrad
# ones taking the last images of the data gradient)
@pytest.mark.parametrize("B", [1, 3, 64, 257, 3000, 9000])
@pytest.mark.parametrize("need_dz2", [True, False])
def test_conv3_fc_backward(B, need_dz2):
    torch.manual_seed(7 + B)
    dev = torch.device("cuda")
    ws = weights(dev, B + 3)
    w3, b3, wf, bfc = ws[4], ws[5], ws[6], ws[7]
    z2 = torch.randn(B, 11, 11, 64, device=dev).bfloat16()
    a2, idx2 = pool2_ref(z2)
    pk = packed(ws)
    logits, a3, idx3 = C().cn_conv3_fc_fwd(a2, pk, b3, bfc)
    dl = torch.randn(B, 10, device=dev)
    dw3, db3, dwf, dbf = (torch.empty_like(t) for t in (w3, b3, wf, bfc))
    dz2 = C().cn_conv3_fc_bwd(a2, idx2, a3, idx3, wf, dl, pk, need_dz2, dw3, db3, dwf, dbf)
    # reference: fc backward in fp32, unpool through the kernel's own pool3 argmax
    a3_flat = a3.view(B, 4, 4, 128).permute(0, 3, 1, 2).reshape(B, 2048).float()
    tol = 1e-4 * max(1.0, (B / 256) ** 0.5)  # fp32 sums over B images in a different order than the matmul
    torch.testing.assert_close(dwf, dl.t() @ a3_flat, rtol=1e-4, atol=tol)
    torch.testing.assert_close(dbf, dl.sum(0), rtol=1e-5, atol=tol / 10)
    da3 = (dl @ wf).view(B, 128, 4, 4).permute(0, 2, 3, 1)
    dconv = bf(unpool2x2(da3, idx3.view(B, 4, 4, 128), a3.view(B, 4, 4, 128), 8)).permute(0, 3, 1, 2)
    z2f = z2.permute(0, 3, 1, 2).float().requires_grad_()
    w3q = bf(w3).requires_grad_()
    b3q = b3.clone().requires_grad_()
    F.conv2d(F.max_pool2d(F.relu(z2f), 2, 1), w3q, b3q).backward(dconv)
    assert rel_err(dw3, w3q.grad) < 5e-3
    assert rel_err(db3, b3q.grad) < 5e-3
    if need_dz2:
        assert dz2.shape == (B, 11, 11, 64)
        assert rel_err(dz2.permute(0, 3, 1, 2), z2f.grad) < 1.5e-2
    else:
        assert dz2 is None


@pytest.mark.parametrize("B", [1, 3, 64, 257])
def test_conv2_backward(B):
    torch.manual_seed(11 + B)
    dev = torch.device("cuda")
    ws = weights(dev, B + 4)
    w2, b2 = ws[2], ws[3]
    a1 = torch.relu(torch.randn(B, 13, 13, 32, device=dev)).bfloat16()
    dz2 = torch.randn(B, 11, 11, 64, device=dev).bfloat16()
    dw2, db2 = torch.empty_like(w2), torch.empty_like(b2)
    da1 = C().cn_conv2_bwd(a1, dz2, packed(ws), True, dw2, db2)
    dconv = dz2.float().permute(0, 3, 1, 2)
    x = a1.permute(0, 3, 1, 2).float().requires_grad_()
    wq = bf(w2).requires_grad_()
    bq = b2.clone().requires_grad_()
    F.conv2d(x, wq, bq).backward(dconv)
    assert rel_err(da1.permute(0, 3, 1, 2), x.grad) < 1.5e-2
    assert rel_err(dw2, wq.grad) < 5e-3
    assert rel_err(db2, bq.grad) < 5e-3


@pytest.mark.parametrize("B", [1, 9, 100, 300])
@pytest.mark.parametrize("u8", [True, False])
def test_conv1_wgrad(B, u8):
    torch.manual_seed(13 + B)
    dev = torch.device("cuda")
    ws = weights(dev, B + 5)
    w1, b1 = ws[0], ws[1]
    x, xn, norm = input_batch(B, u8, dev)
    a1, idx = C().cn_conv1_fwd(x, packed(ws), b1, *norm)
    da1 = torch.randn(B, 13, 13, 32, device=dev).bfloat16()
    dw, db = torch.empty_like(w1), torch.empty_like(b1)
    C().cn_conv1_wgrad(x, da1, idx, dw, db, *norm)
    dconv = bf(unpool2x2(da1, conv1_codes(idx) & 3, a1, 26)).permute(0, 3, 1, 2)
    wq = w1.clone().requires_grad_()
    bq = b1.clone().requires_grad_()
    F.conv2d(bf(xn), wq, bq, padding=1).backward(dconv)
    assert rel_err(dw, wq.grad) < 5e-3
    assert rel_err(db, bq.grad) < 5e-3


# 3000: above fc_in_c3_max_batch, the wave-specialised 8-wave kernel (conv12_bwd8_kernel)
@pytest.mark.parametrize("B", [1, 7, 100, 513, 3000])
@pytest.mark.parametrize("u8", [True, False])
def test_conv12_backward_fused(B, u8):
    """Fused conv2 backward + conv1 wgrad (da1 kept in LDS) against the fp32 PyTorch reference of both
    layers, against the separate kernels, and bitwise run to run."""
    torch.manual_seed(17 + B)
    dev = torch.device("cuda")
    ws = weights(dev, B + 6)
    w1, b1, w2, b2 = ws[0], ws[1], ws[2], ws[3]
    x, xn, norm = input_batch(B, u8, dev)
    pk = packed(ws)
    a1, idx1 = C().cn_conv1_fwd(x, pk, b1, *norm)
    dz2 = torch.randn(B, 11, 11, 64, device=dev).bfloat16()
    outs = []
    for _ in range(2):
        g = [torch.empty_like(t) for t in (w2, b2, w1, b1)]
        C().cn_conv12_bwd(x, idx1, a1, dz2, pk, *g, *norm)
        outs.append(g)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    dw2, db2, dw1, db1 = outs[0]
    # separate kernels
    sw2, sb2, sw1, sb1 = (torch.empty_like(t) for t in (w2, b2, w1, b1))
    da1 = C().cn_conv2_bwd(a1, dz2, pk, True, sw2, sb2)
    C().cn_conv1_wgrad(x, da1, idx1, sw1, sb1, *norm)
    for f, r in ((dw2, sw2), (db2, sb2), (dw1, sw1), (db1, sb1)):
        assert rel_err(f, r) < 1e-4
    # fp32 reference of both layers (conv2 on the kernel's a1, conv1 through the kernel's pool1 codes)
    a1q = a1.permute(0, 3, 1, 2).float().requires_grad_()
    w2q = bf(w2).requires_grad_()
    b2q = b2.clone().requires_grad_()
    F.conv2d(a1q, w2q, b2q).backward(dz2.float().permute(0, 3, 1, 2))
    assert rel_err(dw2, w2q.grad) < 5e-3
    assert rel_err(db2, b2q.grad) < 5e-3
    da1_ref = bf(a1q.grad.permute(0, 2, 3, 1))
    dconv = bf(unpool2x2(da1_ref, conv1_codes(idx1) & 3, a1, 26)).permute(0, 3, 1, 2)
    w1q = w1.clone().requires_grad_()
    b1q = b1.clone().requires_grad_()
    F.conv2d(bf(xn), w1q, b1q, padding=1).backward(dconv)
    assert rel_err(dw1, w1q.grad) < 1.5e-2
    assert rel_err(db1, b1q.grad) < 1.5e-2


def test_wgrad_deterministic():
    """Slab reductions and the dgrad K-group sums run in a fixed order: two identical backward calls
    are bitwise equal."""
    dev = torch.device("cuda")
    ws = weights(dev, 9)
    B = 333
    a2, idx2 = pool2_ref(torch.randn(B, 11, 11, 64, device=dev).bfloat16())
    pk = packed(ws)
    logits, a3, idx3 = C().cn_conv3_fc_fwd(a2, pk, ws[5], ws[7])
    dl = torch.randn(B, 10, device=dev)
    outs = []
    for _ in range(2):
        g = [torch.empty_like(t) for t in (ws[4], ws[5], ws[6], ws[7])]
        dz2 = C().cn_conv3_fc_bwd(a2, idx2, a3, idx3, ws[6], dl, pk, True, *g)
        outs.append(g + [dz2])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


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


@pytest.mark.parametrize("B,u8", [(1, True), (100, True), (300, False), (1031, True), (5000, True)])
def test_fused_forward_matches_separate_kernels(B, u8):
    """cn_forward_fused (conv1 -> conv2 -> conv3 + fc1 in one launch, a1 / a2 handed over in LDS) writes
    the same a1 / idx1 / a2 / idx2 / a3 / idx3 / packed bytes as the three-launch path, and the same
    logits (bit-identical where the separate path also runs fc1 inside conv3's launch, B <= 4096)."""
    torch.manual_seed(B)
    ws = weights("cuda", seed=B)
    w1, b1, w2, b2, w3, b3, wf, bfc = ws
    if u8:
        x = torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device="cuda")
        norm = NORM_U8
    else:
        x = torch.randn(B, 1, 28, 28, device="cuda")
        norm = NORM_F32
    a1, i1, pk = C().cn_conv1_fwd_pack(x, w1, w2, w3, wf, b1, *norm)
    a2, i2 = C().cn_conv2_fwd(a1, pk, b2)
    lg, a3, i3 = C().cn_conv3_fc_fwd(a2, pk, b3, bfc)
    bufs = C().cn_forward_buffers(x)
    lg_f, a3_f, i3_f = C().cn_forward_fused(x, w1, b1, w2, b2, w3, b3, wf, bfc, *norm, *bufs)
    torch.cuda.synchronize()
    for name, want, got in (("a1", a1, bufs[0]), ("idx1", i1, bufs[1]), ("a2", a2, bufs[2]), ("idx2", i2, bufs[3]),
                            ("packed", pk, bufs[4]), ("a3", a3, a3_f), ("idx3", i3, i3_f)):
        assert torch.equal(want, got), name
    if B <= 4096:
        assert torch.equal(lg, lg_f)
    else:
        torch.testing.assert_close(lg_f, lg, rtol=1e-4, atol=1e-4)


def test_fc_backward_inside_conv3_launch_matches_separate():
    """B <= 2048: the fc1 backward runs as the first workgroups of the conv3 backward launch and the conv3
    roles form the compact gradient themselves; B = 2049 takes the separate fc1 launch.  With a zero
    logits gradient for the extra image, dz2 of the shared 2048 images is bit-identical and the weight
    gradients agree to summation order."""
    torch.manual_seed(11)
    dev = torch.device("cuda")
    ws = weights(dev, 13)
    w3, b3, wf, bfc = ws[4], ws[5], ws[6], ws[7]
    pk = packed(ws)
    B = 2049
    z2 = torch.randn(B, 11, 11, 64, device=dev).bfloat16()
    a2, idx2 = pool2_ref(z2)
    logits, a3, idx3 = C().cn_conv3_fc_fwd(a2, pk, b3, bfc)
    dl = torch.randn(B, 10, device=dev)
    dl[-1] = 0
    outs = []
    for n in (B - 1, B):
        g = [torch.empty_like(t) for t in (w3, b3, wf, bfc)]
        dz2 = C().cn_conv3_fc_bwd(a2[:n].contiguous(), idx2[:n].contiguous(), a3[:n].contiguous(),
                                  idx3[:n].contiguous(), wf, dl[:n].contiguous(), pk, True, *g)
        outs.append((dz2, g))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0][: B - 1])
    for a, b in zip(outs[0][1], outs[1][1]):  # other slab partitions: other fp32 summation orders
        assert float((a - b).norm() / b.norm()) < 1e-5
