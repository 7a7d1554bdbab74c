"""Per-block forward agreement of the NHWC kernel path vs a bf16-emulating ATen oracle."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from ringdp import models  # noqa: E402
from ringdp.ops.nhwc import MaxPoolNHWC, to_nhwc  # noqa: E402
from ringdp.models.resnet import _fused  # noqa: E402


class R(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


def cos(a, b):
    return float(F.cosine_similarity(a.reshape(1, -1).float(), b.reshape(1, -1).float()))


arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
res = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.manual_seed(0)
m = getattr(models, arch)(num_classes=10).cuda()
for mod in m.modules():
    if isinstance(mod, torch.nn.Conv2d):
        mod.weight.data = mod.weight.data.bfloat16().float()
ref = copy.deepcopy(m)
for mod in ref.modules():
    if isinstance(mod, (torch.nn.Conv2d, torch.nn.BatchNorm2d, torch.nn.ReLU)):
        mod.register_forward_hook(lambda mm, i, o: R.apply(o))
x = torch.randn(32, 3, res, res, device="cuda")
h = to_nhwc(x)
h = _fused(h, m.conv1, m.bn1, True)
hr = ref.relu(ref.bn1(ref.conv1(x)))
print("stem", cos(h.permute(0, 3, 1, 2), hr))
h = MaxPoolNHWC.apply(h, 3, 2, 1)
hr = ref.maxpool(hr)
print("pool", cos(h.permute(0, 3, 1, 2), hr))
for li, (layer, rlayer) in enumerate(zip((m.layer1, m.layer2, m.layer3, m.layer4),
                                         (ref.layer1, ref.layer2, ref.layer3, ref.layer4))):
    for bi, (blk, rblk) in enumerate(zip(layer, rlayer)):
        # feed the SAME input to both to isolate per-block error
        hin = h
        h = blk.forward_nhwc(hin)
        hr_same = rblk(hin.float().permute(0, 3, 1, 2).contiguous())
        hr = rblk(hr)
        print(f"layer{li+1}.{bi}", "same-input", round(cos(h.permute(0, 3, 1, 2), hr_same), 5),
              "chained", round(cos(h.permute(0, 3, 1, 2), hr), 5))
