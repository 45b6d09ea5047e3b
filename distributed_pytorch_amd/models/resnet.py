"""ResNet-50 (v1.5: stride on the 3x3 conv) for the BASELINE.json stress config
("ResNet-50 ImageNet-shaped bf16 8xMI355X DDP") — new scope, the reference has only VGG.

``ResNet`` is built from the NHWC kernel layers (ops/layers.py): every conv runs the gfx950
implicit-GEMM kernels (bf16 MFMA, or x3 fp32-grade), every BatchNorm is fused with its ReLU /
residual-add+ReLU, the stem max-pool is the native NHWC pool, and the head (global average pool +
Linear + softmax-CE) is one autograd node over head.hip + gemm_f32.hip (fp32 matrix cores)
(``model(x, target)`` returns the loss; ``model(x)`` the logits).
Parameter / buffer names and shapes (state_dict) match torchvision's ``resnet50`` so checkpoints
interchange.  ``ResNetRef`` is the same network from stock torch NCHW modules: the numerics
oracle for tests.
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import functional as Fn
from ..ops.layers import BatchNorm2d, Conv2d, MaxPool2d

LAYERS = {"resnet50": [3, 4, 6, 3], "resnet101": [3, 4, 23, 3], "resnet152": [3, 8, 36, 3]}


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int, downsample: bool, impl: str):
        super().__init__()
        cout = width * 4
        self.conv1 = Conv2d(cin, width, 1, 1, 0, impl)
        self.bn1 = BatchNorm2d(width, "relu")
        self.conv2 = Conv2d(width, width, 3, stride, 1, impl)
        self.bn2 = BatchNorm2d(width, "relu")
        self.conv3 = Conv2d(width, cout, 1, 1, 0, impl)
        self.bn3 = BatchNorm2d(cout, "add_relu")
        self.downsample = (nn.Sequential(Conv2d(cin, cout, 1, stride, 0, impl), BatchNorm2d(cout, "none"))
                           if downsample else None)
        # x's gradient has two contributions (conv1, and the identity or the downsample conv): they
        # are summed inside the last one's data-gradient reduction instead of by autograd (GradJoin)
        self._join = Fn.GradJoin(2)

    def forward(self, x):
        j = self._join if (self.training and torch.is_grad_enabled() and x.requires_grad) else None
        if j is not None:
            j.reset()
            # x made by a BN backward that sums a second gradient operand on load: the join may leave
            # its stash to it instead of an add pass; the hook adds it if autograd summed x's gradient
            j.defer = Fn.DEFER_JOIN and bool(getattr(x, "_dpa_sum_on_load", False))
            j.key = None
            if j.defer:
                x.register_hook(j.guard)
        out = self.bn1(self.conv1(x, j))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:  # the downsample BN is applied inside bn3's add (one pass on GPU)
            return self.bn3(self.conv3(out), self.downsample[0](x, j), res_bn=self.downsample[1])
        return self.bn3(self.conv3(out), x, res_join=j)


class ResNet(nn.Module):
    """Input NHWC fp32 [N,H,W,3]; output logits [N, num_classes] (fp32).  With impl "bf16" the
    activations between layers are bf16 tensors; parameters, BN statistics and the head are fp32."""

    def __init__(self, layers: List[int], num_classes: int = 1000, impl: str = "bf16"):
        super().__init__()
        self.impl = impl
        self.conv1 = Conv2d(3, 64, 7, 2, 3, impl)
        self.bn1 = BatchNorm2d(64, "relu")
        self.maxpool = MaxPool2d(3, 2, 1)
        cin = 64
        for li, (n, width, stride) in enumerate(zip(layers, (64, 128, 256, 512), (1, 2, 2, 2))):
            blocks = []
            for b in range(n):
                s = stride if b == 0 else 1
                blocks.append(Bottleneck(cin, width, s, b == 0, impl))
                cin = width * 4
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))
        self.fc = nn.Linear(cin, num_classes)
        self.fc.weight._dpa_direct = self.fc.bias._dpa_direct = True  # the head writes their optimizer slots
        self._init()

    def _init(self):
        # torchvision resnet init: kaiming_normal_(fan_out, relu) convs, BN (1, 0)
        for m in self.modules():
            if isinstance(m, Conv2d):
                w = torch.empty(m.cout, m.cin, m.k, m.k)
                nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")
                with torch.no_grad():
                    m.weight.zero_()
                    m.weight[..., :m.cin].copy_(w.permute(0, 2, 3, 1))

    def features(self, x):
        mp = self.maxpool
        x = self.bn1(self.conv1(x), pool=(mp.k, mp.stride, mp.padding))  # BN + ReLU + max-pool, one pass on GPU
        return self.layer4(self.layer3(self.layer2(self.layer1(x))))

    def forward(self, x, target=None):
        """Logits, or with ``target`` the batch-mean cross-entropy through the fused head."""
        if self.training:
            Fn.clear_deferred()
        f = self.features(x)
        if target is not None:
            return Fn.head_ce(f, self.fc.weight, self.fc.bias, target)
        return Fn.head_logits(f, self.fc.weight, self.fc.bias)


def resnet50(num_classes: int = 1000, impl: str = "bf16") -> ResNet:
    return ResNet(LAYERS["resnet50"], num_classes, impl)


# ---------------------------------------------------------------- stock-torch oracle (NCHW)
class _RefBottleneck(nn.Module):
    def __init__(self, cin, width, stride, downsample):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.downsample = (nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
                           if downsample else None)

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        identity = self.downsample(x) if self.downsample is not None else x
        return F.relu(out + identity)


class ResNetRef(nn.Module):
    """Input NCHW."""

    def __init__(self, layers: List[int], num_classes: int = 1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        cin = 64
        for li, (n, width, stride) in enumerate(zip(layers, (64, 128, 256, 512), (1, 2, 2, 2))):
            blocks = []
            for b in range(n):
                blocks.append(_RefBottleneck(cin, width, stride if b == 0 else 1, b == 0))
                cin = width * 4
            setattr(self, f"layer{li + 1}", nn.Sequential(*blocks))
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))
