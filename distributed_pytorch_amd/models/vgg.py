"""VGG family for 3x32x32 inputs / 10 classes — the reference model (``/root/reference/model.py``).

Two faces of the same network:

* ``VGG11()`` … ``VGG19()`` return a plain ``torch.nn.Module`` with the reference's structure
  and parameter/buffer names (``layers.{i}.*`` Sequential of Conv2d(3x3,s1,p1,bias) →
  BatchNorm2d → ReLU(inplace) with MaxPool2d(2,2) at each ``'M'``, then ``fc1 = Linear(512,10)``;
  model.py:3-50).  Its ``state_dict`` has the reference's 58 keys for VGG-11, so checkpoints are
  interchangeable with ``model.VGG11()``.
* ``VGGSpec`` — the static layer plan (channels, spatial sizes, pool flags, state-dict key names)
  consumed by :class:`distributed_pytorch_amd.engine.VGGEngine`, the hand-scheduled MI355X
  trainer.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

import torch.nn as nn

CFG = {
    "VGG11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "VGG19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"],
}


def make_layers(cfg) -> nn.Sequential:
    layers: list = []
    c = 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(c, v, kernel_size=3, stride=1, padding=1, bias=True), nn.BatchNorm2d(v),
                       nn.ReLU(inplace=True)]
            c = v
    return nn.Sequential(*layers)


class VGG(nn.Module):
    """VGG for 3x32x32 input, 10 classes (reference model.py:30-46)."""

    def __init__(self, name: str = "VGG11", num_classes: int = 10):
        super().__init__()
        self.name = name
        self.layers = make_layers(CFG[name])
        self.fc1 = nn.Linear(512, num_classes)

    def forward(self, x):
        y = self.layers(x)
        y = y.view(y.size(0), -1)
        return self.fc1(y)


def VGG11(num_classes: int = 10) -> VGG:
    return VGG("VGG11", num_classes)


def VGG13(num_classes: int = 10) -> VGG:
    return VGG("VGG13", num_classes)


def VGG16(num_classes: int = 10) -> VGG:
    return VGG("VGG16", num_classes)


def VGG19(num_classes: int = 10) -> VGG:
    return VGG("VGG19", num_classes)


@dataclass
class ConvLayer:
    idx: int          # position in the reference Sequential (conv module index)
    cin: int          # true input channels (3 for the first layer)
    cin_pad: int      # channels as stored by the engine (first layer padded to 4 or 8)
    cout: int
    hw: int           # input (= conv output) spatial size
    pool: bool        # followed by MaxPool2d(2,2)
    conv_key: str = ""
    bn_key: str = ""


@dataclass
class VGGSpec:
    name: str
    convs: List[ConvLayer] = field(default_factory=list)
    num_classes: int = 10
    fc_in: int = 512
    in_hw: int = 32

    @classmethod
    def from_name(cls, name: str = "VGG11", num_classes: int = 10, in_hw: int = 32, in_pad: int = 4) -> "VGGSpec":
        """in_pad: channels the 3-channel input is zero-padded to (4 for the fp32 kernels, 8 for
        the bf16-plane kernels, whose 16-byte operand chunks are 8 channels)."""
        cfg = CFG[name]
        spec = cls(name=name, num_classes=num_classes, in_hw=in_hw)
        c, hw, mi = 3, in_hw, 0
        for i, v in enumerate(cfg):
            if v == "M":
                spec.convs[-1].pool = True
                hw //= 2
                mi += 1
                continue
            layer = ConvLayer(idx=mi, cin=c, cin_pad=in_pad if c == 3 else c, cout=v, hw=hw, pool=False,
                              conv_key=f"layers.{mi}", bn_key=f"layers.{mi + 1}")
            spec.convs.append(layer)
            mi += 3
            c = v
        if hw != 1 or c != 512:
            raise ValueError(f"{name} at {in_hw}x{in_hw} does not flatten to 512 features")
        return spec

    def param_names(self) -> List[str]:
        """Reference ``named_parameters()`` order (model.py:18-40)."""
        names = []
        for l in self.convs:
            names += [f"{l.conv_key}.weight", f"{l.conv_key}.bias", f"{l.bn_key}.weight", f"{l.bn_key}.bias"]
        return names + ["fc1.weight", "fc1.bias"]
