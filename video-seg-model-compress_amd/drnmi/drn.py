"""DRN-D backbone definitions: the parameter containers behind DRNSeg.

Mirrors the public surface of the reference lmodels/drn.py (same factory names,
same module attribute names, so state_dict keys are identical and reference
checkpoints load unchanged):

  conv3x3                 lmodels/drn.py:27-29
  BasicBlock              lmodels/drn.py:32-65   (expansion 1)
  Bottleneck              lmodels/drn.py:68-106  (expansion 4)
  DRN (arch 'D')          lmodels/drn.py:109-259 (_make_layer :177-199, _make_conv_layers :201-211)
  drn_d_22 / 38 / 54      lmodels/drn.py:361-393 (also 24 / 40 / 56 / 105 / 107)

These modules hold parameters and describe the graph; they do not compute.  The
forward pass runs through drnmi.engine (HIP kernels via the C-ABI).  Calling a
block's forward directly raises, so nothing can silently fall back to ATen.
"""
from __future__ import annotations

import math

import torch.nn as nn

BatchNorm = nn.BatchNorm2d


def conv3x3(in_planes, out_planes, stride=1, padding=1, dilation=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride,
                     padding=padding, bias=False, dilation=dilation)


class _NoEagerForward:
    def forward(self, *args, **kwargs):  # pragma: no cover - guard
        raise RuntimeError(
            f"{type(self).__name__}.forward is not an eager op in drnmi: run the whole "
            "network through DRNSeg (HIP engine)")


class BasicBlock(_NoEagerForward, nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None,
                 dilation=(1, 1), residual=True):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride, padding=dilation[0], dilation=dilation[0])
        self.bn1 = BatchNorm(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes, padding=dilation[1], dilation=dilation[1])
        self.bn2 = BatchNorm(planes)
        self.downsample = downsample
        self.stride = stride
        self.residual = residual


class Bottleneck(_NoEagerForward, nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None,
                 dilation=(1, 1), residual=True):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.bn1 = BatchNorm(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride,
                               padding=dilation[1], bias=False, dilation=dilation[1])
        self.bn2 = BatchNorm(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = BatchNorm(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


class DRN(_NoEagerForward, nn.Module):
    """Arch 'D' dilated residual network (output stride 8)."""

    def __init__(self, block, layers, num_classes=1000,
                 channels=(16, 32, 64, 128, 256, 512, 512, 512),
                 out_map=False, out_middle=False, pool_size=28, arch="D"):
        super().__init__()
        if arch != "D":
            raise NotImplementedError("drnmi builds the DRN-D family (north_star scope)")
        self.inplanes = channels[0]
        self.out_map = out_map
        self.out_dim = channels[-1]
        self.out_middle = out_middle
        self.arch = arch
        self.block = block

        self.layer0 = nn.Sequential(
            nn.Conv2d(3, channels[0], kernel_size=7, stride=1, padding=3, bias=False),
            BatchNorm(channels[0]),
            nn.ReLU(inplace=True))
        self.layer1 = self._make_conv_layers(channels[0], layers[0], stride=1)
        self.layer2 = self._make_conv_layers(channels[1], layers[1], stride=2)
        self.layer3 = self._make_layer(block, channels[2], layers[2], stride=2)
        self.layer4 = self._make_layer(block, channels[3], layers[3], stride=2)
        self.layer5 = self._make_layer(block, channels[4], layers[4], dilation=2, new_level=False)
        self.layer6 = None if layers[5] == 0 else \
            self._make_layer(block, channels[5], layers[5], dilation=4, new_level=False)
        self.layer7 = None if layers[6] == 0 else \
            self._make_conv_layers(channels[6], layers[6], dilation=2)
        self.layer8 = None if layers[7] == 0 else \
            self._make_conv_layers(channels[7], layers[7], dilation=1)

        if num_classes > 0:
            self.avgpool = nn.AvgPool2d(pool_size)
            self.fc = nn.Conv2d(self.out_dim, num_classes, kernel_size=1, stride=1, padding=0, bias=True)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, BatchNorm):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _make_layer(self, block, planes, blocks, stride=1, dilation=1, new_level=True, residual=True):
        assert dilation == 1 or dilation % 2 == 0
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False),
                BatchNorm(planes * block.expansion))
        first_dil = (1, 1) if dilation == 1 else (dilation // 2 if new_level else dilation, dilation)
        mods = [block(self.inplanes, planes, stride, downsample, dilation=first_dil, residual=residual)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            mods.append(block(self.inplanes, planes, residual=residual, dilation=(dilation, dilation)))
        return nn.Sequential(*mods)

    def _make_conv_layers(self, channels, convs, stride=1, dilation=1):
        mods = []
        for i in range(convs):
            mods.extend([
                nn.Conv2d(self.inplanes, channels, kernel_size=3, stride=stride if i == 0 else 1,
                          padding=dilation, bias=False, dilation=dilation),
                BatchNorm(channels),
                nn.ReLU(inplace=True)])
            self.inplanes = channels
        return nn.Sequential(*mods)


_DRN_D = {
    "drn_d_22": (BasicBlock, [1, 1, 2, 2, 2, 2, 1, 1]),
    "drn_d_24": (BasicBlock, [1, 1, 2, 2, 2, 2, 2, 2]),
    "drn_d_38": (BasicBlock, [1, 1, 3, 4, 6, 3, 1, 1]),
    "drn_d_40": (BasicBlock, [1, 1, 3, 4, 6, 3, 2, 2]),
    "drn_d_54": (Bottleneck, [1, 1, 3, 4, 6, 3, 1, 1]),
    "drn_d_56": (Bottleneck, [1, 1, 3, 4, 6, 3, 2, 2]),
    "drn_d_105": (Bottleneck, [1, 1, 3, 4, 23, 3, 1, 1]),
    "drn_d_107": (Bottleneck, [1, 1, 3, 4, 23, 3, 2, 2]),
}


def _factory(name):
    block, layers = _DRN_D[name]

    def make(pretrained=False, **kwargs):
        if pretrained:
            raise RuntimeError(
                f"{name}(pretrained=True) fetches weights from http://dl.yf.io (reference "
                "lmodels/drn.py:13-24); no network here — load a local state_dict instead")
        return DRN(block, layers, arch="D", **kwargs)

    make.__name__ = name
    return make


drn_d_22 = _factory("drn_d_22")
drn_d_24 = _factory("drn_d_24")
drn_d_38 = _factory("drn_d_38")
drn_d_40 = _factory("drn_d_40")
drn_d_54 = _factory("drn_d_54")
drn_d_56 = _factory("drn_d_56")
drn_d_105 = _factory("drn_d_105")
drn_d_107 = _factory("drn_d_107")

ARCHS = tuple(_DRN_D)
