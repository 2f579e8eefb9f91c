"""Row-walking 3x3 128 -> 128 conv (csrc/conv_row128.hip, tile 23; not routed by default): the D-22 layer4 BasicBlock convs
without a downsample (lmodels/drn.py:27-29, :49-65), BN folded, optional residual, ReLU.

Oracle: a plain fp32 torch restatement on the same bf16 operands (weights as the packed bf16 rows
with the scale folded).  Tolerance (bf16 perf mode, written here): the output is rounded to bf16
once, and the kernel sums the two K halves in fp32 in its own order, so |gpu - ref| <=
2^-7 |ref| + 1e-3 max|ref|; against the staggered 128-channel tile (tile 19, same operands) the
same bound holds and at least 99 % of the outputs are identical.
"""
from __future__ import annotations

import ctypes

import pytest
import torch
import torch.nn.functional as F

from drnmi import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape,with_res,relu", [
    ((1, 3, 5), True, True), ((2, 17, 70), False, True), ((1, 40, 130), True, False),
    ((3, 33, 200), True, True), ((2, 4, 256), False, True), ((8, 128, 256), True, True),
])
def test_row128_matches_reference(shape, with_res, relu):
    n, h, w = shape
    g = torch.Generator().manual_seed(h * 13 + w)
    x = (torch.randn(n, h, w, 128, generator=g) * 0.7).bfloat16().to(DEV)
    wt = (torch.randn(128, 128, 3, 3, generator=g) * (2.0 / 1152) ** 0.5).to(DEV)
    sc = (torch.rand(128, generator=g) + 0.5).to(DEV)
    sh = (torch.rand(128, generator=g) - 0.5).to(DEV)
    res = (torch.randn(n, h, w, 128, generator=g) * 0.5).bfloat16().to(DEV) if with_res else None
    kw = dict(stride=1, padding=1, dilation=1, relu=relu, fold_scale=True)
    got = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=23, **kw)
    torch.cuda.synchronize()
    wf = (wt * sc.view(-1, 1, 1, 1)).bfloat16().float()
    r = F.conv2d(x.float().permute(0, 3, 1, 2), wf, padding=1) + sh.view(1, -1, 1, 1)
    if with_res:
        r = r + res.float().permute(0, 3, 1, 2)
    if relu:
        r = torch.relu(r)
    r = r.permute(0, 2, 3, 1)
    err = (got.float() - r).abs()
    assert bool((err <= 2 ** -7 * r.abs() + 1e-3 * r.abs().max()).all()), err.max().item()
    if w % 256 == 0:                        # the staggered 128-channel tile takes whole 256-pixel rows
        st = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=19, **kw)
        torch.cuda.synchronize()
        assert (st == got).float().mean().item() >= 0.99


def test_row128_kernel_name():
    a = _lib.ConvArgs()
    a.n, a.h, a.w, a.cin, a.ho, a.wo, a.cout, a.cout_pad = 8, 128, 256, 128, 128, 256, 128, 128
    a.ks, a.stride, a.pad, a.dil, a.k, a.k_pad = 3, 1, 1, 1, 1152, 1152
    a.y_sn, a.y_sp, a.y_sc = 128 * 256 * 128, 128, 1
    a.dtype, a.out_dtype, a.tile, a.algo = _lib.DRNMI_BF16, _lib.DRNMI_BF16, 23, _lib.ALGO_IGEMM
    a.x = a.wgt = a.shift = a.y = 16
    assert _lib.load().drnmi_conv_kernel_name(ctypes.byref(a)).decode() == "conv_row128_kernel<false>"
    a.tile = -1                                 # not routed by default (DRNMI_ROW128=1 routes it)
    assert _lib.load().drnmi_conv_kernel_name(ctypes.byref(a)).decode() == "conv_stag128_kernel"
