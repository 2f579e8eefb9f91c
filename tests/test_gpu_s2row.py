"""Row-walking stride-2 3x3 conv (csrc/conv_s2row.hip, tile id 20): the BasicBlock conv1 of DRN-D
layer3.0 (32 -> 64) and layer4.0 (64 -> 128), lmodels/drn.py:27-29 conv3x3 + :49-52 (stride 2),
BN folded (scale into the bf16 weights, shift as the accumulator start), ReLU.

Oracle: the conv_big BK-32 / BK-64 tiles the engine used for these convs before -- same packed
weights, same per-accumulator K order and MFMA, same start value and epilogue -- so the outputs
must be bit-identical (torch.equal), on ragged shapes (image edges, strips past the last column,
odd heights) and with ReLU off.  A plain fp32 torch conv bounds both (bf16 tolerance, written
below) so the pair cannot agree on a wrong answer.
"""
from __future__ import annotations

import ctypes

import pytest
import torch
import torch.nn.functional as F

from drnmi import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _args(x, wpk, k, sh, y, cin, cout, relu, tile):
    n, h, w, _ = x.shape
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    a = _lib.ConvArgs()
    a.x, a.wgt, a.scale, a.shift, a.res, a.y = x.data_ptr(), wpk.data_ptr(), None, sh.data_ptr(), None, y.data_ptr()
    a.y_sn, a.y_sp, a.y_sc = ho * wo * cout, cout, 1
    a.n, a.h, a.w, a.cin = n, h, w, cin
    a.ho, a.wo, a.cout, a.cout_pad = ho, wo, cout, wpk.shape[0]
    a.ks, a.stride, a.pad, a.dil = 3, 2, 1, 1
    a.k, a.k_pad = k, wpk.shape[1]
    a.relu, a.dtype, a.out_dtype, a.tile, a.algo = 1 if relu else 0, _lib.DRNMI_BF16, _lib.DRNMI_BF16, tile, _lib.ALGO_IGEMM
    return a


@pytest.mark.parametrize("cin", [32, 64])
@pytest.mark.parametrize("shape,relu", [
    ((1, 5, 9), True), ((2, 17, 70), True), ((1, 40, 130), False), ((3, 64, 248), True),
    ((2, 129, 257), True), ((8, 512, 1024), True),
])
def test_s2row_bit_identical_to_conv_big(cin, shape, relu):
    n, h, w = shape
    if cin == 64:                                   # layer4.0 conv1 runs at half layer3.0's size
        h, w = (h + 1) // 2, (w + 1) // 2
    cout = 2 * cin
    g = torch.Generator().manual_seed(11 + cin + h)
    x = (torch.randn(n, h, w, cin, generator=g) * 0.7).bfloat16().to(DEV)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (2 / (9 * cin)) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    shv = torch.randn(cout, generator=g) * 0.3
    wpk, k = ops.pack_conv_weight((wt * sc.view(-1, 1, 1, 1)).to(DEV), cin, torch.bfloat16)
    sh = torch.zeros(wpk.shape[0], device=DEV)
    sh[:cout] = shv.to(DEV)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    lib = _lib.load()
    outs = {}
    for tile in (-1, 20, 6 if cin == 32 else 7):    # auto, forced s2row, conv_big BK-32 / BK-64 64-wide tile
        y = torch.full((n, ho, wo, cout), float("nan"), device=DEV, dtype=torch.bfloat16)
        a = _args(x, wpk, k, sh, y, cin, cout, relu, tile)
        name = lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode()
        if tile in (-1, 20):
            assert name.startswith(f"conv_s2row_kernel<{cin}, "), name
        else:
            assert name.startswith("conv_big_kernel<3, 64, 1"), name
        _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())), "s2row")
        torch.cuda.synchronize()
        outs[tile] = y
    ref_tile = 6 if cin == 32 else 7
    assert not torch.isnan(outs[20].float()).any()
    assert torch.equal(outs[-1], outs[20])
    assert torch.equal(outs[20], outs[ref_tile]), \
        f"{int((outs[20] != outs[ref_tile]).sum())} of {outs[20].numel()} differ"
    # fp32 torch restatement (bf16 tolerance: the folded weights and the output are bf16-rounded)
    if n * h * w <= 3 * 64 * 248:
        wf = wpk[:cout, :k].float().view(cout, 3, 3, cin).permute(0, 3, 1, 2)
        r = F.conv2d(x.float().permute(0, 3, 1, 2), wf, stride=2, padding=1) + sh[:cout].view(1, -1, 1, 1)
        if relu:
            r = torch.relu(r)
        r = r.permute(0, 2, 3, 1)
        err = (outs[20].float() - r).abs()
        assert bool((err <= 2 ** -7 * r.abs() + 1e-3 * r.abs().max()).all())


def test_s2row_refuses_other_shapes():
    x = torch.zeros(1, 8, 8, 64, device=DEV, dtype=torch.bfloat16)
    wpk, k = ops.pack_conv_weight(torch.zeros(64, 64, 3, 3, device=DEV), 64, torch.bfloat16)   # 64 -> 64: not taken
    sh = torch.zeros(wpk.shape[0], device=DEV)
    y = torch.empty(1, 4, 4, 64, device=DEV, dtype=torch.bfloat16)
    a = _args(x, wpk, k, sh, y, 64, 64, True, 20)
    lib = _lib.load()
    assert lib.drnmi_conv_kernel_name(ctypes.byref(a)) is None
    assert lib.drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())) == -2


@pytest.mark.parametrize("shape", [(1, 3, 5), (2, 17, 70), (1, 40, 130), (3, 33, 200), (8, 256, 512)])
def test_s1x2row_bit_identical_to_halo(shape):
    """Layer3.0 conv2 + the folded 1x1 stride-2 downsample (conv_s1x2row_kernel, tile 21) against
    conv_halo's x2 form (tile 17): same packed [W2 | W_ds | 0] rows, K order, start and epilogue."""
    n, h, w = shape
    h2, w2 = 2 * h, 2 * w
    g = torch.Generator().manual_seed(h * 7 + w)
    x = (torch.randn(n, h, w, 64, generator=g) * 0.7).bfloat16().to(DEV)
    x2 = (torch.randn(n, h2, w2, 32, generator=g) * 0.7).bfloat16().to(DEV)
    wt = (torch.randn(64, 64, 3, 3, generator=g) / 24).bfloat16()
    wd = (torch.randn(64, 32, 1, 1, generator=g) / 5.7).bfloat16()
    kp = 640
    wpk = torch.zeros(128, kp, dtype=torch.bfloat16)
    wpk[:64, :576] = wt.permute(0, 2, 3, 1).reshape(64, 576)
    wpk[:64, 576:608] = wd.reshape(64, 32)
    wpk = wpk.to(DEV)
    sh = torch.zeros(128, device=DEV)
    sh[:64] = (torch.randn(64, generator=g) * 0.3).to(DEV)
    lib = _lib.load()
    outs = {}
    for tile in (-1, 21, 17):
        y = torch.full((n, h, w, 64), float("nan"), device=DEV, dtype=torch.bfloat16)
        a = _lib.ConvArgs()
        a.x, a.wgt, a.scale, a.shift, a.res, a.y = x.data_ptr(), wpk.data_ptr(), None, sh.data_ptr(), None, y.data_ptr()
        a.y_sn, a.y_sp, a.y_sc = h * w * 64, 64, 1
        a.n, a.h, a.w, a.cin, a.ho, a.wo, a.cout, a.cout_pad = n, h, w, 64, h, w, 64, 128
        a.ks, a.stride, a.pad, a.dil = 3, 1, 1, 1
        a.k, a.k_pad = 608, kp
        a.relu, a.dtype, a.out_dtype, a.tile, a.algo = 1, _lib.DRNMI_BF16, _lib.DRNMI_BF16, tile, _lib.ALGO_IGEMM
        a.x2, a.cin2, a.h2, a.w2, a.stride2 = x2.data_ptr(), 32, h2, w2, 2
        name = lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode()
        assert name == ("conv_halo_kernel<64, 1, 64>" if tile == 17 else "conv_s1x2row_kernel"), name
        _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())), "s1x2row")
        torch.cuda.synchronize()
        outs[tile] = y
    assert not torch.isnan(outs[21].float()).any()
    assert torch.equal(outs[-1], outs[21])
    assert torch.equal(outs[21], outs[17]), f"{int((outs[21] != outs[17]).sum())} of {outs[21].numel()} differ"
    if n * h * w <= 3 * 33 * 200:
        r = F.conv2d(x.float().permute(0, 3, 1, 2), wt.float().to(DEV), padding=1) \
            + F.conv2d(x2.float().permute(0, 3, 1, 2), wd.float().to(DEV), stride=2) + sh[:64].view(1, -1, 1, 1)
        r = torch.relu(r).permute(0, 2, 3, 1)
        err = (outs[21].float() - r).abs()
        assert bool((err <= 2 ** -7 * r.abs() + 1e-3 * r.abs().max()).all())
