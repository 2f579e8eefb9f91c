"""Labels-only head on NHWC logits (drnmi_up8_labels_nhwc, csrc/ops.hip up8_labels_oct_kernel<.., true>)
and the seg conv's NHWC fp32 store it reads (conv_tile.h store_tile, 16-B rows): the video path's
DRNSeg.segment (lmodels/drnseg.py:285-299 up + LogSoftmax, seg_video_old_no_plot.py:166 argmax).

Oracle: the NCHW head the engine used before (drnmi_up8_logsoftmax_argmax, itself checked against
the fp32 torch restatement in test_gpu_kernels) -- same values, same per-pixel arithmetic, so the
labels must be identical, including at exact and near ties between classes.
"""
from __future__ import annotations

import ctypes

import pytest
import torch

from drnmi import _lib, drnseg, engine
from drnmi.drnseg import INFO_MEAN, INFO_STD
from drnmi.weights import bilinear_up_kernel

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _up_plane():
    return torch.from_numpy(bilinear_up_kernel(16)).float().contiguous().to(DEV)


@pytest.mark.parametrize("shape", [(1, 1, 1), (2, 5, 7), (3, 17, 33), (8, 128, 256)])
@pytest.mark.parametrize("ldt", [torch.uint8, torch.int64])
def test_labels_nhwc_match_nchw_head(shape, ldt):
    n, h, w = shape
    g = torch.Generator().manual_seed(h * 31 + w)
    logits = torch.randn(n, 19, h, w, generator=g) * 3
    # exact ties and near ties (the fallback path): copy class 4 into class 11 (+ tiny offsets)
    logits[:, 11] = logits[:, 4]
    logits[:, 12, ::2] = logits[:, 4, ::2] + 2 ** -20
    logits = logits.to(DEV)
    cs = 20
    nhwc = torch.full((n, h, w, cs), float("nan"), device=DEV)
    nhwc[..., :19] = logits.permute(0, 2, 3, 1)
    up = _up_plane()
    code = _lib.DRNMI_I64 if ldt == torch.int64 else _lib.DRNMI_U8
    a = torch.empty(n, 8 * h, 8 * w, dtype=ldt, device=DEV)
    b = torch.empty_like(a)
    lib = _lib.load()
    st = ctypes.c_void_p(_lib.stream_ptr())
    _lib.check(lib.drnmi_up8_logsoftmax_argmax(logits.data_ptr(), up.data_ptr(), None, a.data_ptr(), code, n, 19,
                                               h, w, st), "nchw head")
    _lib.check(lib.drnmi_up8_labels_nhwc(nhwc.data_ptr(), cs, up.data_ptr(), b.data_ptr(), code, n, 19, h, w, st),
               "nhwc head")
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def _smooth_logits(n, h, w, seed):
    """Spatially smooth logits (bilinearly enlarged coarse noise): large same-argmax regions, the
    fast path of up8_labels_tile_kernel, with engineered top-2 margins around its guard."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(seed)
    coarse = torch.randn(n, 19, h // 6 + 2, w // 6 + 2, generator=g) * 4
    x = F.interpolate(coarse, size=(h, w), mode="bilinear", align_corners=True)
    top2 = torch.topk(x, 2, dim=1)
    # every 7th pixel: runner-up moved to best - d with d around the guard (2^-16 .. 2^-13)
    sel = torch.zeros(h, w, dtype=torch.bool)
    sel.view(-1)[::7] = True
    d = torch.tensor([2 ** -17, 2 ** -16, 1.1 * 2 ** -16, 2 ** -15, 1.5 * 2 ** -15, 2 ** -13, 2 ** -12])
    dd = d[torch.arange(h * w) % len(d)].view(h, w)
    i2 = top2.indices[:, 1]
    newv = top2.values[:, 0] - dd
    x.scatter_(1, i2.unsqueeze(1), torch.where(sel, newv, top2.values[:, 1]).unsqueeze(1))
    return x


@pytest.mark.parametrize("shape", [(2, 40, 64), (1, 128, 256), (3, 9, 130)])
@pytest.mark.parametrize("up", ["bilinear", "random", "negative"])
@pytest.mark.parametrize("seg2", [False, True])
def test_labels_fast_path_identical(shape, up, seg2):
    """up8_labels_tile_kernel (NHWC / SEG2 entry points): windows whose 4 taps share an argmax with a
    margin above the guard are written without per-pixel work; labels must equal the oct head's
    (NCHW) bit for bit, with margins engineered around the guard, non-bilinear up weights and a
    negative weight (which disables the fast path)."""
    n, h, w = shape
    logits = _smooth_logits(n, h, w, h * 7 + w + (1 if seg2 else 0))
    if up == "bilinear":
        upw = _up_plane()
    else:
        g = torch.Generator().manual_seed(5)
        upw = (torch.rand(16, 16, generator=g) * 0.3).float()
        if up == "negative":
            upw[3, 5] = -0.01
        upw = upw.contiguous().to(DEV)
    cs = 20
    lib = _lib.load()
    st = ctypes.c_void_p(_lib.stream_ptr())
    a = torch.empty(n, 8 * h, 8 * w, dtype=torch.uint8, device=DEV)
    b = torch.empty_like(a)
    if seg2:   # the head sums (bias + partial 0) + partial 1: feed the NCHW head that same sum
        g = torch.Generator().manual_seed(9)
        bias = torch.randn(20, generator=g) * 0.1
        p0 = torch.randn(n, h, w, cs, generator=g)
        p1 = logits.permute(0, 2, 3, 1).contiguous()
        p1 = torch.cat([p1, torch.zeros(n, h, w, 1)], dim=3) - p0
        summed = ((bias.view(1, 1, 1, cs) + p0) + p1)[..., :19].permute(0, 3, 1, 2).contiguous().to(DEV)
        parts = torch.stack([p0, p1]).contiguous().to(DEV)
        bias = bias.to(DEV)
        _lib.check(lib.drnmi_up8_logsoftmax_argmax(summed.data_ptr(), upw.data_ptr(), None, a.data_ptr(),
                                                   _lib.DRNMI_U8, n, 19, h, w, st), "nchw head")
        _lib.check(lib.drnmi_up8_labels_seg2(parts.data_ptr(), cs, bias.data_ptr(), upw.data_ptr(), b.data_ptr(),
                                             _lib.DRNMI_U8, n, 19, h, w, st), "seg2 head")
    else:
        lg = logits.to(DEV)
        nhwc = torch.full((n, h, w, cs), float("nan"), device=DEV)
        nhwc[..., :19] = lg.permute(0, 2, 3, 1)
        _lib.check(lib.drnmi_up8_logsoftmax_argmax(lg.data_ptr(), upw.data_ptr(), None, a.data_ptr(), _lib.DRNMI_U8,
                                                   n, 19, h, w, st), "nchw head")
        _lib.check(lib.drnmi_up8_labels_nhwc(nhwc.data_ptr(), cs, upw.data_ptr(), b.data_ptr(), _lib.DRNMI_U8,
                                             n, 19, h, w, st), "nhwc head")
    torch.cuda.synchronize()
    assert torch.equal(a, b), f"{int((a != b).sum())} labels differ"


@pytest.mark.parametrize("amp", [3e-5, 1e-3, 0.05])
@pytest.mark.parametrize("seg2", [False, True])
def test_labels_candidate_pruning_identical(amp, seg2):
    """The slow blocks' candidate-class pruning (a class is skipped when its largest tap logit sits a
    guard below the best smallest one, up8_labels_tile_kernel): labels equal the oct head's bit for
    bit when the logits are compressed so that margins between classes are near the 2^-16 tie rule
    and the pruning guard (amp 3e-5: most blocks tie or nearly tie; 1e-3 / 0.05: a few candidates per
    block, some classes close to the threshold)."""
    import torch.nn.functional as F
    n, h, w = 2, 24, 40
    g = torch.Generator().manual_seed(int(amp * 1e6) + (7 if seg2 else 0))
    coarse = torch.randn(n, 19, h // 4 + 2, w // 4 + 2, generator=g)
    logits = (F.interpolate(coarse, size=(h, w), mode="bilinear", align_corners=True) * amp).contiguous()
    upw = _up_plane()
    cs = 20
    lib = _lib.load()
    st = ctypes.c_void_p(_lib.stream_ptr())
    a = torch.empty(n, 8 * h, 8 * w, dtype=torch.uint8, device=DEV)
    b = torch.empty_like(a)
    lg = logits.to(DEV)
    _lib.check(lib.drnmi_up8_logsoftmax_argmax(lg.data_ptr(), upw.data_ptr(), None, a.data_ptr(), _lib.DRNMI_U8,
                                               n, 19, h, w, st), "nchw head")
    if seg2:   # partial 0 = 0, bias = 0: the SEG2 sum (0 + 0) + p1 is p1 exactly
        parts = torch.zeros(2, n, h, w, cs, device=DEV)
        parts[1, ..., :19] = lg.permute(0, 2, 3, 1)
        bias = torch.zeros(cs, device=DEV)
        _lib.check(lib.drnmi_up8_labels_seg2(parts.data_ptr(), cs, bias.data_ptr(), upw.data_ptr(), b.data_ptr(),
                                             _lib.DRNMI_U8, n, 19, h, w, st), "seg2 head")
    else:
        nhwc = torch.zeros(n, h, w, cs, device=DEV)
        nhwc[..., :19] = lg.permute(0, 2, 3, 1)
        _lib.check(lib.drnmi_up8_labels_nhwc(nhwc.data_ptr(), cs, upw.data_ptr(), b.data_ptr(), _lib.DRNMI_U8,
                                             n, 19, h, w, st), "nhwc head")
    torch.cuda.synchronize()
    assert torch.equal(a, b), f"{int((a != b).sum())} labels differ"


def test_labels_nhwc_rejects_bad_args():
    lib = _lib.load()
    x = torch.zeros(1, 4, 4, 20, device=DEV)
    up = _up_plane()
    lab = torch.empty(1, 32, 32, dtype=torch.uint8, device=DEV)
    st = ctypes.c_void_p(_lib.stream_ptr())
    assert lib.drnmi_up8_labels_nhwc(x.data_ptr(), 18, up.data_ptr(), lab.data_ptr(), _lib.DRNMI_U8, 1, 19, 4, 4, st) == -1
    assert lib.drnmi_up8_labels_nhwc(x.data_ptr(), 20, up.data_ptr(), lab.data_ptr(), _lib.DRNMI_U8, 1, 21, 4, 4, st) == -2


@pytest.mark.parametrize("arch,hw", [("drn_d_22", (64, 128)), ("drn_d_22", (96, 200)), ("drn_d_38", (64, 96))])
def test_segment_labels_nhwc_identical(arch, hw):
    m = drnseg.build(arch, 19, seed=3, device=torch.device(DEV), precision="bf16").eval()
    g = torch.Generator(device=DEV).manual_seed(9)
    frames = torch.randint(0, 256, (2, *hw, 3), dtype=torch.uint8, device=DEV, generator=g)
    old = engine.LABELS_NHWC, engine.SEG_FUSE
    try:
        engine.SEG_FUSE = False
        engine.LABELS_NHWC = False
        ref = m.segment(frames, INFO_MEAN, INFO_STD, False).clone()
        engine.LABELS_NHWC = True
        got = m.segment(frames, INFO_MEAN, INFO_STD, False)
        plans = list(m._plans.values())
        assert plans and all(p.labels_path() == "nhwc" for p in plans), "the bf16 plan must take the NHWC logits path"
    finally:
        engine.LABELS_NHWC, engine.SEG_FUSE = old
    assert torch.equal(ref, got)


@pytest.mark.parametrize("arch,n", [("drn_d_22", 1), ("drn_d_22", 2), ("drn_d_38", 1), ("drn_d_54", 1)])
def test_segment_seg_fused_into_last_conv(arch, n):
    """DRN-D at 1024 x 2048 (layer8 on the staggered tile): the seg classifier folded into layer8's
    epilogue (drnmi_conv_stag_seg) + the SEG2 head against the separate seg conv + NHWC head.  The
    logits differ only by fp32 summation order (two 256-channel partials): bound 2^-16 max|logit|;
    labels may flip only at near ties.  Every architecture whose plan routes the fusion is covered
    (D-38 / D-54 share D-22's 512-channel layer8)."""
    m = drnseg.build(arch, 19, seed=4, device=torch.device(DEV), precision="bf16").eval()
    g = torch.Generator(device=DEV).manual_seed(2)
    frames = torch.randint(0, 256, (n, 1024, 2048, 3), dtype=torch.uint8, device=DEV, generator=g)
    old = engine.SEG_FUSE
    try:
        engine.SEG_FUSE = False
        ref = m.segment(frames, INFO_MEAN, INFO_STD, False).clone()
        plan = next(iter(m._plans.values()))
        logits = plan.bufs["logits_nhwc"].view(n, 128, 256, 20)[..., :19].clone()
        engine.SEG_FUSE = True
        plan.refresh_weight_ptrs()                     # re-derives the labels path with the flag on
        assert plan.labels_path() == "seg2"
        got = m.segment(frames, INFO_MEAN, INFO_STD, False)
    finally:
        engine.SEG_FUSE = old
    part = plan.bufs["seg_part"].view(2, n, 128, 256, 20)
    seg = plan.packed.graph.nodes[plan.seg_idx]
    fused = (seg.shift[:19].view(1, 1, 1, 19) + part[0, ..., :19]) + part[1, ..., :19]
    err = (fused - logits).abs().max().item()
    assert err <= 2 ** -16 * logits.abs().max().item() + 1e-6, err
    agree = (got == ref).float().mean().item()
    print(f"{arch} seg-fused labels agreement {agree:.6f}, logits max |diff| {err:.3e}")
    assert agree >= 0.9995


@pytest.mark.parametrize("n", [1, 2])
def test_seg_fused_w1_matches_stag_bit_identical(n):
    """The seg-fused layer8 launch on the one-wave-per-SIMD tile (conv_w1_seg_kernel, the default)
    == the staggered tile's (conv_stag_seg_kernel, forced with tile 19): same K order and MFMA order
    per accumulator, the same seg MFMAs per partial and the same wc 0 + wc 1 order, so the partial
    logits are equal bit for bit."""
    m = drnseg.build("drn_d_22", 19, seed=7, device=torch.device(DEV), precision="bf16").eval()
    g = torch.Generator(device=DEV).manual_seed(5)
    frames = torch.randint(0, 256, (n, 1024, 2048, 3), dtype=torch.uint8, device=DEV, generator=g)
    got = m.segment(frames, INFO_MEAN, INFO_STD, False).clone()
    plan = next(iter(m._plans.values()))
    assert plan.labels_path() == "seg2"
    j = plan.seg_fused["conv"]
    lib = _lib.load()
    assert lib.drnmi_conv_stag_seg_kernel_name(ctypes.byref(plan.args[j])).decode() == "conv_w1_seg_kernel"
    part_w1 = plan.bufs["seg_part"].clone()
    plan.args[j].tile = 19
    try:
        assert lib.drnmi_conv_stag_seg_kernel_name(ctypes.byref(plan.args[j])).decode() == "conv_stag_seg_kernel"
        ref = m.segment(frames, INFO_MEAN, INFO_STD, False)
        part_stag = plan.bufs["seg_part"].clone()
    finally:
        plan.args[j].tile = -1
    torch.cuda.synchronize()
    assert torch.equal(part_w1, part_stag)
    assert torch.equal(got, ref)


def test_seg_fused_int8_w1_matches_stag():
    """int8 nets: the seg-fused layer8 launch on the one-wave-per-SIMD int8 tile
    (conv_w1_i8_seg_kernel, the default) == the staggered one (conv_i8_stag_seg_kernel, tile 19):
    integer partials, so equal bit for bit."""
    m = drnseg.build("drn_d_22", 19, seed=8, device=torch.device(DEV))
    g = torch.Generator(device=DEV).manual_seed(13)
    frames = torch.randint(0, 256, (2, 256, 2048, 3), dtype=torch.uint8, device=DEV, generator=g)
    m.calibrate_int8(frames[:1])
    m.set_precision("int8")
    got = m.segment(frames, INFO_MEAN, INFO_STD, False).clone()
    plan = [p for k, p in m._plans.items() if k[0] == "int8"][0]
    assert plan.labels_path() == "seg2" and plan.seg_fused["i8"]
    j = plan.seg_fused["conv"]
    lib = _lib.load()
    assert lib.drnmi_conv_stag_seg_kernel_name(ctypes.byref(plan.args[j])).decode() == "conv_w1_i8_seg_kernel"
    part_w1 = plan.bufs["seg_part"].clone()
    plan.args[j].tile = 19
    try:
        assert lib.drnmi_conv_stag_seg_kernel_name(ctypes.byref(plan.args[j])).decode() == "conv_i8_stag_seg_kernel"
        ref = m.segment(frames, INFO_MEAN, INFO_STD, False)
        part_stag = plan.bufs["seg_part"].clone()
    finally:
        plan.args[j].tile = -1
    torch.cuda.synchronize()
    assert torch.equal(part_w1, part_stag)
    assert torch.equal(got, ref)


def test_segment_labels_nhwc_identical_int8():
    """int8 nets (C5): the int8 seg conv writes the same fp32 values as NHWC rows (store_tile_i8's
    16-B path) -- labels identical to the NCHW-planes head."""
    m = drnseg.build("drn_d_22", 19, seed=5, device=torch.device(DEV))
    g = torch.Generator(device=DEV).manual_seed(11)
    frames = torch.randint(0, 256, (2, 128, 256, 3), dtype=torch.uint8, device=DEV, generator=g)
    m.calibrate_int8(frames)
    m.set_precision("int8")
    old = engine.LABELS_NHWC
    try:
        engine.LABELS_NHWC = False
        ref = m.segment(frames, INFO_MEAN, INFO_STD, False).clone()
        engine.LABELS_NHWC = True
        got = m.segment(frames, INFO_MEAN, INFO_STD, False)
        plans = [p for k, p in m._plans.items() if k[0] == "int8"]
        assert plans and all(p.labels_path() == "nhwc" for p in plans), "the int8 plan must take the NHWC logits path"
    finally:
        engine.LABELS_NHWC = old
    assert torch.equal(ref, got)


def test_segment_seg_fused_int8_exact():
    """int8 nets (C5): the int8 seg conv folded into layer8's int8 epilogue (conv_i8_stag_seg_kernel:
    the int8 values layer8 would store times the int8 seg weights, int32 partials per 256-channel
    block) + drnmi_up8_labels_seg2_i8.  Integer sums are exact, so (float)(p0 + p1) * scale + shift
    must equal the separate int8 seg conv's fp32 logits bit for bit, and the labels must be equal."""
    m = drnseg.build("drn_d_22", 19, seed=6, device=torch.device(DEV))
    g = torch.Generator(device=DEV).manual_seed(12)
    frames = torch.randint(0, 256, (2, 256, 2048, 3), dtype=torch.uint8, device=DEV, generator=g)
    m.calibrate_int8(frames[:1])
    m.set_precision("int8")
    old = engine.SEG_FUSE
    try:
        engine.SEG_FUSE = False
        ref = m.segment(frames, INFO_MEAN, INFO_STD, False).clone()
        plan = [p for k, p in m._plans.items() if k[0] == "int8"][0]
        assert plan.labels_path() == "nhwc"
        lh, lw = plan.shapes["logits"]
        logits = plan.bufs["logits_nhwc"].view(2, lh, lw, 20)[..., :19].clone()
        engine.SEG_FUSE = True
        plan.refresh_weight_ptrs()
        assert plan.labels_path() == "seg2" and plan.seg_fused["i8"]
        got = m.segment(frames, INFO_MEAN, INFO_STD, False)
    finally:
        engine.SEG_FUSE = old
    torch.cuda.synchronize()
    part = plan.bufs["seg_part"].view(2, 2, lh, lw, 20)
    seg = plan.packed.graph.nodes[plan.seg_idx]
    acc = (part[0] + part[1])[..., :19]
    rebuilt = acc.float() * seg.scale[:19].view(1, 1, 1, 19)
    rebuilt = rebuilt + seg.shift[:19].view(1, 1, 1, 19)
    assert torch.equal(rebuilt, logits)
    assert torch.equal(got, ref)
