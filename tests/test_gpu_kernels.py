"""Per-kernel parity on the GPU: HIP kernels vs the CPU fp32 oracle (torch CPU ops).

Tolerances (written here, per precision):
  fp32 parity mode: |y - ref| <= 2e-5 * max|ref| + 1e-6   (exact-fp32 MFMA, different sum order)
  bf16 perf mode  : reference computed on bf16-rounded operands; |y - ref| <= 1.5e-2 * max|ref|
                    (bf16 output rounding 2^-9 plus fp32 accumulation-order differences)
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from drnmi import _lib, ops
from oracle import drn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"

CONV_CASES = [
    # cin, cout, ks, stride, dil, h, w, residual, relu
    (16, 16, 3, 1, 1, 37, 45, False, True),
    (16, 32, 3, 2, 1, 40, 52, False, True),
    (32, 64, 3, 2, 1, 33, 31, False, True),
    (64, 64, 3, 1, 1, 20, 24, True, True),
    (32, 64, 1, 2, 1, 33, 31, False, False),
    (128, 256, 3, 1, 2, 16, 20, False, True),
    (256, 256, 3, 1, 2, 12, 16, True, True),
    (256, 512, 3, 1, 4, 16, 16, False, True),
    (512, 512, 3, 1, 4, 11, 13, True, True),
    (512, 512, 3, 1, 2, 16, 32, False, True),
    (512, 19, 1, 1, 1, 16, 32, False, False),
    (64, 256, 1, 1, 1, 15, 17, True, True),    # bottleneck conv3
    (256, 64, 1, 1, 1, 15, 17, False, True),   # bottleneck conv1
]


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def _ref_conv(x, w, sc, sh, res, stride, pad, dil, relu):
    y = F.conv2d(x, w, stride=stride, padding=pad, dilation=dil)
    y = y * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("case", range(len(CONV_CASES)))
def test_conv_bn_act(case, prec):
    cin, cout, ks, stride, dil, h, w, has_res, relu = CONV_CASES[case]
    n = 2
    pad = dil * (ks // 2)
    x = _rand((n, cin, h, w), 1 + case)
    wt = _rand((cout, cin, ks, ks), 100 + case, (2.0 / (ks * ks * cout)) ** 0.5)
    sc = torch.rand(cout, generator=torch.Generator().manual_seed(7)) + 0.5
    sh = torch.rand(cout, generator=torch.Generator().manual_seed(8)) - 0.5
    ho = (h + 2 * pad - dil * (ks - 1) - 1) // stride + 1
    wo = (w + 2 * pad - dil * (ks - 1) - 1) // stride + 1
    res = _rand((n, cout, ho, wo), 200 + case) if has_res else None
    dt = torch.float32 if prec == "fp32" else torch.bfloat16
    if prec == "bf16":
        x, wt = x.bfloat16().float(), wt.bfloat16().float()
        res = res.bfloat16().float() if res is not None else None
    ref = _ref_conv(x, wt, sc, sh, res, stride, pad, dil, relu)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, dt)
    rd = res.permute(0, 2, 3, 1).contiguous().to(DEV, dt) if res is not None else None
    y = ops.conv2d_bn_act(xd, wt.to(DEV), sc.to(DEV), sh.to(DEV), rd, stride, pad, dil, relu)
    torch.cuda.synchronize()
    got = y.float().permute(0, 3, 1, 2).cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    if prec == "fp32":
        assert err <= 2e-5 * scale + 1e-6, f"max err {err} (scale {scale})"
    else:
        # bf16 operands are exact inputs here (pre-rounded), products exact, fp32 accumulation and
        # epilogue: the only errors are the output's bf16 rounding (<= 2^-9 |v|) and the fp32
        # summation order, so elementwise |got - ref| <= 2^-8 |ref| + 1e-3 max|ref|
        bound = 2.0 ** -8 * ref.abs() + 1e-3 * scale
        worst = ((got - ref).abs() - bound).max().item()
        assert worst <= 0, f"max err {err} (scale {scale}), bound exceeded by {worst}"


@pytest.mark.parametrize("tile", [0, 1, 2, 3])
def test_conv_all_tiles(tile):
    n, cin, cout, h, w = 1, 64, 128, 19, 23
    x = _rand((n, cin, h, w), 5)
    wt = _rand((cout, cin, 3, 3), 6, 0.05)
    ref = F.conv2d(x, wt, padding=2, dilation=2)
    y = ops.conv2d_bn_act(x.permute(0, 2, 3, 1).contiguous().to(DEV), wt.to(DEV), padding=2, dilation=2,
                          tile=tile)
    got = y.permute(0, 3, 1, 2).cpu()
    assert (got - ref).abs().max().item() <= 2e-5 * ref.abs().max().item() + 1e-6


def test_stem_7x7_padded_input():
    """layer0: 7x7 conv over 3 channels stored with channel stride 8 (zero pad)."""
    x = _rand((2, 3, 41, 67), 9)
    wt = _rand((16, 3, 7, 7), 10, 0.1)
    ref = F.conv2d(x, wt, padding=3)
    xd = ops.nchw_to_nhwc(x.to(DEV), 8, torch.float32)
    y = ops.conv2d_bn_act(xd, wt.to(DEV), padding=3)
    got = y.permute(0, 3, 1, 2).cpu()
    assert (got - ref).abs().max().item() <= 2e-5 * ref.abs().max().item() + 1e-6


def test_seg_conv_writes_nchw_fp32_logits():
    x = _rand((2, 512, 9, 14), 11)
    wt = _rand((19, 512, 1, 1), 12, 0.05)
    b = _rand((19,), 13, 0.1)
    ref = F.conv2d(x, wt, b)
    y = ops.conv2d_bn_act(x.permute(0, 2, 3, 1).contiguous().to(DEV), wt.to(DEV), None, b.to(DEV),
                          out_nchw_fp32=True)
    assert y.shape == (2, 19, 9, 14)
    assert (y.cpu() - ref).abs().max().item() <= 2e-5 * ref.abs().max().item() + 1e-6


@pytest.mark.parametrize("ysp", [20, 28, 64])
def test_fp32_nhwc_store_stays_in_its_channels(ysp):
    """bf16 in, fp32 NHWC out (conv_big's 16-B fp32 epilogue): rows of ysp floats.  ysp 20 =
    round_up(19, 4) is the labels head's padded-row layout; 28 / 64 are channel slices of a wider
    buffer, whose channels past cout must keep their sentinel."""
    n, h, w, cin, cout = 2, 9, 14, 512, 19
    g = torch.Generator().manual_seed(90 + ysp)
    x = torch.randn(n, h, w, cin, generator=g).bfloat16()
    wt = torch.randn(cout, cin, 1, 1, generator=g) * 0.05
    b = torch.randn(cout, generator=g) * 0.1
    wpk, k = ops.pack_conv_weight(wt.to(DEV), cin, torch.bfloat16)
    sc = torch.ones(wpk.shape[0], device=DEV)
    sh = torch.zeros(wpk.shape[0], device=DEV)
    sh[:cout] = b.to(DEV)
    y = torch.full((n, h, w, ysp), 7.0, device=DEV)
    xd = x.to(DEV)
    a = _lib.ConvArgs()
    a.x, a.wgt, a.scale, a.shift, a.res, a.y = xd.data_ptr(), wpk.data_ptr(), sc.data_ptr(), sh.data_ptr(), None, \
        y.data_ptr()
    a.y_sn, a.y_sp, a.y_sc = h * w * ysp, ysp, 1
    a.n, a.h, a.w, a.cin, a.ho, a.wo, a.cout, a.cout_pad = n, h, w, cin, h, w, cout, wpk.shape[0]
    a.ks, a.stride, a.pad, a.dil, a.k, a.k_pad, a.relu = 1, 1, 0, 1, k, wpk.shape[1], 0
    a.dtype, a.out_dtype, a.tile, a.algo = _lib.DRNMI_BF16, _lib.DRNMI_F32, -1, _lib.ALGO_IGEMM
    _lib.check(_lib.load().drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())), "conv")
    torch.cuda.synchronize()
    got = y.cpu()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wt.bfloat16().float(), b).permute(0, 2, 3, 1)
    assert (got[..., :cout] - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    if ysp > 20:
        assert bool((got[..., cout:] == 7.0).all())


def test_frame_ingest_bit_exact(golden_forward):
    for case in ["d22_1x64x128", "d22_1x300x300"]:
        frames = torch.from_numpy(golden_forward[case + "/frames"]).to(DEV)
        out = ops.frame_ingest(frames, O.INFO_MEAN, O.INFO_STD, dtype=torch.float32)
        got = out[..., :3].permute(0, 3, 1, 2).cpu().numpy()
        np.testing.assert_array_equal(got, golden_forward[case + "/input"])
        assert torch.count_nonzero(out[..., 3:]).item() == 0


def test_frame_ingest_bgr_swap():
    fr = torch.randint(0, 256, (1, 5, 7, 3), dtype=torch.uint8)
    a = ops.frame_ingest(fr.to(DEV), O.INFO_MEAN, O.INFO_STD, bgr=True)
    b = ops.frame_ingest(fr.flip(-1).contiguous().to(DEV), O.INFO_MEAN, O.INFO_STD, bgr=False)
    torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("h,w", [(8, 16), (38, 38), (5, 3), (1, 1)])
def test_up8_logsoftmax_argmax(h, w):
    from drnmi.weights import bilinear_up_kernel
    c = 19
    logits = _rand((2, c, h, w), 21, 3.0)
    upw = torch.from_numpy(bilinear_up_kernel(16))
    sd = {"up.weight": upw.expand(c, 1, 16, 16).contiguous()}
    ref = O.up_logsoftmax(sd, logits)
    lp, lab = ops.up8_logsoftmax_argmax(logits.to(DEV), upw.to(DEV))
    assert lp.shape == ref.shape
    assert (lp.cpu() - ref).abs().max().item() <= 2e-5
    ref_lab = O.labels_of(ref)
    srt = ref.sort(dim=1).values
    margin = srt[:, -1] - srt[:, -2]
    diff = lab.cpu() != ref_lab
    assert not bool((diff & (margin > 1e-5)).any())
    _, lab8 = ops.up8_logsoftmax_argmax(logits.to(DEV), upw.to(DEV), want_logprobs=False,
                                        label_dtype=torch.uint8)
    assert torch.equal(lab8.cpu().long(), lab.cpu())
    _, lab64 = ops.up8_logsoftmax_argmax(logits.to(DEV), upw.to(DEV), want_logprobs=False,
                                         label_dtype=torch.int64)   # labels-only 8-row kernel, int64
    assert torch.equal(lab64.cpu(), lab.cpu())


@pytest.mark.parametrize("use_bits,from_disk", [(False, False), (True, False), (True, True)])
def test_mask_apply_bit_exact(use_bits, from_disk, tmp_path):
    """Pruner.apply_masks through the HIP kernel == w * m on the CPU, bit for bit (incl. -0.0)."""
    import json
    from drnmi import pruners as P
    from drnmi.drnseg import DRNSeg
    from drnmi.weights import synth_state_dict
    m = DRNSeg("drn_d_22", 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, 0))
    layers = ["layer.0.0.weight", "layer.3.0.conv2.weight", "layer.6.1.conv2.weight", "seg.weight"]
    cfg = {"pruner_type": "block", "configs": [{"layer_set": layers, "sparsity": 0.5, "block_height": 4,
           "block_width": 4, "sub_rows": -1, "sub_cols": -1, "collapse_tensor": True}]}
    jp = tmp_path / "c.json"
    jp.write_text(json.dumps(cfg))
    pr = P.BlockPruner(str(jp), on_gpu=True)
    pr.generate_masks(m)
    if from_disk:   # 1-bit on-disk masks: load seeds the bit cache the kernel reads directly
        pr.save_masks(tmp_path / "m.npz")
        pr = P.BlockPruner(str(jp), on_gpu=True).load_masks(tmp_path / "m.npz")
        assert set(pr._bits_cache) == set(layers)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    ref = O.apply_masks({k: before[k] for k in layers}, {k: pr.mask_dict[k].cpu() for k in layers})
    m = m.to(DEV)
    pr.apply_masks(m, use_bits=use_bits)
    torch.cuda.synchronize()
    sd = m.state_dict()
    for k in layers:
        a = sd[k].cpu().view(torch.int32)
        b = ref[k].contiguous().view(torch.int32)
        assert torch.equal(a, b), k
    for k, v in before.items():
        if k not in layers:
            assert torch.equal(sd[k].cpu(), v), k


PATCH_CASES = [  # cin(stored), cout, ks, stride, h, w  — the bf16 LDS-patch kernel shapes
    (16, 16, 3, 1, 37, 131),
    (16, 32, 3, 2, 41, 133),
    (32, 64, 3, 2, 19, 70),
    (8, 16, 7, 1, 23, 77),
]


@pytest.mark.parametrize("case", range(len(PATCH_CASES)))
def test_patch_conv_bf16(case):
    from drnmi import _lib
    cin, cout, ks, stride, h, w = PATCH_CASES[case]
    n, pad = 2, ks // 2
    x = _rand((n, cin, h, w), 31 + case).bfloat16().float()
    wt = _rand((cout, cin, ks, ks), 41 + case, (2.0 / (ks * ks * cout)) ** 0.5).bfloat16().float()
    sc = torch.rand(cout, generator=torch.Generator().manual_seed(1)) + 0.5
    sh = torch.rand(cout, generator=torch.Generator().manual_seed(2)) - 0.5
    ref = _ref_conv(x, wt, sc, sh, None, stride, pad, 1, True)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV, torch.bfloat16)
    y = ops.conv2d_bn_act(xd, wt.to(DEV), sc.to(DEV), sh.to(DEV), None, stride, pad, 1, True,
                          algo=_lib.ALGO_PATCH)
    got = y.float().permute(0, 3, 1, 2).cpu()
    y2 = ops.conv2d_bn_act(xd, wt.to(DEV), sc.to(DEV), sh.to(DEV), None, stride, pad, 1, True)
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 1.5e-2 * scale
    # the two bf16 algorithms agree to bf16 output rounding
    assert (got - y2.float().permute(0, 3, 1, 2).cpu()).abs().max().item() <= 1e-2 * scale


F32_PATCH_CASES = [  # cin(stored), cout, ks, stride, h, w -- the exact-fp32 patch kernel shapes
    (16, 16, 3, 1, 37, 131),
    (16, 32, 3, 2, 41, 133),
    (8, 16, 7, 1, 23, 77),
    (16, 16, 3, 1, 1, 1),
    (16, 32, 3, 2, 2, 3),
    (8, 16, 7, 1, 70, 5),
]


@pytest.mark.parametrize("case", range(len(F32_PATCH_CASES)))
def test_patch_conv_f32(case):
    """patch_f32_kernel (f32-input MFMA = an fmaf chain per output, conv_igemm's K order) vs the f32
    implicit GEMM it replaces in the fp32 mode (bit-identical) and vs the fp64 conv."""
    cin, cout, ks, stride, h, w = F32_PATCH_CASES[case]
    n, pad = 2, ks // 2
    creal = 3 if cin == 8 else cin
    x = torch.zeros(n, cin, h, w)
    x[:, :creal] = _rand((n, creal, h, w), 131 + case)
    wt = torch.zeros(cout, cin, ks, ks)
    wt[:, :creal] = _rand((cout, creal, ks, ks), 141 + case, (2.0 / (ks * ks * cout)) ** 0.5)
    sc = torch.rand(cout, generator=torch.Generator().manual_seed(11)) + 0.5
    sh = torch.rand(cout, generator=torch.Generator().manual_seed(12)) - 0.5
    ref = _ref_conv(x.double(), wt.double(), sc.double(), sh.double(), None, stride, pad, 1, True)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    name = ops_kernel_name(xd, wt, stride, pad, _lib.ALGO_PATCH)
    assert name.startswith("patch_f32_kernel"), name
    y = ops.conv2d_bn_act(xd, wt.to(DEV), sc.to(DEV), sh.to(DEV), None, stride, pad, 1, True, algo=_lib.ALGO_PATCH)
    yi = ops.conv2d_bn_act(xd, wt.to(DEV), sc.to(DEV), sh.to(DEV), None, stride, pad, 1, True)
    torch.cuda.synchronize()
    got = y.permute(0, 3, 1, 2).cpu().double()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    err_i = (yi.permute(0, 3, 1, 2).cpu().double() - ref).abs().max().item()
    print(f"{name} {F32_PATCH_CASES[case]}: max-abs vs fp64 {err:.2e} (igemm {err_i:.2e}, |y| {scale:.2f})")
    assert err <= 1e-5 * scale + 1e-6
    assert torch.equal(y, yi)


def ops_kernel_name(xd, wt, stride, pad, algo):
    """drnmi_conv_kernel_name of the fp32 launch ops.conv2d_bn_act would make for these operands."""
    n, h, w, cs = xd.shape
    cout, _, ks, _ = wt.shape
    wpk, k = ops.pack_conv_weight(wt, cs, torch.float32)
    a = _lib.ConvArgs()
    a.n, a.h, a.w, a.cin = n, h, w, cs
    a.ks, a.stride, a.pad, a.dil = ks, stride, pad, 1
    a.ho, a.wo = (h + 2 * pad - ks) // stride + 1, (w + 2 * pad - ks) // stride + 1
    a.cout, a.cout_pad, a.k, a.k_pad = cout, wpk.shape[0], k, wpk.shape[1]
    a.dtype = a.out_dtype = _lib.DRNMI_F32
    a.y_sp, a.y_sc = cout, 1
    a.tile, a.algo = -1, algo
    return _lib.load().drnmi_conv_kernel_name(ctypes.byref(a)).decode()


@pytest.mark.parametrize("hw", [(45, 83), (9, 301), (130, 67), (1, 1)])
def test_stem_u8_f32_ingest_bit_exact(hw):
    """Exact-fp32 stem from uint8 frames, centre-tap identity weights: the output is the normalised
    frame itself, bit for bit equal to the reference ToTensor + Normalize (oracle preprocess_u8) and
    to drnmi_frame_ingest_u8, zero padding at every edge."""
    h, w = hw
    frames = torch.randint(0, 256, (3, h, w, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(h + w))
    wt = torch.zeros(16, 3, 7, 7)
    for c in range(3):
        wt[c, c, 3, 3] = 1.0
    y = ops.stem_u8(frames.to(DEV), wt, torch.ones(16), torch.zeros(16), O.INFO_MEAN, O.INFO_STD, relu=False,
                    dtype=torch.float32)
    ref = O.preprocess_u8(frames.numpy())
    assert torch.equal(y.cpu()[..., :3].permute(0, 3, 1, 2), ref)
    assert torch.count_nonzero(y[..., 3:]).item() == 0


@pytest.mark.parametrize("hw", [(45, 83), (33, 130), (64, 64)])
def test_stem_u8_f32_conv(hw):
    """Exact-fp32 fused-ingest stem vs the fp64 conv of the reference-normalised frame, and vs the
    two-launch fp32 path (drnmi_frame_ingest_u8 + the NHWC8 stem); BGR flag."""
    frames = torch.randint(0, 256, (2, hw[0], hw[1], 3), dtype=torch.uint8,
                           generator=torch.Generator().manual_seed(6))
    wt = _rand((16, 3, 7, 7), 51, 0.1)
    sc = torch.rand(16, generator=torch.Generator().manual_seed(4)) + 0.5
    sh = torch.rand(16, generator=torch.Generator().manual_seed(5)) - 0.5
    x = O.preprocess_u8(frames.numpy())
    ref = _ref_conv(x.double(), wt.double(), sc.double(), sh.double(), None, 1, 3, 1, True)
    y = ops.stem_u8(frames.to(DEV), wt, sc.to(DEV), sh.to(DEV), O.INFO_MEAN, O.INFO_STD, dtype=torch.float32)
    got = y.permute(0, 3, 1, 2).cpu().double()
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 1e-5 * scale + 1e-6
    # the NHWC8 form (SRC 1) stages the same normalised values in the same K order, and both are
    # conv_igemm's order on drnmi_frame_ingest_u8's input: bit-identical to the two-launch path
    xi = ops.frame_ingest(frames.to(DEV), O.INFO_MEAN, O.INFO_STD, dtype=torch.float32)
    y2 = ops.conv2d_bn_act(xi, wt.to(DEV), sc.to(DEV), sh.to(DEV), None, 1, 3, 1, True, algo=_lib.ALGO_PATCH)
    yi = ops.conv2d_bn_act(xi, wt.to(DEV), sc.to(DEV), sh.to(DEV), None, 1, 3, 1, True)
    assert torch.equal(y2, y)
    assert torch.equal(yi, y)
    yb = ops.stem_u8(frames.flip(-1).contiguous().to(DEV), wt, sc.to(DEV), sh.to(DEV), O.INFO_MEAN,
                     O.INFO_STD, bgr=True, dtype=torch.float32)
    assert torch.equal(yb, y)


@pytest.mark.parametrize("hw", [(45, 83), (64, 128), (9, 301), (130, 67)])
def test_stem_u8_ingest_bit_exact(hw):
    """Centre-tap identity weights: the stem outputs the normalised frame itself, which must
    equal the reference ToTensor+Normalize (oracle preprocess_u8) rounded to bf16, bit for bit,
    including the zero padding at every image edge (frame widths with W*3 % 4 != 0 too)."""
    h, w = hw
    frames = torch.randint(0, 256, (3, h, w, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(h * w))
    wt = torch.zeros(16, 3, 7, 7)
    for c in range(3):
        wt[c, c, 3, 3] = 1.0
    y = ops.stem_u8(frames.to(DEV), wt, torch.ones(16), torch.zeros(16), O.INFO_MEAN, O.INFO_STD, relu=False)
    ref = O.preprocess_u8(frames.numpy()).bfloat16()            # [N,3,H,W]
    got = y.cpu()[..., :3].permute(0, 3, 1, 2)
    assert torch.equal(got, ref)
    assert torch.count_nonzero(y[..., 3:]).item() == 0


@pytest.mark.parametrize("hw", [(45, 83), (33, 130)])
def test_stem_u8_fused_ingest(hw):
    frames = torch.randint(0, 256, (2, hw[0], hw[1], 3), dtype=torch.uint8,
                           generator=torch.Generator().manual_seed(3))
    wt = _rand((16, 3, 7, 7), 50, 0.1).bfloat16().float()
    sc = torch.rand(16, generator=torch.Generator().manual_seed(4)) + 0.5
    sh = torch.rand(16, generator=torch.Generator().manual_seed(5)) - 0.5
    x = O.preprocess_u8(frames.numpy()).bfloat16().float()
    ref = _ref_conv(x, wt, sc, sh, None, 1, 3, 1, True)
    y = ops.stem_u8(frames.to(DEV), wt, sc.to(DEV), sh.to(DEV), O.INFO_MEAN, O.INFO_STD)
    got = y.float().permute(0, 3, 1, 2).cpu()
    assert (got - ref).abs().max().item() <= 1.5e-2 * ref.abs().max().item()
    yb = ops.stem_u8(frames.flip(-1).contiguous().to(DEV), wt, sc.to(DEV), sh.to(DEV), O.INFO_MEAN,
                     O.INFO_STD, bgr=True)
    assert torch.equal(yb, y)


@pytest.mark.parametrize("shape", [(64, 128, 3, 2, 1, 37, 51), (128, 256, 3, 1, 2, 33, 40),
                                   (512, 512, 3, 1, 4, 24, 40), (256, 512, 1, 1, 1, 20, 30),
                                   (64, 128, 1, 2, 1, 37, 51), (32, 64, 3, 2, 1, 41, 53), (32, 64, 1, 2, 1, 41, 53),
                                   (64, 256, 1, 1, 1, 19, 23), (128, 256, 3, 1, 1, 29, 35),
                                   (64, 64, 3, 1, 1, 37, 70), (128, 128, 3, 1, 1, 21, 131),
                                   (64, 128, 3, 1, 2, 19, 67), (128, 64, 3, 1, 1, 9, 200)])
def test_dma_conv_matches_register_staged(shape):
    """bf16 LDS-DMA kernel (tile 4) vs the register-staged bf16 tile 0 on the same inputs."""
    cin, cout, ks, stride, dil, h, w = shape
    pad = dil * (ks // 2)
    x = _rand((3, cin, h, w), 61).bfloat16()
    wt = _rand((cout, cin, ks, ks), 62, (2.0 / (ks * ks * cout)) ** 0.5)
    sc = torch.rand(cout, generator=torch.Generator().manual_seed(63)) + 0.5
    sh = torch.rand(cout, generator=torch.Generator().manual_seed(64)) - 0.5
    ho = (h + 2 * pad - dil * (ks - 1) - 1) // stride + 1
    wo = (w + 2 * pad - dil * (ks - 1) - 1) // stride + 1
    res = _rand((3, ho, wo, cout), 65).bfloat16().to(DEV)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    a = ops.conv2d_bn_act(xd, wt.to(DEV), sc.to(DEV), sh.to(DEV), res, stride, pad, dil, True, tile=0).float()
    ref = _ref_conv(x.float(), wt.bfloat16().float(), sc, sh, res.float().permute(0, 3, 1, 2).cpu(), stride,
                    pad, dil, True)
    ran = 0
    from drnmi import _lib
    for t in range(4, _lib.load().drnmi_conv_num_tiles()):   # every LDS-DMA variant that takes the shape
        try:
            b = ops.conv2d_bn_act(xd, wt.to(DEV), sc.to(DEV), sh.to(DEV), res, stride, pad, dil, True,
                                  tile=t).float()
        except RuntimeError as e:
            assert "EINVAL" in str(e) or "ENOTSUP" in str(e)
            continue
        ran += 1
        assert (a - b).abs().max().item() <= 1e-2 * a.abs().max().item(), f"tile {t}"
        assert (b.permute(0, 3, 1, 2).cpu() - ref).abs().max().item() <= 1.5e-2 * ref.abs().max().item()
    assert ran >= (1 if cin < 64 else 3)


@pytest.mark.parametrize("shape", [(512, 512, 3, 1, 4, 20, 37), (256, 256, 3, 1, 2, 33, 40), (256, 512, 1, 1, 1, 20, 30),
                                   (64, 64, 3, 1, 1, 37, 70), (128, 128, 3, 1, 1, 21, 131), (64, 128, 3, 2, 1, 37, 51),
                                   (32, 64, 1, 2, 1, 41, 53), (512, 19, 1, 1, 1, 17, 23)])
def test_null_scale_seeds_accumulator(shape):
    """scale = NULL (BN scale folded into the weights): the LDS-DMA kernels start from
    shift + residual; result matches the scaled launch within bf16 rounding, every variant."""
    from drnmi import _lib
    cin, cout, ks, stride, dil, h, w = shape
    pad = dil * (ks // 2)
    x = _rand((2, h, w, cin), 71).bfloat16().to(DEV)
    wt = _rand((cout, cin, ks, ks), 72, (2.0 / (ks * ks * cout)) ** 0.5).to(DEV)
    sc = (torch.rand(cout, generator=torch.Generator().manual_seed(73)) + 0.5).to(DEV)
    sh = (torch.rand(cout, generator=torch.Generator().manual_seed(74)) - 0.5).to(DEV)
    ho = (h + 2 * pad - dil * (ks - 1) - 1) // stride + 1
    wo = (w + 2 * pad - dil * (ks - 1) - 1) // stride + 1
    seg = cout == 19
    res = None if seg else _rand((2, ho, wo, cout), 75).bfloat16().to(DEV)
    ran = 0
    for t in [-1] + list(range(4, _lib.load().drnmi_conv_num_tiles())):
        kw = dict(stride=stride, padding=pad, dilation=dil, relu=not seg, out_nchw_fp32=seg, tile=t)
        try:
            a = ops.conv2d_bn_act(x, wt, sc, sh, res, **kw).float()
            b = ops.conv2d_bn_act(x, wt, sc, sh, res, fold_scale=True, **kw).float()
        except RuntimeError as e:
            assert "EINVAL" in str(e) or "ENOTSUP" in str(e)
            continue
        ran += 1
        assert (a - b).abs().max().item() <= 1.5e-2 * a.abs().max().item(), f"tile {t}"
    assert ran >= 2


@pytest.mark.parametrize("n,h,w,cin,cout,dil,with_res,fold", [
    (2, 9, 256, 256, 256, 2, True, True), (1, 5, 512, 512, 512, 4, True, True),
    (2, 6, 256, 128, 256, 2, False, True), (1, 4, 256, 512, 512, 1, False, False),
    (3, 3, 256, 64, 256, 4, True, True), (1, 2, 768, 256, 512, 1, True, True)])
def test_strip_kernel_bit_identical(n, h, w, cin, cout, dil, with_res, fold):
    """Strip-staged B (tile 18, conv_strip_kernel: one DMA of 256 + 2 dil input pixels per
    (channel block, tap row), read by the three kw taps at row offset kw*dil) == the per-tap
    gather of the same 256 x 256 tile (tile 5) bit for bit, and auto-routing takes it for
    wo % 256 == 0.  Image borders (top/bottom rows, left/right strip ends) are in every case."""
    g = torch.Generator().manual_seed(90 + h * w + cin)
    x = torch.randn(n, h, w, cin, generator=g).bfloat16().to(DEV)
    wt = (torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cout)) ** 0.5).to(DEV)
    sc = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    sh = (torch.rand(cout, generator=g) - 0.5).to(DEV)
    res = torch.randn(n, h, w, cout, generator=g).bfloat16().to(DEV) if with_res else None
    kw = dict(stride=1, padding=dil, dilation=dil, relu=True, fold_scale=fold)
    a = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=5, **kw)
    b = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=18, **kw)
    auto = ops.conv2d_bn_act(x, wt, sc, sh, res, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(auto, b)
    ref = _ref_conv(x.float().permute(0, 3, 1, 2).cpu(), wt.bfloat16().float().cpu(), sc.cpu(), sh.cpu(),
                    res.float().permute(0, 3, 1, 2).cpu() if with_res else None, 1, dil, dil, True)
    assert (b.float().permute(0, 3, 1, 2).cpu() - ref).abs().max().item() <= 1.5e-2 * ref.abs().max().item()


@pytest.mark.parametrize("n,h,w,cin,cout,dil,with_res,fold", [
    (2, 9, 256, 256, 256, 2, True, True), (1, 5, 512, 512, 512, 4, True, True),
    (2, 6, 256, 128, 256, 2, False, True), (1, 4, 256, 512, 512, 1, False, False),
    (1, 2, 768, 256, 512, 1, True, True), (1, 3, 256, 128, 256, 3, True, False)])
def test_stag_kernel_bit_identical(n, h, w, cin, cout, dil, with_res, fold):
    """conv_stag_kernel (tile 19: the strip tile with waves 4-7 half a K step behind their SIMD
    partners, two barriers per step) == conv_strip_kernel (tile 18) bit for bit: same K order,
    same MFMA order per accumulator, same epilogue.  Borders and dil 1..4 as in the strip test."""
    g = torch.Generator().manual_seed(190 + h * w + cin)
    x = torch.randn(n, h, w, cin, generator=g).bfloat16().to(DEV)
    wt = (torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cout)) ** 0.5).to(DEV)
    sc = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    sh = (torch.rand(cout, generator=g) - 0.5).to(DEV)
    res = torch.randn(n, h, w, cout, generator=g).bfloat16().to(DEV) if with_res else None
    kw = dict(stride=1, padding=dil, dilation=dil, relu=True, fold_scale=fold)
    a = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=18, **kw)
    b = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=19, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("n,h,w,cin,cout,dil,with_res", [
    (2, 9, 256, 256, 256, 2, True), (1, 5, 512, 512, 512, 4, True), (2, 6, 256, 128, 256, 2, False),
    (1, 4, 256, 512, 512, 1, False), (1, 2, 768, 256, 512, 1, True), (1, 3, 256, 128, 256, 3, True)])
def test_w1_kernel_bit_identical(n, h, w, cin, cout, dil, with_res):
    """conv_w1_kernel (tile 22: the stag256 tile as 4 waves of 128 x 128, one wave per SIMD, one
    barrier per K step) == conv_stag_kernel (tile 19) bit for bit: same K order, same MFMA order per
    accumulator, same accumulator start and epilogue.  Borders and dil 1..4 as in the strip test."""
    g = torch.Generator().manual_seed(390 + h * w + cin)
    x = torch.randn(n, h, w, cin, generator=g).bfloat16().to(DEV)
    wt = (torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cout)) ** 0.5).to(DEV)
    sc = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    sh = (torch.rand(cout, generator=g) - 0.5).to(DEV)
    res = torch.randn(n, h, w, cout, generator=g).bfloat16().to(DEV) if with_res else None
    kw = dict(stride=1, padding=dil, dilation=dil, relu=True, fold_scale=True)
    a = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=19, **kw)
    b = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=22, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("n,h,w,cin,cout,dil,with_res", [
    (2, 5, 256, 128, 128, 1, True), (1, 6, 512, 128, 128, 1, False), (1, 4, 256, 128, 128, 2, True),
    (2, 3, 256, 256, 256, 4, True), (1, 4, 256, 512, 256, 3, False)])
def test_w1h_kernel_bit_identical(n, h, w, cin, cout, dil, with_res):
    """conv_w1h_kernel (tile 23: 128 x 128 tiles of 4 waves of 64 x 64, two workgroups per CU) ==
    conv_stag128 / conv_stag (tile 19) bit for bit: the same K order and accumulator start."""
    g = torch.Generator().manual_seed(490 + h * w + cin + cout)
    x = torch.randn(n, h, w, cin, generator=g).bfloat16().to(DEV)
    wt = (torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cout)) ** 0.5).to(DEV)
    sc = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    sh = (torch.rand(cout, generator=g) - 0.5).to(DEV)
    res = torch.randn(n, h, w, cout, generator=g).bfloat16().to(DEV) if with_res else None
    kw = dict(stride=1, padding=dil, dilation=dil, relu=True, fold_scale=True)
    a = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=19, **kw)
    b = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=23, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_w1_kernel_refuses_unfolded_scale():
    """tile 22 serves only the BN-scale-folded launches (accumulators start from shift + residual)."""
    x = torch.randn(1, 4, 256, 256, device=DEV).bfloat16()
    wt = torch.randn(256, 256, 3, 3, device=DEV) * 0.02
    sc = torch.rand(256, device=DEV) + 0.5
    with pytest.raises(RuntimeError, match="ENOTSUP"):
        ops.conv2d_bn_act(x, wt, sc, None, None, padding=1, dilation=1, tile=22, fold_scale=False)


@pytest.mark.parametrize("n,h,w,dil,with_res", [(2, 5, 256, 1, True), (1, 4, 512, 1, False), (1, 6, 256, 2, True)])
def test_stag128_matches_halo_bit_identical(n, h, w, dil, with_res):
    """128 -> 128 3x3 (D-22 layer4) on the staggered 128-channel tile (conv_stag128_kernel, tile
    19) == the halo kernel (tile 17): same (channel block, tap) K order, same substep order, same
    accumulator start (shift + residual), so the same bits."""
    g = torch.Generator().manual_seed(290 + h * w)
    x = torch.randn(n, h, w, 128, generator=g).bfloat16().to(DEV)
    wt = (torch.randn(128, 128, 3, 3, generator=g) * (2.0 / (9 * 128)) ** 0.5).to(DEV)
    sc = (torch.rand(128, generator=g) + 0.5).to(DEV)
    sh = (torch.rand(128, generator=g) - 0.5).to(DEV)
    res = torch.randn(n, h, w, 128, generator=g).bfloat16().to(DEV) if with_res else None
    kw = dict(stride=1, padding=dil, dilation=dil, relu=True, fold_scale=True)
    # the halo kernel's patch does not fit LDS at dil 2 with 128 channels: conv_big's 128 x 256
    # tile (tile 4, same K order and accumulator start) is the reference there
    a = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=17 if dil == 1 else 4, **kw)
    b = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=19, **kw)
    auto = ops.conv2d_bn_act(x, wt, sc, sh, res, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(auto, b)


def test_stag_kernel_refuses_cin_not_multiple_of_128():
    x = torch.randn(1, 4, 256, 64, device=DEV).bfloat16()
    wt = torch.randn(256, 64, 3, 3, device=DEV) * 0.02
    with pytest.raises(RuntimeError, match="ENOTSUP"):
        ops.conv2d_bn_act(x, wt, padding=1, dilation=1, tile=19)


def test_strip_kernel_refuses_unaligned_rows():
    x = torch.randn(1, 4, 200, 256, device=DEV).bfloat16()
    wt = torch.randn(256, 256, 3, 3, device=DEV) * 0.02
    with pytest.raises(RuntimeError, match="ENOTSUP"):
        ops.conv2d_bn_act(x, wt, padding=2, dilation=2, tile=18)


def test_forced_tile_larger_than_weights_is_rejected():
    """A 256-channel tile over a 128-row packed weight must be refused, not read past it."""
    x = torch.randn(1, 16, 16, 128, device=DEV).bfloat16()
    wt = torch.randn(128, 128, 3, 3, device=DEV) * 0.05
    with pytest.raises(RuntimeError, match="EINVAL"):
        ops.conv2d_bn_act(x, wt, padding=1, tile=5)


@pytest.mark.parametrize("dt", [(torch.uint8, torch.uint8), (torch.int64, torch.int64), (torch.uint8, torch.int64)])
def test_confusion_matrix_matches_fast_hist(dt):
    from drnmi import metrics
    g = torch.Generator().manual_seed(9)
    pred = torch.randint(0, 19, (2, 61, 97), generator=g)
    label = torch.randint(0, 21, (2, 61, 97), generator=g)
    label[label >= 19] = 255                      # ignore label
    ref = O.fast_hist(pred.numpy().reshape(-1), label.numpy().reshape(-1), 19)
    h = metrics.fast_hist(pred.to(DEV, dt[0]), label.to(DEV, dt[1]), 19)
    h = metrics.fast_hist(pred.to(DEV, dt[0]), label.to(DEV, dt[1]), 19, hist=h)   # accumulates
    np.testing.assert_array_equal(h.cpu().numpy(), 2 * ref)
    np.testing.assert_allclose(metrics.per_class_iu(h), O.per_class_iu(2 * ref))
    assert metrics.miou(h) == round(float(np.nanmean(O.per_class_iu(ref))) * 100, 2)


X6_CASES = [
    # (n, h, w, cin, cout, ks, stride, pad, dil, res)
    (1, 20, 36, 512, 512, 3, 1, 4, 4, True),     # layer6-shaped, dilation 4, 256-channel tile
    (2, 11, 13, 256, 256, 3, 1, 2, 2, False),    # ragged pixel tile, dilation 2
    (1, 16, 16, 128, 128, 3, 1, 1, 1, True),     # 128-channel tile
    (1, 17, 15, 32, 64, 3, 2, 1, 1, False),      # cin 32, stride 2, 64-channel tile
    (1, 16, 16, 64, 128, 1, 2, 0, 1, False),     # 1x1 stride-2 downsample
]


@pytest.mark.parametrize("case", X6_CASES)
def test_conv_x6_fp32_accuracy(case):
    """DRNMI_F32X3 (split-bf16, 6 products) vs an fp64 conv: as close as the exact-f32 kernel."""
    _x6_case(case, split=False)


@pytest.mark.parametrize("case", [X6_CASES[0], X6_CASES[1], X6_CASES[2]])
def test_conv_x6_split_k(case):
    """The split-K launch (caller workspace, grids of few tiles): partial sums + the epilogue
    kernel, as accurate as the unsplit kernel (fp64 reference, same bound)."""
    _x6_case(case, split=True)


@pytest.mark.parametrize("case", [X6_CASES[0], X6_CASES[2], X6_CASES[4]])
def test_conv_x6_variants_bit_identical(case):
    """Every conv_x6 tile variant (forced through drnmi_conv_args.tile: 256 / 128 / 64 channels,
    8- and 4-wave, and the 128 x 128 / 64 x 128 two-per-CU tiles) keeps each accumulator's MFMA
    order: the outputs are bit-identical to the auto variant's."""
    outs = {}
    for v in (-1, 0, 1, 2, 3, 4, 5):
        y = _x6_case(case, split=False, tile=v, check=v == -1)
        if y is not None:
            outs[v] = y
    assert len(outs) >= 3
    for v, y in outs.items():
        assert torch.equal(y, outs[-1]), v


def test_conv_x6_two_per_cu_split_k():
    """The two-workgroups-per-CU tile under a forced split-K (tile = 4 + 6 * 2): as accurate as the
    unsplit kernel."""
    _x6_case(X6_CASES[0], split=True, tile=4 + 6 * 2)


@pytest.mark.parametrize("case", [X6_CASES[1], X6_CASES[2], (2, 24, 20, 64, 256, 1, 1, 0, 1, False)])
def test_conv_x6_bn_stats_partials(case):
    """drnmi_conv_args.stats: the conv_x6 epilogue's per-channel fp64 sums of y and y^2 (one row
    per 64-pixel wave slice) match fp64 sums over the stored y, and drnmi_bn_stats_partials_f32
    gives the batch mean / invstd / running stats of drnmi_bn_stats_f32 over y."""
    n, h, w, cin, cout, ks, s, pad, dil, _ = case
    y, args, keep = _x6_case(case, split=False, check=False, stats=True)
    rows = y.numel() // cout
    G = _lib.load().drnmi_conv_stats_rows(ctypes.byref(args))
    part = keep["stats"].view(2, G, cout).cpu().numpy()
    yd = y.reshape(rows, cout).double().cpu().numpy()
    np.testing.assert_allclose(part[0].sum(0), yd.sum(0), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(part[1].sum(0), (yd * yd).sum(0), rtol=1e-12, atol=1e-9)
    lib = _lib.load()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    sp = ctypes.c_void_p(_lib.stream_ptr())
    outs = []
    for fused in (True, False):
        mean, invstd = torch.empty(cout, device=DEV), torch.empty(cout, device=DEV)
        rm, rv = torch.zeros(cout, device=DEV), torch.ones(cout, device=DEV)
        if fused:
            _lib.check(lib.drnmi_bn_stats_partials_f32(vp(keep["stats"]), G, rows, cout, 1e-5, 0.1, vp(mean),
                                                       vp(invstd), vp(rm), vp(rv), None, sp), "partials")
        else:
            ws = torch.empty(lib.drnmi_reduce_workspace_bytes(rows, cout), dtype=torch.uint8, device=DEV)
            _lib.check(lib.drnmi_bn_stats_f32(vp(y), rows, cout, 1e-5, 0.1, vp(mean), vp(invstd), vp(rm), vp(rv),
                                              None, vp(ws), sp), "stats")
        outs.append([t.cpu() for t in (mean, invstd, rm, rv)])
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=2e-7, atol=1e-9)


def test_conv_x6_bn_stats_refused_with_split_k():
    """A split-K plan cannot write the statistics: the launch is refused, nothing runs."""
    y, args, keep = _x6_case(X6_CASES[0], split=True, check=False, stats="query")
    assert _lib.load().drnmi_conv_stats_rows(ctypes.byref(args)) == 0
    args.stats = keep["y"].data_ptr()
    assert _lib.load().drnmi_conv2d_bn_act(ctypes.byref(args), ctypes.c_void_p(_lib.stream_ptr())) == -1


def _x6_case(case, split, tile=-1, check=True, stats=False):
    import torch.nn.functional as F
    from drnmi import ops
    from drnmi.engine import split3_bf16
    n, h, w, cin, cout, ks, s, pad, dil, res = case
    g = torch.Generator().manual_seed(cin + cout + ks)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, ks, ks, generator=g) / (cin * ks * ks) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g)
    y64 = F.conv2d(x.double(), wt.double(), stride=s, padding=pad, dilation=dil) * sc.double().view(1, -1, 1, 1) \
        + sh.double().view(1, -1, 1, 1)
    r = None
    if res:
        r = torch.randn(y64.shape, generator=g)
        y64 = y64 + r.double()
    y64 = torch.relu(y64)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    rd = r.permute(0, 2, 3, 1).contiguous().to(DEV) if res else None
    f32 = ops.conv2d_bn_act(xd, wt.to(DEV), sc.to(DEV), sh.to(DEV), rd, stride=s, padding=pad, dilation=dil,
                            relu=True)
    wpk, k = ops.pack_conv_weight(wt.to(DEV), cin, torch.float32)
    planes = split3_bf16(wpk)
    scp = torch.ones(wpk.shape[0], device=DEV)
    shp = torch.zeros(wpk.shape[0], device=DEV)
    scp[:cout], shp[:cout] = sc.to(DEV), sh.to(DEV)
    ho = (h + 2 * pad - dil * (ks - 1) - 1) // s + 1
    wo = (w + 2 * pad - dil * (ks - 1) - 1) // s + 1
    y = torch.empty(n, ho, wo, cout, device=DEV)
    a = _lib.ConvArgs()
    a.x, a.wgt, a.scale, a.shift = xd.data_ptr(), planes.data_ptr(), scp.data_ptr(), shp.data_ptr()
    a.res = rd.data_ptr() if res else None
    a.y = y.data_ptr()
    a.y_sn, a.y_sp, a.y_sc = ho * wo * cout, cout, 1
    a.n, a.h, a.w, a.cin = n, h, w, cin
    a.ho, a.wo, a.cout, a.cout_pad = ho, wo, cout, wpk.shape[0]
    a.ks, a.stride, a.pad, a.dil = ks, s, pad, dil
    a.k, a.k_pad = k, wpk.shape[1]
    a.relu, a.dtype, a.out_dtype, a.tile, a.algo = 1, _lib.DRNMI_F32X3, _lib.DRNMI_F32, tile, _lib.ALGO_IGEMM
    name = _lib.load().drnmi_conv_kernel_name(ctypes.byref(a)).decode()
    assert name.startswith("conv_x6_kernel")
    bco = int(name.split("<")[1].split(",")[1]) * int(name.split(",")[2])
    if (cout + bco - 1) // bco * bco > wpk.shape[0]:
        return None                                   # a forced tile wider than the packed rows
    keep = {"y": y}
    if split:
        nb = _lib.load().drnmi_conv_workspace_bytes(ctypes.byref(a))
        assert nb > 0, "these geometries leave most CUs idle: the launch must split"
        ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
        a.ws, a.ws_bytes = ws.data_ptr(), nb
        keep["ws"] = ws
        name += f" split-K {nb // (4 * n * ho * wo * cout)}"
    if stats == "query":
        return y, a, keep
    if stats:
        rows = _lib.load().drnmi_conv_stats_rows(ctypes.byref(a))
        assert rows > 0
        keep["stats"] = torch.full((2 * rows * cout,), float("nan"), dtype=torch.float64, device=DEV)
        a.stats = keep["stats"].data_ptr()
    _lib.check(_lib.load().drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())), "x6")
    torch.cuda.synchronize()
    ref = y64.permute(0, 2, 3, 1).numpy()
    e_x6 = np.abs(y.cpu().double().numpy() - ref).max()
    e_f32 = np.abs(f32.cpu().double().numpy() - ref).max()
    scale = np.abs(ref).max()
    print(f"{name} {case}: max-abs vs fp64 {e_x6:.2e} (exact-f32 kernel {e_f32:.2e}, |y| {scale:.1f})")
    if check:
        assert e_x6 <= max(4 * e_f32, 1e-6 * scale)
    return (y, a, keep) if stats else y


@pytest.mark.parametrize("case", [
    # (n, h, w, cin, cout, ks, dil, cin2, stride2, h2, w2)
    (2, 16, 24, 256, 256, 3, 2, 128, 1, 16, 24),     # layer5.0: conv2 + 1x1 downsample 128 -> 256
    (1, 12, 20, 512, 512, 3, 4, 256, 1, 12, 20),     # layer6.0: dilation 4, 256 -> 512
    (1, 9, 13, 256, 1024, 1, 1, 512, 2, 18, 26),     # Bottleneck conv3 + stride-2 downsample
    (2, 33, 70, 64, 64, 3, 1, 32, 2, 66, 140),       # layer3.0: halo conv2 + 1x1 s2 downsample 32 -> 64
    (1, 20, 40, 128, 128, 3, 1, 64, 2, 40, 80),      # layer4.0: halo conv2 + 1x1 s2 downsample 64 -> 128
    (3, 7, 130, 64, 64, 3, 1, 32, 2, 13, 259),       # ragged blocks, odd x2 extent
    (2, 5, 256, 256, 256, 3, 2, 128, 1, 5, 256),     # layer5.0 on whole 256-pixel rows: conv_stag_x2_kernel
    (2, 4, 256, 128, 128, 3, 1, 64, 2, 8, 512),      # layer4.0 on whole rows: conv_stag128_x2_kernel (vs halo)
    (1, 4, 512, 512, 512, 3, 4, 256, 1, 4, 512),     # layer6.0 on whole rows: conv_stag_x2_kernel
])
def test_conv_fused_downsample(case):
    """drnmi_conv_args.x2: y = relu(conv(x, w) + conv1x1_s(x2, w2) + shift) as one launch (the
    downsample folded into the block's last conv) vs torch fp32 on the same bf16 operands.
    conv_big takes cin2 % 64 == 0 (k_pad = k); the halo kernel (64/128-channel 3x3) takes cin2
    32/64 with weight rows zero-padded to 64-column steps, and on a shape both take the two are
    bit-identical (same K order and accumulator start)."""
    n, h, w, cin, cout, ks, dil, cin2, s2, h2, w2 = case
    g = torch.Generator().manual_seed(cin + cin2)
    x = (torch.randn(n, h, w, cin, generator=g)).to(torch.bfloat16)
    x2 = (torch.randn(n, h2, w2, cin2, generator=g)).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, ks, ks, generator=g) / (cin * ks * ks) ** 0.5).to(torch.bfloat16)
    wd = (torch.randn(cout, cin2, 1, 1, generator=g) / cin2 ** 0.5).to(torch.bfloat16)
    sh = torch.randn(cout, generator=g)
    pad = dil if ks == 3 else 0
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wt.float(), padding=pad, dilation=dil) \
        + F.conv2d(x2.float().permute(0, 3, 1, 2), wd.float(), stride=s2) + sh.view(1, -1, 1, 1)
    ref = torch.relu(ref).permute(0, 2, 3, 1)
    k1 = ks * ks * cin
    halo = cin in (64, 128) and cout in (64, 128) and ks == 3
    kp = (k1 + cin2 + 63) // 64 * 64 if halo else k1 + cin2
    wpk = torch.zeros(cout, kp, dtype=torch.bfloat16)
    wpk[:, :k1] = wt.permute(0, 2, 3, 1).reshape(cout, k1)
    wpk[:, k1:k1 + cin2] = wd.reshape(cout, cin2)
    ho, wo = h, w
    y = torch.empty(n, ho, wo, cout, dtype=torch.bfloat16, device=DEV)
    xd, x2d, wpd, shd = x.to(DEV), x2.to(DEV), wpk.to(DEV), sh.to(DEV)
    a = _lib.ConvArgs()
    a.x, a.wgt, a.scale, a.shift, a.res, a.y = xd.data_ptr(), wpd.data_ptr(), None, shd.data_ptr(), None, y.data_ptr()
    a.y_sn, a.y_sp, a.y_sc = ho * wo * cout, cout, 1
    a.n, a.h, a.w, a.cin, a.ho, a.wo, a.cout, a.cout_pad = n, h, w, cin, ho, wo, cout, cout
    a.ks, a.stride, a.pad, a.dil = ks, 1, pad, dil
    a.k, a.k_pad = k1 + cin2, kp
    a.relu, a.dtype, a.out_dtype, a.tile, a.algo = 1, _lib.DRNMI_BF16, _lib.DRNMI_BF16, -1, _lib.ALGO_IGEMM
    a.x2, a.cin2, a.h2, a.w2, a.stride2 = x2d.data_ptr(), cin2, h2, w2, s2
    name = _lib.load().drnmi_conv_kernel_name(ctypes.byref(a)).decode()
    stag = ks == 3 and wo % 256 == 0 and cin % 128 == 0 and kp == k1 + cin2
    s1x2 = halo and cin == 64 and cout == 64 and cin2 == 32 and s2 == 2 and dil == 1   # conv_s1x2row_kernel
    # whole-row strip shapes: conv_w1h_x2 at 128 channels (layer4.0), else the staggered x2 tile (the
    # conv_w1 / 256-channel conv_w1h x2 forms measured slower inside the network: profiles/r11_w1h)
    assert name.startswith("conv_w1h_x2_kernel" if stag and cout <= 128 else "conv_stag_x2_kernel" if stag
                           else "conv_s1x2row_kernel" if s1x2 else "conv_halo_kernel" if halo else "conv_big_kernel"), name
    _lib.check(_lib.load().drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())), "fused ds")
    torch.cuda.synchronize()
    err = (y.float().cpu() - ref).abs().max().item()
    print(f"{name} {case}: max-abs {err:.3e} (|y| {ref.abs().max().item():.2f})")
    assert err <= 0.02 * max(1.0, ref.abs().max().item())
    if stag:                              # == conv_big's X2 form of the same 256 x 256 tile (tile 5) / the halo kernel
        yb = torch.empty_like(y)
        a.y, a.tile = yb.data_ptr(), 17 if halo else 5
        _lib.check(_lib.load().drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())), "fused ds big")
        torch.cuda.synchronize()
        assert torch.equal(yb, y)
        # the staggered x2 tiles (tile 19: conv_stag128_x2 / conv_stag_x2) and both conv_w1 forms
        for t in (19, 22, 23):
            if t == 22 and cout % 256:
                continue
            a.y, a.tile = yb.data_ptr(), t
            yb.zero_()
            _lib.check(_lib.load().drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())), f"x2 tile {t}")
            torch.cuda.synchronize()
            assert torch.equal(yb, y), t
        a.y, a.tile = y.data_ptr(), -1
    if halo and kp == k1 + cin2:          # conv_big takes it too (tile 4: the 128 x 256 X2 form)
        yb = torch.empty_like(y)
        a.y, a.tile = yb.data_ptr(), 4
        _lib.check(_lib.load().drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())), "fused ds big")
        torch.cuda.synchronize()
        assert torch.equal(yb, y)
        a.y = y.data_ptr()
    # no kernel without x2 support may take it silently
    a.tile = 0
    assert _lib.load().drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr())) < 0


def test_bf16_fused_downsample_network_matches_unfused(golden_forward):
    """The bf16 network with the downsamples folded (default) vs the separate launches: the fused
    form skips one bf16 rounding of the residual, so the two agree to bf16 noise."""
    from drnmi import engine
    from drnmi.drnseg import build
    case = "d22_2x128x256"
    m = build("drn_d_22", 19, seed=int(golden_forward[case + "/meta"][0]), device=DEV, precision="bf16")
    frames = torch.from_numpy(golden_forward[case + "/frames"]).to(DEV)
    pk_plan = m.plan(2, 128, 256)
    assert len(pk_plan.skip) == 4          # layer3.0 / layer4.0 (halo) and layer5.0 / layer6.0 (conv_big)
    fused = m.segment(frames).long()
    engine.FUSE_DOWNSAMPLE = False
    try:
        m2 = build("drn_d_22", 19, seed=int(golden_forward[case + "/meta"][0]), device=DEV, precision="bf16")
        assert not m2.plan(2, 128, 256).skip
        unfused = m2.segment(frames).long()
    finally:
        engine.FUSE_DOWNSAMPLE = True
    ref = torch.from_numpy(golden_forward[case + "/labels"]).long().to(DEV)
    agree = (fused == unfused).float().mean().item()
    a_f = (fused == ref).float().mean().item()
    a_u = (unfused == ref).float().mean().item()
    print(f"fused vs unfused labels {agree:.4f}; vs reference fused {a_f:.4f} unfused {a_u:.4f}")
    assert agree >= 0.99 and a_f >= 0.98


@pytest.mark.parametrize("shape", [(2, 45, 83), (1, 64, 128), (3, 33, 130), (1, 9, 301), (2, 130, 67)])
def test_stem_layer1_fused_bit_identical(shape):
    """drnmi_stem_layer1 (one launch, the stem output never leaves the CU) vs stem_dma_kernel +
    patch_dma_kernel<16, 16, ...> (two launches): bit-identical, including the zero padding of
    layer1 at every image edge, ragged tiles and frame widths with W*3 % 4 != 0; BGR too."""
    n, h, w = shape
    g = torch.Generator().manual_seed(h * w)
    frames = torch.randint(0, 256, (n, h, w, 3), dtype=torch.uint8, generator=g).to(DEV)
    w0 = _rand((16, 3, 7, 7), 91, 0.1)
    w1 = _rand((16, 16, 3, 3), 92, 0.2)
    sc0, sh0 = torch.rand(16, generator=g) + 0.5, torch.rand(16, generator=g) - 0.5
    sc1, sh1 = torch.rand(16, generator=g) + 0.5, torch.rand(16, generator=g) - 0.5
    for bgr in (False, True):
        y0 = ops.stem_u8(frames, w0, sc0.to(DEV), sh0.to(DEV), O.INFO_MEAN, O.INFO_STD, bgr=bgr)
        two = ops.conv2d_bn_act(y0, w1.to(DEV), sc1.to(DEV), sh1.to(DEV), None, 1, 1, 1, True,
                                algo=_lib.ALGO_PATCH)
        one = ops.stem_layer1_u8(frames, w0, sc0.to(DEV), sh0.to(DEV), w1.to(DEV), sc1.to(DEV), sh1.to(DEV),
                                 O.INFO_MEAN, O.INFO_STD, bgr=bgr)
        torch.cuda.synchronize()
        assert torch.equal(one, two), (bgr, (one.float() - two.float()).abs().max().item())


def test_stem_fused_network_matches_two_launch():
    """The bf16 video path with the stem fused gives the same labels as with the stem and layer1
    as two launches (bit-identical layer1 output => identical network); the fused front
    (layer0..layer2 in one launch, test_front.py) is switched off for both."""
    from drnmi import engine
    from drnmi.drnseg import build
    from drnmi.weights import synth_frames
    engine.FUSE_FRONT = False
    try:
        m = build("drn_d_22", 19, seed=3, device=DEV, precision="bf16")
        frames = torch.from_numpy(synth_frames(11, 2, 136, 200)).to(DEV)
        assert m.plan(2, 136, 200).stem_fused and not m.plan(2, 136, 200).front_fused
        fused = m.segment(frames)
        engine.FUSE_STEM = False
        try:
            m2 = build("drn_d_22", 19, seed=3, device=DEV, precision="bf16")
            assert not m2.plan(2, 136, 200).stem_fused
            two = m2.segment(frames)
        finally:
            engine.FUSE_STEM = True
    finally:
        engine.FUSE_FRONT = True
    assert torch.equal(fused, two)



def test_up8_labels_only_matches_logprob_argmax_at_near_ties():
    """The labels-only head skips the log-softmax except where the top two up-sampled logits
    are within 2^-16; there it must reproduce torch.max over the log-probs exactly, including
    the lower-index choice when the rounding of (v - max) - lse merges the top two."""
    from drnmi.weights import bilinear_up_kernel
    c, h, w = 19, 24, 40
    g = torch.Generator().manual_seed(77)
    logits = torch.randn(2, c, h, w, generator=g) * 3
    # near-ties between classes 3 and 11 (11 ahead by a few ulp) on every input pixel
    logits[:, 11] = logits[:, 3] + logits[:, 3].abs() * 2.0 ** -22
    logits[:, 3] += 4.0                     # make them the top two
    logits[:, 11] += 4.0
    upw = torch.from_numpy(bilinear_up_kernel(16)).to(DEV)
    lp, lab = ops.up8_logsoftmax_argmax(logits.to(DEV), upw)
    _, lab8 = ops.up8_logsoftmax_argmax(logits.to(DEV), upw, want_logprobs=False, label_dtype=torch.uint8)
    torch.cuda.synchronize()
    assert torch.equal(lab8.long(), lab)
    assert torch.equal(lab, torch.max(lp, 1)[1])
    assert int((lab == 3).sum()) > 0 and int((lab == 11).sum()) > 0


def test_split3_kernel_matches_engine_split():
    """drnmi_split3_bf16 (the fp32x fine-tune's per-step weight split) == engine.split3_bf16 bit
    for bit, including denormal-range residuals and large magnitudes; w1 + w2 + w3 == w."""
    from drnmi import _lib
    from drnmi.engine import split3_bf16
    g = torch.Generator().manual_seed(77)
    w = (torch.randn(129, 577, generator=g) * torch.logspace(-30, 30, 577).view(1, -1)).float().to(DEV)
    out = torch.empty(3, 129, 577, dtype=torch.bfloat16, device=DEV)
    _lib.check(_lib.load().drnmi_split3_bf16(w.data_ptr(), w.numel(), out.data_ptr(), _lib.stream_ptr(w.device)),
               "split3")
    ref = split3_bf16(w)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    s = out[0].double() + out[1].double() + out[2].double()
    assert (s - w.double()).abs().max().item() <= 2.0 ** -24 * w.double().abs().max().item()
