"""Functional host wrappers of the C-ABI (one call = one HIP launch on the current stream).

These are the per-op entry points (the engine prebuilds the same argument structs once
per plan).  Tensors must already live on the ROCm device; nothing here computes on the
host or falls back to ATen.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .engine import COUT_ALIGN, K_ALIGN, _round_up

_CODE = {torch.float32: _lib.DRNMI_F32, torch.bfloat16: _lib.DRNMI_BF16}


def pack_conv_weight(weight: torch.Tensor, cin_stride: int, dtype: torch.dtype):
    """[cout, cin, k, k] fp32 -> [cout_pad][k_pad] with k = (kh*ks + kw)*cin_stride + ci."""
    cout, cin, kh, kw = weight.shape
    k = kh * kw * cin_stride
    wp = torch.zeros(cout, kh, kw, cin_stride, device=weight.device, dtype=torch.float32)
    wp[..., :cin] = weight.float().permute(0, 2, 3, 1)
    full = torch.zeros(_round_up(cout, COUT_ALIGN), _round_up(k, K_ALIGN), device=weight.device,
                       dtype=torch.float32)
    full[:cout, :k] = wp.reshape(cout, k)
    return full.to(dtype).contiguous(), k


def conv2d_bn_act(x_nhwc: torch.Tensor, weight: torch.Tensor, scale=None, shift=None, residual=None,
                  stride=1, padding=0, dilation=1, relu=False, out_nchw_fp32=False, tile=-1,
                  packed=None, algo=_lib.ALGO_IGEMM, fold_scale=False):
    """y = act(conv(x) * scale + shift [+ residual]) on NHWC x (channel stride = x.shape[3]).
    fold_scale: multiply the scale into the packed weights and launch with scale = NULL."""
    n, h, w, cs = x_nhwc.shape
    cout, cin, ks, _ = weight.shape
    dt = x_nhwc.dtype
    if fold_scale and packed is None:   # (with `packed`, the caller folded the scale already)
        if scale is not None:
            weight = weight * scale.to(weight.device).float().view(-1, 1, 1, 1)
    if packed is None:
        wpk, k = pack_conv_weight(weight, cs, dt)
    else:
        wpk, k = packed
    cout_pad = wpk.shape[0]
    dev = x_nhwc.device
    sc = torch.ones(cout_pad, device=dev)
    sh = torch.zeros(cout_pad, device=dev)
    if scale is not None:
        sc[:cout] = scale.float()
    if shift is not None:
        sh[:cout] = shift.float()
    ho = (h + 2 * padding - dilation * (ks - 1) - 1) // stride + 1
    wo = (w + 2 * padding - dilation * (ks - 1) - 1) // stride + 1
    if out_nchw_fp32:
        y = torch.empty(n, cout, ho, wo, device=dev, dtype=torch.float32)
        strides = (cout * ho * wo, 1, ho * wo)
        out_code = _lib.DRNMI_F32
    else:
        y = torch.empty(n, ho, wo, cout, device=dev, dtype=dt)
        strides = (ho * wo * cout, cout, 1)
        out_code = _CODE[dt]
    a = _lib.ConvArgs()
    a.x, a.wgt, a.shift = x_nhwc.data_ptr(), wpk.data_ptr(), sh.data_ptr()
    a.scale = None if fold_scale else sc.data_ptr()
    a.res = residual.data_ptr() if residual is not None else None
    a.y = y.data_ptr()
    a.y_sn, a.y_sp, a.y_sc = strides
    a.n, a.h, a.w, a.cin = n, h, w, cs
    a.ho, a.wo, a.cout, a.cout_pad = ho, wo, cout, cout_pad
    a.ks, a.stride, a.pad, a.dil = ks, stride, padding, dilation
    a.k, a.k_pad = k, wpk.shape[1]
    a.relu = 1 if relu else 0
    a.dtype, a.out_dtype = _CODE[dt], out_code
    a.tile = tile
    a.algo = algo
    lib = _lib.load()
    _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr(dev))), "conv2d_bn_act")
    return y


def nchw_to_nhwc(x: torch.Tensor, c_pad: int, dtype=torch.float32):
    n, c, h, w = x.shape
    out = torch.empty(n, h, w, c_pad, device=x.device, dtype=dtype)
    lib = _lib.load()
    _lib.check(lib.drnmi_nchw_to_nhwc(x.contiguous().data_ptr(), out.data_ptr(), n, c, h, w, c_pad, _CODE[dtype],
                                      ctypes.c_void_p(_lib.stream_ptr(x.device))), "nchw_to_nhwc")
    return out


def frame_ingest(frames_u8: torch.Tensor, mean, std, bgr=False, dtype=torch.float32):
    n, h, w, _ = frames_u8.shape
    out = torch.empty(n, h, w, 8, device=frames_u8.device, dtype=dtype)
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    lib = _lib.load()
    _lib.check(lib.drnmi_frame_ingest_u8(frames_u8.contiguous().data_ptr(), out.data_ptr(), n, h, w, m, s,
                                         1 if bgr else 0, _CODE[dtype],
                                         ctypes.c_void_p(_lib.stream_ptr(frames_u8.device))), "frame_ingest")
    return out


def up8_logsoftmax_argmax(logits: torch.Tensor, up_plane: torch.Tensor, want_logprobs=True,
                          label_dtype=torch.int64):
    n, c, h, w = logits.shape
    dev = logits.device
    lp = torch.empty(n, c, 8 * h, 8 * w, device=dev, dtype=torch.float32) if want_logprobs else None
    lab = torch.empty(n, 8 * h, 8 * w, device=dev, dtype=label_dtype) if label_dtype is not None else None
    code = _lib.DRNMI_I64 if label_dtype == torch.int64 else _lib.DRNMI_U8
    lib = _lib.load()
    _lib.check(lib.drnmi_up8_logsoftmax_argmax(
        logits.contiguous().data_ptr(), up_plane.float().contiguous().data_ptr(),
        lp.data_ptr() if lp is not None else None, lab.data_ptr() if lab is not None else None,
        code, n, c, h, w, ctypes.c_void_p(_lib.stream_ptr(dev))), "up8_logsoftmax_argmax")
    return lp, lab


def _stem_u8_args(frames_u8, weight, scale, shift, mean, std, bgr, relu, dtype=torch.bfloat16):
    """ConvArgs of the fused-ingest 7x7 stem (PATCH, src_u8) + the tensors they point into.
    dtype: bf16 (stem_dma_kernel) or fp32 (the exact-fp32 patch_f32_kernel)."""
    from .engine import STEM_U8_K
    n, h, w, _ = frames_u8.shape
    cout = weight.shape[0]
    dev = frames_u8.device
    wp = torch.zeros(cout, 7, 8, 4, device=dev)
    wp[:, :, :7, :3] = weight.float().to(dev).permute(0, 2, 3, 1)
    full = torch.zeros(_round_up(cout, COUT_ALIGN), STEM_U8_K, device=dev)
    full[:cout] = wp.reshape(cout, STEM_U8_K)
    wpk = full.to(dtype).contiguous()
    sc = torch.ones(wpk.shape[0], device=dev)
    sh = torch.zeros(wpk.shape[0], device=dev)
    sc[:cout] = scale.float()
    sh[:cout] = shift.float()
    a = _lib.ConvArgs()
    a.x, a.wgt, a.scale, a.shift, a.res = frames_u8.data_ptr(), wpk.data_ptr(), sc.data_ptr(), sh.data_ptr(), None
    a.y_sn, a.y_sp, a.y_sc = h * w * cout, cout, 1
    a.n, a.h, a.w, a.cin = n, h, w, 4
    a.ho, a.wo, a.cout, a.cout_pad = h, w, cout, wpk.shape[0]
    a.ks, a.stride, a.pad, a.dil = 7, 1, 3, 1
    a.k = a.k_pad = STEM_U8_K
    a.relu = 1 if relu else 0
    a.dtype = a.out_dtype = _CODE[dtype]
    a.tile = -1
    a.algo = _lib.ALGO_PATCH
    a.src_u8 = 1
    a.bgr = 1 if bgr else 0
    for i in range(3):
        a.mean[i], a.std[i] = float(mean[i]), float(std[i])
    return a, (wpk, sc, sh)


def stem_u8(frames_u8: torch.Tensor, weight: torch.Tensor, scale, shift, mean, std, bgr=False, relu=True,
            dtype=torch.bfloat16):
    """Fused ingest + 7x7 stem: uint8 [N,H,W,3] -> NHWC [N,H,W,cout] in `dtype` (bf16 patch kernel, or
    fp32: the exact-fp32 patch kernel)."""
    n, h, w, _ = frames_u8.shape
    a, keep = _stem_u8_args(frames_u8, weight, scale, shift, mean, std, bgr, relu, dtype)
    y = torch.empty(n, h, w, weight.shape[0], device=frames_u8.device, dtype=dtype)
    a.y = y.data_ptr()
    lib = _lib.load()
    _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr(frames_u8.device))), "stem_u8")
    return y


def stem_layer1_u8(frames_u8: torch.Tensor, w0: torch.Tensor, scale0, shift0, w1: torch.Tensor, scale1, shift1,
                   mean, std, bgr=False):
    """drnmi_stem_layer1: uint8 frames -> stem 7x7 3->16 + BN + ReLU -> 3x3 16->16 + BN + ReLU in one
    launch (the stem output stays on chip) -> bf16 NHWC [N,H,W,16]."""
    n, h, w, _ = frames_u8.shape
    dev = frames_u8.device
    a0, keep0 = _stem_u8_args(frames_u8, w0, scale0, shift0, mean, std, bgr, True)
    wpk, k = pack_conv_weight(w1, 16, torch.bfloat16)
    sc = torch.ones(wpk.shape[0], device=dev)
    sh = torch.zeros(wpk.shape[0], device=dev)
    sc[:16], sh[:16] = scale1.float(), shift1.float()
    y = torch.empty(n, h, w, 16, device=dev, dtype=torch.bfloat16)
    a1 = _lib.ConvArgs()
    a1.x, a1.wgt, a1.scale, a1.shift, a1.res, a1.y = a0.x, wpk.data_ptr(), sc.data_ptr(), sh.data_ptr(), None, \
        y.data_ptr()
    a1.y_sn, a1.y_sp, a1.y_sc = h * w * 16, 16, 1
    a1.n, a1.h, a1.w, a1.cin, a1.ho, a1.wo, a1.cout, a1.cout_pad = n, h, w, 16, h, w, 16, wpk.shape[0]
    a1.ks, a1.stride, a1.pad, a1.dil, a1.k, a1.k_pad, a1.relu = 3, 1, 1, 1, k, wpk.shape[1], 1
    a1.dtype = a1.out_dtype = _lib.DRNMI_BF16
    a1.tile, a1.algo = -1, _lib.ALGO_PATCH
    lib = _lib.load()
    _lib.check(lib.drnmi_stem_layer1(ctypes.byref(a0), ctypes.byref(a1), ctypes.c_void_p(_lib.stream_ptr(dev))),
               "stem_layer1")
    return y


def resize_bilinear_u8(frames_u8: torch.Tensor, size) -> torch.Tensor:
    """uint8 HWC3 frames [N,H,W,3] -> [N,oh,ow,3] with Pillow's Image.resize(BILINEAR) arithmetic,
    bit-identical (T.Resize((300, 300)) of seg_video_old_no_plot.py:126-127).  size = (oh, ow)."""
    n, h, w, c = frames_u8.shape
    if frames_u8.dtype != torch.uint8 or c != 3:
        raise ValueError("resize_bilinear_u8 expects uint8 [N,H,W,3] frames")
    oh, ow = int(size[0]), int(size[1])
    lib = _lib.load()
    nbytes = lib.drnmi_resize_workspace_bytes(n, h, w, oh, ow, 3)
    if nbytes < 0:
        raise ValueError("resize_bilinear_u8: bad sizes")
    dev = frames_u8.device
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out = torch.empty(n, oh, ow, 3, dtype=torch.uint8, device=dev)
    _lib.check(lib.drnmi_resize_bilinear_u8(frames_u8.contiguous().data_ptr(), n, h, w, out.data_ptr(), oh, ow,
                                            ws.data_ptr(), nbytes, ctypes.c_void_p(_lib.stream_ptr(dev))),
               "resize_bilinear_u8")
    return out


def resize_bilinear_f32(planes: torch.Tensor, size, out: torch.Tensor | None = None,
                        accumulate: bool = False) -> torch.Tensor:
    """fp32 [..., H, W] planes -> [..., oh, ow] with Pillow's 'F'-mode Image.resize(BILINEAR)
    arithmetic (resize_4d_tensor, semantic_seg.py:471-504); accumulate: out += resized."""
    *lead, h, w = planes.shape
    if planes.dtype != torch.float32:
        raise ValueError("resize_bilinear_f32 expects fp32 planes")
    oh, ow = int(size[0]), int(size[1])
    npl = 1
    for d in lead:
        npl *= d
    dev = planes.device
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs out=")
        out = torch.empty(*lead, oh, ow, dtype=torch.float32, device=dev)
    elif tuple(out.shape) != (*lead, oh, ow) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous fp32 tensor of the resized shape")
    lib = _lib.load()
    nbytes = lib.drnmi_resize_workspace_bytes(npl, h, w, oh, ow, 4)
    if nbytes < 0:
        raise ValueError("resize_bilinear_f32: bad sizes")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    _lib.check(lib.drnmi_resize_bilinear_f32(planes.contiguous().data_ptr(), npl, h, w, out.data_ptr(), oh, ow,
                                             1 if accumulate else 0, ws.data_ptr(), nbytes,
                                             ctypes.c_void_p(_lib.stream_ptr(dev))), "resize_bilinear_f32")
    return out


def argmax_nchw(x: torch.Tensor, label_dtype=torch.int64) -> torch.Tensor:
    """numpy x.argmax(axis=1) over fp32 NCHW (first maximum wins) -> [N,H,W] labels."""
    n, c, h, w = x.shape
    lab = torch.empty(n, h, w, dtype=label_dtype, device=x.device)
    code = _lib.DRNMI_U8 if label_dtype == torch.uint8 else _lib.DRNMI_I64
    _lib.check(_lib.load().drnmi_argmax_nchw_f32(x.contiguous().data_ptr(), n, c, h * w, lab.data_ptr(), code,
                                                 ctypes.c_void_p(_lib.stream_ptr(x.device))), "argmax_nchw")
    return lab
