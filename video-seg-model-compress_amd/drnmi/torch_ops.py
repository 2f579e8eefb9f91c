"""PyTorch-ROCm custom ops (`torch.ops.drnmi.*`) over the C-ABI of include/drnmi.h.

The reference's hot path is ATen ops called from Python (lmodels/drnseg.py:295-299 ->
lmodels/drn.py:213-259, pruners/Pruner.py:17-20, semantic_seg.py:445).  drnmi exposes the same
work as registered torch operators, so it composes with the dispatcher like any ATen op:
  * each op has a fake (meta) kernel: FakeTensorMode / torch.compile tracing sees the output
    shapes and dtypes without a GPU;
  * the real kernels are registered for the "cuda" (= ROCm HIP) device only: calling an op on a
    CPU tensor raises (there is no CPU fallback by design);
  * every launch goes to the current stream, so `torch.cuda.graph` captures a whole
    `segment()` and replays it.

Ops (schema -> reference):
  drnmi::conv2d_bn_act(Tensor x_nhwc, Tensor w_packed, Tensor? scale, Tensor shift,
                       Tensor? residual, int cout, int ks, int stride, int pad, int dil,
                       bool relu, bool out_nchw_fp32) -> Tensor
      conv3x3/1x1/7x7 + BatchNorm (eval, folded) + residual + ReLU
      (lmodels/drn.py:27-29, :49-65, :86-106, :132-137, :181-186, :201-211; drnseg.py:278-284)
  drnmi::up8_logsoftmax_argmax(Tensor logits, Tensor up_plane, bool emit_logprobs,
                               bool labels_u8) -> (Tensor labels, Tensor logprobs)
      up (ConvTranspose2d k16 s8 p4, bilinear) + LogSoftmax + torch.max(., 1)
      (lmodels/drnseg.py:257-299, semantic_seg.py:445); logprobs is empty when not emitted
  drnmi::mask_apply_(Tensor(a!)[] weights, Tensor[] masks) -> ()
      Pruner.apply_masks: w *= mask in place (pruners/Pruner.py:17-20)
  drnmi::segment(Tensor frames_u8, int model, float[] mean, float[] std, bool bgr) -> Tensor
      the seg_video per-frame loop body (seg_video_old_no_plot.py:157-169): normalise ->
      model(img)[0] -> torch.max(final, 1), uint8 labels
  drnmi::forward(Tensor x, int model) -> (Tensor log_probs, Tensor logits)
      DRNSeg.forward in eval mode (lmodels/drnseg.py:295-299)
  drnmi::predict(Tensor x, int model) -> Tensor
      torch.max(model(x)[0], 1)[1] (semantic_seg.py:444-445), int64 labels
`model` is the handle of a live drnmi.drnseg.DRNSeg (its packed weights and launch plans are
the op's state; DRNSeg.segment / forward / predict pass their own handle).
"""
from __future__ import annotations

import ctypes
import itertools
import weakref

import torch

from . import _lib

_CODE = {torch.float32: _lib.DRNMI_F32, torch.bfloat16: _lib.DRNMI_BF16}

# ------------------------------------------------------------------ model handles
_MODELS: dict[int, weakref.ref] = {}
_NEXT = itertools.count(1)


def register_model(model) -> int:
    h = next(_NEXT)
    _MODELS[h] = weakref.ref(model, lambda _r, h=h: _MODELS.pop(h, None))
    return h


def _model(handle: int):
    ref = _MODELS.get(int(handle))
    m = ref() if ref is not None else None
    if m is None:
        raise RuntimeError(f"drnmi: model handle {handle} is not live")
    return m


def _conv_out(h, k, s, p, d):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1


# ------------------------------------------------------------------ conv2d_bn_act
@torch.library.custom_op("drnmi::conv2d_bn_act", mutates_args=(), device_types="cuda")
def conv2d_bn_act(x_nhwc: torch.Tensor, w_packed: torch.Tensor, scale: torch.Tensor | None,
                  shift: torch.Tensor, residual: torch.Tensor | None, cout: int, ks: int, stride: int, pad: int,
                  dil: int, relu: bool, out_nchw_fp32: bool) -> torch.Tensor:
    n, h, w, cs = x_nhwc.shape
    if x_nhwc.dtype not in _CODE or w_packed.dtype != x_nhwc.dtype:
        raise TypeError("drnmi::conv2d_bn_act: x and w_packed must share dtype fp32 or bf16")
    k = ks * ks * cs
    if w_packed.dim() != 2 or w_packed.shape[0] < cout or w_packed.shape[1] < k:
        raise ValueError(f"drnmi::conv2d_bn_act: w_packed {tuple(w_packed.shape)} too small for cout {cout}, k {k}")
    if shift.dtype != torch.float32 or shift.numel() < w_packed.shape[0]:
        raise ValueError("drnmi::conv2d_bn_act: shift must be fp32 [cout_pad]")
    if scale is not None and (scale.dtype != torch.float32 or scale.numel() < w_packed.shape[0]):
        raise ValueError("drnmi::conv2d_bn_act: scale must be fp32 [cout_pad]")
    ho, wo = _conv_out(h, ks, stride, pad, dil), _conv_out(w, ks, stride, pad, dil)
    x = x_nhwc.contiguous()
    if out_nchw_fp32:
        y = torch.empty(n, cout, ho, wo, device=x.device, dtype=torch.float32)
        strides, out_code = (cout * ho * wo, 1, ho * wo), _lib.DRNMI_F32
    else:
        y = torch.empty(n, ho, wo, cout, device=x.device, dtype=x.dtype)
        strides, out_code = (ho * wo * cout, cout, 1), _CODE[x.dtype]
    if residual is not None and (residual.dtype != x.dtype or residual.numel() != n * ho * wo * cout):
        raise ValueError("drnmi::conv2d_bn_act: residual must be NHWC [n, ho, wo, cout] in x's dtype")
    a = _lib.ConvArgs()
    a.x, a.wgt = x.data_ptr(), w_packed.data_ptr()
    a.scale = scale.data_ptr() if scale is not None else None
    a.shift = shift.data_ptr()
    a.res = residual.contiguous().data_ptr() if residual is not None else None
    a.y = y.data_ptr()
    a.y_sn, a.y_sp, a.y_sc = strides
    a.n, a.h, a.w, a.cin = n, h, w, cs
    a.ho, a.wo, a.cout, a.cout_pad = ho, wo, cout, w_packed.shape[0]
    a.ks, a.stride, a.pad, a.dil = ks, stride, pad, dil
    a.k, a.k_pad = k, w_packed.shape[1]
    a.relu = 1 if relu else 0
    a.dtype, a.out_dtype = _CODE[x.dtype], out_code
    a.tile, a.algo = -1, _lib.ALGO_IGEMM
    _lib.check(_lib.load().drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(_lib.stream_ptr(x.device))),
               "drnmi::conv2d_bn_act")
    return y


@conv2d_bn_act.register_fake
def _(x_nhwc, w_packed, scale, shift, residual, cout, ks, stride, pad, dil, relu, out_nchw_fp32):
    n, h, w, _ = x_nhwc.shape
    ho, wo = _conv_out(h, ks, stride, pad, dil), _conv_out(w, ks, stride, pad, dil)
    if out_nchw_fp32:
        return x_nhwc.new_empty((n, cout, ho, wo), dtype=torch.float32)
    return x_nhwc.new_empty((n, ho, wo, cout))


# ------------------------------------------------------------------ head
@torch.library.custom_op("drnmi::up8_logsoftmax_argmax", mutates_args=(), device_types="cuda")
def up8_logsoftmax_argmax(logits: torch.Tensor, up_plane: torch.Tensor, emit_logprobs: bool,
                          labels_u8: bool) -> tuple[torch.Tensor, torch.Tensor]:
    if logits.dtype != torch.float32 or logits.dim() != 4:
        raise TypeError("drnmi::up8_logsoftmax_argmax: logits must be fp32 NCHW")
    if up_plane.shape != (16, 16) or up_plane.dtype != torch.float32:
        raise ValueError("drnmi::up8_logsoftmax_argmax: up_plane must be fp32 [16, 16]")
    n, c, h, w = logits.shape
    dev = logits.device
    lab = torch.empty(n, 8 * h, 8 * w, device=dev, dtype=torch.uint8 if labels_u8 else torch.int64)
    lp = torch.empty((n, c, 8 * h, 8 * w) if emit_logprobs else (0,), device=dev, dtype=torch.float32)
    _lib.check(_lib.load().drnmi_up8_logsoftmax_argmax(
        logits.contiguous().data_ptr(), up_plane.contiguous().data_ptr(), lp.data_ptr() if emit_logprobs else None,
        lab.data_ptr(), _lib.DRNMI_U8 if labels_u8 else _lib.DRNMI_I64, n, c, h, w,
        ctypes.c_void_p(_lib.stream_ptr(dev))), "drnmi::up8_logsoftmax_argmax")
    return lab, lp


@up8_logsoftmax_argmax.register_fake
def _(logits, up_plane, emit_logprobs, labels_u8):
    n, c, h, w = logits.shape
    lab = logits.new_empty((n, 8 * h, 8 * w), dtype=torch.uint8 if labels_u8 else torch.int64)
    lp = logits.new_empty((n, c, 8 * h, 8 * w) if emit_logprobs else (0,))
    return lab, lp


# ------------------------------------------------------------------ mask apply
@torch.library.custom_op("drnmi::mask_apply_", mutates_args=("weights",), device_types="cuda")
def mask_apply_(weights: list[torch.Tensor], masks: list[torch.Tensor]) -> None:
    """w *= m for every pair, one launch; masks fp32 (weight-shaped) or int32 bit words
    (bit i of word i/32, drnmi_mask_apply_bits_f32)."""
    if len(weights) != len(masks) or not weights:
        raise ValueError("drnmi::mask_apply_: need matching non-empty weight / mask lists")
    bits = masks[0].dtype == torch.int32
    for w, m in zip(weights, masks):
        if w.dtype != torch.float32 or not w.is_contiguous():
            raise TypeError("drnmi::mask_apply_: weights must be contiguous fp32")
        if (m.dtype == torch.int32) != bits or not m.is_contiguous() or m.device != w.device:
            raise TypeError("drnmi::mask_apply_: masks must all be fp32 or all int32 bit words, on the weight's device")
        need = (w.numel() + 31) // 32 if bits else w.numel()
        if m.numel() != need or (not bits and m.dtype != torch.float32):
            raise ValueError("drnmi::mask_apply_: mask size does not match its weight")
    k = len(weights)
    lib = _lib.load()
    fn = lib.drnmi_mask_apply_bits_f32 if bits else lib.drnmi_mask_apply_f32
    _lib.check(fn(k, (ctypes.c_void_p * k)(*[w.data_ptr() for w in weights]),
                  (ctypes.c_void_p * k)(*[m.data_ptr() for m in masks]),
                  (ctypes.c_int64 * k)(*[w.numel() for w in weights]),
                  ctypes.c_void_p(_lib.stream_ptr(weights[0].device))), "drnmi::mask_apply_")


@mask_apply_.register_fake
def _(weights, masks):
    return None


# ------------------------------------------------------------------ whole-network ops
def _out_hw(model, h: int, w: int):
    """Label-map size of DRNSeg at input h x w: 8 x the 1/8-resolution logits size (300 -> 304)."""
    shapes = {"input": (h, w)}
    for nd in model._graph.nodes:          # follow the value graph (downsample branches too)
        c = nd.conv
        ih, iw = shapes[nd.src]
        shapes[nd.dst] = (_conv_out(ih, c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0]),
                          _conv_out(iw, c.kernel_size[1], c.stride[1], c.padding[1], c.dilation[1]))
    lh, lw = shapes["logits"]
    return 8 * lh, 8 * lw, lh, lw


@torch.library.custom_op("drnmi::segment", mutates_args=(), device_types="cuda")
def segment(frames_u8: torch.Tensor, model: int, mean: list[float], std: list[float], bgr: bool) -> torch.Tensor:
    return _model(model)._segment_impl(frames_u8, mean, std, bgr, None)


@segment.register_fake
def _(frames_u8, model, mean, std, bgr):
    n, h, w, _ = frames_u8.shape
    oh, ow, _, _ = _out_hw(_model(model), h, w)
    return frames_u8.new_empty((n, oh, ow), dtype=torch.uint8)


@torch.library.custom_op("drnmi::forward", mutates_args=(), device_types="cuda")
def forward(x: torch.Tensor, model: int) -> tuple[torch.Tensor, torch.Tensor]:
    return _model(model)._forward_impl(x)


@forward.register_fake
def _(x, model):
    m = _model(model)
    n, _, h, w = x.shape
    oh, ow, lh, lw = _out_hw(m, h, w)
    return (x.new_empty((n, m.classes, oh, ow), dtype=torch.float32),
            x.new_empty((n, m.classes, lh, lw), dtype=torch.float32))


@torch.library.custom_op("drnmi::predict", mutates_args=(), device_types="cuda")
def predict(x: torch.Tensor, model: int) -> torch.Tensor:
    return _model(model)._predict_impl(x)


@predict.register_fake
def _(x, model):
    n, _, h, w = x.shape
    oh, ow, _, _ = _out_hw(_model(model), h, w)
    return x.new_empty((n, oh, ow), dtype=torch.int64)


__all__ = ["conv2d_bn_act", "up8_logsoftmax_argmax", "mask_apply_", "segment", "forward", "predict",
           "register_model"]
