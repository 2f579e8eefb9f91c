"""DRNSeg — drop-in for the reference segmentation module, run on HIP kernels.

Reference API (kept): semantic_seg.py:126-164 / lmodels/drnseg.py:268-305
  DRNSeg(model_name, classes, pretrained_model=None, pretrained=True, use_torch_up=False)
  forward(x: fp32 [B,3,H,W]) -> (log_probs fp32 [B,C,8h,8w], logits fp32 [B,C,h,w])
  optim_parameters()  -> layer + seg params (up excluded)
  state_dict keys     layer.{0..8}.*, seg.weight, seg.bias, up.weight
                      (load_state_dict also accepts the seg_video "base." prefix,
                       log.txt:18-170, and a DataParallel/DDP "module." prefix)

Differences by design:
  * forward runs the fused HIP plan (drnmi.engine) on a ROCm device, as the registered
    custom op torch.ops.drnmi.forward (drnmi.torch_ops; also .predict / .segment).  It never
    falls back to ATen; on CPU it raises.  In train mode it runs the fine-tune path
    (drnmi.train: batch-stat BN, autograd through the HIP backward kernels, fp32).
  * use_torch_up=True keeps the reference's nn.UpsamplingBilinear2d(scale_factor=8) head
    (lmodels/drnseg.py:285-287: bilinear, align_corners=True, output 8h x 8w) on its own
    fused HIP kernel (drnmi_up8_bilinear_logsoftmax_argmax).
  * precision: "fp32" (default; the reference's arithmetic, parity mode, exact-fp32
    MFMA), "fp32x" (fp32-accurate arithmetic on the bf16 MFMA pipe: exact 3-way bf16 splits,
    6 products, for every conv with cin >= 32; parity gates as fp32, ~3x faster), "bf16"
    (perf mode, fp32 accumulation) or "int8" (W8A8 for the cin >= 64 convs,
    config C5; needs calibrate_int8() first — the reference has no quantisation, so this
    mode is ours) via set_precision().
  * segment(frames_u8) is the fused seg_video path (seg_video_old_no_plot.py:157-169:
    normalise -> model(img)[0] -> torch.max(final, 1)) producing uint8 labels without
    materialising the 19-plane log-prob tensor.
  * model_name is honoured (lmodels/drnseg.py:272 always builds D-22; semantic_seg.py
    :130-131 builds model_name — we follow the driver copy).
"""
from __future__ import annotations

import json
import math
import os

import torch
import torch.nn as nn

from . import _lib, drn, torch_ops
from .engine import PackedNet, Plan, lower_drnseg
from .weights import bilinear_up_kernel

# info.json:1 (Cityscapes normalisation used by every reference driver)
INFO_MEAN = (0.29010095242892997, 0.32808144844279574, 0.28696394422942517)
INFO_STD = (0.1829540508368939, 0.18656561047509476, 0.18447508988480435)


def fill_up_weights(up: nn.ConvTranspose2d) -> None:
    """Bilinear kernel into every depthwise plane (lmodels/drnseg.py:257-266)."""
    k = up.weight.shape[2]
    w = torch.from_numpy(bilinear_up_kernel(k))
    with torch.no_grad():
        up.weight.copy_(w.expand_as(up.weight))


class DRNSeg(nn.Module):
    def __init__(self, model_name, classes, pretrained_model=None, pretrained=True,
                 use_torch_up=False):
        super().__init__()
        factory = getattr(drn, model_name, None)
        if factory is None:
            raise KeyError(f"unknown model {model_name!r}; known: {drn.ARCHS}")
        model = factory(pretrained=pretrained, num_classes=1000)
        if pretrained_model is not None:
            model.load_state_dict(pretrained_model)
        self.layer = nn.Sequential(*list(model.children())[:-2])
        self.seg = nn.Conv2d(model.out_dim, classes, kernel_size=1, bias=True)
        self.softmax = nn.LogSoftmax(dim=1)
        n = self.seg.kernel_size[0] * self.seg.kernel_size[1] * self.seg.out_channels
        self.seg.weight.data.normal_(0, math.sqrt(2.0 / n))
        self.seg.bias.data.zero_()
        if use_torch_up:
            self.up = nn.UpsamplingBilinear2d(scale_factor=8)
        else:
            up = nn.ConvTranspose2d(classes, classes, 16, stride=8, padding=4, output_padding=0,
                                    groups=classes, bias=False)
            fill_up_weights(up)
            up.weight.requires_grad = False
            self.up = up
        self.use_torch_up = bool(use_torch_up)
        self.model_name = model_name
        self.classes = classes
        self.precision = "fp32"
        self.block_sparse = False    # opt-in: measured slower than dense below ~60 % zero units
        self._graph = lower_drnseg(self.layer, self.seg)
        self._act_scales = None      # int8: per-value activation scales (calibrate_int8)
        self._packed = {}
        self._plans = {}
        self._pack_key = None
        self._key_tensors = None     # cached parameter/buffer list of the repack key
        self._key_ids = None         # ids of the parameter/buffer/submodule objects it was built from
        self._key_dicts = []         # the modules' _parameters/_buffers/_modules dicts behind them
        self.timing_hook = None      # optional per-launch callback (bench.py's HIP events)
        self._handle = torch_ops.register_model(self)   # torch.ops.drnmi.* state handle

    # copies and unpickled modules register a handle of their own: the handle keys the
    # torch.ops.drnmi.* state, and a copied integer would dispatch to the ORIGINAL model's
    # weights.  Packed weights and launch plans hold device pointers of this instance: not copied.
    def __getstate__(self):
        st = self.__dict__.copy()
        st.pop("_handle", None)
        st.update(_packed={}, _plans={}, _pack_key=None, _key_tensors=None, _key_ids=None, _key_dicts=[],
                  timing_hook=None)
        st.pop("_train_runner", None)
        return st

    def __setstate__(self, st):
        super().__setstate__(st)
        self._handle = torch_ops.register_model(self)

    # ----------------------------------------------------------------- reference API
    def optim_parameters(self, memo=None):
        for param in self.layer.parameters():
            yield param
        for param in self.seg.parameters():
            yield param

    def forward(self, x: torch.Tensor):
        if self.training:
            # fine-tune path: batch-stat BN + autograd through the HIP backward kernels
            if x.device.type != "cuda":
                raise RuntimeError("drnmi.DRNSeg runs on the HIP engine only (no CPU fallback by design)")
            if self.precision not in ("fp32", "fp32x"):
                raise NotImplementedError("the fine-tune path runs in fp32 (the reference's arithmetic) or fp32x "
                                          "(fp32-accurate split-bf16 forward/dgrad convs)")
            from .train import train_forward
            return train_forward(self, x)
        if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] != 3:
            raise ValueError("DRNSeg.forward expects fp32 [B,3,H,W]")
        self._check_device(x)
        return torch.ops.drnmi.forward(x, self._handle)

    # ----------------------------------------------------------------- fused paths
    def predict(self, x: torch.Tensor) -> torch.Tensor:
        """torch.max(model(x)[0], 1)[1] (semantic_seg.py:444-445) as one fused pass: int64 labels."""
        if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] != 3:
            raise ValueError("DRNSeg.predict expects fp32 [B,3,H,W]")
        self._check_device(x)
        return torch.ops.drnmi.predict(x, self._handle)

    def segment(self, frames_u8: torch.Tensor, mean=INFO_MEAN, std=INFO_STD, bgr: bool = False,
                labels: torch.Tensor | None = None, size=None) -> torch.Tensor:
        """Video path: uint8 HWC frames [B,H,W,3] on the GPU -> uint8 label maps [B,8h,8w].

        Fuses ToTensorVideoImage + Normalize (data_transforms.py:256-281, :109-125) into the
        ingest kernel and model(img)[0] + torch.max(final,1) into the head kernel.  Runs as
        torch.ops.drnmi.segment (graph-capturable); `labels=` writes into a caller buffer.
        size=(oh, ow): first resize the frames on the GPU exactly as seg_video's
        T.Resize((300, 300)) does on each PIL frame (seg_video_old_no_plot.py:126-127;
        Pillow BILINEAR arithmetic, drnmi_resize_bilinear_u8)."""
        if frames_u8.dtype != torch.uint8 or frames_u8.dim() != 4 or frames_u8.shape[3] != 3:
            raise ValueError("segment expects uint8 [B,H,W,3] frames")
        self._check_device(frames_u8)
        if size is not None and tuple(size) != tuple(frames_u8.shape[1:3]):
            from .ops import resize_bilinear_u8
            frames_u8 = resize_bilinear_u8(frames_u8, size)
        if labels is not None:
            return self._segment_impl(frames_u8, mean, std, bgr, labels)
        return torch.ops.drnmi.segment(frames_u8, self._handle, [float(v) for v in mean],
                                       [float(v) for v in std], bool(bgr))

    # bodies of the torch.ops.drnmi ops (drnmi/torch_ops.py)
    def _forward_impl(self, x: torch.Tensor):
        plan, stream = self._prepare(x.shape[0], x.shape[2], x.shape[3], x.device)
        x = x.contiguous()
        plan.ingest_nchw(x, stream)
        plan.run_backbone(stream, self.timing_hook)
        oh, ow = plan.out_hw
        logprobs = torch.empty(x.shape[0], self.classes, oh, ow, dtype=torch.float32, device=x.device)
        self._head(plan, stream, logprobs, None)
        logits = plan.bufs["logits"].clone()
        return logprobs, logits

    def _predict_impl(self, x: torch.Tensor) -> torch.Tensor:
        plan, stream = self._prepare(x.shape[0], x.shape[2], x.shape[3], x.device)
        plan.ingest_nchw(x.contiguous(), stream)
        plan.run_backbone(stream, self.timing_hook)
        oh, ow = plan.out_hw
        labels = torch.empty(x.shape[0], oh, ow, dtype=torch.int64, device=x.device)
        self._head(plan, stream, None, labels)
        return labels

    def _segment_impl(self, frames_u8, mean, std, bgr, labels):
        plan, stream = self._prepare(frames_u8.shape[0], frames_u8.shape[1], frames_u8.shape[2],
                                     frames_u8.device)
        plan.ingest_u8(frames_u8.contiguous(), mean, std, bgr, stream)
        path = plan.labels_path(self.use_torch_up)
        plan.run_backbone(stream, self.timing_hook, labels_only=path != "nchw")
        oh, ow = plan.out_hw
        if labels is None:
            labels = torch.empty(frames_u8.shape[0], oh, ow, dtype=torch.uint8, device=frames_u8.device)
        elif labels.shape != (frames_u8.shape[0], oh, ow) or labels.dtype not in (torch.uint8, torch.int64) \
                or not labels.is_contiguous() or labels.device != frames_u8.device:
            raise ValueError(f"labels must be a contiguous uint8/int64 [{frames_u8.shape[0]}, {oh}, {ow}] tensor "
                             f"on {frames_u8.device}")
        hook, head_idx = self.timing_hook, len(plan.packed.graph.nodes)   # (the head's launch index)
        if hook is not None:
            hook(head_idx, None, True)
        if path == "seg2":
            plan.head_labels_seg2(self._up_plane(plan.packed.device), stream, labels)
        elif path == "nhwc":
            plan.head_labels_nhwc(self._up_plane(plan.packed.device), stream, labels)
        else:
            self._head(plan, stream, None, labels)
        if hook is not None:
            hook(head_idx, None, False)
        return labels

    def _head(self, plan, stream, logprobs, labels):
        if self.use_torch_up:
            plan.head_bilinear(stream, logprobs, labels)
        else:
            plan.head(self._up_plane(plan.packed.device), stream, logprobs, labels)

    @staticmethod
    def _check_device(t: torch.Tensor):
        if t.device.type != "cuda":
            raise RuntimeError("drnmi.DRNSeg runs on the HIP engine only: move the model and input "
                               "to a ROCm device (no CPU fallback by design)")

    # ----------------------------------------------------------------- configuration
    def set_precision(self, precision: str) -> "DRNSeg":
        if precision not in ("fp32", "fp32x", "bf16", "int8"):
            raise ValueError("precision must be 'fp32', 'fp32x', 'bf16' or 'int8'")
        self.precision = precision
        return self

    @torch.no_grad()
    def calibrate_int8(self, frames_u8: torch.Tensor, mean=INFO_MEAN, std=INFO_STD, bgr: bool = False):
        """Per-tensor activation scales for precision "int8": the bf16 engine runs the
        calibration frames (uint8 [B,H,W,3] on the GPU) and every activation's scale is
        absmax / 127 (drnmi_absmax on the HBM buffer).  Re-packs the int8 weights."""
        import ctypes
        prev = self.precision
        self.precision = "bf16"
        try:
            plan, stream = self._prepare(frames_u8.shape[0], frames_u8.shape[1], frames_u8.shape[2],
                                         frames_u8.device, keep_all=True)
            plan.ingest_u8(frames_u8.contiguous(), mean, std, bgr, stream)
            plan.run_backbone(stream)
            lib = _lib.load()
            amax = torch.empty(1, dtype=torch.float32, device=frames_u8.device)
            scales = {}
            values = set(plan.packed.graph.channels)             # graph values only (not the
            for v, buf in plan.bufs.items():                      # head's logits_nhwc / seg_part buffers)
                if v in ("input", "logits") or v not in values:
                    continue
                _lib.check(lib.drnmi_absmax(buf.data_ptr(), _lib.DRNMI_BF16, buf.numel(), amax.data_ptr(),
                                            ctypes.c_void_p(stream)), "absmax")
                a = float(amax.item())
                scales[v] = a / 127.0 if a > 0 else 1.0
        finally:
            self.precision = prev
            self._plans = {k: p for k, p in self._plans.items() if not k[-1]}   # drop the keep_all plan
        self._act_scales = scales
        self._packed.pop("int8", None)
        self._plans = {k: p for k, p in self._plans.items() if k[0] != "int8"}
        self._pack_key = None
        return scales

    def set_block_sparse(self, enabled: bool) -> "DRNSeg":
        """bf16: let pruned (all-zero) 16 x 32 weight units skip their MFMAs (opt-in; results are
        bit-identical either way; layers with < SPARSE_MIN_ZERO_UNITS zero units stay dense).
        Takes effect at the next pack."""
        self.block_sparse = bool(enabled)
        for pk in self._packed.values():
            pk.block_sparse = self.block_sparse
        self._pack_key = None
        return self

    def plan(self, n, h, w, device=None, keep_all=False) -> Plan:
        device = device or next(self.parameters()).device
        plan, _ = self._prepare(n, h, w, torch.device(device), keep_all=keep_all)
        return plan

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self._key_tensors = None
        fixed = {}
        for k, v in state_dict.items():
            if k.startswith("module."):
                k = k[len("module."):]
            if k.startswith("base."):
                k = "layer." + k[len("base."):]
            fixed[k] = v
        return super().load_state_dict(fixed, strict=strict, assign=assign)

    # ----------------------------------------------------------------- internals
    def _up_plane(self, device):
        return self.up.weight[0, 0].detach().to(device, torch.float32).contiguous()

    def _apply(self, fn, *args, **kwargs):
        self._key_tensors = None          # .to() / .cuda() / .float() may swap tensors
        return super()._apply(fn, *args, **kwargs)

    def _state_key(self):
        """Repack key: every parameter/buffer's storage and version counter (an in-place update
        -- optimizer step, apply_masks, load_state_dict -- bumps the version).  The tensor list
        is cached (building it cost ~0.6 ms per call); _apply / load_state_dict reset it, and a
        Parameter or buffer swapped in anywhere in the tree (conv.weight = nn.Parameter(...))
        changes the object ids checked here, which rebuilds it."""
        ts = self._key_tensors
        ids = tuple(id(v) for d in self._key_dicts for v in d.values()) if ts is not None else None
        if ts is None or ids != self._key_ids:
            ts = self._key_tensors = list(self.parameters()) + list(self.buffers())
            self._key_dicts = [d for mod in self.modules() for d in (mod._parameters, mod._buffers, mod._modules)]
            self._key_ids = tuple(id(v) for d in self._key_dicts for v in d.values())
        return (self.precision, tuple((t.data_ptr(), t._version) for t in ts))

    def _prepare(self, n, h, w, device, keep_all=False):
        if device.type != "cuda":
            raise RuntimeError("drnmi.DRNSeg runs on the HIP engine only: move the model and input "
                               "to a ROCm device (no CPU fallback by design)")
        if self.training:
            raise RuntimeError("predict()/segment() are inference paths: call .eval() first "
                               "(train-mode forward is DRNSeg.forward)")
        _lib.load()
        key = self._state_key()
        if key != self._pack_key:
            if self.precision in self._packed:
                self._packed[self.precision].pack()
                for pkey, plan in list(self._plans.items()):
                    if pkey[0] == self.precision:
                        try:
                            plan.refresh_weight_ptrs()
                        except RuntimeError:      # the repack changed the plan's launch structure
                            del self._plans[pkey]
            self._pack_key = key
        if self.precision == "int8" and self._act_scales is None:
            raise RuntimeError("precision 'int8' needs activation scales: call calibrate_int8(frames) first")
        pk = self._packed.get(self.precision)
        if pk is None:
            pk = PackedNet(self._graph, self.precision, device, block_sparse=self.block_sparse,
                           act_scales=self._act_scales)
            self._packed[self.precision] = pk
        pkey = (self.precision, n, h, w, keep_all)
        plan = self._plans.get(pkey)
        if plan is None:
            plan = Plan(pk, n, h, w, keep_all=keep_all)
            self._plans[pkey] = plan
        return plan, _lib.stream_ptr(device)


def load_info(path: str):
    with open(path) as f:
        info = json.load(f)
    return tuple(info["mean"]), tuple(info["std"])


def build(model_name: str = "drn_d_22", classes: int = 19, seed: int | None = 0, device="cuda",
          precision: str = "fp32") -> DRNSeg:
    """DRNSeg with hash-initialised weights (drnmi.weights), in eval mode, on `device`."""
    from .weights import synth_state_dict
    m = DRNSeg(model_name, classes, pretrained=False)
    if seed is not None:
        m.load_state_dict(synth_state_dict(m, seed))
    return m.to(device).eval().set_precision(precision)


__all__ = ["DRNSeg", "fill_up_weights", "build", "INFO_MEAN", "INFO_STD", "load_info",
           "os"]
