"""Fine-tune path: train-mode DRNSeg forward/backward, CrossEntropyLoss, SGD — on HIP kernels.

Reference training step (semantic_seg.py:166-230):

    model.train()
    output = model(input)[0]                      # DRNSeg.forward, BN on batch statistics
    loss = criterion(output, target)              # CrossEntropyLoss(ignore_index=255), :817
    optimizer.zero_grad(); loss.backward()        # autograd through ~70 ATen ops
    optimizer.step()                              # SGD(momentum, weight_decay), :963-966
    if pruner: pruner.apply_masks(model)          # :213-214

Here the same step keeps that exact user-facing shape: `DRNSeg.forward` in train mode is one
autograd.Function whose forward runs the fp32 HIP plan (conv -> batch-stat BN -> ReLU/residual
per node, then up x8 + LogSoftmax) and whose backward runs the HIP backward kernels in reverse
node order (include/drnmi.h "Fine-tune path"), writing every parameter's .grad directly.  A
gradient-ready callback per node lets the data-parallel wrapper (drnmi.parallel) launch the
bucketed RCCL all-reduce of finished buckets while earlier layers are still in backward.
`CrossEntropyLoss` and `SGD` below are the HIP drop-ins for the criterion and optimizer (the
optimizer can fuse the pruner's mask into the update: `SGD(..., pruner=p)`).

Precision: fp32 (the reference trains in fp32; model.set_precision("fp32"), the default) or
"fp32x": the forward and data-gradient convs with >= 32 input channels run on the fp32-accurate
split-bf16 kernel (csrc/conv_x6.hip: exact 3-way bf16 split of weights and activations, the six
products above 2^-24, fp32 accumulation, 2.5 PF / 6 peak) instead of the exact-f32 MFMA
(157 TF), and so do their weight gradients (drnmi_conv_wgrad_f32x3, the same split on dy and x);
BN, the head and the small-channel convs stay exact fp32.
Activations NHWC with a power-of-two channel stride, like the inference engine.  There is no
CPU or ATen fallback.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from .engine import COUT_ALIGN, K_ALIGN, X6_PATCH_SHAPES, _conv_out, _pow2_at_least, _round_up

F32 = _lib.DRNMI_F32
# TrainRunner default (tests switch it off to compare against the per-layer packs)
BATCHED_PACK = True
# BN batch statistics from the conv_x6 epilogue where the launch can write them (tests switch it
# off to compare against the separate statistics pass over y)
FUSED_BN_STATS = True
# fp32x data gradient of a stride-2 conv as four parity-class convs of dy (tests switch it off to
# compare against the zero-inserted conv, which it reproduces bit for bit when neither splits K)
S2_CLASS_DGRAD = True
# conv_x6 training launches may split K where their tiles leave CUs idle (tests switch it off for
# bit-for-bit comparisons of launch forms: a split sums the same products in another association)
X6_SPLIT_K = True


def _vp(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class _NodeState:
    """Per-node packed weights (forward / dgrad layouts) cached across steps."""

    __slots__ = ("wf", "wd", "wfx", "wdx", "k", "k_pad", "cout_pad", "kd", "kd_pad", "rows_d", "shift", "patch",
                 "dpatch", "dys", "s2_step", "s2_cls", "s2_planes")

    def __init__(self):
        self.wf = self.wd = self.wfx = self.wdx = self.shift = None
        self.patch = self.dpatch = False
        self.dys = None
        self.s2_step = self.s2_cls = self.s2_planes = None   # stride-2 dgrad parity classes (per step)


class TrainRunner:
    """Executes one DRNSeg's train-mode forward and backward on the HIP kernels."""

    def __init__(self, model):
        self.model = model
        self.graph = model._graph
        self.cstride = {"input": 8}
        for v, c in self.graph.channels.items():
            if v != "input":
                self.cstride[v] = _pow2_at_least(c)
        self.nodes = self.graph.nodes
        self.state = [_NodeState() for _ in self.nodes]
        self._red_ws = None
        self._wg_ws = None
        self._cv_ws = None
        self._st_ws = None
        self._step_id = 0               # backward passes run (keys the per-step stride-2 class planes)
        self._zeros = None
        self.grad_ready = None          # callback(list[Parameter]) after each node's grads land
        self.grad_scale = 1.0           # multiplies dL/dlogprobs (DDP averaging: 1 / world_size)
        self._flat = None               # flat gradient buffer (views = param.grad)
        self._flat_params = None
        self.debug_value_grads = None   # dict -> filled with {value: NHWC grad clone} (diagnostics)
        # batched re-pack (drnmi_pack_conv_weights_batched): after the first step has allocated every
        # packed buffer, each forward re-packs all forward and dgrad weights (+ fp32x planes) in one
        # launch instead of ~4 launches per layer; the table is rebuilt when a buffer moves
        self.batched_pack = BATCHED_PACK
        self._pack_key = None
        self._pack_prec = None
        self._pack_tab = None
        self._pack_total = 0
        self._packed_now = False

    # ------------------------------------------------------------------ helpers
    def _ws(self, attr, nbytes, device):
        buf = getattr(self, attr)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            setattr(self, attr, buf)
        return buf

    def _zeros_f32(self, n, device):
        if self._zeros is None or self._zeros.numel() < n:
            self._zeros = torch.zeros(max(n, 4096), dtype=torch.float32, device=device)
        return self._zeros

    def ordered_params(self):
        """Parameters in the order backward finishes them (seg first, then nodes reversed)."""
        out = []
        for nd in reversed(self.nodes):
            ps = [nd.conv.weight] + ([nd.conv.bias] if nd.conv.bias is not None else [])
            if nd.bn is not None:
                ps += [nd.bn.weight, nd.bn.bias]
            out += [p for p in ps if p is not None]
        return out

    def _ensure_flat_grads(self, device):
        """param.grad of every trainable parameter is a view of one flat fp32 buffer laid out
        in backward order (contiguous all-reduce buckets).  Returns {param: accumulate?}."""
        params = [p for p in self.ordered_params() if p.requires_grad]
        if self._flat_params is None or [id(p) for p in self._flat_params] != [id(p) for p in params]:
            total = sum(p.numel() for p in params)
            self._flat = torch.zeros(total, dtype=torch.float32, device=device)
            self._flat_params = params
            self._views = {}
            off = 0
            for p in params:
                self._views[id(p)] = self._flat[off:off + p.numel()].view_as(p)
                off += p.numel()
        acc = {}
        for p in params:
            if p.grad is None:
                p.grad = self._views[id(p)]
                acc[id(p)] = False
            else:
                if not (p.grad.is_contiguous() and p.grad.dtype == torch.float32 and p.grad.device == p.device):
                    raise RuntimeError("drnmi train: existing .grad must be contiguous fp32 on the device")
                acc[id(p)] = True
        return acc

    def _pack(self, nd, st, device, stream):
        lib = _lib.load()
        conv = nd.conv
        cout, cin, ks, _ = conv.weight.shape
        cs = self.cstride[nd.src]
        if st.wf is None:
            st.k = ks * ks * cs
            st.k_pad = _round_up(st.k, K_ALIGN)
            st.cout_pad = _round_up(cout, COUT_ALIGN)
            st.wf = torch.empty(st.cout_pad, st.k_pad, dtype=torch.float32, device=device)
            st.shift = torch.zeros(st.cout_pad, dtype=torch.float32, device=device)
        w = conv.weight.detach()
        if not (w.is_contiguous() and w.dtype == torch.float32):
            raise RuntimeError(f"{nd.name}: expected a contiguous fp32 weight")
        if not self._packed_now:
            _lib.check(lib.drnmi_pack_conv_weight(_vp(w), cout, cin, ks, cs, st.cout_pad, st.k_pad, 0, None, F32,
                                                  _vp(st.wf), stream), f"pack {nd.name}")
            # fp32x: the full-resolution small-channel convs (stem, layer1, layer2 shapes) run on
            # the split-bf16 patch kernels, as in the inference engine (engine.X6_PATCH_SHAPES)
            st.patch = self.model.precision == "fp32x" and not nd.out_fp32_nchw and \
                (cs, cout, ks, conv.stride[0], conv.dilation[0]) in X6_PATCH_SHAPES
            st.wfx = self._split(st.wf, cs, st.k, st.k_pad, patch=st.patch, out=st.wfx)
        if conv.bias is not None:
            st.shift[:cout].copy_(conv.bias.detach())

    def _pack_dgrad(self, nd, st, device, stream):
        lib = _lib.load()
        cout, cin, ks, _ = nd.conv.weight.shape
        dys = self.cstride[nd.dst] if not nd.out_fp32_nchw else _pow2_at_least(cout)
        if st.wd is None:
            st.kd = ks * ks * dys
            st.kd_pad = _round_up(st.kd, K_ALIGN)
            st.rows_d = _round_up(cin, COUT_ALIGN)
            st.wd = torch.empty(st.rows_d, st.kd_pad, dtype=torch.float32, device=device)
        st.dys = dys
        if self._packed_now:                      # packed with the forward weights (batched launch)
            return dys
        _lib.check(lib.drnmi_pack_conv_weight(_vp(nd.conv.weight.detach()), cout, cin, ks, dys, st.rows_d,
                                              st.kd_pad, 1, None, F32, _vp(st.wd), stream), f"pack dgrad {nd.name}")
        # fp32x: a data gradient whose (stride-1) conv is a patch-kernel shape (layer1's 16 -> 16
        # at full resolution) runs split-bf16 on the patch kernel, not on the f32 igemm
        st.dpatch = self.model.precision == "fp32x" and \
            (dys, cin, ks, 1, nd.conv.dilation[0]) in X6_PATCH_SHAPES
        st.wdx = self._split(st.wd, dys, st.kd, st.kd_pad, patch=st.dpatch, out=st.wdx)
        return dys

    def _s2_classes(self, nd, st, device, stream):
        """The parity classes of a stride-2 conv's data gradient in fp32x (drnmi_dgrad_s2_class_planes):
        [(a, b, ksc, planes)] for the classes some tap reaches, their weight planes gathered from this
        step's packed dgrad planes; None when the layer keeps the zero-insert path (not conv_x6, a
        dilated conv, or a class whose taps would start above its pixel).  Cached per step."""
        if st.s2_step == self._step_id:
            return st.s2_cls
        st.s2_step, st.s2_cls = self._step_id, None
        cout, cin, ks, _ = nd.conv.weight.shape
        p, d = nd.conv.padding[0], nd.conv.dilation[0]
        dys = self._pack_dgrad(nd, st, device, stream)
        if st.wdx is None or st.dpatch or d != 1 or dys % 8 != 0 or st.kd != st.kd_pad:
            return None
        pad_d = d * (ks - 1) - p
        parts = []
        for a_ in (0, 1):
            k0 = (pad_d - a_) % 2
            nh = (ks - k0 + 1) // 2 if k0 < ks else 0
            if nh and (a_ - pad_d + k0) // 2 != 0:       # the class conv would need a nonzero pad
                return None
            parts.append((k0, nh))
        lib = _lib.load()
        cls = []
        cache = st.s2_planes or {}
        for a_ in (0, 1):
            for b_ in (0, 1):
                nh, nw = parts[a_][1], parts[b_][1]
                if nh == 0 or nw == 0:
                    continue
                ksc = max(nh, nw)
                kpc = ksc * ksc * dys
                buf = cache.get((a_, b_))
                if buf is None or buf.shape != (3, st.rows_d, kpc):
                    buf = torch.empty(3, st.rows_d, kpc, dtype=torch.bfloat16, device=device)
                    cache[(a_, b_)] = buf
                _lib.check(lib.drnmi_dgrad_s2_class_planes(_vp(st.wdx), st.rows_d, st.kd_pad, dys, ks, pad_d, a_, b_,
                                                           ksc, _vp(buf), kpc, stream), f"dgrad classes {nd.name}")
                cls.append((a_, b_, ksc, buf))
        st.s2_planes = cache
        st.s2_cls = cls
        return cls

    def _batched_pack(self, device, stream) -> bool:
        """Re-pack every forward and dgrad weight (and fp32x planes) of the network in one launch
        (drnmi_pack_conv_weights_batched), bit-identical to the per-layer calls.  Needs the buffers
        of a previous step (False on the first step, or when disabled)."""
        if not self.batched_pack:
            return False
        if self._pack_prec != self.model.precision:   # a per-layer step sets the new mode's buffers
            self._pack_prec = self.model.precision
            self._pack_key = None
            return False
        key = [self.model.precision]
        for nd, st in zip(self.nodes, self.state):
            if st.wf is None or (nd.src != "input" and st.wd is None):
                return False
            key.append((nd.conv.weight.data_ptr(), st.wf.data_ptr(), st.wfx.data_ptr() if st.wfx is not None else 0,
                        st.wd.data_ptr() if st.wd is not None else 0,
                        st.wdx.data_ptr() if st.wdx is not None else 0))
        key = tuple(key)
        if key != self._pack_key:
            rows = []
            total = 0
            for nd, st in zip(self.nodes, self.state):
                cout, cin, ks, _ = nd.conv.weight.shape
                w = nd.conv.weight.detach()
                if not (w.is_contiguous() and w.dtype == torch.float32):
                    return False
                ents = [(st.wf, st.wfx, self.cstride[nd.src], st.cout_pad, st.k_pad, 0)]
                if st.wd is not None:
                    ents.append((st.wd, st.wdx, st.dys, st.rows_d, st.kd_pad, 1))
                for out, planes, kst, rows_pad, k_pad, mode in ents:
                    rows.append([w.data_ptr(), out.data_ptr(), planes.data_ptr() if planes is not None else 0,
                                 cout, cin, ks, kst, rows_pad, k_pad, mode, total, 0])
                    total += rows_pad * k_pad
            tab = torch.tensor(rows, dtype=torch.int64)
            tot = ctypes.c_int64(0)
            _lib.check(_lib.load().drnmi_pack_table_check(ctypes.c_void_p(tab.data_ptr()), len(rows),
                                                          ctypes.byref(tot)), "pack table")
            self._pack_tab = tab.to(device)
            self._pack_total = int(tot.value)
            self._pack_key = key
        _lib.check(_lib.load().drnmi_pack_conv_weights_batched(_vp(self._pack_tab), self._pack_tab.shape[0],
                                                               self._pack_total, ctypes.c_void_p(stream)),
                   "batched weight pack")
        return True

    def _split(self, wpk, cin_stride, k, k_pad, patch=False, out=None):
        """fp32x: the three bf16 planes of a packed fp32 weight, for the convs conv_x6 takes
        (>= 32 input channels, k == k_pad) or the split-bf16 patch kernels take (`patch`); None
        keeps the launch on the exact-f32 kernel.  `out`: the previous step's planes (reused)."""
        if self.model.precision != "fp32x" or (not patch and (cin_stride < 32 or k != k_pad)):
            return None
        # one HIP pass (drnmi_split3_bf16), bit-identical to engine.split3_bf16
        if out is None or out.shape != (3,) + tuple(wpk.shape):
            out = torch.empty((3,) + tuple(wpk.shape), dtype=torch.bfloat16, device=wpk.device)
        _lib.check(_lib.load().drnmi_split3_bf16(_vp(wpk), wpk.numel(), _vp(out), _lib.stream_ptr(wpk.device)),
                   "split3_bf16")
        return out

    def _conv(self, x, cin_stride, h, w, wpk, k, k_pad, cout_pad, cout, ks, stride, pad, dil, y, y_strides,
              shift, res, n, ho, wo, stream, what, wx=None, algo=_lib.ALGO_IGEMM, want_stats=False, y_sr=0,
              split=True):
        """One drnmi_conv2d_bn_act launch.  want_stats: let a conv_x6 launch write the BN statistics
        partials of its output (self._st_ws); returns their row count, 0 when it cannot."""
        a = _lib.ConvArgs()
        a.x, a.wgt, a.scale, a.shift = x.data_ptr(), (wx if wx is not None else wpk).data_ptr(), None, shift.data_ptr()
        a.res = res.data_ptr() if res is not None else None
        a.y = y.data_ptr()
        a.y_sn, a.y_sp, a.y_sc = y_strides
        a.y_sr = y_sr
        a.n, a.h, a.w, a.cin = n, h, w, cin_stride
        a.ho, a.wo, a.cout, a.cout_pad = ho, wo, cout, cout_pad
        a.ks, a.stride, a.pad, a.dil = ks, stride, pad, dil
        a.k, a.k_pad = k, k_pad
        a.relu = 0
        a.dtype = a.out_dtype = F32
        if wx is not None:
            a.dtype = _lib.DRNMI_F32X3           # fp32x: conv_x6 (fp32 in/out, bf16 weight planes)
        a.tile, a.algo = -1, algo
        lib = _lib.load()
        if wx is not None and algo == _lib.ALGO_IGEMM and split and X6_SPLIT_K:
            # split-K scratch for the launches whose tiles would leave CUs idle (the 1/8-res layers)
            nb = lib.drnmi_conv_workspace_bytes(ctypes.byref(a))
            if nb > 0:
                ws = self._ws("_cv_ws", nb, y.device)
                a.ws, a.ws_bytes = ws.data_ptr(), ws.numel()
        rows = 0
        if want_stats and wx is not None and algo == _lib.ALGO_IGEMM:
            rows = lib.drnmi_conv_stats_rows(ctypes.byref(a))
            if rows > 0:
                a.stats = self._ws("_st_ws", 2 * rows * cout * 8, y.device).data_ptr()
        _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(stream)), what)
        return max(rows, 0)

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, save: bool):
        """Train-mode forward; returns (logprobs, logits, saved) — saved is None if not save."""
        lib = _lib.load()
        dev = x.device
        stream = _lib.stream_ptr(dev)
        n, _, h, w = x.shape
        vals = {}
        shapes = {"input": (h, w)}
        xin = torch.empty(n, h, w, 8, dtype=torch.float32, device=dev)
        _lib.check(lib.drnmi_nchw_to_nhwc(x.data_ptr(), xin.data_ptr(), n, 3, h, w, 8, F32, ctypes.c_void_p(stream)),
                   "nchw_to_nhwc")
        vals["input"] = xin
        self._packed_now = False
        self._packed_now = self._batched_pack(dev, stream)
        per_node = []
        logits = None
        for nd, st in zip(self.nodes, self.state):
            c = nd.conv
            ih, iw = shapes[nd.src]
            ks, s, p, d = c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0]
            oh, ow = _conv_out(ih, ks, s, p, d), _conv_out(iw, ks, s, p, d)
            shapes[nd.dst] = (oh, ow)
            self._pack(nd, st, dev, ctypes.c_void_p(stream))
            cout = c.out_channels
            cs_in = self.cstride[nd.src]
            if nd.out_fp32_nchw:        # seg 1x1 + bias -> fp32 NCHW logits
                logits = torch.empty(n, cout, oh, ow, dtype=torch.float32, device=dev)
                self._conv(vals[nd.src], cs_in, ih, iw, st.wf, st.k, st.k_pad, st.cout_pad, cout, ks, s, p, d,
                           logits, (cout * oh * ow, 1, oh * ow), st.shift, None, n, oh, ow, stream, nd.name, st.wfx)
                vals[nd.dst] = logits
                per_node.append(None)
                continue
            cs = self.cstride[nd.dst]
            if cs != cout:
                raise NotImplementedError("train path: channel count must be a power of two")
            rows = n * oh * ow
            y = torch.empty(rows, cs, dtype=torch.float32, device=dev)
            bn = nd.bn
            if bn.momentum is None or not bn.track_running_stats:
                raise NotImplementedError("BatchNorm2d with momentum=None / no running stats")
            # conv_x6 launches write the BN statistics partials in their epilogue (no pass over y)
            g_rows = self._conv(vals[nd.src], cs_in, ih, iw, st.wf, st.k, st.k_pad, st.cout_pad, cout, ks, s, p,
                                d, y, (oh * ow * cs, cs, 1), st.shift, None, n, oh, ow, stream, nd.name, st.wfx,
                                _lib.ALGO_PATCH if st.patch else _lib.ALGO_IGEMM, want_stats=FUSED_BN_STATS)
            mean = torch.empty(cs, dtype=torch.float32, device=dev)
            invstd = torch.empty(cs, dtype=torch.float32, device=dev)
            if g_rows > 0:
                # the epilogue wrote [2][g_rows][cout] partials (row stride = cout); cs == cout here
                # (checked above), so the finalize reads them with the same channel count
                _lib.check(lib.drnmi_bn_stats_partials_f32(
                    _vp(self._st_ws), g_rows, rows, cs, float(bn.eps), float(bn.momentum), _vp(mean), _vp(invstd),
                    _vp(bn.running_mean), _vp(bn.running_var), _vp(bn.num_batches_tracked), ctypes.c_void_p(stream)),
                    f"bn_stats {nd.name}")
            else:
                ws = self._ws("_red_ws", lib.drnmi_reduce_workspace_bytes(rows, cs), dev)
                _lib.check(lib.drnmi_bn_stats_f32(_vp(y), rows, cs, float(bn.eps), float(bn.momentum), _vp(mean),
                                                  _vp(invstd), _vp(bn.running_mean), _vp(bn.running_var),
                                                  _vp(bn.num_batches_tracked), _vp(ws), ctypes.c_void_p(stream)),
                           f"bn_stats {nd.name}")
            for b in (bn.running_mean, bn.running_var, bn.num_batches_tracked):
                torch.autograd.graph.increment_version(b)
            z = torch.empty(rows, cs, dtype=torch.float32, device=dev)
            res = vals[nd.res] if nd.res else None
            _lib.check(lib.drnmi_bn_act_f32(_vp(y), _vp(mean), _vp(invstd), _vp(bn.weight.detach()),
                                            _vp(bn.bias.detach()), _vp(res), 1 if nd.relu else 0, rows, cs, _vp(z),
                                            ctypes.c_void_p(stream)), f"bn_act {nd.name}")
            vals[nd.dst] = z
            per_node.append((y, mean, invstd) if save else None)
        lh, lw = shapes["logits"]
        logprobs = torch.empty(n, logits.shape[1], 8 * lh, 8 * lw, dtype=torch.float32, device=dev)
        if self.model.use_torch_up:      # UpsamplingBilinear2d(8) head (lmodels/drnseg.py:285-287)
            up = None
            _lib.check(lib.drnmi_up8_bilinear_logsoftmax_argmax(logits.data_ptr(), logprobs.data_ptr(), None,
                                                                _lib.DRNMI_U8, n, logits.shape[1], lh, lw,
                                                                ctypes.c_void_p(stream)), "up8_bilinear_logsoftmax")
        else:
            up = self.model._up_plane(dev)
            _lib.check(lib.drnmi_up8_logsoftmax_argmax(logits.data_ptr(), up.data_ptr(), logprobs.data_ptr(), None,
                                                       _lib.DRNMI_U8, n, logits.shape[1], lh, lw,
                                                       ctypes.c_void_p(stream)), "up8_logsoftmax")
        saved = None
        if save:
            saved = {"vals": vals, "shapes": shapes, "nodes": per_node, "n": n, "up": up}
        return logprobs, logits, saved

    # ------------------------------------------------------------------ backward
    def backward(self, saved, logprobs, logits, g_lp, g_logits):
        lib = _lib.load()
        self._step_id += 1
        dev = logprobs.device
        stream = _lib.stream_ptr(dev)
        sp = ctypes.c_void_p(stream)
        vals, shapes, n = saved["vals"], saved["shapes"], saved["n"]
        acc = self._ensure_flat_grads(dev)
        ncls, lh, lw = logits.shape[1], logits.shape[2], logits.shape[3]
        # head: LogSoftmax backward + transpose of the bilinear up-conv
        dlog = torch.empty_like(logits)
        du = torch.empty_like(logprobs) if g_lp is not None else None
        glp = g_lp.contiguous() if g_lp is not None else None
        glg = g_logits.contiguous() if g_logits is not None else None
        if saved["up"] is None:          # use_torch_up: transpose of the bilinear x8
            _lib.check(lib.drnmi_up8_bilinear_lsm_bwd_f32(_vp(glp), _vp(logprobs) if glp is not None else None,
                                                          _vp(glg), float(self.grad_scale), n, ncls, lh, lw, _vp(du),
                                                          _vp(dlog), sp), "up8_bilinear_lsm_bwd")
        else:
            _lib.check(lib.drnmi_up8_lsm_bwd_f32(_vp(glp), _vp(logprobs) if glp is not None else None, _vp(glg),
                                                 _vp(saved["up"]), float(self.grad_scale), n, ncls, lh, lw, _vp(du),
                                                 _vp(dlog), sp), "up8_lsm_bwd")
        del du
        grads = {}          # value -> NHWC fp32 gradient buffer
        for idx in range(len(self.nodes) - 1, -1, -1):
            nd, st = self.nodes[idx], self.state[idx]
            c = nd.conv
            cout, cin, ks, _ = c.weight.shape
            s, p, d = c.stride[0], c.padding[0], c.dilation[0]
            ih, iw = shapes[nd.src]
            oh, ow = shapes[nd.dst]
            rows = n * oh * ow
            done = []
            if nd.out_fp32_nchw:
                dys = _pow2_at_least(cout)
                dy = torch.empty(rows, dys, dtype=torch.float32, device=dev)
                _lib.check(lib.drnmi_nchw_to_nhwc(dlog.data_ptr(), dy.data_ptr(), n, cout, oh, ow, dys, F32, sp),
                           "seg grad nhwc")
                if c.bias is not None and c.bias.requires_grad:
                    ws = self._ws("_red_ws", lib.drnmi_reduce_workspace_bytes(rows, dys), dev)
                    _lib.check(lib.drnmi_channel_sum_f32(_vp(dy), rows, dys, cout, _vp(c.bias.grad),
                                                         1 if acc[id(c.bias)] else 0, _vp(ws), sp), "seg bias grad")
                    done.append(c.bias)
            else:
                dys = self.cstride[nd.dst]
                dz = grads.pop(nd.dst, None)
                if dz is None:
                    raise RuntimeError(f"no gradient reached {nd.name}")
                if self.debug_value_grads is not None:
                    self.debug_value_grads[nd.dst] = dz.detach().clone()
                y, mean, invstd = saved["nodes"][idx]
                z = vals[nd.dst]
                bn = nd.bn
                dres = None
                dres_acc = 0
                if nd.res:
                    dres = grads.get(nd.res)
                    if dres is None:
                        dres = torch.empty_like(vals[nd.res])
                        grads[nd.res] = dres
                    else:
                        dres_acc = 1
                gw, gb = bn.weight, bn.bias
                ws = self._ws("_red_ws", lib.drnmi_reduce_workspace_bytes(rows, dys), dev)
                gacc = 1 if (gw.requires_grad and acc[id(gw)]) else 0
                if nd.relu and not nd.res:
                    # residual-free BN + ReLU: the mask is recomputed from y (z is not read)
                    _lib.check(lib.drnmi_bn_relu_bwd_y_f32(
                        _vp(dz), _vp(y), _vp(mean), _vp(invstd), _vp(gw.detach()), _vp(gb.detach()), rows, dys,
                        _vp(dz), _vp(gw.grad) if gw.requires_grad else None,
                        _vp(gb.grad) if gb.requires_grad else None, gacc, _vp(ws), sp), f"bn_bwd {nd.name}")
                else:
                    _lib.check(lib.drnmi_bn_act_bwd_f32(
                        _vp(dz), _vp(z), _vp(y), _vp(mean), _vp(invstd), _vp(gw.detach()), 1 if nd.relu else 0,
                        rows, dys, _vp(dz), _vp(dres), dres_acc,
                        _vp(gw.grad) if gw.requires_grad else None, _vp(gb.grad) if gb.requires_grad else None,
                        gacc, _vp(ws), sp), f"bn_bwd {nd.name}")
                if gw.requires_grad and gb.requires_grad and acc[id(gw)] != acc[id(gb)]:
                    raise RuntimeError("BN weight/bias grads must be both set or both None")
                done += [q for q in (gw, gb) if q.requires_grad]
                dy = dz
            # weight gradient
            if c.weight.requires_grad:
                wa = _lib.WgradArgs()
                wa.dy, wa.x, wa.dw = dy.data_ptr(), vals[nd.src].data_ptr(), c.weight.grad.data_ptr()
                wa.n, wa.h, wa.w, wa.cin, wa.cin_stride = n, ih, iw, cin, self.cstride[nd.src]
                wa.ho, wa.wo, wa.cout, wa.dy_stride = oh, ow, cout, dys
                wa.ks, wa.stride, wa.pad, wa.dil = ks, s, p, d
                wa.accumulate = 1 if acc[id(c.weight)] else 0
                # fp32x: every weight gradient is split-bf16 (the forward's small-channel layers
                # run split on the patch kernels as well); fp32 sizes only its own partials
                x3 = self.model.precision == "fp32x"
                nb = (lib.drnmi_conv_wgrad_workspace_bytes if x3 else lib.drnmi_conv_wgrad_f32_workspace_bytes)(
                    ctypes.byref(wa))
                if nb < 0:
                    raise RuntimeError(f"wgrad {nd.name}: bad geometry")
                ws = self._ws("_wg_ws", nb, dev)
                wa.ws, wa.ws_bytes = ws.data_ptr(), ws.numel()
                wg = lib.drnmi_conv_wgrad_f32x3 if x3 else lib.drnmi_conv_wgrad_f32
                _lib.check(wg(ctypes.byref(wa), sp), f"wgrad {nd.name}")
                done.append(c.weight)
            if self.grad_ready is not None and done:
                self.grad_ready(done)
            # data gradient (not needed for the network input)
            classes = (self._s2_classes(nd, st, dev, sp) if nd.src != "input" and s == 2 and S2_CLASS_DGRAD
                       else None)
            if classes is not None:
                # stride 2: four parity-class convs of dy itself, no zero-inserted copy
                cs_src = self.cstride[nd.src]
                prev = grads.get(nd.src)
                if prev is not None:
                    out = prev
                elif len(classes) < 4:          # pixels no tap reaches keep a zero gradient
                    out = torch.zeros(n * ih * iw, cs_src, dtype=torch.float32, device=dev)
                else:
                    out = torch.empty(n * ih * iw, cs_src, dtype=torch.float32, device=dev)
                flat = out.view(-1)
                for (a_, b_, ksc, planes) in classes:
                    ho_c, wo_c = (ih - a_ + 1) // 2, (iw - b_ + 1) // 2
                    if ho_c <= 0 or wo_c <= 0:
                        continue
                    base = (a_ * iw + b_) * cs_src
                    view = flat[base:]
                    self._conv(dy, dys, oh, ow, None, ksc * ksc * dys, ksc * ksc * dys, st.rows_d, cin, ksc, 1, 0,
                               1, view, (ih * iw * cs_src, 2 * cs_src, 1), self._zeros_f32(st.rows_d, dev),
                               view if prev is not None else None, n, ho_c, wo_c, stream,
                               f"dgrad {nd.name} class {a_}{b_}", planes, y_sr=2 * iw * cs_src, split=False)
                grads[nd.src] = out
            elif nd.src != "input":
                dys_d = self._pack_dgrad(nd, st, dev, sp)
                assert dys_d == dys
                cs_src = self.cstride[nd.src]
                src = dy
                hu, wu = oh, ow
                pad_d = d * (ks - 1) - p
                if s > 1:
                    hu, wu = ih + 2 * p - d * (ks - 1), iw + 2 * p - d * (ks - 1)
                    src = torch.empty(n * hu * wu, dys, dtype=torch.float32, device=dev)
                    _lib.check(lib.drnmi_zero_insert_f32(_vp(dy), n, oh, ow, dys, s, hu, wu, _vp(src), sp),
                               f"zero_insert {nd.name}")
                prev = grads.get(nd.src)
                out = prev if prev is not None else torch.empty(n * ih * iw, cs_src, dtype=torch.float32, device=dev)
                patch = st.dpatch and prev is None       # the patch kernels take no residual
                self._conv(src, dys, hu, wu, st.wd, st.kd, st.kd_pad, st.rows_d, cin, ks, 1, pad_d, d, out,
                           (ih * iw * cs_src, cs_src, 1), self._zeros_f32(st.rows_d, dev), prev, n, ih, iw,
                           stream, f"dgrad {nd.name}", st.wdx if (patch or not st.dpatch) else None,
                           _lib.ALGO_PATCH if patch else _lib.ALGO_IGEMM)
                grads[nd.src] = out
            del dy


class _TrainFn(torch.autograd.Function):
    """DRNSeg train-mode forward as one autograd node; backward = the HIP backward kernels."""

    @staticmethod
    def forward(ctx, runner, x, *params):
        ctx.set_materialize_grads(False)
        lp, logits, saved = runner.forward(x, save=True)
        ctx.runner = runner
        ctx.saved = saved
        ctx.outs = (lp, logits)
        return lp, logits

    @staticmethod
    def backward(ctx, g_lp, g_logits):
        lp, logits = ctx.outs
        if g_lp is not None or g_logits is not None:
            ctx.runner.backward(ctx.saved, lp, logits, g_lp, g_logits)
        ctx.saved = None
        # parameter grads were written straight into .grad (flat buffer views)
        return (None,) * len(ctx.needs_input_grad)


def train_forward(model, x: torch.Tensor):
    """DRNSeg.forward in train mode (batch-stat BN, autograd through the HIP backward)."""
    runner = getattr(model, "_train_runner", None)
    if runner is None:
        runner = TrainRunner(model)
        model._train_runner = runner
    if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] != 3:
        raise ValueError("DRNSeg.forward expects fp32 [B,3,H,W]")
    x = x.contiguous()
    params = [p for p in runner.ordered_params() if p.requires_grad]
    if torch.is_grad_enabled() and params:
        return _TrainFn.apply(runner, x, *params)
    lp, logits, _ = runner.forward(x, save=False)
    return lp, logits


# ====================================================================== criterion
class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lp, target, ignore_index):
        lib = _lib.load()
        n, c = lp.shape[0], lp.shape[1]
        hw = lp[0, 0].numel()
        dev = lp.device
        loss = torch.empty((), dtype=torch.float32, device=dev)
        count = torch.empty((), dtype=torch.float32, device=dev)
        ws = torch.empty(lib.drnmi_ce_workspace_bytes(), dtype=torch.uint8, device=dev)
        sp = ctypes.c_void_p(_lib.stream_ptr(dev))
        _lib.check(lib.drnmi_ce_loss_f32(_vp(lp), _vp(target), n, c, hw, int(ignore_index), _vp(loss), _vp(count),
                                         _vp(ws), sp), "ce_loss")
        ctx.save_for_backward(lp, target, count)
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, g):
        lp, target, count = ctx.saved_tensors
        lib = _lib.load()
        n, c = lp.shape[0], lp.shape[1]
        hw = lp[0, 0].numel()
        glp = torch.empty_like(lp)
        g = g.contiguous().to(torch.float32)
        _lib.check(lib.drnmi_ce_loss_bwd_f32(_vp(lp), _vp(target), n, c, hw, int(ctx.ignore_index), _vp(g),
                                             _vp(count), _vp(glp), ctypes.c_void_p(_lib.stream_ptr(lp.device))),
                   "ce_loss_bwd")
        return glp, None, None


class CrossEntropyLoss(torch.nn.Module):
    """nn.CrossEntropyLoss(ignore_index=255) drop-in (semantic_seg.py:817) on the HIP kernels.

    Like the reference it is applied to DRNSeg's log-probs (model(x)[0]), i.e. it computes
    mean over target != ignore_index of logsumexp(lp) - lp[target] (a second log-softmax,
    semantic_seg.py:197-198).  Only mean reduction and no class weights (the reference's use)."""

    def __init__(self, weight=None, ignore_index: int = -100, reduction: str = "mean"):
        super().__init__()
        if weight is not None or reduction != "mean":
            raise NotImplementedError("class weights / reduction != 'mean' are not used by the reference")
        self.ignore_index = ignore_index

    def forward(self, logprobs: torch.Tensor, target: torch.Tensor):
        if not logprobs.is_cuda:
            raise RuntimeError("drnmi CrossEntropyLoss runs on the HIP kernels (no CPU fallback)")
        if logprobs.dtype != torch.float32:
            raise ValueError("expected fp32 log-probs")
        if target.dtype != torch.int64:
            raise ValueError("expected int64 targets (semantic_seg.py:195 target.long())")
        if target.shape != (logprobs.shape[0],) + tuple(logprobs.shape[2:]):
            raise ValueError(f"target shape {tuple(target.shape)} does not match {tuple(logprobs.shape)}")
        return _CEFn.apply(logprobs.contiguous(), target.contiguous(), self.ignore_index)


# ====================================================================== optimizer
class SGD(torch.optim.Optimizer):
    """torch.optim.SGD drop-in (semantic_seg.py:963-966) whose step is one multi-tensor HIP
    launch per 48 parameters.  With `pruner=` the pruner's masks are applied inside the same
    pass (replacing the separate Pruner.apply_masks after optimizer.step(), :213-214);
    state['momentum_buffer'] matches torch's, so state_dict()/load_state_dict() interoperate."""

    def __init__(self, params, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, pruner=None,
                 model=None):
        if lr < 0 or momentum < 0 or weight_decay < 0:
            raise ValueError("invalid SGD hyper-parameters")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))
        self.pruner = pruner
        self._mask_of = {}
        if pruner is not None:
            if model is None:
                raise ValueError("SGD(pruner=...) needs model= to resolve mask keys to parameters")
            self.attach_pruner(pruner, model)

    def attach_pruner(self, pruner, model):
        self.pruner = pruner
        named = dict(model.named_parameters())
        self._mask_of = {}
        for key in pruner.mask_dict:
            for cand in (key, "module." + key, key[len("module."):] if key.startswith("module.") else None):
                if cand is not None and cand in named:
                    self._mask_of[id(named[cand])] = key
                    break
            else:
                raise KeyError(key)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for group in self.param_groups:
            ps, gs, bs, ns, ms, fs = [], [], [], [], [], []
            mom = group["momentum"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise RuntimeError("drnmi SGD: parameters/grads must be contiguous fp32 on the ROCm device")
                st = self.state[p]
                first = 0
                if mom != 0:
                    buf = st.get("momentum_buffer")
                    if buf is None:
                        buf = torch.empty_like(p)
                        st["momentum_buffer"] = buf
                        first = 1
                    bs.append(buf)
                ps.append(p)
                gs.append(p.grad)
                ns.append(p.numel())
                fs.append(first)
                key = self._mask_of.get(id(p))
                ms.append(self.pruner._mask_bits(key, p.device) if key is not None else None)
            if not ps:
                continue
            k = len(ps)
            arr = lambda ts: (ctypes.c_void_p * k)(*[t.data_ptr() if t is not None else None for t in ts])
            mask_arr = arr(ms) if any(m is not None for m in ms) else None
            _lib.check(lib.drnmi_sgd_step_f32(
                k, arr(ps), arr(gs), arr(bs) if mom != 0 else None, (ctypes.c_int64 * k)(*ns), mask_arr,
                (ctypes.c_int32 * k)(*fs), float(group["lr"]), float(mom), float(group["dampening"]),
                float(group["weight_decay"]), 1 if group["nesterov"] else 0,
                ctypes.c_void_p(_lib.stream_ptr(ps[0].device))), "sgd_step")
            for p in ps:
                torch.autograd.graph.increment_version(p)
        return loss
