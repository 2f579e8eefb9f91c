"""Execution engine: packs a DRN-D + seg head into HIP-kernel launch plans.

The reference runs DRNSeg.forward as ~70 ATen ops per frame (lmodels/drnseg.py:
295-299 -> lmodels/drn.py:213-259).  Here the same network is lowered once into a
list of fused launches on the C-ABI (include/drnmi.h):

  ingest / NCHW->NHWC  -> stem conv7x7+BN+ReLU -> conv3x3+BN+ReLU ... ->
  [block: conv+BN+ReLU, (1x1 downsample+BN), conv+BN+residual+ReLU] ... ->
  seg 1x1+bias (fp32 NCHW logits) -> up x8 + log-softmax + argmax

Activations are NHWC in HBM (channel stride = a power of two >= 8), in bf16 (perf
mode) or fp32 (parity mode).  BN is folded into per-channel scale/shift applied in
the conv epilogue (eval semantics, lmodels/drn.py:7 BatchNorm2d in .eval()).
Weights are re-packed lazily whenever any parameter/buffer changes (tracked by the
tensors' version counters), so Pruner.apply_masks or a load_state_dict is picked up.
"""
from __future__ import annotations

import ctypes
import dataclasses
from dataclasses import dataclass, field

import torch
import torch.nn as nn

from . import _lib
from .drn import BasicBlock, Bottleneck

BN_EPS_DEFAULT = 1e-5
K_ALIGN = 32
COUT_ALIGN = 128

DTYPES = {"fp32": (torch.float32, _lib.DRNMI_F32), "bf16": (torch.bfloat16, _lib.DRNMI_BF16),
          "fp32x": (torch.float32, _lib.DRNMI_F32)}
# fp32x: fp32 activations everywhere (the fp32 mode's buffers); the convs with cin >= X6_MIN_CIN
# and ks 1/3 run fp32-accurate split-bf16 arithmetic (csrc/conv_x6.hip, dtype DRNMI_F32X3), the
# full-resolution small-channel stem / layer1 / layer2 stay on the exact f32 MFMA kernels.
X6_MIN_CIN = 32
TORCH_OF_CODE = {_lib.DRNMI_F32: torch.float32, _lib.DRNMI_BF16: torch.bfloat16, _lib.DRNMI_I8: torch.int8}
# W8A8 (config C5): convs whose input channel stride is >= this run on the int8 MFMA kernel
# (conv_i8_kernel: K steps of 64/128 int8 channels); the full-resolution small-channel layers
# (stem, layer1-3: ~5 % of D-22's FLOPs) stay bf16.
INT8_MIN_CIN = 64
# ... and whose output has at least this many channels.  256: D-22's 128-channel layer4.0 stays on
# the bf16 row / staggered kernels (s2row, stag128 with the downsample folded in), which beat the
# int8 tiles there: 1786-1788 vs 1750-1755 fps interleaved (profiles/r6_int8_fusions).
INT8_MIN_COUT = 256
# ... except the 128 -> 128 3x3 stride-1 convs without a folded downsample (D-22 layer4.1): the
# int8 128 x 128 tile (conv_w1h_i8_kernel, odd tap-group counts) serves them (INT8_LAYER4 = False
# keeps them bf16)
INT8_LAYER4 = True

# (cin_stride, cout, ks, stride, dil) served by the LDS-patch kernel (bf16 only; include/drnmi.h)
# (32 -> 64 stride 2 runs faster on the K-32 LDS-DMA implicit GEMM: 67 vs 108 us per 4 frames)
PATCH_SHAPES = {(8, 16, 7, 1, 1), (16, 16, 3, 1, 1), (16, 32, 3, 2, 1)}
# fp32 and fp32x inference: the same full-resolution layers on the exact-fp32 patch kernel
# (csrc/patch_f32.hip, f32-input MFMA; the stem reads the uint8 frame on the segment() path) --
# faster than the split-bf16 patch kernels (2.0 vs 2.4 ms per 8-frame step) and exact fp32
F32_PATCH_SHAPES = PATCH_SHAPES
# the fp32x fine-tune keeps these layers on the split-bf16 patch kernels (drnmi/train.py)
X6_PATCH_SHAPES = PATCH_SHAPES
STEM_U8_K = 224     # fused u8 stem: k = kh*32 + kw*4 + c


def _pow2_at_least(c: int, lo: int = 8) -> int:
    p = lo
    while p < c:
        p *= 2
    return p


def _round_up(v: int, a: int) -> int:
    return (v + a - 1) // a * a


@dataclass
class ConvNode:
    """One fused conv launch: y = act(conv(x) * scale + shift [+ res])."""
    name: str                    # state_dict prefix of the conv weight (e.g. "layer.3.0.conv1")
    conv: nn.Conv2d
    bn: nn.BatchNorm2d | None    # None -> bias (seg) or identity scale
    src: str                     # value names in the plan
    dst: str
    res: str | None = None
    relu: bool = True
    out_fp32_nchw: bool = False  # seg logits
    cin_stride: int = 0          # filled by packing
    # packed device tensors
    wpk: torch.Tensor | None = None
    scale: torch.Tensor | None = None
    shift: torch.Tensor | None = None
    k: int = 0
    k_pad: int = 0
    cout_pad: int = 0
    scale_folded: bool = False   # BN scale multiplied into wpk; launched with scale = NULL
    unit_mask: torch.Tensor | None = None   # block-sparsity map of wpk (MFMA skips zero units)
    zero_unit_frac: float = 0.0
    # W8A8 (precision "int8"): int8 wpk, scale = weight scale x input scale x BN scale
    i8: bool = False
    x_val: str = ""              # value the launch reads (src, or "q:src" = its int8 copy)
    r_val: str | None = None
    res_scale: float = 0.0
    out_scale: float = 0.0       # 1 / scale of an int8 output (0: bf16 / fp32 output)
    x6: bool = False             # fp32x: wpk holds three bf16 planes, launched as DRNMI_F32X3
    # fused 1x1 downsample (bf16): this node's launch also computes the residual branch
    # (include/drnmi.h drnmi_conv_args.x2); ds_of names the folded-away downsample node
    fused: dict | None = None    # {"wpk", "shift", "k", "x2_val", "stride2", "ds": node index}
    fused_into: int = -1         # downsample node: index of the conv that computes it


@dataclass
class Graph:
    nodes: list = field(default_factory=list)
    stage_outputs: dict = field(default_factory=dict)   # "layer0".."layer8" -> value name
    channels: dict = field(default_factory=dict)        # value -> logical channels


def lower_drnseg(layer: nn.Sequential, seg: nn.Conv2d, prefix: str = "layer") -> Graph:
    """Walk DRNSeg.layer (= DRN children[:-2]) and emit ConvNodes.

    Follows lmodels/drn.py forward order (:213-259): layer0 .. layer8, with
    BasicBlock (:49-65) / Bottleneck (:86-106) residual structure."""
    g = Graph()
    cur = "input"
    g.channels[cur] = 3
    vid = [0]

    def new(c):
        vid[0] += 1
        name = f"v{vid[0]}"
        g.channels[name] = c
        return name

    for li, stage in enumerate(layer):
        sname = f"{prefix}.{li}"
        mods = list(stage)
        if mods and isinstance(mods[0], nn.Conv2d):
            # conv-bn-relu triples (layer0 stem, _make_conv_layers)
            for j in range(0, len(mods), 3):
                conv, bn = mods[j], mods[j + 1]
                dst = new(conv.out_channels)
                g.nodes.append(ConvNode(f"{sname}.{j}", conv, bn, cur, dst, relu=True))
                cur = dst
        else:
            for bi, blk in enumerate(mods):
                bname = f"{sname}.{bi}"
                if isinstance(blk, BasicBlock) or type(blk).__name__ == "BasicBlock":
                    t = new(blk.conv1.out_channels)
                    g.nodes.append(ConvNode(f"{bname}.conv1", blk.conv1, blk.bn1, cur, t, relu=True))
                    res = None
                    if blk.residual:
                        res = cur
                        if blk.downsample is not None:
                            res = new(blk.downsample[0].out_channels)
                            g.nodes.append(ConvNode(f"{bname}.downsample.0", blk.downsample[0],
                                                    blk.downsample[1], cur, res, relu=False))
                    out = new(blk.conv2.out_channels)
                    g.nodes.append(ConvNode(f"{bname}.conv2", blk.conv2, blk.bn2, t, out, res=res, relu=True))
                    cur = out
                elif isinstance(blk, Bottleneck) or type(blk).__name__ == "Bottleneck":
                    t1 = new(blk.conv1.out_channels)
                    g.nodes.append(ConvNode(f"{bname}.conv1", blk.conv1, blk.bn1, cur, t1, relu=True))
                    t2 = new(blk.conv2.out_channels)
                    g.nodes.append(ConvNode(f"{bname}.conv2", blk.conv2, blk.bn2, t1, t2, relu=True))
                    res = cur
                    if blk.downsample is not None:
                        res = new(blk.downsample[0].out_channels)
                        g.nodes.append(ConvNode(f"{bname}.downsample.0", blk.downsample[0],
                                                blk.downsample[1], cur, res, relu=False))
                    out = new(blk.conv3.out_channels)
                    g.nodes.append(ConvNode(f"{bname}.conv3", blk.conv3, blk.bn3, t2, out, res=res, relu=True))
                    cur = out
                else:
                    raise TypeError(f"unsupported block {type(blk)} at {bname}")
        g.stage_outputs[f"layer{li}"] = cur
    logits = "logits"
    g.channels[logits] = seg.out_channels
    g.nodes.append(ConvNode("seg", seg, None, cur, logits, relu=False, out_fp32_nchw=True))
    return g


def _fold_bn(bn: nn.BatchNorm2d):
    """Eval-mode BatchNorm as y = x*scale + shift (lmodels/drn.py:7)."""
    invstd = torch.rsqrt(bn.running_var.float() + bn.eps)
    w = bn.weight.float() if bn.weight is not None else torch.ones_like(invstd)
    b = bn.bias.float() if bn.bias is not None else torch.zeros_like(invstd)
    scale = w * invstd
    shift = b - bn.running_mean.float() * scale
    return scale, shift


class PackedNet:
    """Device-resident packed weights for one precision.

    Owns its own copy of the graph's ConvNodes: the packed tensors (wpk, scale, shift, unit
    masks, int8 fields) of one precision never overwrite another precision's, so a Plan of
    any PackedNet stays valid while other precisions are packed."""

    def __init__(self, graph: Graph, precision: str, device, block_sparse: bool = True,
                 act_scales: dict | None = None):
        self.graph = Graph(nodes=[dataclasses.replace(nd) for nd in graph.nodes],
                           stage_outputs=dict(graph.stage_outputs), channels=dict(graph.channels))
        self.block_sparse = block_sparse
        self.precision = precision
        # int8 nets run their small-channel layers in bf16: "base" is that precision
        self.base = "bf16" if precision == "int8" else precision
        self.tdtype, self.code = DTYPES[self.base]
        self.device = device
        self.cstride = {"input": 8}
        for v, c in graph.channels.items():
            if v != "input":
                self.cstride[v] = _pow2_at_least(c)
        self.act_scales = dict(act_scales or {})
        self.vcode = {}            # value -> dtype code where it differs from self.code
        self.quant_after = {}      # node index -> values quantised (bf16 -> "q:" int8) after it
        self.i8_nodes = set()
        if precision == "int8":
            self._int8_layout()
        self.pack()

    def _int8_layout(self):
        """Which launches run W8A8 and which values are int8 in HBM.  A value is int8 when an
        int8 launch produces it and only int8 launches read it; a bf16 value read by an int8
        launch gets an int8 copy "q:<value>" quantised right after its producer."""
        g = self.graph
        # (cout >= 128 too: the int8 tiles are 128 channels wide; the 64-channel layer3 convs keep
        # the bf16 halo kernel)
        producer = {nd.dst: i for i, nd in enumerate(g.nodes)}

        def layer4_shape(nd):
            c = nd.conv
            if not INT8_LAYER4 or (c.in_channels, c.out_channels, c.kernel_size[0], c.stride[0], c.groups) != \
                    (128, 128, 3, 1, 1) or self.cstride[nd.src] != 128:
                return False
            # a block conv2 whose residual is a downsample keeps the bf16 tile with it folded in
            return not (nd.res and nd.res in producer and g.nodes[producer[nd.res]].name.endswith("downsample.0"))
        elig = {i for i, nd in enumerate(g.nodes)
                if self.cstride[nd.src] >= INT8_MIN_CIN and nd.conv.kernel_size[0] in (1, 3)
                and (nd.conv.out_channels >= INT8_MIN_COUT or nd.out_fp32_nchw or layer4_shape(nd))}
        readers = {}
        for i, nd in enumerate(g.nodes):
            for v in (nd.src, nd.res):
                if v:
                    readers.setdefault(v, []).append(i)
        for i in elig:
            nd = g.nodes[i]
            if not nd.out_fp32_nchw and readers.get(nd.dst) and all(j in elig for j in readers[nd.dst]):
                self.vcode[nd.dst] = _lib.DRNMI_I8
        need = {v for i in elig for v in (g.nodes[i].src, g.nodes[i].res) if v}
        missing = sorted(v for v in need | set(self.vcode) if v not in self.act_scales)
        if missing:
            raise RuntimeError(f"int8: no calibrated activation scale for {missing} (DRNSeg.calibrate_int8)")
        for v in sorted(need):
            if self.vcode.get(v) != _lib.DRNMI_I8:
                if v == "input":
                    raise NotImplementedError("int8 launch reading the network input")
                self.quant_after.setdefault(producer[v], []).append(v)
        self.i8_nodes = elig

    def value_code(self, v: str) -> int:
        if v.startswith("q:"):
            return _lib.DRNMI_I8
        return self.vcode.get(v, self.code)

    def pack(self):
        with torch.no_grad():
            for ni, nd in enumerate(self.graph.nodes):
                conv = nd.conv
                w = conv.weight.detach().to(self.device, torch.float32)
                cout, cin, kh, kw = w.shape
                if kh != kw:
                    raise NotImplementedError("square kernels only")
                cs = self.cstride[nd.src]
                nd.cin_stride = cs
                wp = torch.zeros(cout, kh, kw, cs, device=self.device, dtype=torch.float32)
                wp[..., :cin] = w.permute(0, 2, 3, 1)
                nd.k = kh * kw * cs
                nd.k_pad = _round_up(nd.k, K_ALIGN)
                nd.cout_pad = _round_up(cout, COUT_ALIGN)
                full = torch.zeros(nd.cout_pad, nd.k_pad, device=self.device, dtype=torch.float32)
                full[:cout, :nd.k] = wp.reshape(cout, nd.k)
                nd.wpk = full.to(self.tdtype).contiguous()
                scale = torch.ones(nd.cout_pad, device=self.device)
                shift = torch.zeros(nd.cout_pad, device=self.device)
                if nd.bn is not None:
                    s, b = _fold_bn(nd.bn)
                    scale[:cout] = s.to(self.device)
                    shift[:cout] = b.to(self.device)
                elif conv.bias is not None:
                    shift[:cout] = conv.bias.detach().to(self.device, torch.float32)
                nd.scale, nd.shift = scale.contiguous(), shift.contiguous()
                nd.i8, nd.x_val, nd.r_val, nd.res_scale, nd.out_scale = False, nd.src, nd.res, 0.0, 0.0
                nd.x6 = False
                if ni in self.i8_nodes:
                    self._pack_int8(nd, full, scale, cout)
                    continue
                if self.precision == "fp32x" and cs >= X6_MIN_CIN and kh in (1, 3):
                    nd.x6 = True
                    nd.wpk = split3_bf16(full)
                    nd.scale_folded = False
                    nd.unit_mask, nd.zero_unit_frac = None, 0.0
                    continue
                # bf16 LDS-DMA kernels: fold the BN scale into the weights so the kernel starts its
                # accumulators from shift + residual (include/drnmi.h: scale may be NULL)
                nd.scale_folded = self.base == "bf16" and _fused_init_route(nd, cs)
                if nd.scale_folded:
                    nd.wpk = (full * scale[:, None]).to(self.tdtype).contiguous()
                nd.unit_mask, nd.zero_unit_frac = None, 0.0
                if nd.scale_folded and self.block_sparse:
                    nd.unit_mask, nd.zero_unit_frac = _unit_mask(nd.wpk, self.code)
            self._fuse_downsamples()
            # fused-ingest stem weights (bf16 patch kernel reads uint8 frames directly)
            self.stem_u8_w = None
            stem = self.graph.nodes[0]
            w = stem.conv.weight.detach().to(self.device, torch.float32)
            if self.base in ("bf16", "fp32x", "fp32") and tuple(w.shape[1:]) == (3, 7, 7) and \
                    _uses_patch(stem, self.cstride["input"], self.base):
                wp = torch.zeros(w.shape[0], 7, 8, 4, device=self.device, dtype=torch.float32)
                wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
                full = torch.zeros(stem.cout_pad, STEM_U8_K, device=self.device, dtype=torch.float32)
                full[:w.shape[0]] = wp.reshape(w.shape[0], STEM_U8_K)
                # (fp32 / fp32x: the f32 weights in the same kh*32 + kw*4 + c layout, patch_f32.hip SRC 0)
                self.stem_u8_w = full.to(self.tdtype).contiguous()
            self._front_packs = {}
            self.front_eligible = self._front_shapes_ok()
            self.block64_pairs = self._block64_pairs()
            self._block64_packs = {}

    def _front_shapes_ok(self) -> bool:
        """The fused video front (drnmi_video_front_u8: layer0 + layer1 + layer2 of every DRN-D,
        lmodels/drn.py:132-137, :201-211) takes exactly 7x7 3->16 s1, 3x3 16->16 s1, 3x3 16->32 s2,
        bf16 activations (also in int8 nets, whose small-channel layers stay bf16)."""
        nodes = self.graph.nodes
        if self.base != "bf16" or len(nodes) < 4 or not FUSE_FRONT:
            return False
        want = [(3, 16, 7, 1, 3, 1), (16, 16, 3, 1, 1, 1), (16, 32, 3, 2, 1, 1)]
        for nd, (ci, co, k, st, pd, dl) in zip(nodes[:3], want):
            c = nd.conv
            if (c.in_channels, c.out_channels, c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0]) != \
                    (ci, co, k, st, pd, dl) or c.groups != 1 or nd.bn is None or nd.res is not None or \
                    not nd.relu or nd.i8 or nd.out_fp32_nchw:
                return False
        return nodes[1].src == nodes[0].dst and nodes[2].src == nodes[1].dst and self.cstride[nodes[2].dst] == 32

    def _block64_pairs(self) -> list[int]:
        """Node indices i where nodes i, i+1 are a plain 64-channel BasicBlock (lmodels/drn.py:49-65:
        conv3x3 64 -> 64 + BN + ReLU, conv3x3 + BN + residual = the block input + ReLU, stride 1,
        dilation 1, no downsample) in bf16: drnmi_basic_block64 runs them as one launch."""
        if self.base != "bf16" or not FUSE_BLOCK64 or self.block_sparse:
            return []
        nodes = self.graph.nodes
        out = []
        for i in range(len(nodes) - 1):
            a, b = nodes[i], nodes[i + 1]
            ok = True
            for nd in (a, b):
                c = nd.conv
                ok &= (c.in_channels, c.out_channels, c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0],
                       c.groups) == (64, 64, 3, 1, 1, 1, 1) and nd.bn is not None and nd.relu and not nd.i8 \
                    and not nd.x6 and not nd.out_fp32_nchw and not nd.fused and nd.fused_into < 0
            ok = ok and a.res is None and b.src == a.dst and b.res == a.src and \
                all(self.cstride[v] == 64 for v in (a.src, a.dst, b.dst)) and \
                self.value_code(a.src) == self.value_code(a.dst) == self.value_code(b.dst) == _lib.DRNMI_BF16
            if ok and (not out or out[-1] + 1 < i):
                out.append(i)
        return out

    def block64_pack(self, i: int) -> torch.Tensor:
        """Device copy of drnmi_block64_pack for the block at nodes i, i+1 (cleared by every repack)."""
        t = self._block64_packs.get(i)
        if t is None:
            import numpy as np
            lib = _lib.load()
            arrs = []
            for nd in self.graph.nodes[i:i + 2]:
                arrs += [nd.conv.weight.detach().float().cpu().contiguous().numpy(),
                         nd.scale[:64].float().cpu().contiguous().numpy(), nd.shift[:64].float().cpu().contiguous().numpy()]
            out = np.zeros(int(lib.drnmi_block64_pack_bytes()), dtype=np.uint8)
            _lib.check(lib.drnmi_block64_pack(*[x.ctypes.data_as(ctypes.c_void_p) for x in arrs],
                                              out.ctypes.data_as(ctypes.c_void_p)), "block64_pack")
            t = torch.from_numpy(out).to(self.device)
            self._block64_packs[i] = t
        return t

    def front_pack(self, mean, std, bgr: bool) -> torch.Tensor:
        """Device copy of drnmi_front_pack for these weights and this normalisation (cached per
        (mean, std, bgr); cleared by every repack)."""
        key = (tuple(float(v) for v in mean), tuple(float(v) for v in std), bool(bgr))
        t = self._front_packs.get(key)
        if t is None:
            import numpy as np
            lib = _lib.load()
            arrs = []
            for nd in self.graph.nodes[:3]:
                arrs += [nd.conv.weight.detach().float().cpu().contiguous().numpy(),
                         nd.scale.float().cpu().contiguous().numpy(), nd.shift.float().cpu().contiguous().numpy()]
            arrs += [np.asarray(key[0], dtype=np.float32), np.asarray(key[1], dtype=np.float32)]
            out = np.zeros(int(lib.drnmi_front_pack_bytes()), dtype=np.uint8)
            _lib.check(lib.drnmi_front_pack(*[a.ctypes.data_as(ctypes.c_void_p) for a in arrs], 1 if bgr else 0,
                                            out.ctypes.data_as(ctypes.c_void_p)), "front_pack")
            t = torch.from_numpy(out).to(self.device)
            self._front_packs[key] = t
        return t


    def _fuse_downsamples(self):
        """bf16: fold each BasicBlock / Bottleneck 1x1 downsample (lmodels/drn.py:181-186) into the
        block's last conv as extra K columns -- [W2 | W_ds] over [im2col(t) ; x sampled at the
        downsample stride], both BN scales already folded into the weights, shifts summed -- so
        the residual branch is one GEMM segment instead of a launch that writes it to HBM and a
        residual read.  Only where the last conv already runs on conv_big (the LDS-DMA kernel
        that takes x2); plans with keep_all (parity taps, calibration) keep the separate launch."""
        g = self.graph
        for nd in g.nodes:
            nd.fused, nd.fused_into = None, -1
        if self.base != "bf16" or not FUSE_DOWNSAMPLE:
            return
        producer = {nd.dst: i for i, nd in enumerate(g.nodes)}
        reads = {}
        for nd in g.nodes:
            for v in (nd.src, nd.res):
                if v:
                    reads[v] = reads.get(v, 0) + 1
        for i, nd in enumerate(g.nodes):
            j = producer.get(nd.res) if nd.res else None
            if j is None or nd.i8 or nd.x6 or not nd.scale_folded or nd.unit_mask is not None:
                continue
            ds = g.nodes[j]
            if (not ds.name.endswith("downsample.0") or ds.relu or ds.i8 or not ds.scale_folded
                    or ds.conv.kernel_size[0] != 1 or ds.conv.padding[0] != 0 or reads.get(nd.res) != 1):
                continue
            cin2 = self.cstride[ds.src]
            if ds.cout_pad != nd.cout_pad or nd.k_pad != nd.k:
                continue
            # conv_big takes cin2 % 64 == 0 with k_pad == k; the halo kernel (layer3/4 3x3,
            # cin2 32 or 64) takes rows zero-padded to whole 64-column steps
            k = nd.k + cin2
            if cin2 % 64 == 0 and _route_name(nd, nd.cin_stride).startswith("conv_big") and \
                    _route_name(nd, nd.cin_stride, cin2).startswith("conv_big"):
                k_pad = k
            elif cin2 in (32, 64) and _route_name(nd, nd.cin_stride).startswith("conv_halo") and \
                    _route_name(nd, nd.cin_stride, cin2, (k + 63) // 64 * 64).startswith("conv_halo"):
                k_pad = (k + 63) // 64 * 64
            else:
                continue
            parts = [nd.wpk, ds.wpk[:, :cin2]]
            if k_pad > k:
                parts.append(torch.zeros(nd.wpk.shape[0], k_pad - k, dtype=nd.wpk.dtype, device=nd.wpk.device))
            nd.fused = {"wpk": torch.cat(parts, dim=1).contiguous(),
                        "shift": (nd.shift + ds.shift).contiguous(), "k": k, "k_pad": k_pad,
                        "x2_val": ds.src, "stride2": ds.conv.stride[0], "ds": j}
            ds.fused_into = i

    def _pack_int8(self, nd: ConvNode, full: torch.Tensor, bn_scale: torch.Tensor, cout: int):
        """Per-output-channel symmetric int8 weights (oracle/int8_oracle.py quantize_weight_rows):
        s_w = absmax / 127, q = clamp(rint(w * 127 / absmax)); the epilogue scale is
        s_w * s_x * bn_scale, so acc * scale is the dequantised, BN-scaled conv output."""
        a = full.abs().amax(dim=1)
        pos = a > 0
        inv = torch.where(pos, 127.0 / torch.where(pos, a, torch.ones_like(a)), torch.ones_like(a))
        nd.wpk = torch.round(full * inv[:, None]).clamp_(-127, 127).to(torch.int8).contiguous()
        sw = torch.where(pos, a / 127.0, torch.ones_like(a))
        sx = float(self.act_scales[nd.src])
        nd.scale = (sw * sx * bn_scale).float().contiguous()
        nd.scale_folded = False
        nd.unit_mask, nd.zero_unit_frac = None, 0.0
        nd.i8 = True
        nd.x_val = nd.src if self.vcode.get(nd.src) == _lib.DRNMI_I8 else "q:" + nd.src
        if nd.res:
            nd.r_val = nd.res if self.vcode.get(nd.res) == _lib.DRNMI_I8 else "q:" + nd.res
            nd.res_scale = float(self.act_scales[nd.res])
        if self.vcode.get(nd.dst) == _lib.DRNMI_I8:
            nd.out_scale = 1.0 / float(self.act_scales[nd.dst])


def split3_bf16(w: torch.Tensor) -> torch.Tensor:
    """fp32 [R, K] -> bf16 [3, R, K] planes with w = w1 + w2 + w3 (round-to-nearest-even at each
    step; the residuals are exact in fp32), the weight side of the fp32x arithmetic
    (include/drnmi.h DRNMI_F32X3)."""
    w = w.float()
    w1 = w.to(torch.bfloat16)
    r1 = w - w1.float()
    w2 = r1.to(torch.bfloat16)
    w3 = (r1 - w2.float()).to(torch.bfloat16)
    return torch.stack([w1, w2, w3]).contiguous()


# Below this fraction of all-zero 16 x 32 units the dense kernel is used: skipping costs scalar
# flag loads and breaks the MFMA/LDS interleave, measured break-even near 50 %.
SPARSE_MIN_ZERO_UNITS = 0.5


def _unit_mask(wpk: torch.Tensor, code: int):
    """Block-sparsity map of packed weights (include/drnmi.h drnmi_weight_unit_mask): one bit per
    16 x 32 unit.  Returned only when enough units are all-zero (pruned) to pay for the
    per-step flag loads; the count is read back once per (re)pack, never in the launch loop."""
    rows, kp = wpk.shape
    wpr = (kp + 1023) // 1024
    mask = torch.empty((rows // 16) * wpr, dtype=torch.int32, device=wpk.device)
    cnt = torch.empty(1, dtype=torch.int32, device=wpk.device)
    lib = _lib.load()
    _lib.check(lib.drnmi_weight_unit_mask(wpk.data_ptr(), code, rows, kp, mask.data_ptr(), cnt.data_ptr(),
                                          ctypes.c_void_p(_lib.stream_ptr(wpk.device))), "weight_unit_mask")
    units = (rows // 16) * (kp // 32)
    zero = 1.0 - int(cnt.item()) / units
    return (mask, zero) if zero >= SPARSE_MIN_ZERO_UNITS else (None, zero)


def _uses_patch(nd: ConvNode, cin_stride: int, precision: str) -> bool:
    if nd.i8:
        return False
    c = nd.conv
    shape = (cin_stride, c.out_channels, c.kernel_size[0], c.stride[0], c.dilation[0])
    if nd.res is not None or nd.out_fp32_nchw:
        return False
    return (precision == "bf16" and shape in PATCH_SHAPES) or (precision in ("fp32", "fp32x") and shape in F32_PATCH_SHAPES)


# bf16: fold 1x1 downsamples into the block's last conv (PackedNet._fuse_downsamples)
FUSE_DOWNSAMPLE = True
# bf16 video path: the uint8 stem and the 3x3 16->16 layer1 conv run as one kernel
# (drnmi_stem_layer1); the stem output is never written.  Plans with keep_all keep two launches.
FUSE_STEM = True
# bf16 video path: layer0 + layer1 + layer2 as one launch from the uint8 frames (drnmi_video_front_u8);
# neither 16-channel full-resolution activation is written.  Plans with keep_all keep separate launches.
FUSE_FRONT = True
# 64-channel BasicBlocks (D-22 layer3.1) as one drnmi_basic_block64 launch (False: two conv launches)
FUSE_BLOCK64 = True


def _route_name(nd: ConvNode, cin_stride: int, cin2: int = 0, k_pad: int | None = None) -> str:
    """Kernel the bf16 launch of `nd` (optionally with a fused cin2-channel second input, weight
    rows of k_pad columns) goes to, probed on a 16x16 map through drnmi_conv_kernel_name
    (routing does not depend on size)."""
    c = nd.conv
    a = _lib.ConvArgs()
    a.n, a.h, a.w, a.cin = 1, 16, 16, cin_stride
    a.ks, a.stride, a.pad, a.dil = c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0]
    a.ho = _conv_out(16, a.ks, a.stride, a.pad, a.dil)
    a.wo = a.ho
    a.cout, a.cout_pad = c.out_channels, nd.cout_pad
    a.k = a.ks * a.ks * cin_stride + cin2
    a.k_pad = a.k if k_pad is None else k_pad
    a.dtype, a.out_dtype, a.y_sp, a.y_sc = _lib.DRNMI_BF16, _lib.DRNMI_BF16, c.out_channels, 1
    a.scale = None
    a.tile, a.algo = -1, _lib.ALGO_IGEMM
    if cin2:
        a.x2, a.cin2, a.h2, a.w2, a.stride2 = 1, cin2, 16 * c.stride[0], 16 * c.stride[0], 1
    name = _lib.load().drnmi_conv_kernel_name(ctypes.byref(a))
    return name.decode() if name is not None else ""


def _fused_init_route(nd: ConvNode, cin_stride: int) -> bool:
    """True when the bf16 launch of `nd` goes to conv_big / conv_pp / conv_halo (the kernels
    that take scale = NULL and seed the accumulators with shift + residual).  Routing does not
    depend on the spatial size, so a 16x16 probe decides it."""
    if _uses_patch(nd, cin_stride, "bf16"):
        return False
    c = nd.conv
    a = _lib.ConvArgs()
    a.n, a.h, a.w, a.cin = 1, 16, 16, cin_stride
    a.ks, a.stride, a.pad, a.dil = c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0]
    a.ho = _conv_out(16, a.ks, a.stride, a.pad, a.dil)
    a.wo = a.ho
    a.cout, a.cout_pad, a.k, a.k_pad = c.out_channels, nd.cout_pad, nd.k, nd.k_pad
    a.dtype = _lib.DRNMI_BF16
    if nd.out_fp32_nchw:
        a.out_dtype, a.y_sp, a.y_sc = _lib.DRNMI_F32, 1, a.ho * a.wo
    else:
        a.out_dtype, a.y_sp, a.y_sc = _lib.DRNMI_BF16, c.out_channels, 1
    a.tile, a.algo = -1, _lib.ALGO_IGEMM
    name = _lib.load().drnmi_conv_kernel_name(ctypes.byref(a))
    return name is not None and name.decode().startswith(("conv_big", "conv_pp", "conv_halo"))


def _conv_out(h, k, s, p, d):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1


# segment(): NHWC logits rows for the labels head, and the seg classifier folded into the last conv
# (drnmi_conv_stag_seg); tests switch these module flags off to compare with the unfused path
LABELS_NHWC = True
SEG_FUSE = True


class Plan:
    """Launch plan for one (batch, H, W, precision): shapes, buffers, C-ABI arg structs."""

    def __init__(self, packed: PackedNet, n: int, h: int, w: int, keep_all: bool = False):
        self.packed = packed
        self.n, self.h, self.w = n, h, w
        dev = packed.device
        g = packed.graph
        self.shapes = {"input": (h, w)}
        for nd in g.nodes:
            c = nd.conv
            ih, iw = self.shapes[nd.src]
            self.shapes[nd.dst] = (_conv_out(ih, c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0]),
                                   _conv_out(iw, c.kernel_size[1], c.stride[1], c.padding[1], c.dilation[1]))
        lh, lw = self.shapes["logits"]
        self.out_hw = (8 * lh, 8 * lw)

        # Liveness-based buffer reuse (exact-size, per-dtype pool).  Launches read nd.x_val /
        # nd.r_val (an int8 copy "q:<v>" of a bf16 value in int8 nets), and a fused conv its
        # downsample's input instead of the residual (PackedNet._fuse_downsamples).
        self.fuse = not keep_all
        for nd in g.nodes:
            if not nd.x_val:
                nd.x_val, nd.r_val = nd.src, nd.res
        self.skip = {i for i, nd in enumerate(g.nodes) if self.fuse and nd.fused_into >= 0}
        reads_of = {}
        for i, nd in enumerate(g.nodes):
            if i in self.skip:
                reads_of[i] = set()
            elif self.fuse and nd.fused:
                reads_of[i] = {nd.x_val, nd.fused["x2_val"]}
            else:
                reads_of[i] = {nd.x_val, nd.r_val} - {None}
        last_use = {}
        for i in range(len(g.nodes)):
            for v in reads_of[i]:
                last_use[v] = i
        self.bufs = {}
        pool = {}
        self.bufs["input"] = torch.empty(n * h * w * 8, dtype=packed.tdtype, device=dev)

        def alloc(v, numel):
            td = TORCH_OF_CODE[packed.value_code(v)]
            lst = pool.get((numel, td))
            self.bufs[v] = lst.pop() if lst else torch.empty(numel, dtype=td, device=dev)

        for i, nd in enumerate(g.nodes):
            if i in self.skip:
                continue                          # computed inside the block's last conv
            oh, ow = self.shapes[nd.dst]
            if nd.out_fp32_nchw:
                self.bufs[nd.dst] = torch.empty(n, nd.conv.out_channels, oh, ow, dtype=torch.float32, device=dev)
            else:
                alloc(nd.dst, n * oh * ow * packed.cstride[nd.dst])
            for v in packed.quant_after.get(i, []):
                alloc("q:" + v, n * oh * ow * packed.cstride[v])
            if not keep_all:
                for v in reads_of[i] - {"input"}:
                    if last_use.get(v) == i and v in self.bufs and v != nd.dst:
                        t = self.bufs[v]
                        pool.setdefault((t.numel(), t.dtype), []).append(t)
        self.keep_all = keep_all
        self._reads_of = reads_of
        self.args = [None if i in self.skip else self._conv_args(nd) for i, nd in enumerate(g.nodes)]
        self.stem_u8 = self._stem_u8_args()
        self.stem_fused = self._stem_fusable(reads_of)
        self.front_fused = self._front_fusable(reads_of)
        self.front_pack_t = None
        self._norm = None                          # (mean, std, bgr) of the last ingest_u8
        # fused 64-channel BasicBlocks: the first conv's output has no other reader
        self.block64 = {}
        lib = _lib.load()
        for i in getattr(packed, "block64_pairs", []):
            # (int8 nets: the block output's int8 copy for layer4 is quantised after the launch)
            if self.fuse and not any(g.nodes[i].dst in reads_of[j] for j in range(len(g.nodes)) if j != i + 1) and \
                    not packed.quant_after.get(i) and \
                    lib.drnmi_block64_supported(n, *self.shapes[g.nodes[i].dst]):
                self.block64[i] = packed.block64_pack(i)
        self._setup_seg_nhwc()
        self.src = "nchw"

    # labels-only video path: the seg conv writes fp32 NHWC rows of SEG_NHWC_CS floats (16-B
    # stores instead of 19 strided planes) and drnmi_up8_labels_nhwc reads them; same values,
    # same labels.  Only where the seg conv runs on conv_big (bf16 input), on the int8 tile
    # (int8 nets: store_tile_i8's 16-B fp32 rows) or on conv_x6 (fp32x) and the 19-class head.
    SEG_NHWC_CS = 20

    def _setup_seg_nhwc(self):
        self.seg_idx, self.seg_nhwc_args, self.seg_fused = -1, None, None
        nodes = self.packed.graph.nodes
        idx = [i for i, nd in enumerate(nodes) if nd.out_fp32_nchw]
        if len(idx) != 1 or self.args[idx[0]] is None:
            return
        i = idx[0]
        nd, a0 = nodes[i], self.args[i]
        if nd.conv.out_channels != 19 or nd.conv.kernel_size[0] != 1:
            return
        cs = self.SEG_NHWC_CS
        lh, lw = self.shapes[nd.dst]
        a = _lib.ConvArgs()
        ctypes.pointer(a)[0] = a0
        a.y_sn, a.y_sp, a.y_sc = lh * lw * cs, cs, 1
        name = _lib.load().drnmi_conv_kernel_name(ctypes.byref(a))   # (routing does not read a.y)
        if name is None or not name.decode().startswith(("conv_big_kernel", "conv_i8_kernel", "conv_i8_occ2_kernel",
                                                        "conv_x6_kernel")):
            return
        if "logits_nhwc" not in self.bufs:      # only plans whose seg conv writes the NHWC rows
            self.bufs["logits_nhwc"] = torch.empty(self.n * lh * lw * cs, dtype=torch.float32,
                                                   device=self.packed.device)
        a.y = self.bufs["logits_nhwc"].data_ptr()
        self.seg_idx, self.seg_nhwc_args = i, a
        self._setup_seg_fused(i)

    def _setup_seg_fused(self, i: int):
        """The seg classifier folded into its producer's epilogue (drnmi_conv_stag_seg) when that
        producer is a 512-channel staggered-tile conv whose output nothing else reads: bf16 nets
        (fp32 partial logits, bias added by the head) and int8 nets (the int8 seg conv on the
        producer's int8 output: int32 partials, the seg conv's dequant applied by the head)."""
        self.seg_fused = None
        if not SEG_FUSE or not self.fuse:
            return
        nodes = self.packed.graph.nodes
        seg = nodes[i]
        prod = [j for j, nd in enumerate(nodes) if nd.dst == seg.x_val and j not in self.skip]
        if len(prod) != 1 or seg.x_val != seg.src or seg.r_val:
            return
        j = prod[0]
        a = self.args[j]
        if a is None or j in self.block64 or (j - 1) in self.block64 or j <= 2 or self.packed.quant_after.get(j):
            return
        if any(nodes[j].dst in self._reads_of[k] for k in range(len(nodes)) if k != i):
            return
        i8 = seg.i8 and nodes[j].i8
        if i8 != (seg.i8 or nodes[j].i8) or (not i8 and not seg.scale_folded):
            return
        if a.cout != 512 or a.res or a.x2 or seg.k != a.cout or seg.cout_pad < 32 or (a.scale and not i8):
            return
        if i8 and a.out_dtype != _lib.DRNMI_I8:
            return
        name = _lib.load().drnmi_conv_kernel_name(ctypes.byref(a))
        # (a plain 512-channel launch runs conv_w1 unfused; fused, drnmi_conv_stag_seg's staggered tile)
        if name is None or name.decode() not in (("conv_i8_stag_kernel", "conv_w1_i8_kernel") if i8 else ("conv_stag_kernel", "conv_w1_kernel")):
            return
        lh, lw = self.shapes[seg.dst]
        if "seg_part" not in self.bufs:
            self.bufs["seg_part"] = torch.empty(2 * self.n * lh * lw * self.SEG_NHWC_CS,
                                                dtype=torch.int32 if i8 else torch.float32, device=self.packed.device)
        self.seg_fused = {"conv": j, "seg_w": seg.wpk.data_ptr(), "seg_k_pad": seg.k_pad, "seg_rows": seg.cout_pad,
                          "bias": seg.shift.data_ptr(), "i8": i8, "scale": seg.scale.data_ptr()}

    def labels_path(self, use_torch_up: bool = False) -> str:
        """How segment() produces labels on this plan: "seg2" (seg folded into the last conv),
        "nhwc" (NHWC logits rows) or "nchw" (the logits planes)."""
        if use_torch_up or not LABELS_NHWC or self.seg_nhwc_args is None:
            return "nchw"
        return "seg2" if self.seg_fused is not None else "nhwc"

    def _front_fusable(self, reads_of) -> bool:
        """layer0..layer2 run as one drnmi_video_front_u8 launch on the u8 path when the packed net
        takes it, each intermediate has exactly one reader and the frame shape is supported."""
        pk = self.packed
        nodes = pk.graph.nodes
        if not (self.fuse and getattr(pk, "front_eligible", False)):
            return False
        for i in (0, 1):
            if any(nodes[i].dst in reads_of[j] for j in range(len(nodes)) if j != i + 1) or pk.quant_after.get(i):
                return False
        if pk.quant_after.get(2):
            return False
        return bool(_lib.load().drnmi_front_supported(self.n, self.h, self.w))

    def _stem_fusable(self, reads_of) -> bool:
        """The u8 stem and layer1 can run as one launch (drnmi_stem_layer1) when layer1 is the
        stem output's only reader and the library takes the pair."""
        nodes = self.packed.graph.nodes
        if not (FUSE_STEM and self.fuse and self.stem_u8 is not None and len(nodes) > 1):
            return False
        if self.args[1] is None or nodes[1].x_val != nodes[0].dst:
            return False
        if any(nodes[0].dst in reads_of[i] for i in range(2, len(nodes))) or self.packed.quant_after.get(0):
            return False
        lib = _lib.load()
        return lib.drnmi_stem_layer1_kernel_name(ctypes.byref(self.stem_u8), ctypes.byref(self.args[1])) is not None

    def _conv_args(self, nd: ConvNode) -> _lib.ConvArgs:
        pk = self.packed
        c = nd.conv
        ih, iw = self.shapes[nd.src]
        oh, ow = self.shapes[nd.dst]
        a = _lib.ConvArgs()
        a.x = self.bufs[nd.x_val].data_ptr()
        a.wgt = nd.wpk.data_ptr()
        a.scale = None if nd.scale_folded else nd.scale.data_ptr()
        a.shift = nd.shift.data_ptr()
        fused = nd.fused if self.fuse else None
        a.res = self.bufs[nd.r_val].data_ptr() if (nd.r_val and not fused) else None
        a.y = self.bufs[nd.dst].data_ptr()
        cout = c.out_channels
        if nd.out_fp32_nchw:
            a.y_sn, a.y_sp, a.y_sc = cout * oh * ow, 1, oh * ow
            a.out_dtype = _lib.DRNMI_F32
        else:
            cs = pk.cstride[nd.dst]
            if nd.res and pk.cstride[nd.res] != cout:
                raise NotImplementedError("residual channel stride must equal cout")
            a.y_sn, a.y_sp, a.y_sc = oh * ow * cs, cs, 1
            a.out_dtype = pk.value_code(nd.dst)
            if cs != cout:
                raise NotImplementedError("activation channel padding beyond the stem input")
        a.n, a.h, a.w, a.cin = self.n, ih, iw, nd.cin_stride
        a.ho, a.wo, a.cout, a.cout_pad = oh, ow, cout, nd.cout_pad
        a.ks, a.stride, a.pad, a.dil = c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0]
        a.k, a.k_pad = nd.k, nd.k_pad
        a.relu = 1 if nd.relu else 0
        a.dtype = _lib.DRNMI_F32X3 if nd.x6 else pk.value_code(nd.x_val)
        a.tile = -1
        a.algo = _lib.ALGO_PATCH if _uses_patch(nd, nd.cin_stride, pk.base) else _lib.ALGO_IGEMM
        a.res_scale, a.out_scale = nd.res_scale, nd.out_scale
        a.unit_mask = nd.unit_mask.data_ptr() if nd.unit_mask is not None else None
        if fused:
            f = fused
            a.wgt, a.shift, a.res = f["wpk"].data_ptr(), f["shift"].data_ptr(), None
            a.k, a.k_pad = f["k"], f["k_pad"]
            a.x2 = self.bufs[f["x2_val"]].data_ptr()
            a.cin2 = pk.cstride[f["x2_val"]]
            a.h2, a.w2 = self.shapes[f["x2_val"]]
            a.stride2 = f["stride2"]
        return a

    def _stem_u8_args(self) -> _lib.ConvArgs | None:
        pk = self.packed
        if pk.stem_u8_w is None:
            return None
        a = _lib.ConvArgs()
        ctypes.pointer(a)[0] = self.args[0]
        a.algo = _lib.ALGO_PATCH
        a.src_u8 = 1
        a.cin = 4
        a.k = a.k_pad = STEM_U8_K
        a.wgt = pk.stem_u8_w.data_ptr()
        return a

    def refresh_weight_ptrs(self):
        nodes = self.packed.graph.nodes
        skip = {i for i, nd in enumerate(nodes) if self.fuse and nd.fused_into >= 0}
        if skip != self.skip:
            raise RuntimeError("repack changed the downsample fusion of a live plan")
        for i, nd in enumerate(nodes):
            if i in self.skip:
                continue
            self.args[i] = self._conv_args(nd)
        self.front_pack_t = None
        if self._norm is not None and self.front_fused:   # a u8 plan may run again without a new ingest
            self.front_pack_t = self.packed.front_pack(*self._norm)
        for i in list(self.block64):
            self.block64[i] = self.packed.block64_pack(i)
        self._setup_seg_nhwc()
        if self.stem_u8 is not None:
            nd = self.packed.graph.nodes[0]
            self.stem_u8.wgt = self.packed.stem_u8_w.data_ptr()
            self.stem_u8.scale = nd.scale.data_ptr()
            self.stem_u8.shift = nd.shift.data_ptr()

    # ------------------------------------------------------------------ execution
    def run_backbone(self, stream: int, timing_hook=None, labels_only: bool = False):
        """labels_only: the seg conv writes the NHWC logits for head_labels_nhwc (when the plan has
        that form, seg_nhwc_args); the NCHW logits buffer is then not written."""
        lib = _lib.load()
        segf = self.seg_fused if labels_only and self.seg_nhwc_args is not None else None
        front = self.src == "u8" and self.front_fused
        fused_stem = self.src == "u8" and self.stem_fused and not front
        nodes = self.packed.graph.nodes
        blocks = self.block64
        for i, (a, nd) in enumerate(zip(self.args, nodes)):
            if a is None or (i == 1 and fused_stem) or (front and i in (1, 2)) or (i - 1) in blocks:
                continue                          # folded into another launch
            if i in blocks:                       # conv1 + conv2 of a 64-channel BasicBlock
                if timing_hook is not None:
                    timing_hook(i, nd, True)
                h, w = self.shapes[nd.dst]
                _lib.check(lib.drnmi_basic_block64(self.bufs[nd.x_val].data_ptr(), blocks[i].data_ptr(),
                                                   self.bufs[nodes[i + 1].dst].data_ptr(), self.n, h, w,
                                                   ctypes.c_void_p(stream)), f"basic_block64 {nd.name}")
                if timing_hook is not None:
                    timing_hook(i, nd, False)
                for v in self.packed.quant_after.get(i + 1, ()):
                    self._quantize(lib, v, stream)
                continue
            if front and i == 0:
                if timing_hook is not None:
                    timing_hook(0, nd, True)
                _lib.check(lib.drnmi_video_front_u8(self.stem_u8.x, self.front_pack_t.data_ptr(),
                                                    self.bufs[self.packed.graph.nodes[2].dst].data_ptr(),
                                                    self.n, self.h, self.w, ctypes.c_void_p(stream)), "video_front_u8")
                if timing_hook is not None:
                    timing_hook(0, nd, False)
                continue
            if i == 0 and self.src == "u8":
                a = self.stem_u8
            if labels_only and i == self.seg_idx and self.seg_nhwc_args is not None:
                if segf is not None:
                    continue                      # folded into its producer's epilogue
                a = self.seg_nhwc_args
            if segf is not None and i == segf["conv"]:
                if timing_hook is not None:
                    timing_hook(i, nd, True)
                _lib.check(lib.drnmi_conv_stag_seg(ctypes.byref(a), segf["seg_w"], segf["seg_k_pad"], segf["seg_rows"],
                                                   self.bufs["seg_part"].data_ptr(), ctypes.c_void_p(stream)),
                           f"conv_stag_seg {nd.name}")
                if timing_hook is not None:
                    timing_hook(i, nd, False)
                continue
            if timing_hook is not None:
                timing_hook(i, nd, True)
            if i == 0 and fused_stem:
                _lib.check(lib.drnmi_stem_layer1(ctypes.byref(a), ctypes.byref(self.args[1]), ctypes.c_void_p(stream)),
                           "stem_layer1")
            else:
                _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), ctypes.c_void_p(stream)), f"conv {nd.name}")
            if timing_hook is not None:
                timing_hook(i, nd, False)
            for v in self.packed.quant_after.get(i, ()):
                self._quantize(lib, v, stream)

    def _quantize(self, lib, v: str, stream: int):
        """bf16 value -> its int8 copy "q:<v>" (include/drnmi.h drnmi_quantize_i8)."""
        src, dst = self.bufs[v], self.bufs["q:" + v]
        _lib.check(lib.drnmi_quantize_i8(src.data_ptr(), self.packed.value_code(v), dst.data_ptr(), dst.numel(),
                                         1.0 / float(self.packed.act_scales[v]), ctypes.c_void_p(stream)),
                   f"quantize_i8 {v}")

    def ingest_nchw(self, x: torch.Tensor, stream: int):
        self.src = "nchw"
        lib = _lib.load()
        n, c, h, w = x.shape
        _lib.check(lib.drnmi_nchw_to_nhwc(x.data_ptr(), self.bufs["input"].data_ptr(), n, c, h, w, 8,
                                          self.packed.code, ctypes.c_void_p(stream)), "nchw_to_nhwc")

    def ingest_u8(self, frames: torch.Tensor, mean, std, bgr: bool, stream: int):
        """uint8 HWC frames in.  The stem kernel reads them directly (normalisation fused) on every
        precision whose stem runs on a patch kernel; otherwise a separate ingest kernel writes the
        normalised NHWC8 input."""
        n, h, w, _ = frames.shape
        if (n, h, w) != (self.n, self.h, self.w):
            raise ValueError("frames shape does not match the plan")
        if self.stem_u8 is not None:
            a = self.stem_u8
            a.x = frames.data_ptr()
            a.bgr = 1 if bgr else 0
            for i in range(3):
                a.mean[i] = float(mean[i])
                a.std[i] = float(std[i])
            if self.front_fused:
                self.front_pack_t = self.packed.front_pack(mean, std, bgr)
            self._norm = (tuple(mean), tuple(std), bool(bgr))
            self.src = "u8"
            return
        self.src = "nchw"
        lib = _lib.load()
        m = (ctypes.c_float * 3)(*[float(v) for v in mean])
        s = (ctypes.c_float * 3)(*[float(v) for v in std])
        _lib.check(lib.drnmi_frame_ingest_u8(frames.data_ptr(), self.bufs["input"].data_ptr(), n, h, w,
                                             m, s, 1 if bgr else 0, self.packed.code,
                                             ctypes.c_void_p(stream)), "frame_ingest_u8")

    def head(self, up_w: torch.Tensor, stream: int, logprobs: torch.Tensor | None,
             labels: torch.Tensor | None):
        lib = _lib.load()
        logits = self.bufs["logits"]
        n, c, lh, lw = logits.shape
        lab_dtype = _lib.DRNMI_U8
        if labels is not None and labels.dtype == torch.int64:
            lab_dtype = _lib.DRNMI_I64
        _lib.check(lib.drnmi_up8_logsoftmax_argmax(
            logits.data_ptr(), up_w.data_ptr(),
            logprobs.data_ptr() if logprobs is not None else None,
            labels.data_ptr() if labels is not None else None,
            lab_dtype, n, c, lh, lw, ctypes.c_void_p(stream)), "up8_logsoftmax_argmax")

    def head_labels_nhwc(self, up_w: torch.Tensor, stream: int, labels: torch.Tensor):
        """Labels from the NHWC logits run_backbone(labels_only=True) wrote (drnmi_up8_labels_nhwc)."""
        lh, lw = self.shapes["logits"]
        lab_dtype = _lib.DRNMI_I64 if labels.dtype == torch.int64 else _lib.DRNMI_U8
        _lib.check(_lib.load().drnmi_up8_labels_nhwc(
            self.bufs["logits_nhwc"].data_ptr(), self.SEG_NHWC_CS, up_w.data_ptr(), labels.data_ptr(), lab_dtype,
            self.n, 19, lh, lw, ctypes.c_void_p(stream)), "up8_labels_nhwc")

    def head_labels_seg2(self, up_w: torch.Tensor, stream: int, labels: torch.Tensor):
        """Labels from the partial logits run_backbone(labels_only=True) wrote with the seg folded into
        the last conv (drnmi_up8_labels_seg2)."""
        lh, lw = self.shapes["logits"]
        lab_dtype = _lib.DRNMI_I64 if labels.dtype == torch.int64 else _lib.DRNMI_U8
        sf = self.seg_fused
        if sf["i8"]:
            _lib.check(_lib.load().drnmi_up8_labels_seg2_i8(
                self.bufs["seg_part"].data_ptr(), self.SEG_NHWC_CS, sf["scale"], sf["bias"], up_w.data_ptr(),
                labels.data_ptr(), lab_dtype, self.n, 19, lh, lw, ctypes.c_void_p(stream)), "up8_labels_seg2_i8")
            return
        _lib.check(_lib.load().drnmi_up8_labels_seg2(
            self.bufs["seg_part"].data_ptr(), self.SEG_NHWC_CS, sf["bias"], up_w.data_ptr(),
            labels.data_ptr(), lab_dtype, self.n, 19, lh, lw, ctypes.c_void_p(stream)), "up8_labels_seg2")

    def head_bilinear(self, stream: int, logprobs: torch.Tensor | None, labels: torch.Tensor | None):
        """use_torch_up head: UpsamplingBilinear2d(8) + LogSoftmax + argmax (lmodels/drnseg.py:285-287)."""
        lib = _lib.load()
        logits = self.bufs["logits"]
        n, c, lh, lw = logits.shape
        lab_dtype = _lib.DRNMI_I64 if labels is not None and labels.dtype == torch.int64 else _lib.DRNMI_U8
        _lib.check(lib.drnmi_up8_bilinear_logsoftmax_argmax(
            logits.data_ptr(), logprobs.data_ptr() if logprobs is not None else None,
            labels.data_ptr() if labels is not None else None, lab_dtype, n, c, lh, lw, ctypes.c_void_p(stream)),
            "up8_bilinear_logsoftmax_argmax")

    def stage_nchw(self, value: str) -> torch.Tensor:
        """fp32 NCHW copy of an intermediate activation (parity taps; keep_all plans).  int8
        values come back dequantised (q * scale) -- a test-side view, not a launch."""
        lib = _lib.load()
        c = self.packed.graph.channels[value]
        oh, ow = self.shapes[value]
        if self.packed.value_code(value) == _lib.DRNMI_I8:
            cs = self.packed.cstride[value]
            q = self.bufs[value].view(self.n, oh, ow, cs)[..., :c]
            return (q.float() * float(self.packed.act_scales[value])).permute(0, 3, 1, 2).contiguous()
        out = torch.empty(self.n, c, oh, ow, dtype=torch.float32, device=self.packed.device)
        _lib.check(lib.drnmi_nhwc_to_nchw(self.bufs[value].data_ptr(), out.data_ptr(), self.n, c, oh, ow,
                                          self.packed.cstride[value], self.packed.value_code(value),
                                          ctypes.c_void_p(_lib.stream_ptr())), "nhwc_to_nchw")
        return out


def conv_flops(plan: Plan):
    """Per-node algorithmic FLOPs (2*M*N*K with the logical Cin, no padding)."""
    out = []
    for nd in plan.packed.graph.nodes:
        c = nd.conv
        oh, ow = plan.shapes[nd.dst]
        m = plan.n * oh * ow
        k = c.in_channels * c.kernel_size[0] * c.kernel_size[1]
        out.append(2.0 * m * c.out_channels * k)
    return out
