"""Algorithmic work and the per-layer roofline of a DRN-D plan.

Per conv node l:  F_l = 2 * M * Cout * (Cin * k * k)       (M = output pixels)
                  B_l = in + weights + out (+ residual)    (activations/weights at the
                        plan's element size; the stem reads the uint8 frame; the seg
                        logits are fp32 and the head writes uint8 labels)
t_l = max(F_l / P_mfma, B_l / BW_hbm),  T* = sum_l t_l,  network fraction = T* / T_measured.
Peaks from /opt/skills/guides/MI355X_MICROARCH.md: HBM 8.0 TB/s, dense bf16 MFMA 2.5 PFLOP/s,
f32-input MFMA 157.3 TFLOP/s.
"""
from __future__ import annotations

HBM_PEAK_BPS = 8.0e12
# int8: dense i8 MFMA = 2x bf16; fp32x: fp32-accurate split-bf16 arithmetic, 6 bf16 MFMAs per fp32
# product (csrc/conv_x6.hip) = 2.5 PF / 6
MFMA_PEAK = {"bf16": 2.5e15, "fp32": 157.3e12, "int8": 5.0e15, "fp32x": 2.5e15 / 6}


def kernel_peak(kernel_name: str, base: str) -> float:
    """MFMA peak of the arithmetic a kernel (named as rocprofv3 names it) runs."""
    if kernel_name.startswith("conv_i8") or "_i8_" in kernel_name:   # conv_i8_*, conv_w1_i8_*, conv_w1h_i8_*
        return MFMA_PEAK["int8"]
    if kernel_name.startswith("conv_x6"):
        return MFMA_PEAK["fp32x"]
    return MFMA_PEAK["fp32" if base == "fp32x" else base]


def node_work(plan):
    """[(name, flops, bytes)] for every conv node, plus the head (up+argmax)."""
    pk = plan.packed
    base = 2 if pk.base == "bf16" else 4        # fp32 / fp32x: fp32 activations
    out = []
    for nd in pk.graph.nodes:
        esz = 1 if nd.i8 else base          # int8 launches: int8 activations and weights
        c = nd.conv
        ih, iw = plan.shapes[nd.src]
        oh, ow = plan.shapes[nd.dst]
        m = plan.n * oh * ow
        cin, cout, k = c.in_channels, c.out_channels, c.kernel_size[0]
        flops = 2.0 * m * cout * cin * k * k
        if nd.src == "input":
            in_b = plan.n * ih * iw * 3 * 1          # uint8 frame
        else:
            in_b = plan.n * ih * iw * cin * esz
        w_b = cout * cin * k * k * esz
        out_b = m * cout * (4 if nd.out_fp32_nchw else esz)
        res_b = m * cout * esz if nd.res else 0
        out.append((nd.name, flops, float(in_b + w_b + out_b + res_b)))
    lh, lw = plan.shapes["logits"]
    c = pk.graph.channels["logits"]
    H, W = plan.out_hw
    head_b = plan.n * c * lh * lw * 4 + plan.n * H * W * 1
    head_f = plan.n * H * W * c * 8.0             # 4 MAC per class per output pixel
    out.append(("head", head_f, float(head_b)))
    return out


def node_peaks(plan):
    """MFMA peak per row of node_work (int8 launches at the i8 rate)."""
    pk = plan.packed
    base = MFMA_PEAK["fp32" if pk.base == "fp32x" else pk.base]
    return [MFMA_PEAK["int8"] if nd.i8 else MFMA_PEAK["fp32x"] if nd.x6 else base
            for nd in pk.graph.nodes] + [base]


def launch_work(plan, video: bool = True):
    """node_work re-cut along the launches the plan really issues (rows stay index-aligned
    with plan.args; an absorbed node's row becomes (name, 0, 0)):
      * a 1x1 downsample folded into its block's last conv (plan.skip, lmodels/drn.py:181-186):
        its FLOPs and its input + weight bytes move into that launch, and the residual tensor
        is neither written by the downsample nor read by the conv;
      * the fused front launch (plan.front_fused: layer0 + layer1 + layer2) or else the fused
        stem + layer1 launch (plan.stem_fused, drn.py:132-137 + :201-211; video=True: the
        uint8-frame segment() path): the 16-channel full-resolution intermediates are neither
        written nor read back."""
    rows = list(node_work(plan))
    nodes = plan.packed.graph.nodes
    esz = 2 if plan.packed.base == "bf16" else 4
    for i in sorted(getattr(plan, "skip", ())):
        j = nodes[i].fused_into
        n_, fj, bj = rows[j]
        oh, ow = plan.shapes[nodes[j].dst]
        res_b = plan.n * oh * ow * nodes[j].conv.out_channels * (1 if nodes[j].i8 else esz)
        fi, bi = rows[i][1], rows[i][2]
        rows[j] = (n_, fj + fi, bj - res_b + (bi - res_b))
        rows[i] = (rows[i][0], 0.0, 0.0)
    if video and getattr(plan, "front_fused", False):
        # layer0 + layer1 + layer2 in one launch (drnmi_video_front_u8): neither full-resolution
        # 16-channel intermediate is written or read back
        mid = 0.0
        for k in (0, 1):
            hk, wk = plan.shapes[nodes[k].dst]
            mid += plan.n * hk * wk * nodes[k].conv.out_channels * esz
        rows[0] = (rows[0][0], rows[0][1] + rows[1][1] + rows[2][1], rows[0][2] + rows[1][2] + rows[2][2] - 2 * mid)
        rows[1] = (rows[1][0], 0.0, 0.0)
        rows[2] = (rows[2][0], 0.0, 0.0)
    elif video and getattr(plan, "stem_fused", False):
        h0, w0 = plan.shapes[nodes[0].dst]
        mid = plan.n * h0 * w0 * nodes[0].conv.out_channels * esz
        rows[0] = (rows[0][0], rows[0][1] + rows[1][1], rows[0][2] + rows[1][2] - 2 * mid)
        rows[1] = (rows[1][0], 0.0, 0.0)
    for i in getattr(plan, "block64", {}):
        # a 64-channel BasicBlock in one launch (drnmi_basic_block64): the intermediate is neither
        # written nor read back, and the block input is read once (conv1 and the residual)
        hb, wb = plan.shapes[nodes[i].dst]
        mid = plan.n * hb * wb * 64 * esz
        rows[i] = (rows[i][0], rows[i][1] + rows[i + 1][1], rows[i][2] + rows[i + 1][2] - 3 * mid)
        rows[i + 1] = (rows[i + 1][0], 0.0, 0.0)
    segf = getattr(plan, "seg_fused", None)
    if video and segf is not None and plan.labels_path() == "seg2":
        # the seg classifier in the last conv's epilogue (drnmi_conv_stag_seg): the conv's output is
        # neither written nor read back, nor are the fp32 logits; the two partial-logit planes are
        # written by it and read by the head instead
        j, i = segf["conv"], plan.seg_idx
        oh, ow = plan.shapes[nodes[j].dst]
        act = plan.n * oh * ow * nodes[j].conv.out_channels * (1 if nodes[j].i8 else esz)   # int8 nets: int8
        lh, lw = plan.shapes[nodes[i].dst]
        logits = plan.n * lh * lw * nodes[i].conv.out_channels * 4
        part = 2 * plan.n * lh * lw * plan.SEG_NHWC_CS * 4
        rows[j] = (rows[j][0], rows[j][1] + rows[i][1], rows[j][2] + rows[i][2] - 2 * act - logits + part)
        rows[i] = (rows[i][0], 0.0, 0.0)
        rows[-1] = (rows[-1][0], rows[-1][1], rows[-1][2] - logits + part)
    return rows


def _t_star(rows, peaks):
    return sum(max(f / pk_, b / HBM_PEAK_BPS) for (_, f, b), pk_ in zip(rows, peaks))


def network_roofline(plan, video: bool = True):
    """T* two ways: per layer (every conv charged its unfused bytes) and the fused floor (the
    launches the plan issues, charged the bytes they move: launch_work).  The fused floor is the
    smaller, honest bound; bench.py reports frac against it."""
    rows = node_work(plan)
    peaks = node_peaks(plan)
    fused = launch_work(plan, video)
    return {
        "flops": sum(f for _, f, _ in rows),
        "bytes": sum(b for _, _, b in rows),
        "fused_bytes": sum(b for _, _, b in fused),
        "t_star_s": _t_star(rows, peaks),
        "t_star_fused_s": _t_star(fused, peaks),
        "t_mfma_s": sum(f / pk_ for (_, f, _), pk_ in zip(rows, peaks)),
        "t_hbm_s": sum(b for _, _, b in rows) / HBM_PEAK_BPS,
    }
