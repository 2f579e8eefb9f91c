"""ORACLE — test infrastructure only (never imported by the product path).

CPU fp32 restatement of the reference DRN-D segmentation forward, written as plain
functional torch-CPU ops over a state_dict, so it does not depend on the reference's
module classes nor on drnmi's.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this file.

Pinned by: tests/golden/*.npz produced by tests/golden/make_golden.py, which runs
the reference's own lmodels/drnseg.py / drn.py modules in this container with the
same hash-initialised state_dicts (tests/test_oracle_golden.py checks max-abs 0 on
logits / log-probs and exact labels).

Reference anchors (paths relative to the reference repo):
  conv3x3                       lmodels/drn.py:27-29
  BasicBlock.forward            lmodels/drn.py:49-65
  Bottleneck.forward            lmodels/drn.py:86-106
  DRN.__init__ (arch D layout)  lmodels/drn.py:109-176 ; _make_layer :177-199 ;
                                _make_conv_layers :201-211 ; forward :213-259
  DRNSeg head                   lmodels/drnseg.py:268-299 (seg 1x1+bias, up convT k16 s8 p4
                                groups=C, LogSoftmax over dim 1)
  per-pixel argmax              semantic_seg.py:445 / seg_video_old_no_plot.py:166
  preprocessing                 data_transforms.py:109-125 (Normalize), :256-281
                                (ToTensorVideoImage); constants info.json:1
  BN (eval)                     nn.BatchNorm2d, eps 1e-5 (lmodels/drn.py:7)
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

# (block kind, blocks per layer) — lmodels/drn.py:361-393
ARCHS = {
    "drn_d_22": ("basic", [1, 1, 2, 2, 2, 2, 1, 1]),
    "drn_d_24": ("basic", [1, 1, 2, 2, 2, 2, 2, 2]),
    "drn_d_38": ("basic", [1, 1, 3, 4, 6, 3, 1, 1]),
    "drn_d_40": ("basic", [1, 1, 3, 4, 6, 3, 2, 2]),
    "drn_d_54": ("bottleneck", [1, 1, 3, 4, 6, 3, 1, 1]),
    "drn_d_56": ("bottleneck", [1, 1, 3, 4, 6, 3, 2, 2]),
}

INFO_MEAN = (0.29010095242892997, 0.32808144844279574, 0.28696394422942517)
INFO_STD = (0.1829540508368939, 0.18656561047509476, 0.18447508988480435)


_TRAIN = {"on": False}


def _bn(sd, p, x):
    """BatchNorm2d (lmodels/drn.py:7): eval uses running stats; train mode (the fine-tune
    path) normalises by batch stats and updates the running stats in place (momentum 0.1,
    unbiased running var) and num_batches_tracked."""
    if _TRAIN["on"]:
        if (p + ".num_batches_tracked") in sd:
            sd[p + ".num_batches_tracked"] += 1
        return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                            sd[p + ".bias"], training=True, momentum=0.1, eps=1e-5)
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], training=False, momentum=0.0, eps=1e-5)


def _conv(sd, p, x, stride=1, padding=0, dilation=1, bias=False):
    return F.conv2d(x, sd[p + ".weight"], sd[p + ".bias"] if bias else None,
                    stride=stride, padding=padding, dilation=dilation)


def _conv_layers(sd, p, x, n, stride, dilation):
    """_make_conv_layers (lmodels/drn.py:201-211): [conv3x3 s/d -> BN -> ReLU] x n."""
    for i in range(n):
        x = _conv(sd, f"{p}.{3 * i}", x, stride=stride if i == 0 else 1, padding=dilation, dilation=dilation)
        x = F.relu(_bn(sd, f"{p}.{3 * i + 1}", x))
    return x


def _basic(sd, p, x, stride, dil):
    """BasicBlock.forward (lmodels/drn.py:49-65), residual=True for arch D."""
    out = F.relu(_bn(sd, p + ".bn1", _conv(sd, p + ".conv1", x, stride, dil[0], dil[0])))
    out = _bn(sd, p + ".bn2", _conv(sd, p + ".conv2", out, 1, dil[1], dil[1]))
    res = x
    if (p + ".downsample.0.weight") in sd:
        res = _bn(sd, p + ".downsample.1", _conv(sd, p + ".downsample.0", x, stride))
    return F.relu(out + res)


def _bottleneck(sd, p, x, stride, dil):
    """Bottleneck.forward (lmodels/drn.py:86-106)."""
    out = F.relu(_bn(sd, p + ".bn1", _conv(sd, p + ".conv1", x)))
    out = F.relu(_bn(sd, p + ".bn2", _conv(sd, p + ".conv2", out, stride, dil[1], dil[1])))
    out = _bn(sd, p + ".bn3", _conv(sd, p + ".conv3", out))
    res = x
    if (p + ".downsample.0.weight") in sd:
        res = _bn(sd, p + ".downsample.1", _conv(sd, p + ".downsample.0", x, stride))
    return F.relu(out + res)


def _res_layer(sd, p, x, kind, nblocks, stride, dilation, new_level):
    """_make_layer (lmodels/drn.py:177-199): first block gets stride and
    dilation (1,1) | (d//2 if new_level else d, d); the rest (d, d)."""
    blk = _basic if kind == "basic" else _bottleneck
    first = (1, 1) if dilation == 1 else ((dilation // 2) if new_level else dilation, dilation)
    x = blk(sd, f"{p}.0", x, stride, first)
    for b in range(1, nblocks):
        x = blk(sd, f"{p}.{b}", x, 1, (dilation, dilation))
    return x


def backbone(sd, arch, x, prefix="layer"):
    """DRN-D trunk through layer8 (lmodels/drn.py:213-259), returns (x, stage outputs)."""
    kind, layers = ARCHS[arch]
    stages = {}
    x = F.relu(_bn(sd, f"{prefix}.0.1", _conv(sd, f"{prefix}.0.0", x, 1, 3)))
    stages["layer0"] = x
    x = _conv_layers(sd, f"{prefix}.1", x, layers[0], 1, 1)
    stages["layer1"] = x
    x = _conv_layers(sd, f"{prefix}.2", x, layers[1], 2, 1)
    stages["layer2"] = x
    x = _res_layer(sd, f"{prefix}.3", x, kind, layers[2], 2, 1, True)
    stages["layer3"] = x
    x = _res_layer(sd, f"{prefix}.4", x, kind, layers[3], 2, 1, True)
    stages["layer4"] = x
    x = _res_layer(sd, f"{prefix}.5", x, kind, layers[4], 1, 2, False)
    stages["layer5"] = x
    idx = 6
    if layers[5] > 0:
        x = _res_layer(sd, f"{prefix}.{idx}", x, kind, layers[5], 1, 4, False)
        stages["layer6"] = x
        idx += 1
    if layers[6] > 0:
        x = _conv_layers(sd, f"{prefix}.{idx}", x, layers[6], 1, 2)
        stages["layer7"] = x
        idx += 1
    if layers[7] > 0:
        x = _conv_layers(sd, f"{prefix}.{idx}", x, layers[7], 1, 1)
        stages["layer8"] = x
    return x, stages


def up_logsoftmax(sd, logits):
    """up = depthwise ConvTranspose2d(C, C, 16, stride 8, pad 4) + LogSoftmax(dim 1)
    (lmodels/drnseg.py:285-299).  Without "up.weight" in sd (DRNSeg(use_torch_up=True)): up =
    nn.UpsamplingBilinear2d(scale_factor=8) (lmodels/drnseg.py:285-287), i.e. bilinear with
    align_corners=True."""
    if "up.weight" not in sd:
        y = F.interpolate(logits, scale_factor=8, mode="bilinear", align_corners=True)
        return F.log_softmax(y, dim=1)
    c = logits.shape[1]
    y = F.conv_transpose2d(logits, sd["up.weight"], None, stride=8, padding=4, groups=c)
    return F.log_softmax(y, dim=1)


@torch.no_grad()
def drnseg_forward(sd, arch, x):
    """(log_probs, logits, stages) of DRNSeg.forward for a state_dict (keys layer.*/seg.*/up.*;
    no up.weight = the use_torch_up head)."""
    sd = {k: v.float() for k, v in sd.items()}
    feat, stages = backbone(sd, arch, x.float())
    logits = _conv(sd, "seg", feat, bias=True)
    return up_logsoftmax(sd, logits), logits, stages


def labels_of(logprobs):
    """torch.max(final, 1)[1] (semantic_seg.py:445)."""
    return torch.max(logprobs, 1)[1]


def preprocess_u8(frames_hwc: np.ndarray, mean=INFO_MEAN, std=INFO_STD) -> torch.Tensor:
    """uint8 [N,H,W,3] -> fp32 [N,3,H,W]: x.float().div(255) then (x - m) / s per channel,
    the op order of ToTensorVideoImage + Normalize (data_transforms.py:256-281, :109-125)."""
    t = torch.from_numpy(np.ascontiguousarray(frames_hwc)).permute(0, 3, 1, 2).contiguous()
    t = t.float().div(255)
    for c in range(3):
        t[:, c].sub_(mean[c]).div_(std[c])
    return t


TRAINABLE_SUFFIXES = (".weight", ".bias")


def trainable_keys(sd):
    """optim_parameters() of DRNSeg (semantic_seg.py:160-164): every layer.* / seg.* weight and
    bias (convs and BN affine), excluding up.weight."""
    return [k for k in sd if k.endswith(TRAINABLE_SUFFIXES) and not k.startswith("up.")]


def drnseg_train_steps(sd, arch, inputs, targets, lr=0.01, momentum=0.9, weight_decay=1e-4,
                       masks=None, ignore_index=255, dtype=torch.float32):
    """The reference fine-tune loop body (semantic_seg.py:166-230) for len(inputs) steps:
    train-mode forward, CrossEntropyLoss(ignore_index) on the log-probs (:817, :197-198),
    zero_grad, backward, torch.optim.SGD(momentum, weight_decay) step (:963-966), then
    Pruner.apply_masks (:213-214).  Returns (losses, grads of the LAST step, final state_dict);
    sd is not modified.  dtype=torch.float64 gives the exact-arithmetic yardstick the fp32
    implementations (the reference's and ours) are both measured against."""
    sd = {k: v.detach().clone() for k, v in sd.items()}
    for k, v in sd.items():
        if v.is_floating_point():
            sd[k] = v.to(dtype)
    keys = trainable_keys(sd)
    params = [sd[k].requires_grad_(True) for k in keys]
    opt = torch.optim.SGD(params, lr, momentum=momentum, weight_decay=weight_decay)
    losses, grads = [], {}
    _TRAIN["on"] = True
    try:
        for x, t in zip(inputs, targets):
            feat, _ = backbone(sd, arch, x.to(dtype))
            logits = _conv(sd, "seg", feat, bias=True)
            lp = up_logsoftmax(sd, logits)
            loss = F.cross_entropy(lp, t.long(), ignore_index=ignore_index)
            opt.zero_grad()
            loss.backward()
            grads = {k: sd[k].grad.detach().clone() for k in keys}
            opt.step()
            if masks:
                with torch.no_grad():
                    for k, m in masks.items():
                        sd[k].mul_(m.to(dtype))
            losses.append(float(loss.detach()))
    finally:
        _TRAIN["on"] = False
    out = {k: v.detach().clone() for k, v in sd.items()}
    return losses, grads, out


def apply_masks(weights: dict, masks: dict) -> dict:
    """Pruner.apply_masks (pruners/Pruner.py:17-20): w *= mask, elementwise in fp32."""
    return {k: (weights[k] * masks[k]) if k in masks else weights[k] for k in weights}


def fast_hist(pred: np.ndarray, label: np.ndarray, n: int) -> np.ndarray:
    """semantic_seg.py:293-296: n x n confusion over 0 <= label < n."""
    k = (label >= 0) & (label < n)
    return np.bincount(n * label[k].astype(int) + pred[k], minlength=n ** 2).reshape(n, n)


def per_class_iu(hist: np.ndarray) -> np.ndarray:
    """semantic_seg.py:299-300."""
    return np.diag(hist) / (hist.sum(1) + hist.sum(0) - np.diag(hist))
