"""Evaluation drivers on the GPU: the callers of the hot path in semantic_seg.py (SURVEY.md §8a
rows a18/a19, §8f row 4), same names and arguments.

  test(eval_data_loader, model, num_classes, has_gt=True)        semantic_seg.py:429-468
  val_miou(val_loader, model, num_classes, args=None, has_gt=True) semantic_seg.py:638-671
  test_ms(eval_data_loader, model, num_classes, scales, has_gt=True) semantic_seg.py:507-557
  resize_4d_tensor(tensor, width, height)                         semantic_seg.py:471-504

Everything per image stays on the device: the forward (DRNSeg, HIP engine), the Pillow-exact
bilinear resize of every log-prob plane and the fp32 scale sum (drnmi_resize_bilinear_f32,
accumulate), the argmax (drnmi_argmax_nchw_f32) and the confusion matrix (drnmi_confusion_matrix).
Only the 19 x 19 histogram ever comes back to the host.  Deviations: no save_vis / output_dir
(image writing is out of scope), and the loader's tensors are moved to the model's device.
"""
from __future__ import annotations

import numpy as np
import torch

from . import metrics, ops


def resize_4d_tensor(tensor: torch.Tensor, width: int, height: int) -> torch.Tensor:
    """[N, C, h, w] fp32 -> [N, C, height, width] with Pillow's Image.resize(BILINEAR) 'F'-mode
    arithmetic per plane (the reference runs it per channel in threads on the CPU).  Returns the
    tensor itself when the size already matches, as the reference does."""
    if tensor.size(2) == height and tensor.size(3) == width:
        return tensor
    return ops.resize_bilinear_f32(tensor.float().contiguous(), (height, width))


def _device_of(model):
    return next(model.parameters()).device


def _miou_of(hist: torch.Tensor) -> float:
    ious = metrics.per_class_iu(hist) * 100
    return round(float(np.nanmean(ious)), 2)


def _unwrap(model):
    """The DRNSeg inside a DataParallel / DDP wrapper (semantic_seg.py:812 and :1074 hand the
    wrapped model to val_miou; the multigpu script hands a DDP one)."""
    while hasattr(model, "module") and not hasattr(model, "predict"):
        model = model.module
    return model


def test(eval_data_loader, model, num_classes, has_gt=True, **_unused):
    """Single-scale eval loop: model(image)[0] -> torch.max(final, 1) -> fast_hist (on the GPU)."""
    model.eval()
    model = _unwrap(model)
    dev = _device_of(model)
    hist = torch.zeros(num_classes, num_classes, dtype=torch.int64, device=dev)
    for it, batch in enumerate(eval_data_loader):
        image = batch[0].to(dev)
        pred = model.predict(image)                  # fused forward + argmax (int64 labels)
        if has_gt:
            metrics.fast_hist(pred, batch[1].to(dev).long().reshape(pred.shape), num_classes, hist)
    if has_gt:
        return _miou_of(hist)
    return None


def val_miou(val_loader, model, num_classes, args=None, has_gt=True):
    """semantic_seg.py:638-671 -- the same loop over (image, label) batches."""
    return test(val_loader, model, num_classes, has_gt=has_gt)


def test_ms(eval_data_loader, model, num_classes, scales, has_gt=True, **_unused):
    """Multi-scale eval: the log-probs of the image and of its len(scales) rescaled copies (the
    loader's SegListMS items: image, label, name, *scaled images) are each resized to the input
    size and summed in fp32 in the reference's order, then argmax(axis=1) and fast_hist."""
    model.eval()
    model = _unwrap(model)
    dev = _device_of(model)
    hist = torch.zeros(num_classes, num_classes, dtype=torch.int64, device=dev)
    num_scales = len(scales)
    preds = []
    for it, input_data in enumerate(eval_data_loader):
        label = input_data[1] if has_gt else None
        h, w = input_data[0].size()[2:4]
        images = [input_data[0]]
        images.extend(input_data[-num_scales:])
        final = None
        for image in images:
            out = model(image.to(dev))[0]
            if final is None:
                final = resize_4d_tensor(out, w, h).clone()   # 0 + out_0: the sum's first term is exact
            elif out.size(2) == h and out.size(3) == w:
                final += out
            else:                                             # final += resize(out), fp32, in order
                ops.resize_bilinear_f32(out, (h, w), out=final, accumulate=True)
        pred = ops.argmax_nchw(final)
        preds.append(pred)
        if has_gt:
            metrics.fast_hist(pred, label.to(dev).long().reshape(pred.shape), num_classes, hist)
    if has_gt:
        return _miou_of(hist)
    return preds


__all__ = ["resize_4d_tensor", "test", "val_miou", "test_ms"]
