"""Segmentation metrics on the GPU (the eval caller of the hot path).

  fast_hist      semantic_seg.py:293-296  -> drnmi_confusion_matrix (HIP, int64 hist)
  per_class_iu   semantic_seg.py:299-300  (19x19 host math)
  miou           semantic_seg.py:468      round(nanmean(iou) * 100, 2)
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

_CODES = {torch.uint8: _lib.DRNMI_U8, torch.int64: _lib.DRNMI_I64}


def fast_hist(pred: torch.Tensor, label: torch.Tensor, n: int, hist: torch.Tensor | None = None) -> torch.Tensor:
    """Accumulate the n x n confusion matrix (rows = label, cols = pred) on the device."""
    if pred.shape != label.shape:
        raise ValueError("pred and label shapes differ")
    if pred.dtype not in _CODES or label.dtype not in _CODES:
        raise TypeError("pred/label must be uint8 or int64")
    if not (pred.is_cuda and label.is_cuda):
        raise RuntimeError("fast_hist runs on the HIP kernel: tensors must be on a ROCm device")
    if pred.device != label.device:
        raise RuntimeError("pred and label are on different devices")
    if not 0 < n <= 32:
        raise ValueError("n must be in 1..32 (drnmi_confusion_matrix)")
    if hist is None:
        hist = torch.zeros(n, n, dtype=torch.int64, device=pred.device)
    elif (hist.dtype != torch.int64 or tuple(hist.shape) != (n, n) or not hist.is_contiguous()
          or hist.device != pred.device):
        raise ValueError(f"hist must be a contiguous int64 ({n}, {n}) tensor on {pred.device}")
    pred, label = pred.contiguous(), label.contiguous()
    lib = _lib.load()
    _lib.check(lib.drnmi_confusion_matrix(pred.data_ptr(), _CODES[pred.dtype], label.data_ptr(),
                                          _CODES[label.dtype], pred.numel(), n, hist.data_ptr(),
                                          ctypes.c_void_p(_lib.stream_ptr(pred.device))), "confusion_matrix")
    return hist


def per_class_iu(hist) -> np.ndarray:
    h = hist.cpu().numpy() if isinstance(hist, torch.Tensor) else np.asarray(hist)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.diag(h) / (h.sum(1) + h.sum(0) - np.diag(h))


def miou(hist) -> float:
    return round(float(np.nanmean(per_class_iu(hist))) * 100, 2)
