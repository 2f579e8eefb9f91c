"""CPU restatement of the reference's eval-side resampling (TEST INFRASTRUCTURE ONLY: imported by
tests/ as the checker, never by the product path).

  resize_4d_tensor   semantic_seg.py:471-504: every fp32 plane through
                     Image.fromarray(plane).resize((w, h), Image.BILINEAR) (Pillow 'F' mode)
  multiscale_pred    semantic_seg.py:537-543: sum of the resized outputs in fp32, argmax(axis=1)
  resize_frame_u8    seg_video_old_no_plot.py:124-127: Image.fromarray(frame, 'RGB') then
                     T.Resize((300, 300)) -- torchvision's PIL path is Image.resize(size[::-1],
                     BILINEAR); torchvision itself is not importable in this image, so the Pillow
                     call it makes is used directly (noted in DESIGN.md)
Pillow (12.2 here and on the GPU box) is the arithmetic the reference calls, so these are the
reference's own numbers, not a re-derivation.
"""
from __future__ import annotations

import numpy as np
from PIL import Image


def resize_4d_tensor(arr: np.ndarray, width: int, height: int) -> np.ndarray:
    arr = np.asarray(arr, dtype=np.float32)
    if arr.shape[2] == height and arr.shape[3] == width:
        return arr
    out = np.empty((arr.shape[0], arr.shape[1], height, width), dtype=np.float32)
    for j in range(arr.shape[1]):
        for i in range(arr.shape[0]):
            out[i, j] = np.array(Image.fromarray(arr[i, j]).resize((width, height), Image.BILINEAR))
    return out


def multiscale_pred(outputs, width: int, height: int) -> np.ndarray:
    final = sum([resize_4d_tensor(o, width, height) for o in outputs])
    return final.argmax(axis=1)


def resize_frame_u8(frame_hwc: np.ndarray, size) -> np.ndarray:
    """size = (oh, ow) as T.Resize takes it."""
    img = Image.fromarray(np.ascontiguousarray(frame_hwc), "RGB")
    return np.array(img.resize((int(size[1]), int(size[0])), Image.BILINEAR))
