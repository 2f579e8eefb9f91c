"""ORACLE — test infrastructure only (never imported by the product path).

numpy restatement of drnmi's W8A8 convolution (BASELINE config C5, include/drnmi.h
drnmi_conv_args int8 fields) and of the int8 quantiser (drnmi_quantize_i8).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this file.

Parity status: the reference has NO quantisation code (a grep for
quant/int8/qint finds nothing), so the int8 scheme itself is ours and "parity unpinned" against
the reference.  What this file pins is the arithmetic: every int8 launch is checked bit for bit
against it on the launch's own inputs (tests/test_gpu_int8.py), and the int8 network is gated
against the reference's fp32 forward (oracle/drn_oracle.py, pinned by the reference goldens)
by label agreement.

Arithmetic (one fp32 rounding per step, no fused multiply-add):
  acc  = sum_k x_i8[m, k] * w_i8[c, k]                (exact int32; k = (kh*ks + kw)*cin + ci,
                                                       the packed layout of lmodels/drn.py:27-29
                                                       conv3x3 / :181-186 downsample / 1x1 seg)
  v    = fl(fl(float(acc) * scale[c]) + shift[c])    (BN folded: lmodels/drn.py:7 eval BN)
  v    = fl(v + fl(float(res) * res_scale))           (residual add, lmodels/drn.py:60-63)
  v    = max(v, 0) if relu
  out  = clamp(rint(fl(v * out_scale)), -127, 127)   (int8 out; rint = round half to even)
       | bf16(v) (round to nearest even) | v (fp32 out)
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def quantize_i8(x: np.ndarray, inv_scale: float) -> np.ndarray:
    """drnmi_quantize_i8: clamp(rint(x * inv_scale), -127, 127), x already fp32-representable."""
    v = np.rint(x.astype(F32) * F32(inv_scale))
    return np.clip(v, -127, 127).astype(np.int8)


def bf16_bits(v: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 (round to nearest even) as uint16 bit patterns (finite inputs)."""
    b = v.astype(F32).view(np.uint32).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) >> 16
    return b.astype(np.uint16)


def bf16_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(F32)


def im2col_nhwc(x: np.ndarray, ks: int, stride: int, pad: int, dil: int):
    """x [n, h, w, c] -> cols [n*ho*wo, ks*ks*c] with column (kh*ks + kw)*c + ci, zero padding."""
    n, h, w, c = x.shape
    ho = (h + 2 * pad - dil * (ks - 1) - 1) // stride + 1
    wo = (w + 2 * pad - dil * (ks - 1) - 1) // stride + 1
    xp = np.zeros((n, h + 2 * pad, w + 2 * pad, c), dtype=x.dtype)
    xp[:, pad:pad + h, pad:pad + w] = x
    cols = np.empty((n, ho, wo, ks * ks, c), dtype=x.dtype)
    for kh in range(ks):
        for kw in range(ks):
            r0, c0 = kh * dil, kw * dil
            cols[:, :, :, kh * ks + kw] = xp[:, r0:r0 + stride * (ho - 1) + 1:stride,
                                             c0:c0 + stride * (wo - 1) + 1:stride]
    return cols.reshape(n * ho * wo, ks * ks * c), ho, wo


def conv_i8(x: np.ndarray, wpk: np.ndarray, scale: np.ndarray, shift: np.ndarray, cout: int,
            ks: int, stride: int, pad: int, dil: int, relu: bool, res: np.ndarray | None = None,
            res_scale: float = 0.0, out: str = "i8", out_scale: float = 1.0) -> np.ndarray:
    """One int8 conv launch.  x int8 NHWC [n, h, w, cin]; wpk int8 [cout_pad, k_pad] packed;
    res int8 [n, ho, wo, cout].  Returns NHWC [n, ho, wo, cout]: int8, uint16 bf16 bits or fp32."""
    n = x.shape[0]
    cols, ho, wo = im2col_nhwc(x, ks, stride, pad, dil)
    k = cols.shape[1]
    acc = cols.astype(np.int64) @ wpk[:cout, :k].astype(np.int64).T      # exact
    assert np.abs(acc).max(initial=0) < 2 ** 31
    v = acc.astype(np.int32).astype(F32) * scale[:cout].astype(F32)
    v = (v + shift[:cout].astype(F32)).astype(F32)
    if res is not None:
        v = v + res.reshape(-1, cout).astype(F32) * F32(res_scale)
    if relu:
        v = np.maximum(v, F32(0))
    v = v.reshape(n, ho, wo, cout)
    if out == "i8":
        return np.clip(np.rint(v * F32(out_scale)), -127, 127).astype(np.int8)
    if out == "bf16":
        return bf16_bits(v)
    return v.astype(F32)


def quantize_weight_rows(w: np.ndarray):
    """Per-output-channel symmetric int8 of packed fp32 weights [rows, k]:
    s = absmax / 127 (1 for all-zero rows), q = clamp(rint(w * (127 / absmax)), -127, 127).
    Mirrors drnmi/engine.py _quantize_rows (host packing); returns (q int8, s fp32)."""
    a = np.abs(w).max(axis=1).astype(F32)
    inv = np.where(a > 0, F32(127) / np.where(a > 0, a, F32(1)), F32(1)).astype(F32)
    q = np.clip(np.rint(w.astype(F32) * inv[:, None]), -127, 127).astype(np.int8)
    s = np.where(a > 0, a / F32(127), F32(1)).astype(F32)
    return q, s
