"""Lane-level numpy restatement of csrc/front.hip (drnmi_video_front_u8) -- TEST INFRASTRUCTURE.

It reads the blob drnmi_front_pack writes and replays the kernel's pixel-pair MFMA dataflow
(v_mfma_f32_32x32x16 fragment layouts, the f16 frame image 1024 + u8, the border-case stem
shifts, the left/right-neighbour operands of the 3x3 convs, bf16 rounding of every stored
activation) with float64 sums.  The CPU test checks it against a plain fp32 torch restatement
of layer0..layer2 (lmodels/drn.py:132-137, :201-211 on the normalised frame,
data_transforms.py:109-125) -- which pins the packing and the dataflow without a GPU -- and the
GPU test checks the kernel against it.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

PACK_FRAGS = (11, 12, 9)


def bf16_round(x: np.ndarray) -> np.ndarray:
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(torch.bfloat16).float().numpy()


def pack_front(lib, w0, s0, b0, w1, s1, b1, w2, s2, b2, mean, std, bgr) -> np.ndarray:
    """drnmi_front_pack on host float32 arrays -> uint8 blob."""
    out = np.zeros(int(lib.drnmi_front_pack_bytes()), dtype=np.uint8)
    arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (w0, s0, b0, w1, s1, b1, w2, s2, b2, mean, std)]
    ptrs = [a.ctypes.data_as(ctypes.c_void_p) for a in arrs]
    rc = lib.drnmi_front_pack(*ptrs, 1 if bgr else 0, out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
    return out


def unpack(blob: np.ndarray):
    fs, f1, f2 = PACK_FRAGS
    off = 0
    frags = []
    for nf, dt in ((fs, np.float16), (f1, None), (f2, None)):
        raw = blob[off:off + nf * 64 * 16].view(np.uint16).reshape(nf, 64, 8)
        if dt is np.float16:
            v = raw.view(np.float16).astype(np.float64)
        else:
            v = (raw.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
        # A[m][i][k] = frag[m][i + 32 h][e], k = 8 h + e
        a = np.concatenate([v[:, :32, :], v[:, 32:, :]], axis=2)      # [m][32][16]
        frags.append(a)
        off += nf * 64 * 16
    c0 = blob[off:off + 64 * 16 * 4].view(np.float32).reshape(8, 8, 16).astype(np.float64)[:7, :7]
    off += 64 * 16 * 4
    c1 = blob[off:off + 64].view(np.float32).astype(np.float64)
    off += 64
    c2 = blob[off:off + 128].view(np.float32).astype(np.float64)
    return frags[0], frags[1], frags[2], c0, c1, c2


def _case(v, size):
    """border case index of the kernel: 0, 1, 2 | 3 interior | 4, 5, 6"""
    return np.where(v < 3, v, np.where(v >= size - 3, 6 - (size - 1 - v), 3))


def emulate(blob: np.ndarray, frames: np.ndarray) -> np.ndarray:
    """frames uint8 [n][H][W][3] -> layer2 output float32 [n][(H+1)//2][(W+1)//2][32] (bf16 values)."""
    As, A1, A2, C0, C1, C2 = unpack(blob)
    n, H, W, _ = frames.shape
    H2, W2 = (H + 1) // 2, (W + 1) // 2
    # f16 image of every frame row: value 1024 + byte, padded with zeros outside the image
    pad = 12
    img = np.zeros((n, H + 16, 3 * (W + 2 * pad)), dtype=np.float64)
    img[:, 8:8 + H, 3 * pad:3 * (pad + W)] = 1024.0 + frames.reshape(n, H, 3 * W).astype(np.float64)

    def img_row(fr):                    # [n][bytes] of frame row fr (zeros outside)
        return img[:, fr + 8, :]

    # stem over pixel pairs (c, c+1), c odd, covering every column in [0, W)
    cs = np.arange(-1, W, 2)                                   # pair left columns
    npair = cs.size
    stem = np.zeros((n, H, W, 16), dtype=np.float32)
    for q in range(H):
        rc = int(_case(np.array(q), H))
        D = np.zeros((n, npair, 32))
        # window of pair c: pixels c-3 .. c+4 -> bytes 3(c-3) .. +24 in image coords (+3 pad)
        b0 = 3 * (cs - 3 + pad)
        idx = b0[:, None] + np.arange(24)[None, :]            # [npair][24]
        for kh in range(7):
            win = img_row(q - 3 + kh)[:, idx]                 # [n][npair][24]
            B = win[:, :, 0:16]                               # P: chunks 0 (h=0), 1 (h=1)
            D += B @ As[kh].T
        for t in range(4):
            wa = img_row(q - 3 + 2 * t)[:, idx][:, :, 16:24]
            wb = img_row(q - 2 + 2 * t)[:, idx][:, :, 16:24]
            B = np.concatenate([wa, wb], axis=2)
            D += B @ As[7 + t].T
        # D row i -> (sp = (i>>2)&1, co = (i&3) + 4(i>>3))
        for i in range(32):
            sp, co = (i >> 2) & 1, (i & 3) + 4 * (i >> 3)
            col = cs + sp
            ok = (col >= 0) & (col < W)
            cc = np.clip(_case(col, W), 0, 6)
            v = D[:, :, i] + C0[rc, cc, co][None, :]
            stem[:, q, col[ok], co] = np.maximum(v[:, ok], 0.0)
    stem = bf16_round(stem).astype(np.float64)

    def shifted(t, rows, cols):
        """t [n][H][W][C] sampled at (rows, cols) grids with zero outside"""
        Hh, Ww = t.shape[1], t.shape[2]
        out = np.zeros((t.shape[0], len(rows), len(cols), t.shape[3]))
        rr = np.asarray(rows)
        cc = np.asarray(cols)
        rok = (rr >= 0) & (rr < Hh)
        cok = (cc >= 0) & (cc < Ww)
        sub = t[:, np.clip(rr, 0, Hh - 1)][:, :, np.clip(cc, 0, Ww - 1)]
        return sub * (rok[None, :, None, None] & cok[None, None, :, None])

    # layer1 over the same pairs
    l1 = np.zeros((n, H, W, 16), dtype=np.float32)
    rows = np.arange(H)
    D = np.zeros((n, H, npair, 32)) + 0.0
    for kh in range(3):
        sr = rows - 1 + kh
        own0 = shifted(stem, sr, cs)          # pixel c (sp 0)
        own1 = shifted(stem, sr, cs + 1)      # pixel c + 1
        left = shifted(stem, sr, cs - 1)
        right = shifted(stem, sr, cs + 2)
        Ba = np.concatenate([own0[..., 0:8], own1[..., 0:8]], axis=3)
        Bb = np.concatenate([own0[..., 8:16], own1[..., 8:16]], axis=3)
        Lra = np.concatenate([left[..., 0:8], right[..., 0:8]], axis=3)
        Lrb = np.concatenate([left[..., 8:16], right[..., 8:16]], axis=3)
        D += Ba @ A1[4 * kh].T + Bb @ A1[4 * kh + 1].T + Lra @ A1[4 * kh + 2].T + Lrb @ A1[4 * kh + 3].T
    for i in range(32):
        sp, co = (i >> 2) & 1, (i & 3) + 4 * (i >> 3)
        col = cs + sp
        ok = (col >= 0) & (col < W)
        l1[:, :, col[ok], co] = np.maximum(D[:, :, ok, i] + C1[co], 0.0)
    l1 = bf16_round(l1).astype(np.float64)

    # layer2: output x uses layer1 columns 2x-1 (kw 0), 2x (kw 1), 2x+1 (kw 2)
    xs = np.arange(W2)
    ys = np.arange(H2)
    D = np.zeros((n, H2, W2, 32))
    for kh in range(3):
        lr = 2 * ys - 1 + kh
        p0 = shifted(l1, lr, 2 * xs - 1)
        p1 = shifted(l1, lr, 2 * xs)
        p2 = shifted(l1, lr, 2 * xs + 1)
        Ba = np.concatenate([p0[..., 0:8], p1[..., 0:8]], axis=3)
        Bb = np.concatenate([p0[..., 8:16], p1[..., 8:16]], axis=3)
        Br = p2
        D += Ba @ A2[3 * kh].T + Bb @ A2[3 * kh + 1].T + Br @ A2[3 * kh + 2].T
    out = np.maximum(D + C2[None, None, None, :], 0.0)
    return bf16_round(out)


def torch_reference(frames: np.ndarray, w0, s0, b0, w1, s1, b1, w2, s2, b2, mean, std, bgr=False) -> np.ndarray:
    """fp32 restatement of layer0..layer2 (eval BN folded as scale/shift) on the normalised frame,
    NHWC [n][H2][W2][32]."""
    x = torch.from_numpy(frames).float()
    if bgr:
        x = x.flip(-1)
    x = x.permute(0, 3, 1, 2) / 255.0
    m = torch.tensor(mean, dtype=torch.float32).view(1, 3, 1, 1)
    s = torch.tensor(std, dtype=torch.float32).view(1, 3, 1, 1)
    x = (x - m) / s

    def cbr(x, w, sc, sh, stride, pad):
        y = torch.nn.functional.conv2d(x, torch.from_numpy(w), stride=stride, padding=pad)
        return torch.relu(y * torch.from_numpy(sc).view(1, -1, 1, 1) + torch.from_numpy(sh).view(1, -1, 1, 1))

    x = cbr(x, w0, s0, b0, 1, 3)
    x = cbr(x, w1, s1, b1, 1, 1)
    x = cbr(x, w2, s2, b2, 2, 1)
    return x.permute(0, 2, 3, 1).contiguous().numpy()


def random_params(seed: int = 0):
    g = np.random.default_rng(seed)
    w0 = g.normal(0, np.sqrt(2 / (49 * 16)), (16, 3, 7, 7)).astype(np.float32)
    w1 = g.normal(0, np.sqrt(2 / (9 * 16)), (16, 16, 3, 3)).astype(np.float32)
    w2 = g.normal(0, np.sqrt(2 / (9 * 32)), (32, 16, 3, 3)).astype(np.float32)
    s0, s1, s2 = (g.uniform(0.5, 1.5, c).astype(np.float32) for c in (16, 16, 32))
    b0, b1, b2 = (g.uniform(-0.3, 0.3, c).astype(np.float32) for c in (16, 16, 32))
    return w0, s0, b0, w1, s1, b1, w2, s2, b2
