"""Fused video front (drnmi_video_front_u8, csrc/front.hip): layer0 + layer1 + layer2 from the
uint8 frame in one launch.

CPU: the host packing (drnmi_front_pack) replayed by the lane-level emulator (tests/front_emul.py)
against a plain fp32 torch restatement of lmodels/drn.py:132-137, :201-211 on the normalised frame
(data_transforms.py:109-125) -- borders, ragged strips and the BGR flag included.
GPU: the kernel against the emulator (same packed parameters, same roundings of the stored
activations) and the network with the front against the reference labels.

Tolerances (bf16 perf mode, written here): the emulator vs the fp32 restatement differs by the bf16
roundings of the folded weights and of the two stored 16-channel activations plus the output's own
rounding: |emu - ref| <= 2^-6 |ref| + 6e-3 max|ref|.  The kernel vs the emulator differs only in the
fp32 accumulation order (float64 in the emulator), i.e. an occasional one-ulp flip of a stored bf16
intermediate: |gpu - emu| <= 2^-7 |emu| + 2e-3 max|emu|, and at most 0.5 % of the outputs beyond
2^-8 |emu| + 1e-4.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import front_emul as fe
from drnmi import _lib

MEAN, STD = [0.29010095, 0.32808144, 0.28696345], [0.1829540508, 0.18656234, 0.18447035]
SHAPES = [(2, 20, 44, False), (1, 9, 12, True), (1, 33, 64, False), (2, 70, 128, True)]


def _params(seed=1):
    return fe.random_params(seed)


def _frames(n, h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (n, h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("n,h,w,bgr", SHAPES)
def test_front_pack_emulation_matches_reference(n, h, w, bgr):
    lib = _lib.load()
    p = _params()
    fr = _frames(n, h, w, h * w)
    blob = fe.pack_front(lib, *p, MEAN, STD, bgr)
    emu = fe.emulate(blob, fr)
    ref = fe.torch_reference(fr, *p, MEAN, STD, bgr)
    assert emu.shape == ref.shape == (n, (h + 1) // 2, (w + 1) // 2, 32)
    bound = 2.0 ** -6 * np.abs(ref) + 6e-3 * np.abs(ref).max()
    d = np.abs(emu - ref)
    assert (d <= bound).all(), float((d - bound).max())


def test_front_supported_shapes():
    lib = _lib.load()
    assert lib.drnmi_front_supported(8, 1024, 2048) == 1
    assert lib.drnmi_front_supported(1, 300, 300) == 1
    assert lib.drnmi_front_supported(1, 7, 64) == 0          # h < 8
    assert lib.drnmi_front_supported(1, 64, 126) == 0        # w % 4 != 0
    assert lib.drnmi_front_supported(400, 1024, 2048) == 0   # > 2^31 frame bytes
    assert lib.drnmi_front_pack_bytes() > 0


def _run_gpu(blob, fr):
    lib = _lib.load()
    n, h, w, _ = fr.shape
    x = torch.from_numpy(fr).cuda()
    pk = torch.from_numpy(blob).cuda()
    y = torch.full((n, (h + 1) // 2, (w + 1) // 2, 32), float("nan"), dtype=torch.bfloat16, device="cuda")
    _lib.check(lib.drnmi_video_front_u8(x.data_ptr(), pk.data_ptr(), y.data_ptr(), n, h, w,
                                        _lib.stream_ptr()), "video_front_u8")
    torch.cuda.synchronize()
    return y.float().cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,bgr", SHAPES + [(3, 130, 260, False), (3, 512, 1024, False)])
def test_front_kernel_matches_emulation(n, h, w, bgr):
    """Every output element written (no NaN left), and equal to the emulator up to accumulation order.
    (3, 512, 1024): 13,824 rows of work over the persistent waves, so every wave walks several rows
    and ranges cross strip / frame boundaries (re-primed walks)."""
    lib = _lib.load()
    p = _params(2)
    fr = _frames(n, h, w, 7 * h + w)
    blob = fe.pack_front(lib, *p, MEAN, STD, bgr)
    got = _run_gpu(blob, fr)
    assert not np.isnan(got).any()
    emu = fe.emulate(blob, fr)
    d = np.abs(got - emu)
    scale = np.abs(emu).max()
    assert (d <= 2.0 ** -7 * np.abs(emu) + 2e-3 * scale).all(), float(d.max())
    assert float((d > 2.0 ** -8 * np.abs(emu) + 1e-4).mean()) <= 5e-3


@pytest.mark.gpu
def test_front_network_labels():
    """D-22 bf16 video path with the fused front (default) vs the stem+layer1 / layer2 launches and
    vs the fp32 oracle labels at 256x512: same bf16-mode label gates as the rest of the network."""
    from drnmi import engine
    from drnmi.drnseg import build
    from drnmi.weights import synth_frames
    from oracle import drn_oracle as O
    fr_np = synth_frames(21, 2, 256, 512)
    frames = torch.from_numpy(fr_np).cuda()
    m = build("drn_d_22", 19, seed=5, device="cuda", precision="bf16")
    assert m.plan(2, 256, 512).front_fused
    lab = m.segment(frames).long()
    engine.FUSE_FRONT = False
    try:
        m2 = build("drn_d_22", 19, seed=5, device="cuda", precision="bf16")
        assert not m2.plan(2, 256, 512).front_fused
        lab2 = m2.segment(frames).long()
    finally:
        engine.FUSE_FRONT = True
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_lp, _, _ = O.drnseg_forward(sd, "drn_d_22", O.preprocess_u8(fr_np))
    ref = torch.max(ref_lp, 1)[1]
    agree = float((lab == lab2).float().mean())
    a_front = float((lab.cpu() == ref).float().mean())
    a_sep = float((lab2.cpu() == ref).float().mean())
    print(f"front vs separate launches {agree:.4f}; vs fp32 oracle: front {a_front:.4f}, separate {a_sep:.4f}")
    assert agree >= 0.99 and a_front >= 0.99           # measured 0.9937 / 0.9951
