"""Micro-benchmark of the fused video front (drnmi_video_front_u8) on n x 1024 x 2048 frames:
HIP-event time per launch (on the launch stream), algorithmic FLOPs and HBM bytes, and the
same work as the previous launches (stem_l1 + layer2 patch kernel) for comparison."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "video-seg-model-compress_amd"), os.path.join(REPO, "tests"), REPO]
from drnmi import _lib  # noqa: E402
import front_emul as fe  # noqa: E402


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    n = int(os.environ.get("N", "8"))
    H, W = int(os.environ.get("H", "1024")), int(os.environ.get("W", "2048"))
    lib = _lib.load()
    p = fe.random_params(3)
    blob = fe.pack_front(lib, *p, [0.29, 0.33, 0.29], [0.18, 0.19, 0.18], False)
    pk = torch.from_numpy(blob).cuda()
    fr = torch.randint(0, 256, (n, H, W, 3), dtype=torch.uint8, device="cuda")
    y = torch.empty(n, (H + 1) // 2, (W + 1) // 2, 32, dtype=torch.bfloat16, device="cuda")
    st = _lib.stream_ptr()

    def run():
        _lib.check(lib.drnmi_video_front_u8(fr.data_ptr(), pk.data_ptr(), y.data_ptr(), n, H, W,
                                            ctypes.c_void_p(st)), "front")

    us = timeit(run)
    macs = n * H * W * (147 + 144) * 16 + n * ((H + 1) // 2) * ((W + 1) // 2) * 144 * 32
    byts = n * H * W * 3 + y.numel() * 2
    print(f"front n={n} {H}x{W}: {us:.1f} us  {2 * macs / us / 1e6:.1f} TFLOP/s "
          f"({2 * macs / us / 1e6 / 2500:.3f} of 2.5 PF)  {byts / us / 1e3:.0f} GB/s  "
          f"floor mfma {2 * macs / 2.5e15 * 1e6:.1f} us hbm {byts / 8e12 * 1e6:.1f} us")

    # the launches it replaces: stem_l1 (layer0 + layer1) + layer2 on the patch kernel
    if os.environ.get("CMP", "1") == "1":
        from drnmi.drnseg import build
        from drnmi import engine
        engine.FUSE_FRONT = False
        m = build("drn_d_22", 19, seed=0, device="cuda", precision="bf16")
        plan = m.plan(n, H, W)
        m.segment(fr)
        a1 = plan.args[1]

        def old():
            _lib.check(lib.drnmi_stem_layer1(ctypes.byref(plan.stem_u8), ctypes.byref(a1), ctypes.c_void_p(st)), "sl1")
            _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(plan.args[2]), ctypes.c_void_p(st)), "l2")

        us2 = timeit(old)
        print(f"stem_l1 + layer2 launches: {us2:.1f} us")


if __name__ == "__main__":
    main()
