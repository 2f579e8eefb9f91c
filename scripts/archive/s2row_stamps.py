"""Diagnostic: per-workgroup clock stamps of conv_s2row_kernel (library built with
scripts/build_variant_src.sh s2stamp conv_s2row.hip -DDRNMI_S2_STAMP=1, selected by
DRNMI_LIB=.../libdrnmi_s2stamp.so).  Splits one launch into dispatch skew (workgroup start times),
the first ring fill (weights + 3 input row pairs), the first row step and the rest.
python scripts/s2row_stamps.py [batch]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "video-seg-model-compress_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from drnmi import _lib, ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
lib = _lib.load()
lib.drnmi_diag_s2_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.drnmi_diag_s2_stamps_clear.argtypes = []
TILE = 21   # conv_s2row (csrc/conv_big.hip kS2Row)
for name, cin, cout, h, w in [("l4.0c1 64->128 s2", 64, 128, 256, 512), ("l3.0c1 32->64 s2", 32, 64, 512, 1024)]:
    x = torch.randn(B, h, w, cin, device="cuda").bfloat16()
    wt = torch.randn(cout, cin, 3, 3, device="cuda") * 0.05
    packed = ops.pack_conv_weight(wt, cin, torch.bfloat16)
    for _ in range(20):
        ops.conv2d_bn_act(x, wt, None, None, None, 2, 1, 1, True, tile=TILE, packed=packed, fold_scale=True)
    torch.cuda.synchronize()
    for rep in range(3):
        assert lib.drnmi_diag_s2_stamps_clear() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.conv2d_bn_act(x, wt, None, None, None, 2, 1, 1, True, tile=TILE, packed=packed, fold_scale=True)
        e1.record()
        torch.cuda.synchronize()
        buf = np.zeros((8192, 8), dtype=np.uint64)
        assert lib.drnmi_diag_s2_stamps(buf.ctypes.data_as(ctypes.c_void_p), 8192) == 0
        st = buf[buf[:, 0] != 0].astype(np.float64)
        r0, t0, t_fill, t_step1, t_end, rows, r1, segs = st.T
        clk = (t_end - t0) / ((r1 - r0) / 100e6)          # shader clock from memtime / realtime (100 MHz)
        ghz = np.median(clk) / 1e9
        us = lambda cyc: cyc / (ghz * 1e3)                  # noqa: E731
        rs = (r0 - r0.min()) / 100.0                        # us since the first workgroup started
        re_ = (r1 - r0.min()) / 100.0
        print(f"{name} B={B} rep {rep}: event {e0.elapsed_time(e1) * 1e3:.1f} us, {len(st)} WGs, clock {ghz:.2f} GHz, "
              f"span of stamps {re_.max():.1f} us")
        print(f"  WG start  us: p50 {np.median(rs):.1f} p90 {np.percentile(rs, 90):.1f} max {rs.max():.1f}; "
              f"WG end us: min {re_.min():.1f} p50 {np.median(re_):.1f} max {re_.max():.1f}")
        print(f"  per WG us: total p50 {us(np.median(t_end - t0)):.1f} | first fill {us(np.median(t_fill - t0)):.1f} "
              f"| first step {us(np.median(t_step1 - t_fill)):.2f} | rest {us(np.median(t_end - t_step1)):.1f} "
              f"for {np.median(rows) - 1:.0f} rows ({us(np.median((t_end - t_step1) / np.maximum(rows - 1, 1))):.2f} us/row), "
              f"segments p50 {np.median(segs):.0f} max {segs.max():.0f}")
