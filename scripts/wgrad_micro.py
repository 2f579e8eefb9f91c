"""Diagnostic: the fp32x weight-gradient kernels on D-54 fine-tune shapes (2 x 128 x 96 pixels),
timed with HIP events; run under rocprofv3 --pmc for counters.  python scripts/wgrad_micro.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import _lib  # noqa: E402

SHAPES = [  # name, cin, cout, ks, dil, h, w
    ("layer7.0 conv1 2048->512 d2", 2048, 512, 3, 2, 128, 96),
    ("layer6 conv2 512->512 d4", 512, 512, 3, 4, 128, 96),
    ("layer5 conv3 256->1024 1x1", 256, 1024, 1, 1, 128, 96),
]
lib = _lib.load()
n = 2
for name, cin, cout, ks, dil, h, w in SHAPES:
    pad = dil * (ks // 2)
    x = torch.randn(n * h * w, cin, device="cuda")
    dy = torch.randn(n * h * w, cout, device="cuda")
    dw = torch.empty(cout, cin, ks, ks, device="cuda")
    a = _lib.WgradArgs()
    a.dy, a.x, a.dw = dy.data_ptr(), x.data_ptr(), dw.data_ptr()
    a.n, a.h, a.w, a.cin, a.cin_stride = n, h, w, cin, cin
    a.ho, a.wo, a.cout, a.dy_stride = h, w, cout, cout
    a.ks, a.stride, a.pad, a.dil = ks, 1, pad, dil
    a.accumulate = 0
    nb = lib.drnmi_conv_wgrad_workspace_bytes(ctypes.byref(a))
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    a.ws, a.ws_bytes = ws.data_ptr(), nb
    sp = ctypes.c_void_p(_lib.stream_ptr())
    for _ in range(2):
        _lib.check(lib.drnmi_conv_wgrad_f32x3(ctypes.byref(a), sp), "wgrad")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        _lib.check(lib.drnmi_conv_wgrad_f32x3(ctypes.byref(a), sp), "wgrad")
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 5 * 1e3
    fl = 2.0 * n * h * w * cout * cin * ks * ks
    print(f"{name:32s} {us:8.1f} us/call (incl. reduce) {fl / us / 1e6:6.1f} TF  ws {nb / 2**20:.0f} MiB", flush=True)
