"""Vendor-library ceilings for the conv shapes of scripts/conv_micro.py (diagnostic only):
hipBLASLt GEMM of the equivalent implicit-GEMM size (M = B*Ho*Wo, N = Cout, K = Cin*k*k, bf16)
and MIOpen conv2d (channels_last bf16).  python scripts/vendor_micro.py [batch]"""
import sys

import torch
import torch.nn.functional as F

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
SHAPES = [  # name, cin, cout, ks, stride, dil, H, W
    ("l8 512x512 d1", 512, 512, 3, 1, 1, 128, 256),
    ("l6 512x512 d4", 512, 512, 3, 1, 4, 128, 256),
    ("l5 256x256 d2", 256, 256, 3, 1, 2, 128, 256),
    ("l4 128x128", 128, 128, 3, 1, 1, 128, 256),
    ("l3 64x64", 64, 64, 3, 1, 1, 256, 512),
    ("l6 ds 256->512 1x1", 256, 512, 1, 1, 1, 128, 256),
]


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


for name, cin, cout, ks, st, dil, h, w in SHAPES:
    pad = dil * (ks // 2)
    m, k = B * h * w, cin * ks * ks
    flops = 2.0 * m * cout * k
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    bt = torch.randn(k, cout, device="cuda", dtype=torch.bfloat16)
    t_gemm = timeit(lambda: torch.mm(a, bt))
    del a, bt
    x = torch.randn(B, cin, h, w, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    wt = torch.randn(cout, cin, ks, ks, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    try:
        t_conv = timeit(lambda: F.conv2d(x, wt, None, st, pad, dil))
        conv = f"{t_conv:8.1f}us {flops / t_conv / 1e6:7.1f}TF"
    except RuntimeError as e:  # noqa: BLE001
        conv = f"error {str(e)[:40]}"
    print(f"{name:22s} | hipBLASLt gemm {t_gemm:8.1f}us {flops / t_gemm / 1e6:7.1f}TF | MIOpen conv {conv}",
          flush=True)
