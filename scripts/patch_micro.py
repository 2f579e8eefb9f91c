"""Micro-benchmark of the full-resolution patch kernels (stem u8 7x7, layer1 16->16, layer2
16->32 s2) at 1024x2048, batch B (diagnostic).  python scripts/patch_micro.py [batch]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import _lib, ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
H, W = 1024, 2048
dev = "cuda"
frames = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev)
w0 = torch.randn(16, 3, 7, 7, device=dev) * 0.1
one16, zero16 = torch.ones(16, device=dev), torch.zeros(16, device=dev)
x1 = torch.randn(B, H, W, 16, device=dev).bfloat16()
w1 = torch.randn(16, 16, 3, 3, device=dev) * 0.1
w2 = torch.randn(32, 16, 3, 3, device=dev) * 0.1
only = os.environ.get("ONLY", "")
cases = [
    ("stem u8 7x7 3->16", 2.0 * B * H * W * 16 * 147,
     lambda: ops.stem_u8(frames, w0, one16, zero16, (0.3, 0.3, 0.3), (0.2, 0.2, 0.2))),
    ("stem+layer1 fused", 2.0 * B * H * W * 16 * (147 + 144),
     lambda: ops.stem_layer1_u8(frames, w0, one16, zero16, w1, one16, zero16, (0.3, 0.3, 0.3), (0.2, 0.2, 0.2))),
    ("layer1 3x3 16->16", 2.0 * B * H * W * 16 * 144,
     lambda: ops.conv2d_bn_act(x1, w1, None, None, None, 1, 1, 1, True, algo=_lib.ALGO_PATCH)),
    ("layer2 3x3 s2 16->32", 2.0 * B * H * W / 4 * 32 * 144,
     lambda: ops.conv2d_bn_act(x1, w2, None, None, None, 2, 1, 1, True, algo=_lib.ALGO_PATCH)),
]
for name, flops, fn in cases:
    if only and not name.startswith(only):
        continue
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 5 * 1e3)
    print(f"{name:24s} {best:8.1f} us {flops / best / 1e6:7.1f} TF", flush=True)
