"""Diagnostic: time the halo-family kernels on the DRN-D-22 layer3/layer4 3x3 shapes (bf16,
8 frames of 1024x2048 input, BN scale folded = the engine's launch), by forced tile id:
17 = conv_halo_kernel (tile 18, the rolling-window experiment, is in git history:
commit dc4061a).  python scripts/halo_micro.py [tiles...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import ops  # noqa: E402

TILES = [int(t) for t in sys.argv[1:]] or [17]
B = int(os.environ.get("B", "8"))
SHAPES = [("l3 64x64 +res", 64, 64, 256, 512), ("l4 128x128 +res", 128, 128, 128, 256)]
for name, cin, cout, h, w in SHAPES:
    x = torch.randn(B, h, w, cin, device="cuda").bfloat16()
    wt = torch.randn(cout, cin, 3, 3, device="cuda") * 0.05
    sh = torch.randn(cout, device="cuda") * 0.1
    res = torch.randn(B, h, w, cout, device="cuda").bfloat16() if os.environ.get("RES", "1") == "1" else None
    packed = ops.pack_conv_weight(wt, cin, torch.bfloat16)
    flops = 2.0 * B * h * w * cout * cin * 9
    line = f"{name:18s}"
    for t in TILES:
        kw = dict(stride=1, padding=1, dilation=1, relu=True, tile=t, packed=packed, fold_scale=True)
        try:
            for _ in range(2):
                ops.conv2d_bn_act(x, wt, None, sh, res, **kw)
            best = 1e9
            for rep in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    ops.conv2d_bn_act(x, wt, None, sh, res, **kw)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
            line += f" | t{t}: {best:7.1f}us {flops / best / 1e6:6.1f}TF"
        except RuntimeError:
            line += f" | t{t}: n/a"
    print(line, flush=True)
