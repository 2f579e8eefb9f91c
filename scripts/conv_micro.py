"""Micro-benchmark of the conv kernels on DRN-D-22 layer shapes (bf16), one process,
interleaved variants (cdna_hip_programming.md rule 24).  python scripts/conv_micro.py [batch]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
TILES = [int(t) for t in os.environ.get("TILES", "4,5,6,16,17").split(",")]
SHAPES = [  # name, cin, cout, ks, stride, dil, H(in), W(in), residual
    ("l8 512x512 d1", 512, 512, 3, 1, 1, 128, 256, False),
    ("l7 512x512 d2", 512, 512, 3, 1, 2, 128, 256, False),
    ("l6 512x512 d4 +res", 512, 512, 3, 1, 4, 128, 256, True),
    ("l6 512x512 d4 nores", 512, 512, 3, 1, 4, 128, 256, False),
    ("l6.0c1 256->512 d4", 256, 512, 3, 1, 4, 128, 256, False),
    ("l5 256x256 d2 +res", 256, 256, 3, 1, 2, 128, 256, True),
    ("l4 128x128 +res", 128, 128, 3, 1, 1, 128, 256, True),
    ("l4.0c1 64->128 s2", 64, 128, 3, 2, 1, 256, 512, False),
    ("l6 ds 256->512 1x1", 256, 512, 1, 1, 1, 128, 256, False),
    ("l3 64x64 +res", 64, 64, 3, 1, 1, 256, 512, True),
    ("l3.0c1 32->64 s2", 32, 64, 3, 2, 1, 512, 1024, False),
    ("l3.0ds 32->64 1x1 s2", 32, 64, 1, 2, 1, 512, 1024, False),
    ("l4.0ds 64->128 1x1 s2", 64, 128, 1, 2, 1, 256, 512, False),
    ("seg 512->19 1x1", 512, 19, 1, 1, 1, 128, 256, False),
]
dev = "cuda"
ONLY = os.environ.get("ONLY")
# scale folded into the weights (scale = NULL: the accumulators start from shift + residual), as the
# engine launches the bf16 convs; FOLD=0 times the unfolded epilogue
FOLD = os.environ.get("FOLD", "1") != "0"
for name, cin, cout, ks, st, dil, h, w, has_res in SHAPES:
    if ONLY and not name.startswith(ONLY):
        continue
    pad = dil * (ks // 2)
    x = torch.randn(B, h, w, cin, device=dev).bfloat16()
    wt = torch.randn(cout, cin, ks, ks, device=dev) * 0.05
    ho = (h + 2 * pad - dil * (ks - 1) - 1) // st + 1
    wo = (w + 2 * pad - dil * (ks - 1) - 1) // st + 1
    res = torch.randn(B, ho, wo, cout, device=dev).bfloat16() if has_res else None
    packed = ops.pack_conv_weight(wt, cin, torch.bfloat16)
    flops = 2.0 * B * ho * wo * cout * cin * ks * ks
    line = f"{name:22s}"
    times = {}
    if ONLY == "l3" and cin == 32:
        pass
    for rep in range(3):
        for t in TILES:
            try:
                for _ in range(2):
                    ops.conv2d_bn_act(x, wt, None, None, res, st, pad, dil, True, tile=t, packed=packed, fold_scale=FOLD)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    ops.conv2d_bn_act(x, wt, None, None, res, st, pad, dil, True, tile=t, packed=packed, fold_scale=FOLD)
                e1.record()
                torch.cuda.synchronize()
                times.setdefault(t, []).append(e0.elapsed_time(e1) / 5 * 1e3)
            except RuntimeError:
                times[t] = None
    for t in TILES:
        if times.get(t):
            us = min(times[t])
            line += f" | t{t}: {us:8.1f}us {flops / us / 1e6:7.1f}TF"
        else:
            line += f" | t{t}: n/a"
    print(line, flush=True)
