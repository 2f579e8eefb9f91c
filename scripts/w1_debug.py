"""conv_w1 (tile 22) vs conv_stag (tile 19) mismatch map on one shape (bring-up diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import ops  # noqa: E402

DEV = "cuda"
for (n, h, w, cin, cout, dil, with_res) in [(2, 9, 256, 256, 256, 2, True), (1, 4, 256, 512, 512, 1, False),
                                            (1, 4, 256, 256, 256, 1, False), (1, 1, 256, 128, 256, 1, False)]:
    g = torch.Generator().manual_seed(390 + h * w + cin)
    x = torch.randn(n, h, w, cin, generator=g).bfloat16().to(DEV)
    wt = (torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cout)) ** 0.5).to(DEV)
    sc = (torch.rand(cout, generator=g) + 0.5).to(DEV)
    sh = (torch.rand(cout, generator=g) - 0.5).to(DEV)
    res = torch.randn(n, h, w, cout, generator=g).bfloat16().to(DEV) if with_res else None
    kw = dict(stride=1, padding=dil, dilation=dil, relu=True, fold_scale=True)
    a = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=19, **kw).float()
    b = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=22, **kw).float()
    b2 = ops.conv2d_bn_act(x, wt, sc, sh, res, tile=22, **kw).float()
    torch.cuda.synchronize()
    d = (a - b).abs()
    bad = d > 0
    print(f"shape n{n} h{h} w{w} cin{cin} cout{cout} dil{dil} res{with_res}: mismatches {int(bad.sum())} of {bad.numel()}, "
          f"max {float(d.max()):.4g}, rerun-identical {bool(torch.equal(b, b2))}")
    if bad.any():
        idx = bad.nonzero()
        px = idx[:, 0] * h * w + idx[:, 1] * w + idx[:, 2]
        tiles = torch.unique(px // 256)
        ch = torch.unique(idx[:, 3])
        print("  tiles:", tiles.tolist()[:20], " pixel%256 range:", int((px % 256).min()), int((px % 256).max()))
        print("  channels:", len(ch), ch.tolist()[:40])
        print("  pixel-in-tile histogram (/16):", torch.bincount((px % 256) // 16, minlength=16).tolist())
        print("  channel histogram (/16):", torch.bincount(idx[:, 3] // 16, minlength=cout // 16).tolist())
