"""conv_w1 bring-up: which K step (tap, 64-channel block) carries the tile-22 vs tile-19 mismatch."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import ops  # noqa: E402

DEV = "cuda"
n, h, w, cin, cout, dil = 1, 4, 256, 256, 256, 1
g = torch.Generator().manual_seed(7)
x = torch.randn(n, h, w, cin, generator=g).bfloat16().to(DEV)
wt = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(DEV)
sh = (torch.rand(cout, generator=g) - 0.5).to(DEV)
kw_ = dict(stride=1, padding=dil, dilation=dil, relu=False, fold_scale=True)
a = ops.conv2d_bn_act(x, wt, None, sh, None, tile=19, **kw_).float()
b = ops.conv2d_bn_act(x, wt, None, sh, None, tile=22, **kw_).float()
print("full:", int((a != b).sum()))
for cb in range(cin // 64):
    for tap in range(9):
        m = torch.zeros_like(wt)
        m[:, cb * 64:(cb + 1) * 64, tap // 3, tap % 3] = 1
        a = ops.conv2d_bn_act(x, wt * m, None, sh, None, tile=19, **kw_).float()
        b = ops.conv2d_bn_act(x, wt * m, None, sh, None, tile=22, **kw_).float()
        bad = (a != b)
        if bad.any():
            idx = bad.nonzero()
            print(f"cb {cb} tap {tap} (step {cb * 9 + tap}): {int(bad.sum())} mismatches, rows {torch.unique(idx[:, 1]).tolist()}, "
                  f"px/16 {torch.unique(idx[:, 2] // 16).tolist()}, ch/16 {torch.unique(idx[:, 3] // 16).tolist()}")
torch.cuda.synchronize()
print("done")
