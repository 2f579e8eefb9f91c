"""Labels-only head on the D-22 batch-8 logits shape (8 x 128 x 256 x 20 fp32 NHWC rows -> 8 x 1024 x
2048 uint8 labels): per-launch time of the NHWC head (up8_labels_tile_kernel) and of the NCHW oct
head on the same logits, the share of 2 x 2 tap windows the fast path takes, and a label checksum.
LOGITS=random (i.i.d. normal logits: no uniform windows) or network (the bf16 D-22 seg logits of 8
random frames, as bench.py's).  python scripts/head_micro.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import _lib, drnseg, engine  # noqa: E402
from drnmi.weights import bilinear_up_kernel  # noqa: E402

n, h, w, cs = 8, 128, 256, 20
mode = os.environ.get("LOGITS", "network")
if mode == "random":
    g = torch.Generator(device="cuda").manual_seed(1)
    logits = torch.randn(n, h, w, cs, device="cuda", generator=g) * 3
else:
    m = drnseg.build("drn_d_22", 19, seed=0, device=torch.device("cuda"), precision="bf16")
    g = torch.Generator(device="cuda").manual_seed(1000)
    frames = torch.randint(0, 256, (n, 8 * h, 8 * w, 3), dtype=torch.uint8, device="cuda", generator=g)
    m.segment(frames)                                   # seg folded into layer8: partial planes
    plan = next(iter(m._plans.values()))
    part = plan.bufs["seg_part"].clone()
    bias = plan.packed.graph.nodes[plan.seg_idx].shift
    engine.SEG_FUSE = False
    plan.refresh_weight_ptrs()
    m.segment(frames)
    logits = plan.bufs["logits_nhwc"].view(n, h, w, cs).clone()
nchw = logits[..., :19].permute(0, 3, 1, 2).contiguous()
up = torch.from_numpy(bilinear_up_kernel(16)).float().cuda()
lab = torch.empty(n, 8 * h, 8 * w, dtype=torch.uint8, device="cuda")
lab2 = torch.empty_like(lab)
lib = _lib.load()
st = ctypes.c_void_p(_lib.stream_ptr())

# share of interior 2 x 2 windows whose taps share the argmax with a margin above the guard
L = logits[..., :19]
top2 = torch.topk(L, 2, dim=-1)
am, marg, best = top2.indices[..., 0], top2.values[..., 0] - top2.values[..., 1], top2.values[..., 0].abs()
same = (am[:, :-1, :-1] == am[:, 1:, :-1]) & (am[:, :-1, :-1] == am[:, :-1, 1:]) & (am[:, :-1, :-1] == am[:, 1:, 1:])
mm = torch.minimum(torch.minimum(marg[:, :-1, :-1], marg[:, 1:, :-1]), torch.minimum(marg[:, :-1, 1:], marg[:, 1:, 1:]))
bm = torch.maximum(torch.maximum(best[:, :-1, :-1], best[:, 1:, :-1]), torch.maximum(best[:, :-1, 1:], best[:, 1:, 1:]))
fast = same & (mm >= 2 ** -16 * (1 + 2 ** -10) + 2 ** -20 * bm)
print(f"logits {mode}: fast-path windows {float(fast.float().mean()):.3f}", flush=True)


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


t_fast = timed(lambda: _lib.check(lib.drnmi_up8_labels_nhwc(logits.data_ptr(), cs, up.data_ptr(), lab.data_ptr(),
                                                             _lib.DRNMI_U8, n, 19, h, w, st), "head"))
t_oct = timed(lambda: _lib.check(lib.drnmi_up8_logsoftmax_argmax(nchw.data_ptr(), up.data_ptr(), None, lab2.data_ptr(),
                                                                  _lib.DRNMI_U8, n, 19, h, w, st), "oct head"))
print(f"nhwc fast-path head {t_fast:7.1f} us   nchw oct head {t_oct:7.1f} us   labels equal {torch.equal(lab, lab2)}   "
      f"label sum {int(lab.sum(dtype=torch.int64))}", flush=True)
if mode != "random":
    t_seg2 = timed(lambda: _lib.check(lib.drnmi_up8_labels_seg2(part.data_ptr(), cs, bias.data_ptr(), up.data_ptr(),
                                                                 lab.data_ptr(), _lib.DRNMI_U8, n, 19, h, w, st), "seg2"))
    print(f"seg2 (two partial planes + bias) fast-path head {t_seg2:7.1f} us", flush=True)
