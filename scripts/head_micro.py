"""Labels-only head (drnmi_up8_labels_nhwc) on the D-22 batch-8 logits shape (8 x 128 x 256 x 20 fp32
rows -> 8 x 1024 x 2048 uint8 labels): per-launch time and a label checksum.  python scripts/head_micro.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import _lib  # noqa: E402
from drnmi.weights import bilinear_up_kernel  # noqa: E402

n, h, w, cs = 8, 128, 256, 20
g = torch.Generator(device="cuda").manual_seed(1)
logits = torch.randn(n, h, w, cs, device="cuda", generator=g) * 3
up = torch.from_numpy(bilinear_up_kernel(16)).float().cuda()
lab = torch.empty(n, 8 * h, 8 * w, dtype=torch.uint8, device="cuda")
lib = _lib.load()
st = ctypes.c_void_p(_lib.stream_ptr())


def run():
    _lib.check(lib.drnmi_up8_labels_nhwc(logits.data_ptr(), cs, up.data_ptr(), lab.data_ptr(), _lib.DRNMI_U8, n, 19,
                                         h, w, st), "head")


for _ in range(3):
    run()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    run()
e1.record()
torch.cuda.synchronize()
print(f"head {e0.elapsed_time(e1) / 20 * 1e3:7.1f} us   label sum {int(lab.sum(dtype=torch.int64))}", flush=True)
