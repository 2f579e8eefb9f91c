"""Fused 64-channel BasicBlock (drnmi_basic_block64) vs the two halo launches it replaces, on the
D-22 layer3.1 shape (8 frames, 256 x 512 x 64 bf16).  python scripts/block64_micro.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-seg-model-compress_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from drnmi import _lib, ops  # noqa: E402
import test_block64 as T  # noqa: E402

N, H, W = int(os.environ.get("N", 8)), 256, 512
lib = _lib.load()
p = T._params(1)
blob = torch.from_numpy(T._pack(lib, p)).cuda()
x = torch.relu(torch.randn(N, H, W, 64, device="cuda")).bfloat16()
y = torch.empty_like(x)
w1, s1, b1, w2, s2, b2 = [t.cuda() for t in p]
st = ctypes.c_void_p(_lib.stream_ptr())


def fused():
    _lib.check(lib.drnmi_basic_block64(x.data_ptr(), blob.data_ptr(), y.data_ptr(), N, H, W, st), "block64")


pk1 = ops.pack_conv_weight(w1, 64, torch.bfloat16)
pk2 = ops.pack_conv_weight(w2, 64, torch.bfloat16)


def halo():   # as the engine launches them: packed weights, scale folded (timing only)
    t = ops.conv2d_bn_act(x, w1, None, None, None, 1, 1, 1, True, tile=17, packed=pk1, fold_scale=True)
    ops.conv2d_bn_act(t, w2, None, None, x, 1, 1, 1, True, tile=17, packed=pk2, fold_scale=True)


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


flops = 2 * 2.0 * N * H * W * 64 * 576
for rep in range(3):
    tf, th = timeit(fused), timeit(halo)
    print(f"layer3.1 {N}x{H}x{W}: fused {tf:7.1f} us ({flops / tf / 1e6:6.1f} TF, {flops / tf / 1e6 / 2500:.3f} of 2.5 PF)"
          f"   two halo launches {th:7.1f} us", flush=True)
ref = T.reference(x.cpu()[:1], p)
fused()
torch.cuda.synchronize()
d = (y[:1].float().cpu() - ref).abs().max()
print(f"frame 0 max |fused - fp32 ref| = {d:.3e}")
