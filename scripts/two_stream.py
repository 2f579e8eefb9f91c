"""Diagnostic: D-22 bf16 seg_video throughput with the batch split over concurrent HIP streams.
(a) one plan of B frames on one stream (what bench.py times); (b) S plans of B/S frames, each on
its own stream, launched back to back so the GPU may overlap one half's kernels with the other's.
python scripts/two_stream.py [B] [S]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import drnseg  # noqa: E402
from drnmi.drnseg import INFO_MEAN, INFO_STD  # noqa: E402
from drnmi.engine import Plan  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
S = int(sys.argv[2]) if len(sys.argv) > 2 else 2
H, W = 1024, 2048
dev = torch.device("cuda")
m = drnseg.build("drn_d_22", 19, seed=0, device=dev, precision="bf16").eval()
g = torch.Generator(device=dev).manual_seed(5)
frames = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
ref = m.segment(frames, INFO_MEAN, INFO_STD, False)
pk = m._packed["bf16"]
sub = B // S
plans = [Plan(pk, sub, H, W) for _ in range(S)]
streams = [torch.cuda.Stream() for _ in range(S)]
up = m._up_plane(dev)
outs = [torch.empty(sub, *plans[0].out_hw, dtype=torch.uint8, device=dev) for _ in range(S)]


def split_step():
    cur = torch.cuda.current_stream()
    for k in range(S):
        streams[k].wait_stream(cur)
    for k in range(S):
        s = streams[k].cuda_stream
        plans[k].ingest_u8(frames[k * sub:(k + 1) * sub], INFO_MEAN, INFO_STD, False, s)
        plans[k].run_backbone(s)
        plans[k].head(up, s, None, outs[k])
    for k in range(S):
        cur.wait_stream(streams[k])


def one_step():
    m.segment(frames, INFO_MEAN, INFO_STD, False)


split_step()
torch.cuda.synchronize()
got = torch.cat(outs)
print("split labels identical:", bool((got == ref).all()), flush=True)


def timeit(fn, steps=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


for rep in range(3):
    t1 = timeit(one_step)
    t2 = timeit(split_step)
    print(f"rep {rep}: one stream {B / t1:8.1f} fps ({t1 * 1e3:.3f} ms)   {S} streams x {sub} "
          f"{B / t2:8.1f} fps ({t2 * 1e3:.3f} ms)", flush=True)
