#!/usr/bin/env python3
"""Fine-tune benchmark (BASELINE.json config C4): DRN-D-54 + RmbPruner 75 % (Ramanujan-block,
8x8 outer blocks, one 2x2 blocklet per blocklet row), Cityscapes-shaped 1024x768 crops,
data-parallel over ranks with the bucketed RCCL gradient all-reduce (drnmi.parallel).

A step is the reference training-loop body (semantic_seg.py:166-230): train-mode forward,
CrossEntropyLoss(ignore_index=255) on the log-probs, zero_grad, backward, SGD(lr 0.01,
momentum 0.9, wd 1e-4) with the pruner's masks applied in the same pass (:213-214).  fp32
throughout (the reference's arithmetic).  Synthetic normalised inputs and labels (10 % ignore)
resident in HBM; hash-initialised weights.

    python bench_finetune.py [--steps K] [--warmup W] [--batch B] [--gpus N]
    torchrun --nproc-per-node N bench_finetune.py --gpus N

`--gpus N` outside torchrun spawns the N rank processes itself (bench.py's launcher); under
torchrun a WORLD_SIZE different from --gpus is refused.  `--stub-step` (test hook, no GPU) runs
a CPU stand-in step over gloo through the same launcher, seeding and max-over-ranks timing.

Prints ONE JSON line (rank 0).  Not the driver's headline bench (bench.py is).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "video-seg-model-compress_amd"))
sys.path.insert(0, REPO)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2, help="crops per GPU per step")
    ap.add_argument("--arch", default="drn_d_54")
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=768)
    ap.add_argument("--no-prune", action="store_true")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp32x"],
                    help="fp32x: the convs (forward, data and weight gradients) on the fp32-accurate "
                         "split-bf16 kernels (conv_x6, X6 patch kernels, wgrad_f32x3); BN and the head stay exact fp32")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stub-step", action="store_true",
                    help="test hook: no GPU; gloo ranks run a CPU stand-in step (a gradient all-reduce of a "
                         "rank-seeded tensor) through the same launcher and timing code")
    return ap.parse_args(argv)


def rmb_pruner(model, on_gpu):
    """RmbPruner 75 % on every conv whose collapsed [Cout, Cin*k*k] matrix tiles into 8x8
    blocks (all but the 3-channel stem), as the shipped rmb configs do (RmbPruner.py:111-125)."""
    from drnmi.pruners import RmbPruner
    layers = [k for k, v in model.state_dict().items()
              if k.startswith("layer.") and k.endswith(".weight") and v.dim() == 4
              and v.shape[0] % 8 == 0 and v[0].numel() % 8 == 0]
    cfg = {"pruner_type": "rmb", "configs": [{"layer_set": layers, "global_bh": 8, "global_bw": 8,
                                              "global_sp": 0.0, "blocklets": [{"bh": 2, "bw": 2, "count": 1}]}]}
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(cfg, f)
        path = f.name
    pr = RmbPruner(path, on_gpu=on_gpu)
    pr.generate_masks(model.cpu() if not on_gpu else model)
    os.unlink(path)
    return pr


def train_flops(model, n, h, w):
    """Algorithmic FLOPs of one step: forward convs F, data-gradient F (except the stem's),
    weight-gradient F — 2*M*Cout*Cin*k*k each (the head's up/log-softmax is negligible)."""
    from drnmi.engine import _conv_out
    shapes = {"input": (h, w)}
    f = 0.0
    for nd in model._graph.nodes:
        c = nd.conv
        ih, iw = shapes[nd.src]
        oh = _conv_out(ih, c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0])
        ow = _conv_out(iw, c.kernel_size[1], c.stride[1], c.padding[1], c.dilation[1])
        shapes[nd.dst] = (oh, ow)
        fl = 2.0 * n * oh * ow * c.out_channels * c.in_channels * c.kernel_size[0] * c.kernel_size[1]
        f += fl * (2 if nd.src == "input" else 3)
    return f


def step_t_star(model, n, h, w, precision):
    """Roofline time of one step's convs at their kernels' MFMA peaks: in fp32x, forward, dgrad
    and wgrad at the split-bf16 rate (2.5 PF / 6) where the HIP path runs them split (conv_x6 and
    every drnmi_conv_wgrad_f32x3, the X6 patch kernels for the stem / layer1 / layer2 forward and
    the layer1 data gradient), else the f32 MFMA (157 TF)."""
    from drnmi.engine import X6_PATCH_SHAPES, _conv_out, _pow2_at_least
    from drnmi.roofline import MFMA_PEAK  # noqa: F401
    shapes = {"input": (h, w)}
    t = 0.0
    f32, x6 = MFMA_PEAK["fp32"], MFMA_PEAK["fp32x"]
    for nd in model._graph.nodes:
        c = nd.conv
        ih, iw = shapes[nd.src]
        oh = _conv_out(ih, c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0])
        ow = _conv_out(iw, c.kernel_size[1], c.stride[1], c.padding[1], c.dilation[1])
        shapes[nd.dst] = (oh, ow)
        fl = 2.0 * n * oh * ow * c.out_channels * c.in_channels * c.kernel_size[0] * c.kernel_size[1]
        cs = 8 if nd.src == "input" else _pow2_at_least(c.in_channels)
        patch = (cs, c.out_channels, c.kernel_size[0], c.stride[0], c.dilation[0]) in X6_PATCH_SHAPES
        fx = precision == "fp32x"
        t += fl / (x6 if fx and (c.in_channels >= 32 or patch) else f32)                 # forward
        if nd.src != "input":
            dpatch = (_pow2_at_least(c.out_channels), c.in_channels, c.kernel_size[0], 1,
                      c.dilation[0]) in X6_PATCH_SHAPES
            t += fl / (x6 if fx and (c.out_channels >= 32 or dpatch) else f32)            # dgrad
        t += fl / (x6 if fx else f32)                                                     # wgrad
    return t


def cpu_baseline(args, seconds):
    """The oracle's fine-tune step (torch-CPU fp32 autograd + torch.optim.SGD) on a bounded
    sample: batch 1 at half the crop size in each dimension, value scaled by the pixel ratio."""
    import torch
    from drnmi.drnseg import DRNSeg
    from drnmi.weights import synth_state_dict
    from oracle import drn_oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    h, w = args.height // 2, args.width // 2
    m = DRNSeg(args.arch, 19, pretrained=False)
    sd = synth_state_dict(m, 0)
    x = torch.randn(1, 3, h, w)
    t = torch.randint(0, 19, (1, h, w))
    n, t0 = 0, time.perf_counter()
    while True:
        O.drnseg_train_steps(sd, args.arch, [x], [t], 0.01, 0.9, 1e-4)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 8:
            break
    ratio = (h * w) / (args.height * args.width)
    return {"value": n / el * ratio, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} oracle fine-tune step(s) (torch-CPU fp32 autograd + torch.optim.SGD) of batch 1 "
                      f"at {h}x{w}, scaled x{ratio:.2f} to {args.height}x{args.width} images/s ({threads} threads)"}


def stub_main(args, world, rank):
    """CPU stand-in of the fine-tune step (no GPU): each rank sums a rank-seeded "gradient" over
    gloo (the DDP all-reduce's role), timed like the real step: barrier, max over ranks."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    g = torch.Generator().manual_seed(2000 + rank)
    grad = torch.randn(4096, generator=g)

    def step():
        buf = grad.clone()
        if world > 1:
            dist.all_reduce(buf)
        return buf

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        red = step()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    out = {"metric": "fine-tune images/s (stub)", "value": world * args.batch * args.steps / el, "unit": "images/s",
           "n_gpus": world, "steps": args.steps, "ms_per_step": el / args.steps * 1e3, "scaling": "weak",
           "reduced_sum": float(red.sum()), "rank_seed": 2000 + rank}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    args = parse(argv)
    import bench
    wr = bench.resolve_world(args, prog="bench_finetune.py")
    if wr is None:                            # --gpus N outside torchrun: spawn the ranks
        sys.exit(bench.spawn_ranks(args.gpus, sys.argv[1:] if argv is None else argv, os.path.abspath(__file__)))
    world, rank, local = wr
    if args.stub_step:
        return stub_main(args, world, rank)
    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from drnmi.dist import max_over_ranks
    from drnmi.drnseg import DRNSeg
    from drnmi.parallel import DistributedDataParallel
    from drnmi.roofline import MFMA_PEAK  # noqa: F401
    from drnmi.train import SGD, CrossEntropyLoss
    from drnmi.weights import synth_state_dict

    m = DRNSeg(args.arch, 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, 0))
    pr = None if args.no_prune else rmb_pruner(m, on_gpu=False)
    m = m.to(dev).train().set_precision(args.precision)
    if pr is not None:
        for k in list(pr.mask_dict):
            pr.mask_dict[k] = pr.mask_dict[k].to(dev)
        pr.on_gpu = True
        pr.apply_masks(m)                          # semantic_seg.py:1063 (before training)
    net = DistributedDataParallel(m, device_ids=[local]) if world > 1 else m
    opt = SGD(m.optim_parameters(), 0.01, momentum=0.9, weight_decay=1e-4, pruner=pr, model=m if pr else None)
    crit = CrossEntropyLoss(ignore_index=255)
    B, H, W = args.batch, args.height, args.width
    g = torch.Generator(device=dev).manual_seed(2000 + rank)
    x = torch.randn(B, 3, H, W, device=dev, generator=g)
    t = torch.randint(0, 19, (B, H, W), device=dev, generator=g)
    t[torch.rand(B, H, W, device=dev, generator=g) < 0.1] = 255

    def step():
        out = net(x)[0]
        loss = crit(out, t)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, device=dev)
    fl = train_flops(m, B, H, W)
    ach = fl * args.steps / el / 1e12
    peak = MFMA_PEAK["fp32"] / 1e12
    t_star = step_t_star(m, B, H, W, args.precision)
    masked = sum(v.numel() for v in pr.mask_dict.values()) if pr else 0
    dens = (sum(int((v != 0).sum()) for v in pr.mask_dict.values()) / masked) if pr else 1.0
    out = {
        "metric": f"fine-tune images/s ({args.arch} + RmbPruner 75%, {H}x{W} crops, DP over RCCL)",
        "value": world * B * args.steps / el,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic normalised inputs + random labels (10% ignore_index), hash-initialised weights",
        "config": {"workload": f"{args.arch} fine-tune step (fwd + CE + bwd + SGD with fused RMB 75% mask), "
                               f"{B} crops/GPU of {H}x{W}", "arch": args.arch, "height": H, "width": W,
                   "crops_per_gpu_step": B, "global_batch": B * world, "mask_density": round(dens, 4),
                   "parallelism": f"dp{world} (bucketed SUM all-reduce overlapped with backward)"},
        "roofline": {"bound": "mfma", "kernel": "whole step (fwd + dgrad + wgrad convs, fp32 MFMA)"
                                                  if args.precision == "fp32" else
                                                  "whole step (fwd and dgrad convs split-bf16 where cin >= 32 or on "
                                                  "the X6 patch kernels, every wgrad split-bf16)",
                     "achieved": round(ach, 2), "peak": peak if args.precision == "fp32" else round(fl / t_star / 1e12, 2),
                     "unit": "TFLOP/s", "frac": round(t_star / (el / args.steps), 4),
                     "traffic": None, "step_tflop": round(fl / 1e12, 3),
                     "peak_note": "conv time at each conv's kernel peak (step_t_star): frac = T* / T"},
        "final_loss": float(loss.detach()),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
