#!/usr/bin/env python3
"""Headline benchmark: DRN-D-22 segmentation of 1024x2048 frames on MI355X (BASELINE.json).

A step = one pass of the seg_video hot loop (reference seg_video_old_no_plot.py:157-169:
normalise -> model(img)[0] -> torch.max(final, 1)) over a batch of synthetic uint8 RGB
frames already resident in HBM: frame ingest -> 22 fused conv launches -> seg -> up x8 +
log-softmax + argmax, producing uint8 label maps.  Frames shard across ranks (one process
per GPU, weak scaling, no collective on the data path; the only collectives are the
timing barrier and the max-over-ranks of the elapsed time).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "video-seg-model-compress_amd"))
sys.path.insert(0, REPO)

METRIC = "frames/sec @1024x2048 DRN-D-22 on 1/2/4/8 MI355X; mIoU vs ref; %HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="frames per GPU per step")
    ap.add_argument("--arch", default="drn_d_22")
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=2048)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "fp32x", "int8"],
                    help="int8: W8A8 for the cin >= 64 convs (config C5), scales calibrated on 2 "
                         "synthetic frames before the timed region")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-events", action="store_true")
    ap.add_argument("--prune", default="", help="block:BHxBW:SPARSITY — BlockPruner masks (collapse_tensor "
                    "False, BlockPruner.py:139-241) on every conv with >=16 input channels (config C3); "
                    "json:PATH — any pruner config (pruner_type dispatch, e.g. the srmbrep D-22 configs "
                    "of config C5)")
    ap.add_argument("--block-sparse", action="store_true", help="unit-skipping MFMA kernels on pruned weights "
                    "(opt-in; the dense kernel is faster below ~60%% zero 16x32 units)")
    ap.add_argument("--host-frames", action="store_true",
                    help="also time the PCIe-inclusive pipeline: frames in pinned host memory, H2D on a copy "
                         "stream overlapped with the previous batch's compute (reported as 'host_frames'; "
                         "the headline value stays HBM-resident)")
    return ap.parse_args()


def pruned_model(args, dev):
    """BASELINE config C3: hash-initialised weights + BlockPruner masks, applied once
    (semantic_seg.py:1063), then the eval engine (which skips the all-zero weight units)."""
    import json
    import tempfile

    import torch
    from drnmi.drnseg import DRNSeg
    from drnmi.pruners import BlockPruner
    from drnmi.weights import synth_state_dict
    m = DRNSeg(args.arch, 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, 0))
    if args.prune.startswith("json:"):
        from drnmi.pruners import make_pruner
        pr = make_pruner(args.prune[len("json:"):], on_gpu=False)
        pr.generate_masks(m, is_static=False)
        layers = list(pr.mask_dict)
    else:
        kind, shape, sp = args.prune.split(":")
        if kind != "block":
            raise SystemExit("--prune: block:BHxBW:SPARSITY or json:PATH")
        bh, bw = (int(v) for v in shape.lower().split("x"))
        layers = [k for k, v in m.state_dict().items() if k.startswith("layer.") and k.endswith(".weight")
                  and v.dim() == 4 and v.shape[1] >= 16 and v.shape[0] % bh == 0 and v.shape[1] % bw == 0]
        cfg = {"pruner_type": "block", "configs": [{"layer_set": layers, "sparsity": float(sp), "block_height": bh,
                                                    "block_width": bw, "sub_rows": -1, "sub_cols": -1,
                                                    "collapse_tensor": False}]}
        with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
            json.dump(cfg, f)
        pr = BlockPruner(f.name, on_gpu=False)
        pr.generate_masks(m, is_static=False)
        os.unlink(f.name)
    with torch.no_grad():
        sd = m.state_dict()
        for k, mk in pr.mask_dict.items():
            sd[k].mul_(mk)
    m = m.to(dev).eval().set_precision("bf16" if args.precision == "int8" else args.precision)
    m.set_block_sparse(args.block_sparse)
    return m, len(layers)


def calibrate(model, args, dev):
    """int8: activation scales from 2 synthetic frames (a different stream than the timed
    frames), then switch the engine to W8A8 (DRNSeg.calibrate_int8)."""
    import torch
    g = torch.Generator(device=dev).manual_seed(77)
    calib = torch.randint(0, 256, (2, args.height, args.width, 3), dtype=torch.uint8, device=dev, generator=g)
    model.calibrate_int8(calib)
    model.set_precision("int8")
    return model


def host_cores() -> int:
    """Every host core this process may run on: the affinity mask (os.sched_getaffinity), capped
    by a cgroup CPU quota when one is set (threads beyond the quota only time-slice)."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            cores = min(cores, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return cores


def cpu_baseline(args, seconds):
    """Reference seg_video CPU loop restated by the oracle (fp32 NCHW torch CPU, batch 1)."""
    import numpy as np
    import torch

    from drnmi.drnseg import DRNSeg
    from drnmi.weights import synth_frames, synth_state_dict
    from oracle import drn_oracle as O

    threads = host_cores()
    torch.set_num_threads(threads)
    m = DRNSeg(args.arch, 19, pretrained=False)
    sd = synth_state_dict(m, 0)
    frames = synth_frames(7, 2, args.height, args.width)

    labels = {}

    def one(i):
        x = O.preprocess_u8(frames[i % 2:i % 2 + 1])
        lp, _, _ = O.drnseg_forward(sd, args.arch, x)
        labels[i % 2] = torch.max(lp, 1)[1][0].cpu().numpy()
        return labels[i % 2]

    one(0)                                   # warm-up frame (untimed)
    n, t0 = 0, time.perf_counter()
    while True:
        one(n)
        n += 1
        el = time.perf_counter() - t0
        if (el >= seconds and n >= 2) or n >= 64:
            break
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": n / el, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} frames of {args.height}x{args.width} after 1 warm-up frame, batch 1, "
                      f"oracle/drn_oracle.py fp32 NCHW torch-CPU ({threads} threads = all affine host cores "
                      f"within the cgroup quota, {cpu_model})"}, (frames, labels)


def parity_vs_ref(args, model, frames, ref_labels, dev):
    """The measured path's labels on the CPU baseline's frames vs the oracle's (the reference
    restated, pinned to its goldens): pixel agreement and mIoU with the reference labels as
    ground truth (BASELINE.json metric "mIoU vs ref"; semantic_seg.py:293-300 fast_hist)."""
    import numpy as np
    import torch

    from drnmi import metrics
    from drnmi.drnseg import INFO_MEAN, INFO_STD
    got = model.segment(torch.from_numpy(frames).to(dev), INFO_MEAN, INFO_STD, False).long()
    ref = torch.from_numpy(np.stack([ref_labels[i] for i in range(len(frames))])).long().to(dev)
    hist = metrics.fast_hist(got.flatten(), ref.flatten(), 19)
    return {"frames": len(frames), "precision": args.precision,
            "label_agreement": float((got == ref).float().mean()),
            "label_mismatches": int((got != ref).sum()),
            "miou_vs_ref": float(metrics.miou(hist.cpu().numpy())),
            "reference": "oracle/drn_oracle.py fp32 torch-CPU forward, same weights and frames"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from drnmi import _lib
    from drnmi.dist import max_over_ranks
    from drnmi.drnseg import INFO_MEAN, INFO_STD, build
    from drnmi.roofline import kernel_peak, network_roofline, node_work

    if args.prune:
        model, n_pruned = pruned_model(args, dev)
    else:
        model = build(args.arch, 19, seed=0, device=dev,
                      precision="bf16" if args.precision == "int8" else args.precision)
    if args.precision == "int8":
        model = calibrate(model, args, dev)
    B, H, W = args.batch, args.height, args.width
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    frames = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    plan = model.plan(B, H, W, device=dev)     # the plan model.segment() runs (same key)
    works = node_work(plan)
    lib = _lib.load()
    import ctypes

    fused_stem = getattr(plan, "stem_fused", False)

    def launched_name(i):
        if fused_stem and i <= 1:            # stem + layer1 in one launch (drnmi_stem_layer1)
            return "" if i == 1 else lib.drnmi_stem_layer1_kernel_name(
                ctypes.byref(plan.stem_u8), ctypes.byref(plan.args[1])).decode()
        a = plan.stem_u8 if (i == 0 and plan.stem_u8 is not None) else plan.args[i]
        if a is None:
            return ""                        # downsample folded into its block's last conv
        return lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode()

    names = [launched_name(i) for i in range(len(plan.args))]
    # useful work of a pruned layer: dense FLOPs x the density of its weights, on
    # dense and sparse kernels alike (the dense kernel multiplies the zeros too)
    nodes = plan.packed.graph.nodes
    density = [float((nd.conv.weight != 0).sum()) / nd.conv.weight.numel() for nd in nodes]
    # a folded-away downsample's FLOPs run inside its block's last conv: attribute them there
    # (its input read too; the residual is never written or read)
    works = list(works)
    for i in sorted(getattr(plan, "skip", ())):
        j = nodes[i].fused_into
        n_, fj, bj = works[j]
        fi, bi = works[i][1], works[i][2]
        oh, ow = plan.shapes[nodes[j].dst]
        res_b = plan.n * oh * ow * nodes[j].conv.out_channels * 2      # the bf16 residual tensor
        # conv2 bytes lose the residual read; the downsample's input + weights (not its output) join
        works[j] = (n_, fj + fi, bj - res_b + (bi - res_b))
        works[i] = (works[i][0], 0.0, 0.0)
    if fused_stem:
        # layer1 runs inside the stem launch; the 16-channel stem output is neither written
        # nor read back
        h0, w0 = plan.shapes[nodes[0].dst]
        mid = plan.n * h0 * w0 * nodes[0].conv.out_channels * 2
        works[0] = (works[0][0], works[0][1] + works[1][1], works[0][2] + works[1][2] - 2 * mid)
        works[1] = (works[1][0], 0.0, 0.0)
        density[0] = density[1] = float(sum((nd.conv.weight != 0).sum() for nd in nodes[:2])) / \
            sum(nd.conv.weight.numel() for nd in nodes[:2])
    dense_flops = {i: w[1] for i, w in enumerate(works)}
    works = [(w[0], w[1] * density[i], w[2]) if i < len(nodes) else w for i, w in enumerate(works)]
    events = []
    pool = [torch.cuda.Event(enable_timing=True) for _ in range(2 * len(names) * max(args.steps, 2))]
    watch = [None]        # None: every launch; else only launches of this kernel name

    def hook(i, nd, before):
        if watch[0] is not None and names[i] != watch[0]:
            return
        ev = pool[len(events)]
        ev.record()
        events.append((i, before, ev))

    def step(timed, x=frames):
        # the public API a seg_video user calls: DRNSeg.segment -> torch.ops.drnmi.segment
        model.timing_hook = hook if (timed and not args.no_kernel_events) else None
        return model.segment(x, INFO_MEAN, INFO_STD, False)

    def collect():
        """per-kernel durations of the recorded launches (the events list is then reset)"""
        torch.cuda.synchronize()
        per_, pend = {}, {}
        for i, before, ev in events:
            if before:
                pend[i] = ev
            else:
                g_ = per_.setdefault(names[i], {"d": [], "f": [], "b": [], "fd": []})
                g_["d"].append(pend.pop(i).elapsed_time(ev) * 1e-3)
                g_["f"].append(works[i][1])
                g_["fd"].append(dense_flops[i])
                g_["b"].append(works[i][2])
        events.clear()
        return per_

    for _ in range(max(args.warmup - 1, 0)):
        step(False)
    # last warm-up step instrumented: it names the dominant kernel (the template instance, as
    # rocprofv3 names it, with the largest total time); inside the timed region only that
    # kernel's launches carry HIP events (events around all ~25 launches cost ~2.7 % per step)
    step(True)
    warm = collect()
    dominant = max(warm, key=lambda k: sum(warm[k]["d"])) if warm else None
    watch[0] = dominant
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, device=dev)   # the slowest rank defines the job
    timed_per = collect()
    # per-kernel table: one fully instrumented step after the timed region
    watch[0] = None
    step(True)
    per = collect()
    if dominant in timed_per:
        per[dominant] = timed_per[dominant]
    model.timing_hook = None
    host = host_frames_run(args, model, step, world, dev) if args.host_frames else None

    durs = timed_per[dominant]["d"] if dominant in timed_per else []
    flops = timed_per[dominant]["f"] if dominant in timed_per else []
    nr = network_roofline(plan)
    total_frames = world * B * args.steps
    out = {
        "metric": METRIC,
        "value": total_frames / el,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": f"synthetic uint8 RGB frames resident in HBM; hash-initialised {args.arch} weights (no checkpoint)"
                + (f"; pruner masks {args.prune}" if args.prune else "")
                + ("; int8 activation scales calibrated on 2 other synthetic frames" if args.precision == "int8" else ""),
        "config": {"workload": f"{args.arch} dense inference, seg_video loop (uint8 frame -> uint8 labels) "
                               f"{H}x{W}, {B} frames/GPU/step",
                   "arch": args.arch, "height": H, "width": W, "frames_per_gpu_step": B,
                   "global_batch": B * world, "parallelism": f"dp{world} (frames sharded, no data-path collective)"},
    }
    if args.prune:
        sparse = [i for i, nm in enumerate(names) if nm.startswith("conv_big_kernel") and nm.endswith("true>")]
        out["config"]["workload"] = out["config"]["workload"].replace("dense inference", f"{args.prune} pruned inference")
        out["config"]["block_sparse"] = {"pruned_layers": n_pruned, "sparse_launches": len(sparse),
                                         "mean_weight_density_of_sparse_launches":
                                             round(sum(density[i] for i in sparse) / max(len(sparse), 1), 4),
                                         "kernels": "K-step compaction" if args.block_sparse else "dense",
                                         "flops": "useful (dense x weight density); dense-equivalent in "
                                                  "roofline.dense_equivalent_achieved"}
    traffic, traffic_src = pmc_traffic(args, dominant) if durs else (None, None)
    if durs:
        avg_d = sum(durs) / len(durs)
        avg_f = sum(flops) / len(flops)
        ach = avg_f / avg_d / 1e12
        peak = kernel_peak(dominant, plan.packed.base) / 1e12
        out["roofline"] = {"bound": "mfma", "kernel": dominant, "achieved": round(ach, 2), "peak": peak,
                           "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": traffic,
                           "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                           "dense_equivalent_achieved": round(sum(per[dominant]["fd"]) / len(durs) / avg_d / 1e12, 2),
                           "launches": len(durs), "avg_launch_us": round(avg_d * 1e6, 2),
                           "avg_launch_gflop": round(avg_f / 1e9, 3),
                           "share_of_step": round(sum(durs) / el, 3)}
        out["kernels_source"] = ("dominant kernel: HIP events around its launches in the timed region; "
                                 "the others: one fully instrumented step after it")
        out["kernels"] = {k: {"launches": len(v["d"]), "avg_us": round(sum(v["d"]) / len(v["d"]) * 1e6, 1),
                              "tflops": round(sum(v["f"]) / sum(v["d"]) / 1e12, 1),
                              "gbps": round(sum(v["b"]) / sum(v["d"]) / 1e9, 1)}
                          for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]["d"]))}
    out["network_roofline"] = {"t_star_ms_per_frame": nr["t_star_s"] / B * 1e3,
                               "measured_ms_per_frame": el / args.steps / B * 1e3,
                               "frac": nr["t_star_s"] / (el / args.steps),
                               "gflop_per_frame": nr["flops"] / B / 1e9, "gb_per_frame": nr["bytes"] / B / 1e9,
                               "achieved_tflops": nr["flops"] * args.steps / el / 1e12}
    if host is not None:
        out["host_frames"] = host
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], (bframes, blabels) = cpu_baseline(args, args.cpu_seconds)
        if not args.prune:                   # the oracle runs the unpruned synthetic weights
            out["parity_vs_ref"] = parity_vs_ref(args, model, bframes, blabels, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_frames_run(args, model, step, world, dev):
    """PCIe-inclusive pipeline (seg_video_old_no_plot.py:123-166 hands host frames to the model):
    uint8 frames in pinned host memory, H2D of batch i+1 on a copy stream while batch i computes,
    two device frame buffers, events order the hand-offs.  Same barrier/max-over-ranks timing."""
    import torch
    import torch.distributed as dist
    from drnmi.dist import max_over_ranks
    B, H, W = args.batch, args.height, args.width
    g = torch.Generator().manual_seed(2000)
    host = [torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, generator=g).pin_memory() for _ in range(2)]
    bufs = [torch.empty(B, H, W, 3, dtype=torch.uint8, device=dev) for _ in range(2)]
    copy = torch.cuda.Stream(device=dev)
    comp = torch.cuda.current_stream(dev)
    loaded = [torch.cuda.Event() for _ in range(2)]
    freed = [torch.cuda.Event() for _ in range(2)]

    def run(n):
        with torch.cuda.stream(copy):
            bufs[0].copy_(host[0], non_blocking=True)
            loaded[0].record(copy)
        for i in range(n):
            cur, nxt = i % 2, (i + 1) % 2
            if i + 1 < n:
                with torch.cuda.stream(copy):
                    if i >= 1:
                        copy.wait_event(freed[nxt])          # batch i-1's compute read bufs[nxt]
                    bufs[nxt].copy_(host[nxt], non_blocking=True)
                    loaded[nxt].record(copy)
            comp.wait_event(loaded[cur])
            step(False, bufs[cur])
            freed[cur].record(comp)

    run(max(args.warmup, 2))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, device=dev)
    return {"value": world * B * args.steps / el, "unit": "frames/s", "ms_per_step": el / args.steps * 1e3,
            "h2d_bytes_per_frame": H * W * 3,
            "note": "frames in pinned host memory, H2D on a copy stream overlapped with compute (not the "
                    "headline: the headline times HBM-resident frames)"}


def pmc_traffic(args, kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC capture of this exact
    workload (profiles/*_pmc_traffic.json, made by scripts/pmc_traffic.sh: FETCH_SIZE x 2 +
    WRITE_SIZE, MI355X_MICROARCH.md §HBM); PMC counters cannot be read inside the timed run."""
    import glob
    want = {"arch": args.arch, "height": args.height, "width": args.width, "frames_per_gpu_step": args.batch,
            "precision": args.precision}
    here = os.path.dirname(os.path.abspath(__file__))
    for f in sorted(glob.glob(os.path.join(here, "profiles", "*_pmc_traffic.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") == want and kernel in d.get("kernels", {}):
            return round(d["kernels"][kernel]["traffic_bytes"]), os.path.relpath(f, here)
    return None, None


if __name__ == "__main__":
    main()
