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

`--gpus N` without a torchrun environment spawns the N rank processes itself (before any GPU
call; one device each, RCCL rendezvous on 127.0.0.1); under torchrun WORLD_SIZE must equal N.
The default bf16 line also carries `exact_mode` (the fp32-accurate split-bf16 engine),
`exact_mode_fp32` (exact fp32 on the f32 MFMA) and `int8_mode` (config C5's W8A8): the other
modes on the same weights and frames, timed in the same process (--exact-steps each), each with
its own dominant-kernel roofline (HIP-event achieved rate, committed PMC traffic and MFMA-busy),
time accounting (per-step spread, launch sum vs step) and parity vs the reference.

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


def parse(argv=None):
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
    ap.add_argument("--no-exact-mode", action="store_true",
                    help="skip the exact_mode (fp32x) sub-measurement of the default bf16 line")
    ap.add_argument("--exact-steps", type=int, default=20,
                    help="timed steps of each sub-line (fp32x / fp32 / int8) of the default bf16 line")
    ap.add_argument("--stub-step", action="store_true",
                    help="test hook: no GPU; gloo ranks run a CPU stand-in step through the same launcher, "
                         "seeding, timing and max-over-ranks code (tests/test_bench_launcher.py)")
    return ap.parse_args(argv)


def spawn_ranks(n: int, argv, script: str | None = None) -> int:
    """`python bench.py --gpus N` outside torchrun: start N rank processes of this script (or of
    `script`: bench_finetune.py uses the same launcher; one per GPU, LOCAL_RANK = RANK = r) with a
    127.0.0.1 rendezvous, before this process touches the GPU, and return the worst exit code.
    The reference's multi-GPU entry does the same through torch.multiprocessing +
    init_process_group (semantic_seg_multigpu.py:467-468)."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__), *argv], env=env))
    rcs = [None] * n
    try:
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
                    if rcs[i] not in (None, 0):      # one rank failed: the others would hang in a collective
                        for q in procs:
                            if q.poll() is None:
                                q.terminate()
            time.sleep(0.05)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return max(abs(rc) for rc in rcs)


def resolve_world(args, environ=os.environ, prog: str = "bench.py"):
    """(world, rank, local_rank) of this process, or None when it must spawn the ranks itself.
    A torchrun environment whose WORLD_SIZE differs from --gpus is refused."""
    if environ.get("WORLD_SIZE") is None:
        if args.gpus > 1:
            return None
        return 1, 0, 0
    world = int(environ["WORLD_SIZE"])
    if world != args.gpus:
        raise SystemExit(f"{prog}: --gpus {args.gpus} but WORLD_SIZE={world} (launch with matching values)")
    return world, int(environ.get("RANK", "0")), int(environ.get("LOCAL_RANK", "0"))


def timed_region(step, steps, world, dev, marks=None, lead=None):
    """K timed steps bracketed by barrier + device sync on both sides; the slowest rank's
    elapsed time defines the job (max over ranks).  Returns (job_seconds, own_seconds).
    `marks`: steps + 1 HIP events recorded at the step boundaries (per-step spread; one event
    per step, on the stream the step launches on).  `lead`: the last untimed warm-up step, run
    after the host-side bookkeeping (collector pass, event collection), so the device is busy up
    to the bracketing sync instead of idling through it (an idle device starts the first timed
    step at a lower clock: +1.5 ms on the first of 20 bf16 steps, BENCH step_ms.max_at_step 0)."""
    import torch
    import torch.distributed as dist
    from drnmi.dist import max_over_ranks
    import gc
    cuda = dev.type == "cuda"
    gc.collect()                 # no collector pause inside the timed steps (re-enabled after them)
    gc.disable()
    if lead is not None:
        lead()
    if cuda:
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    if cuda:
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if marks is not None:
        marks[0].record()
    for k in range(steps):
        step(True)
        if marks is not None:
            marks[k + 1].record()
    if cuda:
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    own = time.perf_counter() - t0
    gc.enable()
    return max_over_ranks(own, device=dev), own


def step_spread(marks):
    """min / median / max of the per-step durations (ms) between consecutive boundary events, the
    slowest step's index, and the time steps spent beyond 1.5x the median (one-off stalls: a 20-40
    ms stall inside one step is what made the 5-step exact-mode line of BENCH_r05 read 4 ms/step
    slower than its kernels)."""
    raw = [a.elapsed_time(b) for a, b in zip(marks, marks[1:])]
    if not raw:
        return None
    d = sorted(raw)
    mid = len(d) // 2
    med = d[mid] if len(d) % 2 else 0.5 * (d[mid - 1] + d[mid])
    stall = sum(x - med for x in raw if x > 1.5 * med)
    return {"min": round(d[0], 4), "median": round(med, 4), "max": round(d[-1], 4), "steps": len(d),
            "max_at_step": raw.index(d[-1]), "stall_ms": round(stall, 3)}


def gather_ranks(vals, world, dev):
    """[[v0, v1, ...] per rank] of a few host floats (per-rank bookkeeping in the JSON line)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=dev)
    if world == 1:
        return [t.tolist()]
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def frame_seed(rank: int) -> int:
    """Per-rank synthetic frame stream: every rank segments different frames."""
    return 1000 + rank


def stub_main(args, world, rank):
    """CPU stand-in for the GPU step (test hook): gloo ranks, per-rank seeded uint8 frames of the
    requested shape, a reduction over them as the 'step'; same timing and JSON fields."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cpu")
    if world > 1:
        dist.init_process_group("gloo")
    g = torch.Generator().manual_seed(frame_seed(rank))
    frames = torch.randint(0, 256, (args.batch, args.height, args.width, 3), dtype=torch.uint8, generator=g)
    acc = [0.0]

    def step(timed):
        acc[0] += float(frames.float().mean())

    for _ in range(args.warmup):
        step(False)
    el, own = timed_region(step, args.steps, world, dev)
    per = gather_ranks([frame_seed(rank), float(frames.long().sum()), own], world, dev)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": world * args.batch * args.steps / el, "unit": "frames/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": el / args.steps * 1e3, "scaling": "weak", "data": "stub (CPU test hook)",
                          "per_rank": [{"rank": r, "frame_seed": int(v[0]), "frame_sum": int(v[1]),
                                        "seconds": v[2]} for r, v in enumerate(per)]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


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


def parity_vs_ref(args, model, frames, ref_labels, dev, precision=None):
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
    return {"frames": len(frames), "precision": precision or args.precision,
            "label_agreement": float((got == ref).float().mean()),
            "label_mismatches": int((got != ref).sum()),
            "miou_vs_ref": float(metrics.miou(hist.cpu().numpy())),
            "reference": "oracle/drn_oracle.py fp32 torch-CPU forward, same weights and frames"}


def measure(args, model, frames, steps, warmup, world, dev, kernel_events=True):
    """Time `steps` seg_video steps of `model` over `frames` (resident in HBM) after `warmup`
    untimed ones.  Returns the job time and the dominant kernel's per-launch HIP-event record
    (timed region) plus a per-kernel table (one fully instrumented step after it)."""
    import ctypes

    import torch
    from drnmi import _lib
    from drnmi.drnseg import INFO_MEAN, INFO_STD
    from drnmi.roofline import launch_work

    B, H, W = frames.shape[0], frames.shape[1], frames.shape[2]
    plan = model.plan(B, H, W, device=dev)     # the plan model.segment() runs (same key)
    lib = _lib.load()
    front = getattr(plan, "front_fused", False)
    fused_stem = getattr(plan, "stem_fused", False) and not front

    blocks = getattr(plan, "block64", {})

    def launched_name(i):
        if front and i <= 2:                 # layer0..layer2 in one launch (drnmi_video_front_u8)
            return "" if i else "front3_kernel"
        if i in blocks:                      # a 64-channel BasicBlock in one launch (drnmi_basic_block64)
            return "block64_kernel"
        if i - 1 in blocks:
            return ""
        if fused_stem and i <= 1:            # stem + layer1 in one launch (drnmi_stem_layer1)
            return "" if i == 1 else lib.drnmi_stem_layer1_kernel_name(
                ctypes.byref(plan.stem_u8), ctypes.byref(plan.args[1])).decode()
        a = plan.stem_u8 if (i == 0 and plan.stem_u8 is not None) else plan.args[i]
        if a is None:
            return ""                        # downsample folded into its block's last conv
        return lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode()

    names = [launched_name(i) for i in range(len(plan.args))]
    path = plan.labels_path()
    if path == "seg2":                         # the seg classifier in the last conv's epilogue (drnmi_conv_stag_seg)
        names[plan.seg_fused["conv"]] = lib.drnmi_conv_stag_seg_kernel_name(
            ctypes.byref(plan.args[plan.seg_fused["conv"]])).decode()
        names[plan.seg_idx] = ""
    # the head launch (index len(nodes), DRNSeg._segment_impl): up x8 + argmax -> uint8 labels
    # (ops.hip drnmi_up8_labels_seg2 / _seg2_i8 / _nhwc launch the tiled uniform-window kernel; NCHW
    # logits the oct kernel)
    i8_head = path == "seg2" and plan.seg_fused["i8"]
    names.append({"seg2": "up8_labels_tile_kernel<19, U8, SEG2%s>" % ("_I8" if i8_head else ""),
                  "nhwc": "up8_labels_tile_kernel<19, U8, NHWC>"}.get(path, "up8_labels_oct_kernel<19, U8>"))
    nodes = plan.packed.graph.nodes
    # per-launch work (roofline.launch_work): a folded downsample's FLOPs and input run inside its
    # block's last conv, the fused stem launch carries layer1; useful work of a pruned layer
    #  = dense FLOPs x the density of its weights, on dense and sparse kernels alike
    works = launch_work(plan)
    density = [float((nd.conv.weight != 0).sum()) / nd.conv.weight.numel() for nd in nodes]
    for k, on in ((3, front), (2, fused_stem)):
        if on:
            density[:k] = [float(sum((nd.conv.weight != 0).sum() for nd in nodes[:k])) /
                           sum(nd.conv.weight.numel() for nd in nodes[:k])] * k
            break
    for i in blocks:                         # the fused block's row carries both convs
        d2 = [float((nd.conv.weight != 0).sum()) for nd in nodes[i:i + 2]]
        density[i] = density[i + 1] = sum(d2) / sum(nd.conv.weight.numel() for nd in nodes[i:i + 2])
    dense_flops = {i: w[1] for i, w in enumerate(works)}
    works = [(w[0], w[1] * density[i], w[2]) if i < len(nodes) else w for i, w in enumerate(works)]
    events = []
    pool = [torch.cuda.Event(enable_timing=True) for _ in range(2 * len(names) * max(steps, 2))]
    watch = [None]        # None: every launch; else only launches of this kernel name

    def hook(i, nd, before):
        if watch[0] is not None and names[i] != watch[0]:
            return
        ev = pool[len(events)]
        ev.record()
        events.append((i, before, ev))

    def step(timed, x=frames):
        # the public API a seg_video user calls: DRNSeg.segment -> torch.ops.drnmi.segment
        model.timing_hook = hook if (timed and kernel_events) else None
        return model.segment(x, INFO_MEAN, INFO_STD, False)

    launches = []         # (node index, seconds) of the last collect(), in launch order

    def collect():
        """per-kernel durations of the recorded launches (the events list is then reset)"""
        torch.cuda.synchronize()
        per_, pend = {}, {}
        launches.clear()
        for i, before, ev in events:
            if before:
                pend[i] = ev
            else:
                d = pend.pop(i).elapsed_time(ev) * 1e-3
                launches.append((i, d))
                g_ = per_.setdefault(names[i], {"d": [], "f": [], "b": [], "fd": []})
                g_["d"].append(d)
                g_["f"].append(works[i][1])
                g_["fd"].append(dense_flops[i])
                g_["b"].append(works[i][2])
        events.clear()
        return per_

    for _ in range(max(warmup - 2, 0)):
        step(False)
    # the next-to-last warm-up step instrumented: it names the dominant kernel (the template
    # instance, as rocprofv3 names it, with the largest total time); inside the timed region only
    # that kernel's launches carry HIP events (events around all ~25 launches cost ~2.7 % per step);
    # the last warm-up step runs inside timed_region, ahead of its opening sync
    step(True)
    warm = collect()
    dominant = max(warm, key=lambda k: sum(warm[k]["d"])) if warm else None
    watch[0] = dominant
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    el, own = timed_region(step, steps, world, dev, marks, lead=(lambda: step(False)) if warmup >= 2 else None)
    timed_per = collect()
    spread = step_spread(marks)
    # per-kernel table: one fully instrumented step after the timed region
    watch[0] = None
    step(True)
    first_last = (events[0][2], events[-1][2]) if events else None
    per = collect()
    inst_span = first_last[0].elapsed_time(first_last[1]) if first_last else None
    # time accounting (per step): the dominant kernel's launches from the timed region, every
    # other launch from the instrumented step; what the launches do not cover is idle time between
    # them (host launch gaps, allocator work, a stall) -- the instrumented step's own span vs its
    # launch sum separates host gaps from a one-off stall in the timed region
    inst_sum = sum(sum(v["d"]) for v in per.values())
    dom_timed = sum(timed_per[dominant]["d"]) / steps if dominant in timed_per else 0.0
    dom_inst = sum(per[dominant]["d"]) if dominant in per else 0.0
    ksum = inst_sum - dom_inst + dom_timed
    step_ms = el / steps * 1e3
    accounting = {"ms_per_step": round(step_ms, 4), "kernel_sum_ms_per_step": round(ksum * 1e3, 4),
                  "unaccounted_ms_per_step": round(step_ms - ksum * 1e3, 4),
                  "unaccounted_frac": round(1.0 - ksum * 1e3 / step_ms, 4),
                  "step_ms": spread,
                  "instrumented_step": {"span_ms": round(inst_span, 4) if inst_span else None,
                                        "kernel_sum_ms": round(inst_sum * 1e3, 4)},
                  "note": "kernel_sum = the dominant kernel's timed-region launches / steps + every other "
                          "launch of one fully instrumented step after the timed region; step_ms = HIP events "
                          "at the timed steps' boundaries"}
    # per launch of that step, keyed by the node that opens it (the conv_stag family's launches
    # differ in K and tile count: the weakest shows here, not in the per-kernel average)
    layers = [{"node": nodes[i].name if i < len(nodes) else "head", "kernel": names[i], "us": round(d * 1e6, 1),
               "gflop": round(works[i][1] / 1e9, 2), "tflops": round(works[i][1] / d / 1e12, 1),
               "gbps": round(works[i][2] / d / 1e9, 1)} for i, d in launches]
    if dominant in timed_per:
        per[dominant] = timed_per[dominant]
    model.timing_hook = None
    return {"el": el, "own": own, "plan": plan, "names": names, "density": density, "per": per,
            "dominant": dominant, "timed": timed_per.get(dominant), "step": step, "layers": layers,
            "accounting": accounting}


def roofline_block(args, m, precision):
    """The dominant kernel's roofline object from a measure() record."""
    from drnmi.roofline import kernel_peak
    t = m["timed"]
    if not t:
        return None, None
    durs, flops = t["d"], t["f"]
    avg_d = sum(durs) / len(durs)
    avg_f = sum(flops) / len(flops)
    ach = avg_f / avg_d / 1e12
    peak = kernel_peak(m["dominant"], m["plan"].packed.base) / 1e12
    traffic, traffic_src = pmc_traffic(args, m["dominant"], precision)
    mfma = pmc_mfma(args, precision)
    mk = mfma.get("kernels", {})
    dom_mfma = mk.get(m["dominant"]) or mk.get(m["dominant"].replace("<f32,", "<float,")) or {}
    # the step's MFMA-pipe utilisation: every kernel's captured busy fraction weighted by its time in
    # this run's per-kernel table (kernels without a capture row are reported as uncovered time)
    wt = cov = 0.0
    tot = sum(sum(v["d"]) for v in m["per"].values())
    for k, v in m["per"].items():
        row = mk.get(k) or mk.get(k.replace("<f32,", "<float,"))
        if row and row.get("mfma_busy") is not None:
            wt += row["mfma_busy"] * sum(v["d"])
            cov += sum(v["d"])
    roof = {"bound": "mfma", "kernel": m["dominant"], "achieved": round(ach, 2), "peak": peak,
            "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": traffic,
            "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
            "mfma_busy": dom_mfma.get("mfma_busy"),
            "eff_clock_ghz": dom_mfma.get("eff_clock_ghz"),
            "mfma_busy_step": round(wt / cov, 4) if cov else None,
            "mfma_busy_step_coverage": round(cov / tot, 4) if tot else None,
            "mfma_busy_source": mfma.get("source"),
            "mfma_busy_norm": mfma.get("norm"),
            "dense_equivalent_achieved": round(sum(t["fd"]) / len(durs) / avg_d / 1e12, 2),
            "launches": len(durs), "avg_launch_us": round(avg_d * 1e6, 2),
            "avg_launch_gflop": round(avg_f / 1e9, 3),
            "share_of_step": round(sum(durs) / m["el"], 3)}
    kernels = {k: {"launches": len(v["d"]), "avg_us": round(sum(v["d"]) / len(v["d"]) * 1e6, 1),
                   "tflops": round(sum(v["f"]) / sum(v["d"]) / 1e12, 1),
                   "gbps": round(sum(v["b"]) / sum(v["d"]) / 1e9, 1)}
               for k, v in sorted(m["per"].items(), key=lambda kv: -sum(kv[1]["d"]))}
    return roof, kernels


def network_block(m, steps, B):
    from drnmi.roofline import network_roofline
    nr = network_roofline(m["plan"])
    step_s = m["el"] / steps
    return {"t_star_ms_per_frame": nr["t_star_fused_s"] / B * 1e3,
            "t_star_per_layer_ms_per_frame": nr["t_star_s"] / B * 1e3,
            "measured_ms_per_frame": step_s / B * 1e3,
            "frac": nr["t_star_fused_s"] / step_s,
            "frac_per_layer": nr["t_star_s"] / step_s,
            "t_star_note": "frac = fused floor (the launches the plan issues, charged the bytes they move: "
                           "drnmi/roofline.py launch_work); frac_per_layer charges every layer its unfused bytes",
            "gflop_per_frame": nr["flops"] / B / 1e9, "gb_per_frame": nr["fused_bytes"] / B / 1e9,
            "gb_per_frame_per_layer": nr["bytes"] / B / 1e9,
            "achieved_tflops": nr["flops"] / step_s / 1e12}


def main(argv=None):
    args = parse(argv)
    wr = resolve_world(args)
    if wr is None:                            # --gpus N outside torchrun: spawn the ranks
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:] if argv is None else argv))
    world, rank, local = wr
    if args.stub_step:
        return stub_main(args, world, rank)
    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from drnmi.drnseg import build

    if args.prune:
        model, n_pruned = pruned_model(args, dev)
    else:
        model = build(args.arch, 19, seed=0, device=dev,
                      precision="bf16" if args.precision == "int8" else args.precision)
    if args.precision == "int8":
        model = calibrate(model, args, dev)
    B, H, W = args.batch, args.height, args.width
    g = torch.Generator(device=dev).manual_seed(frame_seed(rank))
    frames = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    m = measure(args, model, frames, args.steps, args.warmup, world, dev, not args.no_kernel_events)
    el, names, density = m["el"], m["names"], m["density"]
    host = host_frames_run(args, model, m["step"], world, dev) if args.host_frames else None
    per_rank = gather_ranks([frame_seed(rank), m["own"]], world, dev)

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
    if world > 1:
        out["per_rank"] = [{"rank": r, "frame_seed": int(v[0]), "frames": B * args.steps, "seconds": round(v[1], 6)}
                           for r, v in enumerate(per_rank)]
    if args.prune:
        sparse = [i for i, nm in enumerate(names) if nm.startswith("conv_big_kernel") and nm.endswith("true>")]
        out["config"]["workload"] = out["config"]["workload"].replace("dense inference", f"{args.prune} pruned inference")
        out["config"]["block_sparse"] = {"pruned_layers": n_pruned, "sparse_launches": len(sparse),
                                         "mean_weight_density_of_sparse_launches":
                                             round(sum(density[i] for i in sparse) / max(len(sparse), 1), 4),
                                         "kernels": "K-step compaction" if args.block_sparse else "dense",
                                         "flops": "useful (dense x weight density); dense-equivalent in "
                                                  "roofline.dense_equivalent_achieved"}
    roof, kernels = roofline_block(args, m, args.precision)
    if roof is not None:
        out["roofline"] = roof
        out["kernels_source"] = ("dominant kernel: HIP events around its launches in the timed region; "
                                 "the others: one fully instrumented step after it")
        out["kernels"] = kernels
        out["layers"] = m["layers"]
    out["network_roofline"] = network_block(m, args.steps, B)
    out["accounting"] = m["accounting"]
    sp = m["accounting"]["step_ms"] or {}
    out["value_at_median_step"] = round(world * B / sp["median"] * 1e3, 2) if sp.get("median") else None
    if host is not None:
        out["host_frames"] = host
    exact = {}                               # precision -> (sub-line, model)
    if (world == 1 and args.precision == "bf16" and not args.prune and not args.no_exact_mode
            and not args.no_kernel_events):
        # the other precision modes on the same weights and frames, timed in this process (each its
        # own warm-up, >= 20 timed steps, per-step spread and time accounting): the exact-argmax modes
        # (north star: labels bit-exact vs the reference) fp32x (split-bf16, fp32-accurate) and fp32
        # (the reference's own arithmetic on the f32-input MFMA), and int8 (config C5's W8A8)
        for prec, arith in SUB_MODES:
            xm = build(args.arch, 19, seed=0, device=dev, precision="bf16" if prec == "int8" else prec)
            if prec == "int8":
                xm = calibrate(xm, args, dev)
            mx = measure(args, xm, frames, args.exact_steps, SUB_WARMUP, world, dev)
            xroof, xkern = roofline_block(args, mx, prec)
            sp = mx["accounting"]["step_ms"] or {}
            exact[prec] = ({"precision": prec, "value": B * args.exact_steps / mx["el"], "unit": "frames/s",
                            "value_at_median_step": round(B / sp["median"] * 1e3, 2) if sp.get("median") else None,
                            "steps": args.exact_steps, "warmup": SUB_WARMUP,
                            "ms_per_step": mx["el"] / args.exact_steps * 1e3,
                            "roofline": xroof, "network_roofline": network_block(mx, args.exact_steps, B),
                            "accounting": mx["accounting"], "kernels": xkern, "arithmetic": arith}, xm)
            del mx
            torch.cuda.empty_cache()
        out["exact_mode"] = exact["fp32x"][0]
        out["exact_mode_fp32"] = exact["fp32"][0]
        out["int8_mode"] = exact["int8"][0]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], (bframes, blabels) = cpu_baseline(args, args.cpu_seconds)
        if not args.prune:                   # the oracle runs the unpruned synthetic weights
            out["parity_vs_ref"] = parity_vs_ref(args, model, bframes, blabels, dev)
            for prec, (line, xm) in exact.items():
                line["parity_vs_ref"] = parity_vs_ref(args, xm, bframes, blabels, dev, prec)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


SUB_MODES = (
    ("fp32x", "fp32-accurate: exact 3-way bf16 split of weights and activations, the six products above "
              "2^-24 on the bf16 MFMA, fp32 accumulation (peak 2.5 PF / 6)"),
    ("fp32", "exact fp32: f32-input MFMA (v_mfma_f32_16x16x4_f32 = an fmaf chain per output), fp32 "
             "activations, the reference's arithmetic (peak 157.3 TF)"),
    ("int8", "W8A8 (config C5): per-output-channel int8 weights, per-tensor int8 activations calibrated on "
             "2 other synthetic frames, int32 accumulation on the i8 MFMA (peak 5 POPS) for cin >= 64 and "
             "cout >= 256; bf16 below"),
)
SUB_WARMUP = 3


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


def newest_first(pattern):
    """Committed capture files, the latest round first: names start r<round><letters>_ (r9zz_ <
    r10a_ < r10p_), which plain string order gets wrong across the r9 -> r10 boundary."""
    import glob
    import re

    def key(f):
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), m.group(2)) if m else (-1, "")
    return sorted(glob.glob(pattern), key=key, reverse=True)


def pmc_mfma(args, precision=None):
    """Per-kernel MFMA-pipe utilisation and held clock from the newest committed capture of this
    exact workload (profiles/*_pmc_mfma.json, made by scripts/pmc_mfma.sh:
    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)); PMC counters cannot be
    read inside the timed run.  {} when no capture matches."""
    import glob
    want = {"arch": args.arch, "height": args.height, "width": args.width, "frames_per_gpu_step": args.batch,
            "precision": precision or args.precision}
    here = os.path.dirname(os.path.abspath(__file__))
    for f in newest_first(os.path.join(here, "profiles", "*_pmc_mfma.json")):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config") == want and d.get("kernels"):
            return {"kernels": d["kernels"], "source": os.path.relpath(f, here),
                    "norm": "per dispatch SQ_VALU_MFMA_BUSY_CYCLES / ((GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs) "
                            "in a separate rocprofv3 --pmc pass of this workload; mfma_busy_step = those per-kernel "
                            "fractions weighted by each kernel's time in this run's per-kernel table"}
    return {}


def pmc_traffic(args, kernel, precision=None):
    """HBM bytes per launch of `kernel` from the newest committed PMC capture of this exact
    workload (profiles/*_pmc_traffic.json, made by scripts/pmc_traffic.sh: FETCH_SIZE x 2 +
    WRITE_SIZE, MI355X_MICROARCH.md §HBM); PMC counters cannot be read inside the timed run."""
    import glob
    want = {"arch": args.arch, "height": args.height, "width": args.width, "frames_per_gpu_step": args.batch,
            "precision": precision or args.precision}
    here = os.path.dirname(os.path.abspath(__file__))
    for f in newest_first(os.path.join(here, "profiles", "*_pmc_traffic.json")):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        ks = d.get("kernels", {})
        # drnmi_conv_kernel_name spells the fp32 igemm's element type "f32"; rocprof demangles "float"
        for k in (kernel, kernel.replace("<f32,", "<float,")):
            if d.get("config") == want and k in ks:
                return round(ks[k]["traffic_bytes"]), os.path.relpath(f, here)
    return None, None


if __name__ == "__main__":
    main()
