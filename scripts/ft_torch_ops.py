"""Which PyTorch glue ops run inside one fine-tune step (bench_finetune.py's step: forward,
CrossEntropyLoss, zero_grad, backward, SGD) and from where: torch.profiler over one step after
warm-up, aten ops by device time, with the Python frames that issued them.
python scripts/ft_torch_ops.py [--batch 2] [--height 1024] [--width 768]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-seg-model-compress_amd"))


def main():
    import bench_finetune as bf
    args = bf.parse(sys.argv[1:])
    import torch
    from drnmi.drnseg import DRNSeg
    from drnmi.train import SGD, CrossEntropyLoss
    from drnmi.weights import synth_state_dict
    dev = torch.device("cuda", 0)
    m = DRNSeg(args.arch, 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, 0))
    pr = bf.rmb_pruner(m, on_gpu=False)
    m = m.to(dev).train().set_precision(args.precision)
    for k in list(pr.mask_dict):
        pr.mask_dict[k] = pr.mask_dict[k].to(dev)
    pr.on_gpu = True
    pr.apply_masks(m)
    opt = SGD(m.optim_parameters(), 0.01, momentum=0.9, weight_decay=1e-4, pruner=pr, model=m)
    crit = CrossEntropyLoss(ignore_index=255)
    B, H, W = args.batch, args.height, args.width
    g = torch.Generator(device=dev).manual_seed(2000)
    x = torch.randn(B, 3, H, W, device=dev, generator=g)
    t = torch.randint(0, 19, (B, H, W), device=dev, generator=g)
    t[torch.rand(B, H, W, device=dev, generator=g) < 0.1] = 255

    def step():
        out = m(x)[0]
        loss = crit(out, t)
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    ka = prof.key_averages()
    rows = [e for e in ka if e.key.startswith("aten::") and e.count > 0]
    rows.sort(key=lambda e: -e.device_time_total)
    print("aten ops in one step (count, device us total, cpu us total):")
    for e in rows[:30]:
        print(f"  {e.key:40s} {e.count:5d} {e.device_time_total:10.1f} {e.cpu_time_total:10.1f}")
    print("\nby Python stack (top 25, device time):")
    ks = prof.key_averages(group_by_stack_n=6)
    srows = [e for e in ks if e.key.startswith("aten::") and e.device_time_total > 0]
    srows.sort(key=lambda e: -e.device_time_total)
    for e in srows[:25]:
        st = [s for s in e.stack if "site-packages" not in s][:4]
        print(f"  {e.key:30s} n={e.count:4d} dev={e.device_time_total:9.1f}us  <- " + " | ".join(st))


if __name__ == "__main__":
    main()
