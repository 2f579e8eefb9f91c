"""BASELINE.json configs C1, C4 and C5 run end to end on the GPU, each against the oracle.

C1  D-22 dense forward on one 1x3x512x1024 frame (semantic_seg.py:429-468 test() shape), fp32
    and fp32x modes vs the torch-CPU oracle run inside the test: logits <= 1e-3 max-abs, labels
    identical on every pixel.
C2 headline size: D-22 on one 1x3x1024x2048 frame (BASELINE metric shape, the bench's weights
    and its parity frame) in the exact-argmax modes: fp32 labels identical on every pixel; fp32x
    flips bounded to near-ties (oracle top-2 log-prob margin <= 1e-5) and at most 4 pixels.
C4  D-54 + RmbPruner 75 % (tests/golden/rmb_d54_8x8_75.json, masks pinned to the reference's
    RmbPruner by tests/golden/masks.npz) fine-tune step: train-mode forward, CE(ignore 255),
    HIP backward, SGD with the pruner's masks fused into the step (semantic_seg.py:166-230,
    :963-966, :213-214) vs the oracle's fp64 step with the same masks.
C5  D-22 + SRMBRepMasker (the shipped optimal_configs/drn_d_22 50 % config, masks pinned by
    tests/golden/masks.npz srmb_d22_seed11) + int8: every int8 launch bit-exact against
    oracle/int8_oracle.py from its own HBM inputs; labels vs the masked fp32 oracle forward.
"""
import os

import numpy as np
import pytest
import torch

import train_case as TC
from oracle import drn_oracle as O
from oracle import int8_oracle as Q

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _masks_match_golden(golden, tag, mask_dict):
    import hashlib
    for layer, m in mask_dict.items():
        a = m.cpu().numpy()
        sha = hashlib.sha256(np.ascontiguousarray((a != 0).astype(np.uint8)).tobytes()).hexdigest()
        assert sha == str(golden[f"{tag}/sha/{layer}"]), layer


@pytest.mark.parametrize("precision", ["fp32", "fp32x"])
def test_c1_d22_512x1024_fp32_vs_oracle(precision):
    from drnmi.drnseg import build
    from drnmi.weights import synth_frames
    m = build("drn_d_22", 19, seed=5, device=DEV, precision=precision)
    frames = synth_frames(31, 1, 512, 1024)
    x = O.preprocess_u8(frames)
    lp, logits = m(x.to(DEV))
    lab_seg = m.segment(torch.from_numpy(frames).to(DEV))
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_lp, ref_logits, _ = O.drnseg_forward(sd, "drn_d_22", x)
    assert lp.shape == (1, 19, 512, 1024) and logits.shape == (1, 19, 64, 128)
    err = (logits.cpu() - ref_logits).abs().max().item()
    lp_err = (lp.cpu() - ref_lp).abs().max().item()
    top2 = torch.topk(ref_lp, 2, dim=1).values
    margin = (top2[:, 0] - top2[:, 1]).numpy()
    lab = torch.max(lp, 1)[1].cpu().numpy()
    ref_lab = torch.max(ref_lp, 1)[1].numpy()
    diff = lab != ref_lab
    print(f"C1 D-22 1x3x512x1024 {precision}: logits max-abs {err:.2e}, log-probs {lp_err:.2e}, "
          f"labels differ {int(diff.sum())} px ({int((margin <= 1e-4).sum())} px with margin <= 1e-4)")
    assert err <= 1e-3 and lp_err <= 1e-3
    assert int(diff.sum()) == 0                                      # bit-exact argmax
    assert torch.equal(lab_seg.cpu().long(), torch.from_numpy(lab))   # u8 video path == NCHW path


@pytest.mark.parametrize("precision", ["fp32", "fp32x"])
def test_headline_1024x2048_exact_modes_vs_oracle(precision):
    """lmodels/drnseg.py:295-299 + semantic_seg.py:445 at the BASELINE frame size, through the
    video path the bench times (segment: uint8 frame -> labels), on bench.py's weights (seed 0)
    and its first parity frame (synth_frames(7, 2, ...)[0])."""
    from drnmi.drnseg import build
    from drnmi.weights import synth_frames
    m = build("drn_d_22", 19, seed=0, device=DEV, precision=precision)
    frames = synth_frames(7, 2, 1024, 2048)[:1]
    x = O.preprocess_u8(frames)
    lp, logits = m(x.to(DEV))
    lab_seg = m.segment(torch.from_numpy(frames).to(DEV))
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_lp, ref_logits, _ = O.drnseg_forward(sd, "drn_d_22", x)
    err = (logits.cpu() - ref_logits).abs().max().item()
    lp_err = (lp.cpu() - ref_lp).abs().max().item()
    del lp
    top2 = torch.topk(ref_lp, 2, dim=1).values
    margin = (top2[:, 0] - top2[:, 1]).numpy()
    ref_lab = torch.max(ref_lp, 1)[1].numpy()
    lab = lab_seg.cpu().long().numpy()
    diff = lab != ref_lab
    print(f"headline D-22 1x3x1024x2048 {precision}: logits max-abs {err:.2e}, log-probs {lp_err:.2e}, "
          f"labels differ {int(diff.sum())} of {diff.size} px (max oracle margin among them "
          f"{float(margin[diff].max()) if diff.any() else 0.0:.2e}; {int((margin <= 1e-5).sum())} px within 1e-5)")
    assert err <= 1e-3 and lp_err <= 1e-3
    if precision == "fp32":
        assert int(diff.sum()) == 0
    else:
        # fp32x: measured 1 flip of 2,097,152 (an fp32 accumulation-order tie, oracle margin 4.8e-7)
        assert int(diff.sum()) <= 2 and not np.any(diff & (margin > 1e-5))


def test_headline_1024x2048_bf16_vs_oracle():
    """Config C2, the headline path itself: bf16 DRNSeg.segment (the seg_video loop bench.py times:
    uint8 frames -> labels, seg_video_old_no_plot.py:157-169, semantic_seg.py:445) on bench.py's
    seed-0 weights and both of its 1024x2048 parity frames vs the fp32 oracle.  Gates just above
    the measured flips (rounds 4-6: 2,309 of 4,194,304 labels differ, 99.945 %, mIoU vs ref 96.53;
    every bf16 tile change since is bit-identical, so a real regression shows as more flips)."""
    from drnmi import metrics
    from drnmi.drnseg import build
    from drnmi.weights import synth_frames
    m = build("drn_d_22", 19, seed=0, device=DEV, precision="bf16")
    frames = synth_frames(7, 2, 1024, 2048)
    lab = m.segment(torch.from_numpy(frames).to(DEV)).long()
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref = []
    for i in range(len(frames)):
        ref_lp, _, _ = O.drnseg_forward(sd, "drn_d_22", O.preprocess_u8(frames[i:i + 1]))
        ref.append(torch.max(ref_lp, 1)[1])
        del ref_lp
    ref = torch.cat(ref).to(DEV)
    agree = float((lab == ref).float().mean())
    hist = metrics.fast_hist(lab.flatten(), ref.flatten(), 19)
    miou = float(metrics.miou(hist.cpu().numpy()))
    print(f"headline D-22 2x1024x2048 bf16 segment: labels agree {agree:.6f} "
          f"({int((lab != ref).sum())} of {lab.numel()} differ), mIoU vs ref {miou:.2f}")
    assert int((lab != ref).sum()) <= 2600 and miou >= 96.3


@pytest.mark.parametrize("precision", ["fp32", "fp32x"])
def test_c4_d54_rmb75_finetune_step(golden_masks, precision):
    from drnmi.drnseg import DRNSeg
    from drnmi.pruners import RmbPruner
    from drnmi.train import SGD, CrossEntropyLoss
    from drnmi.weights import synth_state_dict
    m = DRNSeg("drn_d_54", 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, 3))        # the weights the golden RMB masks were cut from
    pr = RmbPruner(os.path.join(GOLDEN, "rmb_d54_8x8_75.json"), on_gpu=False)
    pr.generate_masks(m, is_static=False)
    _masks_match_golden(golden_masks, "rmb_d54_8x8", pr.mask_dict)
    masks = {k: v.float() for k, v in pr.mask_dict.items()}
    with torch.no_grad():
        sd = m.state_dict()
        for k, mk in masks.items():
            sd[k].mul_(mk)                           # semantic_seg.py:1063 apply before training
    g = torch.Generator().manual_seed(54)
    x = torch.randn(2, 3, 128, 128, generator=g)
    t = torch.randint(0, 19, (2, 128, 128), generator=g)
    t[torch.rand(t.shape, generator=g) < 0.2] = 255
    losses, g64, f64 = O.drnseg_train_steps(m.state_dict(), "drn_d_54", [x], [t], TC.LR, TC.MOMENTUM, TC.WD,
                                            masks=masks, dtype=torch.float64)
    m = m.to(DEV).train().set_precision(precision)
    for k in list(pr.mask_dict):
        pr.mask_dict[k] = pr.mask_dict[k].to(DEV)
    pr.on_gpu = True
    opt = SGD(m.optim_parameters(), TC.LR, momentum=TC.MOMENTUM, weight_decay=TC.WD, pruner=pr, model=m)
    loss = CrossEntropyLoss(ignore_index=255)(m(x.to(DEV))[0], t.to(DEV))
    opt.zero_grad()
    loss.backward()
    grads = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters() if p.grad is not None}
    opt.step()
    torch.cuda.synchronize()
    assert abs(float(loss) - losses[0]) <= 1e-4 * abs(losses[0])
    worst = 0.0
    for k, gr in grads.items():
        if k.startswith("up."):
            continue
        e = TC.rel_l2(gr.numpy(), g64[k].numpy())
        worst = max(worst, e)
        assert e <= 2e-2, (k, e)          # D-54 tolerance of test_gpu_train (ReLU-at-an-ulp flips)
    worst_p = 0.0
    for k, v in m.state_dict().items():
        if v.is_floating_point() and k in f64:
            e = TC.rel_err(v.detach().double().cpu().numpy(), f64[k].numpy())
            worst_p = max(worst_p, e)
            assert e <= 1e-4, (k, e)
    for k, mk in pr.mask_dict.items():
        w = m.state_dict()[k]
        assert torch.all(w[mk == 0] == 0), k
        assert abs(1 - int((w != 0).sum()) / w.numel() - 0.75) <= 0.01, k
    print(f"C4 D-54 + RMB 75 % step ({precision}): loss {float(loss):.6f} (fp64 {losses[0]:.6f}), grads rel-L2 vs fp64 "
          f"{worst:.2e}, params after the step {worst_p:.2e}")


def check_int8_launches(plan, n):
    """Re-check every int8 launch (and every bf16 -> int8 boundary) of a keep-all plan from its
    own HBM inputs against oracle/int8_oracle.py; returns the number of launches checked."""
    from drnmi import _lib as L
    pk = plan.packed
    for i, vals in pk.quant_after.items():
        for v in vals:
            src = plan.bufs[v].float().cpu().numpy()
            ref = Q.quantize_i8(src, np.float32(1.0 / pk.act_scales[v]))
            np.testing.assert_array_equal(plan.bufs["q:" + v].cpu().numpy(), ref)
    count = 0
    for nd in pk.graph.nodes:
        if not nd.i8:
            continue
        c = nd.conv
        ih, iw = plan.shapes[nd.src]
        oh, ow = plan.shapes[nd.dst]
        x = plan.bufs[nd.x_val].cpu().numpy().reshape(n, ih, iw, pk.cstride[nd.src])
        res = plan.bufs[nd.r_val].cpu().numpy().reshape(n, oh, ow, c.out_channels) if nd.r_val else None
        out = "f32" if nd.out_fp32_nchw else ("i8" if pk.value_code(nd.dst) == L.DRNMI_I8 else "bf16")
        ref = Q.conv_i8(x, nd.wpk.cpu().numpy(), nd.scale.cpu().numpy(), nd.shift.cpu().numpy(), c.out_channels,
                        c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0], nd.relu, res, nd.res_scale,
                        out, nd.out_scale)
        got = plan.bufs[nd.dst].cpu().numpy()
        if out == "f32":
            got = got.transpose(0, 2, 3, 1)
        elif out == "bf16":
            got = got.view(np.uint16).reshape(ref.shape)
        else:
            got = got.reshape(ref.shape)
        np.testing.assert_array_equal(got, ref, err_msg=nd.name)
        count += 1
    return count


def test_c5_d22_srmb50_int8(golden_masks):
    from drnmi import _lib as L
    from drnmi.drnseg import INFO_MEAN, INFO_STD, DRNSeg
    from drnmi.pruners import SRMBRepMasker
    from drnmi.weights import synth_frames, synth_state_dict
    m = DRNSeg("drn_d_22", 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, 0))
    np.random.seed(11)                               # the seed of the golden SRMB masks
    pr = SRMBRepMasker(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    pr.generate_masks(m)
    _masks_match_golden(golden_masks, "srmb_d22_seed11", pr.mask_dict)
    with torch.no_grad():
        sd = m.state_dict()
        for k, mk in pr.mask_dict.items():
            sd[k].mul_(mk)
    m = m.to(DEV).eval()
    frames = torch.from_numpy(synth_frames(57, 2, 128, 256)).to(DEV)
    calib = torch.from_numpy(synth_frames(58, 2, 128, 256)).to(DEV)
    m.set_precision("bf16").calibrate_int8(calib)
    m.set_precision("int8")
    n, h, w = frames.shape[:3]
    plan = m.plan(n, h, w, keep_all=True)
    stream = L.stream_ptr(torch.device(DEV))
    plan.ingest_u8(frames, INFO_MEAN, INFO_STD, False, stream)
    plan.run_backbone(stream)
    torch.cuda.synchronize()
    checked = check_int8_launches(plan, n)
    assert checked >= 10
    lab = m.segment(frames).long().cpu()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_lp, _, _ = O.drnseg_forward(sd, "drn_d_22", O.preprocess_u8(frames.cpu().numpy()))
    agree = float((lab == torch.max(ref_lp, 1)[1]).float().mean())
    m.set_precision("bf16")
    agree_bf16 = float((m.segment(frames).long().cpu() == torch.max(ref_lp, 1)[1]).float().mean())
    print(f"C5 D-22 + SRMB 50 % int8: {checked} int8 launches bit-exact; labels vs masked fp32 oracle "
          f"{agree:.4f} (bf16 {agree_bf16:.4f})")
    assert agree >= 0.93
