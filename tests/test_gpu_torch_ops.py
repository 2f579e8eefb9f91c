"""torch.ops.drnmi custom ops on the GPU: bit-exact against the direct C-ABI (ctypes) path,
torch.cuda.graph capture of segment() replays bit-exactly, and the use_torch_up head
(nn.UpsamplingBilinear2d(8), lmodels/drnseg.py:285-287) forward + fine-tune backward vs the
oracle."""
import ctypes

import numpy as np
import pytest
import torch

import train_case as TC
from drnmi import torch_ops  # noqa: F401  (registers torch.ops.drnmi.* for tests run on their own)
from oracle import drn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_conv_op_matches_capi():
    from drnmi import ops
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(2, 20, 28, 256, device=DEV, generator=g).to(torch.bfloat16)
    wt = torch.randn(256, 256, 3, 3, device=DEV, generator=g) * 0.02
    sc = torch.rand(256, device=DEV, generator=g) + 0.5
    sh = torch.randn(256, device=DEV, generator=g)
    res = torch.randn(2, 20, 28, 256, device=DEV, generator=g).to(torch.bfloat16)
    ref = ops.conv2d_bn_act(x, wt, sc, sh, res, stride=1, padding=2, dilation=2, relu=True)
    wpk, _ = ops.pack_conv_weight(wt, 256, torch.bfloat16)
    scp = torch.ones(wpk.shape[0], device=DEV)
    shp = torch.zeros(wpk.shape[0], device=DEV)
    scp[:256], shp[:256] = sc, sh
    got = torch.ops.drnmi.conv2d_bn_act(x, wpk, scp, shp, res, 256, 3, 1, 2, 2, True, False)
    assert torch.equal(got, ref)


def test_up8_and_mask_ops_match_capi():
    from drnmi import ops
    from drnmi.weights import bilinear_up_kernel
    g = torch.Generator(device=DEV).manual_seed(6)
    logits = torch.randn(2, 19, 9, 13, device=DEV, generator=g) * 4
    up = torch.from_numpy(bilinear_up_kernel(16)).to(DEV)
    lp_ref, lab_ref = ops.up8_logsoftmax_argmax(logits, up, True, torch.int64)
    lab, lp = torch.ops.drnmi.up8_logsoftmax_argmax(logits, up, True, False)
    assert torch.equal(lab, lab_ref) and torch.equal(lp, lp_ref)
    lab8, lp0 = torch.ops.drnmi.up8_logsoftmax_argmax(logits, up, False, True)
    assert lp0.numel() == 0 and torch.equal(lab8.long(), lab_ref)
    w = [torch.randn(64, 32, 3, 3, device=DEV, generator=g), torch.randn(19, 512, 1, 1, device=DEV, generator=g)]
    m = [(torch.rand(t.shape, device=DEV, generator=g) > 0.5).float() for t in w]
    expect = [a * b for a, b in zip(w, m)]
    torch.ops.drnmi.mask_apply_(w, m)
    assert all(torch.equal(a, b) for a, b in zip(w, expect))


@pytest.mark.parametrize("precision", ["bf16", "fp32", "fp32x"])
def test_segment_op_and_graph_capture(precision):
    from drnmi.drnseg import build
    from drnmi.weights import synth_frames
    m = build("drn_d_22", 19, seed=1, device=DEV, precision=precision)
    frames = torch.from_numpy(synth_frames(9, 2, 128, 256)).to(DEV)
    eager = m._segment_impl(frames, (0.29, 0.33, 0.29), (0.18, 0.19, 0.18), False, None)
    via_op = m.segment(frames, (0.29, 0.33, 0.29), (0.18, 0.19, 0.18))
    assert torch.equal(via_op, eager)
    lp, logits = m(torch.randn(1, 3, 64, 128, device=DEV))
    lp2, logits2 = m._forward_impl(torch.zeros(1, 3, 64, 128, device=DEV) + 0)   # plan reuse, no error
    assert lp.shape == lp2.shape and logits.shape == logits2.shape
    # capture the whole video step in a HIP graph (warm-up on a side stream first: packing,
    # plan buffers and kernel attributes are set up outside the capture)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            m.segment(frames)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        captured = m.segment(frames)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(captured, m.segment(frames))
    frames.copy_(torch.from_numpy(synth_frames(10, 2, 128, 256)).to(DEV))   # new input, same buffer
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(captured, m.segment(frames))


def _torch_up_model(seed):
    from drnmi.drnseg import DRNSeg
    from drnmi.weights import synth_state_dict
    m = DRNSeg("drn_d_22", 19, pretrained=False, use_torch_up=True)
    m.load_state_dict(synth_state_dict(m, seed))
    return m


@pytest.mark.parametrize("shape", [(1, 3, 64, 128), (2, 3, 72, 40)])
def test_use_torch_up_forward_vs_oracle(shape):
    m = _torch_up_model(2).to(DEV).eval()
    g = torch.Generator().manual_seed(8)
    x = torch.randn(*shape, generator=g)
    lp, logits = m(x.to(DEV))
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_lp, ref_logits, _ = O.drnseg_forward(sd, "drn_d_22", x)
    assert lp.shape == ref_lp.shape
    e_lg = (logits.cpu() - ref_logits).abs().max().item()
    e_lp = (lp.cpu() - ref_lp).abs().max().item()
    diff = int((torch.max(lp, 1)[1].cpu() != torch.max(ref_lp, 1)[1]).sum())
    print(f"use_torch_up {shape}: logits {e_lg:.2e}, log-probs {e_lp:.2e}, label mismatches {diff}")
    assert e_lg <= 1e-3 and e_lp <= 1e-3 and diff == 0
    assert torch.equal(m.predict(x.to(DEV)), torch.max(lp, 1)[1])


def test_use_torch_up_train_step_vs_oracle():
    from drnmi.train import CrossEntropyLoss
    m = _torch_up_model(4)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(1, 3, 72, 40, generator=g)
    t = torch.randint(0, 19, (1, 72, 40), generator=g)
    t[torch.rand(t.shape, generator=g) < 0.2] = 255
    losses, g64, _ = O.drnseg_train_steps(m.state_dict(), "drn_d_22", [x], [t], 0.0, 0.0, 0.0,
                                          dtype=torch.float64)
    m = m.to(DEV).train()
    lp, logits = m(x.to(DEV))
    loss = CrossEntropyLoss(ignore_index=255)(lp, t.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - losses[0]) <= 1e-4 * abs(losses[0])
    worst = 0.0
    for k, p in m.named_parameters():
        e = TC.rel_l2(p.grad.detach().double().cpu().numpy(), g64[k].numpy())
        worst = max(worst, e)
        assert e <= 1e-3, (k, e)
    print(f"use_torch_up train step: worst grad rel-L2 vs fp64 {worst:.2e}")


def test_bilinear_bwd_kernel_vs_autograd():
    """drnmi_up8_bilinear_lsm_bwd_f32 vs torch-CPU fp32 autograd of interpolate + log_softmax,
    both the log-prob and the logits-only gradient paths, with grad_scale."""
    import torch.nn.functional as F
    from drnmi import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(3)
    for (h, w) in [(6, 9), (1, 3), (2, 2)]:
        logits = (torch.randn(2, 19, h, w, generator=g) * 3).requires_grad_(True)
        lp = F.log_softmax(F.interpolate(logits, scale_factor=8, mode="bilinear", align_corners=True), 1)
        g_lp = torch.randn(lp.shape, generator=g)
        g_lg = torch.randn(logits.shape, generator=g)
        scale = 0.5
        (gref,) = torch.autograd.grad((lp * g_lp).sum() * scale + (logits * g_lg).sum() * scale, logits)
        lpd, glpd, glgd = lp.detach().to(DEV), g_lp.to(DEV), g_lg.to(DEV)
        du = torch.empty_like(lpd)
        out = torch.empty(logits.shape, device=DEV)
        vp = lambda t: ctypes.c_void_p(t.data_ptr())
        _lib.check(lib.drnmi_up8_bilinear_lsm_bwd_f32(vp(glpd), vp(lpd), vp(glgd), scale, 2, 19, h, w, vp(du),
                                                      vp(out), ctypes.c_void_p(_lib.stream_ptr())), "bwd")
        torch.cuda.synchronize()
        np.testing.assert_allclose(out.cpu().numpy(), gref.numpy(), rtol=1e-4, atol=1e-4)


def test_deepcopy_dispatches_to_its_own_weights():
    """a deepcopy with different weights gives different logits (and the original's
    are unchanged)."""
    import copy
    from drnmi.drnseg import build
    m = build("drn_d_22", 19, seed=0, device="cuda", precision="fp32")
    x = torch.rand(1, 3, 64, 128, device="cuda")
    _, l0 = m(x)
    c = copy.deepcopy(m)
    _, lc = c(x)
    assert torch.equal(l0, lc)
    with torch.no_grad():
        c.seg.bias.add_(1.0)
    _, lc2 = c(x)
    _, l1 = m(x)
    assert torch.equal(l1, l0)
    assert torch.allclose(lc2, l0 + 1.0, atol=1e-5)
