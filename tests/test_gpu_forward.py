"""Whole-network parity: drnmi.DRNSeg (HIP engine) vs the reference goldens and the oracle.

north_star gate (fp32 parity mode): logits within 1e-3 max-abs of the reference PyTorch-CPU
forward; argmax label maps identical on EVERY pixel of the golden cases (measured: no pixel
differs; the pixels whose reference top-2 log-prob margin is <= 1e-4, where an fp32
reordering of the same sums could legitimately swap the order, are counted and reported).
bf16 perf mode: argmax agreement >= 0.98 and relative logit error <= 0.03 (measured
0.989-0.993 and ~1.2e-2 in round 1).
"""
import numpy as np
import pytest
import torch

from oracle import drn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = ["d22_1x64x128", "d22_2x128x256", "d38_1x64x128", "d54_1x64x128", "d22_1x300x300"]
ARCH = {"d22": "drn_d_22", "d38": "drn_d_38", "d54": "drn_d_54"}
_MODELS = {}


def model(case, golden):
    from drnmi.drnseg import build
    seed = int(golden[case + "/meta"][0])
    key = (case[:3], seed)
    if key not in _MODELS:
        _MODELS[key] = build(ARCH[case[:3]], 19, seed=seed, device=DEV)
    return _MODELS[key]


@pytest.mark.parametrize("case", CASES)
def test_fp32_forward_matches_reference(case, golden_forward):
    m = model(case, golden_forward).set_precision("fp32")
    x = torch.from_numpy(golden_forward[case + "/input"]).to(DEV)
    lp, logits = m(x)
    torch.cuda.synchronize()
    ref_logits = golden_forward[case + "/logits"]
    err = np.abs(logits.cpu().numpy() - ref_logits).max()
    assert err <= 1e-3, f"logit max-abs {err}"
    if case + "/logprobs" in golden_forward:
        assert np.abs(lp.cpu().numpy() - golden_forward[case + "/logprobs"]).max() <= 1e-3
    if case + "/logprobs_sub7" in golden_forward:
        assert np.abs(lp.cpu().numpy()[:, :, ::7, ::7] - golden_forward[case + "/logprobs_sub7"]).max() <= 1e-3
    labels = torch.max(lp, 1)[1].cpu().numpy()
    ref_lab = golden_forward[case + "/labels"]
    margin = golden_forward[case + "/top2_margin"]
    diff = labels != ref_lab
    print(f"{case}: logit max-abs {err:.2e}, labels differ {int(diff.sum())} px "
          f"({int((margin <= 1e-4).sum())} px with margin <= 1e-4)")
    assert int(diff.sum()) == 0, f"{int(diff.sum())} label mismatches"


@pytest.mark.parametrize("case", ["d22_2x128x256", "d54_1x64x128"])
def test_fp32_stages_match_oracle(case, golden_forward):
    """Per-stage taps (layer0..layer8) of a keep-all plan vs the oracle's stages."""
    m = model(case, golden_forward).set_precision("fp32")
    x = torch.from_numpy(golden_forward[case + "/input"])
    plan = m.plan(x.shape[0], x.shape[2], x.shape[3], keep_all=True)
    from drnmi import _lib
    plan.ingest_nchw(x.to(DEV), _lib.stream_ptr())
    plan.run_backbone(_lib.stream_ptr())
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    _, _, stages = O.drnseg_forward(sd, ARCH[case[:3]], x)
    for name, val in m._graph.stage_outputs.items():
        got = plan.stage_nchw(val).cpu()
        ref = stages[name]
        err = (got - ref).abs().max().item()
        assert err <= 1e-4 * max(1.0, ref.abs().max().item()), f"{name}: {err}"


@pytest.mark.parametrize("precision", ["fp32", "fp32x"])
def test_predict_and_segment_agree(golden_forward, precision):
    case = "d22_1x300x300"
    m = model(case, golden_forward).set_precision(precision)
    frames = torch.from_numpy(golden_forward[case + "/frames"]).to(DEV)
    x = torch.from_numpy(golden_forward[case + "/input"]).to(DEV)
    lab_pred = m.predict(x)
    lab_seg = m.segment(frames)
    m.set_precision("fp32")
    assert lab_seg.dtype == torch.uint8 and lab_seg.shape == (1, 304, 304)
    assert torch.equal(lab_pred.cpu(), lab_seg.cpu().long())
    assert torch.equal(lab_pred.cpu(), torch.from_numpy(golden_forward[case + "/labels"]).long())


@pytest.mark.parametrize("case", ["d22_2x128x256", "d38_1x64x128", "d54_1x64x128"])
def test_bf16_forward_agreement(case, golden_forward):
    m = model(case, golden_forward).set_precision("bf16")
    x = torch.from_numpy(golden_forward[case + "/input"]).to(DEV)
    lp, logits = m(x)
    m.set_precision("fp32")
    ref_logits = golden_forward[case + "/logits"]
    rel = np.abs(logits.cpu().numpy() - ref_logits).max() / np.abs(ref_logits).max()
    labels = torch.max(lp, 1)[1].cpu().numpy()
    agree = (labels == golden_forward[case + "/labels"]).mean()
    print(f"{case} bf16: logit rel err {rel:.3e}, argmax agreement {agree:.4f}")
    assert rel <= 0.03
    # just below the measured agreement (round 4: 0.9939 / 0.9919 / 0.9894): a regression that
    # doubles the mismatch rate fails
    assert agree >= {"d22_2x128x256": 0.990, "d38_1x64x128": 0.988, "d54_1x64x128": 0.985}[case]


def test_weights_repack_after_mask_apply(golden_forward, tmp_path):
    """apply_masks (in place via the C-ABI) must be seen by the next forward."""
    import json
    from drnmi import pruners as P
    from drnmi.drnseg import build
    m = build("drn_d_22", 19, seed=0, device=DEV)
    x = torch.from_numpy(golden_forward["d22_1x64x128/input"]).to(DEV)
    _, l0 = m(x)
    cfg = {"pruner_type": "block", "configs": [{"layer_set": ["layer.8.0.weight"], "sparsity": 0.9,
           "block_height": 1, "block_width": 1, "sub_rows": -1, "sub_cols": -1, "collapse_tensor": True}]}
    jp = tmp_path / "c.json"
    jp.write_text(json.dumps(cfg))
    pr = P.BlockPruner(str(jp))
    pr.generate_masks(m)
    pr.apply_masks(m)
    _, l1 = m(x)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    _, ref, _ = O.drnseg_forward(sd, "drn_d_22", x.cpu())
    assert (l1.cpu() - ref).abs().max().item() <= 1e-3
    assert (l1 - l0).abs().max().item() > 1e-3
    # the repack runs once per weight change, not on every later call (the repack key must be
    # the parameters' state, not a plan key)
    from drnmi.engine import PackedNet
    calls = []
    orig = PackedNet.pack
    PackedNet.pack = lambda self, *a, **k: (calls.append(1), orig(self, *a, **k))[1]
    try:
        for _ in range(3):
            m(x)
        assert not calls
        with torch.no_grad():
            m.seg.bias.add_(0.0)          # in-place: bumps the version counter
        for _ in range(3):
            m(x)
        assert len(calls) == 1
    finally:
        PackedNet.pack = orig


def test_bf16_segment_matches_bf16_forward_labels(golden_forward):
    """bf16 video path (fused u8 stem) vs bf16 NCHW path: same network, near-identical labels."""
    case = "d22_2x128x256"
    m = model(case, golden_forward).set_precision("bf16")
    frames = torch.from_numpy(golden_forward[case + "/frames"]).to(DEV)
    x = torch.from_numpy(golden_forward[case + "/input"]).to(DEV)
    lab_seg = m.segment(frames).long()
    lab_fwd = m.predict(x)
    m.set_precision("fp32")
    agree = (lab_seg == lab_fwd).float().mean().item()
    ref = torch.from_numpy(golden_forward[case + "/labels"]).long().to(DEV)
    agree_ref = (lab_seg == ref).float().mean().item()
    print(f"bf16 segment vs predict agreement {agree:.4f}, vs reference {agree_ref:.4f}")
    assert agree >= 0.99 and agree_ref >= 0.99        # measured 0.9938 / 0.9944


@pytest.mark.parametrize("case", CASES)
def test_fp32x_forward_matches_reference(case, golden_forward):
    """fp32x (fp32-accurate split-bf16 MFMA for every cin >= 32 conv): the fp32 gates."""
    m = model(case, golden_forward).set_precision("fp32x")
    x = torch.from_numpy(golden_forward[case + "/input"]).to(DEV)
    lp, logits = m(x)
    m.set_precision("fp32")
    torch.cuda.synchronize()
    err = np.abs(logits.cpu().numpy() - golden_forward[case + "/logits"]).max()
    labels = torch.max(lp, 1)[1].cpu().numpy()
    diff = int((labels != golden_forward[case + "/labels"]).sum())
    print(f"{case} fp32x: logit max-abs {err:.2e}, labels differ {diff} px")
    assert err <= 1e-3 and diff == 0


def test_fp32x_stages_match_oracle(golden_forward):
    case = "d54_1x64x128"
    m = model(case, golden_forward).set_precision("fp32x")
    x = torch.from_numpy(golden_forward[case + "/input"])
    plan = m.plan(x.shape[0], x.shape[2], x.shape[3], keep_all=True)
    from drnmi import _lib
    plan.ingest_nchw(x.to(DEV), _lib.stream_ptr())
    plan.run_backbone(_lib.stream_ptr())
    assert sum(nd.x6 for nd in plan.packed.graph.nodes) >= 40
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    _, _, stages = O.drnseg_forward(sd, "drn_d_54", x)
    for name, val in m._graph.stage_outputs.items():
        got = plan.stage_nchw(val).cpu()
        ref = stages[name]
        err = (got - ref).abs().max().item()
        assert err <= 1e-4 * max(1.0, ref.abs().max().item()), f"{name}: {err}"
    m.set_precision("fp32")
