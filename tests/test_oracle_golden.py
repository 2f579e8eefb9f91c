"""Pins the CPU oracle (oracle/drn_oracle.py) to golden vectors produced by the
reference's own modules (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import drn_oracle as O

CASES = ["d22_1x64x128", "d22_2x128x256", "d38_1x64x128", "d54_1x64x128", "d22_1x300x300"]
ARCH = {"d22": "drn_d_22", "d38": "drn_d_38", "d54": "drn_d_54"}


def state_dict_for(case, golden):
    from drnmi.drnseg import DRNSeg
    from drnmi.weights import synth_state_dict
    seed = int(golden[case + "/meta"][0])
    m = DRNSeg(ARCH[case[:3]], 19, pretrained=False)
    return synth_state_dict(m, seed)


def test_preprocess_matches_reference(golden_forward):
    for case in CASES:
        frames = golden_forward[case + "/frames"]
        x = O.preprocess_u8(frames)
        np.testing.assert_array_equal(x.numpy(), golden_forward[case + "/input"])


@pytest.mark.parametrize("case", CASES)
def test_oracle_forward_matches_reference(case, golden_forward):
    torch.set_num_threads(8)
    sd = state_dict_for(case, golden_forward)
    x = torch.from_numpy(golden_forward[case + "/input"])
    lp, logits, stages = O.drnseg_forward(sd, ARCH[case[:3]], x)
    ref_logits = golden_forward[case + "/logits"]
    # Same ATen kernels on the same host give max-abs 0; allow CPU-ISA reassociation elsewhere.
    assert np.abs(logits.numpy() - ref_logits).max() <= 1e-5 * max(1.0, np.abs(ref_logits).max())
    labels = O.labels_of(lp).numpy().astype(np.uint8)
    margin = golden_forward[case + "/top2_margin"]
    diff = labels != golden_forward[case + "/labels"]
    assert not np.any(diff & (margin > 1e-4))
    if case + "/logprobs" in golden_forward:
        assert np.abs(lp.numpy() - golden_forward[case + "/logprobs"]).max() <= 1e-4
    if case + "/logprobs_sub7" in golden_forward:
        assert np.abs(lp.numpy()[:, :, ::7, ::7] - golden_forward[case + "/logprobs_sub7"]).max() <= 1e-4
    for k, v in stages.items():
        ref = golden_forward[case + "/stage_sum/" + k]
        got = v.double().sum().item()
        assert abs(got - ref[0]) <= 1e-4 * ref[1] + 1e-6


def test_fast_hist_known_answer():
    label = np.array([0, 0, 1, 1, 2, 2, 255, 1])
    pred = np.array([0, 1, 1, 1, 2, 0, 2, 2])
    h = O.fast_hist(pred, label, 3)
    np.testing.assert_array_equal(h, [[1, 1, 0], [0, 2, 1], [1, 0, 1]])
    iou = O.per_class_iu(h)
    np.testing.assert_allclose(iou, [1 / 3, 2 / 4, 1 / 3])
