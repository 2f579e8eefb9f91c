"""Pins the oracle's fine-tune restatement (oracle/drn_oracle.drnseg_train_steps) to two
reference fine-tune steps (tests/golden/train.npz, made by make_golden.train_cases from the
reference's lmodels/drnseg.DRNSeg + nn.CrossEntropyLoss + torch.optim.SGD + BlockPruner).
CPU only."""
import numpy as np
import torch

import train_case as TC
from oracle import drn_oracle as O


def test_oracle_train_steps_match_reference():
    torch.set_num_threads(8)
    g = TC.load()
    m, pr = TC.model_and_masks(g)
    xs, ts = TC.inputs(g)
    masks = {k: v.float() for k, v in pr.mask_dict.items()}
    losses, grads, final = O.drnseg_train_steps(m.state_dict(), "drn_d_22", xs, ts, TC.LR, TC.MOMENTUM, TC.WD,
                                                masks=masks)
    np.testing.assert_allclose(losses, g[f"{TC.TAG}/losses"], rtol=1e-5)
    nchk = 0
    for k, v in final.items():
        key = f"{TC.TAG}/final/{k}"
        if key in g.files:
            assert TC.rel_err(TC.sample(v.float()).numpy(), g[key]) <= 1e-4, k
            nchk += 1
    for k, v in grads.items():
        key = f"{TC.TAG}/grad/{k}"
        assert key in g.files, k
        assert TC.rel_err(TC.sample(v).numpy(), g[key]) <= 1e-3, k
        s = g[f"{TC.TAG}/grad_sum/{k}"]
        assert abs(float(v.abs().sum()) - s[1]) <= 1e-3 * s[1], k
    assert nchk > 100
    # masked weights stay exactly zero after the steps
    for k, mk in masks.items():
        assert torch.all(final[k][mk == 0] == 0)
