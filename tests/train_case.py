"""Shared setup of the golden fine-tune case (tests/golden/train.npz, make_golden.train_cases):
D-22, hash weights seed 11, BlockPruner masks from tests/golden/block_d22_4x4_sub32.json
(drnmi's generator, bit-identical to the reference's — checked against the stored sha)."""
import hashlib
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TAG = "d22_train"
LR, MOMENTUM, WD = 0.001, 0.9, 1e-4


def load():
    return np.load(os.path.join(GOLDEN, "train.npz"), allow_pickle=False)


def inputs(g):
    xs = [torch.from_numpy(g[f"{TAG}/x{i}"]) for i in range(2)]
    ts = []
    for i in range(2):
        t = torch.from_numpy(g[f"{TAG}/t{i}"].astype(np.int64))
        ts.append(t)
    return xs, ts


def model_and_masks(g):
    """(DRNSeg on CPU with the golden's initial weights, masks dict {key: fp32 tensor})."""
    from drnmi.drnseg import DRNSeg
    from drnmi.pruners import BlockPruner
    from drnmi.weights import synth_state_dict
    seed = int(g[f"{TAG}/meta"][0])
    m = DRNSeg("drn_d_22", 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, seed))
    pr = BlockPruner(os.path.join(GOLDEN, "block_d22_4x4_sub32.json"), on_gpu=False)
    pr.generate_masks(m, is_static=False)
    for k, mk in pr.mask_dict.items():
        sha = hashlib.sha256(np.ascontiguousarray((mk.numpy() != 0).astype(np.uint8)).tobytes()).hexdigest()
        assert sha == str(g[f"{TAG}/mask_sha/{k}"]), k
    with torch.no_grad():
        sd = m.state_dict()
        for k, mk in pr.mask_dict.items():
            sd[k].mul_(mk)
    return m, pr


def sample(v):
    v = v.reshape(-1)
    return v[::97][:256] if v.numel() > 4096 else v


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def rel_l2(a, b):
    """||a - b||_2 / ||b||_2 — the gradient metric: a ReLU whose pre-activation lies within an
    ulp of zero can take either side in two fp32 implementations (or fp32 vs fp64), changing
    that element's gradient path by O(1); such isolated flips dominate a max-abs metric but
    not the norm."""
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
