"""Block-sparse MFMA path (north_star: "MFMA used only on the dense-within-block sub-tiles of the
block-sparse weights"): K steps whose weight slice is all zero for a whole output-channel tile
(pruned blocks covering the tile's rows) are dropped -- no weight DMA, no pixel gather, no MFMA.
Parity gate: the sparse launch is BIT-IDENTICAL to the dense kernel on the same (masked) weights
-- a dropped step only ever contributed exact zeros -- and the masked model matches the oracle
like any dense one."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import drn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def pruned_model(arch, seed, cfg):
    from drnmi.drnseg import DRNSeg
    from drnmi.pruners import BlockPruner
    from drnmi.weights import synth_state_dict
    m = DRNSeg(arch, 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, seed))
    path = os.path.join("/tmp", f"sparse_cfg_{os.getpid()}.json")
    with open(path, "w") as f:
        json.dump(cfg, f)
    pr = BlockPruner(path, on_gpu=False)
    pr.generate_masks(m, is_static=False)
    with torch.no_grad():
        sd = m.state_dict()
        for k, mk in pr.mask_dict.items():
            sd[k].mul_(mk)
    return m.to(DEV).eval()


def conv_layers(m, min_cin=16, bh=16, bw=1):
    return [k for k, v in m.state_dict().items() if k.startswith("layer.") and k.endswith(".weight")
            and v.dim() == 4 and v.shape[1] >= min_cin and v.shape[0] % bh == 0 and v.shape[1] % bw == 0]


def block_cfg(m, bh, bw, sp):
    return {"pruner_type": "block", "configs": [{"layer_set": conv_layers(m, bh=bh, bw=bw), "sparsity": sp,
                                                 "block_height": bh,
                                                 "block_width": bw, "sub_rows": -1, "sub_cols": -1,
                                                 "collapse_tensor": False}]}


@pytest.mark.parametrize("arch,bh,bw,shape", [("drn_d_38", 16, 16, (2, 3, 128, 256)),
                                              ("drn_d_22", 16, 32, (1, 3, 256, 256)),
                                              ("drn_d_38", 256, 64, (2, 3, 128, 256)),
                                              ("drn_d_22", 128, 64, (1, 3, 200, 264))])
def test_sparse_bit_identical_to_dense(arch, bh, bw, shape, monkeypatch):
    from drnmi.drnseg import DRNSeg
    probe = DRNSeg(arch, 19, pretrained=False)
    m = pruned_model(arch, 2, block_cfg(probe, bh, bw, 0.5))
    m.set_precision("bf16")
    from drnmi import engine
    monkeypatch.setattr(engine, "SPARSE_MIN_ZERO_UNITS", 0.05)   # every layer with any zero unit
    monkeypatch.setattr(engine, "FUSE_DOWNSAMPLE", False)        # same launch structure both ways
    x = torch.randn(*shape).to(DEV)
    m.set_block_sparse(True)
    lp_s, lg_s = m(x)
    plan = m.plan(*shape[:1], shape[2], shape[3])
    nodes = m._packed["bf16"].graph.nodes
    frac = {nd.name: round(nd.zero_unit_frac, 3) for nd in nodes if nd.unit_mask is not None}
    assert frac, "no layer took the block-sparse path"
    m.set_block_sparse(False)
    lp_d, lg_d = m(x)
    torch.cuda.synchronize()
    assert torch.equal(lg_s, lg_d) and torch.equal(lp_s, lp_d)
    print(f"{arch} {bh}x{bw}: {len(frac)} sparse layers, zero-unit fractions {sorted(set(frac.values()))}")
    # the masked model in fp32 parity mode still matches the oracle
    m.set_precision("fp32")
    lp, lg = m(x)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    _, ref, _ = O.drnseg_forward(sd, arch, x.cpu())
    assert (lg.cpu() - ref).abs().max().item() <= 1e-3


def test_unit_mask_matches_numpy():
    import ctypes
    from drnmi import _lib
    lib = _lib.load()
    torch.manual_seed(0)
    rows, kp = 256, 4608
    w = torch.randn(rows, kp)
    keep = torch.rand(rows // 16, kp // 32) < 0.4
    w = w * keep.repeat_interleave(16, 0).repeat_interleave(32, 1)
    w[5, 7] = -0.0       # negative zero counts as zero
    wb = w.to(torch.bfloat16).to(DEV)
    wpr = (kp + 1023) // 1024
    mask = torch.empty((rows // 16) * wpr, dtype=torch.int32, device=DEV)
    cnt = torch.empty(1, dtype=torch.int32, device=DEV)
    _lib.check(lib.drnmi_weight_unit_mask(wb.data_ptr(), _lib.DRNMI_BF16, rows, kp, mask.data_ptr(), cnt.data_ptr(),
                                          ctypes.c_void_p(_lib.stream_ptr())), "unit_mask")
    words = mask.cpu().numpy().view(np.uint32).reshape(rows // 16, wpr)
    got = np.zeros((rows // 16, kp // 32), dtype=bool)
    for ku in range(kp // 32):
        got[:, ku] = (words[:, ku // 32] >> (ku % 32)) & 1
    np.testing.assert_array_equal(got, keep.numpy())
    assert int(cnt.item()) == int(keep.sum())
