"""Compact on-disk masks: Pruner.save_masks / load_masks (CPU only).

The reference never persists masks (semantic_seg.py:1085-1092); the format here stores 1 bit
per weight in the word layout drnmi_mask_apply_bits_f32 reads, so a loaded pruner needs no
host repack.  Masks come from the shipped SRMB / BlockPruner configs on hash-initialised D-22."""
import json
import os

import numpy as np
import pytest
import torch

from drnmi import pruners as P

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _model(seed=0):
    from drnmi.drnseg import DRNSeg
    from drnmi.weights import synth_state_dict
    m = DRNSeg("drn_d_22", 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, seed))
    return m


@pytest.mark.parametrize("cfg", ["srmb_d22_1024X768_50.json", "block_d22_4x4_sub32.json"])
def test_roundtrip_bit_exact(tmp_path, cfg):
    np.random.seed(7)
    pr = P.make_pruner(os.path.join(GOLDEN, cfg), on_gpu=False)
    pr.generate_masks(_model())
    path = tmp_path / "masks.npz"
    pr.save_masks(path)
    back = P.make_pruner(os.path.join(GOLDEN, cfg), on_gpu=False).load_masks(path)
    assert list(back.mask_dict) == list(pr.mask_dict)
    n_weights = 0
    for k, m in pr.mask_dict.items():
        b = back.mask_dict[k]
        assert b.dtype == m.dtype and b.shape == m.shape
        assert torch.equal(b, m), k
        n_weights += m.numel()
    # 1 bit per weight (+ npz framing); the fp32 masks are 32 bits per weight
    assert os.path.getsize(path) <= n_weights / 8 * 1.05 + 4096


def test_bits_match_apply_kernel_layout():
    """The stored words are exactly what apply_masks uploads (bit i%32 of word i//32)."""
    rng = np.random.default_rng(3)
    flat = rng.random(1000) < 0.3
    words = P._pack_bits(flat)
    assert words.dtype == np.uint32 and words.size == 32
    for i in (0, 1, 31, 32, 63, 500, 999):
        assert bool((words[i // 32] >> (i % 32)) & 1) == bool(flat[i])
    assert np.array_equal(P._unpack_bits(words, flat.size), flat)


def test_rejects_non_binary_mask(tmp_path):
    pr = P.make_pruner(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    pr.mask_dict["layer.1.0.weight"] = torch.full((16, 16, 3, 3), 0.5)
    with pytest.raises(ValueError):
        pr.save_masks(tmp_path / "bad.npz")


def test_rejects_corrupt_word_count(tmp_path):
    np.savez(tmp_path / "c.npz", format=np.array([1]), layers=np.array(["w"]),
             bits0=np.zeros(3, np.uint32), shape0=np.array([16, 16, 3, 3]), dtype0=np.array(["float32"]))
    pr = P.make_pruner(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    with pytest.raises(ValueError):
        pr.load_masks(tmp_path / "c.npz")


def test_srmb_masks_saved_as_period_tiles(tmp_path):
    """SRMB masks persist as their Kronecker factors (OB, period tile P): bit-identical round trip
    and a file far smaller than even the 1-bit flat form."""
    import numpy as np
    from drnmi import pruners as P
    m = _model()
    np.random.seed(11)
    pr = P.SRMBRepMasker(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    pr.generate_masks(m)
    fac = tmp_path / "srmb.npz"
    pr.save_masks(str(fac))
    with np.load(str(fac)) as z:
        kinds = set(int(k) for k in z["meta"][:, 0])
    assert kinds == {1}                   # every layer stored as (OB, period tile P)
    assert os.path.getsize(fac) < 8192
    flat = tmp_path / "flat.npz"
    pr2 = P.SRMBRepMasker(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    pr2.mask_dict = pr.mask_dict          # no factors: flat bits
    pr2.save_masks(str(flat))
    assert os.path.getsize(fac) * 5 < os.path.getsize(flat)
    back = P.SRMBRepMasker(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False).load_masks(str(fac))
    assert list(back.mask_dict) == list(pr.mask_dict)
    for k in pr.mask_dict:
        assert back.mask_dict[k].dtype == pr.mask_dict[k].dtype
        assert torch.equal(back.mask_dict[k], pr.mask_dict[k]), k
    # a mask edited after generation no longer matches its factors: stored as flat bits
    pr.mask_dict[k] = pr.mask_dict[k].clone()
    pr.mask_dict[k].view(-1)[0] = 1 - pr.mask_dict[k].view(-1)[0]
    pr.save_masks(str(fac))
    back = P.SRMBRepMasker(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False).load_masks(str(fac))
    assert torch.equal(back.mask_dict[k], pr.mask_dict[k])


def test_srmb_non_repetitive_factors(tmp_path):
    import numpy as np
    from drnmi import pruners as P
    m = _model()
    cfg = {"pruner_type": "srmbrep", "configs": [{"layer_set": ["layer.5.0.conv2.weight", "layer.6.0.conv1.weight"],
           "obh": 64, "obw": 64, "cbh": 32, "cbw": 32, "ibh": 1, "ibw": 1, "osp": 0.5, "opat": "RANDOM",
           "isp": 0.75, "ipat": "UROW", "is_repetitive": False, "collapse_tensor": True, "cross_prob": 0.5,
           "is_symmetric": False}]}
    path = tmp_path / "c.json"
    path.write_text(json.dumps(cfg))
    np.random.seed(3)
    pr = P.SRMBRepMasker(str(path), on_gpu=False)
    pr.generate_masks(m)
    f = tmp_path / "m.npz"
    pr.save_masks(str(f))
    back = P.SRMBRepMasker(str(path), on_gpu=False).load_masks(str(f))
    for k in pr.mask_dict:
        assert torch.equal(back.mask_dict[k], pr.mask_dict[k])


def test_checkpoint_carries_masks(tmp_path):
    """save_checkpoint / resume (semantic_seg.py:286-290, :973-990) with the pruner's masks."""
    import numpy as np
    from drnmi import pruners as P
    from drnmi.checkpoint import mask_path, resume, save_checkpoint
    m = _model()
    np.random.seed(11)
    pr = P.SRMBRepMasker(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    pr.generate_masks(m)
    opt = torch.optim.SGD(m.optim_parameters(), 0.01, momentum=0.9)
    state = {"epoch": 3, "arch": "drn_d_22", "state_dict": m.state_dict(), "best_miou": 12.5,
             "optimizer": opt.state_dict(), "dataset": "cityscapes"}
    save_checkpoint(state, True, str(tmp_path), pruner=pr)
    assert os.path.exists(tmp_path / "checkpoint_best.pth.tar")
    assert os.path.exists(mask_path(str(tmp_path / "checkpoint_best.pth.tar")))
    m2 = _model(seed=9)
    pr2 = P.SRMBRepMasker(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    st = resume(str(tmp_path / "checkpoint_best.pth.tar"), m2, torch.optim.SGD(m2.optim_parameters(), 0.01,
                                                                               momentum=0.9), pr2)
    assert st["epoch"] == 3 and st["best_miou"] == 12.5
    for k, v in m.state_dict().items():
        assert torch.equal(m2.state_dict()[k], v), k
    for k in pr.mask_dict:
        assert torch.equal(pr2.mask_dict[k], pr.mask_dict[k])
