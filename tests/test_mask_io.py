"""Compact on-disk masks: Pruner.save_masks / load_masks (CPU only).

The reference never persists masks (semantic_seg.py:1085-1092); the format here stores 1 bit
per weight in the word layout drnmi_mask_apply_bits_f32 reads, so a loaded pruner needs no
host repack.  Masks come from the shipped SRMB / BlockPruner configs on hash-initialised D-22."""
import os

import numpy as np
import pytest
import torch

from drnmi import pruners as P

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _model():
    from drnmi.drnseg import DRNSeg
    from drnmi.weights import synth_state_dict
    m = DRNSeg("drn_d_22", 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, 0))
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
    np.savez(tmp_path / "c.npz", format=np.array([P.MASK_FORMAT_VERSION]), layers=np.array(["w"]),
             bits0=np.zeros(3, np.uint32), shape0=np.array([16, 16, 3, 3]), dtype0=np.array(["float32"]))
    pr = P.make_pruner(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    with pytest.raises(ValueError):
        pr.load_masks(tmp_path / "c.npz")
