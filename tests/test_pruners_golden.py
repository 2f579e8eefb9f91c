"""Mask generators reproduce the reference pruners bit-for-bit (CPU only).

Goldens: tests/golden/masks.npz from the reference's pruners/{SRMBRepMasker,BlockPruner,
RmbPruner}.py run in the build container (tests/golden/make_golden.py), same seeds."""
import hashlib
import json
import os

import numpy as np
import pytest

from drnmi import pruners as P

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def model_for(arch, seed):
    from drnmi.drnseg import DRNSeg
    from drnmi.weights import synth_state_dict
    m = DRNSeg(arch, 19, pretrained=False)
    m.load_state_dict(synth_state_dict(m, seed))
    return m


_MODELS = {}


def cached_model(arch, seed):
    if (arch, seed) not in _MODELS:
        _MODELS[(arch, seed)] = model_for(arch, seed)
    return _MODELS[(arch, seed)]


def sha(m):
    return hashlib.sha256(np.ascontiguousarray((m != 0).astype(np.uint8)).tobytes()).hexdigest()


def check(golden, tag, mask_dict):
    layers = list(golden[tag + "/layers"])
    assert list(mask_dict) == layers
    for layer in layers:
        m = mask_dict[layer].cpu().numpy()
        assert tuple(m.shape) == tuple(golden[f"{tag}/shape/{layer}"])
        assert int(np.count_nonzero(m)) == int(golden[f"{tag}/nnz/{layer}"]), layer
        key = f"{tag}/bits/{layer}"
        if key in golden:
            exp = np.unpackbits(golden[key])[:m.size]
            bad = np.nonzero(exp != (m.reshape(-1) != 0))[0]
            assert bad.size == 0, f"{layer}: {bad.size} mismatches, first {bad[:8]}"
        assert sha(m) == str(golden[f"{tag}/sha/{layer}"]), layer
        if int(golden[f"{tag}/dtype_is_f32/{layer}"]):
            assert m.dtype == np.float32


def write(tmp_path, name, obj):
    p = tmp_path / name
    p.write_text(json.dumps(obj))
    return str(p)


def test_srmb_shipped_config(golden_masks):
    np.random.seed(11)
    pr = P.SRMBRepMasker(os.path.join(GOLDEN, "srmb_d22_1024X768_50.json"), on_gpu=False)
    pr.generate_masks(cached_model("drn_d_22", 0))
    check(golden_masks, "srmb_d22_seed11", pr.mask_dict)


PATS = [("UROW", 0.75), ("CDIA", 0.5), ("CDIASTRIDE", 0.5), ("COLUMN", 0.5), ("CBAND", 0.5),
        ("CCDIA", 0.5), ("CCOLUMN", 0.75), ("GROUP", 0.5), ("RANDOM", 0.5), ("TRANS", 0.5),
        ("TRANS", 0.875), ("RAMANUJAN", 0.75)]


@pytest.mark.parametrize("pi", range(len(PATS)))
@pytest.mark.parametrize("rep", [True, False])
def test_srmb_patterns(pi, rep, golden_masks, tmp_path):
    pat, isp = PATS[pi]
    tag = f"srmb_{pat}{int(isp * 1000)}_{'rep' if rep else 'norep'}_seed{100 + pi}"
    c = json.loads(str(golden_masks[tag + "/config"]))
    jp = write(tmp_path, "c.json", {"pruner_type": "srmbrep", "configs": [c]})
    np.random.seed(100 + pi)
    pr = P.SRMBRepMasker(jp, on_gpu=False)
    pr.generate_masks(cached_model("drn_d_22", 0))
    check(golden_masks, tag, pr.mask_dict)


@pytest.mark.parametrize("tag,seed", [("srmb_nocollapse_seed7", 7), ("srmb_sym_seed8", 8)])
def test_srmb_variants(tag, seed, golden_masks, tmp_path):
    c = json.loads(str(golden_masks[tag + "/config"]))
    jp = write(tmp_path, "c.json", {"pruner_type": "srmbrep", "configs": [c]})
    np.random.seed(seed)
    pr = P.SRMBRepMasker(jp, on_gpu=False)
    pr.generate_masks(cached_model("drn_d_22", 0))
    check(golden_masks, tag, pr.mask_dict)


def test_block_d38_16x16(golden_masks):
    pr = P.BlockPruner(os.path.join(GOLDEN, "block_d38_16x16_50.json"), on_gpu=False)
    pr.generate_masks(cached_model("drn_d_38", 2), is_static=False)
    check(golden_masks, "block_d38_16x16", pr.mask_dict)


def test_block_sub_and_static(golden_masks):
    jp = os.path.join(GOLDEN, "block_d22_4x4_sub32.json")
    pr = P.BlockPruner(jp, on_gpu=False)
    pr.generate_masks(cached_model("drn_d_22", 0), is_static=False)
    check(golden_masks, "block_d22_4x4_sub32", pr.mask_dict)
    np.random.seed(5)
    pr = P.BlockPruner(jp, on_gpu=False)
    pr.generate_masks(cached_model("drn_d_22", 0), is_static=True)
    check(golden_masks, "block_d22_4x4_sub32_static_seed5", pr.mask_dict)


def test_block_elementwise(golden_masks):
    pr = P.BlockPruner(os.path.join(GOLDEN, "block_d22_1x1_75.json"), on_gpu=False)
    pr.generate_masks(cached_model("drn_d_22", 0))
    check(golden_masks, "block_d22_1x1_75", pr.mask_dict)


def test_block_ragged_sub_raises():
    w = np.random.RandomState(0).randn(16, 16, 3, 3).astype(np.float32)
    with pytest.raises(ValueError):
        P.BlockPruner.prune_tensor_as_block(w, 0.5, 4, 4, 32, 32, True)


@pytest.mark.parametrize("tag,cfg", [("rmb_d54_8x8", "rmb_d54_8x8_75.json"),
                                     ("rmb_d54_4x4_sp50", "rmb_d54_4x4_sp50.json")])
def test_rmb(tag, cfg, golden_masks):
    pr = P.RmbPruner(os.path.join(GOLDEN, cfg), on_gpu=False)
    pr.generate_masks(cached_model("drn_d_54", 3), is_static=True)   # is_static accepted, ignored
    check(golden_masks, tag, pr.mask_dict)
    if tag == "rmb_d54_8x8":
        for m in pr.mask_dict.values():
            assert abs(1 - np.count_nonzero(m.numpy()) / m.numel() - 0.75) < 1e-9


def test_bsr_dump_matches_reference(tmp_path):
    d = np.load(os.path.join(GOLDEN, "dumps.npz"), allow_pickle=False)
    mat = d["bsr/mat"]
    pc = P.BlockPrunerConfig(0.5, 2, 2, 4, 4, True)
    mask = P.BlockPruner.generate_mask_by_pruning(mat, pc)
    np.testing.assert_array_equal(mask.astype(np.uint8), d["bsr/mask"])
    bm = P.BlockPruner.generate_block_matrix(mat * mask, 2, 2)
    out = tmp_path / "bsr.txt"
    P.BlockPruner.write_block_matrix_to_file(bm, str(out))
    assert out.read_text() == open(os.path.join(GOLDEN, "bsr_8x8.txt")).read()


def test_reference_block_test_fixture_roundtrip(tmp_path):
    """pruners/block_test.txt (reference fixture): rebuild the dense matrix from its BSR,
    re-dump it with our writer -> byte-identical; 2 kept 2x2 blocks per 4x4 sub-matrix."""
    lines = open(os.path.join(GOLDEN, "block_test.txt")).read().split("\n")
    rows, cols, bh, bw, nnzb = (int(v) for v in lines[:5])
    vals = [int(v) for v in lines[5].split()]
    idx = [int(v) for v in lines[6].split()]
    ptr = [int(v) for v in lines[7].split()]
    dense = np.zeros((rows, cols), dtype=np.int64)
    for rb in range(rows // bh):
        for b in range(ptr[rb], ptr[rb + 1] if rb + 1 < len(ptr) else nnzb):
            blk = np.array(vals[b * bh * bw:(b + 1) * bh * bw]).reshape(bw, bh).T   # column-major
            dense[rb * bh:(rb + 1) * bh, idx[b] * bw:(idx[b] + 1) * bw] = blk
    bm = P.BlockPruner.generate_block_matrix(dense, bh, bw)
    out = tmp_path / "b.txt"
    P.BlockPruner.write_block_matrix_to_file(bm, str(out))
    assert out.read_text() == open(os.path.join(GOLDEN, "block_test.txt")).read()
    keep = (dense != 0).reshape(2, 4, 2, 4).any(axis=(1, 3))
    assert keep.shape == (2, 2)
    blocks = (dense != 0).reshape(4, 2, 4, 2).any(axis=(1, 3))
    for sr in range(2):
        for sc in range(2):
            assert blocks[2 * sr:2 * sr + 2, 2 * sc:2 * sc + 2].sum() == 2


def test_rmb_dump_matches_reference(tmp_path):
    d = np.load(os.path.join(GOLDEN, "dumps.npz"), allow_pickle=False)
    mat = d["rmb/mat"]
    rc = P.RmbPrunerConfig(4, 4, 0.5, [P.BlockletType(2, 2), P.BlockletType(1, 1)], [1, 1])
    out = tmp_path / "rmb.txt"
    mask = P.RmbPruner.prune_tensor_as_rmb(mat, rc, str(out))
    np.testing.assert_array_equal(mask.astype(np.uint8), d["rmb/mask"])
    assert out.read_text() == open(os.path.join(GOLDEN, "rmb_8x8.txt")).read()


def test_make_pruner_dispatch():
    assert isinstance(P.make_pruner(os.path.join(GOLDEN, "rmb_d54_8x8_75.json"), on_gpu=False), P.RmbPruner)
    assert isinstance(P.make_pruner(os.path.join(GOLDEN, "block_d22_1x1_75.json"), on_gpu=False),
                      P.BlockPruner)


def test_print_stats(capsys, tmp_path):
    pr = P.BlockPruner(os.path.join(GOLDEN, "block_d22_1x1_75.json"), on_gpu=False)
    pr.generate_masks(cached_model("drn_d_22", 0))
    pr.print_stats()
    out = capsys.readouterr().out.strip().split("\n")
    assert out[0].startswith("layer.2.0.weight sparsity = ")
