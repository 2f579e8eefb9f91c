"""The hash initialiser is the fixture contract: same seed -> same bits on every host."""
import numpy as np

from drnmi import weights as W


def test_splitmix_known_values():
    # splitmix64 of counters 0,1,2 (published reference sequence for seed 0 state advance)
    z = W.splitmix64(np.array([0, 1, 2], dtype=np.uint64))
    assert [hex(int(v)) for v in z] == ["0xe220a8397b1dcdaf", "0x910a2dec89025cc1", "0x975835de1c9756ce"]


def test_uniform_deterministic():
    a = W.uniform01(3, "layer.0.0.weight", 1000)
    b = W.uniform01(3, "layer.0.0.weight", 1000)
    c = W.uniform01(4, "layer.0.0.weight", 1000)
    np.testing.assert_array_equal(a, b)
    assert not np.array_equal(a, c)
    assert 0.0 <= a.min() and a.max() < 1.0
    assert abs(a.mean() - 0.5) < 0.05


def test_bilinear_kernel():
    w = W.bilinear_up_kernel(16)
    assert w.shape == (16, 16)
    # separable tent, peak 0.9375^2 at the two centre taps (7, 8)
    np.testing.assert_allclose(w[7, 7], (1 - abs(7 / 8 - 15 / 16)) ** 2, rtol=1e-6)
    np.testing.assert_allclose(w, w.T)


def test_state_dict_keys_match_reference_layout():
    from drnmi.drnseg import DRNSeg
    m = DRNSeg("drn_d_22", 19, pretrained=False)
    sd = W.synth_state_dict(m, 0)
    assert len(sd) == 153            # reference log.txt / SURVEY §8b: 153 entries for D-22
    assert "layer.3.0.downsample.0.weight" in sd and "up.weight" in sd and "seg.bias" in sd
    m.load_state_dict(sd)
