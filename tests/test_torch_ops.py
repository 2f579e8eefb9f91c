"""torch.ops.drnmi custom-op registration (CPU-only checks: no kernel launches).

The real kernels are registered for the ROCm ("cuda") device only; the fake kernels give the
dispatcher (FakeTensorMode, torch.compile tracing) output shapes without a GPU."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from drnmi import torch_ops  # noqa: F401  (registers the ops)
from drnmi.drnseg import DRNSeg

OPS = ["conv2d_bn_act", "up8_logsoftmax_argmax", "mask_apply_", "segment", "forward", "predict"]


def test_ops_registered():
    for name in OPS:
        assert hasattr(torch.ops.drnmi, name), name


@pytest.mark.parametrize("arch,h,w,oh,ow", [("drn_d_22", 300, 300, 304, 304), ("drn_d_22", 1024, 2048, 1024, 2048),
                                            ("drn_d_38", 64, 128, 64, 128), ("drn_d_54", 97, 61, 104, 64)])
def test_fake_shapes_whole_network(arch, h, w, oh, ow):
    m = DRNSeg(arch, 19, pretrained=False).eval()
    with FakeTensorMode():
        lab = torch.ops.drnmi.segment(torch.empty(2, h, w, 3, dtype=torch.uint8, device="cuda"), m._handle,
                                      [0.3, 0.3, 0.3], [0.2, 0.2, 0.2], False)
        lp, logits = torch.ops.drnmi.forward(torch.empty(1, 3, h, w, device="cuda"), m._handle)
        pred = torch.ops.drnmi.predict(torch.empty(1, 3, h, w, device="cuda"), m._handle)
    assert lab.shape == (2, oh, ow) and lab.dtype == torch.uint8
    assert lp.shape == (1, 19, oh, ow) and logits.shape == (1, 19, oh // 8, ow // 8)
    assert pred.shape == (1, oh, ow) and pred.dtype == torch.int64


def test_fake_shapes_kernels():
    with FakeTensorMode():
        x = torch.empty(2, 33, 17, 64, dtype=torch.bfloat16, device="cuda")
        w = torch.empty(128, 576, dtype=torch.bfloat16, device="cuda")
        y = torch.ops.drnmi.conv2d_bn_act(x, w, None, torch.empty(128, device="cuda"), None, 128, 3, 2, 1, 1,
                                          True, False)
        seg = torch.ops.drnmi.conv2d_bn_act(x, torch.empty(128, 64, dtype=torch.bfloat16, device="cuda"), None,
                                            torch.empty(128, device="cuda"), None, 19, 1, 1, 0, 1, False, True)
        lab, lp = torch.ops.drnmi.up8_logsoftmax_argmax(torch.empty(2, 19, 5, 7, device="cuda"),
                                                        torch.empty(16, 16, device="cuda"), True, True)
        lab2, lp2 = torch.ops.drnmi.up8_logsoftmax_argmax(torch.empty(2, 19, 5, 7, device="cuda"),
                                                          torch.empty(16, 16, device="cuda"), False, False)
    assert y.shape == (2, 17, 9, 128) and y.dtype == torch.bfloat16
    assert seg.shape == (2, 19, 33, 17) and seg.dtype == torch.float32
    assert lab.shape == (2, 40, 56) and lab.dtype == torch.uint8 and lp.shape == (2, 19, 40, 56)
    assert lab2.dtype == torch.int64 and lp2.numel() == 0


def test_cpu_tensors_have_no_kernel():
    m = DRNSeg("drn_d_22", 19, pretrained=False).eval()
    with pytest.raises(RuntimeError, match="HIP engine only"):
        m(torch.zeros(1, 3, 64, 64))
    with pytest.raises(RuntimeError, match="HIP engine only"):
        m.segment(torch.zeros(1, 64, 64, 3, dtype=torch.uint8))
    with pytest.raises(NotImplementedError):     # no CPU kernel registered for the raw op
        torch.ops.drnmi.mask_apply_([torch.zeros(4)], [torch.ones(4)])


def test_use_torch_up_matches_reference_structure():
    """DRNSeg(use_torch_up=True): the reference's nn.UpsamplingBilinear2d head has no weight
    (lmodels/drnseg.py:285-287), so the state_dict is the convT model's minus up.weight."""
    a = DRNSeg("drn_d_22", 19, pretrained=False)
    b = DRNSeg("drn_d_22", 19, pretrained=False, use_torch_up=True)
    assert set(a.state_dict()) - set(b.state_dict()) == {"up.weight"}
    assert isinstance(b.up, torch.nn.UpsamplingBilinear2d) and b.up.scale_factor == 8
    assert [p is q for p, q in zip(a.optim_parameters(), a.optim_parameters())]
    assert len(list(b.optim_parameters())) == len(list(a.optim_parameters()))


def test_copies_get_their_own_handle():
    """the op handle must follow the instance -- a deepcopy / unpickled DRNSeg
    dispatches to ITS weights, never the original's."""
    import copy
    import pickle
    m = DRNSeg("drn_d_22", 19, pretrained=False).eval()
    for c in (copy.deepcopy(m), pickle.loads(pickle.dumps(m))):
        assert c._handle != m._handle
        assert torch_ops._model(c._handle) is c
        assert torch_ops._model(m._handle) is m
        assert c._graph.nodes[0].conv is c.layer[0][0]           # the lowered graph follows the copy
        assert c._packed == {} and c._plans == {}


def test_repack_key_sees_swapped_parameters():
    m = DRNSeg("drn_d_22", 19, pretrained=False).eval()
    k0 = m._state_key()
    assert m._state_key() == k0
    m.layer[0][0].weight = torch.nn.Parameter(torch.zeros_like(m.layer[0][0].weight))
    k1 = m._state_key()
    assert k1 != k0
    with torch.no_grad():
        m.seg.bias.add_(1.0)                                       # in-place: version bump
    assert m._state_key() != k1


def test_eval_unwraps_data_parallel():
    from drnmi.evaluate import _unwrap
    m = DRNSeg("drn_d_22", 19, pretrained=False)
    wrapped = torch.nn.DataParallel(m)
    assert _unwrap(wrapped) is m and _unwrap(m) is m
