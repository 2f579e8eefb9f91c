"""W8A8 path (BASELINE config C5): int8 conv launches and the int8 quantiser, bit for bit
against oracle/int8_oracle.py, and the int8 network against the reference goldens.

The reference has no quantisation code, so the int8 scheme is ours ("parity unpinned" vs the
reference): the gates are (1) exact arithmetic parity of every int8 launch with the numpy
restatement on the launch's own inputs, (2) label agreement of the int8 network with the
reference fp32 forward (tests/golden/forward.npz).
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import int8_oracle as Q

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib():
    from drnmi import _lib
    return _lib, _lib.load()


def _stream():
    from drnmi import _lib
    return ctypes.c_void_p(_lib.stream_ptr(torch.device(DEV)))


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_quantize_i8_exact(dtype):
    L, lib = _lib()
    g = torch.Generator(device=DEV).manual_seed(3)
    n = 8 * 12347
    x = torch.randn(n, device=DEV, generator=g) * 3.0
    x[:8] = torch.tensor([0.5, 1.5, 2.5, -0.5, -1.5, 300.0, -300.0, 0.0])   # ties and clamps
    x = x.to(torch.bfloat16 if dtype == "bf16" else torch.float32)
    code = L.DRNMI_BF16 if dtype == "bf16" else L.DRNMI_F32
    y = torch.empty(n, dtype=torch.int8, device=DEV)
    inv = 1.0 / 0.037
    L.check(lib.drnmi_quantize_i8(x.data_ptr(), code, y.data_ptr(), n, inv, _stream()), "quantize")
    amax = torch.empty(1, device=DEV)
    L.check(lib.drnmi_absmax(x.data_ptr(), code, n, amax.data_ptr(), _stream()), "absmax")
    torch.cuda.synchronize()
    ref = Q.quantize_i8(x.float().cpu().numpy(), np.float32(inv))
    np.testing.assert_array_equal(y.cpu().numpy(), ref)
    assert amax.item() == x.float().abs().max().item()
    assert lib.drnmi_quantize_i8(x.data_ptr(), code, y.data_ptr(), 12, inv, _stream()) == -1   # n % 8


CONV_CASES = [
    # (n, h, w, cin, cout, ks, stride, pad, dil, res, out)
    (1, 16, 24, 256, 256, 3, 1, 2, 2, True, "i8"),
    (2, 9, 13, 128, 128, 3, 1, 1, 1, False, "i8"),      # ragged pixel tile, 128-wide variant
    (1, 16, 16, 64, 128, 3, 2, 1, 1, False, "i8"),      # cin 64 (64-B rows), stride 2
    (1, 16, 16, 64, 128, 1, 2, 0, 1, False, "i8"),      # 1x1 stride-2 downsample
    (1, 12, 20, 512, 512, 3, 1, 4, 4, False, "bf16"),   # dilation 4, bf16 out
    (1, 10, 10, 512, 19, 1, 1, 0, 1, False, "f32"),     # seg head: cout 19, fp32 NCHW logits
    (1, 10, 10, 512, 19, 1, 1, 0, 1, False, "f32rows20"),  # labels-head NHWC rows (y_sp 20)
    (1, 10, 10, 512, 19, 1, 1, 0, 1, False, "f32slice28"),  # channel slice of a wider fp32 NHWC buffer
    (2, 32, 64, 256, 512, 1, 1, 0, 1, False, "i8"),     # layer6.0 downsample shape (occ2 1x1 tile)
    (1, 9, 17, 128, 256, 1, 1, 0, 1, True, "bf16"),     # ragged 1x1 with a residual
    (1, 8, 8, 256, 256, 3, 1, 1, 1, True, "f32"),
    # whole 256-pixel output rows: the strip-staged int8 kernels (cin % 256 == 0: the staggered
    # conv_i8_stag_kernel; cin 128: conv_i8_strip_kernel)
    (1, 5, 256, 256, 256, 3, 1, 2, 2, True, "i8"),
    (2, 3, 512, 128, 256, 3, 1, 4, 4, False, "bf16"),
    (1, 4, 512, 512, 512, 3, 1, 4, 4, True, "i8"),
    (2, 3, 256, 256, 512, 3, 1, 1, 1, False, "bf16"),
    # long K, no residual, int8 out (conv_w1_i8_kernel's shapes: forced below, not auto-routed)
    (1, 4, 512, 512, 512, 3, 1, 2, 2, False, "i8"),
    (2, 3, 256, 1024, 256, 3, 1, 1, 1, False, "i8"),
    # 128 -> 128 on whole rows, int8 out: the int8 128 x 128 tile (conv_w1h_i8_kernel; cin 128 =
    # 9 K steps, an odd tap-group count), D-22 layer4.1 in int8 nets
    (2, 3, 256, 128, 128, 3, 1, 1, 1, True, "i8"),
    (1, 4, 512, 128, 128, 3, 1, 2, 2, False, "i8"),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_i8_matches_oracle(case):
    L, lib = _lib()
    n, h, w, cin, cout, ks, st, pad, dil, has_res, out = case
    rng = np.random.default_rng(CONV_CASES.index(case))
    x = rng.integers(-127, 128, (n, h, w, cin), dtype=np.int8)
    k = ks * ks * cin
    cout_pad = (cout + 127) // 128 * 128
    wpk = np.zeros((cout_pad, k), np.int8)
    wpk[:cout] = rng.integers(-127, 128, (cout, k), dtype=np.int8)
    scale = np.zeros(cout_pad, np.float32)
    shift = np.zeros(cout_pad, np.float32)
    scale[:cout] = (rng.uniform(0.5, 1.5, cout) / (np.sqrt(k) * 5400.0)).astype(np.float32)   # v ~ N(0, 1)
    shift[:cout] = rng.normal(0, 0.5, cout).astype(np.float32)
    ho = (h + 2 * pad - dil * (ks - 1) - 1) // st + 1
    wo = (w + 2 * pad - dil * (ks - 1) - 1) // st + 1
    res = rng.integers(-127, 128, (n, ho, wo, cout), dtype=np.int8) if has_res else None
    res_scale, out_scale = 0.011, 1.0 / 0.023
    d = {k_: torch.from_numpy(v).to(DEV) for k_, v in
         {"x": x, "w": wpk, "sc": scale, "sh": shift}.items()}
    if res is not None:
        d["res"] = torch.from_numpy(res).to(DEV)
    a = L.ConvArgs()
    a.x, a.wgt, a.scale, a.shift = d["x"].data_ptr(), d["w"].data_ptr(), d["sc"].data_ptr(), d["sh"].data_ptr()
    a.res = d["res"].data_ptr() if res is not None else None
    if out == "f32":
        y = torch.full((n, cout, ho, wo), float("nan"), device=DEV)
        a.y_sn, a.y_sp, a.y_sc, a.out_dtype = cout * ho * wo, 1, ho * wo, L.DRNMI_F32
    elif out.startswith("f32"):                      # NHWC rows of ysp floats, sentinel in the rest
        ysp = int(out[len("f32rows"):] if out.startswith("f32rows") else out[len("f32slice"):])
        y = torch.full((n, ho, wo, ysp), 7.0, device=DEV)
        a.y_sn, a.y_sp, a.y_sc, a.out_dtype = ho * wo * ysp, ysp, 1, L.DRNMI_F32
    else:
        y = torch.zeros((n, ho, wo, cout), dtype=torch.int8 if out == "i8" else torch.int16, device=DEV)
        a.y_sn, a.y_sp, a.y_sc = ho * wo * cout, cout, 1
        a.out_dtype = L.DRNMI_I8 if out == "i8" else L.DRNMI_BF16
    a.y = y.data_ptr()
    a.n, a.h, a.w, a.cin, a.ho, a.wo, a.cout, a.cout_pad = n, h, w, cin, ho, wo, cout, cout_pad
    a.ks, a.stride, a.pad, a.dil, a.k, a.k_pad = ks, st, pad, dil, k, k
    a.relu = 1 if not out.startswith("f32") or has_res else 0
    a.dtype, a.tile, a.algo = L.DRNMI_I8, -1, L.ALGO_IGEMM
    a.res_scale, a.out_scale = res_scale, out_scale
    name = lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode()
    strip = wo % 256 == 0 and ks == 3 and st == 1 and cin >= 128 and cout % 256 == 0
    # conv_w1h_i8_kernel: whole rows, int8 out, cin / cout <= 256 (D-22 layer4.1, layer5)
    w1h = wo % 256 == 0 and ks == 3 and st == 1 and cin % 128 == 0 and cout % 128 == 0 and out == "i8" and \
        cin <= 256 and cout <= 256
    assert name.startswith("conv_w1h_i8_kernel" if w1h else
                           ("conv_i8_stag_kernel" if cin % 256 == 0 else "conv_i8_strip_kernel") if strip
                           else ("conv_i8_kernel<", "conv_i8_occ2_kernel<")), name
    if ks == 1:   # 1x1 launches take the two-workgroups-per-CU tile
        assert name.startswith("conv_i8_occ2_kernel<"), name
    L.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), _stream()), "conv i8")
    torch.cuda.synchronize()
    ref = Q.conv_i8(x, wpk, scale, shift, cout, ks, st, pad, dil, bool(a.relu), res, res_scale,
                    "f32" if out.startswith("f32") else out, out_scale)
    got = y.cpu().numpy()
    if out == "f32":
        got = got.transpose(0, 2, 3, 1)
        np.testing.assert_array_equal(got, ref)
    elif out.startswith("f32"):
        np.testing.assert_array_equal(got[..., :cout], ref)
        if out.startswith("f32slice"):               # a wider buffer's other channels stay untouched
            assert bool((got[..., cout:] == 7.0).all())
    elif out == "bf16":
        np.testing.assert_array_equal(got.view(np.uint16), ref)
    else:
        np.testing.assert_array_equal(got, ref)
        assert np.abs(ref.astype(np.int32)).max() < 127 or (ref == 127).mean() < 0.5   # not all saturated
    if (strip and cin % 256 == 0) or w1h:
        # the int8 strip tiles, forced: tile 19 (conv_i8_stag_kernel) and, with an int8 output,
        # tiles 22 (conv_w1_i8_kernel) and 23 (conv_w1h_i8_kernel) -- the same oracle bits
        for t in ((19, 22, 23) if cin % 256 == 0 and cout % 256 == 0 else (23,)) if out == "i8" else (19,):
            a.tile = t
            y.fill_(0)
            L.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), _stream()), f"conv i8 tile {t}")
            torch.cuda.synchronize()
            got = y.cpu().numpy()
            if out == "f32":
                got = got.transpose(0, 2, 3, 1)
            np.testing.assert_array_equal(got.view(np.uint16) if out == "bf16" else got, ref)
        a.tile = -1


def test_conv_i8_rejects_bad_args():
    L, lib = _lib()
    a = L.ConvArgs()
    x = torch.zeros(64 * 64, dtype=torch.int8, device=DEV)
    a.x = a.wgt = a.y = a.shift = x.data_ptr()
    a.scale = None                                   # int8 needs the combined epilogue scale
    a.n, a.h, a.w, a.cin, a.ho, a.wo, a.cout, a.cout_pad = 1, 8, 8, 64, 8, 8, 64, 128
    a.ks, a.stride, a.pad, a.dil, a.k, a.k_pad = 1, 1, 0, 1, 64, 64
    a.dtype, a.out_dtype, a.tile, a.algo = L.DRNMI_I8, L.DRNMI_I8, -1, L.ALGO_IGEMM
    a.y_sn, a.y_sp, a.y_sc = 64 * 64, 64, 1
    assert lib.drnmi_conv2d_bn_act(ctypes.byref(a), _stream()) == -2
    a.scale = x.data_ptr()
    a.cin, a.k, a.k_pad = 32, 32, 32                 # int8 kernels need cin >= 64
    assert lib.drnmi_conv2d_bn_act(ctypes.byref(a), _stream()) == -2
    a.cin, a.k, a.k_pad = 64, 64, 64
    a.out_dtype = L.DRNMI_U8
    assert lib.drnmi_conv2d_bn_act(ctypes.byref(a), _stream()) == -1


_NET = {}


def _int8_net(golden):
    if "m" not in _NET:
        from drnmi.drnseg import build
        case = "d22_2x128x256"
        seed = int(golden[case + "/meta"][0])
        m = build("drn_d_22", 19, seed=seed, device=DEV)
        frames = torch.from_numpy(golden[case + "/frames"]).to(DEV)
        m.calibrate_int8(frames)
        m.set_precision("int8")
        _NET["m"], _NET["frames"] = m, frames
    return _NET["m"], _NET["frames"]


def test_int8_network_every_launch_exact(golden_forward):
    """Run the int8 D-22 plan with all activations kept and re-check every int8 launch (and the
    bf16 -> int8 boundary quantisation) from its own HBM inputs."""
    from drnmi import _lib as L
    m, frames = _int8_net(golden_forward)
    n, h, w = frames.shape[:3]
    plan = m.plan(n, h, w, keep_all=True)
    pk = plan.packed
    stream = L.stream_ptr(torch.device(DEV))
    plan.ingest_u8(frames, *_norm(), False, stream)
    plan.run_backbone(stream)
    torch.cuda.synchronize()
    i8_nodes = [(i, nd) for i, nd in enumerate(pk.graph.nodes) if nd.i8]
    assert len(i8_nodes) >= 10 and pk.quant_after, "D-22: layer4..seg should run int8"
    for i, vals in pk.quant_after.items():
        for v in vals:
            src = plan.bufs[v].float().cpu().numpy()
            ref = Q.quantize_i8(src, np.float32(1.0 / pk.act_scales[v]))
            np.testing.assert_array_equal(plan.bufs["q:" + v].cpu().numpy(), ref)
    sat = []
    for i, nd in i8_nodes:
        c = nd.conv
        cs_in = pk.cstride[nd.src]
        ih, iw = plan.shapes[nd.src]
        oh, ow = plan.shapes[nd.dst]
        x = plan.bufs[nd.x_val].cpu().numpy().reshape(n, ih, iw, cs_in)
        res = plan.bufs[nd.r_val].cpu().numpy().reshape(n, oh, ow, c.out_channels) if nd.r_val else None
        out = "f32" if nd.out_fp32_nchw else ("i8" if pk.value_code(nd.dst) == L.DRNMI_I8 else "bf16")
        ref = Q.conv_i8(x, nd.wpk.cpu().numpy(), nd.scale.cpu().numpy(), nd.shift.cpu().numpy(), c.out_channels,
                        c.kernel_size[0], c.stride[0], c.padding[0], c.dilation[0], nd.relu, res, nd.res_scale,
                        out, nd.out_scale)
        got = plan.bufs[nd.dst].cpu().numpy()
        if out == "f32":
            got = got.transpose(0, 2, 3, 1)
        elif out == "bf16":
            got = got.view(np.uint16).reshape(ref.shape)
        else:
            got = got.reshape(ref.shape)
            sat.append(float((np.abs(ref.astype(np.int32)) == 127).mean()))
        np.testing.assert_array_equal(got, ref, err_msg=nd.name)
    print(f"int8 launches checked: {len(i8_nodes)}, max saturated fraction {max(sat):.4f}")


def _norm():
    from drnmi.drnseg import INFO_MEAN, INFO_STD
    return INFO_MEAN, INFO_STD


def test_int8_labels_vs_reference(golden_forward):
    """int8 network vs the reference fp32 forward (goldens): argmax agreement."""
    m, frames = _int8_net(golden_forward)
    lab = m.segment(frames).long().cpu().numpy()
    ref = golden_forward["d22_2x128x256/labels"]
    agree = float((lab == ref).mean())
    m.set_precision("bf16")
    lab_bf16 = m.segment(frames).long().cpu().numpy()
    m.set_precision("int8")
    agree_bf16 = float((lab_bf16 == ref).mean())
    print(f"int8 label agreement with the reference fp32 forward {agree:.4f} (bf16: {agree_bf16:.4f})")
    assert agree >= 0.93
