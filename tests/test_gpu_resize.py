"""Pillow-exact bilinear resize on the GPU (seg_video ingest T.Resize, test_ms resize_4d_tensor)
and the multi-scale eval driver, against oracle/eval_oracle.py (Pillow itself, the arithmetic the
reference calls).  Gates: bit-identical bytes / fp32 values / labels / histogram."""
import numpy as np
import pytest
import torch

from oracle import eval_oracle as E

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("h,w,oh,ow", [(640, 1138, 300, 300),     # sample.mp4 frame -> seg_video size
                                       (1024, 2048, 300, 300),
                                       (360, 640, 300, 300),       # Road_1101.mp4 frame
                                       (97, 61, 300, 300),         # upscale
                                       (300, 517, 300, 300),       # one axis unchanged
                                       (517, 300, 300, 300),
                                       (300, 300, 300, 300)])
def test_resize_u8_matches_pillow(h, w, oh, ow):
    from drnmi import ops
    rng = np.random.default_rng(h * 7 + w)
    frames = rng.integers(0, 256, size=(2, h, w, 3), dtype=np.uint8)
    frames[1] = np.clip(np.linspace(0, 255, w)[None, :, None] + rng.normal(0, 20, (h, w, 3)), 0, 255).astype(np.uint8)
    got = ops.resize_bilinear_u8(torch.from_numpy(frames).to(DEV), (oh, ow)).cpu().numpy()
    for i in range(2):
        ref = E.resize_frame_u8(frames[i], (oh, ow))
        bad = int((got[i] != ref).sum())
        assert bad == 0, f"{bad} bytes differ from Pillow"


@pytest.mark.parametrize("h,w,oh,ow", [(64, 128, 512, 1024), (48, 96, 64, 128), (80, 160, 64, 128),
                                       (37, 53, 64, 128), (64, 100, 64, 128)])
def test_resize_f32_matches_pillow(h, w, oh, ow):
    from drnmi import ops
    g = torch.Generator().manual_seed(h + w)
    x = torch.randn(2, 19, h, w, generator=g) * 5
    got = ops.resize_bilinear_f32(x.to(DEV), (oh, ow)).cpu().numpy()
    ref = E.resize_4d_tensor(x.numpy(), ow, oh)
    np.testing.assert_array_equal(got, ref)
    acc = torch.from_numpy(ref).to(DEV) * 0 + 1.5
    ops.resize_bilinear_f32(x.to(DEV), (oh, ow), out=acc, accumulate=True)
    np.testing.assert_array_equal(acc.cpu().numpy(), np.float32(1.5) + ref)


def test_argmax_first_max():
    from drnmi import ops
    x = torch.zeros(2, 5, 3, 4)
    x[0, 2, 0, 0] = 1.0
    x[0, 4, 0, 0] = 1.0          # tie: first index wins
    x[1, :, 1, 1] = torch.tensor([0.0, 3.0, 3.0, -1.0, 2.0])
    lab = ops.argmax_nchw(x.to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(lab, x.numpy().argmax(axis=1))
    lab8 = ops.argmax_nchw(x.to(DEV), torch.uint8).cpu().numpy()
    np.testing.assert_array_equal(lab8, x.numpy().argmax(axis=1))


def test_segment_with_resize_matches_pillow_pipeline():
    """segment(frames, size=(300, 300)) == segment(Pillow-resized frames): the seg_video loop."""
    from drnmi.drnseg import build
    m = build("drn_d_22", 19, seed=3, device=DEV, precision="fp32")
    rng = np.random.default_rng(5)
    frames = rng.integers(0, 256, size=(2, 640, 1138, 3), dtype=np.uint8)
    lab = m.segment(torch.from_numpy(frames).to(DEV), size=(300, 300))
    small = np.stack([E.resize_frame_u8(f, (300, 300)) for f in frames])
    ref = m.segment(torch.from_numpy(small).to(DEV))
    assert lab.shape == (2, 304, 304)
    assert torch.equal(lab, ref)


def test_test_ms_matches_oracle_pipeline():
    """drnmi.evaluate.test_ms (GPU resize + fp32 sum + argmax + histogram) == the reference's
    numpy/Pillow pipeline applied to the same model outputs."""
    from drnmi import evaluate
    from drnmi.drnseg import build
    from oracle import drn_oracle as O
    m = build("drn_d_22", 19, seed=4, device=DEV, precision="fp32")
    g = torch.Generator().manual_seed(2)
    h, w = 96, 160
    scales = [0.5, 0.75, 1.25]
    img = torch.randn(1, 3, h, w, generator=g)
    ms = [torch.nn.functional.interpolate(img, size=(int(h * s), int(w * s)), mode="bilinear", align_corners=False)
          for s in scales]
    label = torch.randint(0, 19, (1, h, w), generator=g)
    label[:, :10] = 255
    loader = [(img, label, "frame0", *ms)]
    miou = evaluate.test_ms(loader, m, 19, scales)
    preds = evaluate.test_ms(loader, m, 19, scales, has_gt=False)[0].cpu().numpy()
    outs = [m(t.to(DEV))[0].cpu().numpy() for t in [img] + ms]
    ref_pred = E.multiscale_pred(outs, w, h)
    np.testing.assert_array_equal(preds, ref_pred)
    hist = O.fast_hist(ref_pred.flatten(), label.numpy().flatten(), 19)
    ref_miou = round(float(np.nanmean(O.per_class_iu(hist) * 100)), 2)
    assert miou == ref_miou
    single = evaluate.test([(img, label)], m, 19)
    pred1 = torch.max(m(img.to(DEV))[0], 1)[1].cpu().numpy()
    h1 = O.fast_hist(pred1.flatten(), label.numpy().flatten(), 19)
    assert single == round(float(np.nanmean(O.per_class_iu(h1) * 100)), 2)
