"""conv_x6 (fp32x) micro-benchmark on the exact-mode / fine-tune shapes: HIP-event time per launch,
fp32-accurate TFLOP/s (peak 2.5 PF / 6) and a SHA-1 of the output bytes (bit-identity across
variants: VARIANTS=auto,3 forces conv_x6 variants through drnmi_conv_args.tile).
python scripts/x6_micro.py"""
import ctypes
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "video-seg-model-compress_amd"))
import torch  # noqa: E402

from drnmi import _lib, ops  # noqa: E402
from drnmi.engine import split3_bf16  # noqa: E402

DEV = "cuda"
SHAPES = [  # name, n, h, w, cin, cout, ks, stride, pad, dil, res, split
    ("l6 512 d4 +res b8", 8, 128, 256, 512, 512, 3, 1, 4, 4, True, False),
    ("l8 512 d1 b8", 8, 128, 256, 512, 512, 3, 1, 1, 1, False, False),
    ("l5 256 d2 +res b8", 8, 128, 256, 256, 256, 3, 1, 2, 2, True, False),
    ("l6 ds 1x1 b8", 8, 128, 256, 256, 512, 1, 1, 0, 1, False, False),
    ("ft l6 512 d4 split", 2, 128, 96, 512, 512, 3, 1, 4, 4, False, True),
    ("l3 64 +res b8", 8, 256, 512, 64, 64, 3, 1, 1, 1, True, False),
    ("l4 128 +res b8", 8, 128, 256, 128, 128, 3, 1, 1, 1, True, False),
    ("l4.0 ds 1x1 s2 b8", 8, 256, 512, 64, 128, 1, 2, 0, 1, False, False),
    ("l5.0 ds 1x1 b8", 8, 128, 256, 128, 256, 1, 1, 0, 1, False, False),
    ("ft 1x1 1024-256", 2, 128, 96, 1024, 256, 1, 1, 0, 1, False, True),
    ("ft 1x1 256-1024", 2, 128, 96, 256, 1024, 1, 1, 0, 1, True, True),
    ("ft 1x1 2048-512", 2, 128, 96, 2048, 512, 1, 1, 0, 1, False, True),
    ("ft 1x1 512-2048", 2, 128, 96, 512, 2048, 1, 1, 0, 1, True, True),
    ("ft 1x1 512-256", 2, 128, 96, 512, 256, 1, 1, 0, 1, False, True),
    ("ft 3x3 256 d2", 2, 128, 96, 256, 256, 3, 1, 2, 2, False, True),
    ("ft l3 1x1 256-64", 2, 256, 192, 256, 64, 1, 1, 0, 1, False, True),
    ("ft l3 1x1 64-256", 2, 256, 192, 64, 256, 1, 1, 0, 1, True, True),
    ("seg 1x1 512-19 b8", 8, 128, 256, 512, 19, 1, 1, 0, 1, False, False),
]
SEL = os.environ.get("SHAPES")
if SEL:
    SHAPES = [sh for sh in SHAPES if any(k in sh[0] for k in SEL.split(","))]
VARIANTS = [(-1 if v == "auto" else int(v)) for v in os.environ.get("VARIANTS", "auto").split(",")]
# SPLITS=1,2,4: force split-K counts on the split shapes (tile = variant + 6 * splits; the variant
# is the auto one when VARIANTS=auto)
SPLITS = [int(v) for v in os.environ.get("SPLITS", "0").split(",")]
lib = _lib.load()
for name, n, h, w, cin, cout, ks, s, pad, dil, res, split in SHAPES:
    g = torch.Generator(device=DEV).manual_seed(cin + cout + ks)
    xd = torch.randn(n, h, w, cin, device=DEV, generator=g)
    wt = torch.randn(cout, cin, ks, ks, device=DEV, generator=g) / (cin * ks * ks) ** 0.5
    ho = (h + 2 * pad - dil * (ks - 1) - 1) // s + 1
    wo = (w + 2 * pad - dil * (ks - 1) - 1) // s + 1
    rd = torch.randn(n, ho, wo, cout, device=DEV, generator=g) if res else None
    wpk, k = ops.pack_conv_weight(wt, cin, torch.float32)
    planes = split3_bf16(wpk)
    scp = torch.rand(wpk.shape[0], device=DEV, generator=g) + 0.5
    shp = torch.randn(wpk.shape[0], device=DEV, generator=g)
    y = torch.empty(n, ho, wo, cout, device=DEV)
    a = _lib.ConvArgs()
    a.x, a.wgt, a.scale, a.shift = xd.data_ptr(), planes.data_ptr(), scp.data_ptr(), shp.data_ptr()
    a.res = rd.data_ptr() if res else None
    a.y = y.data_ptr()
    a.y_sn, a.y_sp, a.y_sc = ho * wo * cout, cout, 1
    a.n, a.h, a.w, a.cin = n, h, w, cin
    a.ho, a.wo, a.cout, a.cout_pad = ho, wo, cout, wpk.shape[0]
    a.ks, a.stride, a.pad, a.dil = ks, s, pad, dil
    a.k, a.k_pad = k, wpk.shape[1]
    a.relu, a.dtype, a.out_dtype, a.tile, a.algo = 1, _lib.DRNMI_F32X3, _lib.DRNMI_F32, -1, _lib.ALGO_IGEMM
    st = ctypes.c_void_p(_lib.stream_ptr())
    combos = [(v, 0) for v in VARIANTS] if not split else [(v, sp) for v in VARIANTS for sp in SPLITS]
    for var, sp in combos:
      a.tile = var
      if sp > 0:
          a.tile = (var if var >= 0 else 0 if cout % 256 == 0 else 3 if cout % 128 == 0 else 2) + 6 * sp
      if split:                       # workspace for this launch's own split count
          a.ws, a.ws_bytes = None, 0
          nb = lib.drnmi_conv_workspace_bytes(ctypes.byref(a))
          ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=DEV)
          a.ws, a.ws_bytes = ws.data_ptr(), nb
      kname = lib.drnmi_conv_kernel_name(ctypes.byref(a))
      if kname is None:
        continue
      kn = kname.decode()
      if (cout + int(kn.split(",")[1]) * int(kn.split(",")[2]) - 1) // (int(kn.split(",")[1]) * int(kn.split(",")[2])) \
              * int(kn.split(",")[1]) * int(kn.split(",")[2]) > wpk.shape[0]:
        continue                      # a forced tile wider than the packed weight rows
      best = None
      for rep in range(3):
        for _ in range(2):
            _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), st), "x6")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            _lib.check(lib.drnmi_conv2d_bn_act(ctypes.byref(a), st), "x6")
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 5 * 1e3
        best = us if best is None else min(best, us)
      flops = 2.0 * n * ho * wo * cout * cin * ks * ks
      sha = hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest()[:12]
      print(f"{name:22s} {kname.decode():28s} S{sp} {best:9.1f} us  {flops / best / 1e6:6.1f} TF  "
            f"({flops / best / 1e6 / (2500 / 6):.3f} of 417)  sha {sha}", flush=True)
