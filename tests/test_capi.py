"""The C-ABI library loads without a GPU and exports every symbol include/drnmi.h declares."""
import ctypes
import os
import re
import subprocess

import numpy as np

from drnmi import _lib
from drnmi.build import LIB_PATH, build

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "drnmi.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(drnmi_[a-z0-9_]+)\s*\(", text)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(_lib.SIGNATURES)


def test_library_exports_every_symbol():
    path = build(verbose=False)
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (drnmi_[a-z0-9_]+)", out))
    missing = set(declared_functions()) - exported
    assert not missing, missing


def test_library_loads_and_reports():
    lib = _lib.load()
    assert lib.drnmi_version().decode().startswith("drnmi ")
    n = lib.drnmi_conv_num_tiles()
    assert n >= 4
    names = [lib.drnmi_conv_tile_name(i).decode() for i in range(n)]
    assert names[0] == "128x128"
    assert lib.drnmi_conv_tile_name(n) is None


def test_argument_validation_without_gpu():
    """Rejected arguments return DRNMI_EINVAL before any HIP call (safe with no device)."""
    lib = _lib.load()
    a = _lib.ConvArgs()
    a.cin = 12          # not a power of two
    assert lib.drnmi_conv2d_bn_act(ctypes.byref(a), None) == -1
    assert lib.drnmi_conv2d_bn_act(None, None) == -1
    assert lib.drnmi_up8_logsoftmax_argmax(None, None, None, None, 2, 1, 19, 8, 8, None) == -1
    assert lib.drnmi_mask_apply_f32(-1, None, None, None, None) == -1
    assert lib.drnmi_mask_apply_f32(0, None, None, None, None) == 0
    # BN-statistics partials: only from an fp32x conv_x6 launch; the finalize validates its inputs
    assert lib.drnmi_conv_stats_rows(None) == -1
    b = _lib.ConvArgs()
    b.n, b.h, b.w, b.cin, b.ho, b.wo, b.cout, b.cout_pad = 1, 8, 8, 64, 8, 8, 64, 128
    b.ks, b.stride, b.pad, b.dil, b.k, b.k_pad = 1, 1, 0, 1, 64, 64
    b.dtype = b.out_dtype = _lib.DRNMI_F32
    assert lib.drnmi_conv_stats_rows(ctypes.byref(b)) == 0          # not fp32x: no partials
    b.stats = 0x1000
    assert lib.drnmi_conv2d_bn_act(ctypes.byref(b), None) == -1    # refused before any launch
    b.dtype = _lib.DRNMI_F32X3
    assert lib.drnmi_conv_stats_rows(ctypes.byref(b)) == 4         # one 256-pixel tile: 4 wave rows
    assert lib.drnmi_bn_stats_partials_f32(None, 4, 64, 64, 1e-5, 0.1, None, None, None, None, None, None) == -1


def test_pack_table_check_without_gpu():
    """The batched weight-pack table is validated on the host (prefix sums, geometry)."""
    lib = _lib.load()
    rows = [[0x1000, 0x2000, 0, 64, 32, 3, 32, 64, 288, 0, 0, 0],
            [0x1000, 0x3000, 0x4000, 64, 32, 3, 64, 32, 576, 1, 64 * 288, 0]]
    tab = np.array(rows, dtype=np.int64)
    tot = ctypes.c_int64(0)
    assert lib.drnmi_pack_table_check(tab.ctypes.data_as(ctypes.c_void_p), 2, ctypes.byref(tot)) == 0
    assert tot.value == 64 * 288 + 32 * 576
    bad = tab.copy()
    bad[1, 10] += 1                                   # wrong prefix
    assert lib.drnmi_pack_table_check(bad.ctypes.data_as(ctypes.c_void_p), 2, ctypes.byref(tot)) == -1
    bad = tab.copy()
    bad[0, 8] = 100                                   # k_pad < ks * ks * kin_stride
    assert lib.drnmi_pack_table_check(bad.ctypes.data_as(ctypes.c_void_p), 2, ctypes.byref(tot)) == -1
    bad = tab.copy()
    bad[0, 6], bad[0, 8] = 34, 308                    # kin_stride not a multiple of 4 (4-column stores)
    assert lib.drnmi_pack_table_check(bad.ctypes.data_as(ctypes.c_void_p), 2, ctypes.byref(tot)) == -1
    bad = tab.copy()
    bad[0, 5], bad[0, 8] = 9, 81 * 32                 # ks > 7 (the LDS tile holds up to 7x7 taps)
    assert lib.drnmi_pack_table_check(bad.ctypes.data_as(ctypes.c_void_p), 2, ctypes.byref(tot)) == -1
    bad = tab.copy()
    bad[1, 2] += 8                                    # planes not 16-B aligned
    assert lib.drnmi_pack_table_check(bad.ctypes.data_as(ctypes.c_void_p), 2, ctypes.byref(tot)) == -1
    assert lib.drnmi_pack_conv_weights_batched(None, 2, 10, None) == -1


def test_fused_second_input_never_routes_to_halo():
    """A conv with a fused second input (x2, the folded 1x1 downsample) must go to a kernel
    that reads x2: the halo kernel takes it only in its fused-downsample form (scale folded,
    no residual, cin2 32/64, rows padded to 64-column steps); anything else must not route
    there, or the downsample term would be dropped silently."""
    lib = _lib.load()
    a = _lib.ConvArgs()
    a.n, a.h, a.w, a.cin, a.ho, a.wo, a.cout, a.cout_pad = 1, 16, 16, 64, 16, 16, 64, 128
    a.ks, a.stride, a.pad, a.dil = 3, 1, 1, 1
    a.k = a.k_pad = 9 * 64
    a.dtype = a.out_dtype = _lib.DRNMI_BF16
    a.y_sp, a.y_sc, a.tile, a.algo = 64, 1, -1, _lib.ALGO_IGEMM
    assert lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode().startswith("conv_halo")
    a.x2, a.cin2, a.h2, a.w2, a.stride2 = 1, 64, 32, 32, 2
    a.k = a.k_pad = 9 * 64 + 64
    # scale = NULL (folded) and no residual: the halo kernel's fused-downsample form takes it
    assert lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode().startswith("conv_halo_kernel")
    a.cin2, a.k, a.k_pad = 32, 9 * 64 + 32, 9 * 64 + 32   # k_pad must be k rounded up to 64
    assert lib.drnmi_conv_kernel_name(ctypes.byref(a)) is None or \
        not lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode().startswith("conv_halo")
    a.k_pad = 9 * 64 + 64
    assert lib.drnmi_conv_kernel_name(ctypes.byref(a)).decode().startswith("conv_halo_kernel")
    sc = (ctypes.c_float * 64)()
    a.scale = ctypes.cast(sc, ctypes.c_void_p).value      # an unfolded scale: not the halo x2 form
    name = lib.drnmi_conv_kernel_name(ctypes.byref(a))
    assert name is None or not name.decode().startswith("conv_halo")


def test_kernel_peak_by_name():
    """bench.py prices the dominant kernel at the peak of the arithmetic it runs: every int8 kernel
    name the library reports (conv_i8_*, conv_w1_i8_*, conv_w1h_i8_*) at the int8 peak, even in
    int8 nets whose base precision is bf16."""
    from drnmi.roofline import MFMA_PEAK, kernel_peak
    for n in ("conv_i8_stag_kernel", "conv_i8_stag_seg_kernel", "conv_w1_i8_kernel", "conv_w1_i8_seg_kernel",
              "conv_w1h_i8_kernel", "conv_i8_occ2_kernel<1, 128, 1, 2, 64>"):
        assert kernel_peak(n, "bf16") == MFMA_PEAK["int8"], n
    for n in ("conv_stag_kernel", "conv_w1_kernel", "conv_w1h_kernel", "conv_w1_seg_kernel", "front3_kernel"):
        assert kernel_peak(n, "bf16") == MFMA_PEAK["bf16"], n
    assert kernel_peak("conv_x6_kernel<3, 128, 2, 4>", "fp32x") == MFMA_PEAK["fp32x"]
    assert kernel_peak("patch_f32_kernel<0, 16, 7, 1, 4, 64>", "fp32x") == MFMA_PEAK["fp32"]
