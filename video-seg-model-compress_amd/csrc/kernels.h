// Internal (non-ABI) launchers shared between the kernel translation units.
#pragma once
#include "common.h"

namespace drnmi {
// Small-channel LDS-patch conv (patch_conv.hip); returns drnmi_status / hipError_t.
int patch_conv_dispatch(const drnmi_conv_args& p, hipStream_t s);
// bf16 LDS-DMA implicit GEMM for cin >= 64, cout % 128 == 0 (conv_big.hip).
bool big_conv_supported(const drnmi_conv_args& p);
int big_conv_dispatch(const drnmi_conv_args& p, int variant, hipStream_t s);  // variant -1 = auto
const char* big_conv_name(const drnmi_conv_args& p, int variant);
const char* patch_conv_name(const drnmi_conv_args& p);
// Exact-fp32 small-channel LDS-patch conv on the f32 MFMA (patch_f32.hip): layer0..layer2 shapes.
int patch_f32_dispatch(const drnmi_conv_args& p, hipStream_t s);
const char* patch_f32_name(const drnmi_conv_args& p);
// Fused uint8 stem + the 3x3 16->16 conv after it (patch_conv.hip).
bool stem_l1_ok(const drnmi_conv_args& p, const drnmi_conv_args& q);
int stem_l1_dispatch(const drnmi_conv_args& p, const drnmi_conv_args& q, hipStream_t s);
int weight_unit_mask(const void* wgt, int dtype, int rows_pad, int k_pad, uint32_t* mask, int* count, hipStream_t s);
// W8A8 LDS-DMA implicit GEMM (conv_big.hip, config C5): dtype DRNMI_I8, cin >= 64.
bool i8_conv_supported(const drnmi_conv_args& p);
int i8_conv_dispatch(const drnmi_conv_args& p, hipStream_t s);
const char* i8_conv_name(const drnmi_conv_args& p);
// Halo-patch 3x3 stride-1 conv, cin/cout 64 or 128 (conv_halo.hip).
bool halo_conv_supported(const drnmi_conv_args& p);
int halo_conv_dispatch(const drnmi_conv_args& p, hipStream_t s);
const char* halo_conv_name(const drnmi_conv_args& p);
// fp32-accurate 6-product split-bf16 implicit GEMM (conv_x6.hip): dtype DRNMI_F32X3, cin >= 32.
bool x6_conv_supported(const drnmi_conv_args& p);
int x6_conv_dispatch(const drnmi_conv_args& p, hipStream_t s);
int64_t x6_conv_workspace_bytes(const drnmi_conv_args& p);
int64_t x6_conv_stats_rows(const drnmi_conv_args& p);
const char* x6_conv_name(const drnmi_conv_args& p);
// The strip tile with staggered SIMD partners (conv_stag.hip): 3x3 stride-1 bf16, wo % 256 == 0,
// cin % 128 == 0 (conv_big.hip's dispatch checks the shape).
hipError_t launch_stag(const drnmi_conv_args& p, hipStream_t s);
// conv_stag_kernel with the seg classifier in its epilogue (drnmi_conv_stag_seg): no activation store,
// partial logits per 256-channel block into part[cout / 256][n ho wo][20] (fp32; int8 nets: int32 sums).
// The same strip tile as 4 waves of 128 x 128 (one wave per SIMD, conv_w1.hip): bf16, no x2,
// cout % 256 == 0; bit-identical to conv_stag_kernel.
hipError_t launch_w1(const drnmi_conv_args& p, hipStream_t s);
// ... as a 128 x 128 tile (conv_w1h_kernel: 4 waves of 64 x 64, two workgroups per CU)
hipError_t launch_w1h(const drnmi_conv_args& p, hipStream_t s);
// ... with the seg classifier in its epilogue (conv_w1_seg_kernel; bf16, partials as launch_stag_seg's)
hipError_t launch_w1_seg(const drnmi_conv_args& p, const void* seg_w, int seg_k_pad, void* part, hipStream_t s);
hipError_t launch_stag_seg(const drnmi_conv_args& p, const void* seg_w, int seg_k_pad, void* part, hipStream_t s);
// Row-walking stride-2 3x3 conv, 32 -> 64 / 64 -> 128 (conv_s2row.hip), bit-identical to conv_big's
// BK-32 / BK-64 tiles; s2row_auto: routed by default where supported.
bool s2row_conv_supported(const drnmi_conv_args& p);
bool s2row_auto(const drnmi_conv_args& p);
int s2row_conv_dispatch(const drnmi_conv_args& p, hipStream_t s);
const char* s2row_conv_name(const drnmi_conv_args& p);
// Row-walking stride-1 3x3 64 -> 64 + folded 1x1 stride-2 downsample from 32 channels (conv_s2row.hip),
// bit-identical to conv_halo's x2 form.
bool s1x2row_conv_supported(const drnmi_conv_args& p);
bool s1x2row_auto(const drnmi_conv_args& p);
int s1x2row_conv_dispatch(const drnmi_conv_args& p, hipStream_t s);
const char* s1x2row_conv_name(const drnmi_conv_args& p);
}  // namespace drnmi
