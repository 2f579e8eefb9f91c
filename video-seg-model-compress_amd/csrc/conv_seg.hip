// The seg classifier: 1x1 conv from a wide bf16 NHWC map to <= 32 classes + bias, fp32 logits at
// any output strides (NCHW for the head) -- DRNSeg.seg, lmodels/drnseg.py:278-284.
//
// On conv_big this launch ran a 64-channel tile over 19 classes through a 4-stage LDS-DMA ring:
// 72 us for the D-22 batch-8 map (128 x 256 x 512 bf16, 268 MB), 3.7 TB/s.  The work is one read
// of the map (32 MACs per input byte at 19 classes: HBM-bound by a factor of ~60), so here no LDS
// is used at all: a wave owns 64 pixels, loads its B fragments (16 B of one pixel per lane)
// straight from global memory into registers (two sets of four K steps: one set in flight under
// the other set's MFMAs), and the 2 x 16-class A fragments per K step come from the 32-row packed weights (L1/L2
// resident).  Per accumulator the K order (32-channel steps, lane group fq = channels 8 fq .. +7),
// the MFMA and the accumulator start (shift when the scale is folded, else 0 and v * scale + shift
// after) are conv_big's BK-32 tile's, so the logits are bit-identical to it.
#include "common.h"
#include "kernels.h"

namespace drnmi {
namespace {

constexpr int kSegFN = 4;        // pixel fragments per wave (64 pixels)
constexpr int kSegKU = 4;        // K steps of B loads in flight

__global__ void __launch_bounds__(256)
conv_seg_kernel(const drnmi_conv_args p) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int M = p.n * p.ho * p.wo;
  const int hw = p.ho * p.wo;
  const int px0 = (blockIdx.x * 4 + wave) * 16 * kSegFN;
  if (px0 >= M) return;
  const int nk = p.cin / 32;
  const uint16_t* __restrict__ x = reinterpret_cast<const uint16_t*>(p.x);
  const uint16_t* __restrict__ wt = reinterpret_cast<const uint16_t*>(p.wgt);
  const bool folded = p.scale == nullptr;

  f32x4 acc[2][kSegFN];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int co = cb * 16 + fq * 4;
    f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (folded) {
      const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);   // padded to cout_pad
      a0 = f32x4{sh.x, sh.y, sh.z, sh.w};
    }
#pragma unroll
    for (int f = 0; f < kSegFN; ++f) acc[cb][f] = a0;
  }
  // pixel rows of this lane's fragments (a ragged last wave re-reads its last pixel)
  const uint16_t* xrow[kSegFN];
#pragma unroll
  for (int f = 0; f < kSegFN; ++f) {
    const int m = px0 + f * 16 + fr;
    xrow[f] = x + static_cast<int64_t>(m < M ? m : M - 1) * p.cin + fq * 8;
  }
  const uint16_t* wrow0 = wt + static_cast<int64_t>(fr) * p.k_pad + fq * 8;
  const uint16_t* wrow1 = wt + static_cast<int64_t>(16 + fr) * p.k_pad + fq * 8;

  // two register sets of kSegKU K steps: the loads of the next set are in flight while the
  // current set's MFMAs run (nk % (2 kSegKU) == 0: seg_conv_supported)
  bf16x8 b0[kSegKU][kSegFN], a0[kSegKU][2], b1[kSegKU][kSegFN], a1[kSegKU][2];
  auto load = [&](int k0, bf16x8 (&b)[kSegKU][kSegFN], bf16x8 (&a)[kSegKU][2]) {
#pragma unroll
    for (int u = 0; u < kSegKU; ++u) {
      const int kt = k0 + u < nk ? k0 + u : nk - 1;    // past the end: a re-read, never used
#pragma unroll
      for (int f = 0; f < kSegFN; ++f) b[u][f] = *reinterpret_cast<const bf16x8*>(xrow[f] + kt * 32);
      a[u][0] = *reinterpret_cast<const bf16x8*>(wrow0 + kt * 32);
      a[u][1] = *reinterpret_cast<const bf16x8*>(wrow1 + kt * 32);
    }
  };
  auto mma = [&](const bf16x8 (&b)[kSegKU][kSegFN], const bf16x8 (&a)[kSegKU][2]) {
#pragma unroll
    for (int u = 0; u < kSegKU; ++u)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int f = 0; f < kSegFN; ++f)
          acc[cb][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][cb], b[u][f], acc[cb][f], 0, 0, 0);
  };
  load(0, b0, a0);
  for (int k0 = 0; k0 < nk; k0 += 2 * kSegKU) {
    load(k0 + kSegKU, b1, a1);
    __builtin_amdgcn_sched_barrier(0);
    mma(b0, a0);
    __builtin_amdgcn_sched_barrier(0);
    if (k0 + 2 * kSegKU < nk) load(k0 + 2 * kSegKU, b0, a0);
    __builtin_amdgcn_sched_barrier(0);
    mma(b1, a1);
    __builtin_amdgcn_sched_barrier(0);
  }

  // lane (fr, fq) holds classes 16 cb + 4 fq + j of pixel px0 + 16 f + fr
#pragma unroll
  for (int f = 0; f < kSegFN; ++f) {
    const int m = px0 + f * 16 + fr;
    if (m >= M) continue;
    const int n = m / hw;
    const int q = m - n * hw;
    const int64_t ybase = static_cast<int64_t>(n) * p.y_sn + static_cast<int64_t>(q) * p.y_sp;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = cb * 16 + fq * 4 + j;
        if (co >= p.cout) break;
        float v = acc[cb][f][j];
        if (!folded) v = v * p.scale[co] + p.shift[co];
        if (p.relu) v = fmaxf(v, 0.f);
        const int64_t off = ybase + static_cast<int64_t>(co) * p.y_sc;
        if (p.out_dtype == DRNMI_BF16) reinterpret_cast<uint16_t*>(p.y)[off] = f32_to_bf16(v);
        else reinterpret_cast<float*>(p.y)[off] = v;
      }
    }
  }
}

}  // namespace

bool seg_conv_supported(const drnmi_conv_args& p) {
  return p.dtype == DRNMI_BF16 && p.ks == 1 && p.stride == 1 && p.pad == 0 && p.cout >= 1 && p.cout <= 32 &&
         p.cout_pad >= 32 && p.cin % (64 * kSegKU) == 0 && p.k == p.cin && p.k_pad >= p.k && p.k_pad % 8 == 0 &&
         p.x2 == nullptr && p.res == nullptr && p.unit_mask == nullptr &&
         (p.out_dtype == DRNMI_F32 || p.out_dtype == DRNMI_BF16) && p.ho == p.h && p.wo == p.w &&
         static_cast<int64_t>(p.n) * p.h * p.w < (int64_t(1) << 31);
}

int seg_conv_dispatch(const drnmi_conv_args& p, hipStream_t s) {
  if (!seg_conv_supported(p)) return DRNMI_ENOTSUP;
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int64_t waves = (M + 16 * kSegFN - 1) / (16 * kSegFN);
  hipLaunchKernelGGL(conv_seg_kernel, dim3(static_cast<unsigned>((waves + 3) / 4)), dim3(256), 0, s, p);
  return static_cast<int>(hipGetLastError());
}

}  // namespace drnmi
