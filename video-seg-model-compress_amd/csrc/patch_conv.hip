// Small-channel direct convolution through an LDS input patch (bf16 MFMA).
//
// The full-resolution DRN-D layers have 3..32 input channels at 2M pixels per frame
// (reference lmodels/drn.py:132-137 layer0 7x7 3->16, :201-211 layer1 3x3 16->16,
// layer2 3x3 s2 16->32): too few channels for the implicit GEMM's 8-channel gathers to
// amortise address math, and every tap of a pixel re-reads the same input bytes.  Here a
// workgroup stages its output tile's input rows once (tile + halo) in LDS, keeps all
// weights in registers, and reads each B fragment (8 channels of one pixel-tap) with one
// LDS access.  MFMA orientation: A = weights (rows = output channels), B = pixels, so the
// accumulator gives each lane 4 consecutive channels of one pixel: 8-byte NHWC stores,
// 16 pixels x cout contiguous per wave instruction.
//
// The stem variant (SRC_U8) reads the uint8 HWC3 frame and applies the reference
// normalisation on load (ToTensorVideoImage + Normalize, data_transforms.py:109-125,
// :256-281; same fp32 op order), so the frame-ingest pass and its 8-channel
// intermediate disappear.  Its K is laid out kh*32 + kw*4 + c (kw < 8, c < 4) so a
// k-step is one kernel row and a fragment is two adjacent pixels x 4 channels.
#include "common.h"
#include "kernels.h"

namespace drnmi {
namespace {

constexpr int kThreads = 256;

template <int CIN, int COUT, int KS, int S, int TR, int TC, bool SRC_U8>
struct PatchCfg {
  static constexpr int CP = SRC_U8 ? 4 : CIN;                  // LDS channels per pixel
  static constexpr int PR = (TR - 1) * S + KS;                 // patch rows
  static constexpr int PCV = (TC - 1) * S + KS + (SRC_U8 ? 1 : 0);  // +1: kw=7 zero tap
  static constexpr int PC = PCV;
  static constexpr int K = SRC_U8 ? KS * 32 : KS * KS * CIN;
  static constexpr int NK = (K + 31) / 32;
  static constexpr int MF = COUT / 16;                         // output-channel fragments
  static constexpr int PF = TR * TC / 16;                      // pixel fragments per tile
  static constexpr int PFW = PF / 4;                           // per wave
  static constexpr int LDS_ELEMS = PR * PC * CP;
  static_assert(PF % 4 == 0, "tile must split over 4 waves");
  static_assert(TC % 16 == 0, "tile columns in 16-pixel fragments");
};

template <int CIN, int COUT, int KS, int S, int TR, int TC, bool SRC_U8>
__global__ void __launch_bounds__(kThreads)
patch_conv_kernel(const drnmi_conv_args p) {
  using C = PatchCfg<CIN, COUT, KS, S, TR, TC, SRC_U8>;
  __shared__ __attribute__((aligned(16))) bf16_t patch[C::LDS_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tiles_w = (p.wo + TC - 1) / TC;
  const int tiles_h = (p.ho + TR - 1) / TR;
  const int b = blockIdx.x;
  const int n = b / (tiles_w * tiles_h);
  const int rem = b - n * tiles_w * tiles_h;
  const int oh0 = (rem / tiles_w) * TR;
  const int ow0 = (rem % tiles_w) * TC;
  const int ih0 = oh0 * S - p.pad;
  const int iw0 = ow0 * S - p.pad;

  // ---- weights -> registers: A fragment (mf, ks) = W[mf*16 + lane&15][ks*32 + 8*(lane>>4) ..+7]
  const bf16_t* __restrict__ wt = reinterpret_cast<const bf16_t*>(p.wgt);
  bf16x8 wa[C::MF][C::NK];
#pragma unroll
  for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
    for (int ks = 0; ks < C::NK; ++ks)
      wa[mf][ks] = *reinterpret_cast<const bf16x8*>(
          wt + static_cast<int64_t>(mf * 16 + (lane & 15)) * p.k_pad + ks * 32 + 8 * (lane >> 4));

  // ---- stage the input patch (zero outside the image = the conv's zero padding)
  if constexpr (SRC_U8) {
    const uint8_t* __restrict__ fr = reinterpret_cast<const uint8_t*>(p.x) +
                                     static_cast<int64_t>(n) * p.h * p.w * 3;
    for (int i = tid; i < C::PR * C::PC; i += kThreads) {
      const int pr = i / C::PC, pc = i - pr * C::PC;
      const int ih = ih0 + pr, iw = iw0 + pc;
      uint2 v = make_uint2(0, 0);
      if (static_cast<unsigned>(ih) < static_cast<unsigned>(p.h) &&
          static_cast<unsigned>(iw) < static_cast<unsigned>(p.w)) {
        const uint8_t* px = fr + (static_cast<int64_t>(ih) * p.w + iw) * 3;
        float c0 = static_cast<float>(px[0]), c1 = static_cast<float>(px[1]), c2 = static_cast<float>(px[2]);
        if (p.bgr) { const float t = c0; c0 = c2; c2 = t; }
        const float v0 = (c0 / 255.0f - p.mean[0]) / p.std[0];
        const float v1 = (c1 / 255.0f - p.mean[1]) / p.std[1];
        const float v2 = (c2 / 255.0f - p.mean[2]) / p.std[2];
        v.x = static_cast<uint32_t>(f32_to_bf16(v0)) | (static_cast<uint32_t>(f32_to_bf16(v1)) << 16);
        v.y = static_cast<uint32_t>(f32_to_bf16(v2));
      }
      *reinterpret_cast<uint2*>(patch + i * 4) = v;
    }
  } else {
    const bf16_t* __restrict__ x = reinterpret_cast<const bf16_t*>(p.x) +
                                   static_cast<int64_t>(n) * p.h * p.w * CIN;
    constexpr int VPP = CIN / 8;  // 16-B vectors per pixel
    for (int i = tid; i < C::PR * C::PC * VPP; i += kThreads) {
      const int pix = i / VPP, v8 = i - pix * VPP;
      const int pr = pix / C::PC, pc = pix - pr * C::PC;
      const int ih = ih0 + pr, iw = iw0 + pc;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (static_cast<unsigned>(ih) < static_cast<unsigned>(p.h) &&
          static_cast<unsigned>(iw) < static_cast<unsigned>(p.w))
        v = *reinterpret_cast<const uint4*>(x + (static_cast<int64_t>(ih) * p.w + iw) * CIN + v8 * 8);
      *reinterpret_cast<uint4*>(patch + pix * CIN + v8 * 8) = v;
    }
  }
  __syncthreads();

  // ---- MFMA: this wave's pixel fragments pf = wave + 4*q
  f32x4 acc[C::MF][C::PFW];
#pragma unroll
  for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
    for (int q = 0; q < C::PFW; ++q) acc[mf][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  int prow[C::PFW], pcol[C::PFW];
#pragma unroll
  for (int q = 0; q < C::PFW; ++q) {
    const int idx = (wave + 4 * q) * 16 + (lane & 15);
    prow[q] = (idx / TC) * S;
    pcol[q] = (idx % TC) * S;
  }
  const int kq = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < C::NK; ++ks) {
#pragma unroll
    for (int q = 0; q < C::PFW; ++q) {
      bf16x8 bv;
      if constexpr (SRC_U8) {
        // k = kh*32 + kw*4 + c: step ks = kernel row kh, fragment = taps kw = 2kq, 2kq+1
        const bf16_t* src = patch + ((prow[q] + ks) * C::PC + pcol[q] + 2 * kq) * 4;
        const uint2 lo = *reinterpret_cast<const uint2*>(src);
        const uint2 hi = *reinterpret_cast<const uint2*>(src + 4);
        const uint4 u = make_uint4(lo.x, lo.y, hi.x, hi.y);
        bv = __builtin_bit_cast(bf16x8, u);
      } else {
        const int k0 = ks * 32 + 8 * kq;
        const int tap = k0 / CIN;
        const int ci = k0 % CIN;
        if (tap < KS * KS) {
          const int kh = tap / KS, kw = tap % KS;
          const uint4 u = *reinterpret_cast<const uint4*>(
              patch + ((prow[q] + kh) * C::PC + pcol[q] + kw) * CIN + ci);
          bv = __builtin_bit_cast(bf16x8, u);
        } else {
          bv = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
        }
      }
#pragma unroll
      for (int mf = 0; mf < C::MF; ++mf)
        acc[mf][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[mf][ks], bv, acc[mf][q], 0, 0, 0);
    }
  }

  // ---- epilogue: lane owns channels co..co+3 of one pixel
  bf16_t* __restrict__ y = reinterpret_cast<bf16_t*>(p.y);
#pragma unroll
  for (int q = 0; q < C::PFW; ++q) {
    const int idx = (wave + 4 * q) * 16 + (lane & 15);
    const int oh = oh0 + idx / TC, ow = ow0 + idx % TC;
    if (oh >= p.ho || ow >= p.wo) continue;
    const int64_t base = static_cast<int64_t>(n) * p.y_sn + static_cast<int64_t>(oh * p.wo + ow) * p.y_sp;
#pragma unroll
    for (int mf = 0; mf < C::MF; ++mf) {
      const int co = mf * 16 + kq * 4;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = acc[mf][q][j] * (p.scale != nullptr ? p.scale[co + j] : 1.f) + p.shift[co + j];
        if (p.relu) v[j] = fmaxf(v[j], 0.f);
      }
      uint2 o;
      o.x = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
      o.y = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      *reinterpret_cast<uint2*>(y + base + co) = o;
    }
  }
}

template <int CIN, int COUT, int KS, int S, int TR, int TC, bool SRC_U8>
hipError_t launch_patch(const drnmi_conv_args& p, hipStream_t s) {
  const int64_t tiles = static_cast<int64_t>(p.n) * ((p.ho + TR - 1) / TR) * ((p.wo + TC - 1) / TC);
  hipLaunchKernelGGL((patch_conv_kernel<CIN, COUT, KS, S, TR, TC, SRC_U8>), dim3(static_cast<unsigned>(tiles)),
                     dim3(kThreads), 0, s, p);
  return hipGetLastError();
}

}  // namespace

int patch_conv_dispatch(const drnmi_conv_args& p, hipStream_t s) {
  if (p.dtype != DRNMI_BF16 || p.out_dtype != DRNMI_BF16 || p.dil != 1 || p.res != nullptr) return DRNMI_ENOTSUP;
  if (p.y_sc != 1 || p.y_sp != p.cout) return DRNMI_ENOTSUP;            // packed NHWC output
  hipError_t e;
  if (p.src_u8) {
    if (p.cin != 4 || p.cout != 16 || p.ks != 7 || p.stride != 1 || p.k != 224 || p.k_pad != 224)
      return DRNMI_ENOTSUP;
    e = launch_patch<4, 16, 7, 1, 4, 64, true>(p, s);
  } else if (p.cin == 8 && p.cout == 16 && p.ks == 7 && p.stride == 1) {
    e = launch_patch<8, 16, 7, 1, 4, 64, false>(p, s);
  } else if (p.cin == 16 && p.cout == 16 && p.ks == 3 && p.stride == 1) {
    e = launch_patch<16, 16, 3, 1, 4, 64, false>(p, s);
  } else if (p.cin == 16 && p.cout == 32 && p.ks == 3 && p.stride == 2) {
    e = launch_patch<16, 32, 3, 2, 4, 64, false>(p, s);
  } else if (p.cin == 32 && p.cout == 64 && p.ks == 3 && p.stride == 2) {
    e = launch_patch<32, 64, 3, 2, 2, 64, false>(p, s);
  } else {
    return DRNMI_ENOTSUP;
  }
  return static_cast<int>(e);
}

const char* patch_conv_name(const drnmi_conv_args& p) {
  if (p.src_u8) return "patch_conv_kernel<4, 16, 7, 1, 4, 64, true>";
  if (p.cin == 8 && p.cout == 16 && p.ks == 7) return "patch_conv_kernel<8, 16, 7, 1, 4, 64, false>";
  if (p.cin == 16 && p.cout == 16 && p.ks == 3 && p.stride == 1) return "patch_conv_kernel<16, 16, 3, 1, 4, 64, false>";
  if (p.cin == 16 && p.cout == 32 && p.ks == 3 && p.stride == 2) return "patch_conv_kernel<16, 32, 3, 2, 4, 64, false>";
  if (p.cin == 32 && p.cout == 64 && p.ks == 3 && p.stride == 2) return "patch_conv_kernel<32, 64, 3, 2, 2, 64, false>";
  return nullptr;
}

}  // namespace drnmi
