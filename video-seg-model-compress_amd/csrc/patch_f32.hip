// Exact-fp32 small-channel convs through an LDS input patch (f32-input MFMA): the fp32
// parity mode's full-resolution layers.
//
// DRN-D's layer0 (7x7 3->16, lmodels/drn.py:132-137), layer1 (3x3 16->16) and layer2 (3x3 s2
// 16->32, :201-211) carry ~5 % of D-22's FLOPs at 2M pixels per frame.  On the generic f32
// implicit GEMM (conv_igemm, 256-row output tiles) 15/16 of every MFMA row block was padding
// for these 16-channel outputs (3-9 TFLOP/s, 43 ms of a 120 ms fp32 step).  Here:
//
// * MFMA orientation: v_mfma_f32_16x16x4_f32 with A = weights (16 output channels x 4 K) and
//   B = 4 K x 16 pixels.  Lane (col = l & 15, kq = l >> 4) supplies W[co = col][k] and
//   x[pixel col][k] for the step's k; the accumulator gives the lane channels 4 kq .. + 3 of
//   pixel col, i.e. one 16-B NHWC store per lane and 16 pixels x 64 B contiguous per row of lanes.
// * K order = conv_igemm's f32 order, so the outputs are bit-identical to the implicit GEMM they
//   replace (and the fp32 labels stay exactly as validated): K runs in 32-deep blocks; in block t,
//   MFMA step j takes k = 32 t + 8 kq + j from lane group kq, j = 0..7 (conv_igemm.hip mma_step
//   <float>).  So lane kq reads 8 consecutive k per block: for 16-channel inputs (k = tap * 16 + ci)
//   half a pixel of tap 2 t + kq / 2 (two ds_read_b128; 5 blocks = 40 MFMAs per 16 x 16 output
//   block for the 144-deep K, the last block half zero-padded as conv_igemm's).  For the 3-channel
//   stem (k = tap * 8 + ci on the NHWC8 input) lane kq's block is tap 4 t + kq, and the steps
//   j >= 3 multiply zero inputs by zero weights in all four lanes groups: fma(0, 0, acc) = acc
//   (acc is never -0 starting from +0), so they are skipped (13 blocks x 3 = 39 MFMAs); a pixel is
//   4 floats in LDS (channel 3 = 0), one ds_read_b128 per block.
// * The stem reads the uint8 HWC3 frame and normalises on load with the reference op order
//   ((c / 255 - mean) / std, ToTensorVideoImage + Normalize, data_transforms.py:109-125,
//   :256-281), the same fp32 sequence as drnmi_frame_ingest_u8 (bit-identical inputs).
// * Persistent workgroups: the next tile's input is loaded into registers while the current one
//   computes; several workgroups per CU overlap one's barrier / staging with another's MFMAs.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace drnmi {
namespace {

constexpr int kF32Threads = 256;

// SRC: 0 = uint8 HWC3 frames (normalised on load), 1 = fp32 NHWC8 (channels 0..3 staged),
//      2 = fp32 NHWC16
template <int SRC, int COUT, int KS, int S, int TR, int TC>
struct F32Cfg {
  static constexpr int CP = SRC == 2 ? 16 : 4;              // floats per LDS pixel
  static constexpr int XS = SRC == 2 ? 16 : 8;              // input channel stride (SRC 1, 2)
  static constexpr int PR = (TR - 1) * S + KS;               // patch rows
  static constexpr int PC = (TC - 1) * S + KS;               // patch columns
  static constexpr int NG = SRC == 2 ? (KS * KS + 1) / 2 : (KS * KS + 3) / 4;   // 32-deep K blocks
  static constexpr int NS = SRC == 2 ? 8 : 3;                // MFMA steps per block
  static constexpr int MF = COUT / 16;                       // output-channel fragments
  static constexpr int PFW = TR * TC / 64;                   // 16-pixel fragments per wave
  static constexpr int UPP = CP / 4;                         // 16-B units per pixel
  static constexpr int NUNITS = PR * PC * (SRC == 0 ? 1 : UPP);
  static constexpr int NPT = (NUNITS + kF32Threads - 1) / kF32Threads;
  static constexpr int LDS_FLOATS = PR * PC * CP;
  static_assert(TC % 16 == 0 && (TR * TC) % 64 == 0, "whole 16-pixel fragments over 4 waves");
  static_assert(COUT % 16 == 0, "16-channel output fragments");
};

template <int SRC, int COUT, int KS, int S, int TR, int TC>
__global__ void __launch_bounds__(kF32Threads)
patch_f32_kernel(const drnmi_conv_args p) {
  using C = F32Cfg<SRC, COUT, KS, S, TR, TC>;
  __shared__ __attribute__((aligned(16))) float patch[C::LDS_FLOATS];
  using Unit = typename std::conditional<SRC == 0, uint32_t, float4>::type;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int col = lane & 15;
  const int kq = lane >> 4;
  const int tiles_w = (p.wo + TC - 1) / TC;
  const int tiles_h = (p.ho + TR - 1) / TR;
  const int ntiles = p.n * tiles_w * tiles_h;

  // ---- weights -> registers: step (t, j) of this lane is W[mf*16 + col][k], k = 32 t + 8 kq + j in
  //   conv_igemm's layouts: k = tap * 16 + ci (SRC 2), tap * 8 + ci (SRC 1); the fused-ingest stem's
  //   packing k = kh * 32 + kw * 4 + ci (STEM_U8_K) holds the same weights (SRC 0)
  const float* __restrict__ wt = reinterpret_cast<const float*>(p.wgt);
  float wa[C::MF][C::NG][C::NS];
  int koff[C::NG];                         // this lane's LDS float offset in block t (from the fragment pixel)
  bool kon[C::NG];                         // the block's tap exists for this lane (else zero weights and input)
#pragma unroll
  for (int t = 0; t < C::NG; ++t) {
    int kbase = -1;
    const int tap = SRC == 2 ? 2 * t + (kq >> 1) : 4 * t + kq;
    const int kh = tap / KS, kw = tap % KS;
    kon[t] = tap < KS * KS;
    koff[t] = kon[t] ? (kh * C::PC + kw) * C::CP + (SRC == 2 ? 8 * (kq & 1) : 0) : 0;
    if (kon[t]) kbase = SRC == 2 ? 32 * t + 8 * kq : SRC == 1 ? tap * 8 : kh * 32 + kw * 4;
#pragma unroll
    for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
      for (int j = 0; j < C::NS; ++j)
        wa[mf][t][j] = kbase >= 0 ? wt[static_cast<int64_t>(mf * 16 + col) * p.k_pad + kbase + j] : 0.f;
  }
  float sc[C::MF][4], sh[C::MF][4];
#pragma unroll
  for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = mf * 16 + kq * 4 + j;
      sc[mf][j] = p.scale != nullptr ? p.scale[co] : 1.f;
      sh[mf][j] = p.shift[co];
    }

  // ---- input patch of a tile -> registers (outside the image: zeros = the conv's padding)
  Unit stage[C::NPT];
  auto load_tile = [&](int b) {
    const int n = b / (tiles_w * tiles_h);
    const int rem = b - n * tiles_w * tiles_h;
    const int ih0 = (rem / tiles_w) * TR * S - p.pad;
    const int iw0 = (rem % tiles_w) * TC * S - p.pad;
#pragma unroll
    for (int u = 0; u < C::NPT; ++u) {
      const int i = tid + u * kF32Threads;
      if constexpr (SRC == 0) {
        const int pr = i / C::PC, pc = i - pr * C::PC;
        const int ih = ih0 + pr, iw = iw0 + pc;
        uint32_t v = 0xffffffffu;                 // marks a padded pixel
        if (i < C::NUNITS && static_cast<unsigned>(ih) < static_cast<unsigned>(p.h) &&
            static_cast<unsigned>(iw) < static_cast<unsigned>(p.w)) {
          const uint8_t* px = reinterpret_cast<const uint8_t*>(p.x) +
                              ((static_cast<int64_t>(n) * p.h + ih) * p.w + iw) * 3;
          v = static_cast<uint32_t>(px[0]) | (static_cast<uint32_t>(px[1]) << 8) |
              (static_cast<uint32_t>(px[2]) << 16);
        }
        stage[u] = v;
      } else {
        const int pix = i / C::UPP, v4 = i - pix * C::UPP;
        const int pr = pix / C::PC, pc = pix - pr * C::PC;
        const int ih = ih0 + pr, iw = iw0 + pc;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < C::NUNITS && static_cast<unsigned>(ih) < static_cast<unsigned>(p.h) &&
            static_cast<unsigned>(iw) < static_cast<unsigned>(p.w))
          v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.x) +
                                               ((static_cast<int64_t>(n) * p.h + ih) * p.w + iw) * C::XS + v4 * 4);
        stage[u] = v;
      }
    }
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int u = 0; u < C::NPT; ++u) {
      const int i = tid + u * kF32Threads;
      if (i >= C::NUNITS) break;
      if constexpr (SRC == 0) {
        // reference normalisation, same fp32 op order (data_transforms.py:109-125, :256-281)
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (stage[u] != 0xffffffffu) {
          float c0 = static_cast<float>(stage[u] & 0xff), c1 = static_cast<float>((stage[u] >> 8) & 0xff),
                c2 = static_cast<float>((stage[u] >> 16) & 0xff);
          if (p.bgr) { const float t = c0; c0 = c2; c2 = t; }
          v.x = (c0 / 255.0f - p.mean[0]) / p.std[0];
          v.y = (c1 / 255.0f - p.mean[1]) / p.std[1];
          v.z = (c2 / 255.0f - p.mean[2]) / p.std[2];
        }
        *reinterpret_cast<float4*>(patch + i * 4) = v;
      } else if constexpr (SRC == 1) {
        float4 v = stage[u];
        v.w = 0.f;                                   // channel 3 of the NHWC8 input (zero padding)
        *reinterpret_cast<float4*>(patch + i * 4) = v;
      } else {
        *reinterpret_cast<float4*>(patch + i * 4) = stage[u];
      }
    }
  };

  int pbase[C::PFW];                                 // fragment pixel's LDS float offset
#pragma unroll
  for (int q = 0; q < C::PFW; ++q) {
    const int idx = (wave + 4 * q) * 16 + col;
    pbase[q] = ((idx / TC) * S * C::PC + (idx % TC) * S) * C::CP;
  }

  int b = blockIdx.x;
  if (b < ntiles) load_tile(b);
  for (; b < ntiles; b += gridDim.x) {
    __syncthreads();                                 // every wave done reading the previous patch
    store_patch();
    __syncthreads();
    if (b + static_cast<int>(gridDim.x) < ntiles) load_tile(b + gridDim.x);   // in flight under the MFMAs

    f32x4 acc[C::MF][C::PFW];
#pragma unroll
    for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
      for (int q = 0; q < C::PFW; ++q) acc[mf][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < C::NG; ++t) {
      float xv[C::PFW][8];
#pragma unroll
      for (int q = 0; q < C::PFW; ++q) {
        const float* src = patch + pbase[q] + koff[t];
        const float4 lo = *reinterpret_cast<const float4*>(src);
        xv[q][0] = lo.x; xv[q][1] = lo.y; xv[q][2] = lo.z; xv[q][3] = lo.w;
        if constexpr (C::NS == 8) {
          const float4 hi = *reinterpret_cast<const float4*>(src + 4);
          xv[q][4] = hi.x; xv[q][5] = hi.y; xv[q][6] = hi.z; xv[q][7] = hi.w;
        }
        if (!kon[t])                         // past the last tap: zero input, as conv_igemm loads it
#pragma unroll
          for (int j = 0; j < C::NS; ++j) xv[q][j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < C::NS; ++j)
#pragma unroll
        for (int q = 0; q < C::PFW; ++q)
#pragma unroll
          for (int mf = 0; mf < C::MF; ++mf)
            acc[mf][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[mf][t][j], xv[q][j], acc[mf][q], 0, 0, 0);
    }

    // ---- epilogue: lane owns channels mf*16 + 4 kq .. + 3 of pixel col of each fragment
    const int n = b / (tiles_w * tiles_h);
    const int rem = b - n * tiles_w * tiles_h;
    const int oh0 = (rem / tiles_w) * TR;
    const int ow0 = (rem % tiles_w) * TC;
#pragma unroll
    for (int q = 0; q < C::PFW; ++q) {
      const int idx = (wave + 4 * q) * 16 + col;
      const int oh = oh0 + idx / TC, ow = ow0 + idx % TC;
      if (oh >= p.ho || ow >= p.wo) continue;
      float* yp = reinterpret_cast<float*>(p.y) + static_cast<int64_t>(n) * p.y_sn +
                  static_cast<int64_t>(oh * p.wo + ow) * p.y_sp;
#pragma unroll
      for (int mf = 0; mf < C::MF; ++mf) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = acc[mf][q][j] * sc[mf][j] + sh[mf][j];
          if (p.relu) v[j] = fmaxf(v[j], 0.f);
        }
        *reinterpret_cast<float4*>(yp + mf * 16 + kq * 4) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

template <int SRC, int COUT, int KS, int S, int TR, int TC>
hipError_t launch_patch_f32(const drnmi_conv_args& p, hipStream_t s) {
  static int slots = 0;
  auto kern = patch_f32_kernel<SRC, COUT, KS, S, TR, TC>;
  if (slots == 0) {
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(kern), kF32Threads, 0) !=
            hipSuccess || blocks <= 0)
      blocks = 1;
    slots = cus * blocks;
  }
  const int64_t tiles = static_cast<int64_t>(p.n) * ((p.ho + TR - 1) / TR) * ((p.wo + TC - 1) / TC);
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(tiles < slots ? tiles : slots)), dim3(kF32Threads), 0, s, p);
  return hipGetLastError();
}

}  // namespace

// Shapes (dtype = out_dtype = DRNMI_F32, packed NHWC output, no residual, dilation 1):
//   src_u8, cin 4, 7x7 3->16 s1 p3, k = k_pad = 224 (STEM_U8_K: kh*32 + kw*4 + c)
//   cin 8, 7x7 3->16 s1 p3, k = 392 (NHWC8 input)
//   cin 16, 3x3 16->16 s1 p1, k = 144
//   cin 16, 3x3 16->32 s2 p1, k = 144
static int f32_shape(const drnmi_conv_args& p) {
  if (p.dtype != DRNMI_F32 || p.out_dtype != DRNMI_F32 || p.dil != 1 || p.res != nullptr || p.y_sc != 1 ||
      p.y_sp != p.cout || p.cout_pad < p.cout)
    return -1;
  if (p.src_u8)
    return (p.cin == 4 && p.cout == 16 && p.ks == 7 && p.stride == 1 && p.pad == 3 && p.k == 224 && p.k_pad == 224) ? 0
                                                                                                                  : -1;
  if (p.cin == 8 && p.cout == 16 && p.ks == 7 && p.stride == 1 && p.pad == 3 && p.k == 392 && p.k_pad >= 392) return 1;
  if (p.cin == 16 && p.cout == 16 && p.ks == 3 && p.stride == 1 && p.pad == 1 && p.k == 144 && p.k_pad >= 144) return 2;
  if (p.cin == 16 && p.cout == 32 && p.ks == 3 && p.stride == 2 && p.pad == 1 && p.k == 144 && p.k_pad >= 144) return 3;
  return -1;
}

int patch_f32_dispatch(const drnmi_conv_args& p, hipStream_t s) {
  hipError_t e;
  switch (f32_shape(p)) {
    case 0: e = launch_patch_f32<0, 16, 7, 1, 4, 64>(p, s); break;
    case 1: e = launch_patch_f32<1, 16, 7, 1, 4, 64>(p, s); break;
    case 2: e = launch_patch_f32<2, 16, 3, 1, 4, 64>(p, s); break;
    case 3: e = launch_patch_f32<2, 32, 3, 2, 4, 32>(p, s); break;
    default: return DRNMI_ENOTSUP;
  }
  return static_cast<int>(e);
}

const char* patch_f32_name(const drnmi_conv_args& p) {
  switch (f32_shape(p)) {
    case 0: return "patch_f32_kernel<0, 16, 7, 1, 4, 64>";
    case 1: return "patch_f32_kernel<1, 16, 7, 1, 4, 64>";
    case 2: return "patch_f32_kernel<2, 16, 3, 1, 4, 64>";
    case 3: return "patch_f32_kernel<2, 32, 3, 2, 4, 32>";
    default: return nullptr;
  }
}

}  // namespace drnmi
