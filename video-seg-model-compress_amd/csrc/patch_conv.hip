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
#include <type_traits>

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


// X6 (fp32x mode, dtype DRNMI_F32X3): fp32 input patch in LDS, weights as three bf16 planes in
// registers, every B fragment split exactly into three bf16 terms and the six products above
// 2^-24 accumulated in fp32 (csrc/conv_x6.hip has the derivation); fp32 NHWC output.
template <int CIN, int COUT, int KS, int S, int TR, int TC, bool SRC_U8, bool X6 = false>
__global__ void __launch_bounds__(kThreads)
patch_conv_kernel(const drnmi_conv_args p) {
  using C = PatchCfg<CIN, COUT, KS, S, TR, TC, SRC_U8>;
  using PT = typename std::conditional<X6, float, bf16_t>::type;
  __shared__ __attribute__((aligned(16))) PT patch[C::LDS_ELEMS];
  // Persistent: each workgroup walks tiles blockIdx.x, +gridDim.x, ...  The next tile's
  // input is loaded into registers while the current one computes (the 4x64-pixel tiles are
  // too short-lived to pay a workgroup dispatch each).
  constexpr int EPU = X6 ? 4 : 8;                           // elements per 16-B unit
  constexpr int NPL = X6 ? 3 : 1;                           // weight planes
  constexpr int VPP = SRC_U8 ? 1 : CIN / EPU;               // staged units per pixel
  constexpr int NUNITS = C::PR * C::PC * VPP;
  constexpr int NPT = (NUNITS + kThreads - 1) / kThreads;    // per thread
  using Unit = typename std::conditional<SRC_U8, uint32_t, uint4>::type;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tiles_w = (p.wo + TC - 1) / TC;
  const int tiles_h = (p.ho + TR - 1) / TR;
  const int ntiles = p.n * tiles_w * tiles_h;

  // ---- weights -> registers: A fragment (mf, ks) = W[mf*16 + lane&15][ks*32 + 8*(lane>>4) ..+7]
  const bf16_t* __restrict__ wt = reinterpret_cast<const bf16_t*>(p.wgt);
  const int64_t plane = static_cast<int64_t>(p.cout_pad) * p.k_pad;
  bf16x8 wa[NPL][C::MF][C::NK];
#pragma unroll
  for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
    for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
      for (int ks = 0; ks < C::NK; ++ks)
        wa[pl][mf][ks] = *reinterpret_cast<const bf16x8*>(
            wt + pl * plane + static_cast<int64_t>(mf * 16 + (lane & 15)) * p.k_pad + ks * 32 + 8 * (lane >> 4));

  // ---- input patch of a tile -> registers (zero outside the image = the conv's padding)
  Unit stage[NPT];
  auto load_tile = [&](int b) {
    const int n = b / (tiles_w * tiles_h);
    const int rem = b - n * tiles_w * tiles_h;
    const int ih0 = (rem / tiles_w) * TR * S - p.pad;
    const int iw0 = (rem % tiles_w) * TC * S - p.pad;
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = tid + u * kThreads;
      const int pix = i / VPP, v8 = i - pix * VPP;
      const int pr = pix / C::PC, pc = pix - pr * C::PC;
      const int ih = ih0 + pr, iw = iw0 + pc;
      const bool ok = i < NUNITS && static_cast<unsigned>(ih) < static_cast<unsigned>(p.h) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(p.w);
      if constexpr (SRC_U8) {
        uint32_t v = 0xffffffffu;                      // marks a padded pixel
        if (ok) {
          const uint8_t* px = reinterpret_cast<const uint8_t*>(p.x) +
                              ((static_cast<int64_t>(n) * p.h + ih) * p.w + iw) * 3;
          v = static_cast<uint32_t>(px[0]) | (static_cast<uint32_t>(px[1]) << 8) |
              (static_cast<uint32_t>(px[2]) << 16);
        }
        stage[u] = v;
      } else {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (ok)
          v = *reinterpret_cast<const uint4*>(reinterpret_cast<const PT*>(p.x) +
                                              ((static_cast<int64_t>(n) * p.h + ih) * p.w + iw) * CIN + v8 * EPU);
        stage[u] = v;
      }
    }
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = tid + u * kThreads;
      if (i >= NUNITS) break;
      if constexpr (SRC_U8) {
        // reference normalisation, same fp32 op order (data_transforms.py:109-125, :256-281)
        float v0 = 0.f, v1 = 0.f, v2 = 0.f;
        if (stage[u] != 0xffffffffu) {
          float c0 = static_cast<float>(stage[u] & 0xff), c1 = static_cast<float>((stage[u] >> 8) & 0xff),
                c2 = static_cast<float>((stage[u] >> 16) & 0xff);
          if (p.bgr) { const float t = c0; c0 = c2; c2 = t; }
          v0 = (c0 / 255.0f - p.mean[0]) / p.std[0];
          v1 = (c1 / 255.0f - p.mean[1]) / p.std[1];
          v2 = (c2 / 255.0f - p.mean[2]) / p.std[2];
        }
        if constexpr (X6) {
          *reinterpret_cast<float4*>(patch + i * 4) = make_float4(v0, v1, v2, 0.f);
        } else {
          uint2 v = make_uint2(0, 0);
          if (stage[u] != 0xffffffffu) {
            v.x = static_cast<uint32_t>(f32_to_bf16(v0)) | (static_cast<uint32_t>(f32_to_bf16(v1)) << 16);
            v.y = static_cast<uint32_t>(f32_to_bf16(v2));
          }
          *reinterpret_cast<uint2*>(patch + i * 4) = v;
        }
      } else {
        *reinterpret_cast<uint4*>(patch + i * EPU) = stage[u];
      }
    }
  };

  int prow[C::PFW], pcol[C::PFW];
#pragma unroll
  for (int q = 0; q < C::PFW; ++q) {
    const int idx = (wave + 4 * q) * 16 + (lane & 15);
    prow[q] = (idx / TC) * S;
    pcol[q] = (idx % TC) * S;
  }
  const int kq = lane >> 4;

  int b = blockIdx.x;
  if (b < ntiles) load_tile(b);
  for (; b < ntiles; b += gridDim.x) {
    __syncthreads();               // every wave done reading the previous patch
    store_patch();
    __syncthreads();
    if (b + static_cast<int>(gridDim.x) < ntiles) load_tile(b + gridDim.x);   // in flight during the MFMAs

    // ---- MFMA: this wave's pixel fragments pf = wave + 4*q
    f32x4 acc[C::MF][C::PFW];
#pragma unroll
    for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
      for (int q = 0; q < C::PFW; ++q) acc[mf][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < C::NK; ++ks) {
#pragma unroll
      for (int q = 0; q < C::PFW; ++q) {
        // the lane's 8 K elements of this pixel fragment: 16 B (bf16) or 32 B (fp32) of the patch
        const PT* src = nullptr;
        if constexpr (SRC_U8) {
          // k = kh*32 + kw*4 + c: step ks = kernel row kh, fragment = taps kw = 2kq, 2kq+1
          src = patch + ((prow[q] + ks) * C::PC + pcol[q] + 2 * kq) * 4;
        } else {
          const int k0 = ks * 32 + 8 * kq;
          const int tap = k0 / CIN;
          const int ci = k0 % CIN;
          if (tap < KS * KS) {
            const int kh = tap / KS, kw = tap % KS;
            src = patch + ((prow[q] + kh) * C::PC + pcol[q] + kw) * CIN + ci;
          }
        }
        if constexpr (X6) {
          float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
          if (src != nullptr) {
            lo = *reinterpret_cast<const float4*>(src);
            hi = *reinterpret_cast<const float4*>(src + 4);
          }
          bf16x8 b1, b2, b3;
          split3(lo, hi, b1, b2, b3);
#pragma unroll
          for (int mf = 0; mf < C::MF; ++mf) {
            f32x4 a = acc[mf][q];
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[2][mf][ks], b1, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[1][mf][ks], b2, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][mf][ks], b3, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[1][mf][ks], b1, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][mf][ks], b2, a, 0, 0, 0);
            acc[mf][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][mf][ks], b1, a, 0, 0, 0);
          }
        } else {
          bf16x8 bv = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
          if constexpr (SRC_U8) {
            const uint2 lo = *reinterpret_cast<const uint2*>(src);
            const uint2 hi = *reinterpret_cast<const uint2*>(src + 4);
            bv = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
          } else if (src != nullptr) {
            bv = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(src));
          }
#pragma unroll
          for (int mf = 0; mf < C::MF; ++mf)
            acc[mf][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][mf][ks], bv, acc[mf][q], 0, 0, 0);
        }
      }
    }

    // ---- epilogue: lane owns channels co..co+3 of one pixel
    const int n = b / (tiles_w * tiles_h);
    const int rem = b - n * tiles_w * tiles_h;
    const int oh0 = (rem / tiles_w) * TR;
    const int ow0 = (rem % tiles_w) * TC;
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
        if constexpr (X6) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.y) + base + co) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          uint2 o;
          o.x = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
          o.y = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.y) + base + co) = o;
        }
      }
    }
  }
}

// ---- LDS-DMA multi-buffered variant for bf16 inputs (layer1 16->16, layer2 16->32 s2).
//
// Persistent workgroups walk their tiles with NB patch buffers in LDS: the patch of tile
// t+NB-1 is DMA'd (buffer_load ... lds, no VGPR round trip, out-of-image pixels = an
// out-of-range buffer offset, which the hardware returns as zeros) while tile t computes.
// A patch is PR rows of PC*CIN*2 contiguous bytes in both global memory and LDS, so a 1-KB
// DMA piece is 64 x 16 B of consecutive patch bytes; each wave issues the same number of
// pieces and of (buffer, out-of-range-dropping) stores per tile, so one counted vmcnt per
// tile retires exactly the patch about to be read.
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

template <int CIN, int COUT, int S, int TR, int TC>
struct DmaCfg {
  static constexpr int PR = (TR - 1) * S + 3;
  static constexpr int PC = (TC - 1) * S + 3;
  static constexpr int ROWB = PC * CIN * 2;                   // bytes per patch row
  static constexpr int PB = (PR * ROWB + 4095) / 4096 * 4096;  // buffer bytes (whole 4-KB rounds)
  static constexpr int P = PB / 4096;                          // DMA pieces per wave per tile
  static constexpr int NB = 3;                                 // patch buffers
  static constexpr int K = 9 * CIN;
  static constexpr int NK = (K + 31) / 32;
  static constexpr int MF = COUT / 16;
  static constexpr int PFW = TR * TC / 16 / 4;                 // pixel fragments per wave
  static constexpr int ST = PFW * (MF % 2 == 0 ? MF / 2 : MF);   // stores per lane per tile (16-B pieces for even MF)
  static constexpr int LDS = NB * PB;
  static_assert(TR * TC % 64 == 0, "tile must split over 4 waves");
};

template <int CIN, int COUT, int S, int TR, int TC>
__global__ void __launch_bounds__(kThreads)
patch_dma_kernel(const drnmi_conv_args p) {
  using C = DmaCfg<CIN, COUT, S, TR, TC>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int kq = lane >> 4;
  const int tiles_w = (p.wo + TC - 1) / TC;
  const int tiles_h = (p.ho + TR - 1) / TR;
  const int ntiles = p.n * tiles_w * tiles_h;
  const int H = p.h, W = p.w;

  const bf16_t* __restrict__ wt = reinterpret_cast<const bf16_t*>(p.wgt);
  bf16x8 wa[C::MF][C::NK];
#pragma unroll
  for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
    for (int ks = 0; ks < C::NK; ++ks)
      wa[mf][ks] = *reinterpret_cast<const bf16x8*>(
          wt + static_cast<int64_t>(mf * 16 + (lane & 15)) * p.k_pad + ks * 32 + 8 * (lane >> 4));
  float sc[C::MF][4], sh[C::MF][4];
#pragma unroll
  for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = mf * 16 + kq * 4 + j;
      sc[mf][j] = p.scale != nullptr ? p.scale[co] : 1.f;
      sh[mf][j] = p.shift[co];
    }

  // DMA pieces: tile-independent (row, column, byte) of this lane's 16 bytes in each piece
  int pc_r[C::P], pc_c[C::P], pc_off[C::P];
#pragma unroll
  for (int j = 0; j < C::P; ++j) {
    const int off = (j * 4 + wave) * 1024 + lane * 16;
    const int r = off / C::ROWB;
    const int rb = off - r * C::ROWB;
    const int c = rb / (CIN * 2);
    pc_r[j] = r < C::PR ? r : (1 << 20);                     // slack bytes: out of range
    pc_c[j] = c;
    pc_off[j] = (r * W + c) * CIN * 2 + (rb - c * CIN * 2);
  }
  const int64_t frame_bytes = static_cast<int64_t>(H) * W * CIN * 2;
  auto issue = [&](int b, int buf) {
    const int n = b / (tiles_w * tiles_h);
    const int rem = b - n * tiles_w * tiles_h;
    const int ih0 = (rem / tiles_w) * TR * S - p.pad;
    const int iw0 = (rem % tiles_w) * TC * S - p.pad;
    const char* fb = reinterpret_cast<const char*>(p.x) + static_cast<int64_t>(n) * frame_bytes;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(fb), 0, static_cast<int>(frame_bytes), 0x00020000);
    const int base = (ih0 * W + iw0) * CIN * 2;
#pragma unroll
    for (int j = 0; j < C::P; ++j) {
      const bool ok = static_cast<unsigned>(ih0 + pc_r[j]) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(iw0 + pc_c[j]) < static_cast<unsigned>(W);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(smem + buf * C::PB + (j * 4 + wave) * 1024), 16,
          ok ? static_cast<unsigned>(base + pc_off[j]) : 0xffffffffu, 0, 0, 0);
    }
  };

  int prow[C::PFW], pcol[C::PFW];
#pragma unroll
  for (int q = 0; q < C::PFW; ++q) {
    const int idx = (wave + 4 * q) * 16 + (lane & 15);
    prow[q] = (idx / TC) * S;
    pcol[q] = (idx % TC) * S;
  }
  int boff[C::NK];                                  // B fragment byte offset of (ks, this lane)
#pragma unroll
  for (int ks = 0; ks < C::NK; ++ks) {
    const int k0 = ks * 32 + 8 * kq;
    const int tap = k0 / CIN, ci = k0 % CIN;
    boff[ks] = tap < 9 ? (((tap / 3) * C::PC + tap % 3) * CIN + ci) * 2 : -1;
  }
  const int64_t ybytes = static_cast<int64_t>(p.n) * p.ho * p.wo * COUT * 2;
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
      p.y, 0, static_cast<int>(ybytes < 0x7fffffff ? ybytes : 0x7fffffff), 0x00020000);

  const int b0 = blockIdx.x;
  const int G = gridDim.x;
  if (b0 < ntiles) issue(b0, 0);
  if (b0 + G < ntiles) issue(b0 + G, 1);
  int t = 0;
  for (int b = b0; b < ntiles; b += G, ++t) {
    // retire tile t's patch: younger ops are stores(t-2), DMA(t+1), stores(t-1)
    if (t >= 2 && b + G < ntiles) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::P + 2 * C::ST) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (b + 2 * G < ntiles) issue(b + 2 * G, (t + 2) % C::NB);
    const char* pt = smem + (t % C::NB) * C::PB;

    f32x4 acc[C::MF][C::PFW];
#pragma unroll
    for (int mf = 0; mf < C::MF; ++mf)
#pragma unroll
      for (int q = 0; q < C::PFW; ++q) acc[mf][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < C::NK; ++ks) {
#pragma unroll
      for (int q = 0; q < C::PFW; ++q) {
        bf16x8 bv = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
        if (boff[ks] >= 0)
          bv = *reinterpret_cast<const bf16x8*>(pt + boff[ks] + (prow[q] * C::PC + pcol[q]) * CIN * 2);
#pragma unroll
        for (int mf = 0; mf < C::MF; ++mf)
          acc[mf][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[mf][ks], bv, acc[mf][q], 0, 0, 0);
      }
    }

    const int n = b / (tiles_w * tiles_h);
    const int rem = b - n * tiles_w * tiles_h;
    const int oh0 = (rem / tiles_w) * TR;
    const int ow0 = (rem % tiles_w) * TC;
#pragma unroll
    for (int q = 0; q < C::PFW; ++q) {
      const int idx = (wave + 4 * q) * 16 + (lane & 15);
      const int oh = oh0 + idx / TC, ow = ow0 + idx % TC;
      const bool ok = oh < p.ho && ow < p.wo;
      const int64_t pix = (static_cast<int64_t>(n) * p.ho + oh) * p.wo + ow;
      uint32_t w[C::MF][2];
#pragma unroll
      for (int mf = 0; mf < C::MF; ++mf) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = acc[mf][q][j] * sc[mf][j] + sh[mf][j];
          if (p.relu) v[j] = fmaxf(v[j], 0.f);
        }
        w[mf][0] = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
        w[mf][1] = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      }
      // every lane issues the store (out-of-range offset = dropped): constant vmcnt per tile
      if constexpr (C::MF % 2 == 0) {
        // 16-B pieces: 64 contiguous bytes per pixel per instruction (common.h swap_halves)
#pragma unroll
        for (int f2 = 0; f2 < C::MF / 2; ++f2) {
          uint4 o = make_uint4(w[2 * f2][0], w[2 * f2][1], w[2 * f2 + 1][0], w[2 * f2 + 1][1]);
          swap_halves(o);
          const unsigned yoff = ok ? static_cast<unsigned>((pix * COUT + f2 * 32 + chunk_of_row(kq) * 8) * 2) : 0xffffffffu;
          typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
          const u32x4_t ov = {o.x, o.y, o.z, o.w};
          __builtin_amdgcn_raw_buffer_store_b128(ov, ys, yoff, 0, 0);
        }
      } else {
#pragma unroll
        for (int mf = 0; mf < C::MF; ++mf) {
          u32x2_t o;
          o.x = w[mf][0];
          o.y = w[mf][1];
          const unsigned yoff = ok ? static_cast<unsigned>((pix * COUT + mf * 16 + kq * 4) * 2) : 0xffffffffu;
          __builtin_amdgcn_raw_buffer_store_b64(o, ys, yoff, 0, 0);
        }
      }
    }
  }
}

// ---- Fused-ingest stem, LDS-DMA pipelined (uint8 HWC3 frames -> 7x7 conv 3->16).
//
// Raw frame bytes are DMA'd (buffer_load_dword ... lds, 4 bytes per lane, one patch row per
// wave instruction, dword-aligned below the row start) two tiles ahead into a 3-slot ring;
// each tile then converts its raw rows into the normalised bf16 patch through a per-channel
// 256-entry table that the workgroup builds once with the reference op order
// ((c / 255 - mean) / std, data_transforms.py:109-125, :256-281), so the conversion is
// bit-identical to the per-pixel division and costs three LDS lookups per pixel.
constexpr int kStemTR = 4, kStemTC = 64;
constexpr int kStemPR = kStemTR + 6, kStemPC = kStemTC + 7;     // +1: the zero kw=7 tap
constexpr int kStemRows = 12;                                    // 3 row loads per wave
constexpr int kStemRawB = kStemRows * 256;                       // one ring slot
constexpr int kStemPatchB = kStemPR * kStemPC * 8;
constexpr int kStemLDS = 3 * kStemRawB + kStemPatchB + 3 * 256 * 2;

__global__ void __launch_bounds__(kThreads)
stem_dma_kernel(const drnmi_conv_args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* raw = smem;
  bf16_t* patch = reinterpret_cast<bf16_t*>(smem + 3 * kStemRawB);
  bf16_t* lut = reinterpret_cast<bf16_t*>(smem + 3 * kStemRawB + kStemPatchB);
  constexpr int NK = 7, PFW = 4, ST = PFW;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int kq = lane >> 4;
  const int H = p.h, W = p.w;
  const int tiles_w = (p.wo + kStemTC - 1) / kStemTC;
  const int tiles_h = (p.ho + kStemTR - 1) / kStemTR;
  const int ntiles = p.n * tiles_w * tiles_h;

  // table: lut[c][v] = bf16((v / 255 - mean[c]) / std[c]) for output channel c
  for (int i = tid; i < 3 * 256; i += kThreads) {
    const int c = i >> 8;
    const float v = static_cast<float>(i & 255);
    lut[i] = f32_to_bf16((v / 255.0f - p.mean[c]) / p.std[c]);
  }
  const bf16_t* __restrict__ wt = reinterpret_cast<const bf16_t*>(p.wgt);
  bf16x8 wa[NK];
#pragma unroll
  for (int ks = 0; ks < NK; ++ks)
    wa[ks] = *reinterpret_cast<const bf16x8*>(wt + static_cast<int64_t>(lane & 15) * p.k_pad + ks * 32 + 8 * kq);
  float sc[4], sh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sc[j] = p.scale != nullptr ? p.scale[kq * 4 + j] : 1.f;
    sh[j] = p.shift[kq * 4 + j];
  }
  const int frame_bytes = H * W * 3;
  const int total = p.n * frame_bytes;          // < 2^31 (stem_dma_ok)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.x), 0, total, 0x00020000);
  auto tile_org = [&](int b, int& n, int& ih0, int& iw0) {
    n = b / (tiles_w * tiles_h);
    const int rem = b - n * tiles_w * tiles_h;
    ih0 = (rem / tiles_w) * kStemTR - p.pad;
    iw0 = (rem % tiles_w) * kStemTC - p.pad;
  };
  auto issue = [&](int b, int slot) {
    int n, ih0, iw0;
    tile_org(b, n, ih0, iw0);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int r = wave + 4 * j;                       // patch row (10, 11: slack)
      const int ih = ih0 + r;
      const int start = n * frame_bytes + (ih * W + iw0) * 3;   // byte of the row's first patch pixel
      const int a0 = start >= 0 ? (start & ~3) : -((-start + 3) & ~3);
      const int o = a0 + lane * 4;
      // a dword straddling the end of the batch would read as zero (out of range): convert()
      // takes those last pixels from global memory directly
      const bool ok = r < kStemPR && static_cast<unsigned>(ih) < static_cast<unsigned>(H) && o >= 0;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(raw + slot * kStemRawB + r * 256), 4,
          ok ? static_cast<unsigned>(o) : 0xffffffffu, 0, 0, 0);
    }
  };
  auto convert = [&](int b, int slot) {
    int n, ih0, iw0;
    tile_org(b, n, ih0, iw0);
    const unsigned char* rb = reinterpret_cast<const unsigned char*>(raw + slot * kStemRawB);
    for (int i = tid; i < kStemPR * kStemPC; i += kThreads) {
      const int pr = i / kStemPC, pc = i - pr * kStemPC;
      const int ih = ih0 + pr, iw = iw0 + pc;
      uint2 v = make_uint2(0, 0);
      if (static_cast<unsigned>(ih) < static_cast<unsigned>(H) && static_cast<unsigned>(iw) < static_cast<unsigned>(W)) {
        const int start = n * frame_bytes + (ih * W + iw0) * 3;
        const int a0 = start >= 0 ? (start & ~3) : -((-start + 3) & ~3);
        const unsigned char* px = rb + pr * 256 + (start - a0) + pc * 3;
        const int pb = start + pc * 3;
        if (pb + 3 > (total & ~3)) px = reinterpret_cast<const unsigned char*>(p.x) + pb;   // batch tail
        int c0 = px[0], c1 = px[1], c2 = px[2];
        if (p.bgr) { const int t = c0; c0 = c2; c2 = t; }
        v.x = static_cast<uint32_t>(lut[c0]) | (static_cast<uint32_t>(lut[256 + c1]) << 16);
        v.y = static_cast<uint32_t>(lut[512 + c2]);
      }
      *reinterpret_cast<uint2*>(patch + i * 4) = v;
    }
  };

  int prow[PFW], pcol[PFW];
#pragma unroll
  for (int q = 0; q < PFW; ++q) {
    const int idx = (wave + 4 * q) * 16 + (lane & 15);
    prow[q] = idx / kStemTC;
    pcol[q] = idx % kStemTC;
  }
  const int64_t ybytes = static_cast<int64_t>(p.n) * p.ho * p.wo * 16 * 2;
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
      p.y, 0, static_cast<int>(ybytes < 0x7fffffff ? ybytes : 0x7fffffff), 0x00020000);

  const int b0 = blockIdx.x;
  const int G = gridDim.x;
  if (b0 < ntiles) issue(b0, 0);
  if (b0 + G < ntiles) issue(b0 + G, 1);
  int t = 0;
  for (int b = b0; b < ntiles; b += G, ++t) {
    // retire tile t's raw rows: younger ops are stores(t-2), rows(t+1), stores(t-1)
    if (t >= 2 && b + G < ntiles) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 + 2 * ST) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (b + 2 * G < ntiles) issue(b + 2 * G, (t + 2) % 3);
    convert(b, t % 3);
    __syncthreads();

    f32x4 acc[PFW];
#pragma unroll
    for (int q = 0; q < PFW; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NK; ++ks) {
#pragma unroll
      for (int q = 0; q < PFW; ++q) {
        // k = kh*32 + kw*4 + c: step ks = kernel row kh, fragment = taps kw = 2kq, 2kq+1
        const bf16_t* src = patch + ((prow[q] + ks) * kStemPC + pcol[q] + 2 * kq) * 4;
        const uint2 lo = *reinterpret_cast<const uint2*>(src);
        const uint2 hi = *reinterpret_cast<const uint2*>(src + 4);
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks], __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y)),
                                                         acc[q], 0, 0, 0);
      }
    }
    int n, oh0, ow0;
    tile_org(b, n, oh0, ow0);
    oh0 += p.pad;
    ow0 += p.pad;
#pragma unroll
    for (int q = 0; q < PFW; ++q) {
      const int idx = (wave + 4 * q) * 16 + (lane & 15);
      const int oh = oh0 + idx / kStemTC, ow = ow0 + idx % kStemTC;
      const bool ok = oh < p.ho && ow < p.wo;
      const int64_t pix = (static_cast<int64_t>(n) * p.ho + oh) * p.wo + ow;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = acc[q][j] * sc[j] + sh[j];
        if (p.relu) v[j] = fmaxf(v[j], 0.f);
      }
      u32x2_t o;
      o.x = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
      o.y = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      __builtin_amdgcn_raw_buffer_store_b64(o, ys, ok ? static_cast<unsigned>((pix * 16 + kq * 4) * 2) : 0xffffffffu,
                                            0, 0);
    }
  }
}

// ---- Fused stem + layer1 (bf16): uint8 frames -> 7x7 3->16 + BN + ReLU -> 3x3 16->16 + BN + ReLU.
//
// The stem's 16-channel full-resolution output (64 MB per 1024x2048 frame) is written by the
// stem and read straight back by layer1 (lmodels/drn.py:132-137, :201-211); here it never
// leaves the CU.  A workgroup owns an 8 x 64 tile of layer1's output; it DMAs the 16 x 73 raw
// frame pixels behind it (two tiles ahead, as stem_dma_kernel), normalises them through the
// per-channel table, computes the 10 x 66 stem outputs the 3x3 conv needs (a wave per 16
// columns, each patch-row fragment feeding up to 7 stem rows; outside the image the stem
// outputs are layer1's zero padding, not stem values),
// keeps them in LDS as bf16, and runs layer1 from there.  Both convs keep the K layouts and
// MFMA orders of stem_dma_kernel and patch_dma_kernel<16, 16, ...>, so the output is
// bit-identical to the two-launch path.
constexpr int kSLTR = 8, kSLTC = 64;                     // layer1 output tile
constexpr int kSLSR = kSLTR + 2, kSLSC = kSLTC + 2;      // stem outputs needed: 10 x 66
constexpr int kSLPR = kSLSR + 6, kSLPC = kSLSC + 7;      // stem input patch 16 x 73 (+1: zero kw=7 tap)
constexpr int kSLRPW = kSLPR / 4;                        // raw rows per wave
constexpr int kSLRawB = kSLPR * 256;                     // raw rows per ring slot
constexpr int kSLPatchB = kSLPR * kSLPC * 8;
constexpr int kSLStemPix = kSLSR * kSLSC;
constexpr int kSLStemB = kSLStemPix * 32;                // 16 bf16 channels per stem pixel
constexpr int kSLLDS = 3 * kSLRawB + kSLPatchB + kSLStemB + 3 * 256 * 2;
static_assert(kSLPatchB % 16 == 0 && kSLStemB % 16 == 0, "16-B aligned LDS regions");
static_assert(kSLPR % 4 == 0 && 2 * kSLSR <= 32 && kSLSR % 2 == 0, "raw rows over 4 waves; edge columns in two groups");

// register-allocated for 3 waves per SIMD (4 spills and runs 10 % slower)
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(3)))
stem_l1_kernel(const drnmi_conv_args p, const drnmi_conv_args q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* raw = smem;
  bf16_t* patch = reinterpret_cast<bf16_t*>(smem + 3 * kSLRawB);
  char* stile = smem + 3 * kSLRawB + kSLPatchB;
  bf16_t* lut = reinterpret_cast<bf16_t*>(stile + kSLStemB);
  constexpr int NK0 = 7, NK1 = 5, PFW = kSLTR * kSLTC / 64, ST = PFW;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int kq = lane >> 4;
  const int H = p.h, W = p.w;
  const int tiles_w = (W + kSLTC - 1) / kSLTC;
  const int tiles_h = (H + kSLTR - 1) / kSLTR;
  const int ntiles = p.n * tiles_w * tiles_h;

  for (int i = tid; i < 3 * 256; i += kThreads) {
    const int c = i >> 8;
    const float v = static_cast<float>(i & 255);
    lut[i] = f32_to_bf16((v / 255.0f - p.mean[c]) / p.std[c]);
  }
  const bf16_t* __restrict__ wt0 = reinterpret_cast<const bf16_t*>(p.wgt);
  const bf16_t* __restrict__ wt1 = reinterpret_cast<const bf16_t*>(q.wgt);
  bf16x8 wa0[NK0], wa1[NK1];
#pragma unroll
  for (int ks = 0; ks < NK0; ++ks)
    wa0[ks] = *reinterpret_cast<const bf16x8*>(wt0 + static_cast<int64_t>(lane & 15) * p.k_pad + ks * 32 + 8 * kq);
#pragma unroll
  for (int ks = 0; ks < NK1; ++ks)
    wa1[ks] = *reinterpret_cast<const bf16x8*>(wt1 + static_cast<int64_t>(lane & 15) * q.k_pad + ks * 32 + 8 * kq);
  float sc0[4], sh0[4], sc1[4], sh1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sc0[j] = p.scale != nullptr ? p.scale[kq * 4 + j] : 1.f;
    sh0[j] = p.shift[kq * 4 + j];
    sc1[j] = q.scale != nullptr ? q.scale[kq * 4 + j] : 1.f;
    sh1[j] = q.shift[kq * 4 + j];
  }
  const int frame_bytes = H * W * 3;
  const int total = p.n * frame_bytes;          // < 2^31 (stem_l1_ok)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.x), 0, total, 0x00020000);
  auto tile_org = [&](int b, int& n, int& oh0, int& ow0) {
    n = b / (tiles_w * tiles_h);
    const int rem = b - n * tiles_w * tiles_h;
    oh0 = (rem / tiles_w) * kSLTR;
    ow0 = (rem % tiles_w) * kSLTC;
  };
  auto issue = [&](int b, int slot) {           // raw rows oh0-4 .. oh0+kSLTR+3 from column ow0-4
    int n, oh0, ow0;
    tile_org(b, n, oh0, ow0);
#pragma unroll
    for (int j = 0; j < kSLRPW; ++j) {
      const int r = wave + 4 * j;
      const int ih = oh0 - 4 + r;
      const int start = n * frame_bytes + (ih * W + ow0 - 4) * 3;
      const int a0 = start >= 0 ? (start & ~3) : -((-start + 3) & ~3);
      const int o = a0 + lane * 4;
      const bool ok = static_cast<unsigned>(ih) < static_cast<unsigned>(H) && o >= 0;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(raw + slot * kSLRawB + r * 256), 4,
          ok ? static_cast<unsigned>(o) : 0xffffffffu, 0, 0, 0);
    }
  };
  // raw bytes -> normalised bf16 patch [12][73][4]; wave w converts the rows it DMA'd
  // (w, w+4, w+8) with the row terms wave-uniform, lanes over the 73 columns
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  auto convert = [&](int b, int slot) {
    int n, oh0, ow0;
    tile_org(b, n, oh0, ow0);
    const int iw0 = ow0 - 4;
    const unsigned char* rb = reinterpret_cast<const unsigned char*>(raw + slot * kSLRawB);
#pragma unroll
    for (int j = 0; j < kSLRPW; ++j) {
      const int r = wv + 4 * j;
      const int ih = oh0 - 4 + r;
      const bool row_ok = static_cast<unsigned>(ih) < static_cast<unsigned>(H);
      const int start = n * frame_bytes + (ih * W + iw0) * 3;
      const int a0 = start >= 0 ? (start & ~3) : -((-start + 3) & ~3);
      // a row that reaches the batch's final partial dword reads global memory instead
      const bool tail = start + kSLPC * 3 > (total & ~3);
      const unsigned char* rowp = tail ? reinterpret_cast<const unsigned char*>(p.x) + start : rb + r * 256 + (start - a0);
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int pc = lane + 64 * h2;
        if (h2 == 1 && pc >= kSLPC) break;
        uint2 v = make_uint2(0, 0);
        if (row_ok && static_cast<unsigned>(iw0 + pc) < static_cast<unsigned>(W)) {
          const unsigned char* px = rowp + pc * 3;
          int c0 = px[0], c1 = px[1], c2 = px[2];
          if (p.bgr) { const int t = c0; c0 = c2; c2 = t; }
          v.x = static_cast<uint32_t>(lut[c0]) | (static_cast<uint32_t>(lut[256 + c1]) << 16);
          v.y = static_cast<uint32_t>(lut[512 + c2]);
        }
        *reinterpret_cast<uint2*>(patch + (r * kSLPC + pc) * 4) = v;
      }
    }
  };

  // layer1 B-fragment offsets (patch_dma_kernel<16, 16, 1, 4, 64>): k = tap * 16 + ci
  int boff[NK1];
#pragma unroll
  for (int ks = 0; ks < NK1; ++ks) {
    const int k0 = ks * 32 + 8 * kq;
    const int tap = k0 / 16, ci = k0 % 16;
    boff[ks] = tap < 9 ? (((tap / 3) * kSLSC + tap % 3) * 16 + ci) * 2 : -1;
  }
  const int64_t ybytes = static_cast<int64_t>(q.n) * q.ho * q.wo * 16 * 2;
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(
      q.y, 0, static_cast<int>(ybytes < 0x7fffffff ? ybytes : 0x7fffffff), 0x00020000);

  const int b0 = blockIdx.x;
  const int G = gridDim.x;
  if (b0 < ntiles) issue(b0, 0);
  if (b0 + G < ntiles) issue(b0 + G, 1);
  int t = 0;
  for (int b = b0; b < ntiles; b += G, ++t) {
    // retire tile t's raw rows: younger ops are stores(t-2), rows(t+1), stores(t-1)
    if (t >= 2 && b + G < ntiles) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(kSLRPW + 2 * ST) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (b + 2 * G < ntiles) issue(b + 2 * G, (t + 2) % 3);
    convert(b, t % 3);
    __syncthreads();

    int n, oh0, ow0;
    tile_org(b, n, oh0, ow0);
    // stem.  Wave w owns stem columns 16w .. 16w+15 over the kSLSR stem rows: patch row r feeds stem
    // row q = r - kh through kernel row kh, so each B fragment is read once and used by up to 7
    // MFMAs (per accumulator the kh order is stem_dma_kernel's: bit-identical).  Columns 64, 65
    // (x kSLSR rows) are two extra groups on waves 0 and 1.
    auto stem_store = [&](const f32x4& acc, int q, int sc) {
      const int ih = oh0 - 1 + q, iw = ow0 - 1 + sc;
      const bool inside = static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                          static_cast<unsigned>(iw) < static_cast<unsigned>(W);
      float v[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v[jj] = acc[jj] * sc0[jj] + sh0[jj];
        if (p.relu) v[jj] = fmaxf(v[jj], 0.f);
        if (!inside) v[jj] = 0.f;                  // layer1's zero padding
      }
      u32x2_t o;
      o.x = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
      o.y = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      *reinterpret_cast<u32x2_t*>(stile + ((q * kSLSC + sc) * 16 + kq * 4) * 2) = o;
    };
    // (two passes of kSLSR / 2 stem rows: half the accumulators live at a time)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      constexpr int HR = kSLSR / 2;
      const int sc = wv * 16 + (lane & 15);
      f32x4 acc[HR];
#pragma unroll
      for (int q = 0; q < HR; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < HR + NK0 - 1; ++r) {
        // k = kh*32 + kw*4 + c: fragment = taps kw = 2kq, 2kq+1 of patch row half*HR + r
        const bf16_t* src = patch + ((half * HR + r) * kSLPC + sc + 2 * kq) * 4;
        const uint2 lo = *reinterpret_cast<const uint2*>(src);
        const uint2 hi = *reinterpret_cast<const uint2*>(src + 4);
        const bf16x8 bv = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
#pragma unroll
        for (int kh = 0; kh < NK0; ++kh) {
          const int q = r - kh;
          if (q >= 0 && q < HR) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa0[kh], bv, acc[q], 0, 0, 0);
        }
      }
#pragma unroll
      for (int q = 0; q < HR; ++q) stem_store(acc[q], half * HR + q, sc);
    }
    if (wv < 2) {
      const int e = wv * 16 + (lane & 15);         // 2 x kSLSR pixels: rows e / 2, columns 64 + e % 2
      const int q = (e < 2 * kSLSR ? e : 2 * kSLSR - 1) / 2, sc = 64 + (e & 1);
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < NK0; ++kh) {
        const bf16_t* src = patch + ((q + kh) * kSLPC + sc + 2 * kq) * 4;
        const uint2 lo = *reinterpret_cast<const uint2*>(src);
        const uint2 hi = *reinterpret_cast<const uint2*>(src + 4);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa0[kh], __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y)),
                                                      acc, 0, 0, 0);
      }
      if (e < 2 * kSLSR) stem_store(acc, q, sc);
    }
    __syncthreads();

    // layer1 from the stem tile
#pragma unroll 2
    for (int qq = 0; qq < PFW; ++qq) {
      const int idx = (wave + 4 * qq) * 16 + (lane & 15);
      const int r = idx / kSLTC, c = idx % kSLTC;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NK1; ++ks) {
        bf16x8 bv = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
        if (boff[ks] >= 0) bv = *reinterpret_cast<const bf16x8*>(stile + boff[ks] + (r * kSLSC + c) * 32);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa1[ks], bv, acc, 0, 0, 0);
      }
      const int oh = oh0 + r, ow = ow0 + c;
      const bool ok = oh < q.ho && ow < q.wo;
      float v[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v[jj] = acc[jj] * sc1[jj] + sh1[jj];
        if (q.relu) v[jj] = fmaxf(v[jj], 0.f);
      }
      u32x2_t o;
      o.x = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
      o.y = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      const unsigned pix = static_cast<unsigned>((n * q.ho + oh) * q.wo + ow);
      __builtin_amdgcn_raw_buffer_store_b64(o, ys, ok ? (pix * 16 + kq * 4) * 2 : 0xffffffffu, 0, 0);
    }
  }
}

int g_num_cus = 0;

template <int CIN, int COUT, int KS, int S, int TR, int TC, bool SRC_U8, bool X6 = false>
hipError_t launch_patch(const drnmi_conv_args& p, hipStream_t s) {
  static int per_cu = 0;
  auto kern = patch_conv_kernel<CIN, COUT, KS, S, TR, TC, SRC_U8, X6>;
  if (per_cu == 0) {
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(kern), kThreads, 0) !=
            hipSuccess || blocks <= 0)
      blocks = 2;
    g_num_cus = cus;
    per_cu = blocks;
  }
  const int64_t tiles = static_cast<int64_t>(p.n) * ((p.ho + TR - 1) / TR) * ((p.wo + TC - 1) / TC);
  const int64_t cap = static_cast<int64_t>(g_num_cus) * per_cu;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(tiles < cap ? tiles : cap)), dim3(kThreads), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_stem_dma(const drnmi_conv_args& p, hipStream_t s) {
  static int per_cu = 0;
  if (per_cu == 0) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(stem_dma_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kStemLDS);
    if (e != hipSuccess) return e;
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(stem_dma_kernel),
                                                     kThreads, kStemLDS) != hipSuccess || blocks <= 0)
      blocks = 1;
    g_num_cus = cus;
    per_cu = blocks;
  }
  const int64_t tiles = static_cast<int64_t>(p.n) * ((p.ho + kStemTR - 1) / kStemTR) * ((p.wo + kStemTC - 1) / kStemTC);
  const int64_t cap = static_cast<int64_t>(g_num_cus) * per_cu;
  hipLaunchKernelGGL(stem_dma_kernel, dim3(static_cast<unsigned>(tiles < cap ? tiles : cap)), dim3(kThreads),
                     kStemLDS, s, p);
  return hipGetLastError();
}

hipError_t launch_stem_l1(const drnmi_conv_args& p, const drnmi_conv_args& q, hipStream_t s) {
  static int per_cu = 0;
  if (per_cu == 0) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(stem_l1_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kSLLDS);
    if (e != hipSuccess) return e;
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(stem_l1_kernel),
                                                     kThreads, kSLLDS) != hipSuccess || blocks <= 0)
      blocks = 1;
    g_num_cus = cus;
    per_cu = blocks;
  }
  const int64_t tiles = static_cast<int64_t>(p.n) * ((p.h + kSLTR - 1) / kSLTR) * ((p.w + kSLTC - 1) / kSLTC);
  const int64_t cap = static_cast<int64_t>(g_num_cus) * per_cu;
  hipLaunchKernelGGL(stem_l1_kernel, dim3(static_cast<unsigned>(tiles < cap ? tiles : cap)), dim3(kThreads),
                     kSLLDS, s, p, q);
  return hipGetLastError();
}

template <int CIN, int COUT, int S, int TR, int TC>
hipError_t launch_patch_dma(const drnmi_conv_args& p, hipStream_t s) {
  using C = DmaCfg<CIN, COUT, S, TR, TC>;
  static int per_cu = 0;
  auto kern = patch_dma_kernel<CIN, COUT, S, TR, TC>;
  if (per_cu == 0) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return e;
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(kern), kThreads,
                                                     C::LDS) != hipSuccess || blocks <= 0)
      blocks = 1;
    g_num_cus = cus;
    per_cu = blocks;
  }
  const int64_t tiles = static_cast<int64_t>(p.n) * ((p.ho + TR - 1) / TR) * ((p.wo + TC - 1) / TC);
  const int64_t cap = static_cast<int64_t>(g_num_cus) * per_cu;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(tiles < cap ? tiles : cap)), dim3(kThreads), C::LDS, s, p);
  return hipGetLastError();
}

}  // namespace

// buffer offsets are 32-bit: one frame of input and the whole output must stay below 2 GB
static bool dma_ok(const drnmi_conv_args& p) {
  return static_cast<int64_t>(p.h) * p.w * p.cin * 2 < (int64_t(1) << 31) &&
         static_cast<int64_t>(p.n) * p.ho * p.wo * p.cout * 2 < (int64_t(1) << 31) && p.pad == 1;
}

static bool stem_dma_ok(const drnmi_conv_args& p) {
  return static_cast<int64_t>(p.n) * p.h * p.w * 3 < (int64_t(1) << 31) &&
         static_cast<int64_t>(p.n) * p.ho * p.wo * 16 * 2 < (int64_t(1) << 31) && p.pad == 3 && p.w >= 8;
}

// fp32x (DRNMI_F32X3 in, fp32 NHWC out): the full-resolution small-channel layers
static int patch_x6_dispatch(const drnmi_conv_args& p, hipStream_t s) {
  if (p.out_dtype != DRNMI_F32 || p.dil != 1 || p.res != nullptr || p.y_sc != 1 || p.y_sp != p.cout)
    return DRNMI_ENOTSUP;
  hipError_t e;
  if (p.src_u8) {
    if (p.cin != 4 || p.cout != 16 || p.ks != 7 || p.stride != 1 || p.k != 224 || p.k_pad != 224)
      return DRNMI_ENOTSUP;
    e = launch_patch<4, 16, 7, 1, 4, 64, true, true>(p, s);
  } else if (p.cin == 8 && p.cout == 16 && p.ks == 7 && p.stride == 1) {
    e = launch_patch<8, 16, 7, 1, 4, 64, false, true>(p, s);
  } else if (p.cin == 16 && p.cout == 16 && p.ks == 3 && p.stride == 1) {
    e = launch_patch<16, 16, 3, 1, 4, 64, false, true>(p, s);
  } else if (p.cin == 16 && p.cout == 32 && p.ks == 3 && p.stride == 2) {
    e = launch_patch<16, 32, 3, 2, 4, 32, false, true>(p, s);
  } else {
    return DRNMI_ENOTSUP;
  }
  return static_cast<int>(e);
}

int patch_conv_dispatch(const drnmi_conv_args& p, hipStream_t s) {
  if (p.dtype == DRNMI_F32X3) return patch_x6_dispatch(p, s);
  if (p.dtype == DRNMI_F32) return patch_f32_dispatch(p, s);       // exact fp32 (patch_f32.hip)
  if (p.dtype != DRNMI_BF16 || p.out_dtype != DRNMI_BF16 || p.dil != 1 || p.res != nullptr) return DRNMI_ENOTSUP;
  if (p.y_sc != 1 || p.y_sp != p.cout) return DRNMI_ENOTSUP;            // packed NHWC output
  hipError_t e;
  if (p.src_u8) {
    if (p.cin != 4 || p.cout != 16 || p.ks != 7 || p.stride != 1 || p.k != 224 || p.k_pad != 224)
      return DRNMI_ENOTSUP;
    e = stem_dma_ok(p) ? launch_stem_dma(p, s) : launch_patch<4, 16, 7, 1, 4, 64, true>(p, s);
  } else if (p.cin == 8 && p.cout == 16 && p.ks == 7 && p.stride == 1) {
    e = launch_patch<8, 16, 7, 1, 4, 64, false>(p, s);
  } else if (p.cin == 16 && p.cout == 16 && p.ks == 3 && p.stride == 1 && dma_ok(p)) {
    e = launch_patch_dma<16, 16, 1, 4, 64>(p, s);
  } else if (p.cin == 16 && p.cout == 32 && p.ks == 3 && p.stride == 2 && dma_ok(p)) {
    e = launch_patch_dma<16, 32, 2, 4, 32>(p, s);
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
  if (p.dtype == DRNMI_F32X3) {
    if (p.src_u8) return "patch_conv_kernel<4, 16, 7, 1, 4, 64, true, true>";
    if (p.cin == 8 && p.cout == 16 && p.ks == 7) return "patch_conv_kernel<8, 16, 7, 1, 4, 64, false, true>";
    if (p.cin == 16 && p.cout == 16 && p.ks == 3) return "patch_conv_kernel<16, 16, 3, 1, 4, 64, false, true>";
    if (p.cin == 16 && p.cout == 32 && p.ks == 3) return "patch_conv_kernel<16, 32, 3, 2, 4, 32, false, true>";
    return nullptr;
  }
  if (p.dtype == DRNMI_F32) return patch_f32_name(p);
  if (p.src_u8) return stem_dma_ok(p) ? "stem_dma_kernel" : "patch_conv_kernel<4, 16, 7, 1, 4, 64, true>";
  if (p.cin == 8 && p.cout == 16 && p.ks == 7) return "patch_conv_kernel<8, 16, 7, 1, 4, 64, false>";
  if (p.cin == 16 && p.cout == 16 && p.ks == 3 && p.stride == 1)
    return dma_ok(p) ? "patch_dma_kernel<16, 16, 1, 4, 64>" : "patch_conv_kernel<16, 16, 3, 1, 4, 64, false>";
  if (p.cin == 16 && p.cout == 32 && p.ks == 3 && p.stride == 2)
    return dma_ok(p) ? "patch_dma_kernel<16, 32, 2, 4, 32>" : "patch_conv_kernel<16, 32, 3, 2, 4, 64, false>";
  if (p.cin == 32 && p.cout == 64 && p.ks == 3 && p.stride == 2) return "patch_conv_kernel<32, 64, 3, 2, 2, 64, false>";
  return nullptr;
}

// stem (uint8 frames, 7x7 3->16, the stem_dma_kernel contract) fused with the 3x3 16->16
// stride-1 conv that consumes it (the patch_dma_kernel<16, 16, ...> contract)
bool stem_l1_ok(const drnmi_conv_args& p, const drnmi_conv_args& q) {
  const bool stem = p.src_u8 && p.dtype == DRNMI_BF16 && p.out_dtype == DRNMI_BF16 && p.cin == 4 && p.cout == 16 &&
                    p.ks == 7 && p.stride == 1 && p.pad == 3 && p.dil == 1 && p.k == 224 && p.k_pad == 224 &&
                    p.res == nullptr && p.x != nullptr && p.wgt != nullptr && p.shift != nullptr && p.n > 0 &&
                    p.h > 0 && p.w >= 8 && p.ho == p.h && p.wo == p.w &&
                    static_cast<int64_t>(p.n) * p.h * p.w * 3 < (int64_t(1) << 31);
  const bool l1 = !q.src_u8 && q.dtype == DRNMI_BF16 && q.out_dtype == DRNMI_BF16 && q.cin == 16 && q.cout == 16 &&
                  q.ks == 3 && q.stride == 1 && q.pad == 1 && q.dil == 1 && q.k == 144 && q.k_pad >= 160 &&
                  q.res == nullptr && q.x2 == nullptr && q.y != nullptr && q.wgt != nullptr && q.shift != nullptr &&
                  q.y_sc == 1 && q.y_sp == 16 && q.n == p.n && q.h == p.h && q.w == p.w && q.ho == q.h && q.wo == q.w &&
                  static_cast<int64_t>(q.n) * q.ho * q.wo * 16 * 2 < (int64_t(1) << 31);
  return stem && l1;
}

int stem_l1_dispatch(const drnmi_conv_args& p, const drnmi_conv_args& q, hipStream_t s) {
  if (!stem_l1_ok(p, q)) return DRNMI_EINVAL;
  return static_cast<int>(launch_stem_l1(p, q, s));
}

}  // namespace drnmi
