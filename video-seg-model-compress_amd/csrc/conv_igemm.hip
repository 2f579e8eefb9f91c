// NHWC implicit-GEMM convolution with a fused BN / bias + residual + ReLU epilogue.
//
// One kernel template covers every convolution of DRN-D (reference lmodels/drn.py):
// the 7x7 stem (layer0, :132-137), the 3x3 dilated convs (conv3x3 :27-29, BasicBlock
// :32-65, _make_conv_layers :201-211), the Bottleneck 1x1/3x3/1x1 (:68-106), the 1x1
// stride-s downsample (:181-186) and the seg 1x1 + bias (lmodels/drnseg.py:278-284).
//
// GEMM view: rows = output pixels (n, oh, ow), cols = output channels, K = (tap, ci)
// with k = tap*cin + ci.  A rows are gathered straight from the NHWC input (each
// 8-channel vector of a pixel is one 16 B / 32 B load; out-of-image taps load zeros,
// which is the conv's zero padding), B rows are the packed weights [cout_pad][k_pad].
// Both operands are register-staged into double-buffered LDS (one barrier per K-step)
// and consumed by MFMA:
//   bf16 mode: v_mfma_f32_16x16x32_bf16, fp32 accumulate (perf mode)
//   fp32 mode: v_mfma_f32_16x16x4_f32 — an exact fp32 fmaf chain (parity mode)
// The per-lane K permutation (lane holds k = 8*(lane>>4) + j) is identical for A and B,
// so one LDS image and one fragment read serve both MFMA shapes.
//
// Workgroup = 4 waves (256 threads), 64-wide wavefronts; tiles are assigned XCD-major
// (blocks b and b+8 share an XCD) so the blocks that share an input row-band and a
// weight panel run under one L2.
#include "common.h"
#include "kernels.h"

#include <cstdio>

namespace drnmi {

namespace {

constexpr int kBK = 32;
constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ void mma_step(f32x4& acc, const T* a, const T* b);

template <>
__device__ __forceinline__ void mma_step<bf16_t>(f32x4& acc, const bf16_t* a, const bf16_t* b) {
  const bf16x8 av = *reinterpret_cast<const bf16x8*>(a);
  const bf16x8 bv = *reinterpret_cast<const bf16x8*>(b);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}

template <>
__device__ __forceinline__ void mma_step<float>(f32x4& acc, const float* a, const float* b) {
  const float4 a0 = reinterpret_cast<const float4*>(a)[0];
  const float4 a1 = reinterpret_cast<const float4*>(a)[1];
  const float4 b0 = reinterpret_cast<const float4*>(b)[0];
  const float4 b1 = reinterpret_cast<const float4*>(b)[1];
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, acc, 0, 0, 0);
}

__device__ __forceinline__ void store_out(void* y, int64_t off, float v, int out_dtype) {
  if (out_dtype == DRNMI_BF16) {
    reinterpret_cast<bf16_t*>(y)[off] = f32_to_bf16(v);
  } else {
    reinterpret_cast<float*>(y)[off] = v;
  }
}

// Bijective XCD-major remap of a 1-D grid (cdna_hip_programming.md §5, "XCD swizzle").
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

template <typename T, int BM, int BN, int WAVES_M, int WAVES_N, int KS>
__global__ void __launch_bounds__(kThreads)
conv_igemm_kernel(const drnmi_conv_args p) {
  constexpr int PAD = sizeof(T) == 2 ? 8 : 4;  // breaks the power-of-two row stride
  constexpr int LDK = kBK + PAD;
  constexpr int WTM = BM / WAVES_M;
  constexpr int WTN = BN / WAVES_N;
  constexpr int FM = WTM / 16;
  constexpr int FN = WTN / 16;
  constexpr int AV = BM * (kBK / 8);
  constexpr int BV = BN * (kBK / 8);
  constexpr int APT = (AV + kThreads - 1) / kThreads;
  constexpr int BPT = (BV + kThreads - 1) / kThreads;
  constexpr int BUF = (BM + BN) * LDK;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per workgroup");
  static_assert(FM >= 1 && FN >= 1, "wave tile at least 16x16");

  __shared__ __attribute__((aligned(16))) T smem[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N;
  const int wn = wave % WAVES_N;

  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const int mt_count = (M + BM - 1) / BM;
  const int nt_count = (p.cout + BN - 1) / BN;      // column tiles past cout would be all padding
  const int tile = xcd_remap(blockIdx.x, mt_count * nt_count);
  const int bm0 = (tile / nt_count) * BM;
  const int bn0 = (tile % nt_count) * BN;

  const int cin = p.cin;
  const int cmask = cin - 1;
  const int lc = 31 - __builtin_clz(cin);
  const int H = p.h, W = p.w, dil = p.dil;
  const T* __restrict__ x = reinterpret_cast<const T*>(p.x);
  const T* __restrict__ wt = reinterpret_cast<const T*>(p.wgt);

  // Per-thread A rows: pixel coordinates are fixed for the whole K loop.
  int a_ih0[APT], a_iw0[APT], a_c[APT], a_row[APT];
  int64_t a_base[APT];
  bool a_on[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int v = tid + i * kThreads;
    a_on[i] = v < AV;
    a_row[i] = v >> 2;
    a_c[i] = v & 3;
    const int m = bm0 + a_row[i];
    a_ih0[i] = -(1 << 28);
    a_iw0[i] = -(1 << 28);
    a_base[i] = 0;
    if (a_on[i] && m < M) {
      const int n = m / hw_o;
      const int r = m - n * hw_o;
      const int oh = r / p.wo;
      const int ow = r - oh * p.wo;
      a_ih0[i] = oh * p.stride - p.pad;
      a_iw0[i] = ow * p.stride - p.pad;
      a_base[i] = static_cast<int64_t>(n) * H * W * cin;
    }
  }

  Vec8<T> ra[APT];
  Vec8<T> rb[BPT];

  auto load_tiles = [&](int kt) {
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      Vec8<T> v = Vec8<T>::zero();
      if (a_on[i]) {
        const int k0 = kt * kBK + 8 * a_c[i];
        const int tap = k0 >> lc;
        const int ci = k0 & cmask;
        if (tap < KS * KS) {
          const int kh = tap / KS;
          const int kw = tap - kh * KS;
          const int ih = a_ih0[i] + kh * dil;
          const int iw = a_iw0[i] + kw * dil;
          if (static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
              static_cast<unsigned>(iw) < static_cast<unsigned>(W)) {
            v = Vec8<T>::load(x + a_base[i] + (static_cast<int64_t>(ih) * W + iw) * cin + ci);
          }
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int v = tid + i * kThreads;
      if (v < BV) {
        const int row = v >> 2;
        const int c = v & 3;
        rb[i] = Vec8<T>::load(wt + static_cast<int64_t>(bn0 + row) * p.k_pad + kt * kBK + 8 * c);
      }
    }
  };

  auto store_tiles = [&](int buf) {
    T* As = smem + buf * BUF;
    T* Bs = As + BM * LDK;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      if (a_on[i]) ra[i].store(As + a_row[i] * LDK + 8 * a_c[i]);
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int v = tid + i * kThreads;
      if (v < BV) rb[i].store(Bs + (v >> 2) * LDK + 8 * (v & 3));
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.k_pad / kBK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();

  const int frag_row = lane & 15;
  const int frag_k = 8 * (lane >> 4);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load_tiles(kt + 1);
    const T* As = smem + cur * BUF;
    const T* Bs = As + BM * LDK;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const T* ap = As + (wm * WTM + fm * 16 + frag_row) * LDK + frag_k;
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const T* bp = Bs + (wn * WTN + fn * 16 + frag_row) * LDK + frag_k;
        mma_step<T>(acc[fm][fn], ap, bp);
      }
    }
    if (more) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // Epilogue: folded BN (or bias), optional residual, optional ReLU, strided store.
  const T* __restrict__ res = reinterpret_cast<const T*>(p.res);
  const int col_l = lane & 15;
  const int row_q = (lane >> 4) * 4;
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = bm0 + wm * WTM + fm * 16 + row_q + j;
      if (m >= M) continue;
      const int n = m / hw_o;
      const int q = m - n * hw_o;
      const int64_t ybase = static_cast<int64_t>(n) * p.y_sn + static_cast<int64_t>(q) * p.y_sp;
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int co = bn0 + wn * WTN + fn * 16 + col_l;
        if (co >= p.cout) continue;
        float v = acc[fm][fn][j] * (p.scale != nullptr ? p.scale[co] : 1.f) + p.shift[co];
        if (res != nullptr) v += Elem<T>::to_f32(res[static_cast<int64_t>(m) * p.cout + co]);
        if (p.relu) v = fmaxf(v, 0.f);
        store_out(p.y, ybase + static_cast<int64_t>(co) * p.y_sc, v, p.out_dtype);
      }
    }
  }
}

struct TileDesc {
  int bm, bn;
  const char* name;
};

constexpr TileDesc kTiles[] = {
    {128, 128, "128x128"},
    {128, 64, "128x64"},
    {256, 32, "256x32"},
    {256, 16, "256x16"},
    // conv_big.hip (bf16, LDS-DMA implicit GEMM, cin >= 32, ks 1/3): cout tile x 256 pixels
    {128, 128, "dma128"}, {256, 256, "dma256"}, {64, 64, "dma64k32"}, {32, 32, "dma32"},
    {256, 256, "dma256k32"}, {128, 128, "dma128k32"},
    {128, 128, "dma128p"}, {256, 256, "dma256p"}, {64, 64, "dma64k32p"}, {32, 32, "dma32p"},
    {256, 256, "dma256k32p"}, {128, 128, "dma128k32p"},   // p = persistent
    {256, 256, "pp256"},                                   // ping-pong 4-phase schedule
    {128, 128, "halo"},                                    // conv_halo.hip, 4x64 pixel block
    {256, 256, "strip256"},                                // conv_big.hip, strip-staged B (3x3, wo % 256 == 0)
    {256, 256, "stag256"},                                 // the strip tile, SIMD partners half a K step apart
    {64, 64, "s2row"},                                     // conv_s2row.hip: stride-2 3x3 32->64 / 64->128 row walk
    {64, 64, "s1x2row"},                                   // conv_s2row.hip: stride-1 3x3 64->64 + 1x1 s2 downsample
    {256, 256, "w1stag256"},                               // conv_w1.hip: the stag256 tile as 4 waves of 128 x 128
    {128, 128, "w1h128"},                                  // conv_w1.hip: 128 x 128 tile, 4 waves of 64 x 64, 2 per CU
};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

template <typename T, int BM, int BN, int WM, int WN, int KS>
hipError_t launch_conv(const drnmi_conv_args& p, hipStream_t stream) {
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int64_t blocks = ((M + BM - 1) / BM) * ((p.cout + BN - 1) / BN);   // (as the kernel's nt_count)
  hipLaunchKernelGGL((conv_igemm_kernel<T, BM, BN, WM, WN, KS>), dim3(static_cast<unsigned>(blocks)),
                     dim3(kThreads), 0, stream, p);
  return hipGetLastError();
}

template <typename T, int KS>
hipError_t dispatch_tile(const drnmi_conv_args& p, int tile, hipStream_t s) {
  switch (tile) {
    case 0: return launch_conv<T, 128, 128, 2, 2, KS>(p, s);
    case 1: return launch_conv<T, 128, 64, 2, 2, KS>(p, s);
    case 2: return launch_conv<T, 256, 32, 4, 1, KS>(p, s);
    case 3: return launch_conv<T, 256, 16, 4, 1, KS>(p, s);
    default: return hipErrorInvalidValue;
  }
}

template <typename T>
hipError_t dispatch_ks(const drnmi_conv_args& p, int tile, hipStream_t s) {
  switch (p.ks) {
    case 1: return dispatch_tile<T, 1>(p, tile, s);
    case 3: return dispatch_tile<T, 3>(p, tile, s);
    case 7: return dispatch_tile<T, 7>(p, tile, s);
    default: return hipErrorInvalidValue;
  }
}

int auto_tile(int cout) {
  if (cout > 64) return 0;
  if (cout > 32) return 1;
  if (cout > 16) return 2;
  return 3;
}

}  // namespace

}  // namespace drnmi

using namespace drnmi;

extern "C" int drnmi_conv_num_tiles(void) { return kNumTiles; }

extern "C" const char* drnmi_conv_tile_name(int tile) {
  return (tile >= 0 && tile < kNumTiles) ? kTiles[tile].name : nullptr;
}

extern "C" int drnmi_conv2d_bn_act(const drnmi_conv_args* a, void* stream) {
  if (a == nullptr) return DRNMI_EINVAL;
  const drnmi_conv_args& p = *a;
  // BN-statistics partials and output row strides: conv_x6 only
  if (p.stats != nullptr && (p.algo != DRNMI_ALGO_IGEMM || x6_conv_stats_rows(p) <= 0)) return DRNMI_EINVAL;
  if (p.y_sr != 0 && (p.algo != DRNMI_ALGO_IGEMM || p.dtype != DRNMI_F32X3 || p.y_sc != 1 || p.y_sr < 0 ||
                      !x6_conv_supported(p)))
    return DRNMI_EINVAL;
  if (p.algo == DRNMI_ALGO_PATCH) {
    if (p.x2 != nullptr) return DRNMI_ENOTSUP;     // fused second input: LDS-DMA kernels only
    if (p.x == nullptr || p.wgt == nullptr || p.y == nullptr || p.shift == nullptr ||
        p.n <= 0 || p.h <= 0 || p.w <= 0 || p.cout > p.cout_pad)
      return DRNMI_EINVAL;
    if (p.ho != (p.h + 2 * p.pad - p.dil * (p.ks - 1) - 1) / p.stride + 1 ||
        p.wo != (p.w + 2 * p.pad - p.dil * (p.ks - 1) - 1) / p.stride + 1)
      return DRNMI_EINVAL;
    return patch_conv_dispatch(p, reinterpret_cast<hipStream_t>(stream));
  }
  if (p.algo != DRNMI_ALGO_IGEMM || p.src_u8) return DRNMI_EINVAL;
  const bool pow2 = p.cin >= 8 && (p.cin & (p.cin - 1)) == 0;
  if (!pow2 || p.n <= 0 || p.h <= 0 || p.w <= 0 || p.ho <= 0 || p.wo <= 0) return DRNMI_EINVAL;
  if (p.cout <= 0 || p.cout > p.cout_pad || p.k != p.ks * p.ks * p.cin + (p.x2 != nullptr ? p.cin2 : 0))
    return DRNMI_EINVAL;
  if (p.k_pad < p.k || p.k_pad % kBK != 0 || p.stride <= 0 || p.dil <= 0 || p.pad < 0) return DRNMI_EINVAL;
  if (p.x == nullptr || p.wgt == nullptr || p.y == nullptr || p.shift == nullptr)
    return DRNMI_EINVAL;
  if (p.dtype == DRNMI_I8) {
    if (p.out_dtype != DRNMI_I8 && p.out_dtype != DRNMI_BF16 && p.out_dtype != DRNMI_F32) return DRNMI_EINVAL;
  } else if (p.dtype == DRNMI_F32X3) {
    if (p.out_dtype != DRNMI_F32) return DRNMI_EINVAL;
  } else if ((p.dtype != DRNMI_BF16 && p.dtype != DRNMI_F32) ||
             (p.out_dtype != DRNMI_BF16 && p.out_dtype != DRNMI_F32)) {
    return DRNMI_EINVAL;
  }
  // Output geometry must be the conv's: ho = (h + 2 pad - dil (ks-1) - 1) / stride + 1 -- except for
  // the row-strided (y_sr) class launches of a stride-2 data gradient, whose taps past the input's
  // bottom / right edge read zeros (an asymmetric pad; conv_x6 bounds-checks every tap)
  if (p.y_sr == 0 && (p.ho != (p.h + 2 * p.pad - p.dil * (p.ks - 1) - 1) / p.stride + 1 ||
                      p.wo != (p.w + 2 * p.pad - p.dil * (p.ks - 1) - 1) / p.stride + 1))
    return DRNMI_EINVAL;
  if (p.dtype == DRNMI_I8) return i8_conv_dispatch(p, reinterpret_cast<hipStream_t>(stream));   // int8: one kernel family
  if (p.dtype == DRNMI_F32X3) return x6_conv_dispatch(p, reinterpret_cast<hipStream_t>(stream));
  if (p.tile >= 4 || (p.tile < 0 && (big_conv_supported(p) || halo_conv_supported(p))))
    return big_conv_dispatch(p, p.tile < 0 ? -1 : p.tile - 4, reinterpret_cast<hipStream_t>(stream));
  if (p.x2 != nullptr) return DRNMI_ENOTSUP;          // fused second input: LDS-DMA kernels only
  const int tile = p.tile < 0 ? auto_tile(p.cout) : p.tile;
  if (tile >= 4 || p.cout_pad % kTiles[tile].bn != 0) return DRNMI_EINVAL;
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  if (M >= (int64_t(1) << 31) / 2) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = p.dtype == DRNMI_BF16 ? dispatch_ks<bf16_t>(p, tile, s) : dispatch_ks<float>(p, tile, s);
  if (e == hipErrorInvalidValue) return DRNMI_ENOTSUP;
  return static_cast<int>(e);
}

extern "C" int64_t drnmi_conv_workspace_bytes(const drnmi_conv_args* a) {
  if (a == nullptr) return -1;
  return a->dtype == DRNMI_F32X3 && a->algo == DRNMI_ALGO_IGEMM ? x6_conv_workspace_bytes(*a) : 0;
}

extern "C" int64_t drnmi_conv_stats_rows(const drnmi_conv_args* a) {
  if (a == nullptr) return -1;
  return a->dtype == DRNMI_F32X3 && a->algo == DRNMI_ALGO_IGEMM ? x6_conv_stats_rows(*a) : 0;
}

extern "C" int drnmi_stem_layer1(const drnmi_conv_args* stem, const drnmi_conv_args* next, void* stream) {
  if (stem == nullptr || next == nullptr) return DRNMI_EINVAL;
  return stem_l1_dispatch(*stem, *next, reinterpret_cast<hipStream_t>(stream));
}

extern "C" const char* drnmi_stem_layer1_kernel_name(const drnmi_conv_args* stem, const drnmi_conv_args* next) {
  if (stem == nullptr || next == nullptr || !stem_l1_ok(*stem, *next)) return nullptr;
  return "stem_l1_kernel";
}

extern "C" int drnmi_weight_unit_mask(const void* wgt, int32_t dtype, int32_t rows_pad, int32_t k_pad,
                                      uint32_t* mask, int32_t* nonzero_units, void* stream) {
  return weight_unit_mask(wgt, dtype, rows_pad, k_pad, mask, nonzero_units, reinterpret_cast<hipStream_t>(stream));
}

extern "C" const char* drnmi_conv_kernel_name(const drnmi_conv_args* a) {
  if (a == nullptr) return nullptr;
  const drnmi_conv_args& p = *a;
  if (p.algo == DRNMI_ALGO_PATCH) return patch_conv_name(p);
  if (p.dtype == DRNMI_I8) return i8_conv_name(p);
  if (p.dtype == DRNMI_F32X3) return x6_conv_name(p);
  if (p.tile >= 4 || (p.tile < 0 && (big_conv_supported(p) || halo_conv_supported(p))))
    return big_conv_name(p, p.tile < 0 ? -1 : p.tile - 4);
  const int tile = p.tile < 0 ? auto_tile(p.cout) : p.tile;
  if (tile > 3 || (p.ks != 1 && p.ks != 3 && p.ks != 7)) return nullptr;
  static const char* tn[4] = {"128, 128, 2, 2", "128, 64, 2, 2", "256, 32, 4, 1", "256, 16, 4, 1"};
  static char buf[8][96];
  static int slot = 0;
  char* b = buf[slot++ & 7];
  snprintf(b, 96, "conv_igemm_kernel<%s, %s, %d>", p.dtype == DRNMI_BF16 ? "bf16" : "f32", tn[tile], p.ks);
  return b;
}
