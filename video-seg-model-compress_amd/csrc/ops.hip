// HBM-bound kernels around the convolutions:
//   * frame ingest (u8 HWC -> normalised NHWC8)      data_transforms.py:109-125, :256-281
//   * NCHW fp32 -> NHWC boundary conversion          lmodels/drnseg.py:295-299 input
//   * fused up x8 + LogSoftmax + argmax             lmodels/drnseg.py:257-299, semantic_seg.py:445
//   * multi-tensor mask apply (float / bit masks)    pruners/Pruner.py:17-20
#include "common.h"

namespace drnmi {
namespace {

template <typename T>
__device__ __forceinline__ T from_f32(float v);
template <>
__device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ bf16_t from_f32<bf16_t>(float v) { return f32_to_bf16(v); }

// ---------------------------------------------------------------- frame ingest
// One thread per pixel: 3 bytes in, 8 channels out (16 B bf16 / 32 B fp32).
template <typename T>
__global__ void __launch_bounds__(256)
frame_ingest_kernel(const uint8_t* __restrict__ frames, T* __restrict__ out, int64_t npix,
                    float m0, float m1, float m2, float s0, float s1, float s2, int bgr) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint8_t* px = frames + i * 3;
  float c0 = static_cast<float>(px[0]);
  float c1 = static_cast<float>(px[1]);
  float c2 = static_cast<float>(px[2]);
  if (bgr) { const float t = c0; c0 = c2; c2 = t; }
  // Same fp32 op sequence as ToTensorVideoImage (x / 255) then Normalize (sub_, div_).
  const float v0 = (c0 / 255.0f - m0) / s0;
  const float v1 = (c1 / 255.0f - m1) / s1;
  const float v2 = (c2 / 255.0f - m2) / s2;
  T* o = out + i * 8;
  Vec8<T> r = Vec8<T>::zero();
  T tmp[8] = {from_f32<T>(v0), from_f32<T>(v1), from_f32<T>(v2), T(0), T(0), T(0), T(0), T(0)};
  r = Vec8<T>::load(tmp);
  r.store(o);
}

// ---------------------------------------------------------------- layout conversion
template <typename T>
__global__ void __launch_bounds__(256)
nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ out, int c, int64_t hw,
                    int c_pad, int64_t total_pix) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= total_pix) return;
  const int64_t n = i / hw;
  const int64_t q = i - n * hw;
  const float* src = x + n * c * hw + q;
  T* dst = out + i * c_pad;
  for (int ch = 0; ch < c_pad; ++ch) {
    dst[ch] = ch < c ? from_f32<T>(src[ch * hw]) : T(0);
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
nhwc_to_nchw_kernel(const T* __restrict__ x, float* __restrict__ out, int c, int64_t hw,
                    int c_stride, int64_t total) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= total) return;  // i indexes the NCHW output
  const int64_t n = i / (c * hw);
  const int64_t r = i - n * c * hw;
  const int64_t ch = r / hw;
  const int64_t q = r - ch * hw;
  out[i] = Elem<T>::to_f32(x[(n * hw + q) * c_stride + ch]);
}

// ---------------------------------------------------------------- up x8 + log-softmax + argmax
// Output pixel (oy, ox) of ConvTranspose2d(k16, s8, p4) receives input rows
// i1 = (oy+4)>>3 (tap ky = oy+4-8*i1 in [0,8)) and i0 = i1-1 (tap ky+8), likewise for
// columns: 4 taps per class.  The 16x16 kernel is shared by every class plane
// (fill_up_weights copies plane 0 into all planes, lmodels/drnseg.py:265-266).
constexpr int kMaxClasses = 32;

template <int LABEL_DTYPE>
__global__ void __launch_bounds__(256)
up8_lsm_kernel(const float* __restrict__ logits, const float* __restrict__ up_w,
               float* __restrict__ logprobs, void* __restrict__ labels, int c, int h, int w) {
  __shared__ float wk[256];
  wk[threadIdx.x] = up_w[threadIdx.x];
  __syncthreads();

  const int H = h * 8, W = w * 8;
  const int ox = blockIdx.x * blockDim.x + threadIdx.x;
  const int oy = blockIdx.y;
  const int n = blockIdx.z;
  if (ox >= W) return;

  const int i1 = (oy + 4) >> 3, i0 = i1 - 1;
  const int ky1 = oy + 4 - 8 * i1, ky0 = ky1 + 8;
  const int j1 = (ox + 4) >> 3, j0 = j1 - 1;
  const int kx1 = ox + 4 - 8 * j1, kx0 = kx1 + 8;
  const bool vi0 = i0 >= 0, vi1 = i1 < h, vj0 = j0 >= 0, vj1 = j1 < w;
  const float w00 = (vi0 && vj0) ? wk[ky0 * 16 + kx0] : 0.f;
  const float w01 = (vi0 && vj1) ? wk[ky0 * 16 + kx1] : 0.f;
  const float w10 = (vi1 && vj0) ? wk[ky1 * 16 + kx0] : 0.f;
  const float w11 = (vi1 && vj1) ? wk[ky1 * 16 + kx1] : 0.f;
  const int ci0 = vi0 ? i0 : 0, ci1 = vi1 ? i1 : 0, cj0 = vj0 ? j0 : 0, cj1 = vj1 ? j1 : 0;

  const int64_t plane = static_cast<int64_t>(h) * w;
  const float* src = logits + static_cast<int64_t>(n) * c * plane;
  float v[kMaxClasses];
  float vmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < kMaxClasses; ++k) {
    if (k < c) {
      const float* s = src + k * plane;
      float a = s[ci0 * w + cj0] * w00;
      a = fmaf(s[ci0 * w + cj1], w01, a);
      a = fmaf(s[ci1 * w + cj0], w10, a);
      a = fmaf(s[ci1 * w + cj1], w11, a);
      v[k] = a;
      vmax = fmaxf(vmax, a);
    }
  }
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxClasses; ++k) {
    if (k < c) sum += expf(v[k] - vmax);
  }
  const float lse = logf(sum);
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int64_t pix = static_cast<int64_t>(oy) * W + ox;
  float best = -INFINITY;
  int arg = 0;
#pragma unroll
  for (int k = 0; k < kMaxClasses; ++k) {
    if (k < c) {
      const float lp = (v[k] - vmax) - lse;
      if (logprobs != nullptr) logprobs[(static_cast<int64_t>(n) * c + k) * HW + pix] = lp;
      if (lp > best) { best = lp; arg = k; }
    }
  }
  if (labels != nullptr) {
    if (LABEL_DTYPE == DRNMI_U8) {
      reinterpret_cast<uint8_t*>(labels)[static_cast<int64_t>(n) * HW + pix] = static_cast<uint8_t>(arg);
    } else {
      reinterpret_cast<int64_t*>(labels)[static_cast<int64_t>(n) * HW + pix] = arg;
    }
  }
}

// Fast path for a compile-time class count: each thread owns 4 consecutive output pixels
// of one row.  Output columns [4q, 4q+4) all read input columns j0 = j1-1, j1 = (q+1)>>1,
// so the 4 taps per class are loaded once for 4 pixels (19 loads per pixel -> ~5), the
// labels go out as one 4-byte store and each log-prob plane as one 16-byte store.
// Same per-pixel arithmetic (and summation order) as up8_lsm_kernel.
template <int NC, int LABEL_DTYPE>
__global__ void __launch_bounds__(256)
up8_lsm_quad_kernel(const float* __restrict__ logits, const float* __restrict__ up_w,
                    float* __restrict__ logprobs, void* __restrict__ labels, int h, int w) {
  __shared__ float wk[256];
  wk[threadIdx.x] = up_w[threadIdx.x];
  __syncthreads();

  const int H = h * 8, W = w * 8;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int oy = blockIdx.y;
  const int n = blockIdx.z;
  if (4 * q >= W) return;

  const int i1 = (oy + 4) >> 3, i0 = i1 - 1;
  const int ky1 = oy + 4 - 8 * i1, ky0 = ky1 + 8;
  const int j1 = (q + 1) >> 1, j0 = j1 - 1;
  const bool vi0 = i0 >= 0, vi1 = i1 < h, vj0 = j0 >= 0, vj1 = j1 < w;
  float w00[4], w01[4], w10[4], w11[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int ox = 4 * q + p;
    const int kx1 = ox + 4 - 8 * j1, kx0 = kx1 + 8;
    w00[p] = (vi0 && vj0) ? wk[ky0 * 16 + kx0] : 0.f;
    w01[p] = (vi0 && vj1) ? wk[ky0 * 16 + kx1] : 0.f;
    w10[p] = (vi1 && vj0) ? wk[ky1 * 16 + kx0] : 0.f;
    w11[p] = (vi1 && vj1) ? wk[ky1 * 16 + kx1] : 0.f;
  }
  const int ci0 = vi0 ? i0 : 0, ci1 = vi1 ? i1 : 0, cj0 = vj0 ? j0 : 0, cj1 = vj1 ? j1 : 0;
  const int64_t plane = static_cast<int64_t>(h) * w;
  const float* src = logits + static_cast<int64_t>(n) * NC * plane;
  float v[NC][4];
  float vmax[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const float* s = src + k * plane;
    const float s00 = s[ci0 * w + cj0], s01 = s[ci0 * w + cj1];
    const float s10 = s[ci1 * w + cj0], s11 = s[ci1 * w + cj1];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float a = s00 * w00[p];
      a = fmaf(s01, w01[p], a);
      a = fmaf(s10, w10[p], a);
      a = fmaf(s11, w11[p], a);
      v[k][p] = a;
      vmax[p] = fmaxf(vmax[p], a);
    }
  }
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int64_t pix = static_cast<int64_t>(oy) * W + 4 * q;
  int arg[4] = {0, 0, 0, 0};
  if (logprobs == nullptr) {
    // Labels only: lp_c = (v_c - max) - lse is a monotone map of v_c, so the argmax of the
    // up-sampled logits is the argmax of the log-probs -- except where the rounding of that map
    // merges the top two (|lp| < 4 + gap, so only gaps below a few 2^-22): there torch.max over
    // the log-probs returns the lower class index.  Pixels whose top-2 gap is under 2^-16 take
    // the log-prob path below (same arithmetic as the logprobs branch), so the labels are those
    // of argmax(log_softmax) bit for bit; the rest skip the 19 exps.
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float best = v[0][p], second = -INFINITY;
#pragma unroll
      for (int k = 1; k < NC; ++k) {
        if (v[k][p] > best) { second = best; best = v[k][p]; arg[p] = k; }
        else if (v[k][p] > second) second = v[k][p];
      }
      if (best - second < 0x1p-16f) {
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < NC; ++k) sum += expf(v[k][p] - vmax[p]);
        const float lse = logf(sum);
        float bl = -INFINITY;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
          const float lp = (v[k][p] - vmax[p]) - lse;
          if (lp > bl) { bl = lp; arg[p] = k; }
        }
      }
    }
  } else {
    float lse[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < NC; ++k) sum += expf(v[k][p] - vmax[p]);
      lse[p] = logf(sum);
    }
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      float lp[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        lp[p] = (v[k][p] - vmax[p]) - lse[p];
        if (lp[p] > best[p]) { best[p] = lp[p]; arg[p] = k; }
      }
      *reinterpret_cast<float4*>(logprobs + (static_cast<int64_t>(n) * NC + k) * HW + pix) =
          make_float4(lp[0], lp[1], lp[2], lp[3]);
    }
  }
  if (labels != nullptr) {
    if (LABEL_DTYPE == DRNMI_U8) {
      const uint32_t packed = static_cast<uint32_t>(arg[0]) | (static_cast<uint32_t>(arg[1]) << 8) |
                              (static_cast<uint32_t>(arg[2]) << 16) | (static_cast<uint32_t>(arg[3]) << 24);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(labels) + static_cast<int64_t>(n) * HW + pix) = packed;
    } else {
      int64_t* o = reinterpret_cast<int64_t*>(labels) + static_cast<int64_t>(n) * HW + pix;
#pragma unroll
      for (int p = 0; p < 4; ++p) o[p] = arg[p];
    }
  }
}

// One output row of 4 pixels of the labels-only head: the up-sampled logits of the 4 taps (kernel
// row ky1 = oy + 4 - 8 i1, columns kx1_0 + p), the argmax with its near-tie fallback through the
// log-softmax (see up8_labels_oct_kernel).  Shared by the oct and the fast-path kernels, so their
// labels are the same arithmetic.
template <int NC>
__device__ __forceinline__ void oct_row_labels(const float (&s00)[NC], const float (&s01)[NC], const float (&s10)[NC],
                                               const float (&s11)[NC], const float* wk, int ky1, int kx1_0, bool vi0,
                                               bool vi1, bool vj0, bool vj1, int (&arg)[4]) {
  const int ky0 = ky1 + 8;
  // two pixels per packed fp32 op (v_pk_mul_f32 / v_pk_fma_f32: the same per-element rounding
  // as the scalar mul + fma chain), then per pixel a running top-2 with one v_med3 per class
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    f32x2_t w00, w01, w10, w11;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int kx1 = kx1_0 + 2 * pp + e, kx0 = kx1 + 8;
      w00[e] = (vi0 && vj0) ? wk[ky0 * 16 + kx0] : 0.f;
      w01[e] = (vi0 && vj1) ? wk[ky0 * 16 + kx1] : 0.f;
      w10[e] = (vi1 && vj0) ? wk[ky1 * 16 + kx0] : 0.f;
      w11[e] = (vi1 && vj1) ? wk[ky1 * 16 + kx1] : 0.f;
    }
    f32x2_t v[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      f32x2_t a = f32x2_t{s00[k], s00[k]} * w00;
      a = __builtin_elementwise_fma(f32x2_t{s01[k], s01[k]}, w01, a);
      a = __builtin_elementwise_fma(f32x2_t{s10[k], s10[k]}, w10, a);
      a = __builtin_elementwise_fma(f32x2_t{s11[k], s11[k]}, w11, a);
      v[k] = a;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      // best >= second throughout, so med3(best, second, x) is the new second for every x
      // (x > best: old best; second < x <= best: x; else second) -- the if / else-if chain
      float best = v[0][e], second = -INFINITY;
      int am = 0;
#pragma unroll
      for (int k = 1; k < NC; ++k) {
        const float x = v[k][e];
        am = x > best ? k : am;
        second = __builtin_amdgcn_fmed3f(best, second, x);
        best = fmaxf(best, x);
      }
      if (best - second < 0x1p-16f) {
        float vmax = -INFINITY;
#pragma unroll
        for (int k = 0; k < NC; ++k) vmax = fmaxf(vmax, v[k][e]);
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < NC; ++k) sum += expf(v[k][e] - vmax);
        const float lse = logf(sum);
        float bl = -INFINITY;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
          const float lp = (v[k][e] - vmax) - lse;
          if (lp > bl) { bl = lp; am = k; }
        }
      }
      arg[2 * pp + e] = am;
    }
  }
}

// oct_row_labels over a candidate subset of the classes (bit k of cm), the four taps' class-k
// logits read from LDS rows tp00[k] .. tp11[k].  The caller guarantees (up8_labels_tile_kernel,
// candidate pruning) that every class outside cm sits more than 2^-16 below the best class at every pixel of
// the block, so the argmax over cm, in class order, is oct_row_labels' argmax whenever the top two
// candidates are >= 2^-16 apart; returns false (no labels) when a pixel's top two are closer, and
// the caller runs the full row.  Same per-class arithmetic as oct_row_labels.
template <int NC>
__device__ __forceinline__ bool oct_row_labels_cand(const float* tp00, const float* tp01, const float* tp10,
                                                    const float* tp11, uint32_t cm, const float* wk, int ky1, int kx1_0,
                                                    int (&arg)[4]) {
  const int ky0 = ky1 + 8;
  f32x2_t w00[2], w01[2], w10[2], w11[2];
#pragma unroll
  for (int pp = 0; pp < 2; ++pp)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int kx1 = kx1_0 + 2 * pp + e, kx0 = kx1 + 8;
      w00[pp][e] = wk[ky0 * 16 + kx0];
      w01[pp][e] = wk[ky0 * 16 + kx1];
      w10[pp][e] = wk[ky1 * 16 + kx0];
      w11[pp][e] = wk[ky1 * 16 + kx1];
    }
  float best[4], second[4];
  int am[4];
  const int k0 = __builtin_ctz(cm);
  bool first = true;
  while (cm != 0) {
    const int k = __builtin_ctz(cm);
    cm &= cm - 1;
    const float a00 = tp00[k], a01 = tp01[k], a10 = tp10[k], a11 = tp11[k];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      f32x2_t v = f32x2_t{a00, a00} * w00[pp];
      v = __builtin_elementwise_fma(f32x2_t{a01, a01}, w01[pp], v);
      v = __builtin_elementwise_fma(f32x2_t{a10, a10}, w10[pp], v);
      v = __builtin_elementwise_fma(f32x2_t{a11, a11}, w11[pp], v);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int px = 2 * pp + e;
        const float x = v[e];
        if (first) {
          best[px] = x;
          second[px] = -INFINITY;
          am[px] = k0;
        } else {
          am[px] = x > best[px] ? k : am[px];
          second[px] = __builtin_amdgcn_fmed3f(best[px], second[px], x);
          best[px] = fmaxf(best[px], x);
        }
      }
    }
    first = false;
  }
  bool ok = true;
#pragma unroll
  for (int px = 0; px < 4; ++px) {
    ok = ok && !(best[px] - second[px] < 0x1p-16f);
    arg[px] = am[px];
  }
  return ok;
}

template <int LABEL_DTYPE>
__device__ __forceinline__ void store_labels4(void* labels, int64_t pix, const int (&arg)[4]) {
  if (LABEL_DTYPE == DRNMI_U8) {
    const uint32_t packed = static_cast<uint32_t>(arg[0]) | (static_cast<uint32_t>(arg[1]) << 8) |
                            (static_cast<uint32_t>(arg[2]) << 16) | (static_cast<uint32_t>(arg[3]) << 24);
    *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(labels) + pix) = packed;
  } else {
    int64_t* o = reinterpret_cast<int64_t*>(labels) + pix;
#pragma unroll
    for (int p = 0; p < 4; ++p) o[p] = arg[p];
  }
}

// int8 nets: the logits of the int8 seg conv from its two int32 partial planes: (float)(p0 + p1) *
// scale + shift, fmul then fadd as store_tile_i8 (no contraction)
template <int NC, typename B>
__device__ __forceinline__ void load_taps_seg2_i8(const int* src, int64_t half, int w, int cs, const B& scale,
                                                  const B& shift, int iy, int ix, float (&d)[NC]) {
#pragma clang fp contract(off)
  constexpr int NC4 = (NC + 3) / 4;
  const int4* r = reinterpret_cast<const int4*>(src + (static_cast<int64_t>(iy) * w + ix) * cs);
#pragma unroll
  for (int k4 = 0; k4 < NC4; ++k4) {
    const int4 a = r[k4], b = r[k4 + half / 4];
    const int e[4] = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * k4 + j < NC) d[4 * k4 + j] = static_cast<float>(e[j]) * scale[4 * k4 + j] + shift[4 * k4 + j];
  }
}

// The 4 taps (19 classes each) of thread q's output block, from NHWC logit rows (cs floats per
// pixel); SEG2: two partial planes and the bias, summed (bias + partial 0) + partial 1.
template <int NC, bool SEG2, typename B>
__device__ __forceinline__ void load_taps_nhwc(const float* src, int64_t half, int w, int cs, const B& bias, int iy,
                                               int ix, float (&d)[NC]) {
  constexpr int NC4 = (NC + 3) / 4;
  const float4* r = reinterpret_cast<const float4*>(src + (static_cast<int64_t>(iy) * w + ix) * cs);
#pragma unroll
  for (int k4 = 0; k4 < NC4; ++k4) {
    float4 v = r[k4];
    if constexpr (SEG2) {
      const float4 v1 = r[k4 + half / 4];
      v = make_float4((bias[4 * k4] + v.x) + v1.x, (bias[4 * k4 + 1] + v.y) + v1.y, (bias[4 * k4 + 2] + v.z) + v1.z,
                      (bias[4 * k4 + 3] + v.w) + v1.w);
    }
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * k4 + j < NC) d[4 * k4 + j] = e[j];
  }
}

// Labels-only head (no log-prob planes requested: the seg_video path).  The 8 output rows
// oy = 8*i1-4 .. 8*i1+3 all read input rows (i1-1, i1), so a thread owns 4 output columns x
// those 8 rows: the 4 taps per class are loaded once for 32 pixels (the quad kernel re-loads
// them for every output row).  Per pixel: the quad kernel's labels-only arithmetic, near-tie
// fallback and argmax order, so the labels are identical.
// NHWC: logits as [n][h][w][cs] fp32 rows (cs % 4 == 0, cs >= NC; the seg conv's labels-only
// output, one float4 per 4 classes) instead of NC planes; the values and the per-pixel arithmetic
// are the same, so are the labels.
// SEG2 (with NHWC): `logits` holds two partial-logit planes [2][n h w][cs] (the seg classifier
// folded into the last conv's epilogue, one partial per 256-channel block) and the logit is
// (bias + partial 0) + partial 1, in that order.
template <int NC, int LABEL_DTYPE, bool NHWC = false, bool SEG2 = false>
__global__ void __launch_bounds__(256)
up8_labels_oct_kernel(const float* __restrict__ logits, const float* __restrict__ up_w,
                      void* __restrict__ labels, int h, int w, int cs = 0, const float* __restrict__ bias = nullptr) {
  __shared__ float wk[256];
  wk[threadIdx.x] = up_w[threadIdx.x];
  __syncthreads();

  const int H = h * 8, W = w * 8;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int i1 = blockIdx.y, i0 = i1 - 1;
  const int n = blockIdx.z;
  if (4 * q >= W) return;

  const int j1 = (q + 1) >> 1, j0 = j1 - 1;
  const bool vi0 = i0 >= 0, vi1 = i1 < h, vj0 = j0 >= 0, vj1 = j1 < w;
  const int ci0 = vi0 ? i0 : 0, ci1 = vi1 ? i1 : 0, cj0 = vj0 ? j0 : 0, cj1 = vj1 ? j1 : 0;
  const int64_t plane = static_cast<int64_t>(h) * w;
  float s00[NC], s01[NC], s10[NC], s11[NC];
  if constexpr (NHWC) {
    const float* src = logits + static_cast<int64_t>(n) * plane * cs;
    const int64_t half = static_cast<int64_t>(gridDim.z) * plane * cs;   // SEG2: second partial plane
    load_taps_nhwc<NC, SEG2>(src, half, w, cs, bias, ci0, cj0, s00);
    load_taps_nhwc<NC, SEG2>(src, half, w, cs, bias, ci0, cj1, s01);
    load_taps_nhwc<NC, SEG2>(src, half, w, cs, bias, ci1, cj0, s10);
    load_taps_nhwc<NC, SEG2>(src, half, w, cs, bias, ci1, cj1, s11);
  } else {
    const float* src = logits + static_cast<int64_t>(n) * NC * plane;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const float* s = src + k * plane;
      s00[k] = s[ci0 * w + cj0];
      s01[k] = s[ci0 * w + cj1];
      s10[k] = s[ci1 * w + cj0];
      s11[k] = s[ci1 * w + cj1];
    }
  }
  const int kx1_0 = 4 * q + 4 - 8 * j1;   // kx1 of column p is kx1_0 + p, kx0 = kx1 + 8
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int oy_begin = max(0, 8 * i1 - 4), oy_end = min(H, 8 * i1 + 4);
  for (int oy = oy_begin; oy < oy_end; ++oy) {
    int arg[4];
    oct_row_labels<NC>(s00, s01, s10, s11, wk, oy + 4 - 8 * i1, kx1_0, vi0, vi1, vj0, vj1, arg);
    store_labels4<LABEL_DTYPE>(labels, static_cast<int64_t>(n) * HW + static_cast<int64_t>(oy) * W + 4 * q, arg);
  }
}

// Labels-only head with a uniform-window fast path (the NHWC / SEG2 / int8-SEG2 logits of
// DRNSeg.segment).  A workgroup owns TI x TJ tap windows (i1, j1) -- window = the 8 x 8 output
// pixels whose taps are the 1/8-res pixels (i1 - 1 .. i1, j1 - 1 .. j1), as in the oct kernel --
// and reads and summarises each of its 1/8-res pixels once.
// Fast path: when the 4 taps are inside the image and share their argmax c with a top-2 margin of
// at least
//     guard = 2^-16 / min_phase(sum w) * (1 + 2^-10) + 2^-20 * max_t |L_t[c]|
// (up-sampling weights all >= 0), every up-sampled logit vector of the window has c on top by more
// than 2^-16: v_c - v_k = sum_t w_t (L_t[c] - L_t[k]) >= min(margin) sum_t w_t, and the computed
// values (one mul + 3 fma, each rounding <= 2^-24 of a partial sum bounded by sum_t w_t |L_t[k]|
// <= sum_t w_t (|L_t[c]| + L_t[c] - L_t[k])) lose less than 2^-21 (2 max|L_t[c]| sum w + the
// margin term) -- so the oct kernel's arithmetic would return c for all 64 pixels without its
// near-tie fallback, and the window's labels are written without any per-pixel work (~79 % of the
// windows on the headline frames).
//   1. its (TI + 1) x (TJ + 1) 1/8-res pixels: logit vector (the entry point's sum, as
//      load_taps_nhwc / load_taps_seg2_i8) to LDS, plus the per-tap summary (argmax, top-2 margin
//      from a med3 chain, |best|, all classes finite);
//   2. one window per thread: the fast path's test (interior, one argmax, margin above the guard)
//      on the four summaries, in the same float operations; a passing window's 64 labels are
//      written at once; the others go to a slow list, with their candidate classes (a class whose
//      largest tap logit sits a guard below the best smallest one can neither win nor come within
//      2^-16 of the winner anywhere in the window: oct_row_labels_cand);
//   3. the slow windows' 16 tasks (8 rows x 2 four-pixel halves) over all threads:
//      oct_row_labels_cand where it decides, else oct_row_labels -- the oct kernel's arithmetic.
//      Border windows (a tap outside the image, zero weight) read their clamped taps from global
//      memory exactly as the oct kernel does.
// Labels are identical to the oct kernel's (test_gpu_head_nhwc.py).  Measured on the bench's network
// logits (scripts/head_micro.py, profiles/r9_head): SEG2 68.5 -> 40.4 us, NHWC 63.5 -> 35.8 us
// against the per-block form this replaced (each 8 x 4 block re-read and re-summarised its taps).
constexpr int kHeadTI = 8, kHeadTJ = 32;             // TI x TJ = 256 windows = one per thread
template <int NC, int LABEL_DTYPE, int SRC>
__global__ void __launch_bounds__(256)
up8_labels_tile_kernel(const void* __restrict__ logits, const float* __restrict__ up_w, void* __restrict__ labels,
                       int h, int w, int cs, const float* __restrict__ bias, const float* __restrict__ scale) {
  constexpr int TI = kHeadTI, TJ = kHeadTJ, PJ = TJ + 1, NPX = (TI + 1) * PJ;
  constexpr int VS = (NC + 3) / 4 * 4;               // LDS floats per pixel vector (16-B rows)
  static_assert(TI * TJ == 256, "one window per thread");
  __shared__ float wk[256];
  __shared__ float wstat[1];
  __shared__ __attribute__((aligned(16))) float vec[NPX][VS];
  __shared__ float smarg[NPX], sabsb[NPX];
  __shared__ int sam[NPX];                           // argmax | 0x100 when every class is finite
  __shared__ int nslow;
  __shared__ unsigned short slist[256];
  __shared__ uint32_t scm[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  wk[tid] = up_w[tid];
  if (tid == 0) nslow = 0;
  __syncthreads();
  if (wave == 0) {                                   // min over the 64 phases of sum w (0 if any w < 0)
    const int ky1 = lane >> 3, kx1 = lane & 7;
    const float a = wk[(ky1 + 8) * 16 + kx1 + 8], b = wk[(ky1 + 8) * 16 + kx1], c = wk[ky1 * 16 + kx1 + 8],
                d = wk[ky1 * 16 + kx1];
    float lo = fminf(fminf(a, b), fminf(c, d)) < 0.f ? 0.f : (a + b) + (c + d);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) lo = fminf(lo, __shfl_xor(lo, o));
    if (lane == 0) wstat[0] = lo;
  }
  const int H = h * 8, W = w * 8;
  const int I0 = blockIdx.y * TI, J0 = blockIdx.x * TJ;
  const int n = blockIdx.z;
  const int64_t plane = static_cast<int64_t>(h) * w;
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int64_t half = static_cast<int64_t>(gridDim.z) * plane * cs;
  constexpr int NCP = (NC + 3) / 4 * 4;
  auto load_px = [&](int iy, int ix, float (&d)[NC]) {
    float bv[NCP], sv[NCP];
#pragma unroll
    for (int k = 0; k < NCP; ++k) {
      bv[k] = SRC != 0 ? bias[k] : 0.f;
      sv[k] = SRC == 2 ? scale[k] : 0.f;
    }
    if constexpr (SRC == 2)
      load_taps_seg2_i8<NC>(static_cast<const int*>(logits) + static_cast<int64_t>(n) * plane * cs, half, w, cs, sv, bv,
                            iy, ix, d);
    else
      load_taps_nhwc<NC, SRC == 1>(static_cast<const float*>(logits) + static_cast<int64_t>(n) * plane * cs, half, w,
                                   cs, bv, iy, ix, d);
  };

  // ---- 1. the tile's 1/8-res pixels (tap rows I0 - 1 .. I0 + TI - 1, columns J0 - 1 .. J0 + TJ - 1)
  for (int px = tid; px < NPX; px += 256) {
    const int iy = I0 - 1 + px / PJ, ix = J0 - 1 + px % PJ;
    if (iy < 0 || iy >= h || ix < 0 || ix >= w) continue;   // only border windows use them (from global)
    float v[NC];
    load_px(iy, ix, v);
    // the per-tap summary: argmax, top-2 margin (running top-2, one v_med3 per class), |best|, finite
    float best = v[0], second = -INFINITY, vmaxabs = fabsf(v[0]);
    int am = 0;
#pragma unroll
    for (int k = 1; k < NC; ++k) {
      const float x = v[k];
      am = x > best ? k : am;
      second = __builtin_amdgcn_fmed3f(best, second, x);
      best = fmaxf(best, x);
      vmaxabs = __builtin_isnan(x) ? INFINITY : fmaxf(vmaxabs, fabsf(x));
    }
    vmaxabs = __builtin_isnan(v[0]) ? INFINITY : vmaxabs;
    smarg[px] = best - second;
    sabsb[px] = fabsf(best);
    sam[px] = am | (vmaxabs < INFINITY ? 0x100 : 0);
    float4* dst = reinterpret_cast<float4*>(vec[px]);
#pragma unroll
    for (int i = 0; i < VS / 4; ++i)
      dst[i] = make_float4(4 * i < NC ? v[4 * i] : 0.f, 4 * i + 1 < NC ? v[4 * i + 1] : 0.f,
                           4 * i + 2 < NC ? v[4 * i + 2] : 0.f, 4 * i + 3 < NC ? v[4 * i + 3] : 0.f);
  }
  __syncthreads();

  // ---- 2. one window per thread
  const float wmin = wstat[0];
  {
    const int ti = tid / TJ, tj = tid % TJ;
    const int i1 = I0 + ti, j1 = J0 + tj;
    if (i1 <= h && j1 <= w) {
      const bool interior = i1 >= 1 && i1 < h && j1 >= 1 && j1 < w;
      bool fast = false;
      int cls = 0;
      uint32_t cm = 0;
      if (interior) {
        const int p[4] = {ti * PJ + tj, ti * PJ + tj + 1, (ti + 1) * PJ + tj, (ti + 1) * PJ + tj + 1};
        cls = sam[p[0]] & 0xff;
        bool same = true, finite = true;
        float mmin = INFINITY, amax = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int a = sam[p[t]];
          same = same && (a & 0xff) == cls;
          finite = finite && (a & 0x100) != 0;
          mmin = fminf(mmin, smarg[p[t]]);
          amax = fmaxf(amax, sabsb[p[t]]);
        }
        fast = same && wmin > 0.f && finite && mmin >= 0x1p-16f / wmin * (1.f + 0x1p-10f) + 0x1p-20f * amax;
        if (!fast && finite && wmin > 0.f) {
          // candidate classes (see oct_row_labels_cand): kept when max_t L_t[k] >= max_j min_t L_t[j] - guard
          float vmaxabs = 0.f, lmax = -INFINITY;
#pragma unroll
          for (int k = 0; k < NC; ++k) {
            const float a0 = vec[p[0]][k], a1 = vec[p[1]][k], a2 = vec[p[2]][k], a3 = vec[p[3]][k];
            vmaxabs = fmaxf(vmaxabs, fmaxf(fmaxf(fabsf(a0), fabsf(a1)), fmaxf(fabsf(a2), fabsf(a3))));
            lmax = fmaxf(lmax, fminf(fminf(a0, a1), fminf(a2, a3)));
          }
          const float thr = lmax - (0x1p-16f / wmin * (1.f + 0x1p-10f) + 0x1p-20f * vmaxabs);
#pragma unroll
          for (int k = 0; k < NC; ++k) {
            const float u = fmaxf(fmaxf(vec[p[0]][k], vec[p[1]][k]), fmaxf(vec[p[2]][k], vec[p[3]][k]));
            cm |= (u >= thr ? 1u : 0u) << k;
          }
        }
      }
      if (fast) {
        const int la[4] = {cls, cls, cls, cls};
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int64_t row = static_cast<int64_t>(n) * HW + static_cast<int64_t>(8 * i1 - 4 + r) * W;
          store_labels4<LABEL_DTYPE>(labels, row + 8 * j1 - 4, la);
          store_labels4<LABEL_DTYPE>(labels, row + 8 * j1, la);
        }
      } else {
        const int at = atomicAdd(&nslow, 1);
        slist[at] = static_cast<unsigned short>(tid);
        scm[at] = cm;
      }
    }
  }
  __syncthreads();

  // ---- 3. the slow windows: 16 tasks each (row r, four-pixel half hh) over the workgroup
  const int ns = nslow;
  for (int tk = tid; tk < 16 * ns; tk += 256) {
    const int e = tk >> 4, r = tk & 7, hh = (tk >> 3) & 1;
    const int wt = slist[e];
    const int ti = wt / TJ, tj = wt % TJ;
    const int i1 = I0 + ti, j1 = J0 + tj;
    const int q = 2 * j1 - 1 + hh;                   // output columns 4 q .. 4 q + 3
    const int oy = 8 * i1 - 4 + r;
    if (q < 0 || 4 * q >= W || oy < 0 || oy >= H) continue;
    const int kx1_0 = 4 * q + 4 - 8 * j1;
    const int64_t pix = static_cast<int64_t>(n) * HW + static_cast<int64_t>(oy) * W + 4 * q;
    const bool vi0 = i1 - 1 >= 0, vi1 = i1 < h, vj0 = j1 - 1 >= 0, vj1 = j1 < w;
    int arg[4];
    float t[4][NC];
    if (vi0 && vi1 && vj0 && vj1) {
      const int p00 = ti * PJ + tj;
      const uint32_t cm = scm[e];
      if (cm != 0) {
        if (oct_row_labels_cand<NC>(vec[p00], vec[p00 + 1], vec[p00 + PJ], vec[p00 + PJ + 1], cm, wk, r, kx1_0, arg)) {
          store_labels4<LABEL_DTYPE>(labels, pix, arg);
          continue;
        }
      }
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        t[0][k] = vec[p00][k];
        t[1][k] = vec[p00 + 1][k];
        t[2][k] = vec[p00 + PJ][k];
        t[3][k] = vec[p00 + PJ + 1][k];
      }
    } else {                                         // border window: the oct kernel's clamped taps
      const int ci0 = vi0 ? i1 - 1 : 0, ci1 = vi1 ? i1 : 0, cj0 = vj0 ? j1 - 1 : 0, cj1 = vj1 ? j1 : 0;
      load_px(ci0, cj0, t[0]);
      load_px(ci0, cj1, t[1]);
      load_px(ci1, cj0, t[2]);
      load_px(ci1, cj1, t[3]);
    }
    oct_row_labels<NC>(t[0], t[1], t[2], t[3], wk, r, kx1_0, vi0, vi1, vj0, vj1, arg);
    store_labels4<LABEL_DTYPE>(labels, pix, arg);
  }
}

// ---------------------------------------------------------------- bilinear x8 (use_torch_up)
// nn.UpsamplingBilinear2d(scale_factor=8) (lmodels/drnseg.py:285-287): bilinear with
// align_corners=True, output 8h x 8w.  Source index and weights as ATen's CPU kernel:
// scale = (in - 1) / (out - 1) in fp32, src = scale * dst, i0 = floor(src), i1 = i0 + (i0 < in-1),
// l1 = src - i0, l0 = 1 - l1; value = l0h * (l0w * x00 + l1w * x01) + l1h * (l0w * x10 + l1w * x11).
__device__ __forceinline__ void bilinear_ac_index(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = out > 1 ? static_cast<float>(in - 1) / static_cast<float>(out - 1) : 0.f;
  const float src = scale * static_cast<float>(dst);
  i0 = static_cast<int>(floorf(src));
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = fminf(fmaxf(src - static_cast<float>(i0), 0.f), 1.f);
  l0 = 1.f - l1;
}

template <int LABEL_DTYPE>
__global__ void __launch_bounds__(256)
up8_bilinear_lsm_kernel(const float* __restrict__ logits, float* __restrict__ logprobs, void* __restrict__ labels,
                        int c, int h, int w) {
  const int H = h * 8, W = w * 8;
  const int ox = blockIdx.x * blockDim.x + threadIdx.x;
  const int oy = blockIdx.y;
  const int n = blockIdx.z;
  if (ox >= W) return;
  int y0, y1, x0, x1;
  float hy0, hy1, wx0, wx1;
  bilinear_ac_index(oy, h, H, y0, y1, hy0, hy1);
  bilinear_ac_index(ox, w, W, x0, x1, wx0, wx1);
  const int64_t plane = static_cast<int64_t>(h) * w;
  const float* src = logits + static_cast<int64_t>(n) * c * plane;
  float v[kMaxClasses];
  float vmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < kMaxClasses; ++k) {
    if (k < c) {
      const float* s = src + k * plane;
      const float top = wx0 * s[y0 * w + x0] + wx1 * s[y0 * w + x1];
      const float bot = wx0 * s[y1 * w + x0] + wx1 * s[y1 * w + x1];
      const float a = hy0 * top + hy1 * bot;
      v[k] = a;
      vmax = fmaxf(vmax, a);
    }
  }
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxClasses; ++k) {
    if (k < c) sum += expf(v[k] - vmax);
  }
  const float lse = logf(sum);
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int64_t pix = static_cast<int64_t>(oy) * W + ox;
  float best = -INFINITY;
  int arg = 0;
#pragma unroll
  for (int k = 0; k < kMaxClasses; ++k) {
    if (k < c) {
      const float lp = (v[k] - vmax) - lse;
      if (logprobs != nullptr) logprobs[(static_cast<int64_t>(n) * c + k) * HW + pix] = lp;
      if (lp > best) { best = lp; arg = k; }
    }
  }
  if (labels != nullptr) {
    if (LABEL_DTYPE == DRNMI_U8) reinterpret_cast<uint8_t*>(labels)[static_cast<int64_t>(n) * HW + pix] = static_cast<uint8_t>(arg);
    else reinterpret_cast<int64_t*>(labels)[static_cast<int64_t>(n) * HW + pix] = arg;
  }
}

// ---------------------------------------------------------------- mask apply
constexpr int kMaskBatch = 32;

struct MaskBatchF32 {
  float* w[kMaskBatch];
  const float* m[kMaskBatch];
  int64_t numel[kMaskBatch];
};

struct MaskBatchBits {
  float* w[kMaskBatch];
  const uint32_t* m[kMaskBatch];
  int64_t numel[kMaskBatch];
};

// blockIdx.y = tensor; grid-stride over float4 groups, scalar tail.
__global__ void __launch_bounds__(256) mask_apply_f32_kernel(const MaskBatchF32 b) {
  const int t = blockIdx.y;
  float* __restrict__ w = b.w[t];
  const float* __restrict__ m = b.m[t];
  const int64_t n = b.numel[t];
  const int64_t n4 = n >> 2;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 wv = reinterpret_cast<float4*>(w)[i];
    const float4 mv = reinterpret_cast<const float4*>(m)[i];
    wv.x *= mv.x; wv.y *= mv.y; wv.z *= mv.z; wv.w *= mv.w;
    reinterpret_cast<float4*>(w)[i] = wv;
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) w[i] *= m[i];
  }
}

// One thread per 32-element group: one mask word, 8 float4 loads/stores.  The multiply
// by 1.0f / 0.0f keeps the reference's exact result (including -0.0 for negative w).
__global__ void __launch_bounds__(256) mask_apply_bits_kernel(const MaskBatchBits b) {
  const int t = blockIdx.y;
  float* __restrict__ w = b.w[t];
  const uint32_t* __restrict__ m = b.m[t];
  const int64_t n = b.numel[t];
  const int64_t groups = (n + 31) >> 5;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < groups; g += stride) {
    const uint32_t bits = m[g];
    const int64_t e0 = g << 5;
    if (e0 + 32 <= n) {
      float4* p = reinterpret_cast<float4*>(w + e0);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float4 v = p[q];
        v.x *= static_cast<float>((bits >> (4 * q + 0)) & 1u);
        v.y *= static_cast<float>((bits >> (4 * q + 1)) & 1u);
        v.z *= static_cast<float>((bits >> (4 * q + 2)) & 1u);
        v.w *= static_cast<float>((bits >> (4 * q + 3)) & 1u);
        p[q] = v;
      }
    } else {
      for (int q = 0; e0 + q < n; ++q) w[e0 + q] *= static_cast<float>((bits >> q) & 1u);
    }
  }
}

// ---------------------------------------------------------------- confusion matrix (eval)
// hist[label * n + pred] += 1 over pixels with 0 <= label < n and pred < n
// (semantic_seg.py:293-296 fast_hist; per-block LDS histogram, one global atomic per bin).
constexpr int kMaxHistClasses = 32;

template <typename TP, typename TL>
__global__ void __launch_bounds__(256)
confusion_kernel(const TP* __restrict__ pred, const TL* __restrict__ label, int64_t npix, int n,
                 unsigned long long* __restrict__ hist) {
  __shared__ unsigned int h[kMaxHistClasses * kMaxHistClasses];
  for (int i = threadIdx.x; i < n * n; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < npix; i += stride) {
    const int64_t l = static_cast<int64_t>(label[i]);
    const int64_t p = static_cast<int64_t>(pred[i]);
    if (l >= 0 && l < n && p >= 0 && p < n) atomicAdd(&h[l * n + p], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n * n; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], static_cast<unsigned long long>(h[i]));
}

inline unsigned grid1d(int64_t n, int block = 256) {
  return static_cast<unsigned>((n + block - 1) / block);
}

}  // namespace
}  // namespace drnmi

using namespace drnmi;

extern "C" int drnmi_frame_ingest_u8(const uint8_t* frames, void* out, int32_t n, int32_t h, int32_t w,
                                     const float* mean3, const float* std3, int32_t bgr,
                                     int32_t out_dtype, void* stream) {
  if (frames == nullptr || out == nullptr || mean3 == nullptr || std3 == nullptr) return DRNMI_EINVAL;
  if (n <= 0 || h <= 0 || w <= 0) return DRNMI_EINVAL;
  const int64_t npix = static_cast<int64_t>(n) * h * w;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (out_dtype == DRNMI_BF16) {
    hipLaunchKernelGGL(frame_ingest_kernel<bf16_t>, dim3(grid1d(npix)), dim3(256), 0, s, frames,
                       reinterpret_cast<bf16_t*>(out), npix, mean3[0], mean3[1], mean3[2], std3[0],
                       std3[1], std3[2], bgr);
  } else if (out_dtype == DRNMI_F32) {
    hipLaunchKernelGGL(frame_ingest_kernel<float>, dim3(grid1d(npix)), dim3(256), 0, s, frames,
                       reinterpret_cast<float*>(out), npix, mean3[0], mean3[1], mean3[2], std3[0],
                       std3[1], std3[2], bgr);
  } else {
    return DRNMI_EINVAL;
  }
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_nchw_to_nhwc(const float* x, void* out, int32_t n, int32_t c, int32_t h, int32_t w,
                                  int32_t c_pad, int32_t out_dtype, void* stream) {
  if (x == nullptr || out == nullptr || n <= 0 || c <= 0 || h <= 0 || w <= 0 || c_pad < c) return DRNMI_EINVAL;
  const int64_t hw = static_cast<int64_t>(h) * w;
  const int64_t total = static_cast<int64_t>(n) * hw;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (out_dtype == DRNMI_BF16) {
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16_t>, dim3(grid1d(total)), dim3(256), 0, s, x,
                       reinterpret_cast<bf16_t*>(out), c, hw, c_pad, total);
  } else if (out_dtype == DRNMI_F32) {
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(grid1d(total)), dim3(256), 0, s, x,
                       reinterpret_cast<float*>(out), c, hw, c_pad, total);
  } else {
    return DRNMI_EINVAL;
  }
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_nhwc_to_nchw(const void* x, float* out, int32_t n, int32_t c, int32_t h, int32_t w,
                                  int32_t c_stride, int32_t in_dtype, void* stream) {
  if (x == nullptr || out == nullptr || n <= 0 || c <= 0 || h <= 0 || w <= 0 || c_stride < c) return DRNMI_EINVAL;
  const int64_t hw = static_cast<int64_t>(h) * w;
  const int64_t total = static_cast<int64_t>(n) * c * hw;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (in_dtype == DRNMI_BF16) {
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<bf16_t>, dim3(grid1d(total)), dim3(256), 0, s,
                       reinterpret_cast<const bf16_t*>(x), out, c, hw, c_stride, total);
  } else if (in_dtype == DRNMI_F32) {
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, dim3(grid1d(total)), dim3(256), 0, s,
                       reinterpret_cast<const float*>(x), out, c, hw, c_stride, total);
  } else {
    return DRNMI_EINVAL;
  }
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_up8_labels_nhwc(const float* logits, int32_t cs, const float* up_w, void* labels,
                                     int32_t label_dtype, int32_t n, int32_t c, int32_t h, int32_t w, void* stream) {
  if (logits == nullptr || up_w == nullptr || labels == nullptr || n <= 0 || h <= 0 || w <= 0) return DRNMI_EINVAL;
  if (c != 19) return DRNMI_ENOTSUP;                   // the 19-class oct kernel
  if (cs < c || cs % 4 != 0 || (reinterpret_cast<uintptr_t>(logits) & 15) != 0) return DRNMI_EINVAL;
  if (label_dtype != DRNMI_U8 && label_dtype != DRNMI_I64) return DRNMI_EINVAL;
  if (h + 1 > 65535 || n > 65535) return DRNMI_EINVAL;
  const dim3 gt(static_cast<unsigned>((w + kHeadTJ) / kHeadTJ), static_cast<unsigned>((h + kHeadTI) / kHeadTI),
                static_cast<unsigned>(n));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (label_dtype == DRNMI_I64)
    hipLaunchKernelGGL((up8_labels_tile_kernel<19, DRNMI_I64, 0>), gt, dim3(256), 0, s, logits, up_w, labels, h, w, cs,
                       nullptr, nullptr);
  else
    hipLaunchKernelGGL((up8_labels_tile_kernel<19, DRNMI_U8, 0>), gt, dim3(256), 0, s, logits, up_w, labels, h, w, cs,
                       nullptr, nullptr);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_up8_labels_seg2(const float* partials, int32_t cs, const float* bias, const float* up_w,
                                     void* labels, int32_t label_dtype, int32_t n, int32_t c, int32_t h, int32_t w,
                                     void* stream) {
  if (partials == nullptr || bias == nullptr || up_w == nullptr || labels == nullptr || n <= 0 || h <= 0 || w <= 0)
    return DRNMI_EINVAL;
  if (c != 19) return DRNMI_ENOTSUP;
  if (cs < 20 || cs % 4 != 0 || (reinterpret_cast<uintptr_t>(partials) & 15) != 0) return DRNMI_EINVAL;
  if (label_dtype != DRNMI_U8 && label_dtype != DRNMI_I64) return DRNMI_EINVAL;
  if (h + 1 > 65535 || n > 65535) return DRNMI_EINVAL;
  const dim3 gt(static_cast<unsigned>((w + kHeadTJ) / kHeadTJ), static_cast<unsigned>((h + kHeadTI) / kHeadTI),
                static_cast<unsigned>(n));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (label_dtype == DRNMI_I64)
    hipLaunchKernelGGL((up8_labels_tile_kernel<19, DRNMI_I64, 1>), gt, dim3(256), 0, s, partials, up_w, labels, h, w, cs,
                       bias, nullptr);
  else
    hipLaunchKernelGGL((up8_labels_tile_kernel<19, DRNMI_U8, 1>), gt, dim3(256), 0, s, partials, up_w, labels, h, w, cs,
                       bias, nullptr);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_up8_labels_seg2_i8(const int32_t* partials, int32_t cs, const float* scale, const float* shift,
                                        const float* up_w, void* labels, int32_t label_dtype, int32_t n, int32_t c,
                                        int32_t h, int32_t w, void* stream) {
  if (partials == nullptr || scale == nullptr || shift == nullptr || up_w == nullptr || labels == nullptr || n <= 0 ||
      h <= 0 || w <= 0)
    return DRNMI_EINVAL;
  if (c != 19) return DRNMI_ENOTSUP;
  if (cs < 20 || cs % 4 != 0 || (reinterpret_cast<uintptr_t>(partials) & 15) != 0) return DRNMI_EINVAL;
  if (label_dtype != DRNMI_U8 && label_dtype != DRNMI_I64) return DRNMI_EINVAL;
  if (h + 1 > 65535 || n > 65535) return DRNMI_EINVAL;
  const dim3 gt(static_cast<unsigned>((w + kHeadTJ) / kHeadTJ), static_cast<unsigned>((h + kHeadTI) / kHeadTI),
                static_cast<unsigned>(n));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (label_dtype == DRNMI_I64)
    hipLaunchKernelGGL((up8_labels_tile_kernel<19, DRNMI_I64, 2>), gt, dim3(256), 0, s, partials, up_w, labels, h, w, cs,
                       shift, scale);
  else
    hipLaunchKernelGGL((up8_labels_tile_kernel<19, DRNMI_U8, 2>), gt, dim3(256), 0, s, partials, up_w, labels, h, w, cs,
                       shift, scale);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_up8_logsoftmax_argmax(const float* logits, const float* up_w, float* logprobs,
                                           void* labels, int32_t label_dtype, int32_t n, int32_t c,
                                           int32_t h, int32_t w, void* stream) {
  if (logits == nullptr || up_w == nullptr || n <= 0 || h <= 0 || w <= 0) return DRNMI_EINVAL;
  if (c <= 0 || c > kMaxClasses) return DRNMI_ENOTSUP;
  if (labels != nullptr && label_dtype != DRNMI_U8 && label_dtype != DRNMI_I64) return DRNMI_EINVAL;
  if (static_cast<int64_t>(h) * 8 > 65535 || n > 65535) return DRNMI_EINVAL;
  const int W = w * 8;
  dim3 grid(static_cast<unsigned>((W + 255) / 256), static_cast<unsigned>(h * 8), static_cast<unsigned>(n));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (c == 19 && logprobs == nullptr && labels != nullptr) {   // labels only: 8-row kernel
    dim3 go(static_cast<unsigned>((W / 4 + 255) / 256), static_cast<unsigned>(h + 1), static_cast<unsigned>(n));
    if (label_dtype == DRNMI_I64) {
      hipLaunchKernelGGL((up8_labels_oct_kernel<19, DRNMI_I64>), go, dim3(256), 0, s, logits, up_w, labels, h, w);
    } else {
      hipLaunchKernelGGL((up8_labels_oct_kernel<19, DRNMI_U8>), go, dim3(256), 0, s, logits, up_w, labels, h, w);
    }
    return static_cast<int>(hipGetLastError());
  }
  if (c == 19) {   // Cityscapes classes: quad kernel
    dim3 gq(static_cast<unsigned>((W / 4 + 255) / 256), static_cast<unsigned>(h * 8), static_cast<unsigned>(n));
    if (label_dtype == DRNMI_I64) {
      hipLaunchKernelGGL((up8_lsm_quad_kernel<19, DRNMI_I64>), gq, dim3(256), 0, s, logits, up_w, logprobs, labels, h, w);
    } else {
      hipLaunchKernelGGL((up8_lsm_quad_kernel<19, DRNMI_U8>), gq, dim3(256), 0, s, logits, up_w, logprobs, labels, h, w);
    }
    return static_cast<int>(hipGetLastError());
  }
  if (label_dtype == DRNMI_I64) {
    hipLaunchKernelGGL(up8_lsm_kernel<DRNMI_I64>, grid, dim3(256), 0, s, logits, up_w, logprobs, labels, c, h, w);
  } else {
    hipLaunchKernelGGL(up8_lsm_kernel<DRNMI_U8>, grid, dim3(256), 0, s, logits, up_w, logprobs, labels, c, h, w);
  }
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_up8_bilinear_logsoftmax_argmax(const float* logits, float* logprobs, void* labels,
                                                    int32_t label_dtype, int32_t n, int32_t c, int32_t h, int32_t w,
                                                    void* stream) {
  if (logits == nullptr || n <= 0 || h <= 0 || w <= 0) return DRNMI_EINVAL;
  if (c <= 0 || c > kMaxClasses) return DRNMI_ENOTSUP;
  if (labels != nullptr && label_dtype != DRNMI_U8 && label_dtype != DRNMI_I64) return DRNMI_EINVAL;
  if (static_cast<int64_t>(h) * 8 > 65535 || n > 65535) return DRNMI_EINVAL;
  const int W = w * 8;
  dim3 grid(static_cast<unsigned>((W + 255) / 256), static_cast<unsigned>(h * 8), static_cast<unsigned>(n));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (label_dtype == DRNMI_I64)
    hipLaunchKernelGGL(up8_bilinear_lsm_kernel<DRNMI_I64>, grid, dim3(256), 0, s, logits, logprobs, labels, c, h, w);
  else
    hipLaunchKernelGGL(up8_bilinear_lsm_kernel<DRNMI_U8>, grid, dim3(256), 0, s, logits, logprobs, labels, c, h, w);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_mask_apply_f32(int32_t ntensors, float* const* weights, const float* const* masks,
                                    const int64_t* numels, void* stream) {
  if (ntensors < 0 || (ntensors > 0 && (weights == nullptr || masks == nullptr || numels == nullptr)))
    return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (int t0 = 0; t0 < ntensors; t0 += kMaskBatch) {
    MaskBatchF32 b{};
    const int cnt = ntensors - t0 < kMaskBatch ? ntensors - t0 : kMaskBatch;
    int64_t maxn = 0;
    for (int i = 0; i < cnt; ++i) {
      b.w[i] = weights[t0 + i];
      b.m[i] = masks[t0 + i];
      b.numel[i] = numels[t0 + i];
      if (b.numel[i] < 0) return DRNMI_EINVAL;
      if (b.numel[i] > 0 && (b.w[i] == nullptr || b.m[i] == nullptr)) return DRNMI_EINVAL;
      if ((reinterpret_cast<uintptr_t>(b.w[i]) | reinterpret_cast<uintptr_t>(b.m[i])) & 15) return DRNMI_EINVAL;
      maxn = b.numel[i] > maxn ? b.numel[i] : maxn;
    }
    if (maxn == 0) continue;
    unsigned gx = grid1d((maxn + 3) / 4);
    gx = gx > 1024 ? 1024 : (gx == 0 ? 1 : gx);
    hipLaunchKernelGGL(mask_apply_f32_kernel, dim3(gx, cnt), dim3(256), 0, s, b);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return DRNMI_OK;
}

extern "C" int drnmi_mask_apply_bits_f32(int32_t ntensors, float* const* weights,
                                         const uint32_t* const* mask_bits, const int64_t* numels,
                                         void* stream) {
  if (ntensors < 0 || (ntensors > 0 && (weights == nullptr || mask_bits == nullptr || numels == nullptr)))
    return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (int t0 = 0; t0 < ntensors; t0 += kMaskBatch) {
    MaskBatchBits b{};
    const int cnt = ntensors - t0 < kMaskBatch ? ntensors - t0 : kMaskBatch;
    int64_t maxn = 0;
    for (int i = 0; i < cnt; ++i) {
      b.w[i] = weights[t0 + i];
      b.m[i] = mask_bits[t0 + i];
      b.numel[i] = numels[t0 + i];
      if (b.numel[i] < 0) return DRNMI_EINVAL;
      if (b.numel[i] > 0 && (b.w[i] == nullptr || b.m[i] == nullptr)) return DRNMI_EINVAL;
      if (reinterpret_cast<uintptr_t>(b.w[i]) & 15) return DRNMI_EINVAL;
      maxn = b.numel[i] > maxn ? b.numel[i] : maxn;
    }
    if (maxn == 0) continue;
    unsigned gx = grid1d((maxn + 31) / 32);
    gx = gx > 1024 ? 1024 : (gx == 0 ? 1 : gx);
    hipLaunchKernelGGL(mask_apply_bits_kernel, dim3(gx, cnt), dim3(256), 0, s, b);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return DRNMI_OK;
}

extern "C" const char* drnmi_version(void) { return "drnmi 0.1.0 gfx950"; }
extern "C" int32_t drnmi_abi_version(void) { return DRNMI_ABI_VERSION; }
extern "C" int64_t drnmi_conv_args_size(void) { return static_cast<int64_t>(sizeof(drnmi_conv_args)); }

extern "C" int drnmi_confusion_matrix(const void* pred, int32_t pred_dtype, const void* label,
                                      int32_t label_dtype, int64_t npix, int32_t nclass, int64_t* hist,
                                      void* stream) {
  if (pred == nullptr || label == nullptr || hist == nullptr || npix < 0) return DRNMI_EINVAL;
  if (nclass <= 0 || nclass > kMaxHistClasses) return DRNMI_ENOTSUP;
  if ((pred_dtype != DRNMI_U8 && pred_dtype != DRNMI_I64) || (label_dtype != DRNMI_U8 && label_dtype != DRNMI_I64))
    return DRNMI_EINVAL;
  if (npix == 0) return DRNMI_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  unsigned g = grid1d(npix);
  g = g > 2048 ? 2048 : g;
  auto* h = reinterpret_cast<unsigned long long*>(hist);
  if (pred_dtype == DRNMI_U8 && label_dtype == DRNMI_U8)
    hipLaunchKernelGGL((confusion_kernel<uint8_t, uint8_t>), dim3(g), dim3(256), 0, s,
                       (const uint8_t*)pred, (const uint8_t*)label, npix, nclass, h);
  else if (pred_dtype == DRNMI_U8)
    hipLaunchKernelGGL((confusion_kernel<uint8_t, int64_t>), dim3(g), dim3(256), 0, s,
                       (const uint8_t*)pred, (const int64_t*)label, npix, nclass, h);
  else if (label_dtype == DRNMI_U8)
    hipLaunchKernelGGL((confusion_kernel<int64_t, uint8_t>), dim3(g), dim3(256), 0, s,
                       (const int64_t*)pred, (const uint8_t*)label, npix, nclass, h);
  else
    hipLaunchKernelGGL((confusion_kernel<int64_t, int64_t>), dim3(g), dim3(256), 0, s,
                       (const int64_t*)pred, (const int64_t*)label, npix, nclass, h);
  return static_cast<int>(hipGetLastError());
}
