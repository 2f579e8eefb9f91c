// Bilinear resize with PIL's arithmetic (the seg_video ingest and the multi-scale eval).
//
//   * seg_video_old_no_plot.py:123-127: every decoded frame goes through T.Resize((300, 300)),
//     which for a PIL image is Image.resize(size, BILINEAR) -- Pillow's separable two-pass
//     resampler (antialiasing: the bilinear support widens with the downscale factor), 8-bit
//     fixed point with 22 fractional bits, horizontal pass first into a uint8 intermediate.
//   * semantic_seg.py:471-504 (resize_4d_tensor, used by test_ms :507-557): each fp32 log-prob
//     plane is resized to the input size with Image.fromarray(plane).resize((w, h), BILINEAR)
//     -- the 'F' mode path: fp32 pixels times double coefficients summed in double, rounded to
//     fp32 after each pass -- and the scales are summed in fp32.
//
// The coefficient tables are Pillow's precompute_coeffs (Resample.c) computed per output
// coordinate on the GPU in double with contraction disabled (the C reference rounds every step),
// so the tables, and therefore every output pixel, are bit-identical to Pillow's.
// Layout: uint8 frames HWC3 [n][h][w][3]; fp32 planes [planes][h][w].
#include "common.h"
#include "kernels.h"

#include <math.h>

namespace drnmi {
namespace {

constexpr int kThreads = 256;
constexpr int kPrecisionBits = 32 - 8 - 2;   // Pillow PRECISION_BITS

struct Axis {
  int in, out, ksize;
  double scale, filterscale, support;
};

Axis make_axis(int in, int out) {
  Axis a;
  a.in = in;
  a.out = out;
  a.scale = static_cast<double>(static_cast<float>(in) - 0.0f) / out;   // (in1 - in0) / outSize, box = (0, in)
  a.filterscale = a.scale < 1.0 ? 1.0 : a.scale;
  a.support = 1.0 * a.filterscale;                                      // bilinear support 1.0
  a.ksize = static_cast<int>(ceil(a.support)) * 2 + 1;
  return a;
}

// one thread per output coordinate: bounds (xmin, xmax) and the normalised double weights
// (Pillow precompute_coeffs), plus their 8-bit fixed-point form (normalize_coeffs_8bpc)
__global__ void __launch_bounds__(kThreads)
coeffs_kernel(int in, int out, int ksize, double scale, double filterscale, double support, int* __restrict__ bounds,
              double* __restrict__ kk, int* __restrict__ kk8) {
#pragma clang fp contract(off)
  const int xx = blockIdx.x * blockDim.x + threadIdx.x;
  if (xx >= out) return;
  const double center = 0.0 + (xx + 0.5) * scale;
  double ww = 0.0;
  const double ss = 1.0 / filterscale;
  int xmin = static_cast<int>(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = static_cast<int>(center + support + 0.5);
  if (xmax > in) xmax = in;
  xmax -= xmin;
  double* k = kk + static_cast<int64_t>(xx) * ksize;
  for (int x = 0; x < xmax; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    const double w = t < 1.0 ? 1.0 - t : 0.0;
    k[x] = w;
    ww += w;
  }
  for (int x = 0; x < xmax; ++x)
    if (ww != 0.0) k[x] /= ww;
  for (int x = xmax; x < ksize; ++x) k[x] = 0.0;
  int* k8 = kk8 + static_cast<int64_t>(xx) * ksize;
  for (int x = 0; x < ksize; ++x)
    k8[x] = k[x] < 0 ? static_cast<int>(-0.5 + k[x] * (1 << kPrecisionBits))
                     : static_cast<int>(0.5 + k[x] * (1 << kPrecisionBits));
  bounds[2 * xx] = xmin;
  bounds[2 * xx + 1] = xmax;
}

__device__ __forceinline__ uint8_t clip8(int v) {
  if (v >= (1 << kPrecisionBits << 8)) return 255;
  if (v <= 0) return 0;
  return static_cast<uint8_t>(v >> kPrecisionBits);
}

// horizontal pass, uint8 HWC3: rows [row0, row0 + rows) of each frame -> tmp [n][rows][ow][3]
__global__ void __launch_bounds__(kThreads)
resize_h_u8_kernel(const uint8_t* __restrict__ src, int n, int h, int w, int row0, int rows, int ow, int ksize,
                   const int* __restrict__ bounds, const int* __restrict__ kk8, uint8_t* __restrict__ dst) {
  const int64_t total = static_cast<int64_t>(n) * rows * ow;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int xx = static_cast<int>(i % ow);
    const int yy = static_cast<int>((i / ow) % rows);
    const int f = static_cast<int>(i / (static_cast<int64_t>(ow) * rows));
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const int* k = kk8 + static_cast<int64_t>(xx) * ksize;
    const uint8_t* row = src + ((static_cast<int64_t>(f) * h + row0 + yy) * w + xmin) * 3;
    int s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < xmax; ++x) {
      s0 += row[3 * x + 0] * k[x];
      s1 += row[3 * x + 1] * k[x];
      s2 += row[3 * x + 2] * k[x];
    }
    uint8_t* o = dst + i * 3;
    o[0] = clip8(s0);
    o[1] = clip8(s1);
    o[2] = clip8(s2);
  }
}

// vertical pass, uint8 HWC3: src [n][sh][ow][3] -> dst [n][oh][ow][3] (bounds already relative to src)
__global__ void __launch_bounds__(kThreads)
resize_v_u8_kernel(const uint8_t* __restrict__ src, int n, int sh, int ow, int oh, int ksize, int shift,
                   const int* __restrict__ bounds, const int* __restrict__ kk8, uint8_t* __restrict__ dst) {
  const int64_t total = static_cast<int64_t>(n) * oh * ow;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int xx = static_cast<int>(i % ow);
    const int yy = static_cast<int>((i / ow) % oh);
    const int f = static_cast<int>(i / (static_cast<int64_t>(ow) * oh));
    const int ymin = bounds[2 * yy] - shift, ymax = bounds[2 * yy + 1];
    const int* k = kk8 + static_cast<int64_t>(yy) * ksize;
    int s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
    for (int y = 0; y < ymax; ++y) {
      const uint8_t* px = src + ((static_cast<int64_t>(f) * sh + ymin + y) * ow + xx) * 3;
      s0 += px[0] * k[y];
      s1 += px[1] * k[y];
      s2 += px[2] * k[y];
    }
    uint8_t* o = dst + i * 3;
    o[0] = clip8(s0);
    o[1] = clip8(s1);
    o[2] = clip8(s2);
  }
}

// fp32 ('F' mode) passes: fp32 x double, summed in double, stored fp32
__global__ void __launch_bounds__(kThreads)
resize_h_f32_kernel(const float* __restrict__ src, int planes, int h, int w, int row0, int rows, int ow, int ksize,
                    const int* __restrict__ bounds, const double* __restrict__ kk, float* __restrict__ dst) {
#pragma clang fp contract(off)
  const int64_t total = static_cast<int64_t>(planes) * rows * ow;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int xx = static_cast<int>(i % ow);
    const int yy = static_cast<int>((i / ow) % rows);
    const int64_t pl = i / (static_cast<int64_t>(ow) * rows);
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const double* k = kk + static_cast<int64_t>(xx) * ksize;
    const float* row = src + (pl * h + row0 + yy) * w + xmin;
    double ss = 0.0;
    for (int x = 0; x < xmax; ++x) ss += static_cast<double>(row[x]) * k[x];
    dst[i] = static_cast<float>(ss);
  }
}

__global__ void __launch_bounds__(kThreads)
resize_v_f32_kernel(const float* __restrict__ src, int planes, int sh, int ow, int oh, int ksize, int shift,
                    const int* __restrict__ bounds, const double* __restrict__ kk, float* __restrict__ dst,
                    int accumulate) {
#pragma clang fp contract(off)
  const int64_t total = static_cast<int64_t>(planes) * oh * ow;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int xx = static_cast<int>(i % ow);
    const int yy = static_cast<int>((i / ow) % oh);
    const int64_t pl = i / (static_cast<int64_t>(ow) * oh);
    const int ymin = bounds[2 * yy] - shift, ymax = bounds[2 * yy + 1];
    const double* k = kk + static_cast<int64_t>(yy) * ksize;
    double ss = 0.0;
    for (int y = 0; y < ymax; ++y) ss += static_cast<double>(src[(pl * sh + ymin + y) * ow + xx]) * k[y];
    const float v = static_cast<float>(ss);
    dst[i] = accumulate ? dst[i] + v : v;
  }
}

// identity pass for an axis Pillow does not resample (copy / accumulate)
__global__ void __launch_bounds__(kThreads)
copy_f32_kernel(const float* __restrict__ src, int64_t total, float* __restrict__ dst, int accumulate) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[i] = accumulate ? dst[i] + src[i] : src[i];
}

template <int LABEL_DTYPE>
__global__ void __launch_bounds__(kThreads)
argmax_nchw_kernel(const float* __restrict__ x, int n, int c, int64_t hw, void* __restrict__ labels) {
  const int64_t total = static_cast<int64_t>(n) * hw;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t b = i / hw, p = i - b * hw;
    const float* v = x + b * c * hw + p;
    float best = v[0];
    int arg = 0;
    for (int k = 1; k < c; ++k) {
      const float t = v[k * hw];
      if (t > best || (t != t && best == best)) {   // numpy argmax: first maximum, NaN wins
        best = t;
        arg = k;
      }
    }
    if (LABEL_DTYPE == DRNMI_U8) reinterpret_cast<uint8_t*>(labels)[i] = static_cast<uint8_t>(arg);
    else reinterpret_cast<int64_t*>(labels)[i] = arg;
  }
}

unsigned grid_of(int64_t n) {
  const int64_t b = (n + kThreads - 1) / kThreads;
  return static_cast<unsigned>(b < 65536 ? (b > 0 ? b : 1) : 65536);
}

struct Plan {
  Axis ax, ay;
  bool need_h, need_v;
  int row0, rows;                 // source rows the vertical pass reads
  int64_t off_bh, off_kh, off_k8h, off_bv, off_kv, off_k8v, off_tmp, bytes;
};

int64_t align256(int64_t v) { return (v + 255) / 256 * 256; }

// Workspace layout and the vertical pass's source-row window (needs the vertical bounds, which
// are only known on the device; the window is bounded instead: the rows of the first and last
// output row's support, computed here with the same double formula on the host).
Plan make_plan(int n, int h, int w, int oh, int ow, int elem) {
  Plan q;
  q.ax = make_axis(w, ow);
  q.ay = make_axis(h, oh);
  q.need_h = ow != w;
  q.need_v = oh != h;
  auto bound = [](const Axis& a, int xx, int& xmin, int& xmax) {
    const double center = 0.0 + (xx + 0.5) * a.scale;
    xmin = static_cast<int>(center - a.support + 0.5);
    if (xmin < 0) xmin = 0;
    xmax = static_cast<int>(center + a.support + 0.5);
    if (xmax > a.in) xmax = a.in;
  };
  int f0, f1, l0, l1;
  bound(q.ay, 0, f0, f1);
  bound(q.ay, oh - 1, l0, l1);
  q.row0 = q.need_h ? f0 : 0;                 // Pillow: ybox_first / ybox_last
  q.rows = q.need_h ? l1 - f0 : h;
  int64_t o = 0;
  q.off_bh = o; o = align256(o + 8LL * ow);
  q.off_kh = o; o = align256(o + 8LL * ow * q.ax.ksize);
  q.off_k8h = o; o = align256(o + 4LL * ow * q.ax.ksize);
  q.off_bv = o; o = align256(o + 8LL * oh);
  q.off_kv = o; o = align256(o + 8LL * oh * q.ay.ksize);
  q.off_k8v = o; o = align256(o + 4LL * oh * q.ay.ksize);
  q.off_tmp = o; o = align256(o + static_cast<int64_t>(n) * q.rows * ow * elem);
  q.bytes = o;
  return q;
}

void launch_coeffs(const Plan& q, char* ws, hipStream_t s) {
  hipLaunchKernelGGL(coeffs_kernel, dim3(grid_of(q.ax.out)), dim3(kThreads), 0, s, q.ax.in, q.ax.out, q.ax.ksize,
                     q.ax.scale, q.ax.filterscale, q.ax.support, reinterpret_cast<int*>(ws + q.off_bh),
                     reinterpret_cast<double*>(ws + q.off_kh), reinterpret_cast<int*>(ws + q.off_k8h));
  hipLaunchKernelGGL(coeffs_kernel, dim3(grid_of(q.ay.out)), dim3(kThreads), 0, s, q.ay.in, q.ay.out, q.ay.ksize,
                     q.ay.scale, q.ay.filterscale, q.ay.support, reinterpret_cast<int*>(ws + q.off_bv),
                     reinterpret_cast<double*>(ws + q.off_kv), reinterpret_cast<int*>(ws + q.off_k8v));
}

bool sizes_ok(int n, int h, int w, int oh, int ow) {
  return n > 0 && h > 0 && w > 0 && oh > 0 && ow > 0 && h < (1 << 24) && w < (1 << 24) && oh < (1 << 24) &&
         ow < (1 << 24);
}

}  // namespace
}  // namespace drnmi

using namespace drnmi;

extern "C" int64_t drnmi_resize_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t oh, int32_t ow,
                                                int32_t elem_bytes) {
  if (!sizes_ok(n, h, w, oh, ow) || (elem_bytes != 3 && elem_bytes != 4)) return -1;
  return make_plan(n, h, w, oh, ow, elem_bytes).bytes;
}

extern "C" int drnmi_resize_bilinear_u8(const uint8_t* src, int32_t n, int32_t h, int32_t w, uint8_t* dst,
                                        int32_t oh, int32_t ow, void* ws, int64_t ws_bytes, void* stream) {
  if (src == nullptr || dst == nullptr || !sizes_ok(n, h, w, oh, ow)) return DRNMI_EINVAL;
  const Plan q = make_plan(n, h, w, oh, ow, 3);
  if (ws == nullptr || ws_bytes < q.bytes) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* wsb = static_cast<char*>(ws);
  launch_coeffs(q, wsb, s);
  const int* bh = reinterpret_cast<const int*>(wsb + q.off_bh);
  const int* bv = reinterpret_cast<const int*>(wsb + q.off_bv);
  uint8_t* tmp = reinterpret_cast<uint8_t*>(wsb + q.off_tmp);
  if (!q.need_h && !q.need_v)
    return static_cast<int>(hipMemcpyAsync(dst, src, static_cast<size_t>(n) * h * w * 3, hipMemcpyDeviceToDevice, s));
  if (q.need_h) {
    uint8_t* out = q.need_v ? tmp : dst;
    hipLaunchKernelGGL(resize_h_u8_kernel, dim3(grid_of(static_cast<int64_t>(n) * q.rows * ow)), dim3(kThreads), 0, s,
                       src, n, h, w, q.row0, q.rows, ow, q.ax.ksize, bh, reinterpret_cast<const int*>(wsb + q.off_k8h),
                       out);
  }
  if (q.need_v) {
    const uint8_t* vin = q.need_h ? tmp : src;
    hipLaunchKernelGGL(resize_v_u8_kernel, dim3(grid_of(static_cast<int64_t>(n) * oh * ow)), dim3(kThreads), 0, s,
                       vin, n, q.need_h ? q.rows : h, ow, oh, q.ay.ksize, q.need_h ? q.row0 : 0, bv,
                       reinterpret_cast<const int*>(wsb + q.off_k8v), dst);
  }
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_resize_bilinear_f32(const float* src, int32_t planes, int32_t h, int32_t w, float* dst,
                                         int32_t oh, int32_t ow, int32_t accumulate, void* ws, int64_t ws_bytes,
                                         void* stream) {
  if (src == nullptr || dst == nullptr || !sizes_ok(planes, h, w, oh, ow)) return DRNMI_EINVAL;
  const Plan q = make_plan(planes, h, w, oh, ow, 4);
  if (ws == nullptr || ws_bytes < q.bytes) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* wsb = static_cast<char*>(ws);
  launch_coeffs(q, wsb, s);
  const int* bh = reinterpret_cast<const int*>(wsb + q.off_bh);
  const int* bv = reinterpret_cast<const int*>(wsb + q.off_bv);
  float* tmp = reinterpret_cast<float*>(wsb + q.off_tmp);
  if (!q.need_h && !q.need_v) {
    hipLaunchKernelGGL(copy_f32_kernel, dim3(grid_of(static_cast<int64_t>(planes) * h * w)), dim3(kThreads), 0, s, src,
                       static_cast<int64_t>(planes) * h * w, dst, accumulate);
    return static_cast<int>(hipGetLastError());
  }
  if (q.need_h) {
    float* out = q.need_v ? tmp : dst;
    if (!q.need_v && accumulate) out = tmp;
    hipLaunchKernelGGL(resize_h_f32_kernel, dim3(grid_of(static_cast<int64_t>(planes) * q.rows * ow)), dim3(kThreads), 0,
                       s, src, planes, h, w, q.row0, q.rows, ow, q.ax.ksize, bh,
                       reinterpret_cast<const double*>(wsb + q.off_kh), out);
    if (!q.need_v && accumulate)
      hipLaunchKernelGGL(copy_f32_kernel, dim3(grid_of(static_cast<int64_t>(planes) * h * ow)), dim3(kThreads), 0, s, tmp,
                         static_cast<int64_t>(planes) * h * ow, dst, 1);
  }
  if (q.need_v) {
    const float* vin = q.need_h ? tmp : src;
    hipLaunchKernelGGL(resize_v_f32_kernel, dim3(grid_of(static_cast<int64_t>(planes) * oh * ow)), dim3(kThreads), 0, s,
                       vin, planes, q.need_h ? q.rows : h, ow, oh, q.ay.ksize, q.need_h ? q.row0 : 0, bv,
                       reinterpret_cast<const double*>(wsb + q.off_kv), dst, accumulate);
  }
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_argmax_nchw_f32(const float* x, int32_t n, int32_t c, int64_t hw, void* labels,
                                     int32_t label_dtype, void* stream) {
  if (x == nullptr || labels == nullptr || n <= 0 || c <= 0 || hw <= 0) return DRNMI_EINVAL;
  if (label_dtype != DRNMI_U8 && label_dtype != DRNMI_I64) return DRNMI_EINVAL;
  if (label_dtype == DRNMI_U8 && c > 256) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (label_dtype == DRNMI_U8)
    hipLaunchKernelGGL(argmax_nchw_kernel<DRNMI_U8>, dim3(grid_of(static_cast<int64_t>(n) * hw)), dim3(kThreads), 0, s,
                       x, n, c, hw, labels);
  else
    hipLaunchKernelGGL(argmax_nchw_kernel<DRNMI_I64>, dim3(grid_of(static_cast<int64_t>(n) * hw)), dim3(kThreads), 0, s,
                       x, n, c, hw, labels);
  return static_cast<int>(hipGetLastError());
}
