// int8 activation helpers for the W8A8 path (BASELINE config C5).
//
// The reference has no quantisation code: the scheme is ours.
//   * weights: per-output-channel symmetric int8, q = rint(w * 127 / absmax_row) (host packing,
//     drnmi/engine.py), the dequant scale folded into the conv epilogue's per-channel scale;
//   * activations: per-tensor symmetric int8 with a calibrated scale s (absmax / 127 over a
//     calibration batch): q = clamp(rint(x * (1/s)), -127, 127).  The conv that produces an int8
//     activation quantises in its epilogue; this file serves the bf16 -> int8 boundary (the first
//     int8 layer's input) and the calibration absmax.
// Both kernels are HBM-bound streams: 16-B loads per lane, grid-stride (no reuse to place).
#include "common.h"
#include "kernels.h"

namespace drnmi {
namespace {

__device__ __forceinline__ int8_t q8(float v, float inv) {
  float r = rintf(__fmul_rn(v, inv));
  r = fminf(fmaxf(r, -127.f), 127.f);
  return static_cast<int8_t>(static_cast<int>(r));
}

// 8 elements per lane per iteration (one 16-B bf16 load -> one 8-B int8 store)
template <typename T>
__global__ void __launch_bounds__(256) quantize_kernel(const T* __restrict__ x, int8_t* __restrict__ y, int64_t n8,
                                                       float inv) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const Vec8<T> v = Vec8<T>::load(x + i * 8);
    const T* e = reinterpret_cast<const T*>(&v);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) lo |= static_cast<uint32_t>(static_cast<uint8_t>(q8(Elem<T>::to_f32(e[j]), inv))) << (8 * j);
#pragma unroll
    for (int j = 0; j < 4; ++j) hi |= static_cast<uint32_t>(static_cast<uint8_t>(q8(Elem<T>::to_f32(e[4 + j]), inv))) << (8 * j);
    *reinterpret_cast<uint2*>(y + i * 8) = make_uint2(lo, hi);
  }
}

// max |x| over n8 * 8 elements into *out (as uint bits: |x| >= 0 orders like its bit pattern;
// NaN (bits above +inf) propagates as the maximum)
template <typename T>
__global__ void __launch_bounds__(256) absmax_kernel(const T* __restrict__ x, int64_t n8, uint32_t* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  uint32_t m = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const Vec8<T> v = Vec8<T>::load(x + i * 8);
    const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t b = __float_as_uint(Elem<T>::to_f32(e[j])) & 0x7fffffffu;
      m = b > m ? b : m;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t t = static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o));
    m = t > m ? t : m;
  }
  __shared__ uint32_t red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t r = red[0];
    for (int w = 1; w < 4; ++w) r = red[w] > r ? red[w] : r;
    atomicMax(out, r);
  }
}

unsigned stream_blocks(int64_t n8) {
  const int64_t b = (n8 + 255) / 256;
  return static_cast<unsigned>(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace
}  // namespace drnmi

using namespace drnmi;

extern "C" int drnmi_quantize_i8(const void* x, int32_t dtype, int8_t* y, int64_t n, float inv_scale, void* stream) {
  if (x == nullptr || y == nullptr || n < 0 || n % 8 != 0 || !(inv_scale > 0.f)) return DRNMI_EINVAL;
  if (n == 0) return DRNMI_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n8 = n / 8;
  if (dtype == DRNMI_BF16)
    hipLaunchKernelGGL(quantize_kernel<bf16_t>, dim3(stream_blocks(n8)), dim3(256), 0, s,
                       static_cast<const bf16_t*>(x), y, n8, inv_scale);
  else if (dtype == DRNMI_F32)
    hipLaunchKernelGGL(quantize_kernel<float>, dim3(stream_blocks(n8)), dim3(256), 0, s,
                       static_cast<const float*>(x), y, n8, inv_scale);
  else
    return DRNMI_EINVAL;
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_absmax(const void* x, int32_t dtype, int64_t n, float* out, void* stream) {
  if (x == nullptr || out == nullptr || n < 0 || n % 8 != 0) return DRNMI_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemsetAsync(out, 0, sizeof(float), s);
  if (e != hipSuccess) return static_cast<int>(e);
  if (n == 0) return DRNMI_OK;
  const int64_t n8 = n / 8;
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  if (dtype == DRNMI_BF16)
    hipLaunchKernelGGL(absmax_kernel<bf16_t>, dim3(stream_blocks(n8)), dim3(256), 0, s,
                       static_cast<const bf16_t*>(x), n8, o);
  else if (dtype == DRNMI_F32)
    hipLaunchKernelGGL(absmax_kernel<float>, dim3(stream_blocks(n8)), dim3(256), 0, s,
                       static_cast<const float*>(x), n8, o);
  else
    return DRNMI_EINVAL;
  return static_cast<int>(hipGetLastError());
}
