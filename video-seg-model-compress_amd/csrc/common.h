// Shared device helpers for the drnmi HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/drnmi.h"

namespace drnmi {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// bf16 stored as raw 16-bit words everywhere in global memory and LDS.
typedef uint16_t bf16_t;

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

// Round-to-nearest-even f32 -> bf16 (NaN kept NaN through the plain cast path).
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int kDtype = DRNMI_F32;
  __device__ __forceinline__ static float to_f32(float v) { return v; }
};
template <> struct Elem<bf16_t> {
  static constexpr int kDtype = DRNMI_BF16;
  __device__ __forceinline__ static float to_f32(bf16_t v) { return bf16_to_f32(v); }
};

// 8 contiguous elements: 16 B of bf16 or 32 B of fp32.
template <typename T> struct Vec8;
template <> struct Vec8<bf16_t> {
  uint4 v;
  __device__ __forceinline__ static Vec8 zero() { Vec8 r; r.v = make_uint4(0, 0, 0, 0); return r; }
  __device__ __forceinline__ static Vec8 load(const bf16_t* p) {
    Vec8 r; r.v = *reinterpret_cast<const uint4*>(p); return r;
  }
  __device__ __forceinline__ void store(bf16_t* p) const { *reinterpret_cast<uint4*>(p) = v; }
};
template <> struct Vec8<float> {
  float4 a, b;
  __device__ __forceinline__ static Vec8 zero() {
    Vec8 r; r.a = make_float4(0.f, 0.f, 0.f, 0.f); r.b = r.a; return r;
  }
  __device__ __forceinline__ static Vec8 load(const float* p) {
    Vec8 r;
    r.a = reinterpret_cast<const float4*>(p)[0];
    r.b = reinterpret_cast<const float4*>(p)[1];
    return r;
  }
  __device__ __forceinline__ void store(float* p) const {
    reinterpret_cast<float4*>(p)[0] = a;
    reinterpret_cast<float4*>(p)[1] = b;
  }
};

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace drnmi
