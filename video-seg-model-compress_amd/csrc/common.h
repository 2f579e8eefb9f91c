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

// Exact three-way split of 8 fp32 values into bf16 fragments, x = x1 + x2 + x3 (round to
// nearest even at each step; x - x1 and (x - x1) - x2 are exact in fp32 by Sterbenz): the
// fp32x arithmetic (include/drnmi.h DRNMI_F32X3).  Works on value pairs: one
// v_cvt_pk_bf16_f32 is a fragment dword, and its halves widen back to fp32 by a shift (low)
// and a mask (high), so no per-element register packing is needed.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16x2(f32x2_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ f32x2_t widen_bf16x2(uint32_t h) {
  return f32x2_t{__uint_as_float(h << 16), __uint_as_float(h & 0xffff0000u)};
}
__device__ __forceinline__ void split3(const float4& lo4, const float4& hi4, bf16x8& b1, bf16x8& b2, bf16x8& b3) {
  const f32x2_t x[4] = {f32x2_t{lo4.x, lo4.y}, f32x2_t{lo4.z, lo4.w}, f32x2_t{hi4.x, hi4.y}, f32x2_t{hi4.z, hi4.w}};
  uint32_t u1[4], u2[4], u3[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u1[i] = pk_bf16x2(x[i]);
    const f32x2_t r1 = x[i] - widen_bf16x2(u1[i]);
    u2[i] = pk_bf16x2(r1);
    u3[i] = pk_bf16x2(r1 - widen_bf16x2(u2[i]));
  }
  b1 = __builtin_bit_cast(bf16x8, make_uint4(u1[0], u1[1], u1[2], u1[3]));
  b2 = __builtin_bit_cast(bf16x8, make_uint4(u2[0], u2[1], u2[2], u2[3]));
  b3 = __builtin_bit_cast(bf16x8, make_uint4(u3[0], u3[1], u3[2], u3[3]));
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

// 16-B row pieces of the MFMA accumulator layout (lane (fr, fq) holds channels 16 fm + 4 fq .. + 3
// of pixel fr): row fq of the 16-lane groups moves chunk s(fq) = (0, 2, 1, 3)[fq] of a 32-channel
// group, and one v_permlane16_swap per dword pair converts (lo: x y, hi: z w) <-> (fragment 2 f2,
// fragment 2 f2 + 1) both ways (conv_tile.h load_residual / store_tile_x4)
__device__ __forceinline__ int chunk_of_row(int fq) { return (fq & 1) * 2 + (fq >> 1); }
__device__ __forceinline__ void swap_halves(uint4& v) {
  const auto a = __builtin_amdgcn_permlane16_swap(v.x, v.z, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(v.y, v.w, false, false);
  v = make_uint4(a[0], b[0], a[1], b[1]);
}

// int8 rows: lane (fr, fq) holds byte quad fq (channels 4 fq .. + 3) of fragments 4 g + k in r[k];
// this 4 x 4 transpose over (register, 16-lane row) leaves fragment 4 g + fq whole in row fq's four
// registers (16 contiguous bytes), and back (it is its own inverse)
__device__ __forceinline__ void transpose_rows4(uint32_t (&r)[4]) {
  const auto a = __builtin_amdgcn_permlane32_swap(r[0], r[2], false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(r[1], r[3], false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
  const auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
  r[0] = c[0];
  r[1] = c[1];
  r[2] = d[0];
  r[3] = d[1];
}

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace drnmi
