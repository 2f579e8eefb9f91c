// Tile machinery shared by the bf16 / int8 LDS-DMA implicit-GEMM conv kernels (conv_big.hip,
// conv_stag.hip): swizzles, element traits, the XCD remap, epilogues and the strip geometry.
// Internal header (anonymous namespace: each translation unit gets its own copies).
#pragma once
#include "common.h"

namespace drnmi {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_void_t;

__device__ uint4 g_zero_page[64];   // zero-initialised: the source of padded taps / rows

constexpr int kBPX = 256;     // pixels per tile
constexpr int kMinCin = 32;   // every K step lies inside one tap

template <int ROWB>
__device__ __forceinline__ int swzb(int row, int chunk) {
  if constexpr (ROWB == 128) return chunk ^ ((row >> 1) & 7);   // 128-B rows
  // 64-B rows: the 16 rows of a fragment read span 4 banks-quads per row residue; the four
  // ds_read_b128 lane groups take chunk patterns (0,1,1,0) / (1,0,0,1) / (2,3,3,2) / (3,2,2,3)
  // over row quarters r >> 2 = 0..3, so XOR-ing 3 into rows 8..15 of each 16 makes every group
  // conflict-free (the former (row >> 2) & 3 left every group 2-way)
  else return chunk ^ (((row >> 3) & 1) * 3);
}
template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) { return swzb<BK * 2>(row, chunk); }   // bf16 rows

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Element traits of the LDS-DMA pipeline.  Both MFMAs consume 64 B of a row per lane group
// (bf16 16x16x32: 32 elements; int8 16x16x64: 64 elements), so the LDS image, swizzle and
// fragment reads are byte-identical; only the element count per K step and the MFMA differ.
// (A and B fragments come from the same row layout, so the dot product does not depend on
// the instruction's k order within the 64-B block.)
template <typename T> struct KT;
template <> struct KT<uint16_t> {
  typedef bf16x8 frag;
  typedef f32x4 acc;
  static constexpr int ESZ = 2;
  __device__ __forceinline__ static acc mma(frag a, frag b, acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct KT<int8_t> {
  typedef i32x4 frag;
  typedef i32x4 acc;
  static constexpr int ESZ = 1;
  __device__ __forceinline__ static acc mma(frag a, frag b, acc c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  }
};

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// index of the n-th set bit of m (n < popcount(m)): binary search on popcounts
__device__ __forceinline__ int nth_set_bit(uint64_t m, int n) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t low = m & ((uint64_t(1) << w) - 1);
    const int c = __popcll(low);
    if (n >= c) {
      n -= c;
      m >>= w;
      pos += w;
    } else {
      m = low;
    }
  }
  return pos;
}

__device__ __forceinline__ int xcd_remap2(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

// Epilogue shared by the conv kernels: lane owns channels co..co+3 of pixel m for FM x 4
// accumulator fragments (folded BN scale/shift, optional residual, ReLU); bf16 NHWC rows get
// one 8-byte store per fragment, other layouts (fp32 / strided seg logits) element stores.
// Accumulator start value.  With a NULL scale (BN scale pre-folded into the weights) the
// tile starts from shift + residual: the residual loads go out with the prologue DMA and
// hide under it, and the epilogue is a plain ReLU + convert + store.
// DEFER: start from zero and add shift + residual in store_tile (keeps the accumulators free of
// VALU work so the compiler can hold them in AGPRs — the 128 x 128-per-wave tiles need that).
template <int FM, int WCO, int FN = 4, bool DEFER = false>
__device__ __forceinline__ void init_tile(const drnmi_conv_args& p, f32x4 (&acc)[FM][FN], int px0, int co0,
                                          int wc, int wp, int fr, int fq) {
  constexpr int PXW = 16 * FN;   // pixels per wave
  if (DEFER || p.scale != nullptr) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const int M = p.n * p.ho * p.wo;
  const uint16_t* __restrict__ res = reinterpret_cast<const uint16_t*>(p.res);
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int co = co0 + wc * WCO + fm * 16 + fq * 4;
    const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);   // padded to cout_pad
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = f32x4{sh.x, sh.y, sh.z, sh.w};
  }
  if (res == nullptr) return;
  // residual loads in groups of 4 pixel fragments (bounds the live registers to FM x 4 uint2)
#pragma unroll
  for (int g = 0; g < FN; g += 4) {
    uint2 rv[FM][4];
#pragma unroll
    for (int f4 = 0; f4 < 4; ++f4) {
      const int m = px0 + wp * PXW + (g + f4) * 16 + fr;
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int co = co0 + wc * WCO + fm * 16 + fq * 4;
        rv[fm][f4] = make_uint2(0, 0);
        if (m < M && co + 3 < p.cout) rv[fm][f4] = *reinterpret_cast<const uint2*>(res + static_cast<int64_t>(m) * p.cout + co);
        else if (m < M) {
          uint16_t t[4] = {0, 0, 0, 0};
          for (int j = 0; j < 4; ++j)
            if (co + j < p.cout) t[j] = res[static_cast<int64_t>(m) * p.cout + co + j];
          rv[fm][f4] = make_uint2(t[0] | (static_cast<uint32_t>(t[1]) << 16), t[2] | (static_cast<uint32_t>(t[3]) << 16));
        }
      }
    }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int f4 = 0; f4 < 4; ++f4) {
        acc[fm][g + f4][0] += bf16_to_f32(static_cast<uint16_t>(rv[fm][f4].x & 0xffff));
        acc[fm][g + f4][1] += bf16_to_f32(static_cast<uint16_t>(rv[fm][f4].x >> 16));
        acc[fm][g + f4][2] += bf16_to_f32(static_cast<uint16_t>(rv[fm][f4].y & 0xffff));
        acc[fm][g + f4][3] += bf16_to_f32(static_cast<uint16_t>(rv[fm][f4].y >> 16));
      }
  }
}

// Residual and output rows as 16-B pieces.  The accumulator layout gives lane (fr, fq) channels
// 16 fm + 4 fq .. + 3 of pixel fr: as 8-B accesses every instruction touches 16 pixels x 32 B, and
// each 128-B line is requested by four instructions.  Here row fq of the 16-lane groups moves the
// 16-B chunk s(fq) = (0, 2, 1, 3)[fq] of a 32-channel group (channels 8 s .. 8 s + 7) and one
// v_permlane16_swap per dword pair converts between the two layouts: swapping the odd rows of the
// low halves with the even rows of the high halves leaves quad fq of the group (fragment 2 f2) in
// the low halves and quad 4 + fq (fragment 2 f2 + 1) in the high halves, and back.  Half the
// instructions, 64 contiguous bytes per pixel; the values are the same, so the sums are.
// (chunk_of_row, swap_halves: common.h)
template <int FM, int WCO, int FN>
__device__ __forceinline__ void load_residual(const drnmi_conv_args& p, uint4 (&rq)[FM / 2][FN], int px0, int co0, int wc,
                                              int wp, int fr, int fq) {
  const uint16_t* __restrict__ res = reinterpret_cast<const uint16_t*>(p.res);
  const int c = co0 + wc * WCO + chunk_of_row(fq) * 8;
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int64_t m = px0 + wp * 16 * FN + fn * 16 + fr;
    // whole 128-B lines, the mirror of store_tile_x4: rq[2 L] / rq[2 L + 1] hold the pieces of
    // pixels 0-7 / 8-15 of groups (2 L, 2 L + 1); add_residual trades them back (lanes fr ^ 8)
    static_assert((FM / 2) % 2 == 0, "line pairs");
    const bool lo = fr < 8;
    const int64_t m0 = m - (lo ? 0 : 8), m1 = m0 + 8;
#pragma unroll
    for (int L = 0; L < FM / 4; ++L) {
      const int ca = c + 2 * L * 32;
      rq[2 * L][fn] = *reinterpret_cast<const uint4*>(res + m0 * p.cout + ca + (lo ? 0 : 32));
      rq[2 * L + 1][fn] = *reinterpret_cast<const uint4*>(res + m1 * p.cout + ca + (lo ? 32 : 0));
    }
  }
}
template <int FM, int FN>
__device__ __forceinline__ void add_residual(f32x4 (&acc)[FM][FN], uint4 (&rq)[FM / 2][FN], int fr) {
  const bool lo = fr < 8;
#pragma unroll
  for (int L = 0; L < FM / 4; ++L)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const uint4 d0 = rq[2 * L][fn], d1 = rq[2 * L + 1][fn];
      const uint4 own = make_uint4(lo ? d0.x : d1.x, lo ? d0.y : d1.y, lo ? d0.z : d1.z, lo ? d0.w : d1.w);
      const uint4 give = make_uint4(lo ? d1.x : d0.x, lo ? d1.y : d0.y, lo ? d1.z : d0.z, lo ? d1.w : d0.w);
      uint4 r;
      r.x = __builtin_amdgcn_update_dpp(0u, give.x, 0x128, 0xf, 0xf, false);
      r.y = __builtin_amdgcn_update_dpp(0u, give.y, 0x128, 0xf, 0xf, false);
      r.z = __builtin_amdgcn_update_dpp(0u, give.z, 0x128, 0xf, 0xf, false);
      r.w = __builtin_amdgcn_update_dpp(0u, give.w, 0x128, 0xf, 0xf, false);
      rq[2 * L][fn] = own;
      rq[2 * L + 1][fn] = r;
    }
#pragma unroll
  for (int f2 = 0; f2 < FM / 2; ++f2)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      swap_halves(rq[f2][fn]);
      const uint32_t w[4] = {rq[f2][fn].x, rq[f2][fn].y, rq[f2][fn].z, rq[f2][fn].w};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4& a = acc[2 * f2 + h][fn];
        a[0] += bf16_to_f32(static_cast<uint16_t>(w[2 * h] & 0xffff));
        a[1] += bf16_to_f32(static_cast<uint16_t>(w[2 * h] >> 16));
        a[2] += bf16_to_f32(static_cast<uint16_t>(w[2 * h + 1] & 0xffff));
        a[3] += bf16_to_f32(static_cast<uint16_t>(w[2 * h + 1] >> 16));
      }
    }
}
// dense bf16 NHWC output (y_sc 1, y_sp cout), shift and residual already in the accumulators:
// ReLU, round, 16-B stores (the rounding and ReLU of store_tile, element for element)
template <int FM, int WCO, int FN>
__device__ __forceinline__ void store_tile_x4(const drnmi_conv_args& p, const f32x4 (&acc)[FM][FN], int px0, int co0,
                                              int wc, int wp, int fr, int fq) {
  uint16_t* __restrict__ y = reinterpret_cast<uint16_t*>(p.y);
  const int c = co0 + wc * WCO + chunk_of_row(fq) * 8;
  const bool relu = p.relu != 0;
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int64_t m = px0 + wp * 16 * FN + fn * 16 + fr;
    uint4 o[FM / 2];
#pragma unroll
    for (int f2 = 0; f2 < FM / 2; ++f2) {
      uint32_t w[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float v[4] = {acc[2 * f2 + h][fn][0], acc[2 * f2 + h][fn][1], acc[2 * f2 + h][fn][2], acc[2 * f2 + h][fn][3]};
        if (relu) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
        }
        w[2 * h] = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
        w[2 * h + 1] = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      }
      o[f2] = make_uint4(w[0], w[1], w[2], w[3]);
      swap_halves(o[f2]);
    }
    // whole 128-B lines: lanes fr and fr ^ 8 (DPP row_ror:8) trade their odd-group chunks, so one
    // instruction writes groups (2 L, 2 L + 1) of pixels 0-7 and the next those of pixels 8-15
    const bool lo = fr < 8;
    const int64_t m0 = m - (lo ? 0 : 8), m1 = m0 + 8;
#pragma unroll
    for (int L = 0; L < FM / 4; ++L) {
      const uint4 a = o[2 * L], b = o[2 * L + 1];
      uint4 r;
      r.x = __builtin_amdgcn_update_dpp(0u, b.x, 0x128, 0xf, 0xf, false);
      r.y = __builtin_amdgcn_update_dpp(0u, b.y, 0x128, 0xf, 0xf, false);
      r.z = __builtin_amdgcn_update_dpp(0u, b.z, 0x128, 0xf, 0xf, false);
      r.w = __builtin_amdgcn_update_dpp(0u, b.w, 0x128, 0xf, 0xf, false);
      const int ca = c + 2 * L * 32, cb = ca + 32;
      const uint4 d0 = make_uint4(lo ? a.x : r.x, lo ? a.y : r.y, lo ? a.z : r.z, lo ? a.w : r.w);
      const uint4 d1 = make_uint4(lo ? r.x : a.x, lo ? r.y : a.y, lo ? r.z : a.z, lo ? r.w : a.w);
      uint16_t* y0 = y + m0 * p.cout + ca + (lo ? 0 : 32);
      uint16_t* y1 = y + m1 * p.cout + ca + (lo ? 32 : 0);
      *reinterpret_cast<uint4*>(y0) = d0;
      *reinterpret_cast<uint4*>(y1) = d1;
    }
    if constexpr ((FM / 2) % 2 == 1) *reinterpret_cast<uint4*>(y + m * p.cout + c + (FM / 2 - 1) * 32) = o[FM / 2 - 1];
  }
}
template <int FM, int WCO, int FN = 4, bool DEFER = false>
__device__ __forceinline__ void store_tile(const drnmi_conv_args& p, const f32x4 (&acc)[FM][FN], int cur_px0,
                                           int cur_co0, int wc, int wp, int fr, int fq) {
  constexpr int PXW = 16 * FN;
  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const uint16_t* __restrict__ res = reinterpret_cast<const uint16_t*>(p.res);
  const bool nhwc16 = p.out_dtype == DRNMI_BF16 && p.y_sc == 1;
  // fp32 NHWC rows, 16-B aligned: one 16-B store per whole 4-channel group inside cout.  A partial
  // group is stored whole only into the pixel's own padding, i.e. when the row is exactly
  // round_up(cout, 4) wide (the labels-only seg logits, SEG_NHWC_CS): those channels get the padded
  // weight rows' values, which no reader uses.  A conv writing a channel slice of a wider buffer
  // (y_sp > round_up(cout, 4)) never touches the channels past cout.
  const bool nhwc32 = p.out_dtype == DRNMI_F32 && p.y_sc == 1 && p.y_sp % 4 == 0 && p.y_sn % 4 == 0 &&
                      (reinterpret_cast<uintptr_t>(p.y) & 15) == 0;
  const bool pad_row = p.y_sp == ((p.cout + 3) & ~3);
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int m = cur_px0 + wp * PXW + fn * 16 + fr;
    if (m >= M) continue;
    const int n = m / hw_o;
    const int q = m - n * hw_o;
    const int64_t ybase = static_cast<int64_t>(n) * p.y_sn + static_cast<int64_t>(q) * p.y_sp;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int co = cur_co0 + wc * WCO + fm * 16 + fq * 4;
      if (co >= p.cout) continue;
      const bool full = co + 3 < p.cout;
      float v[4] = {acc[fm][fn][0], acc[fm][fn][1], acc[fm][fn][2], acc[fm][fn][3]};
      if (p.scale != nullptr) {   // else shift and residual are already in the accumulator
        const float4 sc = *reinterpret_cast<const float4*>(p.scale + co);   // padded to cout_pad
        const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
        v[0] = v[0] * sc.x + sh.x;
        v[1] = v[1] * sc.y + sh.y;
        v[2] = v[2] * sc.z + sh.z;
        v[3] = v[3] * sc.w + sh.w;
      } else if (DEFER) {
        const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
        v[0] += sh.x;
        v[1] += sh.y;
        v[2] += sh.z;
        v[3] += sh.w;
      }
      if ((DEFER || p.scale != nullptr) && res != nullptr) {
        if (full) {
          const uint2 rv = *reinterpret_cast<const uint2*>(res + static_cast<int64_t>(m) * p.cout + co);
          v[0] += bf16_to_f32(static_cast<uint16_t>(rv.x & 0xffff));
          v[1] += bf16_to_f32(static_cast<uint16_t>(rv.x >> 16));
          v[2] += bf16_to_f32(static_cast<uint16_t>(rv.y & 0xffff));
          v[3] += bf16_to_f32(static_cast<uint16_t>(rv.y >> 16));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (co + j < p.cout) v[j] += bf16_to_f32(res[static_cast<int64_t>(m) * p.cout + co + j]);
        }
      }
      if (p.relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      if (nhwc32 && (full || pad_row)) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.y) + ybase + co) = make_float4(v[0], v[1], v[2], v[3]);
      } else if (nhwc16 && full) {
        uint2 o;
        o.x = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
        o.y = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.y) + ybase + co) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (co + j >= p.cout) break;
          const int64_t off = ybase + static_cast<int64_t>(co + j) * p.y_sc;
          if (p.out_dtype == DRNMI_BF16) reinterpret_cast<uint16_t*>(p.y)[off] = f32_to_bf16(v[j]);
          else reinterpret_cast<float*>(p.y)[off] = v[j];
        }
      }
    }
  }
}

template <int FM, int FN>
__device__ __forceinline__ void zero_tile(i32x4 (&acc)[FM][FN]) {
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = i32x4{0, 0, 0, 0};
}

// W8A8 epilogue (include/drnmi.h drnmi_conv_args, int8 fields): one fp32 rounding per step,
// no contraction (fp contract off), so oracle/int8_oracle.py reproduces it bit for bit.
template <int FM, int WCO, int FN>
__device__ __forceinline__ void store_tile_i8(const drnmi_conv_args& p, const i32x4 (&acc)[FM][FN], int cur_px0,
                                              int cur_co0, int wc, int wp, int fr, int fq) {
#pragma clang fp contract(off)   // hipcc contracts a*b+c into v_fma by default (also inside inlined
                                 // __fmul_rn / __fadd_rn): the epilogue is fmul then fadd
  constexpr int PXW = 16 * FN;
  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const int8_t* __restrict__ res = reinterpret_cast<const int8_t*>(p.res);
  const bool packed4 = p.out_dtype == DRNMI_I8 && p.y_sc == 1;
  const bool res4 = (p.cout & 3) == 0;
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int m = cur_px0 + wp * PXW + fn * 16 + fr;
    if (m >= M) continue;
    const int n = m / hw_o;
    const int q = m - n * hw_o;
    const int64_t ybase = static_cast<int64_t>(n) * p.y_sn + static_cast<int64_t>(q) * p.y_sp;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int co = cur_co0 + wc * WCO + fm * 16 + fq * 4;
      if (co >= p.cout) continue;
      const bool full = co + 3 < p.cout;
      const float4 sc = *reinterpret_cast<const float4*>(p.scale + co);   // padded to cout_pad
      const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
      float v[4];
      v[0] = static_cast<float>(acc[fm][fn][0]) * sc.x + sh.x;
      v[1] = static_cast<float>(acc[fm][fn][1]) * sc.y + sh.y;
      v[2] = static_cast<float>(acc[fm][fn][2]) * sc.z + sh.z;
      v[3] = static_cast<float>(acc[fm][fn][3]) * sc.w + sh.w;
      if (res != nullptr) {
        int8_t r[4] = {0, 0, 0, 0};
        const int8_t* rp = res + static_cast<int64_t>(m) * p.cout + co;
        if (full && res4) {
          const uint32_t rw = *reinterpret_cast<const uint32_t*>(rp);
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] = static_cast<int8_t>((rw >> (8 * j)) & 0xff);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (co + j < p.cout) r[j] = rp[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = v[j] + static_cast<float>(r[j]) * p.res_scale;
      }
      if (p.relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      if (p.out_dtype == DRNMI_I8) {
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float t = fminf(fmaxf(rintf(v[j] * p.out_scale), -127.f), 127.f);
          o |= static_cast<uint32_t>(static_cast<uint8_t>(static_cast<int8_t>(static_cast<int>(t)))) << (8 * j);
        }
        int8_t* y = reinterpret_cast<int8_t*>(p.y);
        if (packed4 && full) {
          *reinterpret_cast<uint32_t*>(y + ybase + co) = o;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (co + j >= p.cout) break;
            y[ybase + static_cast<int64_t>(co + j) * p.y_sc] = static_cast<int8_t>((o >> (8 * j)) & 0xff);
          }
        }
      } else if (p.out_dtype == DRNMI_F32 && p.y_sc == 1 && (p.y_sp & 3) == 0 && (p.y_sn & 3) == 0 &&
                 (reinterpret_cast<uintptr_t>(p.y) & 15) == 0 && (full || p.y_sp == ((p.cout + 3) & ~3))) {
        // fp32 NHWC rows: one 16-B store per 4-channel group; a partial group only into the pixel's
        // own padding (rows exactly round_up(cout, 4) wide: the labels head's logits, SEG_NHWC_CS,
        // whose pad channels hold scale/shift padding values nobody reads), never into a wider
        // buffer's neighbouring channels
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.y) + ybase + co) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (co + j >= p.cout) break;
          const int64_t off = ybase + static_cast<int64_t>(co + j) * p.y_sc;
          if (p.out_dtype == DRNMI_BF16) reinterpret_cast<uint16_t*>(p.y)[off] = f32_to_bf16(v[j]);
          else reinterpret_cast<float*>(p.y)[off] = v[j];
        }
      }
    }
  }
}

// store_tile_i8 for whole tiles of a dense int8 NHWC output (y_sc 1, y_sp cout): the same
// per-element arithmetic, residual loads and output stores as 16-B pieces (common.h
// transpose_rows4: row fq moves fragment 4 g + fq whole) instead of 4-B ones
template <int FM, int WCO, int FN>
__device__ __forceinline__ void store_tile_i8_x4(const drnmi_conv_args& p, const i32x4 (&acc)[FM][FN], int px0,
                                                 int co0, int wc, int wp, int fr, int fq) {
#pragma clang fp contract(off)
  static_assert(FM % 4 == 0, "16-B int8 pieces");
  constexpr int NG = FM / 4;                         // 64-B groups of the wave's channels per pixel
  const int8_t* __restrict__ res = reinterpret_cast<const int8_t*>(p.res);
  int8_t* __restrict__ y = reinterpret_cast<int8_t*>(p.y);
  const int cbase = co0 + wc * WCO + fq * 16;
  const bool lo = fr < 8;
  // 128-B lines when the wave's channels span whole lines (NG even): groups (2 L, 2 L + 1) of
  // pixels 0-7, then of pixels 8-15, lanes fr and fr ^ 8 trading the odd group (DPP row_ror:8)
  constexpr bool LINES = NG % 2 == 0;
  auto trade = [](uint4 v) {
    uint4 r;
    r.x = __builtin_amdgcn_update_dpp(0u, v.x, 0x128, 0xf, 0xf, false);
    r.y = __builtin_amdgcn_update_dpp(0u, v.y, 0x128, 0xf, 0xf, false);
    r.z = __builtin_amdgcn_update_dpp(0u, v.z, 0x128, 0xf, 0xf, false);
    r.w = __builtin_amdgcn_update_dpp(0u, v.w, 0x128, 0xf, 0xf, false);
    return r;
  };
  auto sel = [](bool c, uint4 a, uint4 b) {
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
  };
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int64_t m = px0 + wp * 16 * FN + fn * 16 + fr;
    const int64_t m0 = m - (lo ? 0 : 8), m1 = m0 + 8;
    uint4 rq[NG];
    if (res != nullptr) {
      if constexpr (LINES) {
#pragma unroll
        for (int L = 0; L < NG / 2; ++L) {
          const uint4 d0 = *reinterpret_cast<const uint4*>(res + m0 * p.cout + cbase + (2 * L + (lo ? 0 : 1)) * 64);
          const uint4 d1 = *reinterpret_cast<const uint4*>(res + m1 * p.cout + cbase + (2 * L + (lo ? 1 : 0)) * 64);
          rq[2 * L] = sel(lo, d0, d1);
          rq[2 * L + 1] = trade(sel(lo, d1, d0));
        }
      } else {
#pragma unroll
        for (int g = 0; g < NG; ++g) rq[g] = *reinterpret_cast<const uint4*>(res + m * p.cout + cbase + g * 64);
      }
    }
    uint4 out[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      uint32_t rr[4] = {0, 0, 0, 0};
      if (res != nullptr) {
        rr[0] = rq[g].x;
        rr[1] = rq[g].y;
        rr[2] = rq[g].z;
        rr[3] = rq[g].w;
        transpose_rows4(rr);
      }
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int fm = 4 * g + k;
        const int co = co0 + wc * WCO + fm * 16 + fq * 4;
        const float4 sc = *reinterpret_cast<const float4*>(p.scale + co);
        const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
        float v[4];
        v[0] = static_cast<float>(acc[fm][fn][0]) * sc.x + sh.x;
        v[1] = static_cast<float>(acc[fm][fn][1]) * sc.y + sh.y;
        v[2] = static_cast<float>(acc[fm][fn][2]) * sc.z + sh.z;
        v[3] = static_cast<float>(acc[fm][fn][3]) * sc.w + sh.w;
        if (res != nullptr) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[j] = v[j] + static_cast<float>(static_cast<int8_t>((rr[k] >> (8 * j)) & 0xff)) * p.res_scale;
        }
        if (p.relu) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
        }
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float t = fminf(fmaxf(rintf(v[j] * p.out_scale), -127.f), 127.f);
          w |= static_cast<uint32_t>(static_cast<uint8_t>(static_cast<int8_t>(static_cast<int>(t)))) << (8 * j);
        }
        o[k] = w;
      }
      transpose_rows4(o);
      out[g] = make_uint4(o[0], o[1], o[2], o[3]);
    }
    if constexpr (LINES) {
#pragma unroll
      for (int L = 0; L < NG / 2; ++L) {
        const uint4 r = trade(out[2 * L + 1]);
        *reinterpret_cast<uint4*>(y + m0 * p.cout + cbase + (2 * L + (lo ? 0 : 1)) * 64) = sel(lo, out[2 * L], r);
        *reinterpret_cast<uint4*>(y + m1 * p.cout + cbase + (2 * L + (lo ? 1 : 0)) * 64) = sel(lo, r, out[2 * L]);
      }
    } else {
#pragma unroll
      for (int g = 0; g < NG; ++g) *reinterpret_cast<uint4*>(y + m * p.cout + cbase + g * 64) = out[g];
    }
  }
}

template <int WCO, int WC, int NST, int BK, int NWP = 4, int ESZ = 2>
struct BigCfg {
  static constexpr int BCO = WCO * WC;              // output channels per tile
  static constexpr int FM = WCO / 16;               // channel fragments per wave
  static constexpr int NW = NWP * WC;               // waves (WC channel columns x NWP pixel rows)
  static constexpr int PXW = kBPX / NWP;            // pixels per wave
  static constexpr int FN = PXW / 16;               // pixel fragments per wave
  static constexpr int THREADS = 64 * NW;
  static constexpr int ROWB = BK * ESZ;             // bytes per LDS row
  static constexpr int CPR = ROWB / 16;             // 16-B chunks per row
  static constexpr int RPI = 1024 / ROWB;           // rows per 1-KB DMA wave instruction
  static constexpr int SUB = ROWB / 64;             // 64-B MFMA substeps per step
  static constexpr int A_BYTES = BCO * ROWB;
  static constexpr int B_BYTES = kBPX * ROWB;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_INSTR = BCO / RPI / NW;    // DMA instructions per wave per step
  static constexpr int B_INSTR = kBPX / RPI / NW;
  static constexpr int GLDS = A_INSTR + B_INSTR;
  static constexpr int LDS = NST * STAGE;
  static constexpr int GR = FM / 2 > 0 ? FM / 2 : 1;      // MFMA groups per substep
  static constexpr int FPG = FM / GR;                     // channel fragments per group
  static_assert(A_INSTR >= 1 && B_INSTR >= 1, "DMA split");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// STRIP (3x3 stride-1 convs whose tiles are whole 256-pixel runs of one output row, wo % 256
// == 0: DRN-D layer5..8 at 1024x2048): the B operand of the three taps (kh, kw = 0..2) of one
// 64-channel block is the same input row shifted by kw*dil pixels, so it is DMA'd once per
// (channel block, kh) as a strip of 256 + 2 dil pixel rows into one of two strip buffers and the
// three K steps read it at row offset kw*dil.  B DMA drops from 3 x 256 to 256 + 2 dil rows per
// three steps (~8 to ~5.4 DMA pieces per wave per step, 64 to ~43 KB of LDS writes).  The next
// (cb, kh) strip is issued in shares during the current group's three steps.  The K order, the
// MFMAs and the epilogue are unchanged: the output is bit-identical to the non-strip kernel.
constexpr int kStripPieces = 33;                     // ceil((256 + 2 * 4) / 8) 1-KB pieces, dil <= 4
constexpr int kStripBytes = kStripPieces * 1024;

}  // namespace
}  // namespace drnmi
