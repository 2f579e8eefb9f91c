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
#pragma unroll
    for (int f2 = 0; f2 < FM / 2; ++f2) rq[f2][fn] = *reinterpret_cast<const uint4*>(res + m * p.cout + c + f2 * 32);
  }
}
template <int FM, int FN>
__device__ __forceinline__ void add_residual(f32x4 (&acc)[FM][FN], uint4 (&rq)[FM / 2][FN]) {
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
      uint4 o = make_uint4(w[0], w[1], w[2], w[3]);
      swap_halves(o);
      *reinterpret_cast<uint4*>(y + m * p.cout + c + f2 * 32) = o;
    }
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
      if (nhwc16 && full) {
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
