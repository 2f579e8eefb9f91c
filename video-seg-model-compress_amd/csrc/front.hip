// Fused video front (bf16 perf mode): uint8 HWC3 frames -> layer0 7x7 3->16 -> layer1 3x3 16->16
// -> layer2 3x3 stride 2 16->32, each + BN + ReLU, in ONE launch (include/drnmi.h
// drnmi_video_front_u8).  Reference: lmodels/drn.py:132-137 (layer0), :201-211 (layer1, layer2),
// on the frame normalised by data_transforms.py:109-125, :256-281.
//
// Design (gfx950).  The two full-resolution 16-channel activations (64 MB per 1024x2048 frame each
// in bf16) never leave the CU: one wave owns a strip of 30 layer2 columns (64 stem / layer1
// columns) and walks DOWN the frame, so no row is computed twice; everything between the frame
// bytes and the layer2 output stays in registers and a small per-wave LDS area.
//
//  * Pixel-pair MFMAs.  Every conv runs v_mfma_f32_32x32x16 with the 32 B-columns = 32 pixel PAIRS
//    (cols S0 + 2r, S0 + 2r + 1) and the 32 A-rows = (sub-pixel sp, 16 channels): lane (r, h) of an
//    accumulator then holds all 16 channels of pixel S0 + 2r + h, reg j = channel j.  A pair's 7x7
//    window over a frame row is 8 pixels = 24 consecutive bytes = 3 K-chunks of 8, so the stem is
//    11 MFMAs per pair row (K 176 for 2 x 147 useful MACs per channel: 84 %) instead of 14 on
//    single pixels with 4-channel padding.
//  * Exact frame bytes.  1024 + u8 is exact in f16 (bits 0x6400 | u8), so one v_perm_b32 turns
//    two frame bytes into two f16 values; the normalisation (u8 / 255 - mean) / std and the stem's
//    BN scale are folded into the f16 weights, and the offset 1024 plus the mean term come back
//    through the accumulator's starting value, per border case (the reference zero-pads in
//    normalised space: out-of-image taps contribute nothing, so the subtracted constant depends on
//    which taps are inside; 7 x 7 row/column cases, computed on the host in double).
//  * Frame rows are converted once into an LDS ring (8 rows, two copies 4 B apart so every
//    pair window is an 8-B aligned ds_read_b64 pair) and re-read by the 7 stem rows that use them.
//  * A pair row's 16-channel outputs go through a per-wave LDS exchange only to reach the
//    neighbouring pair (the 3x3 convs' left / right taps); the own-pair taps are read the same way.
//    Layer1 is 12 MFMAs per pair row (own pixels, and the left/right neighbours in one B operand:
//    lane half 0 takes pixel 2r-1, half 1 pixel 2r+2); layer2 (stride 2, 32 output channels on the
//    rows, output pixel x = pair r) is 9 MFMAs per output row, all A rows useful.
//  * Skewed, branch-free steps: step j computes stem rows 2j+3, 2j+4, layer1 rows 2j, 2j+1 and
//    layer2 row j-1, each only from rows that EARLIER steps left in LDS, so the step's three MFMA
//    chains are independent and the stem / layer1 epilogues (bf16 pack, ReLU, border masks, LDS
//    writes) run under the later chains' MFMAs.  Border rows / columns are data (zero frame rows,
//    per-lane masks, a per-lane row-case shift read from LDS), not branches, and frame rows are
//    prefetched a step ahead into registers, so the loop waits only for those loads (vmcnt(4):
//    the layer2 stores stay in flight).
//  * Persistent waves: one 64-thread workgroup per SIMD (512 VGPRs: all 32 weight fragments live in
//    registers), each walking a contiguous range of (frame, strip, layer2 row) work; a range start
//    re-primes the walk with three extra steps.
#include <math.h>
#include <string.h>

#include "common.h"
#include "kernels.h"

namespace drnmi {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// ---- packed parameters (drnmi_front_pack): A fragments [frag][lane][8 x 16 bit], then shifts
constexpr int kFS = 11, kF1 = 12, kF2 = 9;             // MFMA A fragments: stem, layer1, layer2
constexpr int kFragB = 64 * 16;
constexpr int kOffL1 = kFS * kFragB;
constexpr int kOffL2 = kOffL1 + kF1 * kFragB;
constexpr int kOffC0 = kOffL2 + kF2 * kFragB;          // float [7 row cases][7 col cases][16]
constexpr int kOffC1 = kOffC0 + 49 * 16 * 4;           // float [16] layer1 shift
constexpr int kOffC2 = kOffC1 + 16 * 4;                // float [32] layer2 shift
constexpr int kPackB = kOffC2 + 32 * 4;

// ---- geometry
constexpr int kCols = 30;                // layer2 columns per strip (pairs 1..30 of 32)
constexpr int kRing = 8;                 // converted frame rows in the LDS ring
constexpr int kRowB = 1040;              // ring row: image byte o at o (copy A) and at kCopyB + o
constexpr int kCopyB = 516;              //   (copy B: 8-B aligned where o % 8 == 4)
constexpr int kXSp = 34 * 16;            // exchange: [plane 2][sp 2][pair slot 34][16 B], pair r at r + 1
constexpr int kXSlot = 4 * kXSp;
constexpr int kXSlots = 6;               // exchange rows per activation (row mod 6)
constexpr int kLdsZero = kRing * kRowB + 2 * kXSlots * kXSlot;
constexpr int kLds = kLdsZero + 49 * 16 * 4;            // + the stem shift table
constexpr uint32_t kF16Hi = 0x64646464u;
#ifndef DRNMI_FR_PIN
#define DRNMI_FR_PIN 0          // 1: keep the step's LDS operand reads ahead of its MFMAs (measured slower: 360 vs 342 us)
#endif
#ifndef DRNMI_FR_AGPRW
#define DRNMI_FR_AGPRW 1        // weight fragments pinned to AGPRs
#endif
#ifndef DRNMI_FR_ABL
#define DRNMI_FR_ABL 0          // diagnostic builds only: bit 0/1/2 skip the stem/layer1/layer2 MFMAs
#endif                          // (operands still read), bit 3 the output stores               // v_perm source of the f16 exponent byte 0x64

struct FrontParams {
  const uint8_t* x;
  const char* pack;
  bf16_t* y;
  int n, h, w, h2, w2, ns;     // ns: strips per frame
  int total;                   // n * ns * h2 layer2 rows of work
  int per_wave;
};

__device__ __forceinline__ uint32_t relu_pk(float a, float b) {
  const uint32_t u = pk_bf16x2(f32x2_t{a, b});
  const s16x2 v = __builtin_elementwise_max(__builtin_bit_cast(s16x2, u), s16x2{0, 0});   // bf16 sign bit
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ f16x8 ld_frag_f16(const char* row, int off) {
  const uint2 lo = *reinterpret_cast<const uint2*>(row + off);
  const uint2 hi = *reinterpret_cast<const uint2*>(row + off + 8);
  return __builtin_bit_cast(f16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}
__device__ __forceinline__ bf16x8 ld_frag_bf16(const char* p) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
}
template <int ABL = 0>
__device__ __forceinline__ f32x16 mfma_f16(const uint4& a, const f16x8& b, const f32x16& c) {
  if constexpr ((DRNMI_FR_ABL & ABL) != 0) {
    asm volatile("" :: "v"(__builtin_bit_cast(u32x4_t, a)), "v"(__builtin_bit_cast(u32x4_t, b)));
    return c;
  } else {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), b, c, 0, 0, 0);
  }
}
template <int ABL = 0>
__device__ __forceinline__ f32x16 mfma_bf16(const uint4& a, const bf16x8& b, const f32x16& c) {
  if constexpr ((DRNMI_FR_ABL & ABL) != 0) {
    asm volatile("" :: "v"(__builtin_bit_cast(u32x4_t, a)), "v"(__builtin_bit_cast(u32x4_t, b)));
    return c;
  } else {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), b, c, 0, 0, 0);
  }
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
front_kernel(const FrontParams a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const ring = smem;
  char* const xs0 = smem + kRing * kRowB;                 // stem rows (slot = row mod 6)
  char* const xs1 = xs0 + kXSlots * kXSlot;               // layer1 rows (slot = row mod 6)
  float* const ctab = reinterpret_cast<float*>(xs1 + kXSlots * kXSlot);   // [7][7][16] stem shifts
  const int lane = threadIdx.x;
  const int r = lane & 31, hh = lane >> 5;

  const uint4* pk = reinterpret_cast<const uint4*>(a.pack);
  uint4 as[kFS], a1[kF1], a2[kF2];
#pragma unroll
  for (int m = 0; m < kFS; ++m) as[m] = pk[m * 64 + lane];
#pragma unroll
  for (int m = 0; m < kF1; ++m) a1[m] = pk[(kFS + m) * 64 + lane];
#pragma unroll
  for (int m = 0; m < kF2; ++m) a2[m] = pk[(kFS + kF1 + m) * 64 + lane];
  if constexpr (DRNMI_FR_AGPRW) {
    // keep the 32 weight fragments in AGPRs (MFMA A operands may be AGPRs): the VGPRs are left to
    // the operand fragments and the accumulators, whose epilogue VALU would otherwise copy them out
#pragma unroll
    for (int m = 0; m < kFS; ++m) { u32x4_t t = __builtin_bit_cast(u32x4_t, as[m]); asm volatile("" : "+a"(t)); as[m] = __builtin_bit_cast(uint4, t); }
#pragma unroll
    for (int m = 0; m < kF1; ++m) { u32x4_t t = __builtin_bit_cast(u32x4_t, a1[m]); asm volatile("" : "+a"(t)); a1[m] = __builtin_bit_cast(uint4, t); }
#pragma unroll
    for (int m = 0; m < kF2; ++m) { u32x4_t t = __builtin_bit_cast(u32x4_t, a2[m]); asm volatile("" : "+a"(t)); a2[m] = __builtin_bit_cast(uint4, t); }
  }
  const float* c1t = reinterpret_cast<const float*>(a.pack + kOffC1);
  const float* c2t = reinterpret_cast<const float*>(a.pack + kOffC2);
  f32x16 c1, c2;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    c1[j] = c1t[j];
    c2[j] = c2t[(j & 3) + 8 * (j >> 2) + 4 * hh];      // 32x32 D row (j&3) + 8(j>>2) + 4h = channel
  }
  for (int i = lane * 16; i < kLdsZero; i += 64 * 16) *reinterpret_cast<uint4*>(smem + i) = make_uint4(0, 0, 0, 0);
  for (int i = lane * 4; i < 49 * 16 * 4; i += 64 * 4)
    *reinterpret_cast<float*>(reinterpret_cast<char*>(ctab) + i) =
        *reinterpret_cast<const float*>(a.pack + kOffC0 + i);

  const int H = a.h, W = a.w;
  const int rowb = 3 * W;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.x), 0, a.n * H * rowb, 0x00020000);
  const __amdgpu_buffer_rsrc_t ys =
      __builtin_amdgcn_make_buffer_rsrc(a.y, 0, a.n * a.h2 * a.w2 * 64, 0x00020000);
  constexpr unsigned kOob = 0x80000000u;                 // buffer offset past num_records: loads 0, stores dropped

  int idx = blockIdx.x * a.per_wave;
  const int end = min(idx + a.per_wave, a.total);
  while (idx < end) {
    const int seg = idx / a.h2;
    const int ya = idx - seg * a.h2;
    const int yb = min(a.h2, ya + (end - idx));
    idx += yb - ya;
    const int n = seg / a.ns, s = seg - n * a.ns;

    const int X0 = kCols * s;
    const int S0 = 2 * X0 - 3;                       // stem / layer1 column of pair 0, sub-pixel 0
    const int col = S0 + 2 * r + hh;                 // this lane's stem / layer1 pixel
    const uint32_t cmask = static_cast<unsigned>(col) < static_cast<unsigned>(W) ? 0xffffffffu : 0u;
    const int ccl = col < 3 ? col : (col >= W - 3 ? 6 - (W - 1 - col) : 3);
    const int cc = ccl < 0 ? 0 : (ccl > 6 ? 6 : ccl);
    // frame bytes: image byte t <-> row byte fb0 + t (fb0 % 4 == 0); lane l converts t = 4l .. 4l+3
    const int fb0 = 6 * X0 - 20;
    const int cb = fb0 + 4 * lane;
    auto bv = [&](int k) { return static_cast<unsigned>(cb + k) < static_cast<unsigned>(rowb); };
    const uint32_t fm0 = (bv(0) ? 0x0000ffffu : 0u) | (bv(1) ? 0xffff0000u : 0u);
    const uint32_t fm1 = (bv(2) ? 0x0000ffffu : 0u) | (bv(3) ? 0xffff0000u : 0u);
    // stem B: pair r's window chunk j at image byte 4 + 12 r + 16 j (f16 image = 2 B per byte)
    const int oP = 4 + 12 * r + 16 * hh;             // P fragments: chunk j = lane half
    const int oX = 36 + 12 * r;                      // X fragments: chunk 2 of rows fr + lane half
    const int rdP = (r & 1) ? oP : kCopyB + oP;
    const int rdX = ((r & 1) ? oX : kCopyB + oX) + hh * kRowB;     // lane half h reads row fr + h
    // exchange offsets (plane 1 = +2 kXSp)
    const int xo_own = hh * kXSp + (r + 1) * 16;
    const int xo_lr = hh ? (r + 2) * 16 : kXSp + r * 16;     // half 0: pixel 2r-1, half 1: 2r+2
    const int xo_r = hh * 2 * kXSp + (r + 2) * 16;          // layer2: pixel 2r+2, channels 8h..
    const int x2 = X0 - 1 + r;
    const bool st_ok = r >= 1 && r <= kCols && x2 < a.w2;
    const int frame_row0 = n * H;
    const float* ctl = ctab + cc * 16;               // this lane's column case

    auto row_ok = [&](int q) { return static_cast<unsigned>(q) < static_cast<unsigned>(H); };
    auto load_row = [&](int fr) -> uint32_t {        // OOB offset for rows outside the frame: 0
      const unsigned off = row_ok(fr) ? static_cast<unsigned>((frame_row0 + fr) * rowb + cb) : kOob;
      return __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    };
    auto ring_put = [&](int fr, uint32_t raw) {
      const bool ok = row_ok(fr);
      const uint32_t f0 = __builtin_amdgcn_perm(kF16Hi, raw, 0x04010400u) & (ok ? fm0 : 0u);
      const uint32_t f1 = __builtin_amdgcn_perm(kF16Hi, raw, 0x04030402u) & (ok ? fm1 : 0u);
      char* row = ring + (fr & (kRing - 1)) * kRowB;
      *reinterpret_cast<uint2*>(row + 8 * lane) = make_uint2(f0, f1);
      *reinterpret_cast<uint32_t*>(row + kCopyB + 8 * lane) = f0;
      *reinterpret_cast<uint32_t*>(row + kCopyB + 8 * lane + 4) = f1;
    };
    auto slot6 = [](int row) { return (row + 12) % 6; };   // rows >= -12
    auto put_x = [&](char* base, int row, const uint32_t (&v)[8]) {
      char* p = base + slot6(row) * kXSlot + xo_own;
      *reinterpret_cast<uint4*>(p) = make_uint4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<uint4*>(p + 2 * kXSp) = make_uint4(v[4], v[5], v[6], v[7]);
    };
    auto row_case = [&](int q) { const int v = q < 3 ? q : (q >= H - 3 ? 6 - (H - 1 - q) : 3); return v < 0 ? 0 : (v > 6 ? 6 : v); };
    auto cinit = [&](int q) -> f32x16 {
      const float4* ct = reinterpret_cast<const float4*>(ctl + row_case(q) * 7 * 16);
      f32x16 c;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 v = ct[i];
        c[4 * i] = v.x; c[4 * i + 1] = v.y; c[4 * i + 2] = v.z; c[4 * i + 3] = v.w;
      }
      return c;
    };

    // Skewed walk: step j computes stem rows 2j+3, 2j+4, layer1 rows 2j, 2j+1 and layer2 row j-1,
    // each from rows the PREVIOUS steps wrote, so the three MFMA chains of a step are independent
    // and the stem / layer1 epilogues run under the later chains' MFMAs.  Steps ya-3 .. yb cover
    // layer2 rows ya .. yb-1 (edge steps compute rows nobody stores).  The frame rows step j reads
    // (2j .. 2j+7) were converted by the end of step j-1.
    const int j0 = ya - 3;
    {
      uint32_t raw[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) raw[i] = load_row(2 * j0 + i);
#pragma unroll
      for (int i = 0; i < 8; ++i) ring_put(2 * j0 + i, raw[i]);
    }
    uint32_t raw0 = load_row(2 * j0 + 8), raw1 = load_row(2 * j0 + 9);
    for (int j = j0; j <= yb; ++j) {
      const int q = 2 * j + 3;                       // stem rows q, q+1
      // ---- operand reads (all from rows written by earlier steps)
      f16x8 bp[8], bx[4], bx2[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) bp[i] = ld_frag_f16(ring + ((2 * j + i) & (kRing - 1)) * kRowB, rdP);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        // X term t of stem row q: chunk 2 of rows q-3+2t+h = 2j+2t+h; of row q+1: 2j+1+2t+h
        // (the kh = 7 half of t = 3 has zero weights; its row aliases a live ring slot)
        bx[t] = ld_frag_f16(ring + ((2 * j + 2 * t) & (kRing - 1)) * kRowB, rdX - ((((2 * j + 2 * t) & (kRing - 1)) == kRing - 1) ? hh * kRing * kRowB : 0));
        bx2[t] = ld_frag_f16(ring + ((2 * j + 1 + 2 * t) & (kRing - 1)) * kRowB, rdX - ((((2 * j + 1 + 2 * t) & (kRing - 1)) == kRing - 1) ? hh * kRing * kRowB : 0));
      }
      const f32x16 ci0 = cinit(q), ci1 = cinit(q + 1);
      bf16x8 o1a[4], o1b[4], lr1a[4], lr1b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const char* sl = xs0 + slot6(2 * j - 1 + i) * kXSlot;
        o1a[i] = ld_frag_bf16(sl + xo_own);
        o1b[i] = ld_frag_bf16(sl + 2 * kXSp + xo_own);
        lr1a[i] = ld_frag_bf16(sl + xo_lr);
        lr1b[i] = ld_frag_bf16(sl + 2 * kXSp + xo_lr);
      }
      bf16x8 o2a[3], o2b[3], rr2[3];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const char* sl = xs1 + slot6(2 * j - 3 + kh) * kXSlot;
        o2a[kh] = ld_frag_bf16(sl + xo_own);
        o2b[kh] = ld_frag_bf16(sl + 2 * kXSp + xo_own);
        rr2[kh] = ld_frag_bf16(sl + xo_r);
      }
      // every operand of the step is in flight before the first MFMA waits on one
      if constexpr (DRNMI_FR_PIN) __builtin_amdgcn_sched_barrier(0);
      // ---- stem (2 x 11 MFMAs)
      f32x16 s0 = ci0, s1 = ci1;
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
        s0 = mfma_f16<1>(as[kh], bp[kh], s0);
        s1 = mfma_f16<1>(as[kh], bp[kh + 1], s1);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s0 = mfma_f16<1>(as[7 + t], bx[t], s0);
        s1 = mfma_f16<1>(as[7 + t], bx2[t], s1);
      }
      // ---- layer1 (2 x 12 MFMAs)
      f32x16 l0 = c1, l1 = c1;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        l0 = mfma_bf16<2>(a1[4 * kh + 0], o1a[kh], l0);
        l1 = mfma_bf16<2>(a1[4 * kh + 0], o1a[kh + 1], l1);
        l0 = mfma_bf16<2>(a1[4 * kh + 1], o1b[kh], l0);
        l1 = mfma_bf16<2>(a1[4 * kh + 1], o1b[kh + 1], l1);
        l0 = mfma_bf16<2>(a1[4 * kh + 2], lr1a[kh], l0);
        l1 = mfma_bf16<2>(a1[4 * kh + 2], lr1a[kh + 1], l1);
        l0 = mfma_bf16<2>(a1[4 * kh + 3], lr1b[kh], l0);
        l1 = mfma_bf16<2>(a1[4 * kh + 3], lr1b[kh + 1], l1);
      }
      // ---- stem epilogue (overlaps the layer1 / layer2 MFMAs)
      {
        const uint32_t m0 = row_ok(q) ? cmask : 0u, m1 = row_ok(q + 1) ? cmask : 0u;
        uint32_t v0[8], v1[8];
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          v0[d] = relu_pk(s0[2 * d], s0[2 * d + 1]) & m0;
          v1[d] = relu_pk(s1[2 * d], s1[2 * d + 1]) & m1;
        }
        put_x(xs0, q, v0);
        put_x(xs0, q + 1, v1);
      }
      // ---- layer2 (9 MFMAs): row j - 1
      f32x16 t2 = c2;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        t2 = mfma_bf16<4>(a2[3 * kh + 0], o2a[kh], t2);
        t2 = mfma_bf16<4>(a2[3 * kh + 1], o2b[kh], t2);
        t2 = mfma_bf16<4>(a2[3 * kh + 2], rr2[kh], t2);
      }
      // ---- layer1 epilogue
      {
        const int p = 2 * j;
        const uint32_t m0 = row_ok(p) ? cmask : 0u, m1 = row_ok(p + 1) ? cmask : 0u;
        uint32_t v0[8], v1[8];
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          v0[d] = relu_pk(l0[2 * d], l0[2 * d + 1]) & m0;
          v1[d] = relu_pk(l1[2 * d], l1[2 * d + 1]) & m1;
        }
        put_x(xs1, p, v0);
        put_x(xs1, p + 1, v1);
      }
      // ---- layer2 epilogue: NHWC bf16 stores, lane half h holds channels 8g + 4h .. + 3
      {
        const int y = j - 1;
        const bool store = st_ok && y >= ya && y < yb && (DRNMI_FR_ABL & 8) == 0;
        const unsigned off =
            store ? static_cast<unsigned>(((static_cast<int>(n) * a.h2 + y) * a.w2 + x2) * 64 + 8 * hh) : kOob;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint2 v = make_uint2(relu_pk(t2[4 * g], t2[4 * g + 1]), relu_pk(t2[4 * g + 2], t2[4 * g + 3]));
          __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{v.x, v.y}, ys, off, 16 * g, 0);
        }
      }
      // ---- frame rows 2j+8, 2j+9 into the ring (over rows 2j, 2j+1: read above), next loads
      ring_put(2 * j + 8, raw0);
      ring_put(2 * j + 9, raw1);
      raw0 = load_row(2 * j + 10);
      raw1 = load_row(2 * j + 11);
    }
  }
}

int g_front_waves = 0;

// ---------------------------------------------------------------- host packing (no GPU)
uint16_t host_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}
uint16_t host_f16(float f) {
  const _Float16 h = static_cast<_Float16>(f);
  uint16_t r;
  memcpy(&r, &h, 2);
  return r;
}
float host_f16_val(uint16_t b) {
  _Float16 h;
  memcpy(&h, &b, 2);
  return static_cast<float>(h);
}

}  // namespace

bool front_ok(int n, int h, int w) {
  return n > 0 && h >= 8 && w >= 8 && w % 4 == 0 && static_cast<int64_t>(n) * h * w * 3 < (int64_t(1) << 31);
}

}  // namespace drnmi

using namespace drnmi;

extern "C" int64_t drnmi_front_pack_bytes(void) { return kPackB; }

extern "C" int drnmi_front_supported(int32_t n, int32_t h, int32_t w) { return front_ok(n, h, w) ? 1 : 0; }

extern "C" int drnmi_front_pack(const float* w0, const float* scale0, const float* shift0, const float* w1,
                                const float* scale1, const float* shift1, const float* w2, const float* scale2,
                                const float* shift2, const float* mean3, const float* std3, int32_t bgr,
                                void* out_host) {
  if (!w0 || !shift0 || !w1 || !shift1 || !w2 || !shift2 || !mean3 || !std3 || !out_host) return DRNMI_EINVAL;
  char* out = static_cast<char*>(out_host);
  memset(out, 0, kPackB);
  auto sc = [](const float* s, int c) { return s ? s[c] : 1.0f; };
  // stem: folded f16 weights W16[co][mc][kh][kw] = w * scale / (255 std[mc])
  uint16_t w16[16][3][7][7];
  for (int co = 0; co < 16; ++co)
    for (int mc = 0; mc < 3; ++mc)
      for (int kh = 0; kh < 7; ++kh)
        for (int kw = 0; kw < 7; ++kw) {
          const double v = static_cast<double>(w0[((co * 3 + mc) * 7 + kh) * 7 + kw]) * sc(scale0, co) /
                           (255.0 * static_cast<double>(std3[mc]));
          w16[co][mc][kh][kw] = host_f16(static_cast<float>(v));
        }
  uint16_t* fs = reinterpret_cast<uint16_t*>(out);
  for (int m = 0; m < kFS; ++m)
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 8; ++e) {
        const int i = l & 31, hq = l >> 5;
        const int sp = (i >> 2) & 1, co = (i & 3) + 4 * (i >> 3);
        int kh, j;
        if (m < 7) { kh = m; j = hq; } else { kh = 2 * (m - 7) + hq; j = 2; }
        uint16_t v = 0;
        if (kh < 7) {
          const int b = 8 * j + e, px = b / 3, c = b % 3;
          const int mc = bgr ? 2 - c : c;
          const int kw = px - sp;
          if (kw >= 0 && kw < 7) v = w16[co][mc][kh][kw];
        }
        fs[(m * 64 + l) * 8 + e] = v;
      }
  // stem starting values per (row case, column case): shift - sum over in-image taps of
  // (1024 W16 + w * scale * mean / std)
  float* c0 = reinterpret_cast<float*>(out + kOffC0);
  for (int rc = 0; rc < 7; ++rc)
    for (int cc = 0; cc < 7; ++cc)
      for (int co = 0; co < 16; ++co) {
        double acc = 0.0;
        for (int kh = 0; kh < 7; ++kh) {
          if (rc < 3 && kh < 3 - rc) continue;          // frame row q - 3 + kh < 0 (q = rc)
          if (rc > 3 && kh > 9 - rc) continue;          // frame row >= H (q = H - 7 + rc)
          for (int kw = 0; kw < 7; ++kw) {
            if (cc < 3 && kw < 3 - cc) continue;
            if (cc > 3 && kw > 9 - cc) continue;
            for (int mc = 0; mc < 3; ++mc) {
              const double wf = static_cast<double>(w0[((co * 3 + mc) * 7 + kh) * 7 + kw]) * sc(scale0, co);
              acc += 1024.0 * static_cast<double>(host_f16_val(w16[co][mc][kh][kw])) +
                     wf * static_cast<double>(mean3[mc]) / static_cast<double>(std3[mc]);
            }
          }
        }
        c0[(rc * 7 + cc) * 16 + co] = static_cast<float>(static_cast<double>(shift0[co]) - acc);
      }
  // layer1: own pixels (2r, 2r+1 on lane halves) and the neighbours (2r-1 | 2r+2)
  uint16_t* f1 = reinterpret_cast<uint16_t*>(out + kOffL1);
  for (int m = 0; m < kF1; ++m)
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 8; ++e) {
        const int i = l & 31, hq = l >> 5;
        const int sp = (i >> 2) & 1, co = (i & 3) + 4 * (i >> 3);
        const int kh = m / 4, f = m % 4;
        const int ch = (f & 1) ? 8 + e : e;
        const int dx = f < 2 ? hq - sp : (hq ? 2 - sp : -1 - sp);
        const int kw = dx + 1;
        uint16_t v = 0;
        if (kw >= 0 && kw < 3) v = host_bf16(w1[((co * 16 + ch) * 3 + kh) * 3 + kw] * sc(scale1, co));
        f1[(m * 64 + l) * 8 + e] = v;
      }
  // layer2: output channel on the A row; own pixels 2x-1, 2x (kw = lane half), right pixel 2x+1
  uint16_t* f2 = reinterpret_cast<uint16_t*>(out + kOffL2);
  for (int m = 0; m < kF2; ++m)
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 8; ++e) {
        const int co = l & 31, hq = l >> 5;
        const int kh = m / 3, f = m % 3;
        const int ch = f == 0 ? e : (f == 1 ? 8 + e : 8 * hq + e);
        const int kw = f < 2 ? hq : 2;
        f2[(m * 64 + l) * 8 + e] = host_bf16(w2[((co * 16 + ch) * 3 + kh) * 3 + kw] * sc(scale2, co));
      }
  float* c1 = reinterpret_cast<float*>(out + kOffC1);
  for (int co = 0; co < 16; ++co) c1[co] = shift1[co];
  float* c2 = reinterpret_cast<float*>(out + kOffC2);
  for (int co = 0; co < 32; ++co) c2[co] = shift2[co];
  return DRNMI_OK;
}

extern "C" int drnmi_video_front_u8(const uint8_t* frames, const void* pack, void* y, int32_t n, int32_t h,
                                    int32_t w, void* stream) {
  if (!frames || !pack || !y || !front_ok(n, h, w)) return DRNMI_EINVAL;
  if (g_front_waves == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    g_front_waves = 4 * cus;                          // one 512-VGPR wave per SIMD
  }
  FrontParams p;
  p.x = frames;
  p.pack = static_cast<const char*>(pack);
  p.y = static_cast<bf16_t*>(y);
  p.n = n;
  p.h = h;
  p.w = w;
  p.h2 = (h + 1) / 2;
  p.w2 = (w + 1) / 2;
  p.ns = (p.w2 + kCols - 1) / kCols;
  p.total = n * p.ns * p.h2;
  const int waves = p.total < g_front_waves ? p.total : g_front_waves;
  p.per_wave = (p.total + waves - 1) / waves;
  const int grid = (p.total + p.per_wave - 1) / p.per_wave;
  hipLaunchKernelGGL(front_kernel, dim3(grid), dim3(64), kLds, static_cast<hipStream_t>(stream), p);
  return static_cast<int>(hipGetLastError());
}
