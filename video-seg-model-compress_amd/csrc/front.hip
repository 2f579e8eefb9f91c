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

#include <type_traits>

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
constexpr int kOffC0 = kOffL2 + kF2 * kFragB;          // float [8 row cases][8 col cases][16]
constexpr int kCTabB = 64 * 16 * 4;                    // case 7 = outside the image: -1e30
constexpr int kOffC1 = kOffC0 + kCTabB;                 // float [16] layer1 shift
constexpr int kOffC2 = kOffC1 + 16 * 4;                // float [32] layer2 shift
constexpr int kPackB = kOffC2 + 32 * 4;

// ---- geometry
constexpr int kCols = 30;                // layer2 columns per strip (pairs 1..30 of 32)
constexpr int kRing = 8;                 // converted frame rows in the LDS ring
constexpr int kRowB = 1040;              // ring row: image byte o at o (copy A) and at kCopyB + o
constexpr int kCopyB = 516;              //   (copy B: 8-B aligned where o % 8 == 4)
constexpr int kXSp = 34 * 16;            // exchange: [plane 2][sp 2][pair slot 34][16 B], pair r at r + 1
constexpr int kXSlot = 4 * kXSp;
constexpr uint32_t kF16Hi = 0x64646464u;            // v_perm source of the f16 exponent byte 0x64
// front3_kernel's pinned MFMA / epilogue interleave: a sched_barrier between groups, epilogue
// values kept where they are computed (else they sink to their first use, out of the MFMA shadow)
// and their inputs read there (else the packing hoists to where they are ready, ahead of MFMAs)
#define FR_SB() __builtin_amdgcn_sched_barrier(0)
#define FR_PINV(x) ({ uint32_t _v = (x); asm volatile("" : "+v"(_v)); _v; })
#define FR_PINF(x) ({ float _f = (x); asm volatile("" : "+v"(_f)); _f; })
constexpr int kFetchAt = 8;               // layer2 MFMA after which the next step's operands are fetched

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
__device__ __forceinline__ f32x16 mfma_f16(const uint4& a, const f16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_bf16(const uint4& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), b, c, 0, 0, 0);
}

// ---- front3_kernel: register-carried rolling windows.  Step j's operands are mostly rows earlier steps already
// hold in registers: the stem's P / X fragments shift by two frame rows per step (only rows 2j+6,
// 2j+7 are read from the ring), layer1's own-pixel operands are the stem outputs S(j-2), S(j-1)
// kept as bf16 registers and only their left/right neighbours come from the LDS exchange, and
// likewise for layer2.  The loop is unrolled by the ring period (4 steps) so every LDS address is
// a per-lane base plus an immediate; ring slot 8 duplicates slot 0 so a lane-half's "row + 1" never
// wraps.  Per step: 22 + 24 + 9 MFMAs against ~14 LDS reads and ~14 LDS writes.
constexpr int kRing3 = kRing + 1;                       // slot 8 = copy of slot 0
constexpr int kX3Slots = 4;                             // exchange rows per activation (row & 3)
constexpr int kLds3Zero = kRing3 * kRowB + 2 * kX3Slots * kXSlot;
constexpr int kLds3 = kLds3Zero + kCTabB + 256;        // + layer1 starts [in | out][16], layer2 [h][16]

template <int N>
using ic = std::integral_constant<int, N>;

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
front3_kernel(const FrontParams a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const ring = smem;
  char* const xs0 = smem + kRing3 * kRowB;                // stem rows (slot = row & 3)
  char* const xs1 = xs0 + kX3Slots * kXSlot;              // layer1 rows (slot = row & 3)
  char* const ctab = xs1 + kX3Slots * kXSlot;             // float [7][7][16] stem shifts
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
  // the 32 weight fragments live in AGPRs (MFMA A operands may be AGPRs): the VGPRs are left to
  // the operand fragments and the accumulators, whose epilogue VALU would otherwise copy them out
#pragma unroll
    for (int m = 0; m < kFS; ++m) { u32x4_t t = __builtin_bit_cast(u32x4_t, as[m]); asm volatile("" : "+a"(t)); as[m] = __builtin_bit_cast(uint4, t); }
#pragma unroll
    for (int m = 0; m < kF1; ++m) { u32x4_t t = __builtin_bit_cast(u32x4_t, a1[m]); asm volatile("" : "+a"(t)); a1[m] = __builtin_bit_cast(uint4, t); }
#pragma unroll
    for (int m = 0; m < kF2; ++m) { u32x4_t t = __builtin_bit_cast(u32x4_t, a2[m]); asm volatile("" : "+a"(t)); a2[m] = __builtin_bit_cast(uint4, t); }
  // layer1 / layer2 starting values live in LDS next to the stem table (re-read every step: the
  // walk's registers are full): c1l[0] = layer1 shift, c1l[1] = -1e30 (pixel outside the image),
  // c2l[h] = layer2 shift of 32x32 D row (j&3) + 8(j>>2) + 4h = channel
  float* const c1l = reinterpret_cast<float*>(ctab + kCTabB);
  float* const c2l = c1l + 32;
  for (int i = lane * 16; i < kLds3Zero; i += 64 * 16) *reinterpret_cast<uint4*>(smem + i) = make_uint4(0, 0, 0, 0);
  for (int i = lane * 4; i < kCTabB; i += 64 * 4)
    *reinterpret_cast<float*>(ctab + i) = *reinterpret_cast<const float*>(a.pack + kOffC0 + i);
  {
    const float* c1t = reinterpret_cast<const float*>(a.pack + kOffC1);
    const float* c2t = reinterpret_cast<const float*>(a.pack + kOffC2);
    const int j = lane & 15, q = lane >> 4;
    if (q == 0) c1l[j] = c1t[j];
    else if (q == 1) c1l[16 + j] = -1e30f;
    else c2l[16 * (q - 2) + j] = c2t[(j & 3) + 8 * (j >> 2) + 4 * (q - 2)];
  }
  __syncthreads();
  auto ld16 = [](const float* t) {
    const float4* v4 = reinterpret_cast<const float4*>(t);
    f32x16 c;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 v = v4[i];
      c[4 * i] = v.x; c[4 * i + 1] = v.y; c[4 * i + 2] = v.z; c[4 * i + 3] = v.w;
    }
    return c;
  };

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
    const int fb0 = 6 * X0 - 20;                     // image byte t <-> row byte fb0 + t
    const int cb = fb0 + 4 * lane;
    auto bv = [&](int k) { return static_cast<unsigned>(cb + k) < static_cast<unsigned>(rowb); };
    const uint32_t fm0 = (bv(0) ? 0x0000ffffu : 0u) | (bv(1) ? 0xffff0000u : 0u);
    const uint32_t fm1 = (bv(2) ? 0x0000ffffu : 0u) | (bv(3) ? 0xffff0000u : 0u);
    // per-lane LDS bases (every other part of an address is an immediate)
    const int oP = 4 + 12 * r + 16 * hh, oX = 36 + 12 * r;
    char* const rP = ring + ((r & 1) ? oP : kCopyB + oP);
    char* const rX = ring + ((r & 1) ? oX : kCopyB + oX) + hh * kRowB;   // lane half h: row + h
    char* const rW = ring + 8 * lane;
    char* const x0own = xs0 + hh * kXSp + (r + 1) * 16;
    char* const x0lr = xs0 + (hh ? (r + 2) * 16 : kXSp + r * 16);      // half 0: pixel 2r-1, 1: 2r+2
    char* const x1own = xs1 + hh * kXSp + (r + 1) * 16;
    char* const x1r = xs1 + hh * 2 * kXSp + (r + 2) * 16;               // pixel 2r+2, channels 8h..
    const char* const ctl = ctab + (cmask ? cc : 7) * 64;      // case 7: outside the image
    const int x2 = X0 - 1 + r;
    const bool st_ok = r >= 1 && r <= kCols && x2 < a.w2;
    const int frame_row0 = n * H;
    const float* const c1m = c1l + (cmask ? 0 : 16);  // layer1 start: -1e30 outside the image
    const float* const c2m = c2l + 16 * hh;
    const unsigned st_base = static_cast<unsigned>((static_cast<int>(n) * a.h2 * a.w2 + x2) * 64 + 8 * hh);

    auto row_ok = [&](int q) { return static_cast<unsigned>(q) < static_cast<unsigned>(H); };
    auto load_row = [&](int fr) -> uint32_t {
      const unsigned off = row_ok(fr) ? static_cast<unsigned>((frame_row0 + fr) * rowb + cb) : kOob;
      return __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    };
    auto conv2 = [&](int fr, uint32_t raw) {
      const bool ok = row_ok(fr);
      return make_uint2(__builtin_amdgcn_perm(kF16Hi, raw, 0x04010400u) & (ok ? fm0 : 0u),
                        __builtin_amdgcn_perm(kF16Hi, raw, 0x04030402u) & (ok ? fm1 : 0u));
    };
    auto load_row_in = [&](int fr) -> uint32_t {     // row known to be inside the frame
      return __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<unsigned>((frame_row0 + fr) * rowb + cb), 0, 0);
    };
    auto conv2_in = [&](uint32_t raw) {
      return make_uint2(__builtin_amdgcn_perm(kF16Hi, raw, 0x04010400u) & fm0,
                        __builtin_amdgcn_perm(kF16Hi, raw, 0x04030402u) & fm1);
    };
    auto ring_put = [&](auto sl_, uint2 f) {        // slot (compile-time) <- converted row
      constexpr int sl = decltype(sl_)::value;
      *reinterpret_cast<uint2*>(rW + sl * kRowB) = f;
      *reinterpret_cast<uint32_t*>(rW + sl * kRowB + kCopyB) = f.x;
      *reinterpret_cast<uint32_t*>(rW + sl * kRowB + kCopyB + 4) = f.y;
      if constexpr (sl == 0) {
        *reinterpret_cast<uint2*>(rW + kRing * kRowB) = f;
        *reinterpret_cast<uint32_t*>(rW + kRing * kRowB + kCopyB) = f.x;
        *reinterpret_cast<uint32_t*>(rW + kRing * kRowB + kCopyB + 4) = f.y;
      }
    };
    auto ldP = [&](int sl) { return ld_frag_f16(rP + sl * kRowB, 0); };
    auto ldX = [&](int sl) { return ld_frag_f16(rX + sl * kRowB, 0); };
    auto put_x = [&](char* own, int sl, const uint32_t (&v)[8]) {
      *reinterpret_cast<uint4*>(own + sl * kXSlot) = make_uint4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<uint4*>(own + sl * kXSlot + 2 * kXSp) = make_uint4(v[4], v[5], v[6], v[7]);
    };
    auto row_case = [&](int q) {
      const int v = q < 3 ? q : (q >= H - 3 ? 6 - (H - 1 - q) : 3);
      return row_ok(q) ? (v < 0 ? 0 : (v > 6 ? 6 : v)) : 7;
    };
    auto cinit_case = [&](int rc) -> f32x16 {
      const float4* ct = reinterpret_cast<const float4*>(ctl + rc * 8 * 64);
      f32x16 c;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 v = ct[i];
        c[4 * i] = v.x; c[4 * i + 1] = v.y; c[4 * i + 2] = v.z; c[4 * i + 3] = v.w;
      }
      return c;
    };
    auto cinit = [&](int q) { return cinit_case(row_case(q)); };
    auto tobf = [&](const uint32_t (&v)[4]) { return __builtin_bit_cast(bf16x8, make_uint4(v[0], v[1], v[2], v[3])); };

    // walk state at step j: P[i] = ring row 2j+i (i < 8), X[t] = rows 2j+2t+h, X2[t] = rows 2j+1+2t+h
    // (the stem's B operands); V[k] = stem row 2j-1+k (bf16 own pixels, planes a | b), LR[k] its
    // left / right neighbour operands; Wl[k] = layer1 row 2j-3+k, Rl[k] its right-neighbour
    // operand; t2p the previous step's layer2 sums
    f16x8 P[8], X[4], X2[4];
    uint32_t V[4][8], LR[4][8], Wl[3][8], Rl[3][4];
    f32x16 t2p;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int d = 0; d < 8; ++d) V[k][d] = LR[k][d] = 0u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int d = 0; d < 8; ++d) Wl[k][d] = 0u;
#pragma unroll
      for (int d = 0; d < 4; ++d) Rl[k][d] = 0u;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) t2p[i] = 0.f;

    // the walk: steps jb .. jl, jb = (ya - 3) rounded down to a multiple of 4 (so the unrolled
    // copies see fixed slots), jl the end of the last whole group of 4 at or after yb; edge steps
    // compute rows nobody stores
    const int jb = (ya - 3) & ~3;
    const int jl = jb + ((yb - jb + 4) & ~3) - 1;
    uint32_t raw0, raw1;
    {
      uint32_t raw[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) raw[i] = load_row(2 * jb + i);
      // ring slot of row 2jb + i = i (2jb % 8 == 0)
      ring_put(ic<0>{}, conv2(2 * jb + 0, raw[0]));
      ring_put(ic<1>{}, conv2(2 * jb + 1, raw[1]));
      ring_put(ic<2>{}, conv2(2 * jb + 2, raw[2]));
      ring_put(ic<3>{}, conv2(2 * jb + 3, raw[3]));
      ring_put(ic<4>{}, conv2(2 * jb + 4, raw[4]));
      ring_put(ic<5>{}, conv2(2 * jb + 5, raw[5]));
      ring_put(ic<6>{}, conv2(2 * jb + 6, raw[6]));
      ring_put(ic<7>{}, conv2(2 * jb + 7, raw[7]));
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) P[i] = ldP(i);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      X[t] = ldX(2 * t);
      X2[t] = ldX(2 * t + 1);
    }
    raw0 = load_row(2 * jb + 8);
    raw1 = load_row(2 * jb + 9);

    auto ld8 = [&](const char* base, uint32_t (&v)[8]) {
      const uint4 va = *reinterpret_cast<const uint4*>(base);
      const uint4 vb = *reinterpret_cast<const uint4*>(base + 2 * kXSp);
      v[0] = va.x; v[1] = va.y; v[2] = va.z; v[3] = va.w;
      v[4] = vb.x; v[5] = vb.y; v[6] = vb.z; v[7] = vb.w;
    };
    // Operands of step j (PH = j & 3), fetched during step j-1's layer2 MFMAs: ring rows 2j+8,
    // 2j+9 (loaded a step earlier) over rows 2j, 2j+1, their successors' loads, the new ring rows
    // 2j+6, 2j+7, the stem rows' neighbour operands and the two older
    // rows' own pixels (rows 2j+1, 2j+2 stay in registers from step j-1).  BORDER: the segment
    // touches the frame's first or last rows (row checks); else every row is inside.
    auto fetch = [&](int j, auto ph_, auto border_) {
      constexpr int PH = decltype(ph_)::value;
      constexpr bool BORDER = decltype(border_)::value != 0;
      constexpr int R0 = 2 * PH;
      if constexpr (BORDER) {
        ring_put(ic<(R0 + 8) & 7>{}, conv2(2 * j + 8, raw0));
        ring_put(ic<(R0 + 9) & 7>{}, conv2(2 * j + 9, raw1));
        raw0 = load_row(2 * j + 10);
        raw1 = load_row(2 * j + 11);
      } else {
        ring_put(ic<(R0 + 8) & 7>{}, conv2_in(raw0));
        ring_put(ic<(R0 + 9) & 7>{}, conv2_in(raw1));
        raw0 = load_row_in(2 * j + 10);
        raw1 = load_row_in(2 * j + 11);
      }
      P[6] = ldP((R0 + 6) & 7);
      P[7] = ldP((R0 + 7) & 7);
      X[3] = ldX((R0 + 6) & 7);
      X2[3] = ldX((R0 + 7) & 7);
#pragma unroll
      for (int k = 0; k < 4; ++k) ld8(x0lr + ((R0 - 1 + k) & 3) * kXSlot, LR[k]);
      ld8(x0own + ((R0 - 1) & 3) * kXSlot, V[0]);
      ld8(x0own + (R0 & 3) * kXSlot, V[1]);
    };
    // layer2 epilogue of row y from its sums: NHWC bf16, lane half h holds channels 8g + 4h .. + 3;
    // piece g of 0..3 (8 B) -- or the packing of piece g (stores issued separately)
    auto l2_store = [&](int y, const uint32_t (&o)[8]) {
      const bool store = st_ok && y >= ya && y < yb;
      const unsigned off = store ? st_base + static_cast<unsigned>(y * a.w2 * 64) : kOob;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{o[2 * g], o[2 * g + 1]}, ys, off, 16 * g, 0);
    };

    // One step (PH = j & 3: ring slot of row 2j + i is (2 PH + i) & 7, exchange slot of row 2j + k is
    // (2 PH + k) & 3).  Pipelined over the step boundary: the previous step's layer2 epilogue runs
    // in the shadows of this step's stem MFMAs, the stem epilogue under the layer1 MFMAs, the
    // layer1 epilogue and the next step's operand fetch under the layer2 MFMAs; the instruction
    // order is pinned (FR_SB).
    auto step = [&](int j, auto ph_, auto border_) {
      constexpr int PH = decltype(ph_)::value;
      constexpr bool BORDER = decltype(border_)::value != 0;
      constexpr int R0 = 2 * PH;
      const int p = 2 * j;                           // layer1 rows p, p+1; stem rows p+3, p+4
      FR_SB();
      // ---- B: stem rows p+3, p+4 (2 x 11 MFMAs) + layer2 epilogue of row j-2 (t2p)
      uint32_t o2[8];
      f32x16 s0 = {}, s1 = {}, l0, cs0, cs1;
#pragma unroll
      for (int i = 0; i < 22; ++i) {
        const int kh = i >> 1;
        if (kh < 7) {
          if ((i & 1) == 0) s0 = mfma_f16(as[kh], P[kh], s0);
          else s1 = mfma_f16(as[kh], P[kh + 1], s1);
        } else {
          const int t = kh - 7;
          if ((i & 1) == 0) s0 = mfma_f16(as[7 + t], X[t], s0);
          else s1 = mfma_f16(as[7 + t], X2[t], s1);
        }
        if (i < 8) o2[i] = FR_PINV(relu_pk(FR_PINF(t2p[2 * i]), FR_PINF(t2p[2 * i + 1])));
        if (i == 9) l2_store(j - 2, o2);
        // later stages' LDS operands, issued a stage ahead: layer1 starting values, the stem rows'
        // border-case offsets (interior segments: row case 3)
        if (i == 12) l0 = ld16(c1m);
        if (i == 14) cs0 = BORDER ? cinit(p + 3) : cinit_case(3);
        if (i == 16) cs1 = BORDER ? cinit(p + 4) : cinit_case(3);
        FR_SB();
      }
      // ---- C: layer1 rows p, p+1 from stem rows p-1 .. p+2 (2 x 12 MFMAs); the stem epilogue
      // adds the stem rows' border-case offsets (pixels outside the image get -1e30: ReLU gives
      // layer1's exact zero padding; interior segments see row case 3 only)
      uint32_t vq0[8], vq1[8];
      f32x16 l1 = l0, t2;
#pragma unroll
      for (int i = 0; i < 24; ++i) {
        if (i == 4) {
          // layer2 operands: layer1 row 2j-3 own pixels, right neighbours of rows 2j-3 .. 2j-1
          ld8(x1own + ((R0 - 3) & 3) * kXSlot, Wl[0]);
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const uint4 v = *reinterpret_cast<const uint4*>(x1r + ((R0 - 3 + k) & 3) * kXSlot);
            Rl[k][0] = v.x; Rl[k][1] = v.y; Rl[k][2] = v.z; Rl[k][3] = v.w;
          }
        }
        if (i == 16) t2 = ld16(c2m);
        const int kh = i / 8, f = (i / 2) % 4, odd = i & 1;
        const uint32_t* src = f < 2 ? V[kh + odd] : LR[kh + odd];
        const int o = (f & 1) * 4;
        const bf16x8 b = tobf({src[o], src[o + 1], src[o + 2], src[o + 3]});
        if (odd) l1 = mfma_bf16(a1[4 * kh + f], b, l1);
        else l0 = mfma_bf16(a1[4 * kh + f], b, l0);
        if (i >= 2 && i < 18) {
          const int d = (i - 2) >> 1;
          if ((i & 1) == 0) vq0[d] = FR_PINV(relu_pk(FR_PINF(s0[2 * d]) + cs0[2 * d], FR_PINF(s0[2 * d + 1]) + cs0[2 * d + 1]));
          else vq1[d] = FR_PINV(relu_pk(FR_PINF(s1[2 * d]) + cs1[2 * d], FR_PINF(s1[2 * d + 1]) + cs1[2 * d + 1]));
        }
        if (i == 18) put_x(x0own, (R0 + 3) & 3, vq0);
        if (i == 20) put_x(x0own, (R0 + 4) & 3, vq1);
        FR_SB();
      }
      // ---- D: layer2 row j-1 from layer1 rows 2j-3 .. 2j-1 (9 MFMAs); the layer1 epilogue and
      // the next step's operand fetch
      uint32_t wp0[8], wp1[8];
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const int kh = i / 3, f = i % 3;
        const uint32_t* src = f < 2 ? Wl[kh] + f * 4 : Rl[kh];
        t2 = mfma_bf16(a2[i], tobf({src[0], src[1], src[2], src[3]}), t2);
        if (i >= 1) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int k = 2 * (i - 1) + e;             // 0 .. 15
            const int d = k >> 1;
            if ((k & 1) == 0) wp0[d] = FR_PINV(relu_pk(FR_PINF(l0[2 * d]), FR_PINF(l0[2 * d + 1])));
            else wp1[d] = FR_PINV(relu_pk(FR_PINF(l1[2 * d]), FR_PINF(l1[2 * d + 1])));
          }
        }
        if (i == kFetchAt) {
          // the next step's operands: the frame windows roll by one step (the stem is done with
          // them) and take the new rows; V[2], V[3] = this step's stem rows
#pragma unroll
          for (int k = 0; k < 6; ++k) P[k] = P[k + 2];
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            X[t] = X[t + 1];
            X2[t] = X2[t + 1];
          }
#pragma unroll
          for (int d = 0; d < 8; ++d) {
            V[2][d] = vq0[d];
            V[3][d] = vq1[d];
          }
          fetch(j + 1, ic<(PH + 1) & 3>{}, border_);
        }
        FR_SB();
      }
      if constexpr (BORDER) {                        // frame top / bottom: rows outside are zero
        const bool ok0 = row_ok(p), ok1 = row_ok(p + 1);
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          wp0[d] = ok0 ? wp0[d] : 0u;
          wp1[d] = ok1 ? wp1[d] : 0u;
        }
      }
      put_x(x1own, R0 & 3, wp0);
      put_x(x1own, (R0 + 1) & 3, wp1);
      // ---- roll the layer1 window by one step
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        Wl[1][d] = wp0[d];
        Wl[2][d] = wp1[d];
      }
      t2p = t2;
    };

    // interior segments skip all row checks: every frame row a stem row reads (<= 2jl+7) is inside
    // and every stem row is of row case 3 (rows fetch() converts past 2jl+7 are never read)
    auto walk = [&](auto border_) {
      fetch(jb, ic<0>{}, border_);
      for (int j = jb; j <= jl; j += 4) {
        step(j + 0, ic<0>{}, border_);
        step(j + 1, ic<1>{}, border_);
        step(j + 2, ic<2>{}, border_);
        step(j + 3, ic<3>{}, border_);
      }
      uint32_t o2[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o2[i] = relu_pk(t2p[2 * i], t2p[2 * i + 1]);
      l2_store(jl - 1, o2);
    };
    if (jb < 0 || 2 * jl + 8 > H) walk(ic<1>{});
    else walk(ic<0>{});
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
  // (1024 W16 + w * scale * mean / std); case 7 (a pixel outside the image) starts from -1e30, so
  // ReLU turns it into the next conv's exact zero padding
  float* c0 = reinterpret_cast<float*>(out + kOffC0);
  for (int i = 0; i < 64 * 16; ++i) c0[i] = -1e30f;
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
        c0[(rc * 8 + cc) * 16 + co] = static_cast<float>(static_cast<double>(shift0[co]) - acc);
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
  hipLaunchKernelGGL(front3_kernel, dim3(grid), dim3(64), kLds3, static_cast<hipStream_t>(stream), p);
  return static_cast<int>(hipGetLastError());
}
