// One-wave-per-SIMD strip convs: conv_w1_kernel and the forms of the same template (below).  Own
// translation unit (their 400-512-register allocations must not be perturbed by the other tiles,
// cdna_hip_programming.md §5.4 rule 19).
//
// conv_w1: the same tile (256 output channels x one 256-pixel run of an output row, 3x3 stride 1,
// cin % 128 == 0), LDS image (two 32-KB weight stages, two 33-KB input strips; DMA'd as in
// conv_stag), K order and per-accumulator MFMA order as conv_stag_kernel -- so the output is
// bit-identical to it -- but 4 waves of 128 channels x 128 pixels instead of 8 waves of 128 x 64:
//
//   * per 32-deep substep a wave reads 8 A + 8 B fragments (16 KB) for 64 MFMAs; the 8-wave tile
//     reads 8 A + 4 B per wave for 32 MFMAs, so the LDS read bytes per MFMA drop by a third (the
//     chip holds its clock under load: LDS read energy per MFMA is one of the levers,
//     cdna_hip_programming.md §5.4 rule 28);
//   * accumulators 8 x 8 x 4 = 256 registers (AGPRs), fragments double-buffered (128 VGPRs);
//   * with no partner wave to fill the matrix pipe, each wave hides its own latencies: one barrier
//     per K step, placed in the middle of the second substep (the MFMAs before it drain while the
//     waves meet), every LDS read issued at least two MFMA groups before its use (counted
//     lgkmcnt), every DMA piece issued a whole K step before the barrier that publishes it.
//
// Schedule of K step t (stage t & 1, strip buffer g & 1, t = 3 g + kw), B_t = the barrier that
// publishes step t's weights (and, for kw = 0, group g's strip); FM x FN fragments per wave
// (conv_w1: 8 x 8):
//   X  groups 0..FM-1 (substep 0): wait for a0[fm] (all b0 landed), issue FM+FN / FM reads of
//      substep 1 (b1 first, then a1), FN MFMAs acc[fm][*] += a0[fm] x b0[*];
//   Y  groups 0..FM/2-1 (substep 1): wait for a1[fm], FN MFMAs;
//      vmcnt lgkmcnt(0) s_barrier = B_{t+1}: every wave's DMA for step t + 1 has landed and
//      every wave has finished reading stage t & 1 and (kw = 2) strip g;
//   Y  groups FM/2..FM-1: issue the reads of step t + 1's substep 0 (b0 first) and the DMA of step
//      t + 2's weights (into stage t & 1, just released; past the last step a re-fetch) and of one
//      third of the next strip (group g' + 1 for t + 1 = 3 g' + k': its buffer was last read in
//      step 3 g' - 1, before B_{3 g'}), spread over the groups' MFMA gaps; FN MFMAs each.
//
// Forms (W1Cfg<WCO, FN> derives the counts above from the tile geometry): conv_w1 (WCO 128, FN 8,
// one workgroup per CU), conv_w1h (WCO 64, FN 4: 128 x 128 tiles, 67 KB of LDS, two workgroups per
// CU, so one tile's prologue and epilogue overlap the other's MFMAs), their x2 forms (the folded
// 1x1 downsample as extra K steps after the taps, as conv_stag_x2), the seg-fused form (the seg
// classifier in the epilogue) and the int8 forms (T = int8_t: the same 128-B rows of 128 channels,
// v_mfma_i32_16x16x64_i8, the W8A8 epilogues; ODDOK walks an odd tap-group count).
// Reference: lmodels/drn.py:27-29 (conv3x3, dilation = padding), :49-65 (BasicBlock convs).
#include "common.h"
#include "conv_tile.h"
#include "kernels.h"

namespace drnmi {
namespace {

// Tile = 2 WCO output channels x 2 (16 FN) pixels (a run of one output row), 4 waves: wc = channel
// half, wp = pixel half.  conv_w1: WCO 128, FN 8 (256 x 256, one wave per SIMD); conv_w1h: WCO 64,
// FN 4 (128 x 128, 67 KB of LDS: two workgroups per CU, so two waves per SIMD from different tiles).
template <int WCO, int FN>
struct W1Cfg {
  static constexpr int FM = WCO / 16;
  static constexpr int BCO = 2 * WCO;
  static constexpr int PXW = 16 * FN;             // pixels per wave
  static constexpr int TPX = 2 * PXW;             // pixels per tile
  static constexpr int AB = BCO * 128;            // one A stage: BCO rows x 64 bf16 channels
  static constexpr int AI = BCO / 32;             // 1-KB weight pieces per wave per K step
  static constexpr int NSP = TPX / 8 + 1;         // strip pieces: TPX + 2 dil rows, dil <= 4
  static constexpr int SB = NSP * 1024;           // one strip buffer
  static constexpr int SH = (NSP + 3) / 4;        // strip shares per wave per tap group
  static constexpr int SPS = (SH + 2) / 3;        // shares per wave per K step (3 steps per group)
  static constexpr int NR = FM + FN;              // fragment reads per wave per substep
  static constexpr int RX = NR / FM;              // substep-1 reads per X group
  // 2 A stages + 2 strips + a 1-KB sink: strip pieces past the strip (j >= NSP) land there, so every
  // wave issues the same DMA sequence without a branch
  static constexpr int SINK = 2 * AB + 2 * SB;
  static constexpr int LDS = SINK + 1024;
  static constexpr int GT = (FM / 2) * (FN - 1);  // MFMA gaps of the Y tail (after the barrier)
  static constexpr int NI = NR + AI + SPS;        // reads + DMA pieces issued in them
  static_assert(AI == FN && RX * FM == NR && RX <= FN - 1 && SPS <= FM && 3 * SPS >= SH && AI % 2 == 0, "w1 geometry");
};

template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

// SEGF (the labels-only video path's last conv, drnmi_conv_stag_seg): the activation is not stored;
// as in conv_stag's SEGF epilogue it becomes the B operand of the seg classifier (1x1 512 -> 19 +
// bias, lmodels/drnseg.py:278-284) and each 256-channel block writes partial logits
// part[block][pixel][20] (wc 0 + wc 1, bias added by the head)
struct W1Seg {
  const void* w;        // seg weights, packed bf16 [>= 32 rows][k_pad] (scale folded), rows 19.. zero
  int k_pad;
  void* part;           // fp32 [cout / 256][n ho wo][20]
};
constexpr int kW1SegCS = 20;

// int8 nets: the seg classifier on the int8 copy of the last conv's output, as conv_stag's
// stag_seg_i8 (the same quantisation, the same fixed permutation of K, integer partial sums: the
// same partials) for a wave of FN pixel groups; xch: a free 2 x 64 x 2 FN x 16-B LDS area
template <int FM, int FN>
__device__ __forceinline__ void w1_seg_i8(const drnmi_conv_args& p, const i32x4 (&acc)[FM][FN], int px0, int co0, int wc,
                                          int wp, int fr, int fq, int lane, const W1Seg& sf, char* xbase) {
#pragma clang fp contract(off)
  static_assert(FM % 4 == 0, "64-channel groups");
  constexpr int NG = FM / 4;
  const int8_t* sw = static_cast<const int8_t*>(sf.w);
  const int cw = co0 + wc * 16 * FM;                 // the wave's first channel
  i32x4 aw[2][NG];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        aw[mt][g][m] = *reinterpret_cast<const int*>(sw + static_cast<int64_t>(16 * mt + fr) * sf.k_pad + cw + 64 * g +
                                                     16 * m + 4 * fq);
  const bool relu = p.relu != 0;
  i32x4 pacc[2][FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    pacc[0][fn] = i32x4{0, 0, 0, 0};
    pacc[1][fn] = i32x4{0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      i32x4 b;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int fm = 4 * g + m;
        const int co = cw + 16 * fm + 4 * fq;
        const float4 sc = *reinterpret_cast<const float4*>(p.scale + co);   // padded to cout_pad
        const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
        const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
        uint32_t o = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = static_cast<float>(acc[fm][fn][e]) * scv[e] + shv[e];
          if (relu) v = fmaxf(v, 0.f);
          const float t = fminf(fmaxf(rintf(v * p.out_scale), -127.f), 127.f);
          o |= static_cast<uint32_t>(static_cast<uint8_t>(static_cast<int8_t>(static_cast<int>(t)))) << (8 * e);
        }
        b[m] = static_cast<int>(o);
      }
      pacc[0][fn] = __builtin_amdgcn_mfma_i32_16x16x64_i8(aw[0][g], b, pacc[0][fn], 0, 0, 0);
      pacc[1][fn] = __builtin_amdgcn_mfma_i32_16x16x64_i8(aw[1][g], b, pacc[1][fn], 0, 0, 0);
    }
  }
  // the two channel halves of the tile (waves wc = 0, 1), added through LDS
  i32x4* xch = reinterpret_cast<i32x4*>(xbase) + (wp * 64 + lane) * (2 * FN);
  if (wc == 1) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) xch[mt * FN + fn] = pacc[mt][fn];
  }
  __syncthreads();
  if (wc == 0) {
    const int M = p.n * p.ho * p.wo;
    int* __restrict__ part = static_cast<int*>(sf.part) + static_cast<int64_t>(co0 / (32 * FM)) * M * kW1SegCS;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int cls = 16 * mt + 4 * fq;
      if (cls >= kW1SegCS) continue;
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const i32x4 o = xch[mt * FN + fn];
        const int64_t m = px0 + wp * 16 * FN + fn * 16 + fr;
        *reinterpret_cast<int4*>(part + m * kW1SegCS + cls) =
            make_int4(pacc[mt][fn][0] + o[0], pacc[mt][fn][1] + o[1], pacc[mt][fn][2] + o[2], pacc[mt][fn][3] + o[3]);
      }
    }
  }
}

// ODDOK: also an odd number of tap groups (int8 at cin 128: 9 K steps of 128 channels)
template <typename T, int WCO, int FN, bool SEGF, bool X2 = false, bool ODDOK = false>
__device__ __forceinline__ void conv_w1_body(const drnmi_conv_args& p, const W1Seg& sf) {
  using C = W1Cfg<WCO, FN>;
  using K = KT<T>;                                   // bf16 / int8: the same 128-B rows (conv_tile.h)
  using FR = typename K::frag;
  using AC = typename K::acc;
  constexpr int ESZ = K::ESZ, BK = 128 / ESZ, CE = 16 / ESZ, FM = C::FM, BCO = C::BCO;
  constexpr int AB = C::AB, AI = C::AI, TPX = C::TPX, PXW = C::PXW, NSP = C::NSP, SB = C::SB, SPS = C::SPS;
  constexpr int NR = C::NR, RX = C::RX;
  static_assert(!SEGF || WCO == 128, "seg fusion: the 256-channel tile");
  static_assert(!(SEGF && X2), "one epilogue extension at a time");
  static_assert(!X2 || ESZ == 2, "the fused downsample: bf16 nets");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave >> 1;                          // channel half (WCO channels)
  const int wp = wave & 1;                           // pixel half (PXW pixels)
  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const int nco = (p.cout + BCO - 1) / BCO;
  const int ntiles = (M / TPX) * nco;
  const int cin = p.cin;
  const int lc = 31 - __builtin_clz(cin);
  const int H = p.h, W = p.w, dil = p.dil;
  const int nk = 9 * cin / BK;
  const int ngroups = nk / 3;                        // even (bf16: cin % 128 == 0), or ODDOK
  const int fr = lane & 15;
  const int fq = lane >> 4;
  const int lrow = lane >> 3;
  const int lslot = lane & 7;

  const int tile = xcd_remap2(blockIdx.x, ntiles);   // XCD-major deal, as conv_stag
  const int px0 = (tile / nco) * TPX;
  const int co0 = (tile % nco) * BCO;
  const int s_n = px0 / hw_o;
  const int s_q = px0 - s_n * hw_o;
  const int s_oh = s_q / p.wo;
  const int s_ow0 = s_q - s_oh * p.wo;
  const int xbytes = p.n * H * W * cin * ESZ;        // < 2^31 (big_conv_supported / i8_conv_supported)
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.x), 0, xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.wgt), 0, p.cout_pad * p.k_pad * ESZ, 0x00020000);
  typedef __attribute__((address_space(3))) void lds_t;
  auto dma = [&](const __amdgpu_buffer_rsrc_t& rs, uint32_t voff, int soff, int lds_byte) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t*)(smem + lds_byte), 16, voff, soff, 0, 0);
  };
  // weight piece i (rows (wave*AI + i)*8 .. +8, 1 KB) of K step kt; the swizzle depends on i only
  // through its parity (AI even)
  uint32_t a_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave * AI + i) * 8 + lrow;
    a_off[i] = ((co0 + r) * p.k_pad + swzb<128>(r, lslot) * CE) * ESZ;
  }
  constexpr uint32_t kOOB = 0x80000000u;             // beyond every buffer (sizes < 2^31)
  auto issue_a = [&](int kt, int stage, int i) __attribute__((always_inline)) {
    const int cb = kt / 9;
    const int tap = kt - cb * 9;
    const int k0 = (tap << lc) + cb * BK;
    dma(rs_w, a_off[i & 1], ((i & ~1) * 8 * p.k_pad + k0) * ESZ, stage * AB + (wave * AI + i) * 1024);
  };
  // strip share sh of group g (channel block g / 3, tap row g % 3): piece j = wave + 4 sh; past the
  // strip (j >= NSP) it reads nothing into the sink, so every wave issues the same count
  auto issue_strip = [&](int g, int buf, int sh) __attribute__((always_inline)) {
    const int j = wave + 4 * sh;
    const bool inside = j < NSP;
    const int R = j * 8 + lrow;
    const int cb = g / 3, kh = g - cb * 3;
    const int ih = s_oh - p.pad + kh * dil;
    const int iw = s_ow0 - p.pad + R;
    const bool ok = inside && R < TPX + 2 * dil && static_cast<unsigned>(iw) < static_cast<unsigned>(W);
    const bool row_ok = static_cast<unsigned>(ih) < static_cast<unsigned>(H);   // wave-uniform
    const uint32_t voff = ok && row_ok ? static_cast<uint32_t>((iw * cin + (lslot ^ (R & 7)) * CE) * ESZ) : kOOB;
    const int soff = row_ok ? ((s_n * H + ih) * W * cin + cb * BK) * ESZ : 0;
    dma(rs_x, voff, soff, inside ? 2 * AB + buf * SB + j * 1024 : C::SINK);
  };

  // fragment-read byte offsets (the swizzles of a lane group's 16 rows do not depend on the
  // fragment index): A rows wc*WCO + 16 fm + fr, B strip rows wp*PXW + 16 fn + fr + kw*dil
  uint32_t a_base[2], b_base[3][2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = wc * WCO + fr;
    a_base[u] = r * 128 + (swzb<128>(r, u * 4 + fq) << 4);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int R = wp * PXW + fr + kw * dil;
      b_base[kw][u] = 2 * AB + R * 128 + (((u * 4 + fq) ^ (R & 7)) << 4);
    }
  }

  AC acc[FM][FN];
  FR a0[FM], b0[FN], a1[FM], b1[FN];
  // The MFMAs are inline asm with the accumulator as an AGPR operand: the 256 accumulator
  // registers stay in the AGPR file for the whole loop (compiler-selected MFMAs shuffled them
  // between the files and spilled: the 128 fragment VGPRs plus addressing leave no room for a
  // second copy).  Hand-placed waits cover the hazards the compiler cannot see through asm: the
  // accumulators are written by v_accvgpr_write before the first MFMA (s_nop after the init) and
  // read by the epilogue after the last one (s_nop after the loop); consecutive MFMAs on one
  // accumulator are 64 MFMAs apart.
  auto mma = [&](AC& c, const FR& a, const FR& b) __attribute__((always_inline)) {
    if constexpr (ESZ == 2) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  };
  auto rd = [&](FR& dst, uint32_t base, auto off_c) __attribute__((always_inline)) {
    constexpr int OFF = decltype(off_c)::value;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(OFF));
  };
  // read n of a substep's list (b[0..FN) then a[0..FM)) of stage ST / strip buffer BF / tap column KW
  auto rd_item = [&](FR (&a)[FM], FR (&b)[FN], auto n_c, auto st_c, auto bf_c, auto kw_c, auto u_c)
                     __attribute__((always_inline)) {
    constexpr int N = decltype(n_c)::value, ST = decltype(st_c)::value, BF = decltype(bf_c)::value;
    constexpr int KW = decltype(kw_c)::value, U = decltype(u_c)::value;
    if constexpr (N < FN) rd(b[N], b_base[KW][U], std::integral_constant<int, BF * SB + N * 2048>{});
    else rd(a[N - FN], a_base[U], std::integral_constant<int, ST * AB + (N - FN) * 2048>{});
  };

  // accumulator start: bf16, shift (+ residual), as conv_stag's split_init (the dispatch, w1_ok,
  // admits only BN-scale-folded launches with a dense bf16 NHWC output: shift + residual start the
  // accumulators, the epilogue is store_tile_x4), loads before the prologue DMA; int8, zero (the
  // W8A8 epilogue applies scale, shift and residual)
  if constexpr (ESZ == 1) {
#pragma unroll
    for (int i = 0; i < AI; ++i) issue_a(0, 0, i);
#pragma unroll
    for (int sh = 0; sh < C::SH; ++sh) issue_strip(0, 0, sh);
    zero_tile(acc);
  } else {
    uint4 rv[FM / 2][FN];
    float4 shv[FM];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) shv[fm] = *reinterpret_cast<const float4*>(p.shift + co0 + wc * WCO + fm * 16 + fq * 4);
    if (p.res != nullptr) load_residual<FM, WCO, FN>(p, rv, px0, co0, wc, wp, fr, fq);
    // prologue: step 0's weights and group 0's whole strip
#pragma unroll
    for (int i = 0; i < AI; ++i) issue_a(0, 0, i);
#pragma unroll
    for (int sh = 0; sh < C::SH; ++sh) issue_strip(0, 0, sh);
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = f32x4{shv[fm].x, shv[fm].y, shv[fm].z, shv[fm].w};
    if (p.res != nullptr) add_residual(acc, rv, fr);
  }
  // the accumulator starts are in their AGPRs before the wait states below (an empty asm that
  // redefines each one: the compiler cannot sink a v_accvgpr_write past it to just before the
  // first MFMA, whose hazard it cannot see through the asm)
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) asm volatile("" : "+a"(acc[fm][fn]));
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");   // B_0
  __builtin_amdgcn_sched_barrier(0);
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using F = std::false_type;
  using T_ = std::true_type;
  // after B_0: step 0's substep-0 fragments (b0 first), step 1's weights (stage 1), share set 0
  // of group 1's strip (buffer 1)
  static_for<NR>([&](auto n_c) __attribute__((always_inline)) { rd_item(a0, b0, n_c, I0{}, I0{}, I0{}, I0{}); });
#pragma unroll
  for (int i = 0; i < AI; ++i) issue_a(1, 1, i);
#pragma unroll
  for (int sh = 0; sh < SPS; ++sh) issue_strip(1, 1, sh);
  __builtin_amdgcn_sched_barrier(0);

  // K step t = 3 g + KW of strip buffer GP; LAST: the final step (no barrier, reads or DMA after it)
  // one MFMA group: acc[FMI][0..FN) += a[FMI] x b[0..FN), with fill(k) issued in the gap after MFMA
  // k (k < FN - 1): with one wave per SIMD every other instruction of the step must sit in the shadow
  // of an MFMA (a 16-cycle issue gap holds about three), or the matrix pipe idles while it issues
  auto mgroup = [&](auto fm_c, FR (&a)[FM], FR (&b)[FN], auto&& fill) __attribute__((always_inline)) {
    constexpr int FMI = decltype(fm_c)::value;
    static_for<FN>([&](auto k_c) __attribute__((always_inline)) {
      constexpr int K = decltype(k_c)::value;
      mma(acc[FMI][K], a[FMI], b[K]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (K < FN - 1) {
        fill(k_c);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  };
  // A fragment set stays allocated until the end of the phase that consumes it (a use the compiler
  // sees): a read issued in the shadow of an MFMA must never be given the registers of that
  // MFMA's own operands (the compiler would reuse them right after their last asm use, while the
  // MFMA may still be reading them); the new reads take the registers of the previous generation
  auto keep = [&](FR (&a)[FM], FR (&b)[FN]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < FM; ++i) asm volatile("" :: "v"(a[i]));
#pragma unroll
    for (int i = 0; i < FN; ++i) asm volatile("" :: "v"(b[i]));
  };
  // weight-piece offsets of the 4 row pairs (i & ~1) * 8 rows, in SGPRs for the loop
  const int a_row = 16 * p.k_pad * ESZ;              // byte offset of 2 x 8 weight rows

  // K step t = 3 g + KW of strip buffer GP; LAST: the final step (no barrier, reads or DMA after it)
  auto step = [&](auto kw_c, auto gp_c, auto last_c, int g) __attribute__((always_inline)) {
    constexpr int KW = decltype(kw_c)::value;
    constexpr int GP = decltype(gp_c)::value;
    constexpr bool LAST = decltype(last_c)::value;
    constexpr int ST = (GP + KW) & 1;                // stage of step t
    constexpr int KWN = KW == 2 ? 0 : KW + 1;        // step t + 1: tap column, strip buffer
    constexpr int GPN = KW == 2 ? GP ^ 1 : GP;
    constexpr int SGB = KW == 2 ? GP : GP ^ 1;       // buffer of the strip DMA'd after B_{t+1}
    const int t = 3 * g + KW;
    using IST = std::integral_constant<int, ST>;
    using IKW = std::integral_constant<int, KW>;
    using IGP = std::integral_constant<int, GP>;
    auto nofill = [](auto) {};
    // ---- X: substep 0; the substep-1 reads (b1 first) in the first RX gaps of each group
    static_for<FM>([&](auto fm_c) __attribute__((always_inline)) {
      constexpr int FMI = decltype(fm_c)::value;
      // a0[FMI] (b0 already): the reads after it are a0[FMI + 1 ..] and this phase's RX x FMI
      asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(FM - 1 - FMI + RX * FMI) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      mgroup(fm_c, a0, b0, [&](auto k_c) __attribute__((always_inline)) {
        constexpr int KK = decltype(k_c)::value;
        if constexpr (KK < RX) rd_item(a1, b1, std::integral_constant<int, RX * FMI + KK>{}, IST{}, IGP{}, IKW{}, I1{});
      });
    });
    keep(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    // ---- Y: substep 1.  The scalars of the DMA after B_{t+1} (t + 1 = 3 g' + k': step t + 2's
    // weights into stage ST, share set k' of group g' + 1's strip into buffer SGB) are computed in
    // the head groups' gaps and pinned there
    const int gn = KW == 2 ? g + 1 : g;              // g'
    int sa = 0, ss = 0, s_ok = 0;
    auto ygroup_head = [&](auto fm_c) __attribute__((always_inline)) {
      constexpr int FMI = decltype(fm_c)::value;
      asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(FM - 1 - FMI) : "memory");   // a1[FMI] (b1 already)
      __builtin_amdgcn_sched_barrier(0);
      mgroup(fm_c, a1, b1, [&](auto k_c) __attribute__((always_inline)) {
        constexpr int KK = decltype(k_c)::value;
        if constexpr (!LAST && FMI == 0 && KK == (FN >= 8 ? 1 : 0)) {
          const int kt = t + 2 < nk ? t + 2 : nk - 1;   // past the end: re-fetch into the idle stage
          const int cb = kt / 9;
          sa = __builtin_amdgcn_readfirstlane((((kt - cb * 9) << lc) + cb * BK) * ESZ);
          __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (!LAST && FMI == 0 && KK == (FN >= 8 ? 3 : 1)) {
          const int g2 = gn + 1 < ngroups ? gn + 1 : ngroups - 1;   // past the end: a buffer never read again
          const int cb = g2 / 3, kh = g2 - cb * 3;
          const int ih = s_oh - p.pad + kh * dil;
          s_ok = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(ih) < static_cast<unsigned>(H) ? 1 : 0);
          ss = __builtin_amdgcn_readfirstlane(s_ok ? ((s_n * H + ih) * W * cin + cb * BK) * ESZ : 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      });
    };
    static_for<(LAST ? FM : FM / 2)>(ygroup_head);
    if constexpr (LAST) {
      (void)nofill;
    } else {
      // B_{t+1}: step t + 1's weights (issued after B_t, before the strip pieces) must have landed;
      // the SPS strip pieces issued after them are needed only when step t + 1 opens a new tap
      // group (KW == 2), else they may stay in flight (their buffer is not read before B_{3 g' + 3})
      if constexpr (KW == 2) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" :: "n"(SPS) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      using ISTN = std::integral_constant<int, ST ^ 1>;
      using IKWN = std::integral_constant<int, KWN>;
      using IGPN = std::integral_constant<int, GPN>;
      // NI items over the GT gaps of the groups after the barrier: b0[0..FN) alternating with the AI
      // (= FN) weight pieces, then a0[0..FM) with the SPS strip pieces after the first SPS of them;
      // gap G issues items [ceil(G NI / GT), ceil((G + 1) NI / GT))
      auto item = [&](auto n_c) __attribute__((always_inline)) {
        constexpr int N = decltype(n_c)::value;
        if constexpr (N < 2 * FN) {
          if constexpr (N % 2 == 0) {
            rd_item(a0, b0, std::integral_constant<int, N / 2>{}, ISTN{}, IGPN{}, IKWN{}, I0{});
          } else {
            constexpr int I = N / 2;
            dma(rs_w, a_off[I & 1], sa + (I >> 1) * a_row, ST * AB + (wave * AI + I) * 1024);
          }
        } else if constexpr (N < 2 * FN + 2 * SPS) {
          if constexpr (N % 2 == 0) {
            rd_item(a0, b0, std::integral_constant<int, FN + (N - 2 * FN) / 2>{}, ISTN{}, IGPN{}, IKWN{}, I0{});
          } else {
            constexpr int SH = (N - 2 * FN - 1) / 2;       // 0..SPS-1 of the share set
            const int sh = SPS * KWN + SH;
            const int j = wave + 4 * sh;
            // branch-free: a piece past the strip reads nothing and lands in the sink
            const bool inside = j < NSP;
            const int R = j * 8 + lrow;
            const int iw = s_ow0 - p.pad + R;
            const bool ok = inside && s_ok && R < TPX + 2 * dil && static_cast<unsigned>(iw) < static_cast<unsigned>(W);
            const uint32_t voff = ok ? static_cast<uint32_t>((iw * cin + (lslot ^ (R & 7)) * CE) * ESZ) : kOOB;
            dma(rs_x, voff, ss, inside ? 2 * AB + SGB * SB + j * 1024 : C::SINK);
          }
        } else {
          rd_item(a0, b0, std::integral_constant<int, FN + SPS + (N - 2 * FN - 2 * SPS)>{}, ISTN{}, IGPN{}, IKWN{}, I0{});
        }
      };
      static_for<FM - FM / 2>([&](auto q_c) __attribute__((always_inline)) {
        constexpr int FMI = FM / 2 + decltype(q_c)::value;
        mgroup(std::integral_constant<int, FMI>{}, a1, b1, [&](auto k_c) __attribute__((always_inline)) {
          constexpr int G = (FMI - FM / 2) * (FN - 1) + decltype(k_c)::value;
          constexpr int LO = (G * C::NI + C::GT - 1) / C::GT, HI = ((G + 1) * C::NI + C::GT - 1) / C::GT;
          static_for<HI - LO>([&](auto d_c) __attribute__((always_inline)) {
            item(std::integral_constant<int, LO + decltype(d_c)::value>{});
          });
        });
      });
    }
    keep(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto group = [&](auto gp_c, auto lastg_c, int g) __attribute__((always_inline)) {
    step(I0{}, gp_c, F{}, g);
    step(I1{}, gp_c, F{}, g);
    step(I2{}, gp_c, lastg_c, g);
  };
  if (ODDOK && (ngroups & 1)) {
    // odd: pairs, then the last group alone (buffer 0; its clamped strip re-fetches land in
    // buffer 1, which the pair before it finished reading at B_{3 (ngroups - 1)})
    for (int g = 0; g < ngroups - 1; g += 2) {
      group(I0{}, F{}, g);
      group(I1{}, F{}, g + 1);
    }
    group(I0{}, T_{}, ngroups - 1);
  } else {
    for (int g = 0; g < ngroups - 2; g += 2) {
      group(I0{}, F{}, g);
      group(I1{}, F{}, g + 1);
    }
    group(I0{}, F{}, ngroups - 2);
    group(I1{}, T_{}, ngroups - 1);
  }
  if constexpr (X2) {
    // the fused 1x1 downsample (x2 != NULL: D-22 layer4.0 / 5.0 / 6.0 conv2) as cin2 / 64 more K
    // steps after the taps, in conv_stag_x2's order (so the same bits): step e reads weight
    // columns 9 cin + 64 e and, as its B strip, pixel R of the tile sampled at stride2 in x2
    // (strip row R, read at tap column 0).  Not pipelined across steps (2-4 per tile): the other
    // workgroup of the CU (conv_w1h) or the partner waves' MFMAs cover the DMA latency
    const int nx2 = p.cin2 / BK;
    const __amdgpu_buffer_rsrc_t rs_x2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(p.x2), 0, p.n * p.h2 * p.w2 * p.cin2 * ESZ, 0x00020000);
    const int x2_row = (s_n * p.h2 + s_oh * p.stride2) * p.w2 * p.cin2 * ESZ;
    auto issue_x2 = [&](int e, int st) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < AI; ++i)
        dma(rs_w, a_off[i & 1], ((i & ~1) * 8 * p.k_pad + 9 * cin + e * BK) * ESZ, st * AB + (wave * AI + i) * 1024);
#pragma unroll
      for (int sh = 0; sh < C::SH; ++sh) {
        const int j = wave + 4 * sh;
        const bool inside = j < NSP;
        const int R = j * 8 + lrow;
        const uint32_t voff = inside && R < TPX
                                  ? static_cast<uint32_t>(((s_ow0 + R) * p.stride2 * p.cin2 + (lslot ^ (R & 7)) * CE) * ESZ)
                                  : kOOB;
        dma(rs_x2, voff, x2_row + e * BK * ESZ, inside ? 2 * AB + st * SB + j * 1024 : C::SINK);
      }
    };
    // every wave is past the loop's last reads; the clamped re-fetches have landed
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    issue_x2(0, 0);
    for (int e = 0; e < nx2; ++e) {
      const int st = e & 1;
      // step e's pieces have landed everywhere, and every wave is done with step e - 1's buffers
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (e + 1 < nx2) issue_x2(e + 1, st ^ 1);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        FR bx[FN], ax[FM];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) bx[fn] = *reinterpret_cast<const FR*>(smem + b_base[0][u] + st * SB + fn * 2048);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) ax[fm] = *reinterpret_cast<const FR*>(smem + a_base[u] + st * AB + fm * 2048);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) mma(acc[fm][fn], ax[fm], bx[fn]);
      }
    }
  }
  // the last MFMAs' results: wait states, then an empty asm that redefines every accumulator, so
  // no epilogue read of an AGPR can be scheduled before the wait (the compiler had hoisted the
  // read of acc[1][0] to right after its last MFMA, which it does not know is one: that read
  // missed the final K step)
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) asm volatile("" : "+a"(acc[fm][fn]));
  if constexpr (ESZ == 1) {
    if constexpr (SEGF) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // the LDS is free
      w1_seg_i8<FM, FN>(p, acc, px0, co0, wc, wp, fr, fq, lane, sf, smem + AB);
    } else {
      // the dispatch (i8_w1_ok) admits only a dense int8 NHWC output: 16-B pieces
      store_tile_i8_x4<FM, WCO, FN>(p, acc, px0, co0, wc, wp, fr, fq);
    }
  } else if constexpr (!SEGF) {
    store_tile_x4<FM, WCO, FN>(p, acc, px0, co0, wc, wp, fr, fq);
  } else {
    // the activation as store_tile_x4 would store it (ReLU, RNE to bf16, 16-B pieces: lane (fr, fq)
    // holds channels 8 s(fq) .. +7 of 32-channel group f2 of pixel fr) times the matching seg weight
    // columns, the same MFMA order per partial as conv_stag's SEGF: the same partial logits
    bf16x8 aw[2][FM / 2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int f2 = 0; f2 < FM / 2; ++f2)
        aw[mt][f2] = *reinterpret_cast<const bf16x8*>(static_cast<const uint16_t*>(sf.w) +
                                                      static_cast<int64_t>(16 * mt + fr) * sf.k_pad + co0 + wc * WCO +
                                                      32 * f2 + chunk_of_row(fq) * 8);
    const bool relu = p.relu != 0;
    f32x4 pacc[2][FN];
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      pacc[0][fn] = f32x4{0.f, 0.f, 0.f, 0.f};
      pacc[1][fn] = f32x4{0.f, 0.f, 0.f, 0.f};
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
        const bf16x8 b = __builtin_bit_cast(bf16x8, o);
        pacc[0][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[0][f2], b, pacc[0][fn], 0, 0, 0);
        pacc[1][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[1][f2], b, pacc[1][fn], 0, 0, 0);
      }
    }
    // the two channel halves (wc 0 + wc 1) through LDS stage 1 (32 KB): the last steps' clamped
    // re-fetches target stage 0 and strip buffer 0 (nk and the group count are even), and every
    // wave is past its last fragment read after the barrier
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float4* xch = reinterpret_cast<float4*>(smem + AB) + (wp * 64 + lane) * (2 * FN);
    if (wc == 1) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          xch[mt * FN + fn] = make_float4(pacc[mt][fn][0], pacc[mt][fn][1], pacc[mt][fn][2], pacc[mt][fn][3]);
    }
    __syncthreads();
    if (wc == 0) {
      float* __restrict__ part = static_cast<float*>(sf.part) + static_cast<int64_t>(co0 / BCO) * M * kW1SegCS;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int cls = 16 * mt + 4 * fq;
        if (cls >= kW1SegCS) continue;
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const float4 o = xch[mt * FN + fn];
          const int64_t m = px0 + wp * PXW + fn * 16 + fr;
          *reinterpret_cast<float4*>(part + m * kW1SegCS + cls) =
              make_float4(pacc[mt][fn][0] + o.x, pacc[mt][fn][1] + o.y, pacc[mt][fn][2] + o.z, pacc[mt][fn][3] + o.w);
        }
      }
    }
  }
}

using W1 = W1Cfg<128, 8>;
using W1H = W1Cfg<64, 4>;

__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
conv_w1_kernel(const drnmi_conv_args p) {
  conv_w1_body<uint16_t, 128, 8, false>(p, W1Seg{nullptr, 0, nullptr});
}

// the 128 x 128 tile (D-22 layer4, 128 -> 128 at K = 1152: 18 K steps per tile); two workgroups per
// CU, so one tile's prologue strip and epilogue overlap the other's MFMAs
__global__ void __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv_w1h_kernel(const drnmi_conv_args p) {
  conv_w1_body<uint16_t, 64, 4, false>(p, W1Seg{nullptr, 0, nullptr});
}

// + the fused 1x1 downsample (x2 != NULL)
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
conv_w1_x2_kernel(const drnmi_conv_args p) {
  conv_w1_body<uint16_t, 128, 8, false, true>(p, W1Seg{nullptr, 0, nullptr});
}
__global__ void __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv_w1h_x2_kernel(const drnmi_conv_args p) {
  conv_w1_body<uint16_t, 64, 4, false, true>(p, W1Seg{nullptr, 0, nullptr});
}

struct W1SegArgs {
  drnmi_conv_args p;
  W1Seg sf;
};
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
conv_w1_seg_kernel(const W1SegArgs a) {
  conv_w1_body<uint16_t, 128, 8, true>(a.p, a.sf);
}

// W8A8 (config C5): int8 rows of 128 channels are the bf16 tile's 128-B rows; v_mfma_i32_16x16x64_i8,
// the W8A8 epilogue (bit-exact against oracle/int8_oracle.py like conv_i8_stag_kernel)
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
conv_w1_i8_kernel(const drnmi_conv_args p) {
  conv_w1_body<int8_t, 128, 8, false>(p, W1Seg{nullptr, 0, nullptr});
}
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
conv_w1_i8_seg_kernel(const W1SegArgs a) {
  conv_w1_body<int8_t, 128, 8, true>(a.p, a.sf);
}
// the int8 128 x 128 tile (D-22 layer4.1 in int8 nets: cin 128 = 9 K steps, an odd tap-group count)
__global__ void __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv_w1h_i8_kernel(const drnmi_conv_args p) {
  conv_w1_body<int8_t, 64, 4, false, false, true>(p, W1Seg{nullptr, 0, nullptr});
}

}  // namespace

static hipError_t w1_attrs() {
  static bool attr_set = false;
  if (!attr_set) {
    for (const void* f : {reinterpret_cast<const void*>(&conv_w1_kernel), reinterpret_cast<const void*>(&conv_w1_seg_kernel),
                          reinterpret_cast<const void*>(&conv_w1_i8_kernel), reinterpret_cast<const void*>(&conv_w1_i8_seg_kernel)}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, W1::LDS);
      if (e != hipSuccess) return e;
    }
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_w1_x2_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, W1::LDS);
    if (e != hipSuccess) return e;
    for (const void* f : {reinterpret_cast<const void*>(&conv_w1h_kernel), reinterpret_cast<const void*>(&conv_w1h_x2_kernel),
                          reinterpret_cast<const void*>(&conv_w1h_i8_kernel)}) {
      const hipError_t e2 = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, W1H::LDS);
      if (e2 != hipSuccess) return e2;
    }
    attr_set = true;
  }
  return hipSuccess;
}

hipError_t launch_w1_seg(const drnmi_conv_args& p, const void* seg_w, int seg_k_pad, void* part, hipStream_t s) {
  const hipError_t e = w1_attrs();
  if (e != hipSuccess) return e;
  W1SegArgs a;
  a.p = p;
  a.sf = W1Seg{seg_w, seg_k_pad, part};
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const dim3 grid(static_cast<unsigned>((M / W1::TPX) * ((p.cout + 255) / 256)));
  if (p.dtype == DRNMI_I8) hipLaunchKernelGGL(conv_w1_i8_seg_kernel, grid, dim3(256), W1::LDS, s, a);
  else hipLaunchKernelGGL(conv_w1_seg_kernel, grid, dim3(256), W1::LDS, s, a);
  return hipGetLastError();
}

hipError_t launch_w1(const drnmi_conv_args& p, hipStream_t s) {
  const hipError_t e0 = w1_attrs();
  if (e0 != hipSuccess) return e0;
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const dim3 grid(static_cast<unsigned>((M / W1::TPX) * ((p.cout + 255) / 256)));
  if (p.dtype == DRNMI_I8) hipLaunchKernelGGL(conv_w1_i8_kernel, grid, dim3(256), W1::LDS, s, p);
  else if (p.x2 != nullptr) hipLaunchKernelGGL(conv_w1_x2_kernel, grid, dim3(256), W1::LDS, s, p);
  else hipLaunchKernelGGL(conv_w1_kernel, grid, dim3(256), W1::LDS, s, p);
  return hipGetLastError();
}

hipError_t launch_w1h(const drnmi_conv_args& p, hipStream_t s) {
  const hipError_t e0 = w1_attrs();
  if (e0 != hipSuccess) return e0;
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const dim3 grid(static_cast<unsigned>((M / W1H::TPX) * ((p.cout + 127) / 128)));
  if (p.dtype == DRNMI_I8) hipLaunchKernelGGL(conv_w1h_i8_kernel, grid, dim3(256), W1H::LDS, s, p);
  else if (p.x2 != nullptr) hipLaunchKernelGGL(conv_w1h_x2_kernel, grid, dim3(256), W1H::LDS, s, p);
  else hipLaunchKernelGGL(conv_w1h_kernel, grid, dim3(256), W1H::LDS, s, p);
  return hipGetLastError();
}

}  // namespace drnmi
