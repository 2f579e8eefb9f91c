// Large-channel NHWC implicit-GEMM convolution, bf16, LDS-DMA staged (the MFMA-bound layers).
//
// Serves every bf16 conv of DRN-D with cin >= 32 and ks 1/3: layer3..layer8 3x3 convs
// (dilation 1/2/4, lmodels/drn.py:27-29, :49-65, :201-211), the 1x1 stride-s downsamples
// (:181-186), the Bottleneck convs (:86-106) and the seg 1x1 + bias (lmodels/drnseg.py:278-284).
// In D-22 at 1024x2048 layer5..8 hold ~85 % of the FLOPs at arithmetic intensity
// 750..2150 FLOP/B: MFMA-bound.
//
// Structure (one output tile = BCO channels x 256 pixels per workgroup):
//   * MFMA v_mfma_f32_16x16x32_bf16 with A = weights (rows = output channels), B = pixels,
//     so the accumulator hands each lane 4 consecutive channels of one pixel (8-byte NHWC
//     stores and residual loads).
//   * K step BK (64, or 32 when cin == 32) = one kernel tap x BK input channels.  Both
//     operand tiles go global -> LDS with global_load_lds_dwordx4 (LDS-DMA: no VGPR round
//     trip, no ds_write issue).  Each pixel row of the B tile is gathered from its own NHWC
//     address -- the implicit-GEMM im2col happens in the DMA source addresses; out-of-image
//     taps read a zero page, which is the conv's zero padding.
//   * NST-stage LDS ring, counted vmcnt + raw s_barrier once per step (a __syncthreads()
//     would drain every DMA in flight).
//   * LDS rows are BK*2 bytes; 16-B chunk c of row r sits at slot c ^ f(r) (applied on the
//     DMA source address because the DMA destination is lane-linear, and on the fragment
//     read): the 16x16x32 fragment reads are bank-conflict free (SQ_LDS_BANK_CONFLICT = 0).
//   * Fragment reads run one MFMA group ahead, and the next step's DMA is issued piece by
//     piece between the MFMA groups of the first substep, so DMA issue cost and LDS latency
//     hide under MFMAs (measured +7..10 % over issuing the DMA as one block).
//   * Each wave owns WCO channels x 64 pixels (WCO/16 x 4 fragments).
//   * Tiles are dealt XCD-major (bijective remap) so the channel tiles of a pixel tile and
//     neighbouring pixel rows share an XCD's L2.
//   * PERSIST: one workgroup per CU walks its tiles; the next tile's first DMA steps are
//     issued before the current tile's epilogue, hiding the pipeline fill and the
//     epilogue (a ~10 us fixed cost per tile otherwise).
#include "common.h"
#include "conv_tile.h"
#include "kernels.h"

// The main-loop schedule is pinned: fragment reads for group q+1 go out before group q's MFMAs
// (sched_barrier between groups) and the next step's DMA pieces are issued without a branch (the
// last steps re-fetch a clamped step into the idle stage).  Without the pins the compiler sinks
// each read next to its MFMAs and waits lgkmcnt(0) on it (no LDS latency hiding).

namespace drnmi {
namespace {


template <typename T, int KS, int WCO, int WC, int NST, int BK, bool PERSIST, int NWP, bool SPARSE, bool X2 = false,
          bool STRIP = false>
__device__ __forceinline__ void conv_big_body(const drnmi_conv_args& p) {
  using K = KT<T>;
  using C = BigCfg<WCO, WC, NST, BK, NWP, K::ESZ>;
  static_assert(!SPARSE || K::ESZ == 2, "unit skipping: bf16 only");
  static_assert(!STRIP || (KS == 3 && NST == 2 && C::ROWB == 128 && !PERSIST && !SPARSE && !X2 && C::NW == 8),
                "strip mode: the 256 x 256 3x3 instantiations with 128-B rows (bf16 BK 64, int8 BK 128)");
  constexpr int CE = 16 / K::ESZ;   // elements per 16-B chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wc = wave / NWP;        // channel column of the tile
  const int wp = wave % NWP;        // PXW-pixel slice of the tile
  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const int nco = (p.cout + C::BCO - 1) / C::BCO;
  const int npx = (M + kBPX - 1) / kBPX;
  const int ntiles = npx * nco;

  const int cin = p.cin;
  const int lc = 31 - __builtin_clz(cin);
  const int H = p.h, W = p.w, dil = p.dil;
  const T* __restrict__ x = reinterpret_cast<const T*>(p.x);
  const T* __restrict__ wt = reinterpret_cast<const T*>(p.wgt);
  const int nk = p.k_pad / BK;
  // fused second input (x2 != NULL: the block's 1x1 downsample folded into this conv, the
  // concatenated-K GEMM [W | W_ds] x [im2col(x) ; x2 sampled at stride2]): the last
  // cin2 / BK K steps read x2 instead of a tap of x
  const T* __restrict__ x2 = reinterpret_cast<const T*>(p.x2);
  const int nk1 = X2 ? (KS * KS * cin) / BK : nk;
  const int fr = lane & 15;       // fragment row (channel or pixel within a 16-block)
  const int fq = lane >> 4;       // 16-B k chunk within a 64-B substep

  // --- DMA assignment.  One wave instruction fills RPI LDS rows (1 KB); lane l fills row
  // RPI*j + l / CPR, slot l % CPR.  Wave w fills A instructions [w*A_INSTR, ...) (weights)
  // and B instructions [w*B_INSTR, ...) (pixels).
  const int lrow = lane / C::CPR;
  const int lslot = lane % C::CPR;
  // weight rows: the swizzle of row (wave*A_INSTR + i)*RPI + lrow depends on i only through its
  // parity, so two offsets + a scalar i*RPI*k_pad cover every piece
  int a_par[2];
  // pixel row i: (ih0, iw0) of tap (0,0) packed as two int16 (ih0 = -16384: no pixel) and the
  // int32 element offset of that tap's chunk (only dereferenced when the tap is inside the
  // image; big_conv_supported / i8_conv_supported bound n*h*w*cin < 2^31 and h, w < 16384)
  uint32_t b_hw[C::B_INSTR];
  int b_off[C::B_INSTR];
  int b2_off[X2 ? C::B_INSTR : 1];   // x2 element offset of the row's chunk (x2 steps)
  const char* zero_src = reinterpret_cast<const char*>(g_zero_page) + lane * 16;
  int s_n = 0, s_oh = 0, s_ow0 = 0;   // STRIP: the tile's image, output row and first column

  auto setup = [&](int px0, int co0) {
    if constexpr (STRIP) {
      s_n = px0 / hw_o;
      const int q = px0 - s_n * hw_o;
      s_oh = q / p.wo;
      s_ow0 = q - s_oh * p.wo;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (wave * C::A_INSTR + i) * C::RPI + lrow;
      a_par[i] = (co0 + r) * p.k_pad + swzb<C::ROWB>(r, lslot) * CE - i * C::RPI * p.k_pad;
    }
    // pixel rows: (ih0, iw0) of tap (0,0) and a base pointer at that tap's chunk (only
    // dereferenced when the tap lies inside the image)
#pragma unroll
    for (int i = 0; i < C::B_INSTR; ++i) {
      const int r = (wave * C::B_INSTR + i) * C::RPI + lrow;
      const int m = px0 + r;
      b_hw[i] = 0xC000C000u;
      b_off[i] = 0;
      if constexpr (X2) b2_off[i] = -1;
      if (m < M) {
        const int n = m / hw_o;
        const int q = m - n * hw_o;
        const int oh = q / p.wo;
        const int ow = q - oh * p.wo;
        const int ih0 = oh * p.stride - p.pad;
        const int iw0 = ow * p.stride - p.pad;
        b_hw[i] = (static_cast<uint32_t>(ih0) << 16) | (static_cast<uint32_t>(iw0) & 0xffffu);
        b_off[i] = ((n * H + ih0) * W + iw0) * cin + swzb<C::ROWB>(r, lslot) * CE;
        if constexpr (X2)
          b2_off[i] = ((n * p.h2 + oh * p.stride2) * p.w2 + ow * p.stride2) * p.cin2 + swzb<C::ROWB>(r, lslot) * CE;
      }
    }
  };

  // K step kt = (channel block cb, tap): taps innermost, so the KS*KS steps that re-read one
  // channel slice of the same pixel neighbourhood run back to back (L2 hits, not MALL).
  struct StepP { int k0, dh, dw; int64_t toff; bool second; };
  auto step_params = [&](int kt) {
    StepP sp;
    sp.second = X2 && kt >= nk1;
    if (sp.second) {                               // x2 step: channels (kt - nk1) * BK of x2
      sp.k0 = KS * KS * cin + (kt - nk1) * BK;
      sp.dh = sp.dw = 0;
      sp.toff = (kt - nk1) * BK;
      return sp;
    }
    const int cb = kt / (KS * KS);
    const int tap = kt - cb * (KS * KS);
    sp.k0 = (tap << lc) + cb * BK;                 // packed weight column: tap * cin + channel
    sp.dh = (tap / KS) * dil;
    sp.dw = (tap - (tap / KS) * KS) * dil;
    sp.toff = (static_cast<int64_t>(sp.dh) * W + sp.dw) * cin + cb * BK;   // uniform over rows
    return sp;
  };
  // one DMA instruction ("piece") of a step: pieces [0, A_INSTR) weights, then pixel rows
  auto issue_piece = [&](const StepP& sp, int stage, int i) {
    if constexpr (STRIP) {                         // A only: B comes as strips
      if (i < C::A_INSTR)
        glds16(wt + (a_par[i & 1] + i * C::RPI * p.k_pad + sp.k0), smem + stage * C::A_BYTES + (wave * C::A_INSTR + i) * 1024);
      return;
    }
    char* sa = smem + stage * C::STAGE;
    if (i < C::A_INSTR) {
      glds16(wt + (a_par[i & 1] + i * C::RPI * p.k_pad + sp.k0), sa + (wave * C::A_INSTR + i) * 1024);
    } else {
      const int j = i - C::A_INSTR;
      const int ih0 = static_cast<int>(b_hw[j]) >> 16;
      const int iw0 = static_cast<int16_t>(b_hw[j] & 0xffffu);
      const bool ok = static_cast<unsigned>(ih0 + sp.dh) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(iw0 + sp.dw) < static_cast<unsigned>(W);
      const void* src = ok ? static_cast<const void*>(x + (b_off[j] + sp.toff)) : static_cast<const void*>(zero_src);
      if constexpr (X2)
        if (sp.second)
          src = b2_off[j] >= 0 ? static_cast<const void*>(x2 + (b2_off[j] + sp.toff)) : static_cast<const void*>(zero_src);
      glds16(src, sa + C::A_BYTES + (wave * C::B_INSTR + j) * 1024);
    }
  };
  auto issue = [&](int kt, int stage) {
    const StepP sp = step_params(kt);
#pragma unroll
    for (int i = 0; i < C::GLDS; ++i) issue_piece(sp, stage, i);
  };
  // STRIP: share sh (0..4) of the strip of group g = K steps 3g..3g+2 (channel block g / 3, tap
  // row kh = g % 3): strip row R = input pixel (oh - pad + kh dil, ow0 - pad + R), 16-B chunk c
  // at slot c ^ (R & 7) (conflict-free for the 16 consecutive rows of a fragment read at any
  // kw*dil offset)
  const int ngroups = nk / 3;
  auto issue_strip = [&](int g, int sh) {
    const int j = wave + 8 * sh;
    if (j >= kStripPieces) return;                 // wave-uniform
    const int R = j * 8 + lrow;
    const int cb = g / 3, kh = g - cb * 3;
    const int ih = s_oh - p.pad + kh * dil;
    const int iw = s_ow0 - p.pad + R;
    const bool ok = R < kBPX + 2 * dil && static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                    static_cast<unsigned>(iw) < static_cast<unsigned>(W);
    const void* src = ok ? static_cast<const void*>(x + ((static_cast<int64_t>(s_n) * H + ih) * W + iw) * cin + cb * BK +
                                                    (lslot ^ (R & 7)) * CE)
                         : static_cast<const void*>(zero_src);
    glds16(src, smem + NST * C::A_BYTES + (g & 1) * kStripBytes + j * 1024);
  };


  typename K::acc acc[C::FM][C::FN];
  int tl = blockIdx.x;
  int tile = xcd_remap2(tl, ntiles);
  int px0 = (tile / nco) * kBPX;
  int co0 = (tile % nco) * C::BCO;
  setup(px0, co0);
  // SPARSE: K-step compaction.  A K step whose weight slice (all BCO rows of this tile x BK
  // packed columns) is zero -- a pruned block covering the tile's rows, BlockPruner.py:139-241 --
  // is dropped entirely: no weight DMA, no pixel-row gather, no MFMA.  Lane q holds the K-step
  // id of live position q (lst0) and q + 64 (lst1), built once per tile from two ballots; a
  // position's step is then a readlane (positions are wave-uniform).  nk <= 128 (dispatch).
  int nlive = nk;
  int lst0 = lane, lst1 = lane + 64;
  if constexpr (SPARSE) {
    const int wpr = (p.k_pad + 1023) >> 10;
    auto step_live = [&](int kt) -> bool {
      if (kt >= nk) return false;
      const int u0 = step_params(kt).k0 >> 5;
      bool any = false;
      for (int rb = co0 >> 4; rb < (co0 + C::BCO) >> 4; ++rb)
        any |= ((p.unit_mask[rb * wpr + (u0 >> 5)] >> (u0 & 31)) & ((1u << C::SUB) - 1)) != 0;
      return any;
    };
    const uint64_t b0 = __ballot(step_live(lane)), b1 = __ballot(step_live(lane + 64));
    const int c0 = __popcll(b0), c1 = __popcll(b1);
    nlive = __builtin_amdgcn_readfirstlane(c0 + c1);   // wave-uniform trip count (scalar loop)
    // position q -> K step: the q-th live step of b0, then of b1
    const int q1 = 64 + lane - c0;                       // b1 index of position 64 + lane
    lst0 = lane < c0 ? nth_set_bit(b0, lane) : (lane - c0 < c1 ? 64 + nth_set_bit(b1, lane - c0) : 0);
    lst1 = q1 < c1 ? 64 + nth_set_bit(b1, q1) : 0;
  }
  auto kt_at = [&](int pos) -> int {
    if constexpr (!SPARSE) return pos;
    return pos < 64 ? __builtin_amdgcn_readlane(lst0, pos) : __builtin_amdgcn_readlane(lst1, pos - 64);
  };
  constexpr bool DEFER = NWP < 4;
  if constexpr (K::ESZ == 2) init_tile<C::FM, WCO, C::FN, DEFER>(p, acc, px0, co0, wc, wp, fr, fq);   // residual loads ahead of the DMA
  else zero_tile(acc);
  for (int t = 0; t < NST - 1 && t < nlive; ++t) issue(kt_at(t), t);
  if constexpr (STRIP) {
#pragma unroll
    for (int sh = 0; sh < 5; ++sh) issue_strip(0, sh);
  }

  while (true) {
    // t runs over the (live) K-step positions; kt_at(t) is the K step itself
    for (int t = 0; t < nlive; ++t) {
      const int cur = t % NST;
      // retire step t: the steps issued after it (min(nlive-1, t+NST-2) - t) may stay in flight
      const int newer = ((nlive - 1) < (t + NST - 2) ? (nlive - 1) : (t + NST - 2)) - t;
      if (NST >= 4 && newer >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * C::GLDS) : "memory");
      else if (NST >= 3 && newer >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::GLDS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);

      const char* sa = smem + cur * (STRIP ? C::A_BYTES : C::STAGE);
      const char* sb = STRIP ? smem + NST * C::A_BYTES + ((t / 3) & 1) * kStripBytes : sa + C::A_BYTES;
      const int kwd = STRIP ? (t % 3) * dil : 0;   // STRIP: strip row offset of this step's tap
      // STRIP: this step also issues shares 2 (t % 3), +1 of the next group's strip (clamped: the
      // last group re-fetches its own strip, identical bytes, into the buffer being read)
      const int sg = (t / 3 + 1 < ngroups) ? t / 3 + 1 : ngroups - 1;
      constexpr int GL = STRIP ? C::A_INSTR + 2 : C::GLDS;
      constexpr int NG = C::SUB * C::GR;
      constexpr int PPG = (GL + C::GR - 1) / C::GR;   // DMA pieces per group (first substep)
      const StepP sp = step_params(kt_at(t + NST - 1 < nlive ? t + NST - 1 : nlive - 1));
      const int nst = (t + NST - 1) % NST;
      constexpr int PFD = 1;                     // fragment prefetch distance in MFMA groups
      constexpr int NAF = PFD + 1;               // A-fragment ring depth
      typename K::frag af[NAF][C::FPG], bfr[2][C::FN];
      auto load_a = [&](typename K::frag (&dst)[C::FPG], int q) {
        const int c = (q / C::GR) * 4 + fq;
#pragma unroll
        for (int h = 0; h < C::FPG; ++h) {
          const int r = wc * WCO + ((q % C::GR) * C::FPG + h) * 16 + fr;
          // unconditional: a branch around an LDS read makes the compiler fall back to lgkmcnt(0)
          dst[h] = *reinterpret_cast<const typename K::frag*>(sa + r * C::ROWB + swzb<C::ROWB>(r, c) * 16);
        }
      };
      auto load_b = [&](typename K::frag (&dst)[C::FN], int sub) {
        const int c = sub * 4 + fq;
#pragma unroll
        for (int fn = 0; fn < C::FN; ++fn) {
          const int r = wp * C::PXW + fn * 16 + fr;
          if constexpr (STRIP) {
            const int R = r + kwd;
            dst[fn] = *reinterpret_cast<const typename K::frag*>(sb + R * C::ROWB + (c ^ (R & 7)) * 16);
          } else {
            dst[fn] = *reinterpret_cast<const typename K::frag*>(sb + r * C::ROWB + swzb<C::ROWB>(r, c) * 16);
          }
        }
      };
      load_b(bfr[0], 0);
#pragma unroll
      for (int q = 0; q < PFD && q < NG; ++q) {
        load_a(af[q % NAF], q);
        if (q > 0 && q % C::GR == 0) load_b(bfr[(q / C::GR) & 1], q / C::GR);
      }
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        // group q's fragments (issued a group ago) land before the next reads go out, so the
        // compiler's wait in front of the MFMAs does not also cover the fresh reads
        // (s_waitcnt lgkmcnt(0) with vmcnt/expcnt at their maxima: LDS-DMA stays in flight)
        if (q + PFD < NG) {
          load_a(af[(q + PFD) % NAF], q + PFD);
          if ((q + PFD) % C::GR == 0) load_b(bfr[((q + PFD) / C::GR) & 1], (q + PFD) / C::GR);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < C::FPG; ++h) {
#pragma unroll
          for (int fn = 0; fn < C::FN; ++fn)
            acc[(q % C::GR) * C::FPG + h][fn] = K::mma(
                af[q % NAF][h], bfr[(q / C::GR) & 1][fn], acc[(q % C::GR) * C::FPG + h][fn]);
        }
        if (q < C::GR) {
#pragma unroll
          for (int k = 0; k < PPG; ++k)
            if constexpr (STRIP) {
              const int i = q * PPG + k;
              if (i < C::A_INSTR) issue_piece(sp, nst, i);
              else if (i < GL) issue_strip(sg, 2 * (t % 3) + (i - C::A_INSTR));
            } else {
              if (q * PPG + k < C::GLDS) issue_piece(sp, nst, q * PPG + k);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // --- next tile: its first DMA steps go out before this tile's epilogue
    const int cur_px0 = px0, cur_co0 = co0;
    bool more = false;
    if constexpr (PERSIST) {
      tl += gridDim.x;
      more = tl < ntiles;
      if (more) {
        tile = xcd_remap2(tl, ntiles);
        px0 = (tile / nco) * kBPX;
        co0 = (tile % nco) * C::BCO;
        // every wave done with the ring, and the clamped re-fetches have landed
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        setup(px0, co0);
        for (int t = 0; t < NST - 1 && t < nk; ++t) issue(t, t);
      }
    }

    if constexpr (K::ESZ == 2) {
      // whole tile inside a dense bf16 NHWC output: 16-B stores (conv_tile.h store_tile_x4)
      bool x4 = false;
      if constexpr (!DEFER && C::FM % 2 == 0)
        x4 = p.scale == nullptr && p.out_dtype == DRNMI_BF16 && p.y_sc == 1 && p.y_sp == p.cout &&
             p.y_sn == static_cast<int64_t>(p.ho) * p.wo * p.cout && cur_px0 + kBPX <= p.n * p.ho * p.wo &&
             cur_co0 + C::BCO <= p.cout;
      if (x4) store_tile_x4<C::FM, WCO, C::FN>(p, acc, cur_px0, cur_co0, wc, wp, fr, fq);
      else store_tile<C::FM, WCO, C::FN, DEFER>(p, acc, cur_px0, cur_co0, wc, wp, fr, fq);
    } else {
      bool x4 = false;
      if constexpr (C::FM % 4 == 0)
        x4 = p.out_dtype == DRNMI_I8 && p.y_sc == 1 && p.y_sp == p.cout &&
             p.y_sn == static_cast<int64_t>(p.ho) * p.wo * p.cout && cur_px0 + kBPX <= p.n * p.ho * p.wo &&
             cur_co0 + C::BCO <= p.cout && (p.res == nullptr || p.cout % 16 == 0);
      if (x4) store_tile_i8_x4<C::FM, WCO, C::FN>(p, acc, cur_px0, cur_co0, wc, wp, fr, fq);
      else store_tile_i8<C::FM, WCO, C::FN>(p, acc, cur_px0, cur_co0, wc, wp, fr, fq);
    }
    if (!more) break;
    if constexpr (K::ESZ == 2) init_tile<C::FM, WCO, C::FN, DEFER>(p, acc, px0, co0, wc, wp, fr, fq);
    else zero_tile(acc);
  }
}

template <int KS, int WCO, int WC, int NST, int BK, bool PERSIST, int NWP, bool SPARSE, bool X2 = false>
__global__ void __launch_bounds__(64 * NWP * WC, 1)
conv_big_kernel(const drnmi_conv_args p) {
  conv_big_body<uint16_t, KS, WCO, WC, NST, BK, PERSIST, NWP, SPARSE, X2>(p);
}

// Strip-staged B operand (see conv_big_body STRIP): the 256 x 256 3x3 tile for wo % 256 == 0.
__global__ void __launch_bounds__(512, 1)
conv_strip_kernel(const drnmi_conv_args p) {
  conv_big_body<uint16_t, 3, 128, 2, 2, 64, false, 4, false, false, true>(p);
}

// int8 strip-staged B: conv_i8_kernel<3, 128, 2, 2, 128> with the STRIP B path (int8 rows of 128
// channels are 128 B, the bf16 layout): same MFMA order, bit-identical to the per-tap gather.
__global__ void __launch_bounds__(512, 1)
conv_i8_strip_kernel(const drnmi_conv_args p) {
  conv_big_body<int8_t, 3, 128, 2, 2, 128, false, 4, false, false, true>(p);
}

// W8A8 (config C5): the same LDS-DMA pipeline over int8 elements, BK int8 channels per K step
// (128-B LDS rows for cin >= 128, 64-B rows for cin == 64), v_mfma_i32_16x16x64_i8 into int32
// accumulators, store_tile_i8 epilogue.
template <int KS, int WCO, int WC, int NST, int BK>
__global__ void __launch_bounds__(64 * 4 * WC, 1)
conv_i8_kernel(const drnmi_conv_args p) {
  conv_big_body<int8_t, KS, WCO, WC, NST, BK, false, 4, false>(p);
}

// the same body at two workgroups per CU (register budget 256, 2 x 24 KB of LDS with 64-B rows):
// the 1x1 launches have 1-2 K steps per tile, so one resident tile per CU leaves its loads and
// stores serialised tile after tile; a second tile overlaps them
template <int KS, int WCO, int WC, int NST, int BK>
__global__ void __launch_bounds__(64 * 4 * WC, 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv_i8_occ2_kernel(const drnmi_conv_args p) {
  conv_big_body<int8_t, KS, WCO, WC, NST, BK, false, 4, false>(p);
}

// --- Ping-pong 256 x 256 schedule (variant "pp256").
//
// Same tile, LDS image and fragment layout as conv_big_kernel<KS, 128, 2, 2, 64>, but each
// 64-deep K step runs as 4 phases, one per quadrant of the wave's 128 x 64 output block
// (16 MFMAs each), and every phase is {load segment} s_barrier {MFMA segment} s_barrier.
// The two waves of a SIMD (w and w + 4: the two channel halves wc) run one barrier apart,
// so on every SIMD one wave issues its LDS fragment reads and DMA pieces while the other
// one runs its MFMA cluster (cdna_hip_programming.md "256^2 8-phase template", T3-T5).
// The stage is split in halves that free up at different phases: the first half (channel
// rows 0-63 of each wc block, pixel rows 0-31 of each 64-pixel block) is read in phase 0,
// the second half in phases 1-2.  Pieces in flight: phases 0-1 of step s stage the second
// half of step s+1, phases 2-3 the first half of step s+2, so every piece has >= 6
// segments to land, with counted vmcnt waits (never 0 in steady state).
template <int KS>
__global__ void __launch_bounds__(512, 1)
conv_pp_kernel(const drnmi_conv_args p) {
  constexpr int BK = 64, ROWB = 128, A_BYTES = 256 * ROWB, STAGE = 2 * A_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar branches)
  const int wc = wave >> 2;
  const int wp = wave & 3;
  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const int nco = p.cout / 256;
  const int npx = (M + kBPX - 1) / kBPX;
  const int ntiles = npx * nco;
  const int tile = xcd_remap2(blockIdx.x, ntiles);
  const int px0 = (tile / nco) * kBPX;
  const int co0 = (tile % nco) * 256;

  const int cin = p.cin;
  const int lc = 31 - __builtin_clz(cin);
  const int H = p.h, W = p.w, dil = p.dil;
  const uint16_t* __restrict__ x = reinterpret_cast<const uint16_t*>(p.x);
  const uint16_t* __restrict__ wt = reinterpret_cast<const uint16_t*>(p.wgt);
  const int nk = p.k_pad / BK;
  const int fr = lane & 15;
  const int fq = lane >> 4;

  // DMA pieces: half h, slot j: weight rows ((2w+j)/8)*128 + h*64 + ((2w+j)%8)*8 .. +8 and
  // pixel rows ((2w+j)/4)*64 + h*32 + ((2w+j)%4)*8 .. +8 (lane -> row + lane/8, chunk lane%8)
  const int lrow = lane >> 3;
  const int lslot = lane & 7;
  int a_off[2][2], a_row0[2][2], b_row0[2][2], b_ih0[2][2], b_iw0[2][2];
  const uint16_t* b_base[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = 2 * wave + j;
      a_row0[h][j] = (q >> 3) * 128 + h * 64 + (q & 7) * 8;
      const int ra = a_row0[h][j] + lrow;
      a_off[h][j] = (co0 + ra) * p.k_pad + swz<BK>(ra, lslot) * 8;
      b_row0[h][j] = (q >> 2) * 64 + h * 32 + (q & 3) * 8;
      const int rb = b_row0[h][j] + lrow;
      const int m = px0 + rb;
      b_ih0[h][j] = -(1 << 28);
      b_iw0[h][j] = -(1 << 28);
      b_base[h][j] = x;
      if (m < M) {
        const int n = m / hw_o;
        const int qq = m - n * hw_o;
        const int oh = qq / p.wo;
        const int ow = qq - oh * p.wo;
        b_ih0[h][j] = oh * p.stride - p.pad;
        b_iw0[h][j] = ow * p.stride - p.pad;
        b_base[h][j] = x + ((static_cast<int64_t>(n) * H + b_ih0[h][j]) * W + b_iw0[h][j]) * cin +
                       swz<BK>(rb, lslot) * 8;
      }
    }
  const char* zero_src = reinterpret_cast<const char*>(g_zero_page) + lane * 16;

  // stage pieces (h, j) of K step kt (one weight piece + one pixel piece)
  auto issue = [&](int kt, int h, int j) {
    const int cb = kt / (KS * KS);                 // channel block outer, tap inner (as conv_big)
    const int tap = kt - cb * (KS * KS);
    const int k0 = (tap << lc) + cb * BK;
    const int dh = (tap / KS) * dil;
    const int dw = (tap - (tap / KS) * KS) * dil;
    const int64_t toff = (static_cast<int64_t>(dh) * W + dw) * cin + cb * BK;
    char* sa = smem + (kt & 1) * STAGE;
    glds16(wt + a_off[h][j] + k0, sa + a_row0[h][j] * ROWB);
    const bool ok = static_cast<unsigned>(b_ih0[h][j] + dh) < static_cast<unsigned>(H) &&
                    static_cast<unsigned>(b_iw0[h][j] + dw) < static_cast<unsigned>(W);
    const void* src = ok ? static_cast<const void*>(b_base[h][j] + toff) : static_cast<const void*>(zero_src);
    glds16(src, sa + A_BYTES + b_row0[h][j] * ROWB);
  };
  auto barrier = [&]() {
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // fragments: channel half hh (4 fragments x 2 substeps), pixel half g (2 x 2)
  auto load_a = [&](bf16x8 (&dst)[4][2], const char* sa, int hh) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const int r = wc * 128 + hh * 64 + f * 16 + fr;
        dst[f][sub] = *reinterpret_cast<const bf16x8*>(sa + r * ROWB + swz<BK>(r, sub * 4 + fq) * 16);
      }
  };
  auto load_b = [&](bf16x8 (&dst)[2][2], const char* sa, int g) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const int r = wp * 64 + g * 32 + f * 16 + fr;
        dst[f][sub] = *reinterpret_cast<const bf16x8*>(sa + A_BYTES + r * ROWB + swz<BK>(r, sub * 4 + fq) * 16);
      }
  };
  f32x4 acc[8][4];
  auto mfma = [&](const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2], int hh, int g) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          acc[hh * 4 + f][g * 2 + e] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f][sub], b[e][sub], acc[hh * 4 + f][g * 2 + e], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  init_tile<8, 128>(p, acc, px0, co0, wc, wp, fr, fq);
  // prologue: step 0 (both halves) and the first half of step 1
  issue(0, 0, 0);
  issue(0, 0, 1);
  issue(0, 1, 0);
  issue(0, 1, 1);
  if (nk > 1) {
    issue(1, 0, 0);
    issue(1, 0, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  barrier();
  if (wc == 1) barrier();   // the second channel half runs one barrier behind

  bf16x8 a_f[4][2], b0[2][2], b1[2][2];
  for (int s = 0; s < nk; ++s) {
    const char* sa = smem + (s & 1) * STAGE;
    const bool n1 = s + 1 < nk, n2 = s + 2 < nk;
    // phase 0: quadrant (channels 0-63, pixels 0-31); retire the second half of step s
    load_a(a_f, sa, 0);
    load_b(b0, sa, 0);
    if (n1) {
      issue(s + 1, 1, 0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    mfma(a_f, b0, 0, 0);
    barrier();
    // phase 1: (channels 0-63, pixels 32-63)
    load_b(b1, sa, 1);
    if (n1) issue(s + 1, 1, 1);
    barrier();
    mfma(a_f, b1, 0, 1);
    barrier();
    // phase 2: (channels 64-127, pixels 32-63)
    load_a(a_f, sa, 1);
    if (n2) issue(s + 2, 0, 0);
    barrier();
    mfma(a_f, b1, 1, 1);
    barrier();
    // phase 3: (channels 64-127, pixels 0-31); retire the first half of step s+1
    if (n2) {
      issue(s + 2, 0, 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (n1) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    barrier();
    mfma(a_f, b0, 1, 0);
    barrier();
  }
  if (wc == 0) barrier();   // balance the barrier count of the two halves

  store_tile<8, 128>(p, acc, px0, co0, wc, wp, fr, fq);
}

template <int KS>
hipError_t launch_pp(const drnmi_conv_args& p, hipStream_t s) {
  constexpr int LDS = 2 * 2 * 256 * 128;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_pp_kernel<KS>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int64_t blocks = ((M + kBPX - 1) / kBPX) * (p.cout / 256);
  hipLaunchKernelGGL((conv_pp_kernel<KS>), dim3(static_cast<unsigned>(blocks)), dim3(512), LDS, s, p);
  return hipGetLastError();
}

int g_num_cus = 0;

template <int KS, int WCO, int WC, int NST, int BK, bool PERSIST, int NWP = 4, bool SPARSE = false, bool X2 = false>
hipError_t launch_big(const drnmi_conv_args& p, hipStream_t s) {
  using C = BigCfg<WCO, WC, NST, BK, NWP>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv_big_kernel<KS, WCO, WC, NST, BK, PERSIST, NWP, SPARSE, X2>),
        hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  int64_t blocks = ((M + kBPX - 1) / kBPX) * ((p.cout + C::BCO - 1) / C::BCO);
  if (PERSIST) {
    if (g_num_cus == 0) {
      int dev = 0, cus = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
      g_num_cus = cus;
    }
    const int64_t per_cu = (160 * 1024) / C::LDS;        // resident workgroups per CU (LDS-bound)
    const int64_t cap = g_num_cus * (per_cu > 0 ? per_cu : 1);
    blocks = blocks < cap ? blocks : cap;
  }
  hipLaunchKernelGGL((conv_big_kernel<KS, WCO, WC, NST, BK, PERSIST, NWP, SPARSE, X2>), dim3(static_cast<unsigned>(blocks)),
                     dim3(C::THREADS), C::LDS, s, p);
  return hipGetLastError();
}

constexpr int kStripLds = 2 * 256 * 128 + 2 * kStripBytes;   // 2 A stages + 2 strips (130 KB)

hipError_t launch_strip(const drnmi_conv_args& p, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_strip_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kStripLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int64_t blocks = (M / kBPX) * ((p.cout + 255) / 256);
  hipLaunchKernelGGL(conv_strip_kernel, dim3(static_cast<unsigned>(blocks)), dim3(512), kStripLds, s, p);
  return hipGetLastError();
}

// Routing is fixed (no environment switches): auto-picked strip launches run conv_w1_kernel (one
// wave per SIMD, 128 x 128 per wave, bit-identical) on the long-K residual-free launches (w1_auto),
// else conv_stag_kernel when cin % 128 == 0 (5-6 % faster than the strip tile, bit-identical),
// else conv_strip_kernel; the other tiles stay reachable through an explicit drnmi_conv_args.tile
// for the bit-identity tests.

// a 256-pixel tile is a run of one output row, the strip of 256 + 2 dil rows fits its buffer
bool strip_ok(const drnmi_conv_args& p) {
  return p.ks == 3 && p.stride == 1 && p.pad == p.dil && p.dil >= 1 && p.dil <= 4 && p.wo % kBPX == 0 &&
         p.x2 == nullptr && p.unit_mask == nullptr && p.cin % 64 == 0 && p.k == 9 * p.cin;
}

// the staggered strip tile (conv_stag.hip): strip geometry, cin % 128 == 0 (an even number of
// 3-step tap groups), optionally with the fused downsample (x2 validated by x2_ok)
bool stag_ok(const drnmi_conv_args& p) {
  const int tco = p.cout <= 128 ? 128 : 256;          // conv_stag128_* / conv_stag_* tile
  return p.ks == 3 && p.stride == 1 && p.pad == p.dil && p.dil >= 1 && p.dil <= 4 && p.wo % kBPX == 0 &&
         p.unit_mask == nullptr && p.cin % 128 == 0 && (p.cout + tco - 1) / tco * tco <= p.cout_pad &&
         (p.x2 == nullptr ? p.k == 9 * p.cin : (p.cin2 % 64 == 0 && p.k == 9 * p.cin + p.cin2));
}

// 128-channel convs (D-22 layer4) go to the staggered 128-channel tile instead of the halo
// kernel when both apply (88-96 vs 102-107 us, profiles/r4c_stag128_vs_halo)
bool halo_preferred(const drnmi_conv_args& p) { return !(big_conv_supported(p) && stag_ok(p)); }

struct Variant {
  int bco, bk;
  const char* name3;
  const char* name1;
};

// tile ids 4 + v in drnmi_conv_args.tile
constexpr Variant kVariants[] = {
    {128, 64, "conv_big_kernel<3, 128, 1, 3, 64, false, 4, false, false>", "conv_big_kernel<1, 128, 1, 3, 64, false, 4, false, false>"},
    {256, 64, "conv_big_kernel<3, 128, 2, 2, 64, false, 4, false, false>", "conv_big_kernel<1, 128, 2, 2, 64, false, 4, false, false>"},
    {64, 32, "conv_big_kernel<3, 64, 1, 4, 32, false, 4, false, false>", "conv_big_kernel<1, 64, 1, 4, 32, false, 4, false, false>"},
    {64, 64, "conv_big_kernel<3, 64, 1, 2, 64, false, 4, false, false>", "conv_big_kernel<1, 64, 1, 2, 64, false, 4, false, false>"},
    {256, 32, "conv_big_kernel<3, 128, 2, 4, 32, false, 4, false, false>", "conv_big_kernel<1, 128, 2, 4, 32, false, 4, false, false>"},
    {128, 32, "conv_big_kernel<3, 128, 1, 4, 32, false, 4, false, false>", "conv_big_kernel<1, 128, 1, 4, 32, false, 4, false, false>"},
    {128, 64, "conv_big_kernel<3, 128, 1, 3, 64, true, 4, false, false>", "conv_big_kernel<1, 128, 1, 3, 64, true, 4, false, false>"},
    {256, 64, "conv_big_kernel<3, 128, 2, 2, 64, true, 4, false, false>", "conv_big_kernel<1, 128, 2, 2, 64, true, 4, false, false>"},
    {64, 32, "conv_big_kernel<3, 64, 1, 4, 32, true, 4, false, false>", "conv_big_kernel<1, 64, 1, 4, 32, true, 4, false, false>"},
    {64, 64, "conv_big_kernel<3, 64, 1, 2, 64, true, 4, false, false>", "conv_big_kernel<1, 64, 1, 2, 64, true, 4, false, false>"},
    {256, 32, "conv_big_kernel<3, 128, 2, 4, 32, true, 4, false, false>", "conv_big_kernel<1, 128, 2, 4, 32, true, 4, false, false>"},
    {128, 32, "conv_big_kernel<3, 128, 1, 4, 32, true, 4, false, false>", "conv_big_kernel<1, 128, 1, 4, 32, true, 4, false, false>"},
    {256, 64, "conv_pp_kernel<3>", "conv_pp_kernel<1>"},
};
constexpr int kPingPong = 12;
constexpr int kHalo = 13;   // conv_halo.hip (tile id 17)
constexpr int kStrip = 14;  // conv_strip_kernel (tile id 18); auto routes variant 1 there when strip_ok
constexpr int kStag = 15;   // conv_stag_kernel (tile id 19): the strip tile with staggered SIMD partners
constexpr int kS2Row = 16;  // conv_s2row_kernel (tile id 20): stride-2 3x3 32 -> 64 / 64 -> 128, row walk
constexpr int kS1X2Row = 17;  // conv_s1x2row_kernel (tile id 21): stride-1 3x3 64 -> 64 + 1x1 s2 downsample 32 -> 64
constexpr int kW1 = 18;      // conv_w1_kernel (tile id 22): the stag256 tile as 4 waves of 128 x 128, one per SIMD
constexpr int kW1H = 19;     // conv_w1h_kernel (tile id 23): 128 x 128 tiles of 4 waves of 64 x 64, two per CU
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

// conv_w1 (conv_w1.hip): the staggered tile's shapes (+ the fused downsample: conv_w1_x2), 256-channel blocks
bool w1_ok(const drnmi_conv_args& p) {
  return stag_ok(p) && p.cout % 256 == 0 && p.scale == nullptr && p.out_dtype == DRNMI_BF16 &&
         p.y_sc == 1 && p.y_sp == p.cout && p.y_sn == static_cast<int64_t>(p.ho) * p.wo * p.cout;
}
// auto-routed where it measured no slower inside the network (same-box interleaved bench A/B,
// profiles/r10m_w1_ab): the long-K residual-free launches (D-22 layer6.1 conv1, layer7).  At
// cin 128 / 256 (18 / 36 K steps) and with a residual its per-tile prologue and epilogue, issued
// by 4 waves instead of 8, cost more than the loop saves (layer5.0 conv1 145 vs 130 us)
bool w1_auto(const drnmi_conv_args& p) { return w1_ok(p) && p.x2 == nullptr && p.cin >= 512 && p.res == nullptr; }
// conv_w1h: the same shapes at 128-channel blocks (a 128-pixel run: wo % 128 == 0 follows from stag_ok)
bool w1h_ok(const drnmi_conv_args& p) {
  return stag_ok(p) && p.cout % 128 == 0 && p.scale == nullptr && p.out_dtype == DRNMI_BF16 &&
         p.y_sc == 1 && p.y_sp == p.cout && p.y_sn == static_cast<int64_t>(p.ho) * p.wo * p.cout;
}
bool w1h_auto(const drnmi_conv_args& p) { return w1h_ok(p) && p.cout <= 128; }

template <int KS, bool PERSIST>
hipError_t launch_base(const drnmi_conv_args& p, int base, hipStream_t s) {
  switch (base) {
    case 0: return launch_big<KS, 128, 1, 3, 64, PERSIST>(p, s);   // 128 x 256 tile, 4 waves, 3 x 48 KB
    case 1: return launch_big<KS, 128, 2, 2, 64, PERSIST>(p, s);   // 256 x 256 tile, 8 waves, 2 x 64 KB
    case 2: return launch_big<KS, 64, 1, 4, 32, PERSIST>(p, s);    //  64 x 256 tile, 4 waves, 4 x 20 KB
    case 3: return launch_big<KS, 64, 1, 2, 64, PERSIST>(p, s);    //  64 x 256 tile, 4 waves, 2 x 40 KB
    case 4: return launch_big<KS, 128, 2, 4, 32, PERSIST>(p, s);   // 256 x 256 tile, 8 waves, 4 x 32 KB
    case 5: return launch_big<KS, 128, 1, 4, 32, PERSIST>(p, s);   // 128 x 256 tile, 4 waves, 4 x 24 KB
    default: return hipErrorInvalidValue;
  }
}

template <int KS, int WCO, int WC, int NST, int BK, bool OCC2 = false>
hipError_t launch_i8(const drnmi_conv_args& p, hipStream_t s) {
  using C = BigCfg<WCO, WC, NST, BK, 4, 1>;
  const void* f;
  if constexpr (OCC2) f = reinterpret_cast<const void*>(&conv_i8_occ2_kernel<KS, WCO, WC, NST, BK>);
  else f = reinterpret_cast<const void*>(&conv_i8_kernel<KS, WCO, WC, NST, BK>);
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int64_t blocks = ((M + kBPX - 1) / kBPX) * ((p.cout + C::BCO - 1) / C::BCO);
  if constexpr (OCC2)
    hipLaunchKernelGGL((conv_i8_occ2_kernel<KS, WCO, WC, NST, BK>), dim3(static_cast<unsigned>(blocks)), dim3(C::THREADS),
                       C::LDS, s, p);
  else
    hipLaunchKernelGGL((conv_i8_kernel<KS, WCO, WC, NST, BK>), dim3(static_cast<unsigned>(blocks)), dim3(C::THREADS),
                       C::LDS, s, p);
  return hipGetLastError();
}

// int8 variants: 0 = 256 x 256 tile / 128-B rows, 1 = 128 x 256 / 128-B, 2 = 256 x 256 / 64-B,
// 3 = 128 x 256 / 64-B (K steps of 128 or 64 int8 channels)
struct I8Variant {
  int bco;
  const char* name3;
  const char* name1;
};
constexpr I8Variant kI8Variants[] = {
    {256, "conv_i8_kernel<3, 128, 2, 2, 128>", "conv_i8_kernel<1, 128, 2, 2, 128>"},
    {128, "conv_i8_kernel<3, 128, 1, 3, 128>", "conv_i8_kernel<1, 128, 1, 3, 128>"},
    {256, "conv_i8_kernel<3, 128, 2, 4, 64>", "conv_i8_kernel<1, 128, 2, 4, 64>"},
    {128, "conv_i8_kernel<3, 128, 1, 4, 64>", "conv_i8_kernel<1, 128, 1, 4, 64>"},
    {128, "conv_i8_occ2_kernel<3, 128, 1, 2, 64>", "conv_i8_occ2_kernel<1, 128, 1, 2, 64>"},
};
constexpr int kI8Occ2 = 4;   // 128 x 256 / 64-B rows, 2 stages, two workgroups per CU

int i8_variant(const drnmi_conv_args& p) {
  const int wide = p.cout % 256 == 0 ? 0 : 1;
  // 1x1: the two-workgroups-per-CU tile (71.6-73.5 vs 86.7-86.9 us for layer5.0 / layer6.0's
  // downsample, 65.6-67.0 for the seg conv: profiles/r6_int8_fusions/occ2_ab.txt)
  return p.ks == 1 && p.cout_pad % kI8Variants[kI8Occ2].bco == 0 ? kI8Occ2 : (p.cin >= 128 ? 0 : 2) + wide;
}

template <int KS>
hipError_t launch_i8_variant(const drnmi_conv_args& p, int v, hipStream_t s) {
  switch (v) {
    case 0: return launch_i8<KS, 128, 2, 2, 128>(p, s);   // 2 x 64 KB
    case 1: return launch_i8<KS, 128, 1, 3, 128>(p, s);   // 3 x 48 KB
    case 2: return launch_i8<KS, 128, 2, 4, 64>(p, s);    // 4 x 32 KB
    case 3: return launch_i8<KS, 128, 1, 4, 64>(p, s);    // 4 x 24 KB
    case kI8Occ2: return launch_i8<KS, 128, 1, 2, 64, true>(p, s);   // 2 x 24 KB, 2 WGs / CU
    default: return hipErrorInvalidValue;
  }
}


template <int KS>
hipError_t launch_sparse(const drnmi_conv_args& p, int base, hipStream_t s) {
  switch (base) {
    case 0: return launch_big<KS, 128, 1, 3, 64, false, 4, true>(p, s);
    case 1: return launch_big<KS, 128, 2, 2, 64, false, 4, true>(p, s);
    case 4: return launch_big<KS, 128, 2, 4, 32, false, 4, true>(p, s);
    case 5: return launch_big<KS, 128, 1, 4, 32, false, 4, true>(p, s);
    default: return hipErrorInvalidValue;
  }
}

const char* sparse_name(int ks, int base) {
  static const char* n3[6] = {"conv_big_kernel<3, 128, 1, 3, 64, false, 4, true, false>",
                              "conv_big_kernel<3, 128, 2, 2, 64, false, 4, true, false>", nullptr, nullptr,
                              "conv_big_kernel<3, 128, 2, 4, 32, false, 4, true, false>",
                              "conv_big_kernel<3, 128, 1, 4, 32, false, 4, true, false>"};
  static const char* n1[6] = {"conv_big_kernel<1, 128, 1, 3, 64, false, 4, true, false>",
                              "conv_big_kernel<1, 128, 2, 2, 64, false, 4, true, false>", nullptr, nullptr,
                              "conv_big_kernel<1, 128, 2, 4, 32, false, 4, true, false>",
                              "conv_big_kernel<1, 128, 1, 4, 32, false, 4, true, false>"};
  return ks == 3 ? n3[base] : n1[base];
}

int auto_variant(const drnmi_conv_args& p) {
  if (p.cin < 64) return p.cout % 256 == 0 ? 4 : p.cout % 128 == 0 ? 5 : 2;   // K steps of 32
  // cout <= 32 (the seg 1x1) also takes the 64-wide BK-32 tile: 57 vs 66 us on the D-22 seg conv
  // at batch 8 (scripts/conv_micro.py) — two workgroups fit per CU where the 32-wide 3 x 36 KB ring fits one
  // 64 -> 128 (D-22 layer4.0 conv1 / downsample, stride 2): the 64-wide BK-32 tile too, two
  // workgroups per CU against one for the 128 x 256 x 3-stage ring: 98 vs 116 us (3x3), 50 vs
  // 75 us (1x1) at batch 8 (scripts/conv_micro.py); the fused-x2 instantiations are bases 0/1
  if (p.cin <= 64 && p.cout % 256 != 0 && p.x2 == nullptr) {
    // cin == 64 3x3 (D-22 layer4.0 conv1, stride 2): the 64-wide tile with 64-channel K steps on a
    // 2 x 40 KB ring halves the K steps of the BK-32 tile at the same DMA bytes: 93.6 vs 102 us
    // at batch 8 (profiles/r3k_tile_64w_bk64_ab.txt)
    if (p.cin == 64 && p.ks == 3) return 3;
    return 2;
  }
  return p.cout % 256 == 0 ? 1 : p.cout % 128 == 0 ? 0 : 2;
}

// one lane per 16 x 32 unit; lanes 0-31 / 32-63 of a wave cover the 32 units of two mask words
template <typename T>
__global__ void __launch_bounds__(256)
unit_mask_kernel(const T* __restrict__ w, int rows_pad, int k_pad, int wpr, uint32_t* __restrict__ mask,
                 int* __restrict__ count) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t word = gid >> 5;
  const int bit = static_cast<int>(gid & 31);
  const int rb = static_cast<int>(word / wpr);
  const int ku = static_cast<int>(word % wpr) * 32 + bit;
  const int nku = k_pad >> 5;
  bool nz = false;
  if (rb < rows_pad / 16 && ku < nku) {
    for (int r = 0; r < 16 && !nz; ++r) {
      const T* row = w + static_cast<int64_t>(rb * 16 + r) * k_pad + ku * 32;
      for (int c = 0; c < 32; ++c) {
        if constexpr (sizeof(T) == 2) nz |= (row[c] & 0x7fff) != 0;
        else nz |= (__float_as_uint(row[c]) & 0x7fffffffu) != 0;
      }
    }
  }
  const uint64_t b = __ballot(nz);
  const int lane = threadIdx.x & 63;
  if (rb < rows_pad / 16) {
    if (lane == 0) mask[word] = static_cast<uint32_t>(b & 0xffffffffu);
    if (lane == 32) mask[word] = static_cast<uint32_t>(b >> 32);
  }
  if (count != nullptr && nz) atomicAdd(count, 1);
}

}  // namespace

bool i8_conv_supported(const drnmi_conv_args& p) {
  return p.dtype == DRNMI_I8 && p.scale != nullptr && p.cin >= 64 && (p.cin & (p.cin - 1)) == 0 &&
         p.cout_pad % 128 == 0 && (p.ks == 1 || p.ks == 3) && p.k == p.ks * p.ks * p.cin && p.k_pad == p.k &&
         static_cast<int64_t>(p.n) * p.h * p.w * p.cin < (int64_t(1) << 31) && p.h < 16384 && p.w < 16384 &&
         (p.out_dtype == DRNMI_F32 || p.out_dtype == DRNMI_BF16 || p.out_dtype == DRNMI_I8);
}

bool i8_strip_ok(const drnmi_conv_args& p) {
  return i8_variant(p) == 0 && p.cin % 128 == 0 && strip_ok(p);
}

hipError_t launch_i8_strip(const drnmi_conv_args& p, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_i8_strip_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kStripLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int64_t blocks = (M / kBPX) * ((p.cout + 255) / 256);
  hipLaunchKernelGGL(conv_i8_strip_kernel, dim3(static_cast<unsigned>(blocks)), dim3(512), kStripLds, s, p);
  return hipGetLastError();
}

// int8 staggered strip tile (conv_stag.hip): 128-channel K steps, so cin % 256 == 0 gives the
// even number of 3-step tap groups the kernel walks in pairs
bool i8_stag_ok(const drnmi_conv_args& p) {
  return i8_strip_ok(p) && p.cin % 256 == 0 && p.x2 == nullptr;
}

// int8 conv_w1 (conv_w1_i8_kernel): the staggered int8 tile's shapes at 256-channel blocks with a
// dense int8 NHWC output (its 16-B epilogue).  Not auto-routed: on the long-K residual-free int8
// launches it measured no faster inside the network (profiles/r11_w1i8: layer6.1 conv1 460 vs 450
// us); the seg-fused layer8 launch (drnmi_conv_stag_seg) takes its SEGF form (431 vs 456 us)
bool i8_w1_ok(const drnmi_conv_args& p) {
  return i8_stag_ok(p) && p.cout % 256 == 0 && p.out_dtype == DRNMI_I8 && p.y_sc == 1 && p.y_sp == p.cout &&
         p.y_sn == static_cast<int64_t>(p.ho) * p.wo * p.cout;
}
// int8 conv_w1h (conv_w1h_i8_kernel: 128 x 128 tiles, two workgroups per CU, odd tap-group counts
// too): whole-row strip geometry, cin % 128 == 0, 128-channel blocks, dense int8 NHWC output;
// auto-routed at cin, cout <= 256 (D-22 layer4.1, layer5 in int8 nets: profiles/r11_int8_layer4)
bool i8_w1h_ok(const drnmi_conv_args& p) {
  return strip_ok(p) && p.cin % 128 == 0 && p.cout % 128 == 0 && p.out_dtype == DRNMI_I8 && p.y_sc == 1 &&
         p.y_sp == p.cout && p.y_sn == static_cast<int64_t>(p.ho) * p.wo * p.cout;
}
bool i8_w1h_pick(const drnmi_conv_args& p) {
  return p.tile == 4 + kW1H || (p.tile < 0 && i8_w1h_ok(p) && (p.cout <= 128 || p.cin == 128 || (p.cin <= 256 && p.cout <= 256)));
}
// tile id 22 forces the one-wave-per-SIMD int8 tile (the bit-identity tests); else the staggered one
bool i8_w1_pick(const drnmi_conv_args& p) { return p.tile == 4 + kW1; }

int i8_conv_dispatch(const drnmi_conv_args& p, hipStream_t s) {
  if (!i8_conv_supported(p)) return DRNMI_ENOTSUP;
  const int v = i8_variant(p);
  if ((p.cout + kI8Variants[v].bco - 1) / kI8Variants[v].bco * kI8Variants[v].bco > p.cout_pad) return DRNMI_EINVAL;
  if (p.ks == 3 && i8_w1h_pick(p)) {
    if (!i8_w1h_ok(p)) return DRNMI_ENOTSUP;
    const hipError_t e = launch_w1h(p, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  if (p.ks == 3 && i8_stag_ok(p)) {
    const bool w1 = i8_w1_pick(p);
    if (w1 && !i8_w1_ok(p)) return DRNMI_ENOTSUP;
    const hipError_t e = w1 ? launch_w1(p, s) : launch_stag(p, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  if (p.ks == 3 && i8_strip_ok(p)) {
    const hipError_t e = launch_i8_strip(p, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  const hipError_t e = p.ks == 3 ? launch_i8_variant<3>(p, v, s) : launch_i8_variant<1>(p, v, s);
  return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
}

const char* i8_conv_name(const drnmi_conv_args& p) {
  if (!i8_conv_supported(p)) return nullptr;
  const int v = i8_variant(p);
  if (p.ks == 3 && i8_w1h_pick(p)) return i8_w1h_ok(p) ? "conv_w1h_i8_kernel" : nullptr;
  if (p.ks == 3 && i8_stag_ok(p)) return !i8_w1_pick(p) ? "conv_i8_stag_kernel" : i8_w1_ok(p) ? "conv_w1_i8_kernel" : nullptr;
  if (p.ks == 3 && i8_strip_ok(p)) return "conv_i8_strip_kernel";
  return p.ks == 3 ? kI8Variants[v].name3 : kI8Variants[v].name1;
}

// second input (fused 1x1 downsample): bf16 NHWC x2 [n][h2][w2][cin2], cin2 a multiple of 64 with
// n*h2*w2*cin2 < 2^31, sampled at (oh*stride2, ow*stride2) inside x2; no residual with it
static bool x2_ok(const drnmi_conv_args& p) {
  if (p.x2 == nullptr) return p.k == p.ks * p.ks * p.cin;
  return p.cin2 >= 64 && p.cin2 % 64 == 0 && p.cin >= 64 && p.res == nullptr && p.unit_mask == nullptr &&
         p.stride2 >= 1 && (p.ho - 1) * p.stride2 < p.h2 && (p.wo - 1) * p.stride2 < p.w2 &&
         static_cast<int64_t>(p.n) * p.h2 * p.w2 * p.cin2 < (int64_t(1) << 31) &&
         p.k == p.ks * p.ks * p.cin + p.cin2;
}

bool big_conv_supported(const drnmi_conv_args& p) {
  return static_cast<int64_t>(p.n) * p.h * p.w * p.cin < (int64_t(1) << 31) && p.h < 16384 && p.w < 16384 &&
         p.dtype == DRNMI_BF16 && p.cin >= kMinCin && (p.cin & (p.cin - 1)) == 0 && p.cout_pad % 128 == 0 &&
         (p.ks == 1 || p.ks == 3) && x2_ok(p) && p.k_pad == p.k &&
         (p.out_dtype == DRNMI_F32 || (p.y_sc == 1 && p.y_sp == p.cout));
}

int big_conv_dispatch(const drnmi_conv_args& p, int variant, hipStream_t s) {
  if (variant == kS2Row || (variant < 0 && s2row_auto(p))) return s2row_conv_dispatch(p, s);
  if (variant == kS1X2Row || (variant < 0 && s1x2row_auto(p))) return s1x2row_conv_dispatch(p, s);
  if (variant == kW1 || variant == kW1H) {
    if (!big_conv_supported(p) || !(variant == kW1 ? w1_ok(p) : w1h_ok(p))) return DRNMI_ENOTSUP;
    const hipError_t e = variant == kW1 ? launch_w1(p, s) : launch_w1h(p, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  // the halo kernel (cin/cout 64-128) stays dense: it beats unit skipping on those shapes
  if (variant == kHalo || (variant < 0 && halo_conv_supported(p) && halo_preferred(p))) return halo_conv_dispatch(p, s);
  if (!big_conv_supported(p)) return DRNMI_ENOTSUP;
  const bool auto_pick = variant < 0;
  if (variant < 0) variant = auto_variant(p);
  if (auto_pick) {
    if (w1_auto(p)) variant = kW1;
    else if (w1h_auto(p)) variant = kW1H;
    else if (stag_ok(p)) variant = kStag;
    else if (variant == 1 && strip_ok(p)) variant = kStrip;
  }
  if (variant == kW1 || variant == kW1H) {
    const hipError_t e = variant == kW1 ? launch_w1(p, s) : launch_w1h(p, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  if (variant == kStrip || variant == kStag) {
    if (variant == kStag ? !stag_ok(p) : (!strip_ok(p) || p.cin < 64)) return DRNMI_ENOTSUP;
    if (variant == kStrip && (p.cout + 255) / 256 * 256 > p.cout_pad) return DRNMI_EINVAL;
    const hipError_t e = variant == kStag ? launch_stag(p, s) : launch_strip(p, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  if (variant >= kNumVariants) return DRNMI_ENOTSUP;
  const Variant& v = kVariants[variant];
  if (p.cin < v.bk) return DRNMI_ENOTSUP;                            // a K step must fit in one tap
  // every weight row a tile's DMA reads must exist: ceil(cout / BCO) * BCO <= cout_pad
  if ((p.cout + v.bco - 1) / v.bco * v.bco > p.cout_pad) return DRNMI_EINVAL;
  hipError_t e;
  if (variant == kPingPong) {
    if (p.cout % 256 != 0 || p.x2 != nullptr) return DRNMI_ENOTSUP;
    e = p.ks == 3 ? launch_pp<3>(p, s) : launch_pp<1>(p, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  const int base = variant % 6;
  const bool persist = variant >= 6;
  if (p.x2 != nullptr) {                  // fused second input: its own instantiation (bases 0 / 1)
    if (persist || (base != 0 && base != 1)) return DRNMI_ENOTSUP;
    if (p.ks == 3) e = base == 1 ? launch_big<3, 128, 2, 2, 64, false, 4, false, true>(p, s)
                                 : launch_big<3, 128, 1, 3, 64, false, 4, false, true>(p, s);
    else e = base == 1 ? launch_big<1, 128, 2, 2, 64, false, 4, false, true>(p, s)
                       : launch_big<1, 128, 1, 3, 64, false, 4, false, true>(p, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  if (p.unit_mask != nullptr && !persist && sparse_name(p.ks, base) != nullptr && p.k_pad / v.bk <= 128) {
    e = p.ks == 3 ? launch_sparse<3>(p, base, s) : launch_sparse<1>(p, base, s);
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  if (p.ks == 3) e = persist ? launch_base<3, true>(p, base, s) : launch_base<3, false>(p, base, s);
  else e = persist ? launch_base<1, true>(p, base, s) : launch_base<1, false>(p, base, s);
  return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
}

const char* big_conv_name(const drnmi_conv_args& p, int variant) {
  if (variant == kS2Row || (variant < 0 && s2row_auto(p))) return s2row_conv_name(p);
  if (variant == kS1X2Row || (variant < 0 && s1x2row_auto(p))) return s1x2row_conv_name(p);
  if (variant == kW1 || variant == kW1H) {
    if (!big_conv_supported(p) || !(variant == kW1 ? w1_ok(p) : w1h_ok(p))) return nullptr;
    if (variant == kW1) return p.x2 != nullptr ? "conv_w1_x2_kernel" : "conv_w1_kernel";
    return p.x2 != nullptr ? "conv_w1h_x2_kernel" : "conv_w1h_kernel";
  }
  if (variant == kHalo || (variant < 0 && halo_conv_supported(p) && halo_preferred(p))) return halo_conv_name(p);
  const bool auto_pick = variant < 0;
  if (variant < 0) variant = auto_variant(p);
  if (auto_pick) {
    if (w1_auto(p)) variant = kW1;
    else if (w1h_auto(p)) variant = kW1H;
    else if (stag_ok(p)) variant = kStag;
    else if (variant == 1 && strip_ok(p)) variant = kStrip;
  }
  if (variant == kW1) return p.x2 != nullptr ? "conv_w1_x2_kernel" : "conv_w1_kernel";
  if (variant == kW1H) return p.x2 != nullptr ? "conv_w1h_x2_kernel" : "conv_w1h_kernel";
  if (variant == kStag) {
    if (!stag_ok(p)) return nullptr;
    if (p.cout <= 128) return p.x2 != nullptr ? "conv_stag128_x2_kernel" : "conv_stag128_kernel";
    return p.x2 != nullptr ? "conv_stag_x2_kernel" : "conv_stag_kernel";
  }
  if (variant == kStrip) return strip_ok(p) && p.cin >= 64 ? "conv_strip_kernel" : nullptr;
  if (variant >= kNumVariants) return nullptr;
  if (p.x2 != nullptr) {
    if (variant != 0 && variant != 1) return nullptr;
    static const char* n[2][2] = {{"conv_big_kernel<1, 128, 1, 3, 64, false, 4, false, true>",
                                   "conv_big_kernel<1, 128, 2, 2, 64, false, 4, false, true>"},
                                  {"conv_big_kernel<3, 128, 1, 3, 64, false, 4, false, true>",
                                   "conv_big_kernel<3, 128, 2, 2, 64, false, 4, false, true>"}};
    return n[p.ks == 3 ? 1 : 0][variant];
  }
  if (p.unit_mask != nullptr && variant < 6 && sparse_name(p.ks, variant) != nullptr &&
      p.k_pad / kVariants[variant].bk <= 128)
    return sparse_name(p.ks, variant);
  return p.ks == 3 ? kVariants[variant].name3 : kVariants[variant].name1;
}

int big_conv_num_variants() { return kNumVariants; }

int weight_unit_mask(const void* wgt, int dtype, int rows_pad, int k_pad, uint32_t* mask, int* count,
                     hipStream_t s) {
  if (wgt == nullptr || mask == nullptr || rows_pad <= 0 || rows_pad % 16 != 0 || k_pad <= 0 || k_pad % 32 != 0)
    return DRNMI_EINVAL;
  const int wpr = (k_pad + 1023) / 1024;
  const int64_t lanes = static_cast<int64_t>(rows_pad / 16) * wpr * 32;
  const unsigned blocks = static_cast<unsigned>((lanes + 255) / 256);
  if (count != nullptr) {
    const hipError_t e = hipMemsetAsync(count, 0, sizeof(int), s);
    if (e != hipSuccess) return static_cast<int>(e);
  }
  if (dtype == DRNMI_BF16)
    hipLaunchKernelGGL(unit_mask_kernel<uint16_t>, dim3(blocks), dim3(256), 0, s,
                       reinterpret_cast<const uint16_t*>(wgt), rows_pad, k_pad, wpr, mask, count);
  else if (dtype == DRNMI_F32)
    hipLaunchKernelGGL(unit_mask_kernel<float>, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const float*>(wgt),
                       rows_pad, k_pad, wpr, mask, count);
  else
    return DRNMI_EINVAL;
  return static_cast<int>(hipGetLastError());
}

}  // namespace drnmi

using namespace drnmi;

// The labels-only video path's last 3x3 conv (D-22 layer8) with the seg classifier folded into its
// epilogue (conv_stag.hip SEGF): same launch geometry and MFMA work as conv_stag_kernel, the
// activation is never stored.  Validated like the conv it replaces plus the seg operands.
extern "C" int drnmi_conv_stag_seg(const drnmi_conv_args* a, const void* seg_w, int32_t seg_k_pad, int32_t seg_rows,
                                   void* partials, void* stream) {
  if (a == nullptr || seg_w == nullptr || partials == nullptr) return DRNMI_EINVAL;
  const drnmi_conv_args& p = *a;
  if (p.x == nullptr || p.wgt == nullptr || p.shift == nullptr) return DRNMI_EINVAL;
  if (p.algo != DRNMI_ALGO_IGEMM || p.src_u8) return DRNMI_EINVAL;
  if (p.dtype == DRNMI_I8) {
    // int8 nets: the conv's int8 output (out_dtype I8, quantised with out_scale) feeds int8 seg
    // weights; int32 partials
    if (p.out_dtype != DRNMI_I8 || p.scale == nullptr) return DRNMI_EINVAL;
    if (p.ho != (p.h + 2 * p.pad - p.dil * (p.ks - 1) - 1) / p.stride + 1 ||
        p.wo != (p.w + 2 * p.pad - p.dil * (p.ks - 1) - 1) / p.stride + 1)
      return DRNMI_EINVAL;
    if (seg_k_pad < p.cout || seg_k_pad % 16 != 0 || seg_rows < 32 || (reinterpret_cast<uintptr_t>(partials) & 15) != 0)
      return DRNMI_EINVAL;
    if (!(i8_conv_supported(p) && p.ks == 3 && i8_stag_ok(p)) || p.res != nullptr || p.cout % 256 != 0 ||
        p.cout_pad < p.cout)
      return DRNMI_ENOTSUP;
    // the one-wave-per-SIMD int8 tile (conv_w1_i8_seg_kernel); tile 19 forces the staggered one
    const hipError_t e = p.tile == 4 + kStag ? launch_stag_seg(p, seg_w, seg_k_pad, partials, reinterpret_cast<hipStream_t>(stream))
                                             : launch_w1_seg(p, seg_w, seg_k_pad, partials, reinterpret_cast<hipStream_t>(stream));
    return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
  }
  if (p.dtype != DRNMI_BF16 || p.out_dtype != DRNMI_BF16) return DRNMI_EINVAL;
  if (p.ho != (p.h + 2 * p.pad - p.dil * (p.ks - 1) - 1) / p.stride + 1 ||
      p.wo != (p.w + 2 * p.pad - p.dil * (p.ks - 1) - 1) / p.stride + 1)
    return DRNMI_EINVAL;
  if (seg_k_pad < p.cout || seg_k_pad % 8 != 0 || seg_rows < 32 || (reinterpret_cast<uintptr_t>(partials) & 15) != 0)
    return DRNMI_EINVAL;
  if (!(big_conv_supported(p) && stag_ok(p)) || p.x2 != nullptr ||
      p.scale != nullptr || p.res != nullptr || p.cout % 256 != 0 || p.cout_pad < p.cout)
    return DRNMI_ENOTSUP;
  // the one-wave-per-SIMD tile (conv_w1_seg_kernel); tile 19 forces the staggered one (the same
  // partial logits, bit for bit: the bit-identity test)
  const hipError_t e = p.tile == 4 + kStag ? launch_stag_seg(p, seg_w, seg_k_pad, partials, reinterpret_cast<hipStream_t>(stream))
                                           : launch_w1_seg(p, seg_w, seg_k_pad, partials, reinterpret_cast<hipStream_t>(stream));
  return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
}

extern "C" const char* drnmi_conv_stag_seg_kernel_name(const drnmi_conv_args* a) {
  if (a == nullptr) return nullptr;
  if (a->dtype == DRNMI_I8) return a->tile == 4 + kStag ? "conv_i8_stag_seg_kernel" : "conv_w1_i8_seg_kernel";
  return a->tile == 4 + kStag ? "conv_stag_seg_kernel" : "conv_w1_seg_kernel";
}
