// Large-channel NHWC implicit-GEMM convolution, bf16, LDS-DMA staged (the MFMA-bound layers).
//
// Serves every conv of DRN-D with cin >= 64 and cout % 128 == 0: layer4..layer8 3x3 convs
// (dilation 1/2/4, lmodels/drn.py:27-29, :49-65, :201-211), the 1x1 stride-s downsamples
// (:181-186) and the Bottleneck convs (:86-106).  In D-22 at 1024x2048 these are ~85 % of
// the FLOPs at arithmetic intensity 190..2150 FLOP/B, i.e. MFMA-bound.
//
// Structure (per workgroup of 4 waves, one output tile of 128 channels x 256 pixels):
//   * MFMA orientation A = weights (rows = output channels), B = pixels, so the
//     accumulator hands each lane 4 consecutive channels of one pixel (8-byte NHWC
//     stores, 8-byte residual loads).
//   * K step = 64 (one kernel tap x 64 input channels, since cin >= 64): both operand
//     tiles are fetched global -> LDS by global_load_lds_dwordx4 (LDS-DMA, no VGPR
//     round trip, no ds_write issue cost).  Each pixel row of the B tile is gathered from
//     its own NHWC address (the implicit-GEMM im2col happens in the DMA addresses);
//     out-of-image taps read a zero page, which is the conv's zero padding.
//   * Three LDS stages (144 KB): the DMAs of steps t+1 and t+2 are in flight while step t
//     is consumed; one raw barrier per step behind a counted vmcnt.
//   * LDS image rows are 128 B; chunk c of row r sits at slot c ^ ((r >> 1) & 7), applied
//     on the DMA source address (the DMA destination is lane-linear) and on the fragment
//     read, which makes the 16x16x32 fragment reads bank-conflict free.
//   * Each wave owns 128 channels x 64 pixels: 8 x 4 fragments, 32 MFMA per 32-deep
//     substep, 128 accumulator registers.
//   * Tiles are dealt XCD-major so the cout tiles of one pixel tile share an L2.
#include "common.h"
#include "kernels.h"

namespace drnmi {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_void_t;

__device__ uint4 g_zero_page[64];   // zero-initialised: the source of padded taps / rows

constexpr int kBPX = 256;     // pixels per tile
constexpr int kMinCin = 32;   // every K step must lie inside one tap (BK 64 needs cin >= 64)

// LDS image rows of BK bf16 (BK*2 bytes).  16-B chunk c of row r sits at slot swz(r, c):
// 128-B rows: c ^ ((r >> 1) & 7); 64-B rows: c ^ ((r >> 2) & 3) -- the rows that share
// banks in a 16x16x32 fragment read then land on different 16-B slots.
template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) {
  if constexpr (BK == 64) return chunk ^ ((row >> 1) & 7);
  else return chunk ^ ((row >> 2) & 3);
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ int xcd_remap2(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

// Tile = (WCO * WC) channels x 256 pixels; 4*WC waves, each wave WCO channels x 64 pixels
// (WCO/16 x 4 MFMA fragments).  NST = LDS ring depth.
template <int KS, int WCO, int WC, int NST, int BK>
struct BigCfg {
  static constexpr int BCO = WCO * WC;
  static constexpr int FM = WCO / 16;
  static constexpr int NW = 4 * WC;
  static constexpr int THREADS = 64 * NW;
  static constexpr int ROWB = BK * 2;               // bytes per LDS row
  static constexpr int CPR = ROWB / 16;             // 16-B chunks per row
  static constexpr int RPI = 1024 / ROWB;           // rows per 1-KB DMA wave instruction
  static constexpr int SUB = BK / 32;               // 32-deep MFMA substeps per step
  static constexpr int A_BYTES = BCO * ROWB;
  static constexpr int B_BYTES = kBPX * ROWB;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_INSTR = BCO / RPI / NW;    // DMA instructions per wave per step
  static constexpr int B_INSTR = kBPX / RPI / NW;
  static constexpr int GLDS = A_INSTR + B_INSTR;
  static constexpr int LDS = NST * STAGE;
};

// OPT bit 0: interleave the DMA issue / fragment reads into the MFMA stream;
// OPT bit 1: raise wave priority around each MFMA group (s_setprio 1 / 0).
template <int KS, int WCO, int WC, int NST, int BK, int OPT>
__global__ void __launch_bounds__(64 * 4 * WC, 1)
conv_big_kernel(const drnmi_conv_args p) {
  constexpr bool IL = (OPT & 1) != 0;
  constexpr bool PRIO = (OPT & 2) != 0;
  using C = BigCfg<KS, WCO, WC, NST, BK>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wc = wave / 4;          // channel half of the tile
  const int wp = wave % 4;          // 64-pixel quarter of the tile
  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const int nco = (p.cout + C::BCO - 1) / C::BCO;
  const int npx = (M + kBPX - 1) / kBPX;
  const int tile = xcd_remap2(blockIdx.x, npx * nco);
  const int px0 = (tile / nco) * kBPX;
  const int co0 = (tile % nco) * C::BCO;

  const int cin = p.cin;
  const int lc = 31 - __builtin_clz(cin);
  const int H = p.h, W = p.w, dil = p.dil;
  const uint16_t* __restrict__ x = reinterpret_cast<const uint16_t*>(p.x);
  const uint16_t* __restrict__ wt = reinterpret_cast<const uint16_t*>(p.wgt);

  // --- DMA assignment.  One wave instruction fills RPI LDS rows (1 KB); lane l fills
  // row RPI*j + l / CPR, slot l % CPR (lane-linear destination; the swizzle is applied to
  // the source chunk).  Wave w fills A instructions [w*A_INSTR, ...) and B [w*B_INSTR, ...).
  const int lrow = lane / C::CPR;
  const int lslot = lane % C::CPR;
  int a_src_off[C::A_INSTR];
#pragma unroll
  for (int i = 0; i < C::A_INSTR; ++i) {
    const int r = (wave * C::A_INSTR + i) * C::RPI + lrow;
    a_src_off[i] = (co0 + r) * p.k_pad + swz<BK>(r, lslot) * 8;
  }
  // pixel rows: (ih0, iw0) of tap (0,0) and a base pointer at that tap's chunk (only
  // dereferenced when the tap lies inside the image)
  int b_ih0[C::B_INSTR], b_iw0[C::B_INSTR];
  const uint16_t* b_base[C::B_INSTR];
#pragma unroll
  for (int i = 0; i < C::B_INSTR; ++i) {
    const int r = (wave * C::B_INSTR + i) * C::RPI + lrow;
    const int m = px0 + r;
    b_ih0[i] = -(1 << 28);
    b_iw0[i] = -(1 << 28);
    b_base[i] = x;
    if (m < M) {
      const int n = m / hw_o;
      const int q = m - n * hw_o;
      const int oh = q / p.wo;
      const int ow = q - oh * p.wo;
      b_ih0[i] = oh * p.stride - p.pad;
      b_iw0[i] = ow * p.stride - p.pad;
      b_base[i] = x + ((static_cast<int64_t>(n) * H + b_ih0[i]) * W + b_iw0[i]) * cin + swz<BK>(r, lslot) * 8;
    }
  }
  const char* zero_src = reinterpret_cast<const char*>(g_zero_page) + lane * 16;

  // one DMA instruction ("piece") of step kt: pieces [0, A_INSTR) weights, then pixels
  struct StepP { int k0, dh, dw; int64_t toff; };
  auto step_params = [&](int kt) {
    StepP sp;
    sp.k0 = kt * BK;
    const int tap = sp.k0 >> lc;
    sp.dh = (tap / KS) * dil;
    sp.dw = (tap - (tap / KS) * KS) * dil;
    sp.toff = (static_cast<int64_t>(sp.dh) * W + sp.dw) * cin + (sp.k0 & (cin - 1));
    return sp;
  };
  auto issue_piece = [&](const StepP& sp, int stage, int i) {
    char* sa = smem + stage * C::STAGE;
    if (i < C::A_INSTR) {
      glds16(wt + a_src_off[i] + sp.k0, sa + (wave * C::A_INSTR + i) * 1024);
    } else {
      const int j = i - C::A_INSTR;
      const bool ok = static_cast<unsigned>(b_ih0[j] + sp.dh) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(b_iw0[j] + sp.dw) < static_cast<unsigned>(W);
      const void* src = ok ? static_cast<const void*>(b_base[j] + sp.toff) : static_cast<const void*>(zero_src);
      glds16(src, sa + C::A_BYTES + (wave * C::B_INSTR + j) * 1024);
    }
  };

  auto issue = [&](int kt, int stage) {
    char* sa = smem + stage * C::STAGE;
    char* sb = sa + C::A_BYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < C::A_INSTR; ++i)
      glds16(wt + a_src_off[i] + k0, sa + (wave * C::A_INSTR + i) * 1024);
    const int tap = k0 >> lc;
    const int ci0 = k0 & (cin - 1);
    const int dh = (tap / KS) * dil;
    const int dw = (tap - (tap / KS) * KS) * dil;
    const int64_t toff = (static_cast<int64_t>(dh) * W + dw) * cin + ci0;   // uniform over rows
#pragma unroll
    for (int i = 0; i < C::B_INSTR; ++i) {
      const bool ok = static_cast<unsigned>(b_ih0[i] + dh) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(b_iw0[i] + dw) < static_cast<unsigned>(W);
      const void* src = ok ? static_cast<const void*>(b_base[i] + toff) : static_cast<const void*>(zero_src);
      glds16(src, sb + (wave * C::B_INSTR + i) * 1024);
    }
  };

  f32x4 acc[C::FM][4];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.k_pad / BK;
  const int fr = lane & 15;       // fragment row (channel or pixel within a 16-block)
  const int fq = lane >> 4;       // 8-element k chunk within a 32-deep substep

  // Ring of NST stages: NST-1 steps in flight while one is consumed.  The DMA of step t is
  // retired by a counted vmcnt (newer steps stay in flight), then published by a raw
  // s_barrier (a __syncthreads() would drain to vmcnt(0)); lgkmcnt(0) first retires this
  // wave's reads of the stage the next DMA overwrites.
  for (int t = 0; t < NST - 1 && t < nk; ++t) issue(t, t);
  for (int t = 0; t < nk; ++t) {
    const int cur = t % NST;
    // steps issued after step t so far: min(nk - 1, t + NST - 2) - t
    const int newer = ((nk - 1) < (t + NST - 2) ? (nk - 1) : (t + NST - 2)) - t;
    if (NST >= 4 && newer >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * C::GLDS) : "memory");
    else if (NST >= 3 && newer >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::GLDS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const char* sa = smem + cur * C::STAGE;
    if constexpr (IL) {
      // Interleaved: fragment reads run one 8-MFMA group ahead and the next step's DMA is
      // issued piece by piece between MFMA groups of the first substep, so the DMA issue
      // cost and the LDS read latency overlap MFMAs instead of preceding them.
      constexpr int GR = C::FM / 2;              // groups of 2 weight fragments x 4 pixel fragments
      constexpr int NG = C::SUB * GR;
      constexpr int PPG = (C::GLDS + GR - 1) / GR;   // DMA pieces per group (first substep)
      const bool nxt = t + NST - 1 < nk;
      const StepP sp = step_params(t + NST - 1);
      const int nst = (t + NST - 1) % NST;
      const char* sb = sa + C::A_BYTES;
      bf16x8 af[2][2], bfr[2][4];
      auto load_a = [&](bf16x8 (&dst)[2], int q) {
        const int c = (q / GR) * 4 + fq;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = wc * WCO + ((q % GR) * 2 + h) * 16 + fr;
          dst[h] = *reinterpret_cast<const bf16x8*>(sa + r * C::ROWB + swz<BK>(r, c) * 16);
        }
      };
      auto load_b = [&](bf16x8 (&dst)[4], int sub) {
        const int c = sub * 4 + fq;
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) {
          const int r = wp * 64 + fn * 16 + fr;
          dst[fn] = *reinterpret_cast<const bf16x8*>(sb + r * C::ROWB + swz<BK>(r, c) * 16);
        }
      };
      load_b(bfr[0], 0);
      load_a(af[0], 0);
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        if (q + 1 < NG) {
          load_a(af[(q + 1) & 1], q + 1);
          if ((q + 1) % GR == 0) load_b(bfr[((q + 1) / GR) & 1], (q + 1) / GR);
        }
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int fn = 0; fn < 4; ++fn)
            acc[(q % GR) * 2 + h][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                af[q & 1][h], bfr[(q / GR) & 1][fn], acc[(q % GR) * 2 + h][fn], 0, 0, 0);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        if (q < GR && nxt) {
#pragma unroll
          for (int k = 0; k < PPG; ++k)
            if (q * PPG + k < C::GLDS) issue_piece(sp, nst, q * PPG + k);
        }
      }
      continue;
    }
    if (t + NST - 1 < nk) issue(t + NST - 1, (t + NST - 1) % NST);
    const char* sb = sa + C::A_BYTES;
#pragma unroll
    for (int s = 0; s < C::SUB; ++s) {
      const int c = s * 4 + fq;
      bf16x8 af[C::FM], bfr[4];
#pragma unroll
      for (int fm = 0; fm < C::FM; ++fm) {
        const int r = wc * WCO + fm * 16 + fr;
        af[fm] = *reinterpret_cast<const bf16x8*>(sa + r * C::ROWB + swz<BK>(r, c) * 16);
      }
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) {
        const int r = wp * 64 + fn * 16 + fr;
        bfr[fn] = *reinterpret_cast<const bf16x8*>(sb + r * C::ROWB + swz<BK>(r, c) * 16);
      }
#pragma unroll
      for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[fm], bfr[fn], acc[fm][fn], 0, 0, 0);
    }
  }

  // --- epilogue: lane owns channels co..co+3 of pixel m, for FM x 4 fragments
  const uint16_t* __restrict__ res = reinterpret_cast<const uint16_t*>(p.res);
  const bool nhwc16 = p.out_dtype == DRNMI_BF16 && p.y_sc == 1;
#pragma unroll
  for (int fn = 0; fn < 4; ++fn) {
    const int m = px0 + wp * 64 + fn * 16 + fr;
    if (m >= M) continue;
    const int n = m / hw_o;
    const int q = m - n * hw_o;
    const int64_t ybase = static_cast<int64_t>(n) * p.y_sn + static_cast<int64_t>(q) * p.y_sp;
#pragma unroll
    for (int fm = 0; fm < C::FM; ++fm) {
      const int co = co0 + wc * WCO + fm * 16 + fq * 4;
      if (co >= p.cout) continue;
      const float4 sc = *reinterpret_cast<const float4*>(p.scale + co);   // padded to cout_pad
      const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
      float v[4] = {acc[fm][fn][0] * sc.x + sh.x, acc[fm][fn][1] * sc.y + sh.y,
                    acc[fm][fn][2] * sc.z + sh.z, acc[fm][fn][3] * sc.w + sh.w};
      const bool full = co + 3 < p.cout;
      if (res != nullptr) {
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

template <int KS, int WCO, int WC, int NST, int BK, int OPT = 0>
hipError_t launch_big(const drnmi_conv_args& p, hipStream_t s) {
  using C = BigCfg<KS, WCO, WC, NST, BK>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_big_kernel<KS, WCO, WC, NST, BK, OPT>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int64_t blocks = ((M + kBPX - 1) / kBPX) * ((p.cout + C::BCO - 1) / C::BCO);
  hipLaunchKernelGGL((conv_big_kernel<KS, WCO, WC, NST, BK, OPT>), dim3(static_cast<unsigned>(blocks)), dim3(C::THREADS),
                     C::LDS, s, p);
  return hipGetLastError();
}

template <int KS>
hipError_t launch_big_variant(const drnmi_conv_args& p, int variant, hipStream_t s) {
  switch (variant) {
    case 0: return launch_big<KS, 128, 1, 3, 64>(p, s);   // 128 x 256 tile, 4 waves, 3 x 48 KB
    case 1: return launch_big<KS, 128, 2, 2, 64>(p, s);   // 256 x 256 tile, 8 waves, 2 x 64 KB
    case 2: return launch_big<KS, 64, 1, 3, 64>(p, s);    //  64 x 256 tile, 4 waves, 3 x 40 KB
    case 3: return launch_big<KS, 32, 1, 3, 64>(p, s);    //  32 x 256 tile, 4 waves, 3 x 36 KB
    case 4: return launch_big<KS, 128, 2, 4, 32>(p, s);   // 256 x 256 tile, 8 waves, 4 x 32 KB (BK 32)
    case 5: return launch_big<KS, 128, 1, 4, 32>(p, s);   // 128 x 256 tile, 4 waves, 4 x 24 KB (BK 32)
    case 6: return launch_big<KS, 128, 2, 2, 64, 1>(p, s);   // = 1, interleaved DMA issue
    case 7: return launch_big<KS, 128, 2, 2, 64, 3>(p, s);   // = 6 + s_setprio around MFMA groups
    case 8: return launch_big<KS, 128, 1, 3, 64, 1>(p, s);   // = 0, interleaved DMA issue
    case 9: return launch_big<KS, 128, 1, 3, 64, 3>(p, s);   // = 8 + s_setprio
    case 10: return launch_big<KS, 64, 1, 3, 64, 1>(p, s);   // = 2, interleaved
    case 11: return launch_big<KS, 32, 1, 3, 64, 1>(p, s);   // = 3, interleaved
    case 12: return launch_big<KS, 64, 1, 4, 32, 1>(p, s);   //  64 x 256, K 32 steps (cin 32)
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool big_conv_supported(const drnmi_conv_args& p) {
  return p.dtype == DRNMI_BF16 && p.cin >= kMinCin && (p.cin & (p.cin - 1)) == 0 && p.cout_pad % 128 == 0 &&
         (p.ks == 1 || p.ks == 3) && p.k == p.ks * p.ks * p.cin && p.k_pad == p.k &&
         (p.out_dtype == DRNMI_F32 || (p.y_sc == 1 && p.y_sp == p.cout));
}

static int auto_variant(const drnmi_conv_args& p) {
  if (p.cin < 64)   // K steps of 32
    return p.cout % 256 == 0 ? 4 : p.cout % 128 == 0 ? 5 : 12;
  return p.cout % 256 == 0 ? 6 : p.cout % 128 == 0 ? 8 : p.cout > 32 ? 12 : 11;
}

int big_conv_dispatch(const drnmi_conv_args& p, int variant, hipStream_t s) {
  if (!big_conv_supported(p)) return DRNMI_ENOTSUP;
  if (variant < 0) variant = auto_variant(p);
  const bool bk32 = variant == 4 || variant == 5 || variant == 12;
  if (!bk32 && p.cin < 64) return DRNMI_ENOTSUP;     // K steps of 64 need cin >= 64
  if (variant > 12) return DRNMI_ENOTSUP;
  // every weight row a tile's DMA reads must exist: ceil(cout / BCO) * BCO <= cout_pad
  static const int bco[13] = {128, 256, 64, 32, 256, 128, 256, 256, 128, 128, 64, 32, 64};
  if ((p.cout + bco[variant] - 1) / bco[variant] * bco[variant] > p.cout_pad) return DRNMI_EINVAL;
  const hipError_t e = p.ks == 3 ? launch_big_variant<3>(p, variant, s) : launch_big_variant<1>(p, variant, s);
  return e == hipErrorInvalidValue ? DRNMI_ENOTSUP : static_cast<int>(e);
}

const char* big_conv_name(const drnmi_conv_args& p, int variant) {
  if (variant < 0) variant = auto_variant(p);
  static const char* names3[] = {"conv_big_kernel<3, 128, 1, 3, 64, 0>", "conv_big_kernel<3, 128, 2, 2, 64, 0>",
                                 "conv_big_kernel<3, 64, 1, 3, 64, 0>", "conv_big_kernel<3, 32, 1, 3, 64, 0>",
                                 "conv_big_kernel<3, 128, 2, 4, 32, 0>", "conv_big_kernel<3, 128, 1, 4, 32, 0>",
                                 "conv_big_kernel<3, 128, 2, 2, 64, 1>", "conv_big_kernel<3, 128, 2, 2, 64, 3>",
                                 "conv_big_kernel<3, 128, 1, 3, 64, 1>", "conv_big_kernel<3, 128, 1, 3, 64, 3>",
                                 "conv_big_kernel<3, 64, 1, 3, 64, 1>", "conv_big_kernel<3, 32, 1, 3, 64, 1>",
                                 "conv_big_kernel<3, 64, 1, 4, 32, 1>"};
  static const char* names1[] = {"conv_big_kernel<1, 128, 1, 3, 64, 0>", "conv_big_kernel<1, 128, 2, 2, 64, 0>",
                                 "conv_big_kernel<1, 64, 1, 3, 64, 0>", "conv_big_kernel<1, 32, 1, 3, 64, 0>",
                                 "conv_big_kernel<1, 128, 2, 4, 32, 0>", "conv_big_kernel<1, 128, 1, 4, 32, 0>",
                                 "conv_big_kernel<1, 128, 2, 2, 64, 1>", "conv_big_kernel<1, 128, 2, 2, 64, 3>",
                                 "conv_big_kernel<1, 128, 1, 3, 64, 1>", "conv_big_kernel<1, 128, 1, 3, 64, 3>",
                                 "conv_big_kernel<1, 64, 1, 3, 64, 1>", "conv_big_kernel<1, 32, 1, 3, 64, 1>",
                                 "conv_big_kernel<1, 64, 1, 4, 32, 1>"};
  if (variant < 0 || variant > 12) return nullptr;
  return p.ks == 3 ? names3[variant] : names1[variant];
}

}  // namespace drnmi
