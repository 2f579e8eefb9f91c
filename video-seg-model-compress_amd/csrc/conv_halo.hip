// Halo-patch 3x3 convolution for the mid-size stride-1 layers (cin 64/128, cout 64/128):
// DRN-D layer3/layer4 BasicBlock convs (lmodels/drn.py:27-29, :49-65; the D-38/54 layer3/4
// Bottleneck 3x3 convs, :86-106, take the same path).
//
// conv_big streams the im2col B operand per K step, so every input pixel is fetched 9 times
// (once per tap) and, at cout <= 128, those DMA pieces outnumber the MFMAs they feed.  Here a
// workgroup owns a 4 x 64 output block and all cout channels; its input neighbourhood
// ((4 + 2 dil) x (64 + 2 dil) pixels x cin) is DMA'd into LDS once, and the 9 taps are read
// from that patch at shifted pixel rows.  Only the weights stream per K step (a small
// LDS-DMA ring shared by every wave).
//
//   * LDS patch rows = pixels (cin * 2 bytes), 16-B chunk c of row r at slot c ^ f(r)
//     (applied on the DMA source and on the fragment read, as in conv_big);
//     out-of-image pixels come from a zero page (the conv's zero padding).
//   * K step = (64-channel block, tap), taps innermost; A = weights [cout][64] per step.
//   * MFMA v_mfma_f32_16x16x32_bf16, A = weights (rows = channels), B = pixels: wave
//     (wc, wp) owns channels wc*64..+64 of output row wp (64 pixels), 4 x 4 fragments.
//   * Fused second input (x2 != NULL: the block's 1x1 stride-s downsample folded into its last
//     conv, lmodels/drn.py:181-186, as in conv_big): cin2 (32 or 64) more K columns
//     [W | W_ds | 0-pad to 64] streamed through the same weight ring as one or two extra 32-wide
//     K halves after the taps; their B fragments (x2 at (oh*s2, ow*s2), 16 B per lane) are
//     plain global loads issued before the patch DMA, so the residual branch is never written
//     to HBM or read back.  k = 9 cin + cin2, k_pad = round_up(k, 64).
#include "common.h"
#include "kernels.h"

namespace drnmi {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_void_t;

__device__ uint4 g_halo_zero[64];   // zero-initialised source of padded pixels

constexpr int kTR = 4, kTC = 64;     // output block: rows x columns
constexpr int kNST = 3;              // weight ring stages (4-5 stages cost a workgroup per CU: slower)

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

template <int ROWB>
__device__ __forceinline__ int hswz(int row, int chunk) {
  // 128-B rows: slot = (row & 1, chunk ^ (row & 7)) gives the 16 lanes of every ds_read_b128
  // group 16 distinct 4-bank slots for ANY row offset (the taps shift the rows by dw), which
  // the earlier (row >> 1) & 7 did not for odd shifts
  if constexpr (ROWB == 128) return chunk ^ (row & 7);
  else return chunk ^ (row & 15);   // 256-B rows span all 64 banks
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// LDS bytes of the patch, rounded up to whole 1-KB DMA pieces
__host__ __device__ constexpr int patch_bytes(int cin, int dil, int tc) {
  return ((kTR + 2 * dil) * (tc + 2 * dil) * cin * 2 + 1023) / 1024 * 1024;
}

template <int CIN, int WC, int TC>
__global__ void __launch_bounds__(256 * WC, 1)
conv_halo_kernel(const drnmi_conv_args p) {
  constexpr int NW = 4 * WC;
  constexpr int FN = TC / 16;            // pixel fragments per wave (one output row)
  constexpr int ROWB = CIN * 2;          // patch row bytes
  constexpr int CPR = ROWB / 16;         // chunks per patch row
  constexpr int RPP = 1024 / ROWB;       // patch rows per DMA piece
  constexpr int COUT_T = 64 * WC;        // channels per tile
  constexpr int A_STAGE = COUT_T * 128;  // weights [COUT_T][64] bf16
  constexpr int A_PIECES = A_STAGE / 1024 / NW;   // per wave per step (2)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;
  char* patch = smem + kNST * A_STAGE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wc = wave >> 2;
  const int wp = wave & 3;
  const int fr = lane & 15;
  const int fq = lane >> 4;
  const int H = p.h, W = p.w, dil = p.dil;
  const int PW = TC + 2 * dil;
  const int PROWS = (kTR + 2 * dil) * PW;
  const int tiles_x = (p.wo + TC - 1) / TC;
  const int tiles_y = (p.ho + kTR - 1) / kTR;
  const int ntiles = p.n * tiles_y * tiles_x;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int n = tile / (tiles_y * tiles_x);
  const int trem = tile - n * tiles_y * tiles_x;
  const int oh0 = (trem / tiles_x) * kTR;
  const int ow0 = (trem - (trem / tiles_x) * tiles_x) * TC;
  const uint16_t* __restrict__ x = reinterpret_cast<const uint16_t*>(p.x);
  const uint16_t* __restrict__ wt = reinterpret_cast<const uint16_t*>(p.wgt);
  constexpr int NCB = CIN / 64;
  const int nk = 9 * NCB;                       // tap steps
  const bool fused = p.x2 != nullptr;
  const int nx = fused ? 1 : 0;                  // x2 steps (cin2 <= 64: one 64-column step)
  const int nk_all = nk + nx;

  // --- accumulator start: 0, or shift + residual when the BN scale is folded into the
  // weights (scale == NULL); those loads go out ahead of the DMA and hide under it
  const uint16_t* __restrict__ res = reinterpret_cast<const uint16_t*>(p.res);
  const int oh = oh0 + wp;
  f32x4 acc[4][FN];
#pragma unroll
  for (int fm = 0; fm < 4; ++fm) {
    const int co = wc * 64 + fm * 16 + fq * 4;
    f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.scale == nullptr) {
      const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
      a0 = f32x4{sh.x, sh.y, sh.z, sh.w};
    }
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = a0;
  }
  // x2 fragments (fused downsample): sub-step j of x2 step e is channel block (2e + j) * 32
  bf16x8 x2f[2][FN];
  if (fused) {
    const uint16_t* __restrict__ x2 = reinterpret_cast<const uint16_t*>(p.x2);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int ow = ow0 + fn * 16 + fr;
        x2f[j][fn] = bf16x8{};
        if (j * 32 < p.cin2 && oh < p.ho && ow < p.wo) {
          const int64_t q = (static_cast<int64_t>(n) * p.h2 + static_cast<int64_t>(oh) * p.stride2) * p.w2 +
                            static_cast<int64_t>(ow) * p.stride2;
          x2f[j][fn] = *reinterpret_cast<const bf16x8*>(x2 + q * p.cin2 + j * 32 + fq * 8);
        }
      }
  }
  // residual loads issued here, added after the patch and weight DMA went out (adding them here
  // made the DMA wait for the residual: two latencies in series per tile)
  const bool add_res = p.scale == nullptr && res != nullptr && oh < p.ho;
  // full output row run (wave-uniform): residual and output as 16-B pieces (common.h swap_halves)
  const bool full_row = oh < p.ho && ow0 + TC <= p.wo;
  uint2 rv[4][FN];
  uint4 rq[2][FN];
  if (add_res && full_row) {
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int64_t m = (static_cast<int64_t>(n) * p.ho + oh) * p.wo + ow0 + fn * 16 + fr;
#pragma unroll
      for (int f2 = 0; f2 < 2; ++f2)
        rq[f2][fn] = *reinterpret_cast<const uint4*>(res + m * p.cout + wc * 64 + f2 * 32 + chunk_of_row(fq) * 8);
    }
  } else if (add_res) {
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int ow = ow0 + fn * 16 + fr;
      const int64_t m = (static_cast<int64_t>(n) * p.ho + oh) * p.wo + (ow < p.wo ? ow : p.wo - 1);
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
        rv[fm][fn] = *reinterpret_cast<const uint2*>(res + m * p.cout + wc * 64 + fm * 16 + fq * 4);
    }
  }

  // --- patch: DMA once (pieces dealt round-robin over the waves)
  {
    const int npieces = (PROWS + RPP - 1) / RPP;
    const char* zero_src = reinterpret_cast<const char*>(g_halo_zero) + lane * 16;
    const int lr = lane / CPR, ls = lane % CPR;
    const int64_t img = static_cast<int64_t>(n) * H;
    for (int pc = wave; pc < npieces; pc += NW) {
      const int row = pc * RPP + lr;
      const int pr = row / PW;
      const int ih = oh0 - p.pad + pr;
      const int iw = ow0 - p.pad + (row - pr * PW);
      const bool ok = row < PROWS && static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(iw) < static_cast<unsigned>(W);
      const void* src = ok ? static_cast<const void*>(x + ((img + ih) * W + iw) * CIN + hswz<ROWB>(row, ls) * 8)
                           : static_cast<const void*>(zero_src);
      glds16(src, patch + pc * 1024);
    }
  }
  // --- weights ring: step kt = (cb, tap) -> packed column tap * CIN + cb * 64
  const int lrow = lane >> 3, lslot = lane & 7;   // 128-B rows, 8 per piece
  int a_off[A_PIECES];
#pragma unroll
  for (int i = 0; i < A_PIECES; ++i) {
    const int r = (wave * A_PIECES + i) * 8 + lrow;
    a_off[i] = r * p.k_pad + (hswz<128>(r, lslot)) * 8;
  }
  auto a_col = [&](int kt) {
    if (kt >= nk) return 9 * CIN + (kt - nk) * 64;   // x2 columns
    const int cb = kt / 9;
    return (kt - cb * 9) * CIN + cb * 64;
  };
  auto issue_a = [&](int kt, int i) {
    glds16(wt + a_off[i] + a_col(kt), ring + (kt % kNST) * A_STAGE + (wave * A_PIECES + i) * 1024);
  };
  for (int t = 0; t < kNST - 1 && t < nk_all; ++t)
#pragma unroll
    for (int i = 0; i < A_PIECES; ++i) issue_a(t, i);
  if (add_res && full_row) {
#pragma unroll
    for (int f2 = 0; f2 < 2; ++f2)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        swap_halves(rq[f2][fn]);
        rv[2 * f2][fn] = make_uint2(rq[f2][fn].x, rq[f2][fn].y);
        rv[2 * f2 + 1][fn] = make_uint2(rq[f2][fn].z, rq[f2][fn].w);
      }
  }
  if (add_res) {
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        acc[fm][fn][0] += bf16_to_f32(static_cast<uint16_t>(rv[fm][fn].x & 0xffff));
        acc[fm][fn][1] += bf16_to_f32(static_cast<uint16_t>(rv[fm][fn].x >> 16));
        acc[fm][fn][2] += bf16_to_f32(static_cast<uint16_t>(rv[fm][fn].y & 0xffff));
        acc[fm][fn][3] += bf16_to_f32(static_cast<uint16_t>(rv[fm][fn].y >> 16));
      }
  }


  for (int t = 0; t < nk; ++t) {
    // retire step t (the patch went out before every weight piece, so it is retired too)
    // younger: the weight pieces of steps t+1 .. t+kNST-2
    if (t + kNST - 2 < nk_all) asm volatile("s_waitcnt vmcnt(%0)" :: "n"((kNST - 2) * A_PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const bool nxt = t + kNST - 1 < nk_all;
    const char* sa = ring + (t % kNST) * A_STAGE;
    const int cb = t / 9;
    const int tap = t - cb * 9;
    const int dh = (tap / 3) * dil, dw = (tap - (tap / 3) * 3) * dil;
    const int prow0 = (wp + dh) * PW + dw;            // patch row of this wave's pixel 0
    // both K halves' fragments are read up front (the second half's reads are in flight under
    // the first half's MFMAs; the two waves of a SIMD run these phases in lockstep after the
    // barrier, so a read issued right before its MFMAs would expose the LDS latency)
    bf16x8 af[2][4], bfr[2][FN];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int r = wc * 64 + f * 16 + fr;
        af[sub][f] = *reinterpret_cast<const bf16x8*>(sa + r * 128 + hswz<128>(r, sub * 4 + fq) * 16);
      }
#pragma unroll
      for (int f = 0; f < FN; ++f) {
        const int pr = prow0 + f * 16 + fr;
        bfr[sub][f] = *reinterpret_cast<const bf16x8*>(patch + pr * ROWB + hswz<ROWB>(pr, cb * 8 + sub * 4 + fq) * 16);
      }
      if (sub == 0 && nxt) {
#pragma unroll
        for (int i = 0; i < A_PIECES; ++i) issue_a(t + kNST - 1, i);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[sub][fm], bfr[sub][fn], acc[fm][fn], 0, 0, 0);
    }
  }
  // fused downsample: the x2 K step (cin2 <= 64: one 64-column weight step), B fragments from
  // registers; a 32-channel x2 has one live K half (the zero-padded second half is skipped).
  // Static fragment indices only: a runtime index would put x2f in scratch memory.
  if (fused) {
    const int t = nk;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const char* sa = ring + (t % kNST) * A_STAGE;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      if (sub * 32 >= p.cin2) break;
      bf16x8 af[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int r = wc * 64 + f * 16 + fr;
        af[f] = *reinterpret_cast<const bf16x8*>(sa + r * 128 + hswz<128>(r, sub * 4 + fq) * 16);
      }
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[fm], x2f[sub][fn], acc[fm][fn], 0, 0, 0);
    }
  }

  // --- epilogue: lane owns channels co..co+3 of pixel (oh0 + wp, ow0 + fn*16 + fr)
  if (oh >= p.ho) return;
  if (full_row && p.scale == nullptr) {   // shift (+ residual) already in the accumulators
    uint16_t* __restrict__ y = reinterpret_cast<uint16_t*>(p.y);
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int64_t m = (static_cast<int64_t>(n) * p.ho + oh) * p.wo + ow0 + fn * 16 + fr;
      uint4 o[2];
#pragma unroll
      for (int f2 = 0; f2 < 2; ++f2) {
        uint32_t w[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float v[4] = {acc[2 * f2 + h][fn][0], acc[2 * f2 + h][fn][1], acc[2 * f2 + h][fn][2], acc[2 * f2 + h][fn][3]};
          if (p.relu) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
          }
          w[2 * h] = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
          w[2 * h + 1] = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
        }
        o[f2] = make_uint4(w[0], w[1], w[2], w[3]);
        swap_halves(o[f2]);
      }
      // whole 128-B lines (the wave's 64 channels of 8 pixels per instruction): lanes fr and
      // fr ^ 8 trade their second-group chunks (as conv_tile.h store_tile_x4)
      const bool lo = fr < 8;
      const int64_t m0 = m - (lo ? 0 : 8), m1 = m0 + 8;
      uint4 r;
      r.x = __builtin_amdgcn_update_dpp(0u, o[1].x, 0x128, 0xf, 0xf, false);
      r.y = __builtin_amdgcn_update_dpp(0u, o[1].y, 0x128, 0xf, 0xf, false);
      r.z = __builtin_amdgcn_update_dpp(0u, o[1].z, 0x128, 0xf, 0xf, false);
      r.w = __builtin_amdgcn_update_dpp(0u, o[1].w, 0x128, 0xf, 0xf, false);
      const uint4 d0 = make_uint4(lo ? o[0].x : r.x, lo ? o[0].y : r.y, lo ? o[0].z : r.z, lo ? o[0].w : r.w);
      const uint4 d1 = make_uint4(lo ? r.x : o[0].x, lo ? r.y : o[0].y, lo ? r.z : o[0].z, lo ? r.w : o[0].w);
      const int c = wc * 64 + chunk_of_row(fq) * 8;
      *reinterpret_cast<uint4*>(y + m0 * p.cout + c + (lo ? 0 : 32)) = d0;
      *reinterpret_cast<uint4*>(y + m1 * p.cout + c + (lo ? 32 : 0)) = d1;
    }
    return;
  }
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int ow = ow0 + fn * 16 + fr;
    if (ow >= p.wo) continue;
    const int64_t m = (static_cast<int64_t>(n) * p.ho + oh) * p.wo + ow;
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
      const int co = wc * 64 + fm * 16 + fq * 4;
      if (co >= p.cout) continue;
      float v[4] = {acc[fm][fn][0], acc[fm][fn][1], acc[fm][fn][2], acc[fm][fn][3]};
      if (p.scale != nullptr) {
        const float4 sc = *reinterpret_cast<const float4*>(p.scale + co);
        const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
        v[0] = v[0] * sc.x + sh.x;
        v[1] = v[1] * sc.y + sh.y;
        v[2] = v[2] * sc.z + sh.z;
        v[3] = v[3] * sc.w + sh.w;
      }
      if (p.scale != nullptr && res != nullptr) {
        const uint2 rv = *reinterpret_cast<const uint2*>(res + m * p.cout + co);
        v[0] += bf16_to_f32(static_cast<uint16_t>(rv.x & 0xffff));
        v[1] += bf16_to_f32(static_cast<uint16_t>(rv.x >> 16));
        v[2] += bf16_to_f32(static_cast<uint16_t>(rv.y & 0xffff));
        v[3] += bf16_to_f32(static_cast<uint16_t>(rv.y >> 16));
      }
      if (p.relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      uint2 o;
      o.x = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
      o.y = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.y) + m * p.cout + co) = o;
    }
  }
}

// output-block width: 64 columns (32 for the 64 -> 64 conv, three workgroups per CU instead of two,
// measured the same: 128.0 vs 128.3 us, D-22 layer3, 8 frames)
constexpr int halo_tc(int /*cin*/, int /*cout*/) { return 64; }

template <int CIN, int WC>
hipError_t launch_halo(const drnmi_conv_args& p, hipStream_t s) {
  constexpr int TC = halo_tc(CIN, 64 * WC);
  const int lds = kNST * 64 * WC * 128 + patch_bytes(CIN, p.dil, TC);
  static int attr_lds = 0;
  if (attr_lds < lds) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_halo_kernel<CIN, WC, TC>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_lds = lds;
  }
  const int64_t tiles = static_cast<int64_t>(p.n) * ((p.ho + kTR - 1) / kTR) * ((p.wo + TC - 1) / TC);
  hipLaunchKernelGGL((conv_halo_kernel<CIN, WC, TC>), dim3(static_cast<unsigned>(tiles)), dim3(256 * WC), lds, s, p);
  return hipGetLastError();
}

}  // namespace

bool halo_conv_supported(const drnmi_conv_args& p) {
  if (p.dtype != DRNMI_BF16 || p.out_dtype != DRNMI_BF16 || p.ks != 3 || p.stride != 1 || p.pad != p.dil)
    return false;
  if ((p.cin != 64 && p.cin != 128) || (p.cout != 64 && p.cout != 128) || p.cout_pad < p.cout)
    return false;
  if (p.y_sc != 1 || p.y_sp != p.cout || p.dil < 1 || p.dil > 8) return false;
  if (p.x2 != nullptr) {
    // fused downsample: cin2 32 or 64 columns after the taps, rows zero-padded to whole 64-column
    // weight steps; the accumulators start from shift only (no residual, scale folded)
    if ((p.cin2 != 32 && p.cin2 != 64) || p.stride2 < 1 || p.res != nullptr || p.scale != nullptr ||
        p.k != 9 * p.cin + p.cin2 || p.k_pad != (p.k + 63) / 64 * 64 || p.h2 < 1 || p.w2 < 1 ||
        (p.ho - 1) * p.stride2 >= p.h2 || (p.wo - 1) * p.stride2 >= p.w2)
      return false;
  } else if (p.k != 9 * p.cin || p.k_pad != p.k) {
    return false;
  }
  const int wc = p.cout / 64;
  return kNST * 64 * wc * 128 + patch_bytes(p.cin, p.dil, halo_tc(p.cin, p.cout)) <= 160 * 1024;
}

int halo_conv_dispatch(const drnmi_conv_args& p, hipStream_t s) {
  if (!halo_conv_supported(p)) return DRNMI_ENOTSUP;
  hipError_t e;
  if (p.cin == 64) e = p.cout == 64 ? launch_halo<64, 1>(p, s) : launch_halo<64, 2>(p, s);
  else e = p.cout == 64 ? launch_halo<128, 1>(p, s) : launch_halo<128, 2>(p, s);
  return static_cast<int>(e);
}

const char* halo_conv_name(const drnmi_conv_args& p) {
  if (p.cin == 64)
    return p.cout == 64 ? "conv_halo_kernel<64, 1, 64>" : "conv_halo_kernel<64, 2, 64>";
  return p.cout == 64 ? "conv_halo_kernel<128, 1, 64>" : "conv_halo_kernel<128, 2, 64>";
}

}  // namespace drnmi
