// Staggered strip conv (bf16): see conv_stag_body.  Own translation unit so its register
// allocation is not perturbed by conv_big.hip's many instantiations (cdna_hip_programming.md
// §5.4 rule 19).
#include "common.h"
#include "conv_tile.h"
#include "kernels.h"

namespace drnmi {
namespace {

// --- Staggered strip kernel (conv_stag_kernel): the strip tile (256 output channels x one
// 256-pixel run of an output row, 3x3 stride 1) with the two waves of every SIMD half a K step
// apart (MI355X_MICROARCH.md "Two waves per SIMD", item 9).
//
// In conv_strip_kernel the SIMD partners w and w + 4 (same pixel slice, channel halves wc = 0/1)
// run in lockstep: after every K-step barrier both issue their fragment reads and wait for them
// before their first MFMA, so the matrix pipe idles on the LDS latency once per step on every
// SIMD.  Here each K step is two phases (one 32-deep substep each) and every phase ends with a
// barrier; waves 4-7 run one phase behind waves 0-3.  In every phase one wave of each SIMD starts
// a fresh step (reads the just-published stage) while its partner runs the second substep of the
// previous one from fragments it prefetched before the barrier.
//
// LDS (as conv_strip_kernel, 130 KB): two A stages (the weight rows of channel half wc are read
// only by waves 4 wc .. 4 wc + 3, which also DMA them) and two B strip buffers.  Hazards, with
// global phase = 2 t + u for waves 0-3 and 2 t + u + 1 for waves 4-7 (step t, substep u):
//   * A rows of half wc for step t + 1 are DMA'd by that half in its phase (t, 0) -- its last
//     read of the stage's previous occupant (step t - 1) was phase (t - 1, 1) -- and retired by
//     the vmcnt at the end of (t, 1), before the barrier that opens (t + 1, 0);
//   * the strip of group g + 1 (K steps 3g + 3 .. 3g + 5) is DMA'd in each wave's phases
//     (3g, 1), (3g + 1, 0), (3g + 1, 1) = global 6g + 1 .. 6g + 4; its buffer's previous group
//     g - 1 was last read in global phase 6g (waves 4-7), and its first reader is global phase
//     6g + 6 (waves 0-3), after the vmcnt at the end of global 6g + 5 at the latest;
//   * every phase ends with s_waitcnt vmcnt(pieces issued in this phase): all older pieces have
//     landed; fragment reads of the second substep may fly across the barrier (same stage, no
//     DMA targets it for two more phases); the last phase of a step waits lgkmcnt(0).
// K order, MFMA order per accumulator and epilogue are conv_strip_kernel's: bit-identical output.
//
// X2 (the block's 1x1 downsample folded in as cin2 / BK extra K steps after the taps, as in
// conv_big's X2 form and in the same K order): the first x2 step's B (256 pixels of x2, one strip
// buffer) is fetched by the last tap group's strip shares; after the staggered loop the waves
// re-align and run the x2 steps unstaggered (one barrier per step, next step's A and B DMA'd
// under the current step's MFMAs).
//
// WCO = channels per wave (tile = 2 WCO output channels x 256 pixels): 128 (the 256-channel tile
// of layer5-8) or 64 (128-channel convs: D-22 layer4); GR = WCO / 32 MFMA groups per substep.
// Tile deal (workgroups go to XCD bid % 8): XCD-major -- XCD x takes a contiguous run of (pixel
// tile, channel block) tiles, i.e. its rows x both channel blocks (an XCD-stationary channel block
// fetched 19 % more at the same time).
__device__ __forceinline__ int stag_tile(int bid, int ntiles, int /*nco*/) { return xcd_remap2(bid, ntiles); }

// SEGF (the labels-only video path's last conv, drnmi_conv_stag_seg): the conv's own output is not
// stored; its epilogue feeds the seg classifier (1x1 512 -> 19 + bias, lmodels/drnseg.py:278-284)
// instead -- per tile, the partial logits over its 256 channels go to part[channel block][pixel][20]
// and the head adds bias + block 0 + block 1 in that order.
struct SegFuse {
  const void* w;        // seg weights, packed [>= 32 rows][k_pad]: bf16 (scale folded) or int8; rows 19.. zero
  int k_pad;
  void* part;           // [nco][n ho wo][kSegCS]: fp32 (bf16 nets) or int32 (int8 nets)
};
constexpr int kSegCS = 20;

// int8 nets (C5): the seg classifier on the int8 copy of the last conv's output.  Each output
// value is quantised exactly as store_tile_i8 stores it (fmul, fadd, ReLU, rint(v * out_scale)
// clamped to +-127; no contraction) and becomes the B operand of v_mfma_i32_16x16x64_i8 whose A
// fragments are the int8 seg weights.  Lane (fr, fq) holds channels 16 fm + 4 fq .. + 3 of
// pixel fr; for the 64-channel group g its 16 bytes are channels 64 g + 16 m + 4 fq + e (m, e =
// 0..3) in that order, and the A fragment takes the seg weights of the same channels: a fixed
// permutation of K, so the int32 sums are exact -- the separate int8 seg conv's accumulators,
// split into per-tile (256-channel) partials whose integer sum is order-free.
template <int FM>
__device__ __forceinline__ void stag_seg_i8(const drnmi_conv_args& p, const int (&acc)[FM][4][4], int px0, int co0, int wc,
                                            int wp, int fr, int fq, const SegFuse& sf, char* smem) {
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
  i32x4 pacc[2][4];
#pragma unroll
  for (int fn = 0; fn < 4; ++fn) {
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
  // the two channel halves of the tile (waves wc = 0, 1), added through LDS (the loop is done with it)
  i32x4* xch = reinterpret_cast<i32x4*>(smem) + (wp * 64 + (fq * 16 + fr)) * 8;
  __syncthreads();
  if (wc == 1) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) xch[mt * 4 + fn] = pacc[mt][fn];
  }
  __syncthreads();
  if (wc == 0) {
    const int M = p.n * p.ho * p.wo;
    int* __restrict__ part = static_cast<int*>(sf.part) + static_cast<int64_t>(co0 / (32 * FM)) * M * kSegCS;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int cls = 16 * mt + 4 * fq;
      if (cls >= kSegCS) continue;
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) {
        const i32x4 o = xch[mt * 4 + fn];
        const int64_t m = px0 + wp * 64 + fn * 16 + fr;
        *reinterpret_cast<int4*>(part + m * kSegCS + cls) =
            make_int4(pacc[mt][fn][0] + o[0], pacc[mt][fn][1] + o[1], pacc[mt][fn][2] + o[2], pacc[mt][fn][3] + o[3]);
      }
    }
  }
}

template <typename T, bool X2, int WCO = 128, bool SEGF = false>
__device__ __forceinline__ void conv_stag_body(const drnmi_conv_args& p, const SegFuse& sf = SegFuse{nullptr, 0, nullptr}) {
  using K = KT<T>;
  constexpr int BK = 128 / K::ESZ;                   // 128-B LDS rows (bf16 64, int8 128 channels)
  using C = BigCfg<WCO, 2, 2, BK, 4, K::ESZ>;
  constexpr int FM = C::FM, GR = FM / 2, AI = C::A_INSTR, BCO = 2 * WCO;
  static_assert(C::ROWB == 128 && C::FN == 4 && (WCO == 128 || WCO == 64) && AI == WCO / 32, "stag tile geometry");
  constexpr int CE = 16 / K::ESZ;
  constexpr int AB = C::A_BYTES;                     // 32 KB per A stage
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave >> 2;                          // channel half; also the stagger group
  const int wp = wave & 3;                           // 64-pixel slice
  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const int nco = (p.cout + BCO - 1) / BCO;
  const int ntiles = (M / kBPX) * nco;
  const int cin = p.cin;
  const int lc = 31 - __builtin_clz(cin);
  const int H = p.h, W = p.w, dil = p.dil;
  const T* __restrict__ x = reinterpret_cast<const T*>(p.x);
  const T* __restrict__ wt = reinterpret_cast<const T*>(p.wgt);
  const int nk = 9 * cin / BK;                       // tap steps: whole groups of 3
  const int ngroups = nk / 3;
  const int nx2 = X2 ? p.cin2 / BK : 0;              // x2 steps after the taps
  const int nk_tot = nk + nx2;
  const int fr = lane & 15;
  const int fq = lane >> 4;
  const int lrow = lane >> 3;
  const int lslot = lane & 7;

  const int tile = stag_tile(blockIdx.x, ntiles, nco);
  const int px0 = (tile / nco) * kBPX;
  const int co0 = (tile % nco) * BCO;
  const int s_n = px0 / hw_o;
  const int s_q = px0 - s_n * hw_o;
  const int s_oh = s_q / p.wo;
  const int s_ow0 = s_q - s_oh * p.wo;
  // DMA through buffer resources: per-lane 32-bit byte offsets, out-of-image pixels as an
  // out-of-range offset (the load returns zeros: the conv's zero padding), wave-uniform parts
  // in SGPRs -- one VGPR per stream instead of a 64-bit address and a validity mask
  const int xbytes = p.n * H * W * cin * K::ESZ;     // < 2^31 (big_conv_supported)
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.x), 0, xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.wgt), 0, p.cout_pad * p.k_pad * K::ESZ, 0x00020000);
  typedef __attribute__((address_space(3))) void lds_t;
  auto dma = [&](const __amdgpu_buffer_rsrc_t& rs, uint32_t voff, int soff, int lds_byte) {   // weights
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t*)(smem + lds_byte), 16, voff, soff, 0, 0);
  };
  auto dma_x = [&](const __amdgpu_buffer_rsrc_t& rs, uint32_t voff, int soff, int lds_byte) { // input strips
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t*)(smem + lds_byte), 16, voff, soff, 0, 0);
  };
  // weight rows (wave*4 + i)*8 + lrow: the swizzle depends on i only through its parity
  uint32_t a_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave * AI + i) * 8 + lrow;
    a_off[i] = ((co0 + r) * p.k_pad + swzb<128>(r, lslot) * CE) * K::ESZ;
  }
  constexpr uint32_t kOOB = 0x80000000u;             // beyond every buffer (sizes < 2^31)

  // weight piece i (rows (wave*4 + i)*8 .. +8) of K step kt into A stage `stage`
  auto issue_a = [&](int kt, int stage, int i) {
    const int cb = kt / 9;
    const int tap = kt - cb * 9;
    const int k0 = (X2 && kt >= nk) ? 9 * cin + (kt - nk) * BK : (tap << lc) + cb * BK;
    dma(rs_w, a_off[i & 1], ((i & ~1) * 8 * p.k_pad + k0) * K::ESZ, stage * AB + (wave * AI + i) * 1024);
  };
  // strip share sh of group g (channel block g / 3, tap row g % 3) into strip buffer `buf`
  auto issue_strip = [&](int g, int buf, int sh) {
    const int j = wave + 8 * sh;
    if (j >= kStripPieces) return;                   // wave-uniform
    const int R = j * 8 + lrow;
    const int cb = g / 3, kh = g - cb * 3;
    const int ih = s_oh - p.pad + kh * dil;
    const int iw = s_ow0 - p.pad + R;
    const bool ok = R < kBPX + 2 * dil && static_cast<unsigned>(iw) < static_cast<unsigned>(W);
    const bool row_ok = static_cast<unsigned>(ih) < static_cast<unsigned>(H);   // wave-uniform
    const uint32_t voff = ok && row_ok ? static_cast<uint32_t>((iw * cin + (lslot ^ (R & 7)) * CE) * K::ESZ) : kOOB;
    const int soff = row_ok ? ((s_n * H + ih) * W * cin + cb * BK) * K::ESZ : 0;
    dma_x(rs_x, voff, soff, 2 * AB + buf * kStripBytes + j * 1024);
  };
  // X2: share sh of x2 step e's B -- pixel R of the tile sampled at stride2 in x2, channels
  // e*BK..; strip row R, chunk slot c ^ (R & 7) as the tap strips (read at kw offset 0)
  auto issue_x2 = [&](int e, int buf, int sh) {
    if constexpr (X2) {
      const int j = wave + 8 * sh;
      if (j >= kStripPieces) return;
      const int R = j * 8 + lrow;
      const __amdgpu_buffer_rsrc_t rs_x2 = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<void*>(p.x2), 0, p.n * p.h2 * p.w2 * p.cin2 * K::ESZ, 0x00020000);
      const uint32_t voff = R < kBPX ? static_cast<uint32_t>(((s_ow0 + R) * p.stride2 * p.cin2 + (lslot ^ (R & 7)) * CE) * K::ESZ)
                                     : kOOB;
      const int soff = ((s_n * p.h2 + s_oh * p.stride2) * p.w2 * p.cin2 + e * BK) * K::ESZ;
      dma_x(rs_x2, voff, soff, 2 * AB + buf * kStripBytes + j * 1024);
    }
  };
  auto issue_next_strip = [&](int g, int buf, int sh) {   // the strip of group g + 1 (or x2 step 0)
    if (X2 && g + 1 >= ngroups) issue_x2(0, buf, sh);
    else issue_strip(g + 1 < ngroups ? g + 1 : ngroups - 1, buf, sh);
  };

  // fragment-read byte offsets: the swizzles of the 16 rows a lane group reads do not depend on
  // the fragment index (A: rows 16 apart keep (row >> 1) & 7; B: rows 16 apart keep R & 7), so
  // one base per (substep) / (tap column, substep) and compile-time offsets cover every read
  uint32_t a_base[2], b_base[3][2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int r = wc * WCO + fr;
    a_base[u] = r * 128 + (swzb<128>(r, u * 4 + fq) << 4);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int R = wp * 64 + fr + kw * dil;
      b_base[kw][u] = 2 * AB + R * 128 + (((u * 4 + fq) ^ (R & 7)) << 4);
    }
  }

  typename K::acc acc[FM][4];
  typename K::frag af[2][2], bfr[2][4];
  // fragment reads: inline-asm ds_read_b128 with compile-time offsets and hand-counted lgkmcnt
  // (hipcc's own waits drained every second group: 0.6-0.8 % slower, profiles/r4a_stag_ab)
  auto rd = [&](typename K::frag& dst, uint32_t base, auto off_c) {
    constexpr int OFF = decltype(off_c)::value;
    // base: a byte offset into smem, which is LDS address 0 (the kernel's only LDS object)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(OFF));
  };
  auto load_a = [&](typename K::frag (&dst)[2], auto stage_c, auto u_c, auto qg_c) {
    constexpr int ST = decltype(stage_c)::value, U_ = decltype(u_c)::value, QG = decltype(qg_c)::value;
    rd(dst[0], a_base[U_], std::integral_constant<int, ST * AB + (QG * 2 + 0) * 2048>{});
    rd(dst[1], a_base[U_], std::integral_constant<int, ST * AB + (QG * 2 + 1) * 2048>{});
  };
  auto load_b = [&](typename K::frag (&dst)[4], auto buf_c, auto kw_c, auto u_c) {
    constexpr int BF = decltype(buf_c)::value, KW_ = decltype(kw_c)::value, U_ = decltype(u_c)::value;
    const uint32_t b = b_base[KW_][U_];
    rd(dst[0], b, std::integral_constant<int, BF * kStripBytes + 0 * 2048>{});
    rd(dst[1], b, std::integral_constant<int, BF * kStripBytes + 1 * 2048>{});
    rd(dst[2], b, std::integral_constant<int, BF * kStripBytes + 2 * 2048>{});
    rd(dst[3], b, std::integral_constant<int, BF * kStripBytes + 3 * 2048>{});
  };

  // accumulator start: shift (+ residual).  The residual loads go out before the prologue DMA
  // and are added after it, so their latency and the DMA's overlap (init_tile waited for them
  // before issuing the DMA).  Tiles cover whole 4-channel groups when cout % BCO == 0.
  const bool split_init = K::ESZ == 2 && p.scale == nullptr && p.cout % BCO == 0;
  const bool has_res = split_init && p.res != nullptr;
  // dense bf16 NHWC output: the 16-B store epilogue (store_tile_x4)
  const bool fast_epi = split_init && p.out_dtype == DRNMI_BF16 && p.y_sc == 1 && p.y_sp == p.cout &&
                        p.y_sn == static_cast<int64_t>(hw_o) * p.cout;
  uint4 rv[FM / 2][4];
  float4 shv[FM];
  if constexpr (K::ESZ == 2) {
    if (split_init) {
      // only loads here: a register written from a pending load before the DMA issue would make
      // the compiler wait (vmcnt(0) at the join) ahead of it
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) shv[fm] = *reinterpret_cast<const float4*>(p.shift + co0 + wc * WCO + fm * 16 + fq * 4);
      if (has_res) load_residual<FM, WCO, 4>(p, rv, px0, co0, wc, wp, fr, fq);
    } else {
      init_tile<FM, WCO, 4, false>(p, acc, px0, co0, wc, wp, fr, fq);
    }
  } else {
    zero_tile(acc);
  }
#pragma unroll
  for (int i = 0; i < AI; ++i) issue_a(0, 0, i);
#pragma unroll
  for (int sh = 0; sh < 5; ++sh) issue_strip(0, 0, sh);
  if constexpr (K::ESZ == 2) {
    if (split_init) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) acc[fm][fn] = f32x4{shv[fm].x, shv[fm].y, shv[fm].z, shv[fm].w};
      if (has_res) add_residual(acc, rv, fr);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (wc == 1) {                                     // the stagger: waves 4-7 sit out phase 0
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }

  // one phase = substep U of K step t = 3 g + KW; GP = g & 1 (strip buffer), stage = t & 1
  auto phase = [&](auto kw_c, auto u_c, auto gp_c, int g) {
    constexpr int KW = decltype(kw_c)::value;
    constexpr int U = decltype(u_c)::value;
    constexpr int GP = decltype(gp_c)::value;
    constexpr int STAGE = (GP + KW) & 1;
    const int t = 3 * g + KW;
    const int ta = t + 1 < nk_tot ? t + 1 : nk_tot - 1;   // clamped: past the end, re-fetch into the idle stage
    using IS = std::integral_constant<int, STAGE>;
    using IU = std::integral_constant<int, U>;
    using IG = std::integral_constant<int, GP>;
    using IK = std::integral_constant<int, KW>;
    using Z = std::integral_constant<int, 0>;
    using O = std::integral_constant<int, 1>;
    if constexpr (U == 0) {
      load_b(bfr[0], IG{}, IK{}, Z{});
      load_a(af[0], IS{}, Z{}, Z{});
    }
    auto group_reads = [&](auto qg_c) {
      constexpr int QG = decltype(qg_c)::value;
      if constexpr (QG < GR - 1) {
        load_a(af[(QG + 1) & 1], IS{}, IU{}, std::integral_constant<int, QG + 1>{});
      } else if constexpr (U == 0) {                 // the second substep's first fragments, ahead of the barrier
        load_b(bfr[1], IG{}, IK{}, O{});
        load_a(af[0], IS{}, O{}, Z{});
      }
    };
#pragma unroll
    for (int qg = 0; qg < GR; ++qg) {
      if (qg == 0) group_reads(std::integral_constant<int, 0>{});
      if (qg == 1) group_reads(std::integral_constant<int, 1>{});
      if (qg == 2) group_reads(std::integral_constant<int, 2>{});
      if (qg == 3) group_reads(std::integral_constant<int, 3>{});
      // this group's fragments: everything but the reads issued after them (the next group's
      // 2, or 6 when the second substep's B and first A went out)
      if (qg < GR - 1) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
      else if (U == 0) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) acc[qg * 2 + h][fn] = K::mma(af[qg & 1][h], bfr[U][fn], acc[qg * 2 + h][fn]);
      if constexpr (U == 0) { if (qg < AI) issue_a(ta, STAGE ^ 1, qg); }
      if constexpr (KW == 0 && U == 1) { if (qg < 2) issue_next_strip(g, GP ^ 1, qg); }
      if constexpr (KW == 1 && U == 0) { if (qg == 1) issue_next_strip(g, GP ^ 1, 2); }
      if constexpr (KW == 1 && U == 1) { if (qg < 2) issue_next_strip(g, GP ^ 1, 3 + qg); }
      __builtin_amdgcn_sched_barrier(0);
    }
    // retire every piece issued before this phase; this phase's own stay in flight
    if constexpr (KW == 0 && U == 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(AI) : "memory");
    if constexpr (KW == 0 && U == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    if constexpr (KW == 1 && U == 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(AI + 1) : "memory");
    if constexpr (KW == 1 && U == 1) {
      if (wave == 0) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // shares 3 and 4 (piece 32)
      else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    }
    if constexpr (KW == 2 && U == 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(AI) : "memory");
    if constexpr (KW == 2 && U == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (U == 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  auto group = [&](auto gp_c, int g) {
    phase(I0{}, I0{}, gp_c, g);
    phase(I0{}, I1{}, gp_c, g);
    phase(I1{}, I0{}, gp_c, g);
    phase(I1{}, I1{}, gp_c, g);
    phase(I2{}, I0{}, gp_c, g);
    phase(I2{}, I1{}, gp_c, g);
  };
  for (int g = 0; g < ngroups; g += 2) {             // ngroups even (cin % 128 == 0, dispatch)
    group(I0{}, g);
    group(I1{}, g + 1);
  }
  if (wc == 0) {                                     // waves 0-3 match waves 4-7's last barrier
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (X2) {
    // x2 steps, all waves aligned: step nk + e reads A stage (nk + e) & 1 and strip buffer
    // (ngroups + e) & 1 (both landed: the last phases waited vmcnt(0) before their barriers)
    for (int e = 0; e < nx2; ++e) {
      const int stage = (nk + e) & 1;
      const int buf = (ngroups + e) & 1;
      if (e + 1 < nx2) {
#pragma unroll
        for (int i = 0; i < AI; ++i) issue_a(nk + e + 1, stage ^ 1, i);
#pragma unroll
        for (int sh = 0; sh < 5; ++sh) issue_x2(e + 1, buf ^ 1, sh);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        typename K::frag b4[4];
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          b4[fn] = *reinterpret_cast<const typename K::frag*>(smem + b_base[0][u] + buf * kStripBytes + fn * 2048);
#pragma unroll
        for (int qg = 0; qg < GR; ++qg) {
          typename K::frag a2[2];
#pragma unroll
          for (int h = 0; h < 2; ++h)
            a2[h] = *reinterpret_cast<const typename K::frag*>(smem + a_base[u] + stage * AB + (qg * 2 + h) * 2048);
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int fn = 0; fn < 4; ++fn) acc[qg * 2 + h][fn] = K::mma(a2[h], b4[fn], acc[qg * 2 + h][fn]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped re-fetches
  if constexpr (SEGF && K::ESZ == 1) {
    static_assert(!X2 && WCO == 128, "seg fusion: the 256-channel int8 tile");
    int accv[FM][4][4];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < 4; ++fn)
#pragma unroll
        for (int e = 0; e < 4; ++e) accv[fm][fn][e] = acc[fm][fn][e];
    stag_seg_i8<FM>(p, accv, px0, co0, wc, wp, fr, fq, sf, smem);
    return;
  } else if constexpr (SEGF) {
    // the activation as store_tile_x4 would store it (ReLU, RNE to bf16, 16-B pieces: lane
    // (fr, fq) holds channels 8 s(fq) .. +7 of 32-channel group f2 of pixel fr) is the B operand of
    // the seg GEMM, the A fragments the matching seg weight columns; then the two channel halves
    // of the tile (waves wc = 0, 1) are added in that order through LDS
    static_assert(K::ESZ == 2 && !X2 && WCO == 128, "seg fusion: the 256-channel bf16 tile");
    bf16x8 aw[2][FM / 2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int f2 = 0; f2 < FM / 2; ++f2)
        aw[mt][f2] = *reinterpret_cast<const bf16x8*>(static_cast<const uint16_t*>(sf.w) + static_cast<int64_t>(16 * mt + fr) * sf.k_pad + co0 + wc * WCO +
                                                      32 * f2 + chunk_of_row(fq) * 8);
    const bool relu = p.relu != 0;
    f32x4 pacc[2][4];
#pragma unroll
    for (int fn = 0; fn < 4; ++fn) {
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
    // every wave is past its last fragment read (the loop's last barriers): the LDS is free
    float4* xch = reinterpret_cast<float4*>(smem) + (wp * 64 + lane) * 8;
    if (wc == 1) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) xch[mt * 4 + fn] = make_float4(pacc[mt][fn][0], pacc[mt][fn][1], pacc[mt][fn][2], pacc[mt][fn][3]);
    }
    __syncthreads();
    if (wc == 0) {
      const int M = p.n * p.ho * p.wo;
      float* __restrict__ part = static_cast<float*>(sf.part) + static_cast<int64_t>(co0 / (2 * WCO)) * M * kSegCS;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int cls = 16 * mt + 4 * fq;
        if (cls >= kSegCS) continue;
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) {
          const float4 o = xch[mt * 4 + fn];
          const int64_t m = px0 + wp * 64 + fn * 16 + fr;
          *reinterpret_cast<float4*>(part + m * kSegCS + cls) =
              make_float4(pacc[mt][fn][0] + o.x, pacc[mt][fn][1] + o.y, pacc[mt][fn][2] + o.z, pacc[mt][fn][3] + o.w);
        }
      }
    }
    return;
  }
  if constexpr (K::ESZ == 2) {
    if (fast_epi) store_tile_x4<FM, WCO, 4>(p, acc, px0, co0, wc, wp, fr, fq);
    else store_tile<FM, WCO, 4, false>(p, acc, px0, co0, wc, wp, fr, fq);
  } else {
    // whole tile of a dense int8 NHWC output (M % 256 == 0 here): 16-B pieces
    if (p.out_dtype == DRNMI_I8 && p.y_sc == 1 && p.y_sp == p.cout && p.y_sn == static_cast<int64_t>(hw_o) * p.cout &&
        p.cout % BCO == 0 && (p.res == nullptr || p.cout % 16 == 0))
      store_tile_i8_x4<FM, WCO, 4>(p, acc, px0, co0, wc, wp, fr, fq);
    else
      store_tile_i8<FM, WCO, 4>(p, acc, px0, co0, wc, wp, fr, fq);
  }
}

__global__ void __launch_bounds__(512, 1)
conv_stag_kernel(const drnmi_conv_args p) {
  conv_stag_body<uint16_t, false>(p);
}

// W8A8 (config C5): int8 rows of 128 channels are 128 B, the bf16 layout; v_mfma_i32_16x16x64_i8,
// store_tile_i8 epilogue (bit-exact against oracle/int8_oracle.py like conv_i8_strip_kernel)
__global__ void __launch_bounds__(512, 1)
conv_i8_stag_kernel(const drnmi_conv_args p) {
  conv_stag_body<int8_t, false>(p);
}

// the 128-channel tile (D-22 layer4: 128 -> 128, with the fused 1x1 stride-2 downsample in
// layer4.0 conv2)
__global__ void __launch_bounds__(512, 1)
conv_stag128_kernel(const drnmi_conv_args p) {
  conv_stag_body<uint16_t, false, 64>(p);
}
__global__ void __launch_bounds__(512, 1)
conv_stag128_x2_kernel(const drnmi_conv_args p) {
  conv_stag_body<uint16_t, true, 64>(p);
}

struct StagSegArgs {
  drnmi_conv_args p;
  SegFuse sf;
};
__global__ void __launch_bounds__(512, 1)
conv_stag_seg_kernel(const StagSegArgs a) {
  conv_stag_body<uint16_t, false, 128, true>(a.p, a.sf);
}
__global__ void __launch_bounds__(512, 1)
conv_i8_stag_seg_kernel(const StagSegArgs a) {
  conv_stag_body<int8_t, false, 128, true>(a.p, a.sf);
}

// + the fused 1x1 downsample (x2 != NULL; layer5.0 / layer6.0 conv2 of D-22)
__global__ void __launch_bounds__(512, 1)
conv_stag_x2_kernel(const drnmi_conv_args p) {
  conv_stag_body<uint16_t, true>(p);
}

}  // namespace

constexpr int kStagLds = 2 * 256 * 128 + 2 * kStripBytes;     // 2 A stages + 2 strips (130 KB)
constexpr int kStag128Lds = 2 * 128 * 128 + 2 * kStripBytes;  // 128-channel tile (98 KB)

hipError_t launch_stag_seg(const drnmi_conv_args& p, const void* seg_w, int seg_k_pad, void* part, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    for (const void* f : {reinterpret_cast<const void*>(&conv_stag_seg_kernel), reinterpret_cast<const void*>(&conv_i8_stag_seg_kernel)}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kStagLds);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  StagSegArgs a;
  a.p = p;
  a.sf = SegFuse{seg_w, seg_k_pad, part};
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const dim3 grid(static_cast<unsigned>((M / kBPX) * ((p.cout + 255) / 256)));
  if (p.dtype == DRNMI_I8) hipLaunchKernelGGL(conv_i8_stag_seg_kernel, grid, dim3(512), kStagLds, s, a);
  else hipLaunchKernelGGL(conv_stag_seg_kernel, grid, dim3(512), kStagLds, s, a);
  return hipGetLastError();
}

hipError_t launch_stag(const drnmi_conv_args& p, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    for (const void* f : {reinterpret_cast<const void*>(&conv_stag_kernel), reinterpret_cast<const void*>(&conv_stag_x2_kernel),
                          reinterpret_cast<const void*>(&conv_i8_stag_kernel)}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kStagLds);
      if (e != hipSuccess) return e;
    }
    for (const void* f : {reinterpret_cast<const void*>(&conv_stag128_kernel), reinterpret_cast<const void*>(&conv_stag128_x2_kernel)}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kStag128Lds);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const dim3 grid(static_cast<unsigned>((M / kBPX) * ((p.cout + 255) / 256)));
  if (p.dtype != DRNMI_I8 && p.cout <= 128) {
    const dim3 g128(static_cast<unsigned>((M / kBPX) * ((p.cout + 127) / 128)));
    if (p.x2 != nullptr) hipLaunchKernelGGL(conv_stag128_x2_kernel, g128, dim3(512), kStag128Lds, s, p);
    else hipLaunchKernelGGL(conv_stag128_kernel, g128, dim3(512), kStag128Lds, s, p);
  } else if (p.dtype == DRNMI_I8) {
    hipLaunchKernelGGL(conv_i8_stag_kernel, grid, dim3(512), kStagLds, s, p);
  } else if (p.x2 != nullptr) {
    hipLaunchKernelGGL(conv_stag_x2_kernel, grid, dim3(512), kStagLds, s, p);
  } else {
    hipLaunchKernelGGL(conv_stag_kernel, grid, dim3(512), kStagLds, s, p);
  }
  return hipGetLastError();
}

}  // namespace drnmi
