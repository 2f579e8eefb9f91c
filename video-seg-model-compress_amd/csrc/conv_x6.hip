// fp32-accurate NHWC implicit-GEMM convolution on the bf16 MFMA pipe ("fp32x" precision mode).
//
// The north star's parity gate (logits within 1e-3 of the reference PyTorch-CPU fp32 forward,
// argmax maps bit-exact) needs fp32-class arithmetic; bf16 misses it (98.4 %
// argmax agreement) and the f32-input MFMA runs at 1/16 of the bf16 rate (157 TF).  Here every
// fp32 operand is split exactly into three bf16 terms, x = x1 + x2 + x3 (x1 = bf16(x),
// x2 = bf16(x - x1), x3 = bf16(x - x1 - x2): 24 significant bits, the fp32 significand), and
// the product is formed from the six terms above 2^-24:
//     x*w ~ x1 w1 + (x1 w2 + x2 w1) + (x1 w3 + x2 w2 + x3 w1)
// with fp32 accumulation in v_mfma_f32_16x16x32_bf16 — six bf16 MFMAs per fp32 product, 417 TF
// of fp32-accurate peak (2.65x the f32 MFMA).  The dropped terms are < 2^-24 relative: the
// result is as close to exact as an fp32 FMA chain (measured on the DRN-D goldens: see DESIGN.md).
//
// Serves every conv with cin >= 32 and ks 1/3 in fp32x mode (layer3..8 3x3 convs at dilation
// 1/2/4, the 1x1 downsamples, seg 1x1 + bias; lmodels/drn.py:27-29, :49-65, :86-106,
// :181-186, :201-211, lmodels/drnseg.py:278-284).
//
//   * Weights are pre-split on the host side of the plan: [3][cout_pad][k_pad] bf16 planes.
//   * Activations stay fp32 NHWC in HBM (the fp32 mode's layout); each pixel row of the B tile
//     lands in LDS as fp32 (LDS-DMA, per-lane im2col source addresses, zero page for padding)
//     and is split into its three bf16 fragments in registers right after the fragment read —
//     one split per B fragment feeds FM x 6 MFMAs, so the VALU work hides under the MFMAs.
//   * K step = 32 input channels of one tap; tile = BCO output channels x 256 pixels; each wave
//     owns WCO channels x 64 pixels (FM x 4 fragments); LDS rows XOR-swizzled on the DMA source
//     and on the fragment read; NST-stage ring with counted vmcnt + raw s_barrier; tiles dealt
//     XCD-major.
//   * Epilogue in fp32: v = acc * scale + shift (+ residual), ReLU, fp32 NHWC (or the strided
//     fp32 NCHW seg logits).
#include "common.h"
#include "kernels.h"

namespace drnmi {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_void_t;

__device__ uint4 g_x6_zero[64];   // zero-initialised: the source of padded taps / rows


constexpr int kBK = 32;     // input channels per K step

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// bf16 A rows (64 B): conflict-free for every ds_read_b128 lane group (conv_big.hip swzb<64>)
__device__ __forceinline__ int swz64(int row, int chunk) { return chunk ^ (((row >> 3) & 1) * 3); }
__device__ __forceinline__ int swz128(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }   // fp32 B rows


// x from the lane DPP control CTRL selects, as two 32-bit DPP moves
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(u & 0xffffffffu), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
}
// sum over the 16 lanes of a DPP row, the same in every lane: quad_perm xor 1, xor 2, then
// row_half_mirror (quads 0 <-> 1) and row_mirror (halves) -- a fixed order, ALU only (the
// ds_bpermute form of __shfl_xor cost the short-K launches ~10 % in their epilogue)
__device__ __forceinline__ double row16_sum(double x) {
  x += dpp_f64<0xB1>(x);    // quad_perm [1, 0, 3, 2]
  x += dpp_f64<0x4E>(x);    // quad_perm [2, 3, 0, 1]
  x += dpp_f64<0x141>(x);   // row_half_mirror
  x += dpp_f64<0x140>(x);   // row_mirror
  return x;
}

// one ds_read_b128 at LDS byte address base + OFF (smem is the kernel's only LDS object: byte 0)
template <int OFF, typename V>
__device__ __forceinline__ void ds_rd(V& dst, uint32_t base) {
  static_assert(sizeof(V) == 16 && OFF >= 0 && OFF < 65536, "ds_read_b128 offset");
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(OFF));
}

// Tile = BCO = WCO x WC output channels x BPX = 64 x PS pixels; one wave per (channel column,
// 64-pixel slice).  PS = 4: one workgroup per CU (2- or 3-stage ring in up to 160 KB of LDS);
// PS = 2: a 128 x 128 tile of four waves in <= 80 KB, two workgroups per CU (their barriers
// interleave, and the short-K 1/8-resolution launches get twice the tiles).
template <int WCO, int WC, int PS>
struct X6Cfg {
  static constexpr int BCO = WCO * WC;
  static constexpr int BPX = 64 * PS;
  static constexpr int FM = WCO / 16;
  static constexpr int FN = 4;
  static constexpr int NW = PS * WC;
  static constexpr int THREADS = 64 * NW;
  static constexpr int OCC = PS == 2 ? 2 : 1;       // workgroups per CU the LDS ring is sized for
  static constexpr int A_PLANE = BCO * 64;          // one bf16 plane: BCO rows x 32 K x 2 B
  static constexpr int A_BYTES = 3 * A_PLANE;
  static constexpr int B_BYTES = BPX * 128;         // BPX pixel rows x 32 ch x 4 B
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_PW = A_BYTES / 1024 / NW;  // 1-KB DMA pieces per wave per step
  static constexpr int B_PW = B_BYTES / 1024 / NW;
  static constexpr int GLDS = A_PW + B_PW;
  static constexpr int NST = 3 * STAGE * OCC <= 160 * 1024 ? 3 : 2;
  static constexpr int LDS = NST * STAGE;
  static_assert(A_PW * NW * 1024 == A_BYTES && B_PW * NW * 1024 == B_BYTES, "DMA split");
  static_assert(LDS * OCC <= 160 * 1024, "LDS");
};

template <int KS, int WCO, int WC, int PS>
__global__ void __launch_bounds__(64 * PS * WC, PS == 2 ? 2 : 1)   // X6Cfg::OCC
conv_x6_kernel(const drnmi_conv_args p) {
  using C = X6Cfg<WCO, WC, PS>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wc = wave / PS;          // channel column of the tile
  const int wp = wave % PS;          // 64-pixel slice of the tile
  const int fr = lane & 15;
  const int fq = lane >> 4;
  const int M = p.n * p.ho * p.wo;
  const int hw_o = p.ho * p.wo;
  const int nco = (p.cout + C::BCO - 1) / C::BCO;
  const int npx = (M + C::BPX - 1) / C::BPX;
  const int tile = xcd_remap(blockIdx.x, npx * nco);
  const int px0 = (tile / nco) * C::BPX;
  const int co0 = (tile % nco) * C::BCO;

  const int cin = p.cin;
  const int lc = 31 - __builtin_clz(cin);
  const int H = p.h, W = p.w, dil = p.dil;
  const float* __restrict__ x = reinterpret_cast<const float*>(p.x);
  const uint16_t* __restrict__ wt = reinterpret_cast<const uint16_t*>(p.wgt);
  const int64_t plane_stride = static_cast<int64_t>(p.cout_pad) * p.k_pad;
  // split-K (gridDim.y > 1, drnmi_conv_args.ws): this workgroup runs K steps [kt0, kt0 + nk)
  const int nk_all = p.k_pad / kBK;
  const int kt0 = static_cast<int>(static_cast<int64_t>(nk_all) * blockIdx.y / gridDim.y);
  const int nk = static_cast<int>(static_cast<int64_t>(nk_all) * (blockIdx.y + 1) / gridDim.y) - kt0;
  const char* zero_src = reinterpret_cast<const char*>(g_x6_zero) + lane * 16;

  // --- A pieces: 16 rows of 64 B each; linear row R = plane * BCO + r
  // element offsets < 2^31: 3 planes x cout_pad x k_pad bf16 (x6_conv_dispatch checks)
  int32_t a_off[C::A_PW];
#pragma unroll
  for (int i = 0; i < C::A_PW; ++i) {
    const int R = (wave * C::A_PW + i) * 16 + (lane >> 2);
    const int pl = R / C::BCO, r = R - pl * C::BCO;
    a_off[i] = static_cast<int32_t>(pl * plane_stride + static_cast<int64_t>(co0 + r) * p.k_pad + swz64(r, lane & 3) * 8);
  }
  // --- B pieces: 8 pixel rows of 128 B; (ih0, iw0) of tap (0,0) and the element offset of the
  // row's chunk at that tap (only dereferenced when the tap is inside the image)
  int b_ih[C::B_PW], b_iw[C::B_PW], b_off[C::B_PW];
#pragma unroll
  for (int j = 0; j < C::B_PW; ++j) {
    const int r = (wave * C::B_PW + j) * 8 + (lane >> 3);
    const int m = px0 + r;
    b_ih[j] = -(1 << 28);
    b_iw[j] = -(1 << 28);
    b_off[j] = 0;
    if (m < M) {
      const int n = m / hw_o;
      const int q = m - n * hw_o;
      const int oh = q / p.wo;
      const int ow = q - oh * p.wo;
      b_ih[j] = oh * p.stride - p.pad;
      b_iw[j] = ow * p.stride - p.pad;
      b_off[j] = ((n * H + b_ih[j]) * W + b_iw[j]) * cin + swz128(r, lane & 7) * 4;
    }
  }

  // one DMA piece ("instruction") of K step kt: pieces [0, A_PW) weights, then pixel rows
  struct StepP { int k0, dh, dw, toff; };
  auto step_params = [&](int u) {
    const int kt = kt0 + u;
    StepP sp;
    const int cb = kt / (KS * KS);
    const int tap = kt - cb * (KS * KS);
    sp.k0 = (tap << lc) + cb * kBK;
    sp.dh = (tap / KS) * dil;
    sp.dw = (tap - (tap / KS) * KS) * dil;
    sp.toff = (sp.dh * W + sp.dw) * cin + cb * kBK;
    return sp;
  };
  auto issue_piece = [&](const StepP& sp, int stage, int i) {
    char* sa = smem + stage * C::STAGE;
    if (i < C::A_PW) {
      glds16(wt + (static_cast<uint32_t>(a_off[i]) + sp.k0), sa + (wave * C::A_PW + i) * 1024);
    } else {
      const int j = i - C::A_PW;
      const bool ok = static_cast<unsigned>(b_ih[j] + sp.dh) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(b_iw[j] + sp.dw) < static_cast<unsigned>(W);
      const void* src = ok ? static_cast<const void*>(x + (b_off[j] + sp.toff)) : static_cast<const void*>(zero_src);
      glds16(src, sa + C::A_BYTES + (wave * C::B_PW + j) * 1024);
    }
  };
  auto issue = [&](int kt, int stage) {
    const StepP sp = step_params(kt);
#pragma unroll
    for (int i = 0; i < C::GLDS; ++i) issue_piece(sp, stage, i);
  };

  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int t = 0; t < C::NST - 1 && t < nk; ++t) issue(t, t);

  const uint32_t a_lane = static_cast<uint32_t>((wc * WCO + fr) * 64 + swz64(fr, fq) * 16);
  const uint32_t b_lane0 = static_cast<uint32_t>((wp * 64 + fr) * 128 + swz128(fr, 2 * fq) * 16);
  const uint32_t b_lane1 = static_cast<uint32_t>((wp * 64 + fr) * 128 + swz128(fr, 2 * fq + 1) * 16);
  // A plane `pl` of fragment fm: rows fm * 16 apart keep the swizzle (swz64 reads row bit 3 only)
  auto ds_rd_fm = [&](bf16x8& dst, uint32_t base, int fm, int pl) {
    switch (fm * 3 + pl) {
#define X6_RD(I) case I: ds_rd<(I / 3) * 1024 + (I % 3) * C::A_PLANE>(dst, base); break;
      X6_RD(0) X6_RD(1) X6_RD(2) X6_RD(3) X6_RD(4) X6_RD(5) X6_RD(6) X6_RD(7) X6_RD(8) X6_RD(9) X6_RD(10)
      X6_RD(11) X6_RD(12) X6_RD(13) X6_RD(14) X6_RD(15) X6_RD(16) X6_RD(17) X6_RD(18) X6_RD(19) X6_RD(20)
      X6_RD(21) X6_RD(22) X6_RD(23)
#undef X6_RD
      default: break;
    }
  };
  // per step (each accumulator keeps the six products in the order below, so results are
  // bit-identical to the unpipelined form): B fragments are read and split once (splitting b2 / b3
  // under fm 0's first groups instead spilled 9 VGPRs); the three A
  // planes of fragment fm + 1 are read while fm's MFMAs run, each into the registers a group of
  // fm has just retired (plane 3 after group 1, plane 2 after group 4, plane 1 after group 6),
  // 8-20 MFMAs ahead of their first use
  constexpr int PPF = (C::GLDS + C::FM - 1) / C::FM;
  for (int t = 0; t < nk; ++t) {
    const int newer = ((nk - 1) < (t + C::NST - 2) ? (nk - 1) : (t + C::NST - 2)) - t;
    if (C::NST >= 3 && newer >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(C::GLDS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const bool nxt = t + C::NST - 1 < nk;
    const StepP spn = step_params(nxt ? t + C::NST - 1 : t);
    const int nst = (t + C::NST - 1) % C::NST;

    // A fragment reads as inline-asm ds_read_b128 with compile-time offsets (the swizzle does not
    // depend on fm) and hand-counted lgkmcnt waits: hipcc's own waits drained every read in flight
    // before each group (lgkmcnt(0))
    const uint32_t st_off = static_cast<uint32_t>((t % C::NST) * C::STAGE);
    const uint32_t va = a_lane + st_off, vb0 = b_lane0 + st_off, vb1 = b_lane1 + st_off;
    bf16x8 a3, a2, a1;
    ds_rd<2 * C::A_PLANE>(a3, va);                     // fragment 0's planes, then the B rows
    ds_rd<C::A_PLANE>(a2, va);
    ds_rd<0>(a1, va);
    // the B rows as inline-asm reads too, so fragment fn's pair is waited for alone (fm 0's first
    // three groups run interleaved with the splits below, on each pair as it lands, instead of
    // after an lgkmcnt(0) for all eleven reads: the step's opening burst of LDS reads no longer
    // idles the matrix pipe until its last read returns)
    f32x4 blo[C::FN], bhi[C::FN];
    static_assert(C::FN == 4, "four B fragments");
    ds_rd<C::A_BYTES + 0 * 2048>(blo[0], vb0);
    ds_rd<C::A_BYTES + 0 * 2048>(bhi[0], vb1);
    ds_rd<C::A_BYTES + 1 * 2048>(blo[1], vb0);
    ds_rd<C::A_BYTES + 1 * 2048>(bhi[1], vb1);
    ds_rd<C::A_BYTES + 2 * 2048>(blo[2], vb0);
    ds_rd<C::A_BYTES + 2 * 2048>(bhi[2], vb1);
    ds_rd<C::A_BYTES + 3 * 2048>(blo[3], vb0);
    ds_rd<C::A_BYTES + 3 * 2048>(bhi[3], vb1);
    __builtin_amdgcn_sched_barrier(0);
    // split passes: u1 = bf16(x), u2 = bf16(x - u1), u3 = bf16(x - u1 - u2) (common.h split3)
    bf16x8 b1[C::FN], b2[C::FN], b3[C::FN];
    auto pairs = [&](int fn, int i) {
      const f32x4& v = i < 2 ? blo[fn] : bhi[fn];
      return (i & 1) ? f32x2_t{v.z, v.w} : f32x2_t{v.x, v.y};
    };
    auto split_b1 = [&](int fn) {
      uint32_t u[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) u[i] = pk_bf16x2(pairs(fn, i));
      b1[fn] = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
    };
    auto split_b2 = [&](int fn) {
      const uint4 w1 = __builtin_bit_cast(uint4, b1[fn]);
      const uint32_t v1[4] = {w1.x, w1.y, w1.z, w1.w};
      uint32_t u[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) u[i] = pk_bf16x2(pairs(fn, i) - widen_bf16x2(v1[i]));
      b2[fn] = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
    };
    auto split_b3 = [&](int fn) {
      const uint4 w1 = __builtin_bit_cast(uint4, b1[fn]);
      const uint4 w2 = __builtin_bit_cast(uint4, b2[fn]);
      const uint32_t v1[4] = {w1.x, w1.y, w1.z, w1.w};
      const uint32_t v2[4] = {w2.x, w2.y, w2.z, w2.w};
      uint32_t u[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) u[i] = pk_bf16x2((pairs(fn, i) - widen_bf16x2(v1[i])) - widen_bf16x2(v2[i]));
      b3[fn] = __builtin_bit_cast(bf16x8, make_uint4(u[0], u[1], u[2], u[3]));
    };
    auto grp = [&](int fm, const bf16x8& a, const bf16x8 (&b)[C::FN]) {
#pragma unroll
      for (int fn = 0; fn < C::FN; ++fn) acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[fn], acc[fm][fn], 0, 0, 0);
    };
    // fm 0's group 1 on each B pair as it lands (the reads return in issue order: a3 a2 a1, then
    // the pairs), then its groups 2 / 3 with the b2 / b3 splits of each fragment just ahead of
    // its MFMA; every accumulator keeps its product order
    auto b_wait = [&](auto fn_c) {
      constexpr int FNI = decltype(fn_c)::value;
      // the wait redefines the pair (an asm output): no use of it can be hoisted above the wait
      // (a plain asm wait let the compiler convert all four pairs right after the first one)
      asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(blo[FNI]), "+v"(bhi[FNI]) : "n"(2 * (C::FN - 1 - FNI)) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      split_b1(FNI);
      acc[0][FNI] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3, b1[FNI], acc[0][FNI], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);               // the MFMA goes out before the next wait
    };
#pragma unroll
    for (int fm = 0; fm < C::FM; ++fm) {
      // read order per fragment: a3(fm) after group 1 of fm - 1, a2(fm) after its group 4, a1(fm)
      // after its group 6 (each into the registers that group retired); before group 1 the
      // newer reads in flight are a2(fm), a1(fm)
      if (fm == 0) {
        b_wait(std::integral_constant<int, 0>{});
        b_wait(std::integral_constant<int, 1>{});
        b_wait(std::integral_constant<int, 2>{});
        b_wait(std::integral_constant<int, 3>{});       // 1: a3 b1, every B read landed
      } else {
        asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        grp(fm, a3, b1);                                 // 1: a3 b1
      }
      if (fm + 1 < C::FM) ds_rd_fm(a3, va, fm + 1, 2);
      // branch-free (a branch here let the reads above sink past it, next to their MFMAs): the
      // last step re-fetches its own K step into the stage step t - 1 used, which nobody reads
#pragma unroll
      for (int k = 0; k < PPF; ++k)
        if (fm * PPF + k < C::GLDS) issue_piece(spn, nst, fm * PPF + k);
      // a2(fm) landed: newer in flight a1(fm), a3(fm + 1)
      if (fm + 1 < C::FM) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (fm == 0) {
#pragma unroll
        for (int fn = 0; fn < C::FN; ++fn) {             // 2: a2 b2
          split_b2(fn);
          acc[0][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b2[fn], acc[0][fn], 0, 0, 0);
        }
      } else {
        grp(fm, a2, b2);                                 // 2: a2 b2
      }
      // a1(fm) landed: newer in flight a3(fm + 1)
      if (fm + 1 < C::FM) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (fm == 0) {
#pragma unroll
        for (int fn = 0; fn < C::FN; ++fn) {             // 3: a1 b3
          split_b3(fn);
          acc[0][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b3[fn], acc[0][fn], 0, 0, 0);
        }
      } else {
        grp(fm, a1, b3);                                 // 3: a1 b3
      }
      __builtin_amdgcn_sched_barrier(0);
      grp(fm, a2, b1);                                   // 4: a2 b1
      if (fm + 1 < C::FM) ds_rd_fm(a2, va, fm + 1, 1);
      __builtin_amdgcn_sched_barrier(0);
      grp(fm, a1, b2);                                   // 5: a1 b2
      __builtin_amdgcn_sched_barrier(0);
      grp(fm, a1, b1);                                   // 6: a1 b1
      if (fm + 1 < C::FM) ds_rd_fm(a1, va, fm + 1, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the last step's re-fetch

  // --- split-K: raw fp32 partial sums [split][m][cout]; x6_splitk_epilogue_kernel finishes
  if (gridDim.y > 1) {
    float* __restrict__ part = reinterpret_cast<float*>(p.ws) + static_cast<int64_t>(blockIdx.y) * M * p.cout;
#pragma unroll
    for (int fn = 0; fn < C::FN; ++fn) {
      const int m = px0 + wp * 64 + fn * 16 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int fm = 0; fm < C::FM; ++fm) {
        const int co = co0 + wc * WCO + fm * 16 + fq * 4;
        if (co >= p.cout) continue;
        float* q = part + static_cast<int64_t>(m) * p.cout + co;
        if (co + 3 < p.cout) {
          *reinterpret_cast<float4*>(q) = make_float4(acc[fm][fn][0], acc[fm][fn][1], acc[fm][fn][2], acc[fm][fn][3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (co + j < p.cout) q[j] = acc[fm][fn][j];
        }
      }
    }
    return;
  }

  // --- epilogue: lane owns channels co..co+3 of pixel m, fp32
  const float* __restrict__ res = reinterpret_cast<const float*>(p.res);
  const bool nhwc = p.y_sc == 1;
  // the lane's output row offsets, one per pixel fragment (-1: past the last pixel)
  int64_t ybase_fn[C::FN];
#pragma unroll
  for (int fn = 0; fn < C::FN; ++fn) {
    const int m = px0 + wp * 64 + fn * 16 + fr;
    const int n = m / hw_o;
    const int q = m - n * hw_o;
    const int64_t qo = p.y_sr != 0 ? static_cast<int64_t>(q / p.wo) * p.y_sr + static_cast<int64_t>(q % p.wo) * p.y_sp
                                   : static_cast<int64_t>(q) * p.y_sp;
    ybase_fn[fn] = m < M ? static_cast<int64_t>(n) * p.y_sn + qo : -1;
  }
  // one (fragment fm, pixel fragment fn) of the lane: v = acc * scale + shift (+ res), ReLU,
  // stored; false when the pixel or the channel group lies outside the output
  auto epi = [&](int fm, int fn, float (&v)[4]) -> bool {
    const int m = px0 + wp * 64 + fn * 16 + fr;
    const int co = co0 + wc * WCO + fm * 16 + fq * 4;
    const int64_t ybase = ybase_fn[fn];
    if (ybase < 0 || co >= p.cout) return false;
    const bool full = co + 3 < p.cout;
    const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);   // padded to cout_pad
    v[0] = acc[fm][fn][0];
    v[1] = acc[fm][fn][1];
    v[2] = acc[fm][fn][2];
    v[3] = acc[fm][fn][3];
    if (p.scale != nullptr) {
      const float4 sc = *reinterpret_cast<const float4*>(p.scale + co);
      v[0] = v[0] * sc.x + sh.x;
      v[1] = v[1] * sc.y + sh.y;
      v[2] = v[2] * sc.z + sh.z;
      v[3] = v[3] * sc.w + sh.w;
    } else {
      v[0] += sh.x;
      v[1] += sh.y;
      v[2] += sh.z;
      v[3] += sh.w;
    }
    if (res != nullptr) {
      const float* rp = res + (p.y_sr != 0 ? ybase : static_cast<int64_t>(m) * p.cout) + co;   // y_sr: y's layout
      if (full) {
        const float4 rv = *reinterpret_cast<const float4*>(rp);
        v[0] += rv.x;
        v[1] += rv.y;
        v[2] += rv.z;
        v[3] += rv.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (co + j < p.cout) v[j] += rp[j];
      }
    }
    if (p.relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    float* y = reinterpret_cast<float*>(p.y);
    if (nhwc && full) {
      *reinterpret_cast<float4*>(y + ybase + co) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (co + j < p.cout) y[ybase + static_cast<int64_t>(co + j) * p.y_sc] = v[j];
    }
    return true;
  };
  if (p.stats == nullptr) {
#pragma unroll
    for (int fn = 0; fn < C::FN; ++fn)
#pragma unroll
      for (int fm = 0; fm < C::FM; ++fm) {
        float v[4];
        epi(fm, fn, v);
      }
    return;
  }
  // BN statistics of the stored values (drnmi_conv_args.stats): per channel fragment, the lane's
  // four pixels in fp64, then a fixed xor tree over the 16 lanes of its pixel column; row g = this
  // wave's 64-pixel slice, [2][G][cout] (sums, then sums of squares)
  const int G = npx * PS;
  const int g = (tile / nco) * PS + wp;
#pragma unroll
  for (int fm = 0; fm < C::FM; ++fm) {
    double a1[4] = {0, 0, 0, 0}, a2[4] = {0, 0, 0, 0};
#pragma unroll
    for (int fn = 0; fn < C::FN; ++fn) {
      float v[4];
      if (epi(fm, fn, v)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a1[j] += static_cast<double>(v[j]);
          a2[j] += static_cast<double>(v[j]) * v[j];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a1[j] = row16_sum(a1[j]);
      a2[j] = row16_sum(a2[j]);
    }
    const int co = co0 + wc * WCO + fm * 16 + fq * 4;
    if (fr == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (co + j < p.cout) {
          p.stats[static_cast<int64_t>(g) * p.cout + co + j] = a1[j];
          p.stats[static_cast<int64_t>(G + g) * p.cout + co + j] = a2[j];
        }
    }
  }
}

// split-K finish: v = sum of the partials in split order, then conv_x6's epilogue (scale / shift,
// residual, ReLU, NHWC or strided store); one thread per 4 channels of a pixel.  y and res may
// alias (the fp32x data gradient accumulates the residual gradient in place: out = res = prev):
// every element is read and then written by the same thread, so neither pointer is __restrict__.
__global__ void __launch_bounds__(256) x6_splitk_epilogue_kernel(const drnmi_conv_args p, int splits) {
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int c4 = (p.cout + 3) / 4;
  const int64_t total = M * c4;
  const float* __restrict__ part = reinterpret_cast<const float*>(p.ws);
  const float* res = reinterpret_cast<const float*>(p.res);
  float* y = reinterpret_cast<float*>(p.y);
  const int hw_o = p.ho * p.wo;
  const int64_t pstride = M * p.cout;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t m = i / c4;
    const int co = static_cast<int>(i - m * c4) * 4;
    const bool full = co + 3 < p.cout;
    const int64_t o = m * p.cout + co;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < splits; ++z) {
      if (full) {
        const float4 a = *reinterpret_cast<const float4*>(part + z * pstride + o);
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      } else {
        for (int j = 0; j < 4; ++j)
          if (co + j < p.cout) v[j] += part[z * pstride + o + j];
      }
    }
    const float4 sh = *reinterpret_cast<const float4*>(p.shift + co);
    const float shv[4] = {sh.x, sh.y, sh.z, sh.w};
    if (p.scale != nullptr) {
      const float4 sc = *reinterpret_cast<const float4*>(p.scale + co);
      const float scv[4] = {sc.x, sc.y, sc.z, sc.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = v[j] * scv[j] + shv[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += shv[j];
    }
    const int n = static_cast<int>(m / hw_o);
    const int q = static_cast<int>(m - static_cast<int64_t>(n) * hw_o);
    const int64_t ybase = static_cast<int64_t>(n) * p.y_sn +
                          (p.y_sr != 0 ? static_cast<int64_t>(q / p.wo) * p.y_sr + static_cast<int64_t>(q % p.wo) * p.y_sp
                                       : static_cast<int64_t>(q) * p.y_sp);
    if (res != nullptr) {
      const int64_t ro = p.y_sr != 0 ? ybase + co : o;   // y_sr: the residual has y's layout
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (co + j < p.cout) v[j] += res[ro + j];
    }
    if (p.relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    if (p.y_sc == 1 && full) {
      *reinterpret_cast<float4*>(y + ybase + co) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int j = 0; j < 4; ++j)
        if (co + j < p.cout) y[ybase + static_cast<int64_t>(co + j) * p.y_sc] = v[j];
    }
  }
}

template <int KS, int WCO, int WC, int PS>
hipError_t launch_x6(const drnmi_conv_args& p, int splits, hipStream_t s) {
  using C = X6Cfg<WCO, WC, PS>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_x6_kernel<KS, WCO, WC, PS>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int64_t blocks = ((M + C::BPX - 1) / C::BPX) * ((p.cout + C::BCO - 1) / C::BCO);
  hipLaunchKernelGGL((conv_x6_kernel<KS, WCO, WC, PS>), dim3(static_cast<unsigned>(blocks), splits), dim3(C::THREADS),
                     C::LDS, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || splits == 1) return e;
  const int64_t total = M * ((p.cout + 3) / 4);
  int64_t g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(x6_splitk_epilogue_kernel, dim3(static_cast<unsigned>(g)), dim3(256), 0, s, p, splits);
  return hipGetLastError();
}

// variants: 0 <K, 128, 2, 4> (256 channels x 256 pixels, 8 waves), 1 <K, 128, 1, 4> (128 x 256, 4
// waves), 2 <K, 64, 1, 4> (64 x 256, 4 waves), 3 <K, 64, 2, 4> (128 x 256, 8 waves), 4 <K, 64, 2, 2>
// (128 x 128, 4 waves, two workgroups per CU), 5 <K, 32, 2, 2> (64 x 128, 4 waves of 32 channels,
// two per CU).  A drnmi_conv_args.tile >= 0 forces variant tile % 6 and, when tile >= 6, tile / 6
// split-K partitions (tests, micro-benchmarks; split-K only with a caller workspace).  Every variant
// keeps each accumulator's MFMA order: bit-identical.
constexpr int kNumX6 = 6;
constexpr int kX6Bco[kNumX6] = {256, 128, 64, 128, 128, 64};
constexpr int kX6Bpx[kNumX6] = {256, 256, 256, 256, 128, 128};
constexpr int kX6Occ[kNumX6] = {1, 1, 1, 1, 2, 2};
// seconds per 32-channel K step of one workgroup tile, fitted to scripts/x6_micro.py's sweep on
// the fine-tune shapes (profiles/r8_finetune/x6_micro_variants.txt): the 256 x 256 tile ~4.3 us,
// the 8-wave 128 x 256 ~3.0 us, the two-per-CU 128 x 128 ~2.7 us (its 2.1-3.0 us spread tracks
// how the two resident workgroups overlap; past two rounds the model under-charges it)
constexpr double kX6Step[kNumX6] = {4.3e-6, 3.6e-6, 2.2e-6, 3.0e-6, 2.7e-6, 2.3e-6};
// 128-channel layers take the two-per-CU 128 x 128 tile: D-22 layer4's five launches 1631-1649 ->
// 1510-1568 us against the 8-wave 128 x 256 tile, same box, three interleaved runs each
// (profiles/r9_x6_v5/v4_ab.txt; the 8-wave tile had beaten the 4-wave one, 492 vs 511 us,
// profiles/r7_x6).  64-channel
// layers (and the 19-class seg) take the two-per-CU 64 x 128 tile (eight waves per CU instead of
// four): D-22 layer3 3x3 750 -> 660 us at batch 8, the fine-tune's 1x1 256 -> 64 49 -> 37 us, the
// seg 1x1 512 -> 19 153 -> 142 us (profiles/r9_x6_v5)
int x6_auto_variant(const drnmi_conv_args& p) {
  return p.cout % 256 == 0 ? 0 : p.cout % 128 == 0 ? 4 : p.cout <= 64 ? 5 : 2;
}

int x6_num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// Launch plan (variant, split-K count); split_ok: the launch has (drnmi_conv_args.ws) or is sizing
// (drnmi_conv_workspace_bytes) a caller workspace.  Inference launches (none) take the auto variant
// unsplit.  The fp32x training path (a workspace) picks among the 256- / 128-channel tiles
// and S = 1..4 by a cost model: rounds of resident workgroups x K steps per workgroup x the
// variant's step time, plus the split partials' HBM round trip (S x M x cout fp32 written and
// read) and the output (+ residual) stream.  The default (auto variant, S = 1) is kept unless the
// best plan is >= 5 % faster.  The model is within a few % of the SPLITS sweep (512 -> 512 d4 at
// 2 x 128 x 96: 631 / 580 us modelled for S = 1 / 4, 627 / 580 measured).
struct X6Plan { int v, S; };
X6Plan x6_plan(const drnmi_conv_args& p, bool split_ok) {
  // the partials are [split][m][cout] rows written as float4: only cout % 4 == 0 splits
  if (p.cout % 4 != 0) split_ok = false;
  if (p.tile >= 0) {
    const int v = p.tile % kNumX6;
    int S = p.tile / kNumX6;
    if (!split_ok || S < 1) S = 1;
    if (S > p.k_pad / kBK) S = p.k_pad / kBK;
    return {v, S};
  }
  const int v0 = x6_auto_variant(p);
  if (!split_ok) return {v0, 1};
  const int cus = x6_num_cus();
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  const int nk = p.k_pad / kBK;
  const double out_s = static_cast<double>(M) * p.cout * 4.0 * (p.res != nullptr ? 2 : 1) / 4.5e12;
  auto cost = [&](int v, int S) {
    const int64_t tiles = ((M + kX6Bpx[v] - 1) / kX6Bpx[v]) * ((p.cout + kX6Bco[v] - 1) / kX6Bco[v]);
    const int64_t slots = static_cast<int64_t>(cus) * kX6Occ[v];
    const int64_t rounds = (tiles * S + slots - 1) / slots;
    double t = static_cast<double>(rounds) * ((nk + S - 1) / S) * kX6Step[v] + out_s;
    if (S > 1) t += 2.0 * S * static_cast<double>(M) * p.cout * 4.0 / 4e12 + 4e-6;
    return t;
  };
  const double c0 = cost(v0, 1);
  X6Plan best{v0, 1};
  double bc = c0;
  // Only the auto variant's split counts: with the two-per-CU 128 x 128 tile as a candidate (<= two
  // rounds of it) the plan moved 1/3 of the step's conv_x6 launches onto it and the step's conv_x6
  // time did not move (19.52 -> 19.57 ms, profiles/r8_finetune/x6_plan_v4.txt); variant 4 stays a
  // forced tile for A/B runs.
  const int cands[1] = {v0};
  for (int v : cands) {
    if ((p.cout + kX6Bco[v] - 1) / kX6Bco[v] * kX6Bco[v] > p.cout_pad) continue;
    for (int S = 1; S <= 4 && (S == 1 || nk / S >= 8); ++S) {
      const int64_t tiles = ((M + kX6Bpx[v] - 1) / kX6Bpx[v]) * ((p.cout + kX6Bco[v] - 1) / kX6Bco[v]);
      if (kX6Occ[v] == 2 && tiles * S > 2 * 2 * static_cast<int64_t>(cus)) continue;
      const double c = cost(v, S);
      if (c < 0.95 * c0 && c < bc) {
        best = {v, S};
        bc = c;
      }
    }
  }
  return best;
}
// the workspace a training launch of this geometry needs (its plan with splits allowed); a plan
// that differs from the inference default without splitting asks for a token 256 B, since a
// launch takes the training plan exactly when it is given a workspace
int64_t x6_workspace_bytes(const drnmi_conv_args& p) {
  const X6Plan pl = x6_plan(p, true);
  if (pl.S > 1) return static_cast<int64_t>(pl.S) * p.n * p.ho * p.wo * p.cout * 4;
  return pl.v != x6_plan(p, false).v ? 256 : 0;
}

}  // namespace

bool x6_conv_supported(const drnmi_conv_args& p) {
  return p.dtype == DRNMI_F32X3 && p.out_dtype == DRNMI_F32 && p.cin >= kBK && (p.cin & (p.cin - 1)) == 0 &&
         (p.ks == 1 || p.ks == 2 || p.ks == 3) && p.k == p.ks * p.ks * p.cin && p.k_pad == p.k &&
         static_cast<int64_t>(p.n) * p.h * p.w * p.cin < (int64_t(1) << 31) && p.h < 16384 && p.w < 16384 &&
         (p.y_sc != 1 || p.y_sp == p.cout ||
          (p.y_sr != 0 && p.y_sp % 4 == 0 && p.y_sr % 4 == 0 && p.y_sn % 4 == 0) ||
          // wider NHWC rows (the labels head's 20-float seg logits rows): 16-B aligned, no
          // residual (a residual is read with the output's own packed layout)
          (p.y_sp > p.cout && p.y_sp % 4 == 0 && p.y_sn % 4 == 0 && p.res == nullptr));
}

int64_t x6_conv_workspace_bytes(const drnmi_conv_args& p) {
  return x6_conv_supported(p) ? x6_workspace_bytes(p) : 0;
}

// rows of BN-statistics partials a launch with these arguments writes (0: it cannot -- split K)
int64_t x6_conv_stats_rows(const drnmi_conv_args& p) {
  if (!x6_conv_supported(p)) return 0;
  const X6Plan pl = x6_plan(p, p.ws != nullptr);
  if (pl.S > 1) return 0;
  const int64_t M = static_cast<int64_t>(p.n) * p.ho * p.wo;
  return (M + kX6Bpx[pl.v] - 1) / kX6Bpx[pl.v] * (kX6Bpx[pl.v] / 64);
}

int x6_conv_dispatch(const drnmi_conv_args& p, hipStream_t s) {
  if (!x6_conv_supported(p)) return DRNMI_ENOTSUP;
  const X6Plan pl = x6_plan(p, p.ws != nullptr);
  const int v = pl.v;
  // every weight row a tile's DMA reads must exist in each plane
  if ((p.cout + kX6Bco[v] - 1) / kX6Bco[v] * kX6Bco[v] > p.cout_pad) return DRNMI_EINVAL;
  if (3 * static_cast<int64_t>(p.cout_pad) * p.k_pad >= (int64_t(1) << 31)) return DRNMI_EINVAL;
  const int S = pl.S;
  if (S > 1 && p.stats != nullptr) return DRNMI_EINVAL;   // statistics only from an unsplit launch
  if (p.stats != nullptr && (reinterpret_cast<uintptr_t>(p.stats) & 7) != 0) return DRNMI_EINVAL;
  if (S > 1 && p.ws_bytes < x6_workspace_bytes(p)) return DRNMI_EINVAL;
  if (S > 1 && (reinterpret_cast<uintptr_t>(p.ws) & 15) != 0) return DRNMI_EINVAL;
  hipError_t e;
  if (p.ks == 2) {        // the 2x2 parity-class kernels of a stride-2 conv's data gradient
    switch (v) {
      case 0: e = launch_x6<2, 128, 2, 4>(p, S, s); break;
      case 1: e = launch_x6<2, 128, 1, 4>(p, S, s); break;
      case 2: e = launch_x6<2, 64, 1, 4>(p, S, s); break;
      case 3: e = launch_x6<2, 64, 2, 4>(p, S, s); break;
      case 4: e = launch_x6<2, 64, 2, 2>(p, S, s); break;
      default: e = launch_x6<2, 32, 2, 2>(p, S, s); break;
    }
  } else if (p.ks == 3) {
    switch (v) {
      case 0: e = launch_x6<3, 128, 2, 4>(p, S, s); break;
      case 1: e = launch_x6<3, 128, 1, 4>(p, S, s); break;
      case 2: e = launch_x6<3, 64, 1, 4>(p, S, s); break;
      case 3: e = launch_x6<3, 64, 2, 4>(p, S, s); break;
      case 4: e = launch_x6<3, 64, 2, 2>(p, S, s); break;
      default: e = launch_x6<3, 32, 2, 2>(p, S, s); break;
    }
  } else {
    switch (v) {
      case 0: e = launch_x6<1, 128, 2, 4>(p, S, s); break;
      case 1: e = launch_x6<1, 128, 1, 4>(p, S, s); break;
      case 2: e = launch_x6<1, 64, 1, 4>(p, S, s); break;
      case 3: e = launch_x6<1, 64, 2, 4>(p, S, s); break;
      case 4: e = launch_x6<1, 64, 2, 2>(p, S, s); break;
      default: e = launch_x6<1, 32, 2, 2>(p, S, s); break;
    }
  }
  return static_cast<int>(e);
}

const char* x6_conv_name(const drnmi_conv_args& p) {
  if (!x6_conv_supported(p)) return nullptr;
  static const char* n3[kNumX6] = {"conv_x6_kernel<3, 128, 2, 4>", "conv_x6_kernel<3, 128, 1, 4>",
                                   "conv_x6_kernel<3, 64, 1, 4>", "conv_x6_kernel<3, 64, 2, 4>",
                                   "conv_x6_kernel<3, 64, 2, 2>", "conv_x6_kernel<3, 32, 2, 2>"};
  static const char* n1[kNumX6] = {"conv_x6_kernel<1, 128, 2, 4>", "conv_x6_kernel<1, 128, 1, 4>",
                                   "conv_x6_kernel<1, 64, 1, 4>", "conv_x6_kernel<1, 64, 2, 4>",
                                   "conv_x6_kernel<1, 64, 2, 2>", "conv_x6_kernel<1, 32, 2, 2>"};
  static const char* n2[kNumX6] = {"conv_x6_kernel<2, 128, 2, 4>", "conv_x6_kernel<2, 128, 1, 4>",
                                   "conv_x6_kernel<2, 64, 1, 4>", "conv_x6_kernel<2, 64, 2, 4>",
                                   "conv_x6_kernel<2, 64, 2, 2>", "conv_x6_kernel<2, 32, 2, 2>"};
  const int v = x6_plan(p, p.ws != nullptr).v;
  return p.ks == 3 ? n3[v] : p.ks == 2 ? n2[v] : n1[v];
}

}  // namespace drnmi
