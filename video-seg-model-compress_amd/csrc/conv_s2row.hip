// Row-walking stride-2 3x3 conv (bf16 NHWC, pad 1, BN scale folded): the BasicBlock conv1 of
// DRN-D layer3.0 (32 -> 64) and layer4.0 (64 -> 128) (lmodels/drn.py:27-29 conv3x3, :49-52 with
// stride 2; BN folded from eval running stats).
//
// On conv_big these launches gathered every tap's 256 pixels through an LDS-DMA ring per
// 256-pixel tile: 9 K steps per tile, the ring's fill and the epilogue exposed once per tile
// (121 us / 76 us per D-22 batch-8 step, 3.3 / 2.6 TB/s of algorithmic bytes, against HBM floors of
// ~50 / ~25 us).  Here the work is one read of x and one write of y, streamed:
//   * a workgroup owns an output column strip (OWS = 64 / 32 pixels) of a frame and walks a
//     contiguous range of its output rows; input rows (2 OWS + 1 pixels) arrive by buffer LDS-DMA
//     into a 7-slot ring two steps ahead (step oh reads rows 2 oh - 1 .. 2 oh + 1 and issues rows
//     2 oh + 4, 2 oh + 5), so each input byte crosses HBM once and no tap is re-gathered;
//   * wave (wc, wp) computes output channels 32 wc .. +31 x 32 pixels; its weights (32 rows x
//     9 cin, v_mfma_f32_16x16x32_bf16 A fragments) are loaded once into AGPRs;
//   * pixel rows in LDS: 16-B chunk c of pixel p at granule ((q gpp + c) ^ h(b)) of its 256-B block
//     b (q = p within the block; h(b) = b & 7 for 64-B pixels, 2 b & 15 for 128-B pixels): the
//     stride-2 fragment reads are 2-way (64-B pixels) / conflict-free (128-B pixels);
//   * two workgroups per CU; out-of-image pixels and rows come in as zeros (buffer OOB).
// Per accumulator the K order (32-channel chunks of the packed [cout_pad][9 cin] rows, tap-major),
// the MFMA, the start value (shift) and the epilogue (ReLU, RNE to bf16) are conv_big's BK-32 /
// BK-64 tiles': the output is bit-identical to them (tests/test_gpu_s2row.py).
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

namespace drnmi {
namespace {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// ring depth (input-row slots: 3 in use + 2 per step of DMA lead) and workgroups per CU of the
// cin 32 / cin 64 instantiations
constexpr int kRing32 = 7, kWgs32 = 2, kRing64 = 7, kWgs64 = 2;

constexpr int kSlotB = 9 * 1024;       // input row slot: <= 8448 B used, whole 1-KB DMA pieces
constexpr int kPieces = kSlotB / 1024;
constexpr unsigned kOob = 0x80000000u;
template <int RING>
constexpr int s2_lds_bytes() { return RING * kSlotB + 1024; }   // + slack: reads of discarded columns past a slot, the dummy DMA piece

struct S2Params {
  const uint16_t* x;
  const uint16_t* wgt;
  const float* shift;
  uint16_t* y;
  int n, h, w, ho, wo, k_pad, relu, strips, total, per_wg;
};

template <int CIN>
struct S2Cfg {
  static constexpr int PB = 2 * CIN;             // bytes per input pixel
  static constexpr int GPP = PB / 16;            // 16-B chunks per pixel
  static constexpr int PPB = 256 / PB;           // pixels per 256-B block
  static constexpr int NCW = CIN == 32 ? 2 : 4;  // channel waves (cout = 32 NCW)
  static constexpr int NPW = 4 / NCW;            // pixel waves
  static constexpr int COUT = 32 * NCW;
  static constexpr int OWS = 32 * NPW;           // output columns per strip
  static constexpr int XW = 2 * OWS + 1;         // input columns per strip
  static constexpr int SUBS = CIN / 32;          // 32-channel K chunks per tap
  static constexpr int NKS = 9 * SUBS;           // K chunks
  static constexpr int NE = 2 * NKS;             // (K chunk, pixel fragment) entries per row
  static_assert(XW * PB <= kSlotB - 256, "slot");
};

// LDS byte offset of 16-B chunk c of strip pixel p inside a slot
template <int CIN>
__host__ __device__ __forceinline__ int s2_lds(int p, int c) {
  using C = S2Cfg<CIN>;
  const int b = p / C::PPB, q = p % C::PPB;
  const int h = C::GPP == 4 ? (b & 7) : ((2 * b) & 15);
  return (b << 8) | ((((q * C::GPP) + c) ^ h) << 4);
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int OFF>
__device__ __forceinline__ void ds_rd16(u32x4_t& dst, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(OFF));
}

template <int CIN, int RING, int WGS>
__global__ void __launch_bounds__(256, WGS) __attribute__((amdgpu_waves_per_eu(WGS, WGS)))
conv_s2row_kernel(const S2Params a) {
  using C = S2Cfg<CIN>;
  constexpr int D = (RING - 3) / 2;                  // steps of DMA lead
  static_assert(RING == 3 + 2 * D && D >= 1 && D <= 2, "ring");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wc = wave % C::NCW, wp = wave / C::NCW;
  const int fr = lane & 15, fq = lane >> 4;

  // weights: A fragment (fm, ks) = packed row 32 wc + 16 fm + fr, columns 32 ks + 8 fq .. +7
  // (all loads first, then the AGPR pins: a pin right after each load waits for it)
  u32x4_t wf[C::NKS][2];
#pragma unroll
  for (int ks = 0; ks < C::NKS; ++ks)
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
      wf[ks][fm] = *reinterpret_cast<const u32x4_t*>(a.wgt + static_cast<int64_t>(32 * wc + 16 * fm + fr) * a.k_pad +
                                                     32 * ks + 8 * fq);
  // the AGPR pins wait for every weight load: they come after the first segment's ring-fill DMA
  // is issued, so the weight and input-row latencies overlap (stamps:
  // the fill was 12.2 us of a 40 us workgroup with the pins first, scripts/s2row_stamps.py)
  auto pin_weights = [&]() {
#pragma unroll
    for (int ks = 0; ks < C::NKS; ++ks)
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) asm volatile("" : "+a"(wf[ks][fm]));
  };
  f32x4 cinit[2];
#pragma unroll
  for (int fm = 0; fm < 2; ++fm) {
    const float4 s = *reinterpret_cast<const float4*>(a.shift + 32 * wc + 16 * fm + 4 * fq);
    cinit[fm] = f32x4{s.x, s.y, s.z, s.w};
  }
  const int H = a.h, W = a.w;
  const __amdgpu_buffer_rsrc_t xs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, a.n * H * W * C::PB, 0x00020000);
  const __amdgpu_buffer_rsrc_t ys =
      __builtin_amdgcn_make_buffer_rsrc(a.y, 0, a.n * a.ho * a.wo * C::COUT * 2, 0x00020000);
  typedef __attribute__((address_space(3))) void lds_t;

  // B fragment (fn, kw, sub): output pixel wp 32 + 16 fn + fr -> strip pixel 2 (..) + kw, chunk 4 sub + fq
  uint32_t boff[2][3][C::SUBS];
#pragma unroll
  for (int fn = 0; fn < 2; ++fn)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int sb = 0; sb < C::SUBS; ++sb)
        boff[fn][kw][sb] = static_cast<uint32_t>(s2_lds<CIN>(2 * (32 * wp + 16 * fn + fr) + kw, 4 * sb + fq));
  int idx = blockIdx.x * a.per_wg;
  const int end = min(idx + a.per_wg, a.total);
  // segment state (a run of output rows ya .. yb - 1 of one strip of one image)
  int ya = 0, yb = 0, n = 0, ow0 = 0, img0 = 0;
  uint32_t vo[5];
  const int rowb = W * C::PB;                          // bytes per image row
  auto piece = [&](int k, int r0, int slot0) {         // piece k of rows (r0, r0 + 1); slot0 = slot of r0
    const int i = wave + 4 * k;
    const int dr = i >= kPieces ? 1 : 0;
    const int row = r0 + dr;
    int slot = slot0 + dr;
    slot = slot >= RING ? slot - RING : slot;
    const bool row_ok = static_cast<unsigned>(row) < static_cast<unsigned>(H) && i < 2 * kPieces;
    // wave-uniform by construction; readfirstlane keeps them in SGPRs (a VGPR soffset would
    // make the compiler wrap the load in a waterfall loop)
    const int soff = __builtin_amdgcn_readfirstlane(row_ok ? (img0 + row) * rowb : 0);
    const int dst = __builtin_amdgcn_readfirstlane(i < 2 * kPieces ? slot * kSlotB + (i - dr * kPieces) * 1024 : RING * kSlotB);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xs, (lds_t*)(smem + dst), 16, row_ok ? vo[k] : kOob, soff, 0, 0);
  };
  auto mod_ring = [](int r) { return ((r % RING) + RING) % RING; };
  // next segment: its state and its ring fill, rows 2 ya - 1 .. 2 ya + 2 D (step ya re-issues
  // 2 ya + 2 D: same bytes, no reader yet)
  auto begin_segment = [&]() {
    const int seg = idx / a.ho;
    ya = idx - seg * a.ho;
    yb = min(a.ho, ya + (end - idx));
    idx += yb - ya;
    n = seg / a.strips;
    const int s = seg - n * a.strips;
    ow0 = C::OWS * s;
    const int col0 = 2 * ow0 - 1;                      // image column of strip pixel 0
    img0 = n * H;
    // the 18 DMA pieces of input rows (r0, r0 + 1): wave w issues pieces i = w + 4 k, k < 5 (row
    // i / 9, 1-KB piece i % 9 of its slot); the lane's (pixel, chunk) and the strip/image column
    // test depend only on (k, lane), so the per-step work is a scalar row offset and one select.
    // Waves 2, 3 have no piece 4 (i >= 18): theirs is an all-OOB load into the slack KB after
    // the ring (zeros nobody needs), so every wave issues 5 and the vmcnt counts are uniform.
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int i = wave + 4 * k;
      const int g = (i % kPieces) * 64 + lane;
      const int b = g >> 4;
      const int hb = C::GPP == 4 ? (b & 7) : ((2 * b) & 15);
      const int v = (g & 15) ^ hb;
      const int pp = b * C::PPB + v / C::GPP, c = v % C::GPP;
      const int col = col0 + pp;
      vo[k] = i < 2 * kPieces && pp < C::XW && static_cast<unsigned>(col) < static_cast<unsigned>(W)
                  ? static_cast<unsigned>(col * C::PB + c * 16) : kOob;
    }
#pragma unroll
    for (int r = 0; r <= D; ++r)
#pragma unroll
      for (int k = 0; k < 5; ++k) piece(k, 2 * ya - 1 + 2 * r, mod_ring(2 * ya - 1 + 2 * r));
  };
  bool more = idx < end;
  if (more) begin_segment();
  pin_weights();                                   // waits for the weights only: the fill stays in flight
  while (more) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    int s_lo = mod_ring(2 * ya - 1);                   // slot of row 2 oh - 1
    int s_dma = mod_ring(2 * ya + 2 * D);              // slot of row 2 oh + 2 D
    for (int oh = ya; oh < yb; ++oh) {
      uint32_t rb[3];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int sl = s_lo + kh;
        rb[kh] = static_cast<uint32_t>((sl >= RING ? sl - RING : sl) * kSlotB);
      }
      const int r_dma = 2 * oh + 2 * D, sl_dma = s_dma;
      f32x4 acc[2][2] = {{cinit[0], cinit[0]}, {cinit[1], cinit[1]}};
      constexpr int PF = 4;
      u32x4_t bq[PF + 1];
      auto issue_rd = [&](auto e_c) {
        constexpr int E = decltype(e_c)::value;
        constexpr int KS = E / 2, FN = E % 2;
        constexpr int TAP = KS / C::SUBS, SB = KS % C::SUBS;
        ds_rd16<0>(bq[E % (PF + 1)], rb[TAP / 3] + boff[FN][TAP % 3][SB]);
      };
      static_for<0, PF>(issue_rd);
      auto entry = [&](auto e_c) {
        constexpr int E = decltype(e_c)::value;
        constexpr int KS = E / 2, FN = E % 2;
        if constexpr (E + PF < C::NE) issue_rd(std::integral_constant<int, E + PF>{});
        constexpr int AHEAD = (E + PF < C::NE ? E + PF : C::NE - 1) - E;   // reads issued after entry E's
        asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(AHEAD) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 bv = __builtin_bit_cast(bf16x8, bq[E % (PF + 1)]);
        acc[0][FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[KS][0]), bv, acc[0][FN], 0, 0, 0);
        acc[1][FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[KS][1]), bv, acc[1][FN], 0, 0, 0);
        if constexpr (E < 5) piece(E, r_dma, sl_dma);   // this step's DMA, one piece per MFMA pair
        __builtin_amdgcn_sched_barrier(0);
      };
      static_for<0, C::NE>(entry);

      // epilogue (store_tile_x4's conversion): ReLU, RNE, one 16-B piece per pixel fragment
      const bool relu = a.relu != 0;
      const int obase = (n * a.ho + oh) * a.wo;
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        uint32_t wv[4];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float v[4] = {acc[hh][fn][0], acc[hh][fn][1], acc[hh][fn][2], acc[hh][fn][3]};
          if (relu) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
          }
          wv[2 * hh] = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
          wv[2 * hh + 1] = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
        }
        uint4 o = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        swap_halves(o);
        const int ow = ow0 + 32 * wp + 16 * fn + fr;
        const unsigned ob = ow < a.wo ? static_cast<unsigned>(((obase + ow) * C::COUT + 32 * wc + chunk_of_row(fq) * 8) * 2) : kOob;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{o.x, o.y, o.z, o.w}, ys, ob, 0, 0);
      }
      // retire the DMA pieces of rows 2 oh + 2, 2 oh + 3 (issued D - 1 steps ago; younger ops stay
      // in flight: the 2 stores, and with D = 2 this step's pieces), then publish them and free
      // the slots of 2 oh - 1, 2 oh
      if (D == 1) asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(7)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      s_lo = s_lo + 2 >= RING ? s_lo + 2 - RING : s_lo + 2;
      s_dma = s_dma + 2 >= RING ? s_dma + 2 - RING : s_dma + 2;
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    more = idx < end;
    if (more) begin_segment();
  }
}

// --- Stride-1 3x3 64 -> 64 with the block's 1x1 stride-2 downsample folded in (x2, 32 channels):
// DRN-D layer3.0 conv2 + downsample (lmodels/drn.py:49-65, :181-186), the launch conv_halo's x2
// form served.  Same walk as conv_s2row_kernel with one input row per step: wave (wc, wp) owns
// output channels 32 wc .. +31 x 32 pixels of a 64-column strip; the conv input rows (66 pixels x
// 128 B, chunk c of pixel p at c ^ (p & 7)) arrive two steps ahead into a 5-slot ring, the x2 row
// of each output row (its 64 even pixels (2 oh, 2 ow) gathered by the DMA, 64 B each, chunk c at
// c ^ ((p >> 1) & 3)) into a 3-slot ring.  K: the 18 32-channel tap chunks of the packed
// [W2 | W_ds | 0] rows, then the x2 chunk (k 576 .. 607) -- conv_halo's order, start (the summed
// shifts) and epilogue, so the output is bit-identical to it.
constexpr int kX1Slot = 9 * 1024;     // 66 x 128 B = 8448 B used
constexpr int kX2Slot = 4 * 1024;     // 64 x 64 B
constexpr int kX1Ring = 5, kX2Ring = 3;
constexpr int kS1Lds = kX1Ring * kX1Slot + kX2Ring * kX2Slot + 1024;   // + the dummy DMA piece's KB

struct S1Params {
  const uint16_t* x;
  const uint16_t* x2;
  const uint16_t* wgt;
  const float* shift;
  uint16_t* y;
  int n, h, w, h2, w2, k_pad, relu, strips, total, per_wg;
};

__global__ void __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv_s1x2row_kernel(const S1Params a) {
  constexpr int NKS = 19, NE = 2 * NKS, OWS = 64, XW = 66;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wc = wave & 1, wp = wave >> 1;
  const int fr = lane & 15, fq = lane >> 4;

  u32x4_t wf[NKS][2];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
      wf[ks][fm] = *reinterpret_cast<const u32x4_t*>(a.wgt + static_cast<int64_t>(32 * wc + 16 * fm + fr) * a.k_pad +
                                                     32 * ks + 8 * fq);
  auto pin_weights = [&]() {   // as in conv_s2row_kernel
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) asm volatile("" : "+a"(wf[ks][fm]));
  };
  f32x4 cinit[2];
#pragma unroll
  for (int fm = 0; fm < 2; ++fm) {
    const float4 s = *reinterpret_cast<const float4*>(a.shift + 32 * wc + 16 * fm + 4 * fq);
    cinit[fm] = f32x4{s.x, s.y, s.z, s.w};
  }
  const int H = a.h, W = a.w;
  const __amdgpu_buffer_rsrc_t xs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, a.n * H * W * 128, 0x00020000);
  const __amdgpu_buffer_rsrc_t x2s =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x2), 0, a.n * a.h2 * a.w2 * 64, 0x00020000);
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, a.n * H * W * 128, 0x00020000);
  typedef __attribute__((address_space(3))) void lds_t;

  // B fragments: conv rows (fn, kw, sub): strip pixel 32 wp + 16 fn + fr + kw, chunk 4 sub + fq;
  // x2 (fn): x2 pixel 32 wp + 16 fn + fr, chunk fq
  uint32_t boff[2][3][2], b2off[2];
#pragma unroll
  for (int fn = 0; fn < 2; ++fn) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int p = 32 * wp + 16 * fn + fr + kw, c = 4 * sb + fq;
        boff[fn][kw][sb] = static_cast<uint32_t>(p * 128 + ((c ^ (p & 7)) << 4));
      }
    const int p = 32 * wp + 16 * fn + fr;
    b2off[fn] = static_cast<uint32_t>(kX1Ring * kX1Slot + p * 64 + ((fq ^ ((p >> 1) & 3)) << 4));
  }

  int idx = blockIdx.x * a.per_wg;
  const int end = min(idx + a.per_wg, a.total);
  int ya = 0, yb = 0, n = 0, ow0 = 0;
  // 16 DMA pieces per step: 0..8 the conv row (9 KB slot), 9..12 the x2 row (4 KB), 13..15
  // dummies into the slack KB; wave w issues pieces w + 4 k, k < 4.  Lane offsets (column part)
  // depend only on (k, lane); the row part is a scalar offset.
  uint32_t vo[4];
  auto piece = [&](int k, int row, int slot1, int slot2) {   // conv row `row` (slot1); x2 row of output row row - 1 (slot2)
    const int i = wave + 4 * k;
    int soff = 0, dst = kX1Ring * kX1Slot + kX2Ring * kX2Slot;
    bool ok = false;
    if (i < 9) {
      ok = static_cast<unsigned>(row) < static_cast<unsigned>(H);
      soff = ok ? ((n * H + row) * W) * 128 : 0;
      dst = slot1 * kX1Slot + i * 1024;
    } else if (i < 13) {
      const int r2 = 2 * (row - 1);
      ok = row - 1 >= 0 && row - 1 < H && r2 < a.h2;
      soff = ok ? ((n * a.h2 + r2) * a.w2) * 64 : 0;
      dst = kX1Ring * kX1Slot + slot2 * kX2Slot + (i - 9) * 1024;
    }
    soff = __builtin_amdgcn_readfirstlane(soff);
    dst = __builtin_amdgcn_readfirstlane(dst);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 9 ? xs : x2s, (lds_t*)(smem + dst), 16, ok ? vo[k] : kOob, soff, 0, 0);
  };
  auto m5 = [](int r) { return ((r % kX1Ring) + kX1Ring) % kX1Ring; };
  auto m3 = [](int r) { return ((r % kX2Ring) + kX2Ring) % kX2Ring; };
  // next segment: its state and its ring fill -- conv rows ya - 1 .. ya + 2 with the x2 rows of
  // output rows ya - 2 .. ya + 1 (the first two are never read); step oh then issues conv row
  // oh + 3 and the x2 row of oh + 2
  auto begin_segment = [&]() {
    const int seg = idx / H;
    ya = idx - seg * H;
    yb = min(H, ya + (end - idx));
    idx += yb - ya;
    n = seg / a.strips;
    const int s = seg - n * a.strips;
    ow0 = OWS * s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = wave + 4 * k;
      uint32_t v = kOob;
      if (i < 9) {
        const int g = i * 64 + lane, p = g >> 3, c = (g & 7) ^ (p & 7);
        const int col = ow0 - 1 + p;
        if (p < XW && static_cast<unsigned>(col) < static_cast<unsigned>(W)) v = static_cast<unsigned>(col * 128 + c * 16);
      } else if (i < 13) {
        const int g = (i - 9) * 64 + lane, p = g >> 2, c = (g & 3) ^ ((p >> 1) & 3);
        const int ow = ow0 + p;
        if (ow < W && 2 * ow < a.w2) v = static_cast<unsigned>(2 * ow * 64 + c * 16);
      }
      vo[k] = v;
    }
#pragma unroll
    for (int r = -1; r <= 2; ++r)
#pragma unroll
      for (int k = 0; k < 4; ++k) piece(k, ya + r, m5(ya + r), m3(ya + r - 1));
  };
  bool more = idx < end;
  if (more) begin_segment();
  pin_weights();                                   // waits for the weights only: the fill stays in flight
  while (more) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    int s_lo = m5(ya - 1), s_dma = m5(ya + 3), s2_cur = m3(ya), s2_dma = m3(ya + 2);
    for (int oh = ya; oh < yb; ++oh) {
      uint32_t rb[3];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int sl = s_lo + kh;
        rb[kh] = static_cast<uint32_t>((sl >= kX1Ring ? sl - kX1Ring : sl) * kX1Slot);
      }
      const uint32_t rb2 = static_cast<uint32_t>(s2_cur * kX2Slot);
      const int r_dma = oh + 3, sl1 = s_dma, sl2 = s2_dma;
      f32x4 acc[2][2] = {{cinit[0], cinit[0]}, {cinit[1], cinit[1]}};
      constexpr int PF = 4;
      u32x4_t bq[PF + 1];
      auto issue_rd = [&](auto e_c) {
        constexpr int E = decltype(e_c)::value;
        constexpr int KS = E / 2, FN = E % 2;
        if constexpr (KS < 18) ds_rd16<0>(bq[E % (PF + 1)], rb[KS / 6] + boff[FN][(KS / 2) % 3][KS % 2]);
        else ds_rd16<0>(bq[E % (PF + 1)], rb2 + b2off[FN]);
      };
      static_for<0, PF>(issue_rd);
      auto entry = [&](auto e_c) {
        constexpr int E = decltype(e_c)::value;
        constexpr int KS = E / 2, FN = E % 2;
        if constexpr (E + PF < NE) issue_rd(std::integral_constant<int, E + PF>{});
        constexpr int AHEAD = (E + PF < NE ? E + PF : NE - 1) - E;
        asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(AHEAD) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 bv = __builtin_bit_cast(bf16x8, bq[E % (PF + 1)]);
        acc[0][FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[KS][0]), bv, acc[0][FN], 0, 0, 0);
        acc[1][FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[KS][1]), bv, acc[1][FN], 0, 0, 0);
        if constexpr (E < 4) piece(E, r_dma, sl1, sl2);
        __builtin_amdgcn_sched_barrier(0);
      };
      static_for<0, NE>(entry);

      const bool relu = a.relu != 0;
      const int obase = (n * H + oh) * W;
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        uint32_t wv[4];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float v[4] = {acc[hh][fn][0], acc[hh][fn][1], acc[hh][fn][2], acc[hh][fn][3]};
          if (relu) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
          }
          wv[2 * hh] = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
          wv[2 * hh + 1] = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
        }
        uint4 o = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        swap_halves(o);
        const int ow = ow0 + 32 * wp + 16 * fn + fr;
        const unsigned ob = ow < W ? static_cast<unsigned>(((obase + ow) * 64 + 32 * wc + chunk_of_row(fq) * 8) * 2) : kOob;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{o.x, o.y, o.z, o.w}, ys, ob, 0, 0);
      }
      // retire the pieces issued a step ago (this step's 4 and the 2 stores stay in flight)
      asm volatile("s_waitcnt vmcnt(6)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      s_lo = s_lo + 1 >= kX1Ring ? 0 : s_lo + 1;
      s_dma = s_dma + 1 >= kX1Ring ? 0 : s_dma + 1;
      s2_cur = s2_cur + 1 >= kX2Ring ? 0 : s2_cur + 1;
      s2_dma = s2_dma + 1 >= kX2Ring ? 0 : s2_dma + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    more = idx < end;
    if (more) begin_segment();
  }
}

int g_cus = 0;
constexpr auto kern32 = &conv_s2row_kernel<32, kRing32, kWgs32>;
constexpr auto kern64 = &conv_s2row_kernel<64, kRing64, kWgs64>;

}  // namespace

bool s2row_conv_supported(const drnmi_conv_args& p) {
  const bool c32 = p.cin == 32 && p.cout == 64, c64 = p.cin == 64 && p.cout == 128;
  return p.dtype == DRNMI_BF16 && p.out_dtype == DRNMI_BF16 && (c32 || c64) && p.ks == 3 && p.stride == 2 &&
         p.pad == 1 && p.dil == 1 && p.scale == nullptr && p.res == nullptr && p.x2 == nullptr &&
         p.unit_mask == nullptr && p.k == 9 * p.cin && p.k_pad >= p.k && p.k_pad % 8 == 0 && p.cout_pad >= p.cout &&
         p.n > 0 && p.h >= 1 && p.w >= 1 && p.ho == (p.h - 1) / 2 + 1 && p.wo == (p.w - 1) / 2 + 1 && p.y_sc == 1 &&
         p.y_sp == p.cout && p.y_sn == static_cast<int64_t>(p.ho) * p.wo * p.cout &&
         static_cast<int64_t>(p.n) * p.h * p.w * p.cin * 2 < (int64_t(1) << 31) &&
         static_cast<int64_t>(p.n) * p.ho * p.wo * p.cout * 2 < (int64_t(1) << 31);
}

bool s2row_auto(const drnmi_conv_args& p) { return s2row_conv_supported(p); }

bool s1x2row_conv_supported(const drnmi_conv_args& p) {
  return p.dtype == DRNMI_BF16 && p.out_dtype == DRNMI_BF16 && p.cin == 64 && p.cout == 64 && p.ks == 3 &&
         p.stride == 1 && p.pad == 1 && p.dil == 1 && p.x2 != nullptr && p.cin2 == 32 && p.stride2 == 2 &&
         p.scale == nullptr && p.res == nullptr && p.unit_mask == nullptr && p.k == 9 * 64 + 32 && p.k_pad >= p.k &&
         p.k_pad % 8 == 0 && p.cout_pad >= 64 && p.n > 0 && p.h >= 1 && p.w >= 1 && p.ho == p.h && p.wo == p.w &&
         2 * (p.ho - 1) < p.h2 && 2 * (p.wo - 1) < p.w2 && p.y_sc == 1 && p.y_sp == 64 &&
         p.y_sn == static_cast<int64_t>(p.ho) * p.wo * 64 && static_cast<int64_t>(p.n) * p.h * p.w * 128 < (int64_t(1) << 31) &&
         static_cast<int64_t>(p.n) * p.h2 * p.w2 * 64 < (int64_t(1) << 31);
}

bool s1x2row_auto(const drnmi_conv_args& p) { return s1x2row_conv_supported(p); }

const char* s1x2row_conv_name(const drnmi_conv_args& p) {
  return s1x2row_conv_supported(p) ? "conv_s1x2row_kernel" : nullptr;
}

int s1x2row_conv_dispatch(const drnmi_conv_args& p, hipStream_t st) {
  if (!s1x2row_conv_supported(p)) return DRNMI_ENOTSUP;
  static int wgs = 0;
  if (wgs == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_s1x2row_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kS1Lds);
    if (e != hipSuccess) return static_cast<int>(e);
    wgs = 2 * cus;                                      // two workgroups per CU (58 KB LDS each)
  }
  S1Params a;
  a.x = static_cast<const uint16_t*>(p.x);
  a.x2 = static_cast<const uint16_t*>(p.x2);
  a.wgt = static_cast<const uint16_t*>(p.wgt);
  a.shift = p.shift;
  a.y = static_cast<uint16_t*>(p.y);
  a.n = p.n;
  a.h = p.h;
  a.w = p.w;
  a.h2 = p.h2;
  a.w2 = p.w2;
  a.k_pad = p.k_pad;
  a.relu = p.relu;
  a.strips = (p.w + 63) / 64;
  const int64_t total = static_cast<int64_t>(p.n) * a.strips * p.h;
  if (total >= (int64_t(1) << 31)) return DRNMI_ENOTSUP;
  a.total = static_cast<int>(total);
  a.per_wg = (a.total + wgs - 1) / wgs;
  const int grid = (a.total + a.per_wg - 1) / a.per_wg;
  hipLaunchKernelGGL(conv_s1x2row_kernel, dim3(grid), dim3(256), kS1Lds, st, a);
  return static_cast<int>(hipGetLastError());
}

const char* s2row_conv_name(const drnmi_conv_args& p) {
  if (!s2row_conv_supported(p)) return nullptr;
  static_assert(kRing32 == 7 && kWgs32 == 2 && kRing64 == 7 && kWgs64 == 2, "kernel names below");
  return p.cin == 32 ? "conv_s2row_kernel<32, 7, 2>" : "conv_s2row_kernel<64, 7, 2>";
}

int s2row_conv_dispatch(const drnmi_conv_args& p, hipStream_t st) {
  if (!s2row_conv_supported(p)) return DRNMI_ENOTSUP;
  if (g_cus == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern32), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       s2_lds_bytes<kRing32>());
    if (e == hipSuccess)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern64), hipFuncAttributeMaxDynamicSharedMemorySize,
                              s2_lds_bytes<kRing64>());
    if (e != hipSuccess) return static_cast<int>(e);
    g_cus = cus;
  }
  const bool c32 = p.cin == 32;
  const int wgs = g_cus * (c32 ? kWgs32 : kWgs64);   // persistent: WGS workgroups per CU
  S2Params a;
  a.x = static_cast<const uint16_t*>(p.x);
  a.wgt = static_cast<const uint16_t*>(p.wgt);
  a.shift = p.shift;
  a.y = static_cast<uint16_t*>(p.y);
  a.n = p.n;
  a.h = p.h;
  a.w = p.w;
  a.ho = p.ho;
  a.wo = p.wo;
  a.k_pad = p.k_pad;
  a.relu = p.relu;
  const int ows = p.cin == 32 ? S2Cfg<32>::OWS : S2Cfg<64>::OWS;
  a.strips = (p.wo + ows - 1) / ows;
  const int64_t total = static_cast<int64_t>(p.n) * a.strips * p.ho;
  if (total >= (int64_t(1) << 31)) return DRNMI_ENOTSUP;
  a.total = static_cast<int>(total);
  a.per_wg = (a.total + wgs - 1) / wgs;
  const int grid = (a.total + a.per_wg - 1) / a.per_wg;
  if (c32) hipLaunchKernelGGL(kern32, dim3(grid), dim3(256), s2_lds_bytes<kRing32>(), st, a);
  else hipLaunchKernelGGL(kern64, dim3(grid), dim3(256), s2_lds_bytes<kRing64>(), st, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace drnmi
