// Row-walking 3x3 128 -> 128 conv (bf16 NHWC, stride 1, pad 1, BN scale folded, optional residual,
// ReLU): the D-22 layer4 BasicBlock convs without a downsample (lmodels/drn.py:27-29, :49-65).
//
// On the staggered 128-channel strip tile these launches ran 1024 tiles of 256 pixels x 18 K steps:
// four rounds per CU whose per-tile fill / epilogue and per-phase barriers held the MFMAs to ~0.36
// busy (89-92 us per D-22 batch-8 launch).  Here one persistent workgroup per CU (8 waves) owns a
// 64-column strip of a frame and walks a contiguous range of its rows:
//   * wave (g, kq): output channels 32 g .. +31, K half kq (chunks 18 kq .. 18 kq + 17 of the 36
//     (tap, 32-channel) chunks); its 32 x 576 weights (2 x 18 v_mfma_f32_16x16x32_bf16 A fragments,
//     144 registers) stay in AGPRs for the launch;
//   * input rows (66 pixels x 256 B, 16-B chunk c of pixel p at c ^ (2 p & 15): conflict-free for the
//     fragment reads at any tap offset) arrive by buffer LDS-DMA two steps ahead into a 5-slot ring;
//   * per output row the K-half-1 waves hand their accumulators to the K-half-0 waves through LDS
//     (one barrier), which add them in that order, add the residual (loaded at the start of the
//     step), apply ReLU and store bf16; a second barrier per row advances the ring.
// The accumulation order differs from the strip tile's (two K halves), so the check is numeric
// (tests/test_gpu_row128.py against the fp32 restatement; network label tests).
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

namespace drnmi {
namespace {

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kC = 128;
constexpr int kOWS = 64;                       // output columns per strip
constexpr int kXW = kOWS + 2;                  // input columns per strip
constexpr int kPixB = 256;                     // bytes per input pixel (128 bf16)
constexpr int kSlot = 17 * 1024;               // 66 x 256 B = 16896 B, whole 1-KB DMA pieces
constexpr int kPieces = kSlot / 1024;          // 17
constexpr int kRing = 5;                       // rows oh - 1 .. oh + 3
constexpr int kXch = kRing * kSlot;            // K-half exchange: 4 waves x 64 lanes x 32 floats
constexpr int kDummy = kXch + 4 * 64 * 32 * 4; // the dummy DMA pieces' KB
constexpr int kLds = kDummy + 1024;
constexpr unsigned kOob = 0x80000000u;
constexpr int kNKS = 18;                       // K chunks per wave

struct R128Params {
  const uint16_t* x;
  const uint16_t* wgt;
  const float* shift;
  const uint16_t* res;
  uint16_t* y;
  int n, h, w, k_pad, relu, strips, total, per_wg;
};

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

__device__ __forceinline__ int rswz(int p) { return (2 * p) & 15; }

template <bool RES>
__global__ void __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
conv_row128_kernel(const R128Params a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wave & 3, kq = wave >> 2;
  const int fr = lane & 15, fq = lane >> 4;

  // weights: fragment (ks, mt) = packed row 32 g + 16 mt + fr, columns 32 (18 kq + ks) + 8 fq .. +7
  u32x4_t wf[kNKS][2];
#pragma unroll
  for (int ks = 0; ks < kNKS; ++ks)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
      wf[ks][mt] = *reinterpret_cast<const u32x4_t*>(a.wgt + static_cast<int64_t>(32 * g + 16 * mt + fr) * a.k_pad +
                                                     32 * (kNKS * kq + ks) + 8 * fq);
#pragma unroll
  for (int ks = 0; ks < kNKS; ++ks)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) asm volatile("" : "+a"(wf[ks][mt]));
  f32x4 cinit[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    if (kq == 0) {
      const float4 s = *reinterpret_cast<const float4*>(a.shift + 32 * g + 16 * mt + 4 * fq);
      cinit[mt] = f32x4{s.x, s.y, s.z, s.w};
    } else {
      cinit[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const int H = a.h, W = a.w;
  const int nbytes = a.n * H * W * kPixB;
  const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(RES ? a.res : a.x), 0, nbytes, 0x00020000);
  typedef __attribute__((address_space(3))) void lds_t;

  // B fragment (kw, sub): strip pixel fr + kw (+ 16 fn: a compile-time offset, 16 fn * 256 B, and
  // (2 (p + 16 fn)) & 15 == (2 p) & 15), chunk 4 sub + fq
  uint32_t boff[3][4];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const int p = fr + kw;
      boff[kw][sb] = static_cast<uint32_t>(p * kPixB + (((4 * sb + fq) ^ rswz(p)) << 4));
    }
  float4* const xch = reinterpret_cast<float4*>(smem + kXch) + (g * 64 + lane) * 8;

  int idx = blockIdx.x * a.per_wg;
  const int end = min(idx + a.per_wg, a.total);
  while (idx < end) {
    const int seg = idx / H;
    const int ya = idx - seg * H;
    const int yb = min(H, ya + (end - idx));
    idx += yb - ya;
    const int n = seg / a.strips, s = seg - n * a.strips;
    const int ow0 = kOWS * s;

    // 17 DMA pieces per input row: wave w issues pieces w + 8 k (k < 3); 18..23 are dummies
    uint32_t vo[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int i = wave + 8 * k;
      const int gr = (i % kPieces) * 64 + lane, p = gr >> 4, c = (gr & 15) ^ rswz(p);
      const int col = ow0 - 1 + p;
      vo[k] = i < kPieces && p < kXW && static_cast<unsigned>(col) < static_cast<unsigned>(W)
                  ? static_cast<unsigned>(col * kPixB + c * 16) : kOob;
    }
    auto piece = [&](int k, int row, int slot) {
      const int i = wave + 8 * k;
      const bool ok = i < kPieces && static_cast<unsigned>(row) < static_cast<unsigned>(H);
      const int soff = __builtin_amdgcn_readfirstlane(ok ? (n * H + row) * W * kPixB : 0);
      const int dst = __builtin_amdgcn_readfirstlane(i < kPieces ? slot * kSlot + i * 1024 : kDummy);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xs, (lds_t*)(smem + dst), 16, ok ? vo[k] : kOob, soff, 0, 0);
    };
    auto m5 = [](int r) { return ((r % kRing) + kRing) % kRing; };
    // prologue: rows ya - 1 .. ya + 2 (step oh issues row oh + 3)
#pragma unroll
    for (int r = -1; r <= 2; ++r)
#pragma unroll
      for (int k = 0; k < 3; ++k) piece(k, ya + r, m5(ya + r));
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    int s_lo = m5(ya - 1), s_dma = m5(ya + 3);
    for (int oh = ya; oh < yb; ++oh) {
      const int obase = (n * H + oh) * W;
      uint32_t rb[3];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int sl = s_lo + kh;
        rb[kh] = static_cast<uint32_t>((sl >= kRing ? sl - kRing : sl) * kSlot);
      }
      const int r_dma = oh + 3, sl_dma = s_dma;
      f32x4 acc[2][4];
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) {
        acc[0][fn] = cinit[0];
        acc[1][fn] = cinit[1];
      }
      constexpr int NE = kNKS * 4, PF = 4;
      u32x4_t bq[PF + 1];
      // entry (ks, fn): global chunk 18 KQ + ks = tap * 4 + sub (KQ compile-time: every row base
      // and B offset index is a constant)
      auto mma_row = [&](auto kq_c) {
        constexpr int KQ = decltype(kq_c)::value;
        auto issue_rd = [&](auto e_c) {
          constexpr int E = decltype(e_c)::value;
          constexpr int KS = E / 4, FN = E % 4;
          constexpr int KC = kNKS * KQ + KS, TAP = KC >> 2, SB = KC & 3;
          ds_rd16<FN * 16 * kPixB>(bq[E % (PF + 1)], rb[TAP / 3] + boff[TAP % 3][SB]);
        };
        static_for<0, PF>(issue_rd);
        auto entry = [&](auto e_c) {
          constexpr int E = decltype(e_c)::value;
          constexpr int KS = E / 4, FN = E % 4;
          if constexpr (E + PF < NE) issue_rd(std::integral_constant<int, E + PF>{});
          constexpr int AHEAD = (E + PF < NE ? E + PF : NE - 1) - E;
          asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(AHEAD) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          const bf16x8 bv = __builtin_bit_cast(bf16x8, bq[E % (PF + 1)]);
          acc[0][FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[KS][0]), bv, acc[0][FN], 0, 0, 0);
          acc[1][FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[KS][1]), bv, acc[1][FN], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        };
        static_for<0, NE>(entry);
      };
      if (kq == 0) mma_row(std::integral_constant<int, 0>{});
      else mma_row(std::integral_constant<int, 1>{});

      // the residual of this row (K-half-0 waves), loaded after the MFMAs (no registers held across
      // them; their latency overlaps the K-half handoff)
      uint2 rv[2][4];
      if constexpr (RES) {
        if (kq == 0) {
#pragma unroll
          for (int fn = 0; fn < 4; ++fn) {
            const int ow = ow0 + 16 * fn + fr;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
              const unsigned off = ow < W ? static_cast<unsigned>(((obase + ow) * kC + 32 * g + 16 * mt + 4 * fq) * 2) : kOob;
              const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
              rv[mt][fn] = make_uint2(v[0], v[1]);
            }
          }
        }
      }
      // this step's DMA (row oh + 3, needed two steps on), after the residual loads so that
      // vmcnt(3) below retires the residual with the pieces still in flight
#pragma unroll
      for (int k = 0; k < 3; ++k) piece(k, r_dma, sl_dma);
      // K half 1 -> LDS, barrier, K half 0 adds (h0 + h1), residual, ReLU, bf16 store
      if (kq == 1) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int fn = 0; fn < 4; ++fn) xch[mt * 4 + fn] = make_float4(acc[mt][fn][0], acc[mt][fn][1], acc[mt][fn][2], acc[mt][fn][3]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (kq == 0) {
        if constexpr (RES) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");   // the residual loads (older than the 3 pieces)
        const bool relu = a.relu != 0;
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) {
          const int ow = ow0 + 16 * fn + fr;
          uint32_t wv[4];
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const float4 o = xch[mt * 4 + fn];
            float v[4] = {acc[mt][fn][0] + o.x, acc[mt][fn][1] + o.y, acc[mt][fn][2] + o.z, acc[mt][fn][3] + o.w};
            if constexpr (RES) {
              const f32x2_t r0 = widen_bf16x2(rv[mt][fn].x), r1 = widen_bf16x2(rv[mt][fn].y);
              v[0] += r0[0];
              v[1] += r0[1];
              v[2] += r1[0];
              v[3] += r1[1];
            }
            if (relu) {
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
            }
            wv[2 * mt] = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
            wv[2 * mt + 1] = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
          }
          uint4 o = make_uint4(wv[0], wv[1], wv[2], wv[3]);
          swap_halves(o);
          const unsigned ob = ow < W ? static_cast<unsigned>(((obase + ow) * kC + 32 * g + chunk_of_row(fq) * 8) * 2) : kOob;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{o.x, o.y, o.z, o.w}, ys, ob, 0, 0);
        }
        // retire the pieces issued a step ago (this step's 3 and 4 stores stay in flight)
        asm volatile("s_waitcnt vmcnt(7)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(3)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      s_lo = s_lo + 1 >= kRing ? 0 : s_lo + 1;
      s_dma = s_dma + 1 >= kRing ? 0 : s_dma + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Not routed by default: inside the D-22 bench it measured 87-91 us per launch against 85-88 us
// for the staggered 128-channel tile (profiles/r6_row128); DRNMI_ROW128=1 routes these convs here
// (A/B runs), tile 23 forces it.
bool row128_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("DRNMI_ROW128");
    on = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  return on == 1;
}

}  // namespace

bool row128_conv_supported(const drnmi_conv_args& p) {
  return p.dtype == DRNMI_BF16 && p.out_dtype == DRNMI_BF16 && p.cin == 128 && p.cout == 128 && p.ks == 3 &&
         p.stride == 1 && p.pad == 1 && p.dil == 1 && p.x2 == nullptr && p.scale == nullptr && p.unit_mask == nullptr &&
         p.k == 9 * 128 && p.k_pad >= p.k && p.k_pad % 8 == 0 && p.cout_pad >= 128 && p.n > 0 && p.h >= 1 && p.w >= 1 &&
         p.ho == p.h && p.wo == p.w && p.y_sc == 1 && p.y_sp == 128 && p.y_sn == static_cast<int64_t>(p.ho) * p.wo * 128 &&
         static_cast<int64_t>(p.n) * p.h * p.w * kPixB < (int64_t(1) << 31);
}

bool row128_auto(const drnmi_conv_args& p) { return row128_enabled() && row128_conv_supported(p); }

const char* row128_conv_name(const drnmi_conv_args& p) {
  if (!row128_conv_supported(p)) return nullptr;
  return p.res != nullptr ? "conv_row128_kernel<true>" : "conv_row128_kernel<false>";
}

int row128_conv_dispatch(const drnmi_conv_args& p, hipStream_t st) {
  if (!row128_conv_supported(p)) return DRNMI_ENOTSUP;
  static int wgs = 0;
  if (wgs == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    for (const void* f : {reinterpret_cast<const void*>(&conv_row128_kernel<true>),
                          reinterpret_cast<const void*>(&conv_row128_kernel<false>)}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
      if (e != hipSuccess) return static_cast<int>(e);
    }
    wgs = cus;                                          // one 8-wave workgroup per CU (118 KB LDS)
  }
  R128Params a;
  a.x = static_cast<const uint16_t*>(p.x);
  a.wgt = static_cast<const uint16_t*>(p.wgt);
  a.shift = p.shift;
  a.res = static_cast<const uint16_t*>(p.res);
  a.y = static_cast<uint16_t*>(p.y);
  a.n = p.n;
  a.h = p.h;
  a.w = p.w;
  a.k_pad = p.k_pad;
  a.relu = p.relu;
  a.strips = (p.w + kOWS - 1) / kOWS;
  const int64_t total = static_cast<int64_t>(p.n) * a.strips * p.h;
  if (total >= (int64_t(1) << 31)) return DRNMI_ENOTSUP;
  a.total = static_cast<int>(total);
  a.per_wg = (a.total + wgs - 1) / wgs;
  const int grid = (a.total + a.per_wg - 1) / a.per_wg;
  if (p.res != nullptr) hipLaunchKernelGGL(conv_row128_kernel<true>, dim3(grid), dim3(512), kLds, st, a);
  else hipLaunchKernelGGL(conv_row128_kernel<false>, dim3(grid), dim3(512), kLds, st, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace drnmi
