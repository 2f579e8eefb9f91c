// Fused 64-channel BasicBlock (DRN-D layer3.1; D-38 layer3.1 / 3.2): conv3x3 64 -> 64 + BN + ReLU,
// conv3x3 64 -> 64 + BN + residual + ReLU, bf16 NHWC, stride 1, dilation 1
// (lmodels/drn.py:27-29 conv3x3, :49-65 BasicBlock.forward; BN folded: eval running stats).
//
// The two halo launches wrote the block's intermediate t to HBM and read it back, and each re-ran
// a 9-step K loop per 4 x 64 tile whose prologue / epilogue dominated (MFMA busy 0.31).  Here one
// persistent workgroup walks a 62-column strip of a frame down its rows:
//   * waves 0, 1 compute t row j (conv1, output channels 32 w .. +31) from x rows j-1 .. j+1;
//     waves 2, 3 compute y row j-2 (conv2, channels 32 (w - 2) .. +31) from t rows j-3 .. j-1 and
//     add x row j-2 -- the two convs of a step are independent, and one barrier per row step
//     hands t over;
//   * each wave's 36 weight fragments (32 channels x 576 K as 2 x 18 v_mfma_f32_16x16x32_bf16 A
//     operands: 16-channel row tiles x (tap, 32-channel) K chunks) stay in AGPRs for the whole
//     launch; B fragments are 16-B LDS reads of (tap, 32-channel) chunks of the x / t rows, four
//     16-pixel tiles per row (the 16x16x32 shape holds a higher clock than 32x32x16 at equal
//     cycles per FLOP: MI355X_MICROARCH.md 'DVFS give-back' item 7);
//   * two such workgroups per CU (two waves per SIMD: one's barrier and epilogue bubbles under the
//     other's MFMAs); x rows arrive by buffer LDS-DMA one step ahead into a 5-row ring (the
//     residual row is the oldest), t rows live in a 4-row ring; 128-B pixel rows with the 16-B chunk c at slot
//     c ^ (pixel & 7) (conflict-free for the 16x16x32 fragment reads at any pixel offset);
//   * pixels and rows outside the image are zero in both rings (the convs' zero padding).
#include "common.h"
#include "kernels.h"

#include <cstring>
#include <type_traits>

namespace drnmi {
namespace {

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kC = 64;                 // channels (in = mid = out)
constexpr int kOW = 62;                // output columns per strip
constexpr int kTW = 64;                // t columns per strip (2 blocks of 32): image cols c0 - 1 ..
constexpr int kXW = 66;                // x columns per strip: image cols c0 - 2 ..
constexpr int kRowB = 128;             // bytes per pixel row (64 bf16)
constexpr int kXSlot = 9 * 1024;       // 66 pixel rows (8448 B) padded to whole 1-KB DMA instructions
constexpr int kXRing = 5;              // residual row j-2, conv1 rows j-1 .. j+1, DMA row j+2
constexpr int kTSlot = kTW * kRowB;    // 8192
constexpr int kTRing = 4;
constexpr int kTBase = kXRing * kXSlot;                  // 46080
constexpr int kLds = kTBase + kTRing * kTSlot + 512;     // + slack: conv2 reads t pixels 64, 65 (unstored columns); two workgroups per CU
constexpr int kChunks = 18;            // 9 taps x 2 chunks of 32 channels
constexpr int kSlices = 2 * kChunks;   // A fragments per wave: (chunk, 16-row tile)
constexpr int kFragB = 16;             // bytes per lane per A fragment
constexpr int kPackW = 2 * 2 * kSlices * 64 * kFragB;    // [conv][half][chunk][row tile][lane][8 bf16]
constexpr int kPackBytes = kPackW + 2 * kC * 4;          // + shift1[64], shift2[64]
constexpr unsigned kOob = 0x80000000u;
constexpr int kXPieces = (kXSlot + 1023) / 1024;         // 9 LDS-DMA instructions per x row

struct BlockParams {
  const uint16_t* x;
  const char* pack;
  uint16_t* y;
  int n, h, w, strips, total, per_wg;
};

__device__ __forceinline__ int bswz(int p) { return p & 7; }

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

__global__ void __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
block64_kernel(const BlockParams a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int role = wave >> 1;          // 0: conv1 (t), 1: conv2 (y)
  const int half = wave & 1;           // output channels 32 half .. +31

  // weight fragments -> AGPRs
  u32x4_t wf[kSlices];
  {
    const u32x4_t* pk = reinterpret_cast<const u32x4_t*>(a.pack) + ((role * 2 + half) * kSlices) * 64 + lane;
    // all loads first, then the AGPR pins (a pin right after its load would wait for it: 36
    // serial L2 round trips before the first step)
#pragma unroll
    for (int s = 0; s < kSlices; ++s) wf[s] = pk[s * 64];
  }
  // the pins wait for every weight load: they follow the first segment's ring-fill DMA, so the two latencies overlap (conv_s2row.hip, scripts/s2row_stamps.py)
  auto pin_weights = [&]() {
#pragma unroll
    for (int s = 0; s < kSlices; ++s) asm volatile("" : "+a"(wf[s]));
  };
  // accumulator start: the conv's shift for the 16 D rows this lane holds
  f32x4 cinit[2];
  {
    const float* sh = reinterpret_cast<const float*>(a.pack + kPackW) + role * kC + 32 * half + 4 * ((lane & 63) >> 4);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) cinit[mt] = f32x4{sh[16 * mt], sh[16 * mt + 1], sh[16 * mt + 2], sh[16 * mt + 3]};
  }
  const int H = a.h, W = a.w;
  const __amdgpu_buffer_rsrc_t xs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, a.n * H * W * kRowB, 0x00020000);
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, a.n * H * W * kRowB, 0x00020000);
  typedef __attribute__((address_space(3))) void lds_t;

  // per-lane LDS byte offsets (ring slot added per step): B fragment of pixel tile fn, tap column
  // dw, 32-channel chunk sb: pixel p = 16 fn + fr + dw of the source ring row, 16-B chunk 4 sb + fq
  const int fr = lane & 15, fq = lane >> 4;
  // (p & 7 does not depend on the tile fn: tile fn adds 16 fn * 128 B, a compile-time offset)
  uint32_t boff[3][2];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw)
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      const int p = fr + dw;
      boff[dw][sb] = p * kRowB + (((4 * sb + fq) ^ bswz(p)) << 4);
    }
  // epilogue pieces: D rows 4 fq .. +3 of row tile mt (channels 32 half + 16 mt + 4 fq ..) of pixel
  // tile fn's pixel fr -- conv1: t ring pixel 16 fn + fr;  conv2: residual = x ring pixel 16 fn + fr + 2
  uint32_t eoff[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int p = fr + (role ? 2 : 0);
    eoff[mt] = p * kRowB + (((4 * half + 2 * mt + (fq >> 1)) ^ bswz(p)) << 4) + 8 * (fq & 1);
  }

  int idx = blockIdx.x * a.per_wg;
  const int end = min(idx + a.per_wg, a.total);
  int ya = 0, yb = 0, n = 0, c0 = 0, img0 = 0;
  // x row DMA (all four waves: instruction i = wave + 4 k of the row's 9)
  auto x_dma = [&](int row) {
    const int slot = ((row % kXRing) + kXRing) % kXRing;
    const bool row_ok = static_cast<unsigned>(row) < static_cast<unsigned>(H);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int i = wave + 4 * k;
      if (i >= kXPieces) break;                        // wave-uniform
      const int byte = i * 1024 + lane * 16;
      const int p = byte >> 7, sl = (byte >> 4) & 7;
      const int col = c0 - 2 + p;
      const bool ok = row_ok && p < kXW && static_cast<unsigned>(col) < static_cast<unsigned>(W);
      const unsigned off = ok ? static_cast<unsigned>(((img0 + row) * W + col) * kRowB + ((sl ^ bswz(p)) << 4)) : kOob;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xs, (lds_t*)(smem + slot * kXSlot + i * 1024), 16, off, 0, 0, 0);
    }
  };
  // next segment: its state and its prologue, x rows ya-2 .. ya (steps start at j = ya - 1; step
  // j issues row j + 2)
  auto begin_segment = [&]() {
    const int seg = idx / H;
    ya = idx - seg * H;
    yb = min(H, ya + (end - idx));
    idx += yb - ya;
    n = seg / a.strips;
    const int s = seg - n * a.strips;
    c0 = kOW * s;                                      // first output column of the strip
    img0 = n * H;
    for (int row = ya - 2; row <= ya; ++row) x_dma(row);
  };
  bool more = idx < end;
  if (more) begin_segment();
  pin_weights();                                     // waits for the weights only: the fill stays in flight
  while (more) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    for (int j = ya - 1; j <= yb + 1; ++j) {
      x_dma(j + 2);
      const int xs_m1 = ((j - 1) % kXRing + kXRing) % kXRing;
      // source rows: conv1 x rows j-1 .. j+1, conv2 t rows j-3 .. j-1
      uint32_t rb[3];
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
        rb[dh] = role == 0 ? static_cast<uint32_t>(((xs_m1 + dh) % kXRing) * kXSlot)
                           : static_cast<uint32_t>(kTBase + ((j - 3 + dh) & 3) * kTSlot);
      f32x4 acc[2][4];
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) {
        acc[0][fn] = cinit[0];
        acc[1][fn] = cinit[1];
      }
      // entries (chunk ks = tap * 2 + sb, pixel tile fn): one B read, two MFMAs (row tiles); reads
      // run PF entries ahead with counted lgkmcnt
      constexpr int NE = kChunks * 4, PF = 4;   // B reads in flight
      u32x4_t bq[PF + 1];
      auto issue_rd = [&](auto e_c) {
        constexpr int E = decltype(e_c)::value;
        constexpr int KS = E / 4, FN = E % 4, TAP = KS / 2, SB = KS % 2;
        ds_rd16<FN * 16 * kRowB>(bq[E % (PF + 1)], rb[TAP / 3] + boff[TAP % 3][SB]);
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
        acc[0][FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[2 * KS]), bv, acc[0][FN], 0, 0, 0);
        acc[1][FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[2 * KS + 1]), bv, acc[1][FN], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      };
      static_for<0, NE>(entry);
      if (role == 0) {
        // conv1 epilogue: ReLU -> bf16 into t ring slot j & 3; pixels outside the image (or rows) = 0
        const bool row_ok = static_cast<unsigned>(j) < static_cast<unsigned>(H);
        const uint32_t tb = static_cast<uint32_t>(kTBase + (j & 3) * kTSlot);
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) {
          const int col = c0 - 1 + 16 * fn + fr;
          const bool ok = row_ok && static_cast<unsigned>(col) < static_cast<unsigned>(W);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const f32x4& ac = acc[mt][fn];
            const uint32_t lo = ok ? pk_bf16x2(f32x2_t{fmaxf(ac[0], 0.f), fmaxf(ac[1], 0.f)}) : 0u;
            const uint32_t hi = ok ? pk_bf16x2(f32x2_t{fmaxf(ac[2], 0.f), fmaxf(ac[3], 0.f)}) : 0u;
            *reinterpret_cast<uint2*>(smem + tb + eoff[mt] + fn * 16 * kRowB) = make_uint2(lo, hi);
          }
        }
      } else {
        // conv2 epilogue: + residual (x ring row j - 2), ReLU, bf16 NHWC store (buffer: dropped if not ours)
        const int yrow = j - 2;
        const bool row_ok = yrow >= ya && yrow < yb;
        const uint32_t xb = static_cast<uint32_t>(((yrow % kXRing + kXRing) % kXRing) * kXSlot);
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) {
          const int pc = 16 * fn + fr;                 // strip column
          const int col = c0 + pc;
          const bool ok = row_ok && pc < kOW && col < W;
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const f32x4& ac = acc[mt][fn];
            const unsigned ob = ok ? static_cast<unsigned>(((img0 + yrow) * W + col) * kRowB + (32 * half + 16 * mt + 4 * fq) * 2) : kOob;
            const uint2 rv = *reinterpret_cast<const uint2*>(smem + xb + eoff[mt] + fn * 16 * kRowB);
            const f32x2_t r0 = widen_bf16x2(rv.x), r1 = widen_bf16x2(rv.y);
            const uint32_t lo = pk_bf16x2(f32x2_t{fmaxf(ac[0] + r0[0], 0.f), fmaxf(ac[1] + r0[1], 0.f)});
            const uint32_t hi = pk_bf16x2(f32x2_t{fmaxf(ac[2] + r1[0], 0.f), fmaxf(ac[3] + r1[1], 0.f)});
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{lo, hi}, ys, ob, 0, 0);
          }
        }
      }
      // retire this wave's DMA pieces of row j + 2 (issued at the start of this step; younger: the
      // conv2 waves' 8 stores), then hand the t row and the x row over
      if (role == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    more = idx < end;
    if (more) begin_segment();
  }
}

int g_block_wgs = 0;

}  // namespace
}  // namespace drnmi

using namespace drnmi;

extern "C" int64_t drnmi_block64_pack_bytes(void) { return kPackBytes; }

// OIHW fp32 weights of the block's two 64 -> 64 3x3 convs, eval-BN scale / shift per channel ->
// the kernel's blob: per (conv, 32-channel half, chunk ks = tap * 2 + sb, row tile mt, lane (fr, fq))
// the 8 bf16 A[fr][8 fq + e] = w[32 half + 16 mt + fr][32 sb + 8 fq + e][kh][kw] * scale[..] (RNE),
// then the two shift vectors.
extern "C" int drnmi_block64_pack(const float* w1, const float* scale1, const float* shift1, const float* w2,
                                  const float* scale2, const float* shift2, void* out_host) {
  if (w1 == nullptr || scale1 == nullptr || shift1 == nullptr || w2 == nullptr || scale2 == nullptr ||
      shift2 == nullptr || out_host == nullptr)
    return DRNMI_EINVAL;
  char* out = static_cast<char*>(out_host);
  auto bf = [](float v) -> uint16_t {
    uint32_t u;
    std::memcpy(&u, &v, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return static_cast<uint16_t>(u >> 16);
  };
  const float* ws[2] = {w1, w2};
  const float* sc[2] = {scale1, scale2};
  const float* shv[2] = {shift1, shift2};
  uint16_t* o = reinterpret_cast<uint16_t*>(out);
  for (int cv = 0; cv < 2; ++cv)
    for (int hf = 0; hf < 2; ++hf)
      for (int ks = 0; ks < kChunks; ++ks)
        for (int mt = 0; mt < 2; ++mt) {
          const int tap = ks >> 1, sb = ks & 1, kh = tap / 3, kw = tap % 3;
          for (int ln = 0; ln < 64; ++ln) {
            const int fr = ln & 15, fq = ln >> 4;
            const int co = 32 * hf + 16 * mt + fr;
            for (int e = 0; e < 8; ++e) {
              const int ci = 32 * sb + 8 * fq + e;
              const float v = ws[cv][((co * kC + ci) * 3 + kh) * 3 + kw] * sc[cv][co];
              o[((((cv * 2 + hf) * kChunks + ks) * 2 + mt) * 64 + ln) * 8 + e] = bf(v);
            }
          }
        }
  float* sh = reinterpret_cast<float*>(out + kPackW);
  for (int cv = 0; cv < 2; ++cv)
    for (int c = 0; c < kC; ++c) sh[cv * kC + c] = shv[cv][c];
  return 0;
}

extern "C" int drnmi_block64_supported(int32_t n, int32_t h, int32_t w) {
  return n > 0 && h >= 1 && w >= 1 && static_cast<int64_t>(n) * h * w * kRowB < (int64_t(1) << 31) ? 1 : 0;
}

extern "C" int drnmi_basic_block64(const void* x, const void* pack, void* y, int32_t n, int32_t h, int32_t w,
                                   void* stream) {
  if (x == nullptr || pack == nullptr || y == nullptr || !drnmi_block64_supported(n, h, w)) return DRNMI_EINVAL;
  if (x == y) return DRNMI_EINVAL;                     // the residual is read while y is written
  if (g_block_wgs == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&block64_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    if (e != hipSuccess) return static_cast<int>(e);
    g_block_wgs = 2 * cus;                             // two workgroups per CU (79 KB LDS each); set only
                                                       // once the LDS attribute is in place
  }
  BlockParams p;
  p.x = static_cast<const uint16_t*>(x);
  p.pack = static_cast<const char*>(pack);
  p.y = static_cast<uint16_t*>(y);
  p.n = n;
  p.h = h;
  p.w = w;
  p.strips = (w + kOW - 1) / kOW;
  p.total = n * p.strips * h;
  p.per_wg = (p.total + g_block_wgs - 1) / g_block_wgs;
  const int grid = (p.total + p.per_wg - 1) / p.per_wg;
  hipLaunchKernelGGL(block64_kernel, dim3(grid), dim3(256), kLds, static_cast<hipStream_t>(stream), p);
  return static_cast<int>(hipGetLastError());
}
