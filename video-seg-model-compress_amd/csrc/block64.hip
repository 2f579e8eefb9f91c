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
//   * each wave's 36 weight fragments (32 channels x 576 K, v_mfma_f32_32x32x16_bf16 A operands)
//     stay in AGPRs for the whole launch; B fragments are 16-B LDS reads of (tap, 16-channel)
//     slices of the x / t rows, two 32-pixel blocks per row;
//   * two such workgroups per CU (two waves per SIMD: one's barrier and epilogue bubbles under the
//     other's MFMAs); x rows arrive by buffer LDS-DMA one step ahead into a 5-row ring (the
//     residual row is the oldest), t rows live in a 4-row ring; 128-B pixel rows with the 16-B chunk c at slot
//     c ^ ((pixel >> 1) & 7) (conflict-free ds_read_b128 at any pixel offset);
//   * pixels and rows outside the image are zero in both rings (the convs' zero padding).
#include "common.h"
#include "kernels.h"

#include <cstring>

namespace drnmi {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
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
constexpr int kSlices = 36;            // 9 taps x 4 slices of 16 channels
constexpr int kFragB = 16;             // bytes per lane per A fragment
constexpr int kPackW = 2 * 2 * kSlices * 64 * kFragB;    // [conv][half][slice][lane][8 bf16]
constexpr int kPackBytes = kPackW + 2 * kC * 4;          // + shift1[64], shift2[64]
constexpr unsigned kOob = 0x80000000u;
constexpr int kXPieces = (kXSlot + 1023) / 1024;         // 9 LDS-DMA instructions per x row

struct BlockParams {
  const uint16_t* x;
  const char* pack;
  uint16_t* y;
  int n, h, w, strips, total, per_wg;
};

__device__ __forceinline__ int bswz(int p) { return (p >> 1) & 7; }

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
  const int r = lane & 31, hh = lane >> 5;

  // weight fragments -> AGPRs
  u32x4_t wf[kSlices];
  {
    const u32x4_t* pk = reinterpret_cast<const u32x4_t*>(a.pack) + ((role * 2 + half) * kSlices) * 64 + lane;
    // all loads first, then the AGPR pins (a pin right after its load would wait for it: 36
    // serial L2 round trips before the first step)
#pragma unroll
    for (int s = 0; s < kSlices; ++s) wf[s] = pk[s * 64];
#pragma unroll
    for (int s = 0; s < kSlices; ++s) asm volatile("" : "+a"(wf[s]));
  }
  // accumulator start: the conv's shift for the 16 D rows this lane holds
  f32x16 cinit;
  {
    const float* sh = reinterpret_cast<const float*>(a.pack + kPackW) + role * kC + 32 * half;
#pragma unroll
    for (int q = 0; q < 16; ++q) cinit[q] = sh[(q & 3) + 8 * (q >> 2) + 4 * hh];
  }
  const int H = a.h, W = a.w;
  const __amdgpu_buffer_rsrc_t xs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x), 0, a.n * H * W * kRowB, 0x00020000);
  const __amdgpu_buffer_rsrc_t ys = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, a.n * H * W * kRowB, 0x00020000);
  typedef __attribute__((address_space(3))) void lds_t;

  // per-lane LDS byte offsets (ring slot added per step): B fragment of block b, tap column dw,
  // 16-channel slice cb: pixel p = 32 b + r + dw of the source ring row, chunk 2 cb + h
  uint32_t boff[2][3][4];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int dw = 0; dw < 3; ++dw)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int p = 32 * b + r + dw;
        boff[b][dw][cb] = p * kRowB + (((2 * cb + hh) ^ bswz(p)) << 4);
      }
  // epilogue pieces: D reg group g (4 channels 32 half + 8 g + 4 h ..) of block b's pixel r
  //   conv1: t ring pixel 32 b + r;  conv2: residual = x ring pixel 32 b + r + 2
  uint32_t eoff[2][4];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int p = 32 * b + r + (role ? 2 : 0);
      eoff[b][g] = p * kRowB + (((4 * half + g) ^ bswz(p)) << 4) + 8 * hh;
    }

  int idx = blockIdx.x * a.per_wg;
  const int end = min(idx + a.per_wg, a.total);
  while (idx < end) {
    const int seg = idx / H;
    const int ya = idx - seg * H;
    const int yb = min(H, ya + (end - idx));
    idx += yb - ya;
    const int n = seg / a.strips, s = seg - n * a.strips;
    const int c0 = kOW * s;                            // first output column of the strip
    const int img0 = n * H;

    // x row DMA (all four waves: instruction i = wave + 4 k of the row's 9)
    auto x_dma = [&](int row) {
      const int slot = ((row % kXRing) + kXRing) % kXRing;
      const bool row_ok = static_cast<unsigned>(row) < static_cast<unsigned>(H);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int i = wave + 4 * k;
        if (i >= kXPieces) break;                      // wave-uniform
        const int byte = i * 1024 + lane * 16;
        const int p = byte >> 7, sl = (byte >> 4) & 7;
        const int col = c0 - 2 + p;
        const bool ok = row_ok && p < kXW && static_cast<unsigned>(col) < static_cast<unsigned>(W);
        const unsigned off = ok ? static_cast<unsigned>(((img0 + row) * W + col) * kRowB + ((sl ^ bswz(p)) << 4)) : kOob;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xs, (lds_t*)(smem + slot * kXSlot + i * 1024), 16, off, 0, 0, 0);
      }
    };
    // prologue: x rows ya-2 .. ya (steps start at j = ya - 1; step j issues row j + 2)
    for (int row = ya - 2; row <= ya; ++row) x_dma(row);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    for (int j = ya - 1; j <= yb + 1; ++j) {
      x_dma(j + 2);
      const int xs_m1 = ((j - 1) % kXRing + kXRing) % kXRing;
      f32x16 acc0 = cinit, acc1 = cinit;
      if (role == 0) {
        // conv1: t row j from x rows j-1 .. j+1
        uint32_t rb[3];
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) rb[dh] = static_cast<uint32_t>(((xs_m1 + dh) % kXRing) * kXSlot);
        u32x4_t bq[4];
        // slice order: tap (dh, dw) outer, cb inner; two blocks alternate (independent chains)
#pragma unroll
        for (int q = 0; q < 2 * kSlices + 2; ++q) {
          if (q < 2 * kSlices) {
            const int s2 = q >> 1, b = q & 1;
            const int tap = s2 >> 2, cb = s2 & 3, dh = tap / 3, dw = tap % 3;
            ds_rd16<0>(bq[q & 3], rb[dh] + boff[b][dw][cb]);
          }
          if (q >= 2) {
            const int qq = q - 2;
            const int s2 = qq >> 1, b = qq & 1;
            if (q < 2 * kSlices) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
            else if (q == 2 * kSlices) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8 av = __builtin_bit_cast(bf16x8, wf[s2]);
            const bf16x8 bv = __builtin_bit_cast(bf16x8, bq[qq & 3]);
            if (b == 0) acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc0, 0, 0, 0);
            else acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc1, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        // epilogue: ReLU -> bf16 into t ring slot j & 3; pixels outside the image (or rows) = 0
        const bool row_ok = static_cast<unsigned>(j) < static_cast<unsigned>(H);
        const uint32_t tb = static_cast<uint32_t>(kTBase + (j & 3) * kTSlot);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const f32x16& ac = b ? acc1 : acc0;
          const int col = c0 - 1 + 32 * b + r;
          const bool ok = row_ok && static_cast<unsigned>(col) < static_cast<unsigned>(W);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const uint32_t lo = ok ? pk_bf16x2(f32x2_t{fmaxf(ac[4 * g], 0.f), fmaxf(ac[4 * g + 1], 0.f)}) : 0u;
            const uint32_t hi = ok ? pk_bf16x2(f32x2_t{fmaxf(ac[4 * g + 2], 0.f), fmaxf(ac[4 * g + 3], 0.f)}) : 0u;
            *reinterpret_cast<uint2*>(smem + tb + eoff[b][g]) = make_uint2(lo, hi);
          }
        }
      } else {
        // conv2: y row j - 2 from t rows j-3 .. j-1, + x row j - 2
        uint32_t rb[3];
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) rb[dh] = static_cast<uint32_t>(kTBase + ((j - 3 + dh) & 3) * kTSlot);
        u32x4_t bq[4];
#pragma unroll
        for (int q = 0; q < 2 * kSlices + 2; ++q) {
          if (q < 2 * kSlices) {
            const int s2 = q >> 1, b = q & 1;
            const int tap = s2 >> 2, cb = s2 & 3, dh = tap / 3, dw = tap % 3;
            ds_rd16<0>(bq[q & 3], rb[dh] + boff[b][dw][cb]);
          }
          if (q >= 2) {
            const int qq = q - 2;
            const int s2 = qq >> 1, b = qq & 1;
            if (q < 2 * kSlices) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
            else if (q == 2 * kSlices) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8 av = __builtin_bit_cast(bf16x8, wf[s2]);
            const bf16x8 bv = __builtin_bit_cast(bf16x8, bq[qq & 3]);
            if (b == 0) acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc0, 0, 0, 0);
            else acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc1, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        // epilogue: + residual (x ring row j - 2), ReLU, bf16 NHWC store (buffer: dropped if not ours)
        const int yrow = j - 2;
        const bool row_ok = yrow >= ya && yrow < yb;
        const uint32_t xb = static_cast<uint32_t>(((yrow % kXRing + kXRing) % kXRing) * kXSlot);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const f32x16& ac = b ? acc1 : acc0;
          const int pc = 32 * b + r;                   // strip column
          const int col = c0 + pc;
          const bool ok = row_ok && pc < kOW && col < W;
          const unsigned ob = ok ? static_cast<unsigned>(((img0 + yrow) * W + col) * kRowB + 64 * half + 8 * hh) : kOob;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const uint2 rv = *reinterpret_cast<const uint2*>(smem + xb + eoff[b][g]);
            const f32x2_t r0 = widen_bf16x2(rv.x), r1 = widen_bf16x2(rv.y);
            const uint32_t lo = pk_bf16x2(f32x2_t{fmaxf(ac[4 * g] + r0[0], 0.f), fmaxf(ac[4 * g + 1] + r0[1], 0.f)});
            const uint32_t hi = pk_bf16x2(f32x2_t{fmaxf(ac[4 * g + 2] + r1[0], 0.f), fmaxf(ac[4 * g + 3] + r1[1], 0.f)});
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{lo, hi}, ys, ob, 16 * g, 0);
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
  }
}

int g_block_wgs = 0;

}  // namespace
}  // namespace drnmi

using namespace drnmi;

extern "C" int64_t drnmi_block64_pack_bytes(void) { return kPackBytes; }

// OIHW fp32 weights of the block's two 64 -> 64 3x3 convs, eval-BN scale / shift per channel ->
// the kernel's blob: per (conv, 32-channel half, slice s = tap * 4 + cb, lane (r, h)) the 8 bf16
// A[r][8h + e] = w[32 half + r][16 cb + 8 h + e][kh][kw] * scale[32 half + r] (RNE), then the
// two shift vectors.
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
      for (int s = 0; s < kSlices; ++s) {
        const int tap = s >> 2, cb = s & 3, kh = tap / 3, kw = tap % 3;
        for (int ln = 0; ln < 64; ++ln) {
          const int rr = ln & 31, h = ln >> 5;
          const int co = 32 * hf + rr;
          for (int e = 0; e < 8; ++e) {
            const int ci = 16 * cb + 8 * h + e;
            const float v = ws[cv][((co * kC + ci) * 3 + kh) * 3 + kw] * sc[cv][co];
            o[(((cv * 2 + hf) * kSlices + s) * 64 + ln) * 8 + e] = bf(v);
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
    g_block_wgs = 2 * cus;                             // two workgroups per CU (79 KB LDS each)
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&block64_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    if (e != hipSuccess) return static_cast<int>(e);
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
