// Fine-tune (train-mode) kernels: the backward half of the DRN-D hot path, fp32.
//
// The reference fine-tunes DRNSeg with train-mode BatchNorm, CrossEntropyLoss on the
// log-probs, SGD(momentum, weight_decay) and Pruner.apply_masks after every step
// (semantic_seg.py:166-230, :817, :963-966; pruners/Pruner.py:17-20).  The convs' forward
// and data-gradient (dgrad) passes reuse the implicit-GEMM conv of conv_igemm.hip (dgrad =
// a stride-1 conv of dy with transposed/flipped weights, after a zero-insert for stride-s
// layers); this file holds everything else:
//
//   pack_conv_weight   OIHW fp32 -> packed [rows_pad][k_pad] (forward or dgrad layout)
//   bn stats / apply   train-mode BatchNorm2d: batch mean / biased var, running-stat update
//                      (momentum, unbiased var), y -> relu(bn(y) [+ res])
//   bn backward        relu mask, dgamma / dbeta, dy, residual-branch gradient
//   channel_sum        per-channel column sums (conv bias gradient)
//   conv_wgrad         weight gradient: GEMM over pixels, v_mfma_f32_16x16x4f32, split over
//                      pixel ranges with a fixed-order (deterministic) reduction
//   zero_insert        dy of a stride-s conv spread onto the input grid (dgrad input)
//   up8_lsm_bwd        LogSoftmax backward + transpose of the fixed bilinear up-conv
//   ce_loss            CrossEntropyLoss(ignore_index) forward / backward on log-probs
//   sgd_step           torch.optim.SGD step (momentum, dampening, wd, nesterov) with the
//                      pruner mask (bit-packed) applied in the same pass
//
// Every reduction accumulates in fp64 in a fixed order (no atomics), so results are
// bit-reproducible run to run.
#include "common.h"

namespace drnmi {
namespace {

constexpr int kThreads = 256;

inline bool aligned16(const void* a, const void* b, const void* c) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) == 0;
}

inline unsigned grid_of(int64_t n, int per = kThreads) {
  const int64_t g = (n + per - 1) / per;
  return static_cast<unsigned>(g < 1 ? 1 : (g > 65535 * 16 ? 65535 * 16 : g));
}

// ------------------------------------------------------------------ weight packing
// mode 0 (forward): out[co][ (kh*ks + kw) * kin_stride + ci ] = w[co][ci][kh][kw] * scale[co]
// mode 1 (dgrad):   out[ci][ (kh'*ks + kw') * kin_stride + co ] = w[co][ci][ks-1-kh'][ks-1-kw']
// Everything else in [rows_pad][k_pad] is zero.
template <typename TO>
__global__ void __launch_bounds__(kThreads)
pack_weight_kernel(const float* __restrict__ w, int cout, int cin, int ks, int kin_stride, int rows_pad,
                   int k_pad, int mode, const float* __restrict__ scale, TO* __restrict__ out) {
  const int64_t total = static_cast<int64_t>(rows_pad) * k_pad;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int row = static_cast<int>(i / k_pad);
    const int k = static_cast<int>(i - static_cast<int64_t>(row) * k_pad);
    const int tap = k / kin_stride;
    const int c = k - tap * kin_stride;
    float v = 0.f;
    if (tap < ks * ks) {
      const int kh = tap / ks, kw = tap - (tap / ks) * ks;
      if (mode == 0) {
        if (row < cout && c < cin) {
          v = w[((static_cast<int64_t>(row) * cin + c) * ks + kh) * ks + kw];
          if (scale != nullptr) v *= scale[row];
        }
      } else {
        // row = ci (dgrad output channel), c = co (dgrad input channel)
        if (row < cin && c < cout)
          v = w[((static_cast<int64_t>(c) * cin + row) * ks + (ks - 1 - kh)) * ks + (ks - 1 - kw)];
      }
    }
    if constexpr (sizeof(TO) == 2) out[i] = f32_to_bf16(v);
    else out[i] = v;
  }
}

// All entries of the table in one launch, as LDS-staged transposes.  An element per thread with the
// OIHW source gathered per element ran at ~1 TB/s (0.61 ms of the fp32x fine-tune step): the dgrad
// layout reads w[co][ci] at stride cin * ks * ks per consecutive output.  Here a tile is 32 output
// rows x CT channel columns x all ks * ks taps.  Its source is CT (dgrad) or 32 (forward) runs of
// contiguous floats -- w[co][ci0 .. ci0 + n)[taps] -- read coalesced into LDS.  The tile is then
// written tap by tap, four consecutive k per thread: 16-B fp32 stores, 8-B stores per bf16 plane.
// 37 KB of LDS per workgroup keeps four workgroups (16 waves) per CU on this memory-bound pass.
// Pure data movement plus split3_kernel's arithmetic: bit-identical to the per-layer calls.
constexpr int kPackRows = 32;
constexpr int kPackMaxEntries = 512;
constexpr int kPackLds = kPackRows * (32 * 9 + 1);        // 3x3 taps x 32 columns, run stride + 1
// columns per tile (a multiple of 4): 32 up to 3x3, 4 up to 7x7 (4 x 49 <= 32 x 9)
__device__ __forceinline__ int pack_cols(int taps) { return taps <= 9 ? 32 : 4; }

__global__ void __launch_bounds__(kThreads)
pack_batched_kernel(const int64_t* __restrict__ tab, int n) {
  __shared__ int first[kPackMaxEntries + 1];              // first tile of each entry (prefix sum)
  __shared__ float L[kPackLds];
  const int t = threadIdx.x;
  for (int e = t; e < n; e += kThreads) {
    const int64_t* q = tab + static_cast<int64_t>(e) * DRNMI_PACK_ENTRY_WORDS;
    const int taps = static_cast<int>(q[5] * q[5]);
    first[e + 1] = static_cast<int>(((q[7] + kPackRows - 1) / kPackRows) * ((q[6] + pack_cols(taps) - 1) / pack_cols(taps)));
  }
  __syncthreads();
  if (t == 0) {
    first[0] = 0;
    for (int e = 0; e < n; ++e) first[e + 1] += first[e];
  }
  __syncthreads();
  const int tiles = first[n];
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    int lo = 0, hi = n - 1;                                  // entry: last e with first[e] <= tile
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (first[mid] <= tile) lo = mid;
      else hi = mid - 1;
    }
    const int64_t* q = tab + static_cast<int64_t>(lo) * DRNMI_PACK_ENTRY_WORDS;
    const float* __restrict__ w = reinterpret_cast<const float*>(q[0]);
    float* __restrict__ out = reinterpret_cast<float*>(q[1]);
    bf16_t* __restrict__ pl = reinterpret_cast<bf16_t*>(q[2]);
    const int cout = static_cast<int>(q[3]), cin = static_cast<int>(q[4]), ks = static_cast<int>(q[5]);
    const int kst = static_cast<int>(q[6]), rows_pad = static_cast<int>(q[7]), k_pad = static_cast<int>(q[8]);
    const int mode = static_cast<int>(q[9]);
    const int64_t m = static_cast<int64_t>(rows_pad) * k_pad;
    const int T = ks * ks;
    const int CT = pack_cols(T);
    const int ntc = (kst + CT - 1) / CT;
    const int local = tile - first[lo];
    const int row0 = (local / ntc) * kPackRows;
    const int col0 = (local % ntc) * CT;
    // runs: forward: run r = output row co = row0 + r, its elements ci = col0 + c (c < CT);
    //       dgrad:   run r = column co = col0 + r, its elements ci = row0 + c (c < 32)
    const int nrun = mode == 0 ? kPackRows : CT;
    const int nel = mode == 0 ? CT : kPackRows;
    const int run_co0 = mode == 0 ? row0 : col0;
    const int ci0 = mode == 0 ? col0 : row0;
    const int rlen = nel * T;
    const int rstr = rlen + 1;
    const int nci = cin - ci0 < nel ? cin - ci0 : nel;       // valid elements of a run: nci * T floats
    __syncthreads();                                         // the previous tile's reads of L
    for (int idx = t; idx < nrun * rlen; idx += kThreads) {
      const int r = idx / rlen;
      const int j = idx - r * rlen;
      const int co = run_co0 + r;
      float v = 0.f;
      if (co < cout && j < nci * T) v = w[(static_cast<int64_t>(co) * cin + ci0) * T + j];
      L[r * rstr + j] = v;
    }
    __syncthreads();
    // thread: 4 consecutive columns c4 .. c4 + 3 of (row r, tap); kst % 4 == 0 (table check)
    const int cq = CT / 4;
    for (int idx = t; idx < kPackRows * T * cq; idx += kThreads) {
      const int c4 = (idx % cq) * 4;
      const int rt = idx / cq;
      const int tap = rt % T;
      const int r = rt / T;
      const int row = row0 + r, col = col0 + c4;
      if (row >= rows_pad || col >= kst) continue;
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)   // forward: run r, ci c, tap; dgrad: run c, ci r, flipped tap
        v[u] = mode == 0 ? L[r * rstr + (c4 + u) * T + tap] : L[(c4 + u) * rstr + r * T + (T - 1 - tap)];
      const int64_t o = static_cast<int64_t>(row) * k_pad + tap * kst + col;
      *reinterpret_cast<float4*>(out + o) = make_float4(v[0], v[1], v[2], v[3]);
      if (pl != nullptr) {                                   // split3_kernel's arithmetic
        uint16_t h1[4], h2[4], h3[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bf16_t a = f32_to_bf16(v[u]);
          const float rr = v[u] - bf16_to_f32(a);
          const bf16_t b = f32_to_bf16(rr);
          h1[u] = a;
          h2[u] = b;
          h3[u] = f32_to_bf16(rr - bf16_to_f32(b));
        }
        *reinterpret_cast<uint2*>(pl + o) = make_uint2(h1[0] | (uint32_t(h1[1]) << 16), h1[2] | (uint32_t(h1[3]) << 16));
        *reinterpret_cast<uint2*>(pl + m + o) = make_uint2(h2[0] | (uint32_t(h2[1]) << 16), h2[2] | (uint32_t(h2[3]) << 16));
        *reinterpret_cast<uint2*>(pl + 2 * m + o) = make_uint2(h3[0] | (uint32_t(h3[1]) << 16), h3[2] | (uint32_t(h3[3]) << 16));
      }
    }
    // the k tail past the last tap (k_pad > ks * ks * kst) is zero; column tile 0 writes it
    const int tail = k_pad - T * kst;
    if (col0 == 0 && tail > 0) {
      for (int idx = t; idx < kPackRows * tail; idx += kThreads) {
        const int r = idx / tail;
        const int row = row0 + r;
        if (row >= rows_pad) continue;
        const int64_t o = static_cast<int64_t>(row) * k_pad + T * kst + (idx - r * tail);
        out[o] = 0.f;
        if (pl != nullptr) {
          pl[o] = 0;
          pl[m + o] = 0;
          pl[2 * m + o] = 0;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ column reductions
// Rows x C (C = row stride, a power of two >= 4), fp32 in, fp64 partial sums.
// Block: TPR threads per row (4 channels each, float4), RG = 256 / TPR row groups.
// grid = (G splits, C / (4 * TPR) channel chunks).  Partials ws[2][G][C] (S1, S2).
enum { RED_STATS = 0, RED_BNBWD = 1, RED_SUM = 2 };


struct RedArgs {
  const float* a;       // STATS: y ; BNBWD: dz ; SUM: x
  const float* z;       // BNBWD: z (relu mask), or NULL: the mask is bn_value(y) > 0 (below)
  const float* y;       // BNBWD: y (pre-BN conv output)
  int64_t rows;
  int C;
  int G;
  int64_t rows_per_split;
  int relu;
  double* ws;
  const float* mean;    // BNBWD with z == NULL: the forward's BN terms (gamma / beta NULL-able)
  const float* invstd;
  const float* gamma;
  const float* beta;
};

// The train-mode BN output before ReLU, one rounding order everywhere it is formed: bn_act_kernel
// writes relu(bn_value) and the backward of a residual-free BN + ReLU recomputes the mask
// bn_value(y) > 0 from y instead of reading z (one fp32 tensor less per pass, bit-identical mask).
__device__ __forceinline__ float bn_value(float v, float m, float s, float g, float b) {
  return __builtin_fmaf((v - m) * s, g, b);
}
__device__ __forceinline__ float4 ld4_or(const float* p, int c, float dflt) {
  return p != nullptr ? *reinterpret_cast<const float4*>(p + c) : make_float4(dflt, dflt, dflt, dflt);
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) colred_kernel(const RedArgs r) {
  const int tpr = (r.C / 4) < 64 ? (r.C / 4) : 64;
  const int rg = kThreads / tpr;
  const int t = threadIdx.x;
  const int tc = t % tpr;
  const int tr = t / tpr;
  const int c0 = blockIdx.y * 4 * tpr + 4 * tc;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * r.rows_per_split;
  const int64_t r1 = (r0 + r.rows_per_split) < r.rows ? (r0 + r.rows_per_split) : r.rows;
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  // BNBWD without z: the thread's four channels' forward BN terms (mask = bn_value(y) > 0)
  float bm[4] = {0, 0, 0, 0}, bs[4] = {0, 0, 0, 0}, bg[4] = {1, 1, 1, 1}, bb[4] = {0, 0, 0, 0};
  const bool ymask = MODE == RED_BNBWD && r.relu && r.z == nullptr;
  if (ymask) {
    const float4 m4 = ld4_or(r.mean, c0, 0.f), s4 = ld4_or(r.invstd, c0, 0.f);
    const float4 g4 = ld4_or(r.gamma, c0, 1.f), b4 = ld4_or(r.beta, c0, 0.f);
    bm[0] = m4.x; bm[1] = m4.y; bm[2] = m4.z; bm[3] = m4.w;
    bs[0] = s4.x; bs[1] = s4.y; bs[2] = s4.z; bs[3] = s4.w;
    bg[0] = g4.x; bg[1] = g4.y; bg[2] = g4.z; bg[3] = g4.w;
    bb[0] = b4.x; bb[1] = b4.y; bb[2] = b4.z; bb[3] = b4.w;
  }
  // RB rows' loads go out before their (in-order) fp64 accumulation: the same sums, with that many
  // loads in flight per thread instead of one
  constexpr int RB = 4;
  int64_t row = r0 + tr;
  for (; row + (RB - 1) * rg < r1; row += RB * rg) {
    float4 av[RB], zv[RB], yv[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t off = (row + u * rg) * r.C + c0;
      av[u] = *reinterpret_cast<const float4*>(r.a + off);
      if constexpr (MODE == RED_BNBWD) {
        if (r.relu && !ymask) zv[u] = *reinterpret_cast<const float4*>(r.z + off);
        yv[u] = *reinterpret_cast<const float4*>(r.y + off);
      }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      float a[4] = {av[u].x, av[u].y, av[u].z, av[u].w};
      if constexpr (MODE == RED_STATS) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s1[j] += a[j];
          s2[j] += static_cast<double>(a[j]) * a[j];
        }
      } else if constexpr (MODE == RED_BNBWD) {
        const float y[4] = {yv[u].x, yv[u].y, yv[u].z, yv[u].w};
        if (ymask) {
#pragma unroll
          for (int j = 0; j < 4; ++j) a[j] = bn_value(y[j], bm[j], bs[j], bg[j], bb[j]) > 0.f ? a[j] : 0.f;
        } else if (r.relu) {
          a[0] = zv[u].x > 0.f ? a[0] : 0.f;
          a[1] = zv[u].y > 0.f ? a[1] : 0.f;
          a[2] = zv[u].z > 0.f ? a[2] : 0.f;
          a[3] = zv[u].w > 0.f ? a[3] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s1[j] += a[j];
          s2[j] += static_cast<double>(a[j]) * y[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) s1[j] += a[j];
      }
    }
  }
  for (; row < r1; row += rg) {
    const int64_t off = row * r.C + c0;
    const float4 av = *reinterpret_cast<const float4*>(r.a + off);
    float a[4] = {av.x, av.y, av.z, av.w};
    if constexpr (MODE == RED_STATS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s1[j] += a[j];
        s2[j] += static_cast<double>(a[j]) * a[j];
      }
    } else if constexpr (MODE == RED_BNBWD) {
      const float4 yv = *reinterpret_cast<const float4*>(r.y + off);
      const float y[4] = {yv.x, yv.y, yv.z, yv.w};
      if (ymask) {
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = bn_value(y[j], bm[j], bs[j], bg[j], bb[j]) > 0.f ? a[j] : 0.f;
      } else if (r.relu) {
        const float4 zv = *reinterpret_cast<const float4*>(r.z + off);
        a[0] = zv.x > 0.f ? a[0] : 0.f;
        a[1] = zv.y > 0.f ? a[1] : 0.f;
        a[2] = zv.z > 0.f ? a[2] : 0.f;
        a[3] = zv.w > 0.f ? a[3] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s1[j] += a[j];
        s2[j] += static_cast<double>(a[j]) * y[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) s1[j] += a[j];
    }
  }
  __shared__ double sh1[kThreads * 4], sh2[kThreads * 4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sh1[t * 4 + j] = s1[j];
    sh2[t * 4 + j] = s2[j];
  }
  __syncthreads();
  // thread q < 4*tpr sums channel q of the block over the rg row groups, in order
  if (t < 4 * tpr) {
    const int q_tc = t / 4, q_j = t % 4;
    double a1 = 0, a2 = 0;
    for (int g = 0; g < rg; ++g) {
      a1 += sh1[(g * tpr + q_tc) * 4 + q_j];
      a2 += sh2[(g * tpr + q_tc) * 4 + q_j];
    }
    const int c = blockIdx.y * 4 * tpr + t;
    r.ws[static_cast<int64_t>(blockIdx.x) * r.C + c] = a1;
    r.ws[static_cast<int64_t>(r.G + blockIdx.x) * r.C + c] = a2;
  }
}

int red_splits(int64_t rows, int C) {
  const int tpr = (C / 4) < 64 ? (C / 4) : 64;
  const int chunks = C / (4 * tpr);
  const int rg = kThreads / tpr;
  int64_t g = 1024 / chunks;
  const int64_t by_rows = (rows + 16 * rg - 1) / (16 * rg);   // >= 16 rows per thread
  if (g > by_rows) g = by_rows;
  return static_cast<int>(g < 1 ? 1 : g);
}

template <int MODE>
hipError_t launch_colred(RedArgs& r, hipStream_t s) {
  const int tpr = (r.C / 4) < 64 ? (r.C / 4) : 64;
  r.G = red_splits(r.rows, r.C);
  r.rows_per_split = (r.rows + r.G - 1) / r.G;
  hipLaunchKernelGGL(colred_kernel<MODE>, dim3(r.G, r.C / (4 * tpr)), dim3(kThreads), 0, s, r);
  return hipGetLastError();
}

// finalize.  The G split partials of a channel were summed by one thread in split order: up to
// 1024 dependent fp64 adds per channel on a handful of waves (120 us per BN layer in the
// fine-tune profile, profiles/r2e_finetune_kernel_stats.csv).  Here a block owns 16 channels
// (a 128-B row of partials per split, coalesced) and 16 threads per channel sum 16 contiguous
// runs of splits, which are then added run by run: a fixed order, so the statistics stay
// deterministic.
constexpr int kFinCh = 16;
__device__ __forceinline__ bool split_sums(const double* __restrict__ ws, int G, int C, int& c, double& s1,
                                           double& s2) {
  __shared__ double p1[kThreads], p2[kThreads];
  const int t = threadIdx.x, tc = t % kFinCh, tg = t / kFinCh;
  constexpr int NG = kThreads / kFinCh;
  c = blockIdx.x * kFinCh + tc;
  const int gs = (G + NG - 1) / NG;
  const int g0 = tg * gs, g1 = g0 + gs < G ? g0 + gs : G;
  double a1 = 0, a2 = 0;
  if (c < C) {
#pragma unroll 8
    for (int g = g0; g < g1; ++g) {
      a1 += ws[static_cast<int64_t>(g) * C + c];
      a2 += ws[static_cast<int64_t>(G + g) * C + c];
    }
  }
  p1[t] = a1;
  p2[t] = a2;
  __syncthreads();
  if (t >= kFinCh || c >= C) return false;
  s1 = 0;
  s2 = 0;
  for (int j = 0; j < NG; ++j) {
    s1 += p1[j * kFinCh + tc];
    s2 += p2[j * kFinCh + tc];
  }
  return true;
}
inline unsigned fin_grid(int C) { return static_cast<unsigned>((C + kFinCh - 1) / kFinCh); }

__global__ void __launch_bounds__(kThreads)
bn_stats_final_kernel(const double* __restrict__ ws, int G, int C, int64_t rows, float eps, float momentum,
                      float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ rmean,
                      float* __restrict__ rvar, int64_t* __restrict__ nbt) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt != nullptr) nbt[0] += 1;
  int c;
  double s1, s2;
  if (!split_sums(ws, G, C, c, s1, s2)) return;
  const double m = s1 / static_cast<double>(rows);
  double var = s2 / static_cast<double>(rows) - m * m;
  if (var < 0) var = 0;
  const float mf = static_cast<float>(m);
  const float vf = static_cast<float>(var);
  mean[c] = mf;
  invstd[c] = 1.f / sqrtf(vf + eps);
  if (rmean != nullptr) {
    const float unb = rows > 1 ? static_cast<float>(var * static_cast<double>(rows) / static_cast<double>(rows - 1)) : vf;
    rmean[c] = momentum * mf + (1.f - momentum) * rmean[c];
    rvar[c] = momentum * unb + (1.f - momentum) * rvar[c];
  }
}

// The per-element BN passes walk [rows][C] as float4 lanes with a grid whose total thread count x 4
// is a multiple of C (bn_ew_grid): a thread's channel group never changes along its grid-stride
// loop, so its per-channel terms are loaded once instead of with every float4 (four or five extra
// 16-B loads per 16 B of data held them at ~4.5 TB/s), and each thread keeps ~8 float4s in flight.
inline unsigned bn_ew_grid(int64_t n4, int C) {
  int64_t g = (n4 + kThreads * 8 - 1) / (kThreads * 8);
  const int64_t q = C > 4 * kThreads ? C / (4 * kThreads) : 1;   // g * 4 * kThreads % C == 0
  g = (g + q - 1) / q * q;
  return static_cast<unsigned>(g < q ? q : g);
}

// z = relu?(((y - mean) * invstd) * gamma + beta [+ res]) over [rows][C], float4 lanes
__global__ void __launch_bounds__(kThreads)
bn_act_kernel(const float* __restrict__ y, const float* __restrict__ mean, const float* __restrict__ invstd,
              const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ res,
              int relu, int64_t n4, int C, float* __restrict__ z) {
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i0 >= n4) return;
  // per-channel terms as 16-B loads (c % 4 == 0), once: c is the same for every i of the thread
  const int c = static_cast<int>((i0 * 4) & (C - 1));
  const float4 m4 = *reinterpret_cast<const float4*>(mean + c);
  const float4 s4 = *reinterpret_cast<const float4*>(invstd + c);
  const float4 g4 = ld4_or(gamma, c, 1.f), b4 = ld4_or(beta, c, 0.f);
  const float cm[4] = {m4.x, m4.y, m4.z, m4.w}, cs[4] = {s4.x, s4.y, s4.z, s4.w};
  const float cg[4] = {g4.x, g4.y, g4.z, g4.w}, cb[4] = {b4.x, b4.y, b4.z, b4.w};
  for (int64_t i = i0; i < n4; i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(y)[i];
    float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = bn_value(o[j], cm[j], cs[j], cg[j], cb[j]);
    if (res != nullptr) {
      const float4 rv = reinterpret_cast<const float4*>(res)[i];
      o[0] += rv.x; o[1] += rv.y; o[2] += rv.z; o[3] += rv.w;
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    reinterpret_cast<float4*>(z)[i] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// BN backward finalize: dbeta = S1, dgamma = invstd * (S2 - mean * S1) with S2 = sum(dr * y);
// coefficients for dy = a * (dr - b - (y - mean) * d):
//   a = gamma * invstd, b = S1 / rows, d = invstd^2 * (S2 - mean * S1) / rows
__global__ void __launch_bounds__(kThreads)
bn_bwd_final_kernel(const double* __restrict__ ws, int G, int C, int64_t rows, const float* __restrict__ mean,
                    const float* __restrict__ invstd, const float* __restrict__ gamma, float* __restrict__ dgamma,
                    float* __restrict__ dbeta, int accumulate, float* __restrict__ coef) {
  int c;
  double s1, s2;
  if (!split_sums(ws, G, C, c, s1, s2)) return;
  const double is = invstd[c];
  const double sx = s2 - static_cast<double>(mean[c]) * s1;   // sum(dr * (y - mean))
  const float dg = static_cast<float>(is * sx);
  const float db = static_cast<float>(s1);
  if (dgamma != nullptr) dgamma[c] = accumulate ? dgamma[c] + dg : dg;
  if (dbeta != nullptr) dbeta[c] = accumulate ? dbeta[c] + db : db;
  const double g = gamma != nullptr ? gamma[c] : 1.0;
  coef[c] = static_cast<float>(g * is);
  coef[C + c] = static_cast<float>(s1 / static_cast<double>(rows));
  coef[2 * C + c] = static_cast<float>(is * is * sx / static_cast<double>(rows));
}

__global__ void __launch_bounds__(kThreads)
bn_bwd_apply_kernel(const float* dz, const float* __restrict__ z, const float* __restrict__ y,
                    const float* __restrict__ mean, const float* __restrict__ coef, int relu, int64_t n4, int C,
                    float* dy, float* dres, int dres_acc, const float* __restrict__ invstd,
                    const float* __restrict__ gamma, const float* __restrict__ beta) {
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i0 >= n4) return;
  // per-channel terms once (bn_ew_grid: c is the same for every i of the thread); coef's three
  // rows are C floats each
  const int c = static_cast<int>((i0 * 4) & (C - 1));
  const bool ymask = relu && z == nullptr;             // mask recomputed: bn_value(y) > 0
  const float4 m4 = *reinterpret_cast<const float4*>(mean + c);
  const float4 s4 = ymask ? *reinterpret_cast<const float4*>(invstd + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 g4 = ld4_or(ymask ? gamma : nullptr, c, 1.f), bb4 = ld4_or(ymask ? beta : nullptr, c, 0.f);
  const float4 a4 = *reinterpret_cast<const float4*>(coef + c);
  const float4 b4 = *reinterpret_cast<const float4*>(coef + C + c);
  const float4 d4 = *reinterpret_cast<const float4*>(coef + 2 * C + c);
  const float cm[4] = {m4.x, m4.y, m4.z, m4.w}, cs[4] = {s4.x, s4.y, s4.z, s4.w};
  const float cg[4] = {g4.x, g4.y, g4.z, g4.w}, cbb[4] = {bb4.x, bb4.y, bb4.z, bb4.w};
  const float ca[4] = {a4.x, a4.y, a4.z, a4.w}, cb[4] = {b4.x, b4.y, b4.z, b4.w};
  const float cd[4] = {d4.x, d4.y, d4.z, d4.w};
  for (int64_t i = i0; i < n4; i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const float4 gv = reinterpret_cast<const float4*>(dz)[i];
    float dr[4] = {gv.x, gv.y, gv.z, gv.w};
    const float4 yv = reinterpret_cast<const float4*>(y)[i];
    const float yy[4] = {yv.x, yv.y, yv.z, yv.w};
    if (ymask) {
#pragma unroll
      for (int j = 0; j < 4; ++j) dr[j] = bn_value(yy[j], cm[j], cs[j], cg[j], cbb[j]) > 0.f ? dr[j] : 0.f;
    } else if (relu) {
      const float4 zv = reinterpret_cast<const float4*>(z)[i];
      dr[0] = zv.x > 0.f ? dr[0] : 0.f;
      dr[1] = zv.y > 0.f ? dr[1] : 0.f;
      dr[2] = zv.z > 0.f ? dr[2] : 0.f;
      dr[3] = zv.w > 0.f ? dr[3] : 0.f;
    }
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = ca[j] * (dr[j] - cb[j] - (yy[j] - cm[j]) * cd[j]);
    if (dres != nullptr) {
      float4 rv = make_float4(dr[0], dr[1], dr[2], dr[3]);
      if (dres_acc) {
        const float4 old = reinterpret_cast<const float4*>(dres)[i];
        rv.x += old.x; rv.y += old.y; rv.z += old.z; rv.w += old.w;
      }
      reinterpret_cast<float4*>(dres)[i] = rv;
    }
    reinterpret_cast<float4*>(dy)[i] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

__global__ void __launch_bounds__(kThreads)
colsum_final_kernel(const double* __restrict__ ws, int G, int C, int cvalid, float* __restrict__ out, int acc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cvalid) return;
  double s = 0;
  for (int g = 0; g < G; ++g) s += ws[static_cast<int64_t>(g) * C + c];
  out[c] = acc ? out[c] + static_cast<float>(s) : static_cast<float>(s);
}

// ------------------------------------------------------------------ weight gradient
// dW[co][tap][ci] = sum_m dy[m][co] * x[pix(m, tap)][ci]: C = A * B with A = dy^T (co x m),
// B = im2col(x) (m x k).  Tile 64 co x 64 k per workgroup (4 waves, 32 x 32 each, 2 x 2
// fragments of v_mfma_f32_16x16x4f32), K loop over 32-pixel chunks of the block's pixel
// split.  Operand tiles go to LDS transposed ([row][m]) so one ds_read_b128 feeds 4 MFMAs:
// lane l reads m = mm + 4*(l/16) + {0..3}; MFMA j consumes element j of both operands,
// so the pairing of A and B over m is identical and the 4 MFMAs together cover 16 pixels.
struct WgradP {
  const float* dy;
  const float* x;
  float* ws;
  int dys, cout;
  int n, h, w, cs, ho, wo, ks, stride, pad, dil;
  int K;                 // ks * ks * cs
  int64_t M;
  int64_t pix_per_split;
};

constexpr int kWT = 64;      // tile rows / cols
constexpr int kWM = 32;      // pixels per chunk
constexpr int kWLD = kWM + 4;

// X6 (fp32x fine-tune): the same tiles and chunks, each 32-pixel chunk one K step of
// v_mfma_f32_16x16x32_bf16 on the exact 3-way bf16 splits of both operands (common.h split3),
// the six products above 2^-24 in conv_x6's order -- fp32-class accuracy at the bf16 MFMA rate
// (2.5 PF / 6 = 417 TF against the 157 TF of the f32 MFMA).  Lane (fr, fq) takes pixels
// 8 fq .. 8 fq + 7 of the chunk for its A row and its B column alike, so the pairing over m holds.
template <bool X6>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) wgrad_kernel(const WgradP p) {
  __shared__ __attribute__((aligned(16))) float As[2][kWT][kWLD];
  __shared__ __attribute__((aligned(16))) float Bs[2][kWT][kWLD];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wr = wave >> 1, wcn = wave & 1;
  const int co0 = blockIdx.y * kWT;
  const int kc0 = blockIdx.x * kWT;
  const int64_t m_begin = static_cast<int64_t>(blockIdx.z) * p.pix_per_split;
  int64_t m_end = m_begin + p.pix_per_split;
  if (m_end > p.M) m_end = p.M;
  // the transposed LDS writes As[8 lv + j][lm] hit bank (4 j + lm) % 32 whatever lv is (rows are
  // 36 floats, 8 rows = 288 = 0 mod 32): with 8 pixels x 8 column groups per wave every write was
  // 8-way conflicted; 32 pixels per 32-lane half (lm = t % 32) makes them conflict-free, at 64 B
  // per pixel per load instruction pair instead of 256 B
  const int lm = t & 31;      // pixel row of the chunk this thread loads
  const int lv = t >> 5;      // 8-column group
  const int hw = p.ho * p.wo;
  // B column group: (tap, ci) fixed for the whole loop
  const int kcol = kc0 + 8 * lv;
  const int tap = kcol / p.cs;
  const int ci = kcol - tap * p.cs;
  const bool kval = kcol < p.K && tap < p.ks * p.ks;
  const int kh = kval ? tap / p.ks : 0;
  const int kw = kval ? tap - kh * p.ks : 0;
  const int co = co0 + 8 * lv;

  // The thread's pixel advances by kWM per chunk: (n, oh, ow) are stepped, not divided out of m
  // every chunk (an int64 division per chunk and thread), and two register sets keep two chunks
  // of global loads in flight (chunk c + 2 loads while chunk c computes and chunk c + 1 is staged).
  int64_t m_cur = m_begin + lm;
  int p_n = 0, p_oh = 0, p_ow = 0;
  {
    const int mi = static_cast<int>(m_cur < p.M ? m_cur : 0);   // M < 2^31 (wgrad_check rejects larger)
    p_n = mi / hw;
    const int q = mi - p_n * hw;
    p_oh = q / p.wo;
    p_ow = q - p_oh * p.wo;
  }
  auto load = [&](float (&ra)[8], float (&rb)[8]) {
    const int64_t m = m_cur;
    const int nn = p_n, oh = p_oh, ow = p_ow;
    m_cur += kWM;
    p_ow += kWM;
    while (p_ow >= p.wo) {
      p_ow -= p.wo;
      if (++p_oh == p.ho) {
        p_oh = 0;
        ++p_n;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { ra[j] = 0.f; rb[j] = 0.f; }
    if (m >= m_end) return;
    const float* dr = p.dy + m * p.dys;
    if (co + 8 <= p.dys && co + 8 <= p.cout) {
      const float4 a0 = *reinterpret_cast<const float4*>(dr + co);
      const float4 a1 = *reinterpret_cast<const float4*>(dr + co + 4);
      ra[0] = a0.x; ra[1] = a0.y; ra[2] = a0.z; ra[3] = a0.w;
      ra[4] = a1.x; ra[5] = a1.y; ra[6] = a1.z; ra[7] = a1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (co + j < p.cout) ra[j] = dr[co + j];
    }
    if (kval) {
      const int ih = oh * p.stride - p.pad + kh * p.dil;
      const int iw = ow * p.stride - p.pad + kw * p.dil;
      if (static_cast<unsigned>(ih) < static_cast<unsigned>(p.h) && static_cast<unsigned>(iw) < static_cast<unsigned>(p.w)) {
        const float* xr = p.x + ((static_cast<int64_t>(nn) * p.h + ih) * p.w + iw) * p.cs + ci;
        const float4 b0 = *reinterpret_cast<const float4*>(xr);
        const float4 b1 = *reinterpret_cast<const float4*>(xr + 4);
        rb[0] = b0.x; rb[1] = b0.y; rb[2] = b0.z; rb[3] = b0.w;
        rb[4] = b1.x; rb[5] = b1.y; rb[6] = b1.z; rb[7] = b1.w;
      }
    }
  };
  auto store = [&](int buf, const float (&ra)[8], const float (&rb)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      As[buf][8 * lv + j][lm] = ra[j];
      Bs[buf][8 * lv + j][lm] = rb[j];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15;
  const int fq = lane >> 4;
  auto compute = [&](int buf) {
    if constexpr (X6) {
      // B splits first, then one A row block at a time (fewer live split registers: the kernel
      // fits 128 VGPRs, four waves per SIMD, without spilling); same MFMA order per accumulator
      bf16x8 b[2][3];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const float* br = &Bs[buf][wcn * 32 + f * 16 + fr][8 * fq];
        split3(*reinterpret_cast<const float4*>(br), *reinterpret_cast<const float4*>(br + 4), b[f][0], b[f][1], b[f][2]);
      }
#pragma unroll
      for (int fi = 0; fi < 2; ++fi) {
        if (co0 + wr * 32 + fi * 16 >= p.cout) continue;   // rows past cout (16- and 32-channel layers)
        bf16x8 a[3];
        const float* ar = &As[buf][wr * 32 + fi * 16 + fr][8 * fq];
        split3(*reinterpret_cast<const float4*>(ar), *reinterpret_cast<const float4*>(ar + 4), a[0], a[1], a[2]);
#pragma unroll
        for (int fj = 0; fj < 2; ++fj) {
          f32x4& c = acc[fi][fj];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[fj][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[fj][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[fj][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][0], c, 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int mm = 0; mm < kWM; mm += 16) {
        float4 a4[2], b4[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          a4[f] = *reinterpret_cast<const float4*>(&As[buf][wr * 32 + f * 16 + fr][mm + 4 * fq]);
          b4[f] = *reinterpret_cast<const float4*>(&Bs[buf][wcn * 32 + f * 16 + fr][mm + 4 * fq]);
        }
#pragma unroll
        for (int fi = 0; fi < 2; ++fi) {
          if (co0 + wr * 32 + fi * 16 >= p.cout) continue;
#pragma unroll
          for (int fj = 0; fj < 2; ++fj) {
            acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[fi].x, b4[fj].x, acc[fi][fj], 0, 0, 0);
            acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[fi].y, b4[fj].y, acc[fi][fj], 0, 0, 0);
            acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[fi].z, b4[fj].z, acc[fi][fj], 0, 0, 0);
            acc[fi][fj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[fi].w, b4[fj].w, acc[fi][fj], 0, 0, 0);
          }
        }
      }
    }
  };

  // chunk c computes from LDS buffer c & 1; set X holds chunk c + 1 (staged after the compute),
  // set Y receives chunk c + 2 (its loads fly across the compute of c and the staging of c + 1)
  float r0a[8], r0b[8], r1a[8], r1b[8];
  load(r0a, r0b);
  store(0, r0a, r0b);
  load(r0a, r0b);                                   // chunk 1
  __syncthreads();
  for (int64_t mc = m_begin; mc < m_end; mc += 2 * kWM) {
    load(r1a, r1b);                                 // chunk c + 2 (zeros past the end)
    compute(0);
    if (mc + kWM < m_end) store(1, r0a, r0b);
    __syncthreads();
    if (mc + kWM >= m_end) break;
    load(r0a, r0b);                                 // chunk c + 3
    compute(1);
    if (mc + 2 * kWM < m_end) store(0, r1a, r1b);
    __syncthreads();
  }
  // D[row = 4*(l/16) + r][col = l%16] of each 16x16 fragment; rows = co, cols = k
  float* out = p.ws + static_cast<int64_t>(blockIdx.z) * p.cout * p.K;
#pragma unroll
  for (int fi = 0; fi < 2; ++fi)
#pragma unroll
    for (int fj = 0; fj < 2; ++fj) {
      const int k = kc0 + wcn * 32 + fj * 16 + fr;
      if (k >= p.K) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = co0 + wr * 32 + fi * 16 + 4 * fq + r;
        if (c < p.cout) out[static_cast<int64_t>(c) * p.K + k] = acc[fi][fj][r];
      }
    }
}

// The fp32x weight gradient on a 128 co x 128 k tile (cout and K >= 128): four waves of 64 x 64
// (4 x 4 fragments), so every staged byte feeds twice the MFMAs of the 64 x 64 tile.  Same chunks,
// staging map (32 pixels per 32-lane half: conflict-free transposed writes), two register sets of
// loads in flight, split order and MFMA order per accumulator as wgrad_kernel<true>; the split of a
// B fragment is done once per chunk and reused by the wave's four row blocks.  Two workgroups per
// CU (2 x 2 x 128 x 36 floats of LDS each).
constexpr int kWT2 = 128;
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) wgrad_x6_big_kernel(const WgradP p) {
  __shared__ __attribute__((aligned(16))) float As[2][kWT2][kWLD];
  __shared__ __attribute__((aligned(16))) float Bs[2][kWT2][kWLD];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wr = wave >> 1, wcn = wave & 1;
  const int co0 = blockIdx.y * kWT2;
  const int kc0 = blockIdx.x * kWT2;
  const int64_t m_begin = static_cast<int64_t>(blockIdx.z) * p.pix_per_split;
  int64_t m_end = m_begin + p.pix_per_split;
  if (m_end > p.M) m_end = p.M;
  const int lm = t & 31;      // pixel row of the chunk this thread loads
  const int lv = t >> 5;      // 16-column group
  const int hw = p.ho * p.wo;
  const int kcol = kc0 + 16 * lv;                  // 16 consecutive k stay in one tap (cs % 16 == 0)
  const int tap = kcol / p.cs;
  const int ci = kcol - tap * p.cs;
  const bool kval = kcol < p.K && tap < p.ks * p.ks;
  const int kh = kval ? tap / p.ks : 0;
  const int kw = kval ? tap - kh * p.ks : 0;
  const int co = co0 + 16 * lv;

  int64_t m_cur = m_begin + lm;
  int p_n = 0, p_oh = 0, p_ow = 0;
  {
    const int mi = static_cast<int>(m_cur < p.M ? m_cur : 0);
    p_n = mi / hw;
    const int q = mi - p_n * hw;
    p_oh = q / p.wo;
    p_ow = q - p_oh * p.wo;
  }
  auto load = [&](float4 (&ra)[4], float4 (&rb)[4]) {
    const int64_t m = m_cur;
    const int nn = p_n, oh = p_oh, ow = p_ow;
    m_cur += kWM;
    p_ow += kWM;
    while (p_ow >= p.wo) {
      p_ow -= p.wo;
      if (++p_oh == p.ho) {
        p_oh = 0;
        ++p_n;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ra[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      rb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (m >= m_end) return;
    const float* dr = p.dy + m * p.dys;
    if (co + 16 <= p.dys && co + 16 <= p.cout) {
#pragma unroll
      for (int j = 0; j < 4; ++j) ra[j] = *reinterpret_cast<const float4*>(dr + co + 4 * j);
    } else {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = co + j < p.cout ? dr[co + j] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) ra[j] = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    }
    if (kval) {
      const int ih = oh * p.stride - p.pad + kh * p.dil;
      const int iw = ow * p.stride - p.pad + kw * p.dil;
      if (static_cast<unsigned>(ih) < static_cast<unsigned>(p.h) && static_cast<unsigned>(iw) < static_cast<unsigned>(p.w)) {
        const float* xr = p.x + ((static_cast<int64_t>(nn) * p.h + ih) * p.w + iw) * p.cs + ci;
#pragma unroll
        for (int j = 0; j < 4; ++j) rb[j] = *reinterpret_cast<const float4*>(xr + 4 * j);
      }
    }
  };
  auto store = [&](int buf, const float4 (&ra)[4], const float4 (&rb)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float av[4] = {ra[j].x, ra[j].y, ra[j].z, ra[j].w};
      const float bv[4] = {rb[j].x, rb[j].y, rb[j].z, rb[j].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        As[buf][16 * lv + 4 * j + e][lm] = av[e];
        Bs[buf][16 * lv + 4 * j + e][lm] = bv[e];
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15;
  const int fq = lane >> 4;
  auto compute = [&](int buf) {
    bf16x8 b[4][3];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const float* br = &Bs[buf][wcn * 64 + f * 16 + fr][8 * fq];
      split3(*reinterpret_cast<const float4*>(br), *reinterpret_cast<const float4*>(br + 4), b[f][0], b[f][1], b[f][2]);
    }
#pragma unroll
    for (int fi = 0; fi < 4; ++fi) {
      bf16x8 a[3];
      const float* ar = &As[buf][wr * 64 + fi * 16 + fr][8 * fq];
      split3(*reinterpret_cast<const float4*>(ar), *reinterpret_cast<const float4*>(ar + 4), a[0], a[1], a[2]);
#pragma unroll
      for (int fj = 0; fj < 4; ++fj) {
        f32x4& c = acc[fi][fj];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[fj][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[fj][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[fj][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][0], c, 0, 0, 0);
      }
    }
  };

  float4 r0a[4], r0b[4], r1a[4], r1b[4];
  load(r0a, r0b);
  store(0, r0a, r0b);
  load(r0a, r0b);
  __syncthreads();
  for (int64_t mc = m_begin; mc < m_end; mc += 2 * kWM) {
    load(r1a, r1b);
    compute(0);
    if (mc + kWM < m_end) store(1, r0a, r0b);
    __syncthreads();
    if (mc + kWM >= m_end) break;
    load(r0a, r0b);
    compute(1);
    if (mc + 2 * kWM < m_end) store(0, r1a, r1b);
    __syncthreads();
  }
  float* out = p.ws + static_cast<int64_t>(blockIdx.z) * p.cout * p.K;
#pragma unroll
  for (int fi = 0; fi < 4; ++fi)
#pragma unroll
    for (int fj = 0; fj < 4; ++fj) {
      const int k = kc0 + wcn * 64 + fj * 16 + fr;
      if (k >= p.K) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = co0 + wr * 64 + fi * 16 + 4 * fq + r;
        if (c < p.cout) out[static_cast<int64_t>(c) * p.K + k] = acc[fi][fj][r];
      }
    }
}

// ---- fp32x weight gradient, dy pre-split -----------------------------------------------------
// The 128 x 128 tile above splits every dy and x value in each of the two waves that read it
// (~4.4 VALU instructions per MFMA: VALU-bound, MFMA busy 0.31, profiles/r5r_wgrad_pmc).  Here dy
// is split once per launch into three transposed bf16 planes [plane][co][m] (one HBM pass,
// wgrad_dy_split_kernel) that the tile stages with LDS-DMA like conv_x6's weight planes: the
// kernel splits only x.  Same split3 (RNE) of the same values and the same MFMA order per
// accumulator as wgrad_x6_big_kernel, so the partial sums are bit-identical to it.
constexpr int kPreRows = kWT2;   // dyT rows padded to a multiple of the tile (zero rows)
__device__ float4 g_wgrad_zero[4];   // zero-initialised: the B source outside the image

// LDS byte address of a __shared__ object; one ds_read_b128 at LDS address base + OFF
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)p));
}
template <int OFF, typename V>
__device__ __forceinline__ void ds_rd(V& dst, uint32_t base) {
  static_assert(sizeof(V) == 16 && OFF >= 0 && OFF < 65536, "ds_read_b128 offset");
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(OFF));
}
// one 16-B-per-lane LDS-DMA (global_load_lds_dwordx4) to the wave-uniform LDS address `lds`
// (M0 holds the LDS address; its previous value is restored, as M0 is reserved to the compiler)
__device__ __forceinline__ void dma16(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
__device__ __forceinline__ int pre_swz_a(int row) { return ((row >> 3) & 1) * 3; }          // 64-B bf16 rows
__device__ __forceinline__ int pre_swz_b(int row) { return ((row >> 1) & 1) | (row & 4); }  // 128-B fp32 rows
// transposed B write of row RR (0..15) of a thread's 16-row group: w[k] holds the lane address for
// swizzle value k -> (0, 1, 4, 5)
template <int RR>
__device__ __forceinline__ void pre_wr(const uint32_t (&w)[4], float v) {
  constexpr int k = ((RR >> 1) & 1) | (((RR >> 2) & 1) << 1);
  asm volatile("ds_write_b32 %0, %1 offset:%2" :: "v"(w[k]), "v"(v), "i"(RR * 128) : "memory");
}

__global__ void __launch_bounds__(kThreads)
wgrad_dy_split_kernel(const float* __restrict__ dy, int dys, int cout, int64_t M, int64_t Mp, int Cp,
                      bf16_t* __restrict__ out) {
  // thread: channel co = 64-channel block + t / 4, pixels 8 (t % 4) .. +7 of a 32-pixel group:
  // four lanes write one channel's 64-B row piece per plane; each read instruction is 16
  // consecutive channels (64 B) of 4 pixels
  const int t = threadIdx.x;
  const int64_t ngroups = Mp / 32;
  const int cblocks = Cp / 64;
  const int64_t total = ngroups * cblocks;
  const int64_t pstride = static_cast<int64_t>(Cp) * Mp;
  for (int64_t b = blockIdx.x; b < total; b += gridDim.x) {
    const int cb = static_cast<int>(b % cblocks);
    const int64_t g = b / cblocks;
    const int co = cb * 64 + (t >> 2);
    const int64_t m0 = g * 32 + 8 * (t & 3);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = (co < cout && m0 + j < M) ? dy[(m0 + j) * dys + co] : 0.f;
    bf16x8 h1, h2, h3;
    split3(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), h1, h2, h3);
    bf16_t* o = out + static_cast<int64_t>(co) * Mp + m0;
    *reinterpret_cast<bf16x8*>(o) = h1;
    *reinterpret_cast<bf16x8*>(o + pstride) = h2;
    *reinterpret_cast<bf16x8*>(o + 2 * pstride) = h3;
  }
}

struct WgradPreP {
  WgradP p;
  const bf16_t* dyt;   // [3][Cp][Mp]
  int64_t Mp;
  int Cp;
};

__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) wgrad_x6_pre_kernel(const WgradPreP q) {
  const WgradP& p = q.p;
  // A: [buf][plane][128 rows][64 B] bf16 (16-B chunks swizzled), B: [buf][128 rows][32 floats]
  // (16-B chunks swizzled): 2 x (24 + 16) KB, two workgroups per CU
  __shared__ __attribute__((aligned(16))) char Ab[2][3 * kWT2 * 64];
  __shared__ __attribute__((aligned(16))) float Bs[2][kWT2 * 32];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wr = wave >> 1, wcn = wave & 1;
  const int co0 = blockIdx.y * kWT2;
  const int kc0 = blockIdx.x * kWT2;
  const int64_t m_begin = static_cast<int64_t>(blockIdx.z) * p.pix_per_split;
  int64_t m_end = m_begin + p.pix_per_split;
  if (m_end > p.M) m_end = p.M;
  const int lm = t & 31;
  const int lv = t >> 5;
  const int hw = p.ho * p.wo;
  const int kcol = kc0 + 16 * lv;
  const int tap = kcol / p.cs;
  const int ci = kcol - tap * p.cs;
  const bool kval = kcol < p.K && tap < p.ks * p.ks;
  const int kh = kval ? tap / p.ks : 0;
  const int kw = kval ? tap - kh * p.ks : 0;

  // A DMA: 24 pieces of 1 KB per chunk, 6 per wave; piece gi = plane * 8 + 16-row block.  Sources
  // as element offsets from the block's first row (< 2^31: 3 x 128 rows x Mp), not 64-bit pointers
  // (six of those spilled to scratch, and the reload waited on every load in flight)
  const int64_t plane_stride = static_cast<int64_t>(q.Cp) * q.Mp;
  const bf16_t* a_base = q.dyt + static_cast<int64_t>(co0) * q.Mp;
  int32_t a_off[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int gi = wave * 6 + i;
    const int pl = gi >> 3;
    const int r = (gi & 7) * 16 + (lane >> 2);
    const int c = (lane & 3) ^ pre_swz_a(r);
    a_off[i] = static_cast<int32_t>(pl * plane_stride + static_cast<int64_t>(r) * q.Mp + 8 * c);
  }
  // as inline asm: hipcc models the LDS-DMA builtin's address registers as pending until vmcnt(0)
  // and drained the B loads in flight the first time it reused one
  const uint32_t a_dst = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(lds_addr(&Ab[0][wave * 6 * 1024]))));
  auto dma_a = [&](int buf, int64_t m) {
    const bf16_t* src = a_base + m;
#pragma unroll
    for (int i = 0; i < 6; ++i) dma16(src + a_off[i], a_dst + buf * static_cast<uint32_t>(sizeof(Ab[0])) + i * 1024);
  };

  int64_t m_cur = m_begin + lm;
  int p_n = 0, p_oh = 0, p_ow = 0;
  {
    const int mi = static_cast<int>(m_cur < p.M ? m_cur : 0);
    p_n = mi / hw;
    const int qq = mi - p_n * hw;
    p_oh = qq / p.wo;
    p_ow = qq - p_oh * p.wo;
  }
  // exactly four 16-B loads per call (the zero page outside the image / past the split), so that
  // the chunk-end wait below can leave them in flight with a fixed vmcnt
  auto load = [&](float4 (&rb)[4]) {
    const int64_t m = m_cur;
    const int nn = p_n, oh = p_oh, ow = p_ow;
    m_cur += kWM;
    p_ow += kWM;
    while (p_ow >= p.wo) {
      p_ow -= p.wo;
      if (++p_oh == p.ho) {
        p_oh = 0;
        ++p_n;
      }
    }
    const float* xr = reinterpret_cast<const float*>(g_wgrad_zero);
    const int ih = oh * p.stride - p.pad + kh * p.dil;
    const int iw = ow * p.stride - p.pad + kw * p.dil;
    if (m < m_end && kval && static_cast<unsigned>(ih) < static_cast<unsigned>(p.h) &&
        static_cast<unsigned>(iw) < static_cast<unsigned>(p.w))
      xr = p.x + ((static_cast<int64_t>(nn) * p.h + ih) * p.w + iw) * p.cs + ci;
#pragma unroll
    for (int j = 0; j < 4; ++j) rb[j] = *reinterpret_cast<const float4*>(xr + 4 * j);
  };
  // transposed B writes as inline asm as well (a C++ LDS store made hipcc wait vmcnt(0) for the
  // DMA in flight); row 16 lv + 4 j + e: its swizzle depends on 4 j + e only
  const uint32_t bs_w = lds_addr(&Bs[0][0]) + static_cast<uint32_t>(16 * lv * 128 + 4 * (lm & 3));
  auto store = [&](int buf, const float4 (&rb)[4]) {
    const uint32_t base = bs_w + buf * static_cast<uint32_t>(sizeof(Bs[0]));
    // one lane address per swizzle value (0, 1, 4, 5); the row is the instruction's offset
    const uint32_t w[4] = {base + 16u * ((lm >> 2) ^ 0), base + 16u * ((lm >> 2) ^ 1), base + 16u * ((lm >> 2) ^ 4),
                           base + 16u * ((lm >> 2) ^ 5)};
    pre_wr<0>(w, rb[0].x); pre_wr<1>(w, rb[0].y); pre_wr<2>(w, rb[0].z); pre_wr<3>(w, rb[0].w);
    pre_wr<4>(w, rb[1].x); pre_wr<5>(w, rb[1].y); pre_wr<6>(w, rb[1].z); pre_wr<7>(w, rb[1].w);
    pre_wr<8>(w, rb[2].x); pre_wr<9>(w, rb[2].y); pre_wr<10>(w, rb[2].z); pre_wr<11>(w, rb[2].w);
    pre_wr<12>(w, rb[3].x); pre_wr<13>(w, rb[3].y); pre_wr<14>(w, rb[3].z); pre_wr<15>(w, rb[3].w);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15;
  const int fq = lane >> 4;
  // Fragment reads as inline-asm ds_read_b128 with hand-counted lgkmcnt waits: hipcc cannot tell
  // that the LDS-DMA in flight targets the other buffer, and put a vmcnt(0) before the first C++
  // read of the chunk (draining the B loads issued for two chunks ahead).  The swizzles depend on
  // row bits the fragment offsets (16 rows apart) do not change, so one lane address per operand.
  const uint32_t ab_lds = lds_addr(&Ab[0][0]), bs_lds = lds_addr(&Bs[0][0]);
  uint32_t b_lane[2], a_lane;
  {
    const int rb = wcn * 64 + fr;
    b_lane[0] = bs_lds + static_cast<uint32_t>(rb * 128 + 16 * ((2 * fq) ^ pre_swz_b(rb)));
    b_lane[1] = bs_lds + static_cast<uint32_t>(rb * 128 + 16 * ((2 * fq + 1) ^ pre_swz_b(rb)));
    const int ra = wr * 64 + fr;
    a_lane = ab_lds + static_cast<uint32_t>(ra * 64 + 16 * (fq ^ pre_swz_a(ra)));
  }
  static_assert(sizeof(Bs[0]) == kWT2 * 128 && sizeof(Ab[0]) == 3 * kWT2 * 64, "LDS buffer strides");
  auto compute = [&](int buf) {
    const uint32_t vb0 = b_lane[0] + buf * static_cast<uint32_t>(sizeof(Bs[0]));
    const uint32_t vb1 = b_lane[1] + buf * static_cast<uint32_t>(sizeof(Bs[0]));
    const uint32_t va = a_lane + buf * static_cast<uint32_t>(sizeof(Ab[0]));
    float4 blo[4], bhi[4];
    ds_rd<0>(blo[0], vb0); ds_rd<0>(bhi[0], vb1);
    ds_rd<2048>(blo[1], vb0); ds_rd<2048>(bhi[1], vb1);
    ds_rd<4096>(blo[2], vb0); ds_rd<4096>(bhi[2], vb1);
    ds_rd<6144>(blo[3], vb0); ds_rd<6144>(bhi[3], vb1);
    bf16x8 a[3];
    ds_rd<0>(a[0], va); ds_rd<kWT2 * 64>(a[1], va); ds_rd<2 * kWT2 * 64>(a[2], va);
    // the reads are asm: their results are valid only after the counted wait, and a
    // sched_barrier after each wait keeps the scheduler from hoisting their uses above it
    asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 b[4][3];
#pragma unroll
    for (int f = 0; f < 4; ++f) split3(blo[f], bhi[f], b[f][0], b[f][1], b[f][2]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int fi = 0; fi < 4; ++fi) {
      bf16x8 an[3];
      // the next fragment's three planes (rows 16 apart: +1 KB), read under this one's MFMAs
      switch (fi) {
        case 0: ds_rd<1024>(an[0], va); ds_rd<1024 + kWT2 * 64>(an[1], va); ds_rd<1024 + 2 * kWT2 * 64>(an[2], va); break;
        case 1: ds_rd<2048>(an[0], va); ds_rd<2048 + kWT2 * 64>(an[1], va); ds_rd<2048 + 2 * kWT2 * 64>(an[2], va); break;
        case 2: ds_rd<3072>(an[0], va); ds_rd<3072 + kWT2 * 64>(an[1], va); ds_rd<3072 + 2 * kWT2 * 64>(an[2], va); break;
        default: break;
      }
#pragma unroll
      for (int fj = 0; fj < 4; ++fj) {
        f32x4& c = acc[fi][fj];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[fj][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[fj][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[fj][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[fj][0], c, 0, 0, 0);
      }
      if (fi < 3) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        a[0] = an[0];
        a[1] = an[1];
        a[2] = an[2];
      }
    }
  };

  // Chunk c computes from buffers c & 1.  At the start of its phase the B registers of chunk c + 1
  // (loaded during the previous phase) are written to the other buffer, chunk c + 1's A DMA goes to
  // it as well, then chunk c + 2's B loads are issued into the same registers -- so hipcc's wait for
  // those registers (it cannot count LDS-DMA and waits vmcnt(0)) drains nothing else.  The phase
  // ends with vmcnt(4) (the DMA landed, the four B loads stay in flight across the barrier) +
  // lgkmcnt(0) + s_barrier.  Compiler barriers keep the DMA ahead of the B loads in issue order.
  float4 rb[4];
  dma_a(0, m_begin);
  load(rb);                                        // chunk 0
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  store(0, rb);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  load(rb);                                        // chunk 1
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  int cur = 0;
  for (int64_t mc = m_begin; mc < m_end; mc += kWM, cur ^= 1) {
    store(cur ^ 1, rb);                            // chunk c + 1 (zeros past the split, never read)
    if (mc + kWM < m_end) dma_a(cur ^ 1, mc + kWM);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    load(rb);                                      // chunk c + 2 (the zero page past the split)
    __builtin_amdgcn_sched_barrier(0);
    compute(cur);
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  float* out = p.ws + static_cast<int64_t>(blockIdx.z) * p.cout * p.K;
#pragma unroll
  for (int fi = 0; fi < 4; ++fi)
#pragma unroll
    for (int fj = 0; fj < 4; ++fj) {
      const int k = kc0 + wcn * 64 + fj * 16 + fr;
      if (k >= p.K) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = co0 + wr * 64 + fi * 16 + 4 * fq + r;
        if (c < p.cout) out[static_cast<int64_t>(c) * p.K + k] = acc[fi][fj][r];
      }
    }
}

// ---- fp32x weight gradient of the small-cout convs (cout <= 32: stem, layer1, layer2) ----------
// The 64 x 64 tile left 3/4 of its rows idle at cout 16, and the stem's 8-channel input stride left
// 5/8 of its k columns zero (cin 3): 474 us for 20 GFLOP of the fine-tune step.  Here the MFMA
// operands come straight from global memory into registers -- no LDS, no barriers: lane (fr, fq)
// loads dy[m][16 fm + fr] and x[pix(m, tap)][ci] of its 8 pixels m = m0 + 8 fq + j, as the
// 16x16x32 bf16 A / B layouts ask -- and the k columns are the dense (tap, ci < cin) pairs only
// (147 at the stem instead of 392).  Each wave owns FN 16-column fragments and a contiguous range of
// 32-pixel chunks (one output row segment each: wo % 32 == 0) and writes its own partial sums,
// reduced in split order by wgrad_reduce*_kernel; same split3 and six-product order per
// accumulator as wgrad_kernel<true>.
constexpr int kDirFN = 4;
static bool wgrad_direct_ok(const drnmi_wgrad_args& a) {
  return a.cout <= 32 && a.wo % 32 == 0 && a.ks * a.ks * a.cin <= 4096;
}
static int wgrad_direct_tiles(const drnmi_wgrad_args& a) {
  return (a.ks * a.ks * a.cin + 16 * kDirFN - 1) / (16 * kDirFN);
}
// wave splits: ~2048 waves in all (8 per CU), whole workgroups of 4, <= one chunk per wave
static int wgrad_direct_splits(const drnmi_wgrad_args& a) {
  const int64_t chunks = static_cast<int64_t>(a.n) * a.ho * a.wo / 32;
  int64_t s = 2048 / wgrad_direct_tiles(a);
  if (s > chunks) s = chunks;
  s = (s + 3) / 4 * 4;
  return static_cast<int>(s < 4 ? 4 : s);
}

template <int FM>
__global__ void __launch_bounds__(kThreads) wgrad_x6_direct_kernel(const WgradP p, int cin) {
  const int lane = threadIdx.x & 63;
  const int z = blockIdx.y * 4 + (threadIdx.x >> 6);        // this wave's split
  const int nz = gridDim.y * 4;
  const int fr = lane & 15, fq = lane >> 4;
  const int hw = p.ho * p.wo;
  const int chunks = static_cast<int>(p.M / 32);
  const int c_begin = static_cast<int>(static_cast<int64_t>(chunks) * z / nz);
  const int c_end = static_cast<int>(static_cast<int64_t>(chunks) * (z + 1) / nz);
  const int kdense = p.ks * p.ks * cin;
  // the lane's B column of each fragment: dense column kv -> (tap, ci) -> tap offsets
  int b_dh[kDirFN], b_dw[kDirFN], b_ci[kDirFN];
  bool b_ok[kDirFN];
#pragma unroll
  for (int f = 0; f < kDirFN; ++f) {
    const int kv = (blockIdx.x * kDirFN + f) * 16 + fr;
    b_ok[f] = kv < kdense;
    const int tap = b_ok[f] ? kv / cin : 0;
    b_ci[f] = b_ok[f] ? kv - tap * cin : 0;
    const int kh = tap / p.ks;
    b_dh[f] = kh * p.dil - p.pad;
    b_dw[f] = (tap - kh * p.ks) * p.dil - p.pad;
  }
  f32x4 acc[FM][kDirFN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < kDirFN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c = c_begin; c < c_end; ++c) {
    const int m0 = c * 32;
    const int n = m0 / hw;
    const int q = m0 - n * hw;
    const int oh = q / p.wo;
    const int ow = q - oh * p.wo + 8 * fq;                 // the lane's first pixel (same row)
    const int64_t mrow = static_cast<int64_t>(m0 + 8 * fq) * p.dys;
    float av[FM][8], bv[kDirFN][8];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int co = 16 * fm + fr;
#pragma unroll
      for (int j = 0; j < 8; ++j) av[fm][j] = co < p.cout ? p.dy[mrow + static_cast<int64_t>(j) * p.dys + co] : 0.f;
    }
#pragma unroll
    for (int f = 0; f < kDirFN; ++f) {
      const int ih = oh * p.stride + b_dh[f];
      const bool row_ok = b_ok[f] && static_cast<unsigned>(ih) < static_cast<unsigned>(p.h);
      const float* xr = p.x + (static_cast<int64_t>(n) * p.h + (row_ok ? ih : 0)) * p.w * p.cs + b_ci[f];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int iw = (ow + j) * p.stride + b_dw[f];
        bv[f][j] = row_ok && static_cast<unsigned>(iw) < static_cast<unsigned>(p.w) ? xr[static_cast<int64_t>(iw) * p.cs] : 0.f;
      }
    }
    bf16x8 b[kDirFN][3];
#pragma unroll
    for (int f = 0; f < kDirFN; ++f)
      split3(make_float4(bv[f][0], bv[f][1], bv[f][2], bv[f][3]), make_float4(bv[f][4], bv[f][5], bv[f][6], bv[f][7]),
             b[f][0], b[f][1], b[f][2]);
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      bf16x8 a[3];
      split3(make_float4(av[fm][0], av[fm][1], av[fm][2], av[fm][3]),
             make_float4(av[fm][4], av[fm][5], av[fm][6], av[fm][7]), a[0], a[1], a[2]);
#pragma unroll
      for (int f = 0; f < kDirFN; ++f) {
        f32x4& cc = acc[fm][f];
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[f][0], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[f][1], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[f][2], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[f][0], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[f][1], cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[f][0], cc, 0, 0, 0);
      }
    }
  }
  // C[row = 16 fm + 4 fq + r][col = 16 f + fr] -> ws[z][co][tap * cs + ci] (the reduce skips ci >= cin)
  float* out = p.ws + static_cast<int64_t>(z) * p.cout * p.K;
#pragma unroll
  for (int f = 0; f < kDirFN; ++f) {
    if (!b_ok[f]) continue;
    const int kv = (blockIdx.x * kDirFN + f) * 16 + fr;
    const int tap = kv / cin;
    const int k = tap * p.cs + (kv - tap * cin);
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 16 * fm + 4 * fq + r;
        if (co < p.cout) out[static_cast<int64_t>(co) * p.K + k] = acc[fm][f][r];
      }
  }
}

// dw[co][ci][kh][kw] (+)= sum_z ws[z][co][(kh*ks + kw)*cs + ci]
__global__ void __launch_bounds__(kThreads)
wgrad_reduce_kernel(const float* __restrict__ ws, int splits, int cout, int cin, int cs, int ks, int K,
                    float* __restrict__ dw, int acc) {
  // threads walk the partials' own [co][k] order (k = tap * cs + ci), so each of the `splits`
  // reads is coalesced (walking dw's OIHW order read them ks*ks*... apart); dw is written once
  const int64_t total = static_cast<int64_t>(cout) * K;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int co = static_cast<int>(i / K);
    const int k = static_cast<int>(i - static_cast<int64_t>(co) * K);
    const int tap = k / cs;
    const int ci = k - tap * cs;
    if (ci >= cin) continue;
    // eight splits' loads in flight at a time, summed in split order (one load per add serialised
    // the chain on its latency)
    float s = 0.f;
    const int64_t zs = static_cast<int64_t>(cout) * K;
    int z = 0;
    for (; z + 8 <= splits; z += 8) {
      float a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = ws[(z + u) * zs + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += a[u];
    }
    for (; z < splits; ++z) s += ws[z * zs + i];
    const int64_t o = (static_cast<int64_t>(co) * cin + ci) * ks * ks + tap;   // tap = kh * ks + kw
    dw[o] = acc ? dw[o] + s : s;
  }
}

// Few outputs over many splits (the stem's 16 x 392 partials over 432 splits): one thread per
// output walked its splits as a chain of dependent loads on 18 workgroups (125 us).  Here 8
// threads share an output, each sums a contiguous eighth of the splits (8 loads in flight), and
// the eighths are added in order: a fixed order, so dw stays bit-reproducible.
constexpr int kRedOut = 32;
constexpr int kRedGrp = kThreads / kRedOut;

__global__ void __launch_bounds__(kThreads)
wgrad_reduce_grouped_kernel(const float* __restrict__ ws, int splits, int cout, int cin, int cs, int ks, int K,
                            float* __restrict__ dw, int acc) {
  __shared__ float part[kRedGrp][kRedOut];
  const int t = threadIdx.x;
  const int oi = t % kRedOut, g = t / kRedOut;
  const int64_t total = static_cast<int64_t>(cout) * K;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kRedOut + oi;
  const int z0 = static_cast<int>(static_cast<int64_t>(splits) * g / kRedGrp);
  const int z1 = static_cast<int>(static_cast<int64_t>(splits) * (g + 1) / kRedGrp);
  float s = 0.f;
  if (i < total) {
    const float* p = ws + i;
#pragma unroll 8
    for (int z = z0; z < z1; ++z) s += p[static_cast<int64_t>(z) * total];
  }
  part[g][oi] = s;
  __syncthreads();
  if (g != 0 || i >= total) return;
  const int co = static_cast<int>(i / K);
  const int k = static_cast<int>(i - static_cast<int64_t>(co) * K);
  const int tap = k / cs;
  const int ci = k - tap * cs;
  if (ci >= cin) return;
  float v = part[0][oi];
#pragma unroll
  for (int j = 1; j < kRedGrp; ++j) v += part[j][oi];
  const int64_t o = (static_cast<int64_t>(co) * cin + ci) * ks * ks + tap;
  dw[o] = acc ? dw[o] + v : v;
}

// The pixel range is split so that the launch fills the chip: at least two rounds of the resident
// workgroup slots, and among lo .. 4 lo splits the count whose last round is fullest (the first
// rule alone put D-54 layer7.0's 576 big tiles on 512 slots at one split: 1.125 rounds, the
// second round 1/8 full, 4.6 ms of a 52.8 ms fine-tune step).  Every split holds >= 512 pixels.
static bool wgrad_big_ok(const drnmi_wgrad_args& a) {
  const int K = a.ks * a.ks * a.cin_stride;
  return a.cout >= kWT2 && K >= kWT2 && a.cin_stride % 16 == 0;
}

static void wgrad_plan(const drnmi_wgrad_args& a, bool big, int* splits, int64_t* per) {
  const int K = a.ks * a.ks * a.cin_stride;
  const int tile = big ? kWT2 : kWT;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int64_t slots = (big ? 2 : 4) * static_cast<int64_t>(cus);   // resident workgroups: LDS 73.7 / 36.9 KB
  const int64_t M = static_cast<int64_t>(a.n) * a.ho * a.wo;
  const int64_t tiles = static_cast<int64_t>((a.cout + tile - 1) / tile) * ((K + tile - 1) / tile);
  int64_t smax = (M + 511) / 512;
  if (smax > 512) smax = 512;
  if (smax < 1) smax = 1;
  int64_t lo = (2 * slots + tiles - 1) / tiles;
  if (lo > smax) lo = smax;
  int64_t hi = 4 * lo < smax ? 4 * lo : smax;
  int64_t best_s = 0, best_pp = 0;
  double best_eff = -1.0;
  for (int64_t s = lo; s <= hi; ++s) {
    int64_t pp = (M + s - 1) / s;
    pp = (pp + kWM - 1) / kWM * kWM;
    const int64_t sa = (M + pp - 1) / pp;
    const int64_t wgs = tiles * sa;
    const int64_t rounds = (wgs + slots - 1) / slots;
    const double eff = static_cast<double>(wgs) / static_cast<double>(rounds * slots);
    if (eff > best_eff + 0.02) {     // a larger split count only for a clearly fuller last round
      best_eff = eff;
      best_s = sa;
      best_pp = pp;
    }
  }
  *splits = static_cast<int>(best_s);
  *per = best_pp;
}

// ------------------------------------------------------------------ stride-2 dgrad parity classes
// The data gradient of a stride-2 conv is a stride-1 conv of dy zero-inserted to the input grid
// (zero_insert_kernel below) with the flipped weights: 3/4 of its B rows are zeros.  Split by the
// parity (a, b) of the output pixel, each class is a dense stride-1 conv of dy itself with the
// flipped taps kh' = (pad_d - a) mod 2, + 2, ... (kw' likewise), embedded in a KSC x KSC kernel
// (zero weights where a class has fewer taps in one dimension), written to every other pixel of
// every other row (drnmi_conv_args.y_sr).  Products with the zero rows were exact zeros: the four
// class launches are bit-identical to the zero-inserted conv.  This gathers one class's weight
// planes from the packed dgrad planes ([3][rows][k_pad], k = tap' * kst + co).
__global__ void __launch_bounds__(kThreads)
dgrad_class_planes_kernel(const uint4* __restrict__ in, int rows, int k_pad, int kst, int ks, int kh0, int nh, int kw0,
                          int nw, int ksc, uint4* __restrict__ out, int k_pad_c) {
  const int c8 = kst / 8;
  const int64_t per_plane = static_cast<int64_t>(rows) * ksc * ksc * c8;
  const int64_t total = 3 * per_plane;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int pl = static_cast<int>(i / per_plane);
    int64_t j = i - pl * per_plane;
    const int c = static_cast<int>(j % c8);
    j /= c8;
    const int tc = static_cast<int>(j % (ksc * ksc));
    const int r = static_cast<int>(j / (ksc * ksc));
    const int khc = tc / ksc, kwc = tc - (tc / ksc) * ksc;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (khc < nh && kwc < nw) {
      const int tap = (kh0 + 2 * khc) * ks + (kw0 + 2 * kwc);
      v = in[((static_cast<int64_t>(pl) * rows + r) * k_pad + tap * kst) / 8 + c];
    }
    out[((static_cast<int64_t>(pl) * rows + r) * k_pad_c + tc * kst) / 8 + c] = v;
  }
}

// ------------------------------------------------------------------ zero insert (stride-s dgrad)
__global__ void __launch_bounds__(kThreads)
zero_insert_kernel(const float* __restrict__ dy, int n, int ho, int wo, int c4, int s, int hu, int wu,
                   float* __restrict__ out) {
  const int64_t total = static_cast<int64_t>(n) * hu * wu * c4;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int cv = static_cast<int>(i % c4);
    const int64_t pix = i / c4;
    const int x = static_cast<int>(pix % wu);
    const int y = static_cast<int>((pix / wu) % hu);
    const int b = static_cast<int>(pix / (static_cast<int64_t>(wu) * hu));
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y % s == 0 && x % s == 0 && y / s < ho && x / s < wo)
      v = reinterpret_cast<const float4*>(dy)[((static_cast<int64_t>(b) * ho + y / s) * wo + x / s) * c4 + cv];
    reinterpret_cast<float4*>(out)[i] = v;
  }
}

// ------------------------------------------------------------------ head backward
// du[n][c][p] = scale * (g[n][c][p] - exp(lp[n][c][p]) * sum_c' g[n][c'][p])  (LogSoftmax bwd).
// NC > 0: the class count at compile time (19, the seg head), the pixel's values held in registers
// (one read of g instead of two); NC = 0: any c.  Same operations in the same order either way.
template <int NC>
__global__ void __launch_bounds__(kThreads)
lsm_bwd_kernel(const float* __restrict__ g, const float* __restrict__ lp, int nimg, int c, int64_t hw, float scale,
               float* __restrict__ du) {
  const int64_t total = static_cast<int64_t>(nimg) * hw;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t b = i / hw, p = i - b * hw;
    const int64_t base = b * c * hw + p;
    if constexpr (NC > 0) {
      float gv[NC], lv[NC];
#pragma unroll
      for (int k = 0; k < NC; ++k) {
        gv[k] = g[base + k * hw];
        lv[k] = lp[base + k * hw];
      }
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < NC; ++k) s += gv[k];
#pragma unroll
      for (int k = 0; k < NC; ++k) du[base + k * hw] = scale * (gv[k] - expf(lv[k]) * s);
    } else {
      float s = 0.f;
      for (int k = 0; k < c; ++k) s += g[base + k * hw];
      for (int k = 0; k < c; ++k) {
        const int64_t o = base + k * hw;
        du[o] = scale * (g[o] - expf(lp[o]) * s);
      }
    }
  }
}

// dlogits[n][c][i][j] = sum_{ky,kx} W[ky][kx] * du[n][c][8i-4+ky][8j-4+kx] (+ gscale * g_logits); the
// transpose of ConvTranspose2d(k16, s8, p4) (lmodels/drnseg.py:285-293).  du == NULL: logits-only
// gradient (no log-prob term).  A workgroup owns UBI x UBJ outputs of one plane and stages the
// (8 UBI + 8) x (8 UBJ + 8) du window they read into LDS once (each du value is read by four
// outputs' 16 x 16 windows); every output then sums its 256 products in the same ky-major order,
// skipping the same out-of-image taps: the same result bits as the per-output global gather.
constexpr int kUbI = 4, kUbJ = 32, kUbThreads = kUbI * kUbJ;   // outputs per workgroup, one per thread
constexpr int kUbRows = 8 * kUbI + 8, kUbCols = 8 * kUbJ + 8;
static_assert(kUbCols % 8 == 0, "16-B staging pieces stay inside one skew group");
// column c of a tile row at c + c / 8: output windows start 8 columns apart, so a wave's 32 lanes
// of one row read 9 apart -- distinct banks
constexpr int kUbPitch = kUbCols + kUbCols / 8 + 1;
__global__ void __launch_bounds__(kUbThreads)
up8_bwd_kernel(const float* __restrict__ du, const float* __restrict__ upw, const float* __restrict__ glog,
               float gscale, int nc, int h, int w, float* __restrict__ dlog) {
  __shared__ float wk[256];
  __shared__ float tile[kUbRows * kUbPitch];
  for (int e = threadIdx.x; e < 256; e += kUbThreads) wk[e] = upw[e];
  const int H = 8 * h, W = 8 * w;
  const int64_t plane = blockIdx.z;
  const int i0 = blockIdx.y * kUbI, j0 = blockIdx.x * kUbJ;
  const int y0 = 8 * i0 - 4, x0 = 8 * j0 - 4;        // du window origin
  if (du != nullptr) {
    // 16-B pieces (W = 8 w and x0 = 8 j0 - 4 are multiples of 4: a piece is wholly inside or outside
    // the image), all of a thread's pieces in flight before their LDS writes
    const float* src = du + plane * H * W;
    constexpr int kP4 = kUbCols / 4, kN4 = kUbRows * kP4;
    constexpr int kB = (kN4 + kUbThreads - 1) / kUbThreads;
    float4 v[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int e = threadIdx.x + u * kUbThreads;
      const int r = e / kP4, x = x0 + 4 * (e - r * kP4), y = y0 + r;
      v[u] = (e < kN4 && static_cast<unsigned>(y) < static_cast<unsigned>(H) &&
              static_cast<unsigned>(x) < static_cast<unsigned>(W))
                 ? *reinterpret_cast<const float4*>(src + static_cast<int64_t>(y) * W + x)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int e = threadIdx.x + u * kUbThreads;
      if (e < kN4) {
        const int r = e / kP4, cc = 4 * (e - r * kP4);
        float* t = tile + r * kUbPitch + cc + (cc >> 3);   // the 4 columns share one 8-group
        t[0] = v[u].x;
        t[1] = v[u].y;
        t[2] = v[u].z;
        t[3] = v[u].w;
      }
    }
  }
  __syncthreads();
  const int ii = i0 + threadIdx.x / kUbJ, j = j0 + threadIdx.x % kUbJ;
  if (ii >= h || j >= w) return;
  const float* t0 = tile + 8 * (threadIdx.x / kUbJ) * kUbPitch + 9 * (threadIdx.x % kUbJ);   // (8 ti, 8 tj)
  float s = 0.f;
  for (int ky = 0; ky < 16 && du != nullptr; ++ky) {
    const int y = 8 * ii - 4 + ky;
    if (static_cast<unsigned>(y) >= static_cast<unsigned>(H)) continue;
    const float* row = t0 + ky * kUbPitch;
#pragma unroll
    for (int kx = 0; kx < 16; ++kx) {
      const int x = 8 * j - 4 + kx;
      if (static_cast<unsigned>(x) < static_cast<unsigned>(W)) s += wk[ky * 16 + kx] * row[kx + (kx >> 3)];
    }
  }
  const int64_t i = (plane * h + ii) * w + j;
  if (glog != nullptr) s += gscale * glog[i];   // the logits output's gradient, DDP-averaged like du
  dlog[i] = s;
}

// Transpose of nn.UpsamplingBilinear2d(scale_factor=8) (align_corners=True, lmodels/drnseg.py:
// 285-287): dlogits[i][j] = sum_{oy,ox} wy(oy, i) * wx(ox, j) * du[oy][ox] (+ gscale * g_logits),
// gathered (no atomics, fixed order).  Output row oy touches input rows i0(oy) and i1(oy) with
// i0 non-decreasing in oy, so input row i gathers from the oy window whose i0 is i-1 or i; the
// window is found with the forward's own index arithmetic.
__device__ __forceinline__ void bil_ac(int dst, int in, int out, int& i0, int& i1, float& l0, float& l1) {
  const float scale = out > 1 ? static_cast<float>(in - 1) / static_cast<float>(out - 1) : 0.f;
  const float src = scale * static_cast<float>(dst);
  i0 = static_cast<int>(floorf(src));
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = fminf(fmaxf(src - static_cast<float>(i0), 0.f), 1.f);
  l0 = 1.f - l1;
}

__device__ __forceinline__ float bil_weight(int o, int i, int in, int out) {
  int i0, i1;
  float l0, l1;
  bil_ac(o, in, out, i0, i1, l0, l1);
  return (i0 == i ? l0 : 0.f) + (i1 == i ? l1 : 0.f);
}

__global__ void __launch_bounds__(kThreads)
up8_bilinear_bwd_kernel(const float* __restrict__ du, const float* __restrict__ glog, float gscale, int nc, int h,
                        int w, float* __restrict__ dlog) {
  const int H = 8 * h, W = 8 * w;
  const int64_t total = static_cast<int64_t>(nc) * h * w;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int j = static_cast<int>(i % w);
    const int ii = static_cast<int>((i / w) % h);
    const int64_t plane = i / (static_cast<int64_t>(w) * h);
    float s = 0.f;
    if (du != nullptr) {
      const float* src = du + plane * H * W;
      // candidate windows: o with i0(o) in {i-1, i}, i.e. o*(in-1)/(out-1) in [i-1, i+1), +-2 for
      // rounding; bil_weight() then applies the forward's exact index test
      const float ry = h > 1 ? static_cast<float>(H - 1) / static_cast<float>(h - 1) : static_cast<float>(H);
      const float rx = w > 1 ? static_cast<float>(W - 1) / static_cast<float>(w - 1) : static_cast<float>(W);
      const int oy_lo = max(0, static_cast<int>(floorf((ii - 1) * ry)) - 2);
      const int oy_hi = min(H - 1, static_cast<int>(ceilf((ii + 1) * ry)) + 2);
      const int ox_lo = max(0, static_cast<int>(floorf((j - 1) * rx)) - 2);
      const int ox_hi = min(W - 1, static_cast<int>(ceilf((j + 1) * rx)) + 2);
      for (int oy = oy_lo; oy <= oy_hi; ++oy) {
        const float wy = bil_weight(oy, ii, h, H);
        if (wy == 0.f) continue;
        const float* row = src + static_cast<int64_t>(oy) * W;
        float r = 0.f;
        for (int ox = ox_lo; ox <= ox_hi; ++ox) {
          const float wx = bil_weight(ox, j, w, W);
          if (wx != 0.f) r += wx * row[ox];
        }
        s += wy * r;
      }
    }
    if (glog != nullptr) s += gscale * glog[i];
    dlog[i] = s;
  }
}

// ------------------------------------------------------------------ cross entropy
// per pixel: lse(lp) - lp[t] over t != ignore (CrossEntropyLoss applied to log-probs,
// semantic_seg.py:817 + :197-198); block partials (sum, count) in fp64, fixed order.
constexpr int kCeBlocks = 512;

// one pixel's lse(lp) - lp[t]: NC > 0 holds the NC values in registers (one read instead of three),
// NC = 0 walks any c; same operations in the same order
template <int NC>
__device__ __forceinline__ float ce_pixel(const float* v, int c, int64_t hw, int64_t t) {
  if constexpr (NC > 0) {
    float x[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) x[k] = v[k * hw];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < NC; ++k) mx = fmaxf(mx, x[k]);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) se += expf(x[k] - mx);
    const float lse = mx + logf(se);
    float xt = x[0];
#pragma unroll
    for (int k = 1; k < NC; ++k) xt = k == t ? x[k] : xt;
    return lse - xt;
  } else {
    float mx = -INFINITY;
    for (int k = 0; k < c; ++k) mx = fmaxf(mx, v[k * hw]);
    float se = 0.f;
    for (int k = 0; k < c; ++k) se += expf(v[k * hw] - mx);
    const float lse = mx + logf(se);
    return lse - v[t * hw];
  }
}

template <int NC>
__global__ void __launch_bounds__(kThreads)
ce_fwd_kernel(const float* __restrict__ lp, const int64_t* __restrict__ tgt, int nimg, int c, int64_t hw,
              int64_t ignore, double* __restrict__ ws) {
  const int64_t total = static_cast<int64_t>(nimg) * hw;
  double s = 0, cnt = 0, bad = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t t = tgt[i];
    if (t == ignore) continue;
    if (t < 0 || t >= c) { bad += 1; continue; }
    const int64_t b = i / hw, p = i - b * hw;
    s += static_cast<double>(ce_pixel<NC>(lp + b * c * hw + p, c, hw, t));
    cnt += 1;
  }
  __shared__ double sh[3][kThreads];
  sh[0][threadIdx.x] = s;
  sh[1][threadIdx.x] = cnt;
  sh[2][threadIdx.x] = bad;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + o];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + o];
      sh[2][threadIdx.x] += sh[2][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    ws[blockIdx.x] = sh[0][0];
    ws[kCeBlocks + blockIdx.x] = sh[1][0];
    ws[2 * kCeBlocks + blockIdx.x] = sh[2][0];
  }
}

// the block partials summed in block order by one thread, from LDS (the 64 threads stage them:
// one dependent fp64 add per partial instead of a global load each)
__global__ void __launch_bounds__(64) ce_final_kernel(const double* __restrict__ ws, int blocks, float* __restrict__ loss,
                                                      float* __restrict__ count) {
  __shared__ double sh[3 * kCeBlocks];
  for (int e = threadIdx.x; e < 3 * kCeBlocks; e += 64) sh[e] = ws[e];
  __syncthreads();
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0, cnt = 0, bad = 0;
  for (int b = 0; b < blocks; ++b) {
    s += sh[b];
    cnt += sh[kCeBlocks + b];
    bad += sh[2 * kCeBlocks + b];
  }
  // an out-of-range target is an error in the reference (device assert); surface it as NaN
  loss[0] = bad > 0 ? __builtin_nanf("") : static_cast<float>(s / cnt);
  count[0] = static_cast<float>(cnt);
}

// four consecutive pixels per thread as 16-B pieces (NC > 0, hw % 4 == 0); per-pixel arithmetic
// as ce_bwd_kernel
template <int NC>
__global__ void __launch_bounds__(kThreads)
ce_bwd_v4_kernel(const float* __restrict__ lp, const int64_t* __restrict__ tgt, int nimg, int c, int64_t hw,
                 int64_t ignore, const float* __restrict__ dloss, const float* __restrict__ count,
                 float* __restrict__ glp) {
  const float sc = dloss[0] / count[0];
  const int64_t total4 = static_cast<int64_t>(nimg) * hw / 4;
  const int64_t hw4 = hw / 4;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total4;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t b = i / hw4, p4 = i - b * hw4;
    const int64_t base4 = b * c * hw4 + p4;
    const float4* v4 = reinterpret_cast<const float4*>(lp) + base4;
    float x[4][NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const float4 a = v4[k * hw4];
      x[0][k] = a.x;
      x[1][k] = a.y;
      x[2][k] = a.z;
      x[3][k] = a.w;
    }
    float lse[4];
    int64_t tt[4];
    bool live[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tt[e] = tgt[4 * i + e];
      live[e] = !(tt[e] == ignore || tt[e] < 0 || tt[e] >= c);
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < NC; ++k) mx = fmaxf(mx, x[e][k]);
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < NC; ++k) se += expf(x[e][k] - mx);
      lse[e] = mx + logf(se);
    }
    float4* o4 = reinterpret_cast<float4*>(glp) + base4;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = live[e] ? sc * (expf(x[e][k] - lse[e]) - (k == tt[e] ? 1.f : 0.f)) : 0.f;
      o4[k * hw4] = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

template <int NC>
__global__ void __launch_bounds__(kThreads)
ce_bwd_kernel(const float* __restrict__ lp, const int64_t* __restrict__ tgt, int nimg, int c, int64_t hw,
              int64_t ignore, const float* __restrict__ dloss, const float* __restrict__ count,
              float* __restrict__ glp) {
  const float sc = dloss[0] / count[0];
  const int64_t total = static_cast<int64_t>(nimg) * hw;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t t = tgt[i];
    const int64_t b = i / hw, p = i - b * hw;
    const float* v = lp + b * c * hw + p;
    float* o = glp + b * c * hw + p;
    if (t == ignore || t < 0 || t >= c) {
      for (int k = 0; k < c; ++k) o[k * hw] = 0.f;
      continue;
    }
    if constexpr (NC > 0) {
      float x[NC];
#pragma unroll
      for (int k = 0; k < NC; ++k) x[k] = v[k * hw];
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < NC; ++k) mx = fmaxf(mx, x[k]);
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < NC; ++k) se += expf(x[k] - mx);
      const float lse = mx + logf(se);
#pragma unroll
      for (int k = 0; k < NC; ++k) o[k * hw] = sc * (expf(x[k] - lse) - (k == t ? 1.f : 0.f));
    } else {
      float mx = -INFINITY;
      for (int k = 0; k < c; ++k) mx = fmaxf(mx, v[k * hw]);
      float se = 0.f;
      for (int k = 0; k < c; ++k) se += expf(v[k * hw] - mx);
      const float lse = mx + logf(se);
      for (int k = 0; k < c; ++k) o[k * hw] = sc * (expf(v[k * hw] - lse) - (k == t ? 1.f : 0.f));
    }
  }
}

// ------------------------------------------------------------------ SGD (+ mask)
constexpr int kSgdBatch = 48;
struct SgdBatch {
  float* w[kSgdBatch];
  const float* g[kSgdBatch];
  float* buf[kSgdBatch];
  const uint32_t* mask[kSgdBatch];
  int64_t numel[kSgdBatch];
  int first[kSgdBatch];
};

// torch.optim.SGD (dampening d, nesterov off/on): d_p = g + wd * w;
// buf = first ? d_p : m * buf + (1 - d) * d_p;  d_p = nesterov ? d_p + m * buf : buf;
// w = w - lr * d_p; then w *= mask (Pruner.apply_masks fused, pruners/Pruner.py:17-20).
__global__ void __launch_bounds__(kThreads)
sgd_kernel(const SgdBatch b, float lr, float mom, float damp, float wd, int nesterov) {
  const int t = blockIdx.y;
  float* __restrict__ w = b.w[t];
  const float* __restrict__ g = b.g[t];
  float* __restrict__ buf = b.buf[t];
  const uint32_t* __restrict__ mk = b.mask[t];
  const int64_t n = b.numel[t];
  const int first = b.first[t];
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float d = g[i];
    const float wv = w[i];
    if (wd != 0.f) d = d + wd * wv;
    if (mom != 0.f) {
      float bv;
      if (first) bv = d;
      else bv = mom * buf[i] + (1.f - damp) * d;
      buf[i] = bv;
      d = nesterov ? d + mom * bv : bv;
    }
    float nw = wv - lr * d;
    if (mk != nullptr) nw *= static_cast<float>((mk[i >> 5] >> (i & 31)) & 1u);
    w[i] = nw;
  }
}

}  // namespace
}  // namespace drnmi

using namespace drnmi;

// ================================================================== C-ABI
extern "C" int drnmi_pack_conv_weight(const float* w, int32_t cout, int32_t cin, int32_t ks, int32_t kin_stride,
                                      int32_t rows_pad, int32_t k_pad, int32_t mode, const float* row_scale,
                                      int32_t out_dtype, void* out, void* stream) {
  if (w == nullptr || out == nullptr || cout <= 0 || cin <= 0 || ks <= 0 || kin_stride <= 0 || k_pad <= 0)
    return DRNMI_EINVAL;
  if (mode != 0 && mode != 1) return DRNMI_EINVAL;
  if (k_pad < ks * ks * kin_stride) return DRNMI_EINVAL;
  if (mode == 0 && (rows_pad < cout || kin_stride < cin)) return DRNMI_EINVAL;
  if (mode == 1 && (rows_pad < cin || kin_stride < cout || row_scale != nullptr)) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = static_cast<int64_t>(rows_pad) * k_pad;
  if (out_dtype == DRNMI_F32)
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(grid_of(total)), dim3(kThreads), 0, s, w, cout, cin, ks,
                       kin_stride, rows_pad, k_pad, mode, row_scale, reinterpret_cast<float*>(out));
  else if (out_dtype == DRNMI_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<bf16_t>, dim3(grid_of(total)), dim3(kThreads), 0, s, w, cout, cin, ks,
                       kin_stride, rows_pad, k_pad, mode, row_scale, reinterpret_cast<bf16_t*>(out));
  else
    return DRNMI_EINVAL;
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_pack_table_check(const int64_t* t, int32_t n, int64_t* total_out) {
  if (t == nullptr || n <= 0 || n > kPackMaxEntries) return DRNMI_EINVAL;
  int64_t total = 0;
  for (int e = 0; e < n; ++e) {
    const int64_t* q = t + static_cast<int64_t>(e) * DRNMI_PACK_ENTRY_WORDS;
    const int64_t cout = q[3], cin = q[4], ks = q[5], kst = q[6], rows = q[7], kp = q[8], mode = q[9];
    if (q[0] == 0 || q[1] == 0 || cout <= 0 || cin <= 0 || ks <= 0 || ks > 7 || kst <= 0 || rows <= 0 || kp <= 0)
      return DRNMI_EINVAL;
    if ((mode != 0 && mode != 1) || kp < ks * ks * kst || kp >= (int64_t(1) << 31) || rows >= (int64_t(1) << 31)) return DRNMI_EINVAL;
    if (kst % 4 != 0 || kp % 4 != 0 || ((q[1] | q[2]) & 15) != 0) return DRNMI_EINVAL;   // 4-column stores
    if (mode == 0 && (rows < cout || kst < cin)) return DRNMI_EINVAL;
    if (mode == 1 && (rows < cin || kst < cout)) return DRNMI_EINVAL;
    if (q[10] != total || q[11] != 0) return DRNMI_EINVAL;
    total += rows * kp;
  }
  if (total_out != nullptr) *total_out = total;
  return 0;
}

extern "C" int drnmi_pack_conv_weights_batched(const int64_t* table, int32_t n, int64_t total, void* stream) {
  if (table == nullptr || n <= 0 || n > kPackMaxEntries || total <= 0) return DRNMI_EINVAL;
  // grid-stride over the tiles (their count is known on the device only): 8 workgroups per CU
  hipLaunchKernelGGL(pack_batched_kernel, dim3(2048), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream), table, n);
  return static_cast<int>(hipGetLastError());
}

static bool pow2_ge4(int c) { return c >= 4 && (c & (c - 1)) == 0; }

extern "C" int64_t drnmi_reduce_workspace_bytes(int64_t rows, int32_t channels) {
  if (rows <= 0 || !pow2_ge4(channels)) return -1;
  // partials (2 x G x C doubles) + 3 x C float coefficients
  return static_cast<int64_t>(2) * red_splits(rows, channels) * channels * 8 + 3LL * channels * 4 + 256;
}

extern "C" int drnmi_bn_stats_f32(const float* y, int64_t rows, int32_t C, float eps, float momentum,
                                  float* mean, float* invstd, float* running_mean, float* running_var,
                                  int64_t* num_batches_tracked, void* ws, void* stream) {
  if (y == nullptr || mean == nullptr || invstd == nullptr || ws == nullptr || rows <= 0 || !pow2_ge4(C))
    return DRNMI_EINVAL;
  if ((running_mean == nullptr) != (running_var == nullptr)) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  RedArgs r{};
  r.a = y;
  r.rows = rows;
  r.C = C;
  r.ws = reinterpret_cast<double*>(ws);
  hipError_t e = launch_colred<RED_STATS>(r, s);
  if (e != hipSuccess) return static_cast<int>(e);
  hipLaunchKernelGGL(bn_stats_final_kernel, dim3(fin_grid(C)), dim3(kThreads), 0, s, r.ws, r.G, C, rows, eps,
                     momentum, mean, invstd, running_mean, running_var, num_batches_tracked);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_dgrad_s2_class_planes(const void* planes, int32_t rows, int32_t k_pad, int32_t kst, int32_t ks,
                                           int32_t pad_d, int32_t a, int32_t b, int32_t ksc, void* out, int32_t k_pad_c,
                                           void* stream) {
  if (planes == nullptr || out == nullptr || rows <= 0 || ks <= 0 || ksc <= 0 || kst <= 0 || kst % 8 != 0 ||
      k_pad % 8 != 0 || k_pad < ks * ks * kst || k_pad_c != ksc * ksc * kst || (a != 0 && a != 1) || (b != 0 && b != 1) ||
      ((reinterpret_cast<uintptr_t>(planes) | reinterpret_cast<uintptr_t>(out)) & 15))
    return DRNMI_EINVAL;
  const int kh0 = ((pad_d - a) % 2 + 2) % 2, kw0 = ((pad_d - b) % 2 + 2) % 2;
  const int nh = kh0 < ks ? (ks - kh0 + 1) / 2 : 0, nw = kw0 < ks ? (ks - kw0 + 1) / 2 : 0;
  if (nh > ksc || nw > ksc) return DRNMI_EINVAL;
  const int64_t total = 3LL * rows * ksc * ksc * (kst / 8);
  hipLaunchKernelGGL(dgrad_class_planes_kernel, dim3(grid_of(total)), dim3(kThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const uint4*>(planes), rows, k_pad, kst,
                     ks, kh0, nh, kw0, nw, ksc, reinterpret_cast<uint4*>(out), k_pad_c);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_bn_stats_partials_f32(const double* partials, int64_t G, int64_t rows, int32_t C, float eps,
                                           float momentum, float* mean, float* invstd, float* running_mean,
                                           float* running_var, int64_t* num_batches_tracked, void* stream) {
  if (partials == nullptr || mean == nullptr || invstd == nullptr || G <= 0 || G >= (int64_t(1) << 31) || rows <= 0 ||
      !pow2_ge4(C))
    return DRNMI_EINVAL;
  if ((running_mean == nullptr) != (running_var == nullptr)) return DRNMI_EINVAL;
  hipLaunchKernelGGL(bn_stats_final_kernel, dim3(fin_grid(C)), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                     partials, static_cast<int>(G), C, rows, eps, momentum, mean, invstd, running_mean, running_var,
                     num_batches_tracked);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_bn_act_f32(const float* y, const float* mean, const float* invstd, const float* gamma,
                                const float* beta, const float* res, int32_t relu, int64_t rows, int32_t C,
                                float* z, void* stream) {
  if (y == nullptr || mean == nullptr || invstd == nullptr || z == nullptr || rows <= 0 || !pow2_ge4(C))
    return DRNMI_EINVAL;
  // the per-channel vectors are read as 16-B pieces
  if ((reinterpret_cast<uintptr_t>(mean) | reinterpret_cast<uintptr_t>(invstd) | reinterpret_cast<uintptr_t>(gamma) |
       reinterpret_cast<uintptr_t>(beta)) & 15)
    return DRNMI_EINVAL;
  const int64_t n4 = rows * C / 4;
  hipLaunchKernelGGL(bn_act_kernel, dim3(bn_ew_grid(n4, C)), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                     y, mean, invstd, gamma, beta, res, relu, n4, C, z);
  return static_cast<int>(hipGetLastError());
}

static int bn_bwd_launch(const float* dz, const float* z, const float* y, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, int32_t relu, int64_t rows, int32_t C, float* dy,
                         float* dres, int32_t dres_accumulate, float* dgamma, float* dbeta, int32_t grad_accumulate,
                         void* ws, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  RedArgs r{};
  r.a = dz;
  r.z = z;
  r.y = y;
  r.rows = rows;
  r.C = C;
  r.relu = relu;
  r.ws = reinterpret_cast<double*>(ws);
  r.mean = mean;
  r.invstd = invstd;
  r.gamma = gamma;
  r.beta = beta;
  hipError_t e = launch_colred<RED_BNBWD>(r, s);
  if (e != hipSuccess) return static_cast<int>(e);
  float* coef = reinterpret_cast<float*>(r.ws + static_cast<int64_t>(2) * r.G * C);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(fin_grid(C)), dim3(kThreads), 0, s, r.ws, r.G, C, rows, mean, invstd,
                     gamma, dgamma, dbeta, grad_accumulate, coef);
  e = hipGetLastError();
  if (e != hipSuccess) return static_cast<int>(e);
  const int64_t n4 = rows * C / 4;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(bn_ew_grid(n4, C)), dim3(kThreads), 0, s, dz, z, y, mean, coef, relu, n4,
                     C, dy, dres, dres_accumulate, invstd, gamma, beta);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_bn_act_bwd_f32(const float* dz, const float* z, const float* y, const float* mean,
                                    const float* invstd, const float* gamma, int32_t relu, int64_t rows, int32_t C,
                                    float* dy, float* dres, int32_t dres_accumulate, float* dgamma, float* dbeta,
                                    int32_t grad_accumulate, void* ws, void* stream) {
  if (dz == nullptr || y == nullptr || mean == nullptr || invstd == nullptr || dy == nullptr || ws == nullptr ||
      rows <= 0 || !pow2_ge4(C) || (relu && z == nullptr))
    return DRNMI_EINVAL;
  if (reinterpret_cast<uintptr_t>(mean) & 15) return DRNMI_EINVAL;   // read as 16-B pieces
  return bn_bwd_launch(dz, z, y, mean, invstd, gamma, nullptr, relu, rows, C, dy, dres, dres_accumulate, dgamma, dbeta,
                       grad_accumulate, ws, stream);
}

extern "C" int drnmi_bn_relu_bwd_y_f32(const float* dz, const float* y, const float* mean, const float* invstd,
                                       const float* gamma, const float* beta, int64_t rows, int32_t C, float* dy,
                                       float* dgamma, float* dbeta, int32_t grad_accumulate, void* ws, void* stream) {
  if (dz == nullptr || y == nullptr || mean == nullptr || invstd == nullptr || dy == nullptr || ws == nullptr ||
      rows <= 0 || !pow2_ge4(C))
    return DRNMI_EINVAL;
  if ((reinterpret_cast<uintptr_t>(mean) | reinterpret_cast<uintptr_t>(invstd) | reinterpret_cast<uintptr_t>(gamma) |
       reinterpret_cast<uintptr_t>(beta)) & 15)
    return DRNMI_EINVAL;
  return bn_bwd_launch(dz, nullptr, y, mean, invstd, gamma, beta, 1, rows, C, dy, nullptr, 0, dgamma, dbeta,
                       grad_accumulate, ws, stream);
}

extern "C" int drnmi_channel_sum_f32(const float* x, int64_t rows, int32_t C, int32_t cvalid, float* out,
                                     int32_t accumulate, void* ws, void* stream) {
  if (x == nullptr || out == nullptr || ws == nullptr || rows <= 0 || !pow2_ge4(C) || cvalid <= 0 || cvalid > C)
    return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  RedArgs r{};
  r.a = x;
  r.rows = rows;
  r.C = C;
  r.ws = reinterpret_cast<double*>(ws);
  hipError_t e = launch_colred<RED_SUM>(r, s);
  if (e != hipSuccess) return static_cast<int>(e);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(grid_of(cvalid)), dim3(kThreads), 0, s, r.ws, r.G, C, cvalid, out,
                     accumulate);
  return static_cast<int>(hipGetLastError());
}

static int wgrad_check(const drnmi_wgrad_args* a) {
  if (a == nullptr) return DRNMI_EINVAL;
  if (a->n <= 0 || a->h <= 0 || a->w <= 0 || a->ho <= 0 || a->wo <= 0 || a->cout <= 0 || a->cin <= 0) return DRNMI_EINVAL;
  if (a->cin_stride < 8 || (a->cin_stride & (a->cin_stride - 1)) != 0 || a->cin > a->cin_stride) return DRNMI_EINVAL;
  if (a->dy_stride < a->cout || a->ks <= 0 || a->stride <= 0 || a->dil <= 0 || a->pad < 0) return DRNMI_EINVAL;
  if (a->ho != (a->h + 2 * a->pad - a->dil * (a->ks - 1) - 1) / a->stride + 1 ||
      a->wo != (a->w + 2 * a->pad - a->dil * (a->ks - 1) - 1) / a->stride + 1)
    return DRNMI_EINVAL;
  // pixel indices are int32 inside the tiles (wgrad_kernel / wgrad_x6_*: m_cur, m / hw)
  if (static_cast<int64_t>(a->n) * a->ho * a->wo >= (int64_t(1) << 31)) return DRNMI_EINVAL;
  return DRNMI_OK;
}

// the partials [splits][cout][K] fp32, then (fp32x, 128-tile geometries) the dy planes [3][Cp][Mp]
static int64_t wgrad_partials_bytes(const drnmi_wgrad_args& a, int splits) {
  return (static_cast<int64_t>(splits) * a.cout * a.ks * a.ks * a.cin_stride * 4 + 255) / 256 * 256;
}
// the dy split pass costs ~10 B of HBM per dy element against 2 K flops per element of the tile:
// it pays where K >= 1024 (layer7.0: 3.78 -> 2.72 ms; a 1x1 256 -> 1024 wgrad: 128 -> 234 us)
static bool wgrad_pre_ok(const drnmi_wgrad_args& a) {
  return wgrad_big_ok(a) && a.ks * a.ks * a.cin_stride >= 1024;
}
static int64_t wgrad_pre_bytes(const drnmi_wgrad_args& a) {
  if (!wgrad_pre_ok(a)) return 0;
  const int64_t M = static_cast<int64_t>(a.n) * a.ho * a.wo;
  const int64_t Mp = (M + kWM - 1) / kWM * kWM;
  const int64_t Cp = (a.cout + kPreRows - 1) / kPreRows * kPreRows;
  return 3 * Cp * Mp * 2;
}

// the exact-f32 kernel's own partials (the f32x3 query below also holds the split-bf16 plan and
// its dy planes)
extern "C" int64_t drnmi_conv_wgrad_f32_workspace_bytes(const drnmi_wgrad_args* a) {
  if (wgrad_check(a) != DRNMI_OK) return -1;
  int splits;
  int64_t per;
  wgrad_plan(*a, false, &splits, &per);
  return wgrad_partials_bytes(*a, splits);
}

extern "C" int64_t drnmi_conv_wgrad_workspace_bytes(const drnmi_wgrad_args* a) {
  if (wgrad_check(a) != DRNMI_OK) return -1;
  // room for either kernel (f32 or f32x3): enough for both plans
  int splits;
  int64_t per;
  wgrad_plan(*a, false, &splits, &per);
  int64_t pre = 0;
  if (wgrad_big_ok(*a)) {
    int s2;
    wgrad_plan(*a, true, &s2, &per);
    if (s2 > splits) splits = s2;
    pre = wgrad_pre_bytes(*a);
  }
  if (wgrad_direct_ok(*a) && wgrad_direct_splits(*a) > splits) splits = wgrad_direct_splits(*a);
  return wgrad_partials_bytes(*a, splits) + pre;
}

static int wgrad_launch(const drnmi_wgrad_args* a, bool x6, void* stream) {
  const int rc = wgrad_check(a);
  if (rc != DRNMI_OK) return rc;
  if (a->dy == nullptr || a->x == nullptr || a->dw == nullptr || a->ws == nullptr) return DRNMI_EINVAL;
  if (a->ws_bytes < (x6 ? drnmi_conv_wgrad_workspace_bytes(a) : drnmi_conv_wgrad_f32_workspace_bytes(a)))
    return DRNMI_EINVAL;
  // 16-B loads of dy / x; the dy bf16 planes in ws are LDS-DMA'd and stored as 16-B pieces
  if ((reinterpret_cast<uintptr_t>(a->dy) | reinterpret_cast<uintptr_t>(a->x) | reinterpret_cast<uintptr_t>(a->ws)) & 15)
    return DRNMI_EINVAL;
  if (a->dy_stride % 4 != 0) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  WgradP p{};
  p.dy = a->dy;
  p.x = a->x;
  p.ws = reinterpret_cast<float*>(a->ws);
  p.dys = a->dy_stride;
  p.cout = a->cout;
  p.n = a->n; p.h = a->h; p.w = a->w; p.cs = a->cin_stride;
  p.ho = a->ho; p.wo = a->wo; p.ks = a->ks; p.stride = a->stride; p.pad = a->pad; p.dil = a->dil;
  p.K = a->ks * a->ks * a->cin_stride;
  p.M = static_cast<int64_t>(a->n) * a->ho * a->wo;
  const bool big = x6 && wgrad_big_ok(*a);
  int splits;
  wgrad_plan(*a, big, &splits, &p.pix_per_split);
  const dim3 grid((p.K + kWT - 1) / kWT, (a->cout + kWT - 1) / kWT, splits);
  if (x6 && !big && wgrad_direct_ok(*a)) {
    splits = wgrad_direct_splits(*a);
    const dim3 gd(static_cast<unsigned>(wgrad_direct_tiles(*a)), static_cast<unsigned>(splits / 4));
    if (a->cout <= 16) hipLaunchKernelGGL(wgrad_x6_direct_kernel<1>, gd, dim3(kThreads), 0, s, p, a->cin);
    else hipLaunchKernelGGL(wgrad_x6_direct_kernel<2>, gd, dim3(kThreads), 0, s, p, a->cin);
  } else if (big && wgrad_pre_ok(*a)) {
    WgradPreP q{};
    q.p = p;
    q.Mp = (p.M + kWM - 1) / kWM * kWM;
    q.Cp = (a->cout + kPreRows - 1) / kPreRows * kPreRows;
    int full_splits;
    int64_t per;
    wgrad_plan(*a, false, &full_splits, &per);
    int s2;
    wgrad_plan(*a, true, &s2, &per);
    if (s2 > full_splits) full_splits = s2;
    bf16_t* dyt = reinterpret_cast<bf16_t*>(reinterpret_cast<char*>(a->ws) + wgrad_partials_bytes(*a, full_splits));
    q.dyt = dyt;
    const int64_t blocks = (q.Mp / 32) * (q.Cp / 64);
    hipLaunchKernelGGL(wgrad_dy_split_kernel, dim3(static_cast<unsigned>(blocks < 8192 ? blocks : 8192)), dim3(kThreads),
                       0, s, a->dy, a->dy_stride, a->cout, p.M, q.Mp, q.Cp, dyt);
    const dim3 g2((p.K + kWT2 - 1) / kWT2, (a->cout + kWT2 - 1) / kWT2, splits);
    hipLaunchKernelGGL(wgrad_x6_pre_kernel, g2, dim3(kThreads), 0, s, q);
  } else if (big) {
    const dim3 g2((p.K + kWT2 - 1) / kWT2, (a->cout + kWT2 - 1) / kWT2, splits);
    hipLaunchKernelGGL(wgrad_x6_big_kernel, g2, dim3(kThreads), 0, s, p);
  } else if (x6) {
    hipLaunchKernelGGL(wgrad_kernel<true>, grid, dim3(kThreads), 0, s, p);
  } else {
    hipLaunchKernelGGL(wgrad_kernel<false>, grid, dim3(kThreads), 0, s, p);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return static_cast<int>(e);
  const int64_t total = static_cast<int64_t>(a->cout) * p.K;
  // the grouped form where one thread per output would leave the chip mostly idle on a long chain
  if (splits >= 4 * kRedGrp && total <= 2048 * kThreads)
    hipLaunchKernelGGL(wgrad_reduce_grouped_kernel, dim3(static_cast<unsigned>((total + kRedOut - 1) / kRedOut)),
                       dim3(kThreads), 0, s, p.ws, splits, a->cout, a->cin, a->cin_stride, a->ks, p.K, a->dw,
                       a->accumulate);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_of(total)), dim3(kThreads), 0, s, p.ws, splits, a->cout, a->cin,
                       a->cin_stride, a->ks, p.K, a->dw, a->accumulate);
  return static_cast<int>(hipGetLastError());
}

// fp32 [n] -> bf16 [3][n] planes, w = w1 + w2 + w3 (round to nearest even at each step): the weight
// side of the fp32x arithmetic in one pass (drnmi/engine.py split3_bf16 took six ATen launches per
// weight and step in the fp32x fine-tune)
__global__ void __launch_bounds__(kThreads)
split3_kernel(const float* __restrict__ w, int64_t n, bf16_t* __restrict__ out) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const float x = w[i];
    const bf16_t a = f32_to_bf16(x);
    const float r = x - bf16_to_f32(a);
    const bf16_t b = f32_to_bf16(r);
    out[i] = a;
    out[n + i] = b;
    out[2 * n + i] = f32_to_bf16(r - bf16_to_f32(b));
  }
}

extern "C" int drnmi_split3_bf16(const float* w, int64_t n, void* out, void* stream) {
  if (w == nullptr || out == nullptr || n <= 0) return DRNMI_EINVAL;
  hipLaunchKernelGGL(split3_kernel, dim3(grid_of(n)), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream), w, n,
                     reinterpret_cast<bf16_t*>(out));
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_conv_wgrad_f32(const drnmi_wgrad_args* a, void* stream) { return wgrad_launch(a, false, stream); }
extern "C" int drnmi_conv_wgrad_f32x3(const drnmi_wgrad_args* a, void* stream) { return wgrad_launch(a, true, stream); }

extern "C" int drnmi_zero_insert_f32(const float* dy, int32_t n, int32_t ho, int32_t wo, int32_t c, int32_t stride,
                                     int32_t hu, int32_t wu, float* out, void* stream) {
  if (dy == nullptr || out == nullptr || n <= 0 || ho <= 0 || wo <= 0 || c <= 0 || c % 4 != 0 || stride <= 0 ||
      hu <= 0 || wu <= 0)
    return DRNMI_EINVAL;
  const int64_t total = static_cast<int64_t>(n) * hu * wu * (c / 4);
  hipLaunchKernelGGL(zero_insert_kernel, dim3(grid_of(total)), dim3(kThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), dy, n, ho, wo, c / 4, stride, hu, wu, out);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_up8_lsm_bwd_f32(const float* g_logprobs, const float* logprobs, const float* g_logits,
                                     const float* up_w, float grad_scale, int32_t n, int32_t c, int32_t h, int32_t w,
                                     float* du_ws, float* dlogits, void* stream) {
  if (up_w == nullptr || dlogits == nullptr || n <= 0 || c <= 0 || h <= 0 || w <= 0) return DRNMI_EINVAL;
  if (g_logprobs != nullptr && (logprobs == nullptr || du_ws == nullptr)) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t hw = static_cast<int64_t>(64) * h * w;
  if (g_logprobs != nullptr) {
    if (c == 19)
      hipLaunchKernelGGL(lsm_bwd_kernel<19>, dim3(grid_of(n * hw)), dim3(kThreads), 0, s, g_logprobs, logprobs, n, c, hw,
                         grad_scale, du_ws);
    else
      hipLaunchKernelGGL(lsm_bwd_kernel<0>, dim3(grid_of(n * hw)), dim3(kThreads), 0, s, g_logprobs, logprobs, n, c, hw,
                         grad_scale, du_ws);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  } else if (g_logits == nullptr) {   // logits-only gradient: dlogits = grad_scale * g_logits
    return DRNMI_EINVAL;
  }
  if (static_cast<int64_t>(n) * c > 65535) return DRNMI_EINVAL;   // planes on grid z
  hipLaunchKernelGGL(up8_bwd_kernel, dim3((w + kUbJ - 1) / kUbJ, (h + kUbI - 1) / kUbI, n * c), dim3(kUbThreads), 0, s,
                     g_logprobs != nullptr ? du_ws : nullptr, up_w, g_logits, grad_scale, n * c, h, w, dlogits);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_up8_bilinear_lsm_bwd_f32(const float* g_logprobs, const float* logprobs, const float* g_logits,
                                              float grad_scale, int32_t n, int32_t c, int32_t h, int32_t w,
                                              float* du_ws, float* dlogits, void* stream) {
  if (dlogits == nullptr || n <= 0 || c <= 0 || h <= 0 || w <= 0) return DRNMI_EINVAL;
  if (g_logprobs != nullptr && (logprobs == nullptr || du_ws == nullptr)) return DRNMI_EINVAL;
  if (g_logprobs == nullptr && g_logits == nullptr) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t hw = static_cast<int64_t>(64) * h * w;
  if (g_logprobs != nullptr) {
    if (c == 19)
      hipLaunchKernelGGL(lsm_bwd_kernel<19>, dim3(grid_of(n * hw)), dim3(kThreads), 0, s, g_logprobs, logprobs, n, c, hw,
                         grad_scale, du_ws);
    else
      hipLaunchKernelGGL(lsm_bwd_kernel<0>, dim3(grid_of(n * hw)), dim3(kThreads), 0, s, g_logprobs, logprobs, n, c, hw,
                         grad_scale, du_ws);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  hipLaunchKernelGGL(up8_bilinear_bwd_kernel, dim3(grid_of(static_cast<int64_t>(n) * c * h * w)), dim3(kThreads), 0, s,
                     g_logprobs != nullptr ? du_ws : nullptr, g_logits, grad_scale, n * c, h, w, dlogits);
  return static_cast<int>(hipGetLastError());
}

extern "C" int64_t drnmi_ce_workspace_bytes(void) { return 3LL * kCeBlocks * 8; }

extern "C" int drnmi_ce_loss_f32(const float* logprobs, const int64_t* target, int32_t n, int32_t c, int64_t hw,
                                 int64_t ignore_index, float* loss, float* count, void* ws, void* stream) {
  if (logprobs == nullptr || target == nullptr || loss == nullptr || count == nullptr || ws == nullptr || n <= 0 ||
      c <= 0 || hw <= 0)
    return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (c == 19)
    hipLaunchKernelGGL(ce_fwd_kernel<19>, dim3(kCeBlocks), dim3(kThreads), 0, s, logprobs, target, n, c, hw,
                       ignore_index, reinterpret_cast<double*>(ws));
  else
    hipLaunchKernelGGL(ce_fwd_kernel<0>, dim3(kCeBlocks), dim3(kThreads), 0, s, logprobs, target, n, c, hw,
                       ignore_index, reinterpret_cast<double*>(ws));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return static_cast<int>(e);
  hipLaunchKernelGGL(ce_final_kernel, dim3(1), dim3(64), 0, s, reinterpret_cast<const double*>(ws), kCeBlocks, loss,
                     count);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_ce_loss_bwd_f32(const float* logprobs, const int64_t* target, int32_t n, int32_t c, int64_t hw,
                                     int64_t ignore_index, const float* dloss, const float* count, float* g_logprobs,
                                     void* stream) {
  if (logprobs == nullptr || target == nullptr || dloss == nullptr || count == nullptr || g_logprobs == nullptr ||
      n <= 0 || c <= 0 || hw <= 0)
    return DRNMI_EINVAL;
  if (c == 19 && hw % 4 == 0 && aligned16(logprobs, g_logprobs, nullptr))
    hipLaunchKernelGGL(ce_bwd_v4_kernel<19>, dim3(grid_of(static_cast<int64_t>(n) * hw / 4)), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), logprobs, target, n, c, hw, ignore_index, dloss, count,
                       g_logprobs);
  else if (c == 19)
    hipLaunchKernelGGL(ce_bwd_kernel<19>, dim3(grid_of(static_cast<int64_t>(n) * hw)), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), logprobs, target, n, c, hw, ignore_index, dloss, count,
                       g_logprobs);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<0>, dim3(grid_of(static_cast<int64_t>(n) * hw)), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), logprobs, target, n, c, hw, ignore_index, dloss, count,
                       g_logprobs);
  return static_cast<int>(hipGetLastError());
}

extern "C" int drnmi_sgd_step_f32(int32_t ntensors, float* const* params, const float* const* grads,
                                  float* const* momentum_bufs, const int64_t* numels,
                                  const uint32_t* const* mask_bits, const int32_t* first_step, float lr,
                                  float momentum, float dampening, float weight_decay, int32_t nesterov,
                                  void* stream) {
  if (ntensors < 0 || (ntensors > 0 && (params == nullptr || grads == nullptr || numels == nullptr)))
    return DRNMI_EINVAL;
  if (momentum != 0.f && ntensors > 0 && (momentum_bufs == nullptr || first_step == nullptr)) return DRNMI_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (int t0 = 0; t0 < ntensors; t0 += kSgdBatch) {
    SgdBatch b{};
    const int cnt = ntensors - t0 < kSgdBatch ? ntensors - t0 : kSgdBatch;
    int64_t maxn = 0;
    for (int i = 0; i < cnt; ++i) {
      const int k = t0 + i;
      b.w[i] = params[k];
      b.g[i] = grads[k];
      b.buf[i] = momentum != 0.f ? momentum_bufs[k] : nullptr;
      b.mask[i] = mask_bits != nullptr ? mask_bits[k] : nullptr;
      b.numel[i] = numels[k];
      b.first[i] = momentum != 0.f ? first_step[k] : 0;
      if (b.numel[i] < 0) return DRNMI_EINVAL;
      if (b.numel[i] > 0 && (b.w[i] == nullptr || b.g[i] == nullptr || (momentum != 0.f && b.buf[i] == nullptr)))
        return DRNMI_EINVAL;
      maxn = b.numel[i] > maxn ? b.numel[i] : maxn;
    }
    if (maxn == 0) continue;
    unsigned gx = grid_of(maxn);
    gx = gx > 1024 ? 1024 : gx;
    hipLaunchKernelGGL(sgd_kernel, dim3(gx, cnt), dim3(kThreads), 0, s, b, lr, momentum, dampening, weight_decay,
                       nesterov);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return DRNMI_OK;
}
