// Fused Conv2D(+bias+ReLU)+MaxPool(2x2) kernels for small-channel convolutions (gfx950).
//
// The MNIST CNNs of the reference (model.json conv->relu->...->maxpool, and the
// LeNet-5 of BASELINE.json) have 1-16 input channels on 10-32 pixel images: as separate GEMM, ReLU,
// pool passes they are bound by HBM round trips of the full-resolution activation and by
// 2-byte gathers.  Here a workgroup stages WHOLE images in LDS (zero-padded border) and:
//
//   convpool_fwd    im2col A-fragments are read straight from the LDS image through a per-k offset
//                   table, weights sit in registers, v_mfma_f32_16x16x32_bf16 computes 16 pixels x
//                   16 channels; the 16 MFMA rows are ordered as 4 pool windows x 4 pixels, so every
//                   lane ends up holding one complete 2x2 window of one channel in its 4 accumulator
//                   registers -> bias + max + ReLU in registers, and only the POOLED map (1/4 of the
//                   conv output) plus a 1-byte argmax code (bit2 = "max > 0", relu') reach HBM.
//                   The first layer can read the uint8 dataset through the batch index vector, fusing
//                   the batch gather and u8->bf16 cast.
//   convpool_wgrad  dW = sum_pixels dConv^T * im2col(X): dConv is regenerated in registers from
//                   (dPooled, code) — the full-resolution gradient never exists in memory — and the
//                   bias gradient is an extra "ones" column.  Per-workgroup fp32 slab -> slab_reduce.
//   convpool_dgrad  dX = transposed conv of dConv: dConv is rebuilt in a zero-padded LDS image from
//                   (dPooled, code), A-fragments are 16-byte LDS reads (8 consecutive out channels),
//                   dgrad-layout weights sit in registers.
#include "common.h"
#include "kernels.h"

namespace dfa {

struct CPGeom {
  int B, H, W, C, KH, KW, pad, N, OH, OW, PH, PW, K, Kpad;
  int Hp, Wp, img_elems;  // padded input image in LDS
  int imgs;               // images per workgroup
};

__device__ __forceinline__ long long cp_clamp(long long r, long long n) { return r < 0 ? 0 : (r >= n ? n - 1 : r); }

// Stage images [b0, b0+nimg) into LDS (zero border).  Source: bf16 NHWC, or u8 rows gathered via idx.
__device__ __forceinline__ void stage_images(bf16* xs, const CPGeom& g, const void* x, int x_u8, const long long* idx,
                                             long long nrows, float scale, int b0, int nimg) {
  const int tid = threadIdx.x;
  {
    const int tot8 = (nimg * g.img_elems + 7) / 8;
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
    for (int e = tid; e < tot8; e += blockDim.x) reinterpret_cast<bf16x8*>(xs)[e] = z;
  }
  __syncthreads();
  const int WC = g.W * g.C;
  const int HWC = g.H * WC;
  const int total = nimg * HWC;
  for (int e = tid; e < total; e += blockDim.x) {
    const int i = e / HWC;
    const int r = e - i * HWC;
    const int y = r / WC;
    const int q = r - y * WC;
    bf16 v;
    if (x_u8) {
      const long long row = cp_clamp(idx[b0 + i], nrows);
      v = f2bf((float)reinterpret_cast<const uint8_t*>(x)[row * HWC + r] * scale);
    } else {
      v = reinterpret_cast<const bf16*>(x)[(long long)(b0 + i) * HWC + r];
    }
    xs[i * g.img_elems + ((y + g.pad) * g.Wp + g.pad) * g.C + q] = v;
  }
}

// ------------------------------------------------------------------------------------------------
template <int NT, int NKMAX>
__global__ void __launch_bounds__(256) convpool_fwd_kernel(CPGeom g, const void* x, int x_u8, const long long* idx,
                                                           long long nrows, float scale, const bf16* __restrict__ w,
                                                           const float* __restrict__ bias, bf16* __restrict__ p,
                                                           uint8_t* __restrict__ code) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* lut = reinterpret_cast<int*>(smem);
  bf16* xs = reinterpret_cast<bf16*>(smem + g.Kpad * 4);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b0 = blockIdx.x * g.imgs;
  const int nimg = min(g.imgs, g.B - b0);
  for (int k = tid; k < g.Kpad; k += 256) {
    int v = -1;
    if (k < g.K) {
      const int c = k % g.C, t = k / g.C, ky = t / g.KW, kx = t - ky * g.KW;
      v = (ky * g.Wp + kx) * g.C + c;
    }
    lut[k] = v;
  }
  stage_images(xs, g, x, x_u8, idx, nrows, scale, b0, nimg);
  const int nk = g.Kpad / 32;
  const int Npad = round_up(g.N, 16);
  bf16x8 bfr[NKMAX][NT];
#pragma unroll
  for (int s = 0; s < NKMAX; ++s)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = 16 * t + (lane & 15);
      if (s < nk && n < Npad)
        bfr[s][t] = *reinterpret_cast<const bf16x8*>(w + (long long)n * g.Kpad + 32 * s + 8 * (lane >> 4));
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) bfr[s][t][e] = (bf16)0.f;
    }
  __syncthreads();

  const int npool = g.PH * g.PW;
  const int tpi = (npool + 3) / 4;
  const int total = nimg * tpi;
  const int row = lane & 15;
  for (int tile = wid; tile < total; tile += 4) {
    const int i = tile / tpi;
    const int tw = tile - i * tpi;
    // A-fragment row -> (window, pixel in window)
    const int wg = tw * 4 + (row >> 2);
    const int j = row & 3;
    int base = i * g.img_elems;
    if (wg < npool) {
      const int py = wg / g.PW, px = wg - (wg / g.PW) * g.PW;
      const int oy = 2 * py + (j >> 1), ox = 2 * px + (j & 1);
      base += (oy * g.Wp + ox) * g.C;
    }
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NKMAX; ++s) {
      if (s < nk) {
        const int kb = 32 * s + 8 * (lane >> 4);
        bf16x8 a;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int off = lut[kb + e];
          a[e] = off >= 0 ? xs[base + off] : (bf16)0.f;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x32(a, bfr[s][t], acc[t]);
      }
    }
    // accumulator: col = lane&15 (channel), rows 4*(lane>>4)+r = the 4 pixels of window (lane>>4)
    const int wo = tw * 4 + (lane >> 4);
    if (wo < npool) {
      const long long obase = ((long long)(b0 + i) * npool + wo) * g.N;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = 16 * t + (lane & 15);
        if (n < g.N) {
          float m = acc[t][0];
          int am = 0;
#pragma unroll
          for (int r = 1; r < 4; ++r)
            if (acc[t][r] > m) { m = acc[t][r]; am = r; }
          m += bias ? bias[n] : 0.f;
          p[obase + n] = f2bf(fmaxf(m, 0.f));
          if (code) code[obase + n] = (uint8_t)(am | (m > 0.f ? 4 : 0));
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Weight gradient through the pool: partial[block][n][k] (k == K: bias).
template <int NT, int KTMAX>
__global__ void __launch_bounds__(256) convpool_wgrad_kernel(CPGeom g, const void* x, int x_u8, const long long* idx,
                                                             long long nrows, float scale,
                                                             const bf16* __restrict__ dp,
                                                             const uint8_t* __restrict__ code,
                                                             float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Kt = g.K + 1;
  const int KT = (Kt + 15) / 16;
  const int npool = g.PH * g.PW;
  int* lut = reinterpret_cast<int*>(smem);                                     // [KT*16]
  bf16* xs = reinterpret_cast<bf16*>(smem + round_up(KT * 16 * 4, 16));        // [imgs][img_elems]
  char* after_x = reinterpret_cast<char*>(xs) + round_up(g.imgs * g.img_elems * 2 + 16, 16);
  bf16* dps = reinterpret_cast<bf16*>(after_x);                                // [imgs][npool][N]
  uint8_t* cds = reinterpret_cast<uint8_t*>(after_x + round_up(g.imgs * npool * g.N * 2, 16));
  float* red = reinterpret_cast<float*>(smem);  // aliases everything after the main loop: [4][NT*16][KT*16]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b0 = blockIdx.x * g.imgs;
  const int nimg = min(g.imgs, g.B - b0);
  for (int k = tid; k < KT * 16; k += 256) {
    int v = -1;
    if (k < g.K) {
      const int c = k % g.C, t = k / g.C, ky = t / g.KW, kx = t - ky * g.KW;
      v = (ky * g.Wp + kx) * g.C + c;
    } else if (k == g.K) {
      v = -2;
    }
    lut[k] = v;
  }
  for (int e = tid; e < nimg * npool * g.N; e += 256) {
    const long long o = (long long)b0 * npool * g.N + e;
    dps[e] = dp[o];
    cds[e] = code[o];
  }
  stage_images(xs, g, x, x_u8, idx, nrows, scale, b0, nimg);
  __syncthreads();

  f32x4 acc[NT][KTMAX];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < KTMAX; ++q) acc[t][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int cpi = (npool + 7) / 8;  // 32-pixel chunks (8 windows) per image
  const int total = nimg * cpi;
  const int h = lane >> 4;
  for (int chunk = wid; chunk < total; chunk += 4) {
    const int i = chunk / cpi;
    const int cw = chunk - i * cpi;
    // this lane's 8 reduction elements m = 8h + e  -> windows w0 = 8cw + 2h, w0+1 ; pixel e&3
    const int w0 = cw * 8 + 2 * h;
    int pbase[8];
    bool pval[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int wg = w0 + (e >> 2);
      const int j = e & 3;
      pval[e] = wg < npool;
      const int wgc = pval[e] ? wg : 0;
      const int py = wgc / g.PW, px = wgc - (wgc / g.PW) * g.PW;
      const int oy = 2 * py + (j >> 1), ox = 2 * px + (j & 1);
      pbase[e] = i * g.img_elems + (oy * g.Wp + ox) * g.C;
    }
    bf16x8 afr[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = 16 * t + (lane & 15);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bf16 v = (bf16)0.f;
        const int wg = w0 + (e >> 2);
        if (n < g.N && wg < npool) {
          const int o = (i * npool + wg) * g.N + n;
          const int cd = cds[o];
          if ((cd & 4) && (cd & 3) == (e & 3)) v = dps[o];
        }
        afr[t][e] = v;
      }
    }
#pragma unroll
    for (int q = 0; q < KTMAX; ++q) {
      if (q < KT) {
        const int off = lut[16 * q + (lane & 15)];
        bf16x8 b;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          bf16 v = (bf16)0.f;
          if (pval[e]) {
            if (off >= 0) v = xs[pbase[e] + off];
            else if (off == -2) v = (bf16)1.f;
          }
          b[e] = v;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t][q] = mfma16x16x32(afr[t], b, acc[t][q]);
      }
    }
  }
  __syncthreads();  // everything staged is dead now; reuse LDS for the cross-wave reduction
  const int RW = KT * 16;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < KTMAX; ++q) {
      if (q < KT) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * t + 4 * (lane >> 4) + r;
          const int k = 16 * q + (lane & 15);
          red[(wid * NT * 16 + n) * RW + k] = acc[t][q][r];
        }
      }
    }
  __syncthreads();
  for (int e = tid; e < g.N * Kt; e += 256) {
    const int n = e / Kt, k = e - (e / Kt) * Kt;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) s += red[(ww * NT * 16 + n) * RW + k];
    partial[(long long)blockIdx.x * g.N * Kt + e] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// Data gradient through the pool: dx[b][iy][ix][c] = sum_{ky,kx,n} dConv[iy+pad-ky][ix+pad-kx][n] W[n][ky][kx][c]
struct CPDgrad {
  int Hq, Wq, q_elems, P;  // padded dConv image in LDS, P = KH-1-pad
  int K2, K2pad;           // K2 = KH*KW*N
};

template <int NT, int NKMAX, bool VEC>
__global__ void __launch_bounds__(256) convpool_dgrad_kernel(CPGeom g, CPDgrad d, const bf16* __restrict__ dp,
                                                             const uint8_t* __restrict__ code,
                                                             const bf16* __restrict__ wt, bf16* __restrict__ dx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* lut = reinterpret_cast<int*>(smem);                          // [K2pad]
  bf16* qs = reinterpret_cast<bf16*>(smem + round_up(d.K2pad * 4, 16));  // [imgs][Hq][Wq][N]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b0 = blockIdx.x * g.imgs;
  const int nimg = min(g.imgs, g.B - b0);
  const int npool = g.PH * g.PW;
  for (int k = tid; k < d.K2pad; k += 256) {
    int v = -1;
    if (k < d.K2) {
      const int n = k % g.N, t = k / g.N, ky = t / g.KW, kx = t - ky * g.KW;
      v = ((g.KH - 1 - ky) * d.Wq + (g.KW - 1 - kx)) * g.N + n;
    }
    lut[k] = v;
  }
  {
    const int tot8 = (nimg * d.q_elems + 7) / 8;
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
    for (int e = tid; e < tot8; e += 256) reinterpret_cast<bf16x8*>(qs)[e] = z;
  }
  __syncthreads();
  for (int e = tid; e < nimg * npool * g.N; e += 256) {
    const long long o = (long long)b0 * npool * g.N + e;
    const int cd = code[o];
    if (cd & 4) {
      const int n = e % g.N;
      const int r = e / g.N;
      const int i = r / npool;
      const int wg = r - i * npool;
      const int py = wg / g.PW, px = wg - (wg / g.PW) * g.PW;
      const int oy = 2 * py + ((cd & 3) >> 1), ox = 2 * px + (cd & 1);
      qs[i * d.q_elems + ((oy + d.P) * d.Wq + ox + d.P) * g.N + n] = dp[o];
    }
  }
  const int nk = d.K2pad / 32;
  const int Cpad = round_up(g.C, 16);
  bf16x8 bfr[NKMAX][NT];
#pragma unroll
  for (int s = 0; s < NKMAX; ++s)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = 16 * t + (lane & 15);
      if (s < nk && c < Cpad)
        bfr[s][t] = *reinterpret_cast<const bf16x8*>(wt + (long long)c * d.K2pad + 32 * s + 8 * (lane >> 4));
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) bfr[s][t][e] = (bf16)0.f;
    }
  __syncthreads();

  const int HW = g.H * g.W;
  const int tpi = (HW + 15) / 16;
  const int total = nimg * tpi;
  for (int tile = wid; tile < total; tile += 4) {
    const int i = tile / tpi;
    const int tw = tile - i * tpi;
    const int m = tw * 16 + (lane & 15);
    int base = i * d.q_elems;
    const bool mv = m < HW;
    if (mv) {
      const int iy = m / g.W, ix = m - (m / g.W) * g.W;
      base += (iy * d.Wq + ix) * g.N;
    }
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NKMAX; ++s) {
      if (s < nk) {
        const int kb = 32 * s + 8 * (lane >> 4);
        bf16x8 a;
        if (VEC) {
          const int off = lut[kb];
          if (off >= 0) {
            a = *reinterpret_cast<const bf16x8*>(qs + base + off);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = (bf16)0.f;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int off = lut[kb + e];
            a[e] = off >= 0 ? qs[base + off] : (bf16)0.f;
          }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x32(a, bfr[s][t], acc[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = 16 * t + (lane & 15);
      if (c >= g.C) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mm = tw * 16 + 4 * (lane >> 4) + r;
        if (mm < HW) dx[((long long)(b0 + i) * HW + mm) * g.C + c] = f2bf(acc[t][r]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Deterministic parallel reduction of S fp32 slabs [S][N][Kt] into gw[N][K] (k < K) and gb[N] (k == K).
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ partial, float* __restrict__ gw,
                                                          float* __restrict__ gb, int N, int K, int Kt, int S,
                                                          float scale) {
  __shared__ float red[8][33];
  const int total = N * Kt;
  const int o = blockIdx.x * 32 + (threadIdx.x & 31);
  const int grp = threadIdx.x >> 5;  // 8 groups stride over the slabs
  float s = 0.f;
  if (o < total)
    for (int p = grp; p < S; p += 8) s += partial[(long long)p * total + o];
  red[grp][threadIdx.x & 31] = s;
  __syncthreads();
  if (threadIdx.x < 32 && o < total) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][threadIdx.x];
    const int n = o / Kt, k = o - (o / Kt) * Kt;
    if (k < K)
      gw[(long long)n * K + k] = t * scale;
    else if (gb)
      gb[n] = t * scale;
  }
}

hipError_t slab_reduce(const float* partial, float* gw, float* gb, int N, int K, int Kt, int S, float scale,
                       hipStream_t st) {
  const int total = N * Kt;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(cdiv(total, 32)), dim3(256), 0, st, partial, gw, gb, N, K, Kt, S, scale);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// host side
static CPGeom make_geom(int B, int H, int W, int C, int KH, int KW, int pad, int N) {
  CPGeom g{};
  g.B = B; g.H = H; g.W = W; g.C = C; g.KH = KH; g.KW = KW; g.pad = pad; g.N = N;
  g.OH = H + 2 * pad - KH + 1;
  g.OW = W + 2 * pad - KW + 1;
  g.PH = g.OH / 2;
  g.PW = g.OW / 2;
  g.K = KH * KW * C;
  g.Kpad = round_up(g.K, 32);
  g.Hp = H + 2 * pad;
  g.Wp = W + 2 * pad;
  g.img_elems = round_up(g.Hp * g.Wp * C, 8);
  return g;
}

static const size_t kLdsBudget = 64 * 1024;  // keeps >= 2 workgroups per CU (160 KiB LDS)

bool convpool_supported(int H, int W, int C, int KH, int KW, int pad, int N) {
  CPGeom g = make_geom(1, H, W, C, KH, KW, pad, N);
  if (g.OH <= 0 || g.OW <= 0 || (g.OH & 1) || (g.OW & 1)) return false;
  if (C > 16 || N > 32 || KH > 7 || KW > 7) return false;
  if (g.Kpad / 32 > 16) return false;                 // fwd weight fragments in registers
  if ((g.K + 1 + 15) / 16 > 12) return false;          // wgrad accumulators
  if (round_up(KH * KW * N, 32) / 32 > 16) return false;  // dgrad weight fragments
  const int P = KH - 1 - pad;
  if (P < 0) return false;
  const size_t q_elems = (size_t)(g.OH + 2 * P) * (g.OW + 2 * P) * N;
  if ((size_t)g.img_elems * 2 > kLdsBudget / 2 || q_elems * 2 > kLdsBudget / 2) return false;
  return true;
}

template <int NT, int NKMAX>
static void launch_cp_fwd(const CPGeom& g, size_t lds, const void* x, int x_u8, const long long* idx, long long nrows,
                          float scale, const bf16* w, const float* bias, bf16* p, uint8_t* code, hipStream_t st) {
  hipLaunchKernelGGL((convpool_fwd_kernel<NT, NKMAX>), dim3(cdiv(g.B, g.imgs)), dim3(256), lds, st, g, x, x_u8, idx,
                     nrows, scale, w, bias, p, code);
}

hipError_t convpool_fwd(const void* x, int x_u8, const long long* idx, long long nrows, float scale, int B, int H,
                        int W, int C, int KH, int KW, int pad, int N, const bf16* w, const float* bias, bf16* p,
                        uint8_t* code, hipStream_t st) {
  if (!convpool_supported(H, W, C, KH, KW, pad, N)) return hipErrorInvalidValue;
  CPGeom g = make_geom(B, H, W, C, KH, KW, pad, N);
  const size_t fixed = (size_t)g.Kpad * 4;
  g.imgs = (int)max((size_t)1, (kLdsBudget - fixed) / ((size_t)g.img_elems * 2));
  g.imgs = min(g.imgs, 32);
  // keep at least ~2 workgroups per CU when the batch allows it
  while (g.imgs > 1 && cdiv(B, g.imgs) < 512) g.imgs /= 2;
  const size_t lds = fixed + (size_t)g.imgs * g.img_elems * 2;
  const int nk = g.Kpad / 32;
  const int nt = cdiv(N, 16);
  if (nt == 1) {
    if (nk <= 2) launch_cp_fwd<1, 2>(g, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else if (nk <= 8) launch_cp_fwd<1, 8>(g, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else launch_cp_fwd<1, 16>(g, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
  } else {
    if (nk <= 2) launch_cp_fwd<2, 2>(g, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else if (nk <= 8) launch_cp_fwd<2, 8>(g, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else launch_cp_fwd<2, 16>(g, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
  }
  return hipGetLastError();
}

template <int NT, int KTMAX>
static void launch_cp_wgrad(const CPGeom& g, size_t lds, int grid, const void* x, int x_u8, const long long* idx,
                            long long nrows, float scale, const bf16* dp, const uint8_t* code, float* partial,
                            hipStream_t st) {
  hipLaunchKernelGGL((convpool_wgrad_kernel<NT, KTMAX>), dim3(grid), dim3(256), lds, st, g, x, x_u8, idx, nrows,
                     scale, dp, code, partial);
}

hipError_t convpool_wgrad(const void* x, int x_u8, const long long* idx, long long nrows, float scale, int B, int H,
                          int W, int C, int KH, int KW, int pad, int N, const bf16* dp, const uint8_t* code,
                          float* gw, float* gb, float* workspace, size_t ws_floats, hipStream_t st) {
  if (!convpool_supported(H, W, C, KH, KW, pad, N)) return hipErrorInvalidValue;
  CPGeom g = make_geom(B, H, W, C, KH, KW, pad, N);
  const int Kt = g.K + 1;
  const int KT = cdiv(Kt, 16);
  const int NT = cdiv(N, 16);
  const int npool = g.PH * g.PW;
  const size_t fixed = round_up(KT * 16 * 4, 16);
  const size_t per_img = (size_t)g.img_elems * 2 + round_up(npool * N * 2, 16) + round_up(npool * N, 16) + 32;
  g.imgs = (int)max((size_t)1, (kLdsBudget - fixed) / per_img);
  g.imgs = min(g.imgs, 64);
  while (g.imgs > 1 && cdiv(B, g.imgs) < 512) g.imgs /= 2;
  // slab capacity: fewer, fatter workgroups if the workspace is small
  while ((size_t)cdiv(B, g.imgs) * N * Kt > ws_floats && g.imgs < B) g.imgs *= 2;
  const int grid = cdiv(B, g.imgs);
  if ((size_t)grid * N * Kt > ws_floats) return hipErrorInvalidValue;
  size_t lds = fixed + (size_t)g.imgs * g.img_elems * 2 + 16 + round_up(g.imgs * npool * N * 2, 16) +
               round_up(g.imgs * npool * N, 16) + 64;
  const size_t red_bytes = (size_t)4 * NT * 16 * KT * 16 * 4;
  if (lds < red_bytes) lds = red_bytes;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (NT == 1) {
    if (KT <= 2) launch_cp_wgrad<1, 2>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
    else if (KT <= 4) launch_cp_wgrad<1, 4>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
    else launch_cp_wgrad<1, 12>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
  } else {
    if (KT <= 2) launch_cp_wgrad<2, 2>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
    else if (KT <= 4) launch_cp_wgrad<2, 4>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
    else launch_cp_wgrad<2, 12>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
  }
  DFA_HIP_CHECK(hipGetLastError());
  return slab_reduce(workspace, gw, gb, N, g.K, Kt, grid, 1.f, st);
}

template <int NT, int NKMAX, bool VEC>
static void launch_cp_dgrad(const CPGeom& g, const CPDgrad& d, size_t lds, const bf16* dp, const uint8_t* code,
                            const bf16* wt, bf16* dx, hipStream_t st) {
  hipLaunchKernelGGL((convpool_dgrad_kernel<NT, NKMAX, VEC>), dim3(cdiv(g.B, g.imgs)), dim3(256), lds, st, g, d, dp,
                     code, wt, dx);
}

hipError_t convpool_dgrad(const bf16* dp, const uint8_t* code, const bf16* wt, bf16* dx, int B, int H, int W, int C,
                          int KH, int KW, int pad, int N, hipStream_t st) {
  if (!convpool_supported(H, W, C, KH, KW, pad, N)) return hipErrorInvalidValue;
  CPGeom g = make_geom(B, H, W, C, KH, KW, pad, N);
  CPDgrad d{};
  d.P = KH - 1 - pad;
  d.Hq = g.OH + 2 * d.P;
  d.Wq = g.OW + 2 * d.P;
  d.q_elems = round_up(d.Hq * d.Wq * N, 8);
  d.K2 = KH * KW * N;
  d.K2pad = round_up(d.K2, 32);
  const size_t fixed = round_up(d.K2pad * 4, 16);
  g.imgs = (int)max((size_t)1, (kLdsBudget - fixed) / ((size_t)d.q_elems * 2));
  g.imgs = min(g.imgs, 32);
  while (g.imgs > 1 && cdiv(B, g.imgs) < 512) g.imgs /= 2;
  const size_t lds = fixed + (size_t)g.imgs * d.q_elems * 2;
  const int nk = d.K2pad / 32;
  const int nt = cdiv(C, 16);
  const bool vec = N % 8 == 0;
  if (nt != 1) return hipErrorInvalidValue;
  if (vec) {
    if (nk <= 8) launch_cp_dgrad<1, 8, true>(g, d, lds, dp, code, wt, dx, st);
    else launch_cp_dgrad<1, 16, true>(g, d, lds, dp, code, wt, dx, st);
  } else {
    if (nk <= 8) launch_cp_dgrad<1, 8, false>(g, d, lds, dp, code, wt, dx, st);
    else launch_cp_dgrad<1, 16, false>(g, d, lds, dp, code, wt, dx, st);
  }
  return hipGetLastError();
}

}  // namespace dfa
