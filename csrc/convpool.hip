// Fused Conv2D(+bias+ReLU)+MaxPool(2x2) kernels for small-channel convolutions (gfx950).
//
// The MNIST CNNs of the reference (model.json conv->relu->...->maxpool, and the
// LeNet-5 of BASELINE.json) have 1-16 input channels on 10-32 pixel images: as separate GEMM, ReLU,
// pool passes they are bound by HBM round trips of the full-resolution activation and by
// 2-byte gathers.  Here a workgroup stages WHOLE images in LDS (zero-padded border) and:
//
//   convpool_fwd    im2col A-fragments are read straight from the LDS image through per-lane offset
//                   registers, weights sit in registers, v_mfma_f32_16x16x32_bf16 computes 16 pixels x
//                   16 channels; the 16 MFMA rows are ordered as 4 pool windows x 4 pixels, so every
//                   lane ends up holding one complete 2x2 window of one channel in its 4 accumulator
//                   registers -> bias + max + ReLU in registers, and only the POOLED map (1/4 of the
//                   conv output) plus a 1-byte argmax code (bit2 = "max > 0", relu') reach HBM.
//                   The first layer can read the uint8 dataset through the batch index vector, fusing
//                   the batch gather and u8->bf16 cast.
//   convpool_wgrad  dW = sum_pixels dConv^T * im2col(X): dConv is regenerated in registers from
//                   (dPooled, code) — the full-resolution gradient never exists in memory.  The bias
//                   gradient is summed from the pooled gradient directly.  Per-workgroup fp32 slab ->
//                   slab_reduce (deterministic).
//   convpool_dgrad  dX = transposed conv of dConv: dConv is rebuilt in a zero-padded LDS image from
//                   (dPooled, code), A-fragments are 16-byte LDS reads (8 consecutive out channels),
//                   dgrad-layout weights sit in registers.
//
// Instruction economy (these kernels are issue-bound, not HBM-bound): every per-tile address is a
// table lookup built once per workgroup (no integer division in the tile loops), im2col slots past K
// point at a real LDS element instead of being masked (the matching weight rows are zero padding
// and activations are finite, so they contribute exactly 0), weights / offsets / bias live in
// registers for the whole workgroup.
#include "common.h"
#include "kernels.h"

namespace dfa {

struct CPGeom {
  int B, H, W, C, KH, KW, pad, N, OH, OW, PH, PW, K, Kpad;
  int Hp, Wp, img_elems;  // padded input image in LDS
  int imgs;               // images per workgroup
};

__device__ __forceinline__ long long cp_clamp(long long r, long long n) { return r < 0 ? 0 : (r >= n ? n - 1 : r); }

__device__ __forceinline__ void lds_zero(bf16* p, int elems) {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
  for (int e = threadIdx.x; e < (elems + 7) / 8; e += blockDim.x) reinterpret_cast<bf16x8*>(p)[e] = z;
}

// Stage images [b0, b0+nimg) into LDS (border must already be zero).  Source: bf16 NHWC, or u8
// dataset rows gathered through idx.  One thread per image row segment keeps the divisions out of
// the element loop.
__device__ __forceinline__ void stage_images(bf16* xs, const CPGeom& g, const void* x, int x_u8, const long long* idx,
                                             long long nrows, float scale, int b0, int nimg) {
  const int WC = g.W * g.C;
  const int HWC = g.H * WC;
  const int rows = nimg * g.H;
  // each (image, row) is WC contiguous elements; spread rows over threads, elements over a small loop
  const int tpr = min(64, WC);  // threads per row
  const int rpb = 256 / tpr;    // rows per pass
  const int t = threadIdx.x;
  const int r0 = t / tpr, c0 = t - (t / tpr) * tpr;
  if (r0 >= rpb) return;  // leftover threads when 256 % tpr != 0
  for (int r = r0; r < rows; r += rpb) {
    const int i = r / g.H;
    const int y = r - i * g.H;
    bf16* dst = xs + i * g.img_elems + ((y + g.pad) * g.Wp + g.pad) * g.C;
    if (x_u8) {
      const uint8_t* src = reinterpret_cast<const uint8_t*>(x) + cp_clamp(idx[b0 + i], nrows) * HWC + y * WC;
      for (int c = c0; c < WC; c += tpr) dst[c] = f2bf((float)src[c] * scale);
    } else {
      const bf16* src = reinterpret_cast<const bf16*>(x) + ((long long)(b0 + i) * HWC + y * WC);
      for (int c = c0; c < WC; c += tpr) dst[c] = src[c];
    }
  }
}

// im2col offset of column k inside a padded image (relative to the output pixel's top-left input)
__device__ __forceinline__ int im2col_off(const CPGeom& g, int k) {
  if (k >= g.K) return 0;  // padding column: any finite element (its weight row is zero)
  const int c = k % g.C, t = k / g.C, ky = t / g.KW, kx = t - ky * g.KW;
  return (ky * g.Wp + kx) * g.C + c;
}

// offset (inside a padded image) of conv-output pixel (window wg, pixel j) ; 0 for wg >= npool
__device__ __forceinline__ int window_pixel_off(const CPGeom& g, int wg, int j, int row_stride, int elem) {
  if (wg >= g.PH * g.PW) return 0;
  const int py = wg / g.PW, px = wg - py * g.PW;
  return ((2 * py + (j >> 1)) * row_stride + 2 * px + (j & 1)) * elem;
}

// ------------------------------------------------------------------------------------------------
template <int NT, int NKMAX>
__global__ void __launch_bounds__(256) convpool_fwd_kernel(CPGeom g, const void* x, int x_u8, const long long* idx,
                                                           long long nrows, float scale, const bf16* __restrict__ w,
                                                           const float* __restrict__ bias, bf16* __restrict__ p,
                                                           uint8_t* __restrict__ code) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int npool = g.PH * g.PW;
  const int tpi = (npool + 3) / 4;  // MFMA tiles (4 windows) per image
  int* ttab = reinterpret_cast<int*>(smem);                                          // [tpi*16]
  int* klut = ttab + round_up(tpi * 16, 4);                                          // [Kpad]
  bf16* xs = reinterpret_cast<bf16*>(smem + round_up((round_up(tpi * 16, 4) + g.Kpad) * 4, 16));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // ---- once per workgroup: address tables, zero-bordered image slots, register-resident weights
  for (int e = tid; e < tpi * 16; e += 256) {
    const int row = e & 15;
    ttab[e] = window_pixel_off(g, (e >> 4) * 4 + (row >> 2), row & 3, g.Wp, g.C);
  }
  for (int k = tid; k < g.Kpad; k += 256) klut[k] = im2col_off(g, k);
  lds_zero(xs, g.imgs * g.img_elems);
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
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = 16 * t + (lane & 15);
    bv[t] = (bias && n < g.N) ? bias[n] : 0.f;
  }
  __syncthreads();
  int koff[NKMAX][8];
#pragma unroll
  for (int s = 0; s < NKMAX; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) koff[s][e] = (s < nk) ? klut[32 * s + 8 * (lane >> 4) + e] : 0;

  const int wl = lane >> 4;  // window of this lane's accumulator rows
  // ---- persistent loop over groups of images
  for (int b0 = blockIdx.x * g.imgs; b0 < g.B; b0 += gridDim.x * g.imgs) {
    const int nimg = min(g.imgs, g.B - b0);
    stage_images(xs, g, x, x_u8, idx, nrows, scale, b0, nimg);
    __syncthreads();
    for (int i = 0; i < nimg; ++i) {
      const bf16* xi = xs + i * g.img_elems;
      bf16* pi = p + (long long)(b0 + i) * npool * g.N;
      uint8_t* ci = code ? code + (long long)(b0 + i) * npool * g.N : nullptr;
      for (int tw = wid; tw < tpi; tw += 4) {
        const bf16* xb = xi + ttab[tw * 16 + (lane & 15)];
        f32x4 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NKMAX; ++s) {
          if (s < nk) {
            bf16x8 a;
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = xb[koff[s][e]];
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x32(a, bfr[s][t], acc[t]);
          }
        }
        const int wo = tw * 4 + wl;
        if (wo < npool) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int n = 16 * t + (lane & 15);
            if (n < g.N) {
              float m = acc[t][0];
              int am = 0;
#pragma unroll
              for (int r = 1; r < 4; ++r)
                if (acc[t][r] > m) { m = acc[t][r]; am = r; }
              m += bv[t];
              pi[wo * g.N + n] = f2bf(fmaxf(m, 0.f));
              if (ci) ci[wo * g.N + n] = (uint8_t)(am | (m > 0.f ? 4 : 0));
            }
          }
        }
      }
    }
    __syncthreads();  // image slots are restaged by the next group
  }
}

// ------------------------------------------------------------------------------------------------
// Weight gradient through the pool: partial[block][n][k] (k < K), partial[block][n][K] = bias grad.
template <int NT, int KTMAX>
__global__ void __launch_bounds__(256) convpool_wgrad_kernel(CPGeom g, const void* x, int x_u8, const long long* idx,
                                                             long long nrows, float scale,
                                                             const bf16* __restrict__ dp,
                                                             const uint8_t* __restrict__ code,
                                                             float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Kt = g.K + 1;
  const int KT = (g.K + 15) / 16;  // k-tiles of the weight part
  const int npool = g.PH * g.PW;
  const int cpi = (npool + 7) / 8;  // 32-pixel chunks (8 windows) per image
  int* ctab = reinterpret_cast<int*>(smem);                                     // [cpi*32] pixel offsets
  int* klut = ctab + cpi * 32;                                                  // [KT*16]
  float* bsum = reinterpret_cast<float*>(smem + round_up((cpi * 32 + KT * 16) * 4, 16));  // [32]
  bf16* xs = reinterpret_cast<bf16*>(reinterpret_cast<char*>(bsum) + 128);      // [imgs][img_elems]
  char* after_x = reinterpret_cast<char*>(xs) + round_up(g.imgs * g.img_elems * 2, 16);
  bf16* dps = reinterpret_cast<bf16*>(after_x);                                 // [imgs][npool][N]
  uint8_t* cds = reinterpret_cast<uint8_t*>(after_x + round_up(g.imgs * npool * g.N * 2, 16));
  float* red = reinterpret_cast<float*>(smem);  // aliases all of the above after the main loop

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int e = tid; e < cpi * 32; e += 256) {
    const int m = e & 31;  // m = 4*window_in_chunk + pixel
    ctab[e] = window_pixel_off(g, (e >> 5) * 8 + (m >> 2), m & 3, g.Wp, g.C);
  }
  for (int k = tid; k < KT * 16; k += 256) klut[k] = im2col_off(g, k);
  if (tid < 32) bsum[tid] = 0.f;
  lds_zero(xs, g.imgs * g.img_elems);
  __syncthreads();
  int qoff[KTMAX];
#pragma unroll
  for (int q = 0; q < KTMAX; ++q) qoff[q] = (q < KT) ? klut[16 * q + (lane & 15)] : 0;

  f32x4 acc[NT][KTMAX];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < KTMAX; ++q) acc[t][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the dp/code load loop strides by a multiple of N, so each thread always sees channel tid % N
  // and accumulates that channel's bias gradient in a register
  float bpart = 0.f;
  const int lstride = 256 - 256 % g.N;

  const int h = lane >> 4;
  for (int b0 = blockIdx.x * g.imgs; b0 < g.B; b0 += gridDim.x * g.imgs) {
    const int nimg = min(g.imgs, g.B - b0);
    {
      const int n = nimg * npool * g.N;
      const long long o0 = (long long)b0 * npool * g.N;
      if (tid < lstride) {
        for (int e = tid; e < n; e += lstride) {
          const bf16 dv = dp[o0 + e];
          const int cd = code[o0 + e];
          dps[e] = dv;
          cds[e] = cd;
          if (cd & 4) bpart += (float)dv;
        }
      }
    }
    stage_images(xs, g, x, x_u8, idx, nrows, scale, b0, nimg);
    __syncthreads();
    for (int i = 0; i < nimg; ++i) {
      const bf16* xi = xs + i * g.img_elems;
      const int pbase_i = i * npool * g.N;
      for (int cw = wid; cw < cpi; cw += 4) {
        // reduction slots m = 8h + e of this lane -> windows w0, w0+1 (4 pixels each)
        const int w0 = cw * 8 + 2 * h;
        int pofs[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) pofs[e] = ctab[cw * 32 + 8 * h + e];
        bf16x8 afr[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int n = 16 * t + (lane & 15);
#pragma unroll
          for (int ww = 0; ww < 2; ++ww) {
            int cd = 0;
            bf16 dv = (bf16)0.f;
            if (n < g.N && w0 + ww < npool) {
              const int o = pbase_i + (w0 + ww) * g.N + n;
              cd = cds[o];
              dv = dps[o];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) afr[t][4 * ww + j] = ((cd & 4) && (cd & 3) == j) ? dv : (bf16)0.f;
          }
        }
#pragma unroll
        for (int q = 0; q < KTMAX; ++q) {
          if (q < KT) {
            bf16x8 b;
#pragma unroll
            for (int e = 0; e < 8; ++e) b[e] = xi[pofs[e] + qoff[q]];
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t][q] = mfma16x16x32(afr[t], b, acc[t][q]);
          }
        }
      }
    }
    __syncthreads();  // slots are restaged by the next group
  }
  // bias gradient: per-thread partials of channel tid % N -> LDS
  if (tid < lstride) atomicAdd(&bsum[tid % g.N], bpart);
  __syncthreads();
  const float bias_v = tid < g.N ? bsum[tid] : 0.f;
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
  float* out = partial + (long long)blockIdx.x * g.N * Kt;
  for (int e = tid; e < g.N * g.K; e += 256) {
    const int n = e / g.K, k = e - (e / g.K) * g.K;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) s += red[(ww * NT * 16 + n) * RW + k];
    out[n * Kt + k] = s;
  }
  if (tid < g.N) out[tid * Kt + g.K] = bias_v;
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
  const int HW = g.H * g.W;
  const int tpi = (HW + 15) / 16;
  int* ttab = reinterpret_cast<int*>(smem);  // [tpi*16] input pixel -> qs offset
  int* klut = ttab + tpi * 16;               // [K2pad]
  bf16* qs = reinterpret_cast<bf16*>(smem + round_up((tpi * 16 + d.K2pad) * 4, 16));  // [imgs][Hq][Wq][N]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int npool = g.PH * g.PW;
  for (int e = tid; e < tpi * 16; e += 256) {
    int v = 0;
    if (e < HW) {
      const int iy = e / g.W, ix = e - (e / g.W) * g.W;
      v = (iy * d.Wq + ix) * g.N;
    }
    ttab[e] = v;
  }
  for (int k = tid; k < d.K2pad; k += 256) {
    int v = 0;
    if (k < d.K2) {
      const int n = k % g.N, t = k / g.N, ky = t / g.KW, kx = t - ky * g.KW;
      v = ((g.KH - 1 - ky) * d.Wq + (g.KW - 1 - kx)) * g.N + n;
    }
    klut[k] = v;
  }
  lds_zero(qs, g.imgs * d.q_elems);
  const int nk = d.K2pad / 32;
  const int Cpad = round_up(g.C, 16);
  constexpr int EO = VEC ? 1 : 8;
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
  int koff[NKMAX][EO];
#pragma unroll
  for (int s = 0; s < NKMAX; ++s)
#pragma unroll
    for (int e = 0; e < EO; ++e) koff[s][e] = (s < nk) ? klut[32 * s + 8 * (lane >> 4) + e] : 0;

  const int wn = npool * g.N;
  for (int b0 = blockIdx.x * g.imgs; b0 < g.B; b0 += gridDim.x * g.imgs) {
    const int nimg = min(g.imgs, g.B - b0);
    const long long o0 = (long long)b0 * wn;
    const int ntot = nimg * wn;
    // scatter the routed pooled gradient into the zero full-resolution dConv image
    for (int e = tid; e < ntot; e += 256) {
      const int cd = code[o0 + e];
      if (cd & 4) {
        const int i = e / wn;
        const int r = e - i * wn;
        const int wg = r / g.N, c = r - (r / g.N) * g.N;
        const int py = wg / g.PW, px = wg - (wg / g.PW) * g.PW;
        const int oy = 2 * py + ((cd & 3) >> 1), ox = 2 * px + (cd & 1);
        qs[i * d.q_elems + ((oy + d.P) * d.Wq + ox + d.P) * g.N + c] = dp[o0 + e];
      }
    }
    __syncthreads();
    for (int i = 0; i < nimg; ++i) {
      const bf16* qi = qs + i * d.q_elems;
      bf16* xo = dx + (long long)(b0 + i) * HW * g.C;
      for (int tw = wid; tw < tpi; tw += 4) {
        const bf16* qb = qi + ttab[tw * 16 + (lane & 15)];
        f32x4 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NKMAX; ++s) {
          if (s < nk) {
            bf16x8 a;
            if (VEC) {
              a = *reinterpret_cast<const bf16x8*>(qb + koff[s][0]);
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) a[e] = qb[koff[s][VEC ? 0 : e]];
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
            if (mm < HW) xo[mm * g.C + c] = f2bf(acc[t][r]);
          }
        }
      }
    }
    __syncthreads();
    // restore the zero image: clear exactly the positions scattered above
    for (int e = tid; e < ntot; e += 256) {
      const int cd = code[o0 + e];
      if (cd & 4) {
        const int i = e / wn;
        const int r = e - i * wn;
        const int wg = r / g.N, c = r - (r / g.N) * g.N;
        const int py = wg / g.PW, px = wg - (wg / g.PW) * g.PW;
        const int oy = 2 * py + ((cd & 3) >> 1), ox = 2 * px + (cd & 1);
        qs[i * d.q_elems + ((oy + d.P) * d.Wq + ox + d.P) * g.N + c] = (bf16)0.f;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// Deterministic parallel reduction of S fp32 slabs [S][N][Kt] into gw[N][K] (k < K) and gb[N] (k == K).
// Many slabs (S >= 32): one wave per output, lanes stride the slabs with 4 independent accumulators.
// Few slabs: one thread per output (coalesced across threads), unrolled by 4.
__device__ __forceinline__ void slab_store(float* gw, float* gb, int o, int K, int Kt, float v) {
  const int n = o / Kt, k = o - (o / Kt) * Kt;
  if (k < K)
    gw[(long long)n * K + k] = v;
  else if (gb)
    gb[n] = v;
}

__global__ void __launch_bounds__(256) slab_reduce_wave_kernel(const float* __restrict__ partial,
                                                               float* __restrict__ gw, float* __restrict__ gb, int N,
                                                               int K, int Kt, int S, float scale) {
  const int total = N * Kt;
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (o >= total) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int p = lane;
  for (; p + 192 < S; p += 256) {
    a0 += partial[(long long)p * total + o];
    a1 += partial[(long long)(p + 64) * total + o];
    a2 += partial[(long long)(p + 128) * total + o];
    a3 += partial[(long long)(p + 192) * total + o];
  }
  for (; p < S; p += 64) a0 += partial[(long long)p * total + o];
  const float v = wave_sum((a0 + a1) + (a2 + a3));
  if (lane == 0) slab_store(gw, gb, o, K, Kt, v * scale);
}

__global__ void __launch_bounds__(256) slab_reduce_thread_kernel(const float* __restrict__ partial,
                                                                 float* __restrict__ gw, float* __restrict__ gb,
                                                                 int N, int K, int Kt, int S, float scale) {
  const int total = N * Kt;
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= total) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int p = 0;
  for (; p + 3 < S; p += 4) {
    a0 += partial[(long long)p * total + o];
    a1 += partial[(long long)(p + 1) * total + o];
    a2 += partial[(long long)(p + 2) * total + o];
    a3 += partial[(long long)(p + 3) * total + o];
  }
  for (; p < S; ++p) a0 += partial[(long long)p * total + o];
  slab_store(gw, gb, o, K, Kt, ((a0 + a1) + (a2 + a3)) * scale);
}

hipError_t slab_reduce(const float* partial, float* gw, float* gb, int N, int K, int Kt, int S, float scale,
                       hipStream_t st) {
  const int total = N * Kt;
  if (S >= 32 && (long long)total * 64 <= (1ll << 24))
    hipLaunchKernelGGL(slab_reduce_wave_kernel, dim3(cdiv(total, 4)), dim3(256), 0, st, partial, gw, gb, N, K, Kt, S,
                       scale);
  else
    hipLaunchKernelGGL(slab_reduce_thread_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, partial, gw, gb, N, K, Kt,
                       S, scale);
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
  g.img_elems = round_up(g.Hp * g.Wp * C + 8, 8);  // +8: slack for the finite "padding column" reads
  return g;
}

static const size_t kLdsBudget = 64 * 1024;  // keeps >= 2 workgroups per CU (160 KiB LDS)

bool convpool_supported(int H, int W, int C, int KH, int KW, int pad, int N) {
  CPGeom g = make_geom(1, H, W, C, KH, KW, pad, N);
  if (g.OH <= 0 || g.OW <= 0 || (g.OH & 1) || (g.OW & 1)) return false;
  if (C > 16 || N > 32 || KH > 7 || KW > 7) return false;
  if (g.Kpad / 32 > 16) return false;                     // fwd weight fragments in registers
  if ((g.K + 15) / 16 > 12) return false;                 // wgrad accumulators
  if (round_up(KH * KW * N, 32) / 32 > 16) return false;  // dgrad weight fragments
  const int P = KH - 1 - pad;
  if (P < 0) return false;
  const size_t q_elems = (size_t)(g.OH + 2 * P) * (g.OW + 2 * P) * N;
  if ((size_t)g.img_elems * 2 > kLdsBudget / 2 || q_elems * 2 > kLdsBudget / 2) return false;
  return true;
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// Persistent grid: `wg_per_cu` workgroups per CU, each looping over groups of `imgs` images; the
// per-workgroup setup (tables, weights in registers) is paid once per workgroup, not per group.
static int pick_imgs(int B, size_t fixed, size_t per_img, int wg_per_cu, int* grid) {
  const size_t budget = (160 * 1024) / wg_per_cu;
  int fit = (int)max((size_t)1, (budget > fixed ? budget - fixed : 0) / per_img);
  fit = min(fit, 32);
  const int wg = num_cus() * wg_per_cu;
  int imgs = min(fit, max(1, cdiv(B, wg)));
  *grid = min(wg, cdiv(B, imgs));
  return imgs;
}

template <int NT, int NKMAX>
static void launch_cp_fwd(const CPGeom& g, int grid, size_t lds, const void* x, int x_u8, const long long* idx,
                          long long nrows, float scale, const bf16* w, const float* bias, bf16* p, uint8_t* code,
                          hipStream_t st) {
  hipLaunchKernelGGL((convpool_fwd_kernel<NT, NKMAX>), dim3(grid), dim3(256), lds, st, g, x, x_u8, idx, nrows, scale,
                     w, bias, p, code);
}

hipError_t convpool_fwd(const void* x, int x_u8, const long long* idx, long long nrows, float scale, int B, int H,
                        int W, int C, int KH, int KW, int pad, int N, const bf16* w, const float* bias, bf16* p,
                        uint8_t* code, hipStream_t st) {
  if (!convpool_supported(H, W, C, KH, KW, pad, N)) return hipErrorInvalidValue;
  CPGeom g = make_geom(B, H, W, C, KH, KW, pad, N);
  const int tpi = cdiv(g.PH * g.PW, 4);
  const size_t fixed = round_up((round_up(tpi * 16, 4) + g.Kpad) * 4, 16);
  int grid = 0;
  g.imgs = pick_imgs(B, fixed, (size_t)g.img_elems * 2, 4, &grid);
  const size_t lds = fixed + (size_t)g.imgs * g.img_elems * 2;
  const int nk = g.Kpad / 32;
  const int nt = cdiv(N, 16);
  if (nt == 1) {
    if (nk <= 1) launch_cp_fwd<1, 1>(g, grid, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else if (nk <= 2) launch_cp_fwd<1, 2>(g, grid, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else if (nk <= 5) launch_cp_fwd<1, 5>(g, grid, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else if (nk <= 8) launch_cp_fwd<1, 8>(g, grid, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else launch_cp_fwd<1, 16>(g, grid, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
  } else {
    if (nk <= 2) launch_cp_fwd<2, 2>(g, grid, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else if (nk <= 8) launch_cp_fwd<2, 8>(g, grid, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
    else launch_cp_fwd<2, 16>(g, grid, lds, x, x_u8, idx, nrows, scale, w, bias, p, code, st);
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
  const int KT = cdiv(g.K, 16);
  const int NT = cdiv(N, 16);
  const int npool = g.PH * g.PW;
  const int cpi = cdiv(npool, 8);
  const size_t fixed = round_up((cpi * 32 + KT * 16) * 4, 16) + 128;
  const size_t per_img = (size_t)g.img_elems * 2 + (size_t)npool * N * 3 + 32;
  int grid = 0;
  g.imgs = pick_imgs(B, fixed, per_img, 2, &grid);
  while ((size_t)grid * N * Kt > ws_floats && grid > 1) grid /= 2;
  if ((size_t)grid * N * Kt > ws_floats) return hipErrorInvalidValue;
  size_t lds = fixed + round_up(g.imgs * g.img_elems * 2, 16) + round_up(g.imgs * npool * N * 2, 16) +
               round_up(g.imgs * npool * N, 16);
  const size_t red_bytes = (size_t)4 * NT * 16 * KT * 16 * 4;
  if (lds < red_bytes) lds = red_bytes;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (NT == 1) {
    if (KT <= 2) launch_cp_wgrad<1, 2>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
    else if (KT <= 4) launch_cp_wgrad<1, 4>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
    else if (KT <= 10) launch_cp_wgrad<1, 10>(g, lds, grid, x, x_u8, idx, nrows, scale, dp, code, workspace, st);
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
static void launch_cp_dgrad(const CPGeom& g, const CPDgrad& d, int grid, size_t lds, const bf16* dp,
                            const uint8_t* code, const bf16* wt, bf16* dx, hipStream_t st) {
  hipLaunchKernelGGL((convpool_dgrad_kernel<NT, NKMAX, VEC>), dim3(grid), dim3(256), lds, st, g, d, dp, code, wt, dx);
}

hipError_t convpool_dgrad(const bf16* dp, const uint8_t* code, const bf16* wt, bf16* dx, int B, int H, int W, int C,
                          int KH, int KW, int pad, int N, hipStream_t st) {
  if (!convpool_supported(H, W, C, KH, KW, pad, N)) return hipErrorInvalidValue;
  CPGeom g = make_geom(B, H, W, C, KH, KW, pad, N);
  CPDgrad d{};
  d.P = KH - 1 - pad;
  d.Hq = g.OH + 2 * d.P;
  d.Wq = g.OW + 2 * d.P;
  d.q_elems = round_up(d.Hq * d.Wq * N + 8, 8);
  d.K2 = KH * KW * N;
  d.K2pad = round_up(d.K2, 32);
  const int tpi = cdiv(H * W, 16);
  const size_t fixed = round_up((tpi * 16 + d.K2pad) * 4, 16);
  int grid = 0;
  g.imgs = pick_imgs(B, fixed, (size_t)d.q_elems * 2, 4, &grid);
  const size_t lds = fixed + (size_t)g.imgs * d.q_elems * 2;
  const int nk = d.K2pad / 32;
  const int nt = cdiv(C, 16);
  const bool vec = N % 8 == 0;
  if (nt != 1) return hipErrorInvalidValue;
  if (vec) {
    if (nk <= 8) launch_cp_dgrad<1, 8, true>(g, d, grid, lds, dp, code, wt, dx, st);
    else if (nk <= 13) launch_cp_dgrad<1, 13, true>(g, d, grid, lds, dp, code, wt, dx, st);
    else launch_cp_dgrad<1, 16, true>(g, d, grid, lds, dp, code, wt, dx, st);
  } else {
    if (nk <= 8) launch_cp_dgrad<1, 8, false>(g, d, grid, lds, dp, code, wt, dx, st);
    else launch_cp_dgrad<1, 16, false>(g, d, grid, lds, dp, code, wt, dx, st);
  }
  return hipGetLastError();
}

}  // namespace dfa
