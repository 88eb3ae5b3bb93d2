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
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "diag.h"

#include <array>
#include <map>
#include <mutex>
#include <numeric>

namespace dfa {

struct CPGeom {
  int B, H, W, C, KH, KW, pad, N, OH, OW, PH, PW, K, Kpad;
  int Hp, Wp, img_elems;  // padded input image in LDS
  int imgs;               // images per workgroup
  // forward row-segment layout: k = ky*RLp + (kx*C + c); every 8-slot k group is 8 CONSECUTIVE
  // elements of one padded image row, read with one 16-byte LDS load from one of S shifted copies
  int Cp;                  // LDS channel stride of the forward image (>= C, zero-filled channels)
  int RLp, chunks, Kpad2;  // RLp = round8(KW*Cp), chunks = RLp/8, Kpad2 = round32(KH*RLp)
  int G, S, RowP, ystr, xs_img;  // G = gcd(C,8): copy ci is shifted by ci*G elements, S = 8/G copies
  int pair;                       // forward pair mode (N <= 8): cols 8-15 = pixel x+1 via shifted weights
  int wRLp, wKpad2;               // GLOBAL weight layout (row-segment, KW columns): round8(KW*Cp), row length
  unsigned long long* stamps;     // profiling aid: per-block s_memtime stamps [grid][32] (nullptr = off)
};

static unsigned long long* g_cp_stamps = nullptr;
void convpool_set_stamps(void* buf) { g_cp_stamps = reinterpret_cast<unsigned long long*>(buf); }

// Diagnostic phase stamps (cdna_hip_programming.md §7 "In-kernel stamps"): read SHARES, not lengths.
#define CP_STAMP(slot)                                                                    \
  do {                                                                                    \
    if (g.stamps) {                                                                       \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      unsigned long long t_;                                                              \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if (threadIdx.x == 0 && (slot) < 32) g.stamps[blockIdx.x * 32 + (slot)] = t_;     \
    }                                                                                     \
  } while (0)

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
                                             long long nrows, float scale, int b0, int nimg, int img_stride,
                                             int row_stride, int cp) {
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
    bf16* dst = xs + i * img_stride + (y + g.pad) * row_stride + g.pad * cp;
    for (int c = c0; c < WC; c += tpr) {
      const int d = cp == g.C ? c : (c / g.C) * cp + c % g.C;
      if (x_u8) {
        const uint8_t* src = reinterpret_cast<const uint8_t*>(x) + cp_clamp(idx[b0 + i], nrows) * HWC + y * WC;
        dst[d] = f2bf((float)src[c] * scale);
      } else {
        const bf16* src = reinterpret_cast<const bf16*>(x) + ((long long)(b0 + i) * HWC + y * WC);
        dst[d] = src[c];
      }
    }
  }
}

// ---- Register-staged copies.  A plain "for (e = tid; e < n; e += 256) lds[..] = global[..]" loop
// is a chain of dependent global-load latencies (one round trip per iteration).  Instead every thread
// owns up to CHM fixed chunks of 4 consecutive elements (positions relative to the group start are
// the same for every group, so the index math is done once per workgroup), issues ALL loads of a group
// back to back, then stores.  Requires W*C % 4 == 0 and 4-element-aligned sources (host checks).
template <int CHM>
struct ImgPlan {
  int img[CHM];    // image slot within the group, or a large sentinel
  int soff[CHM];   // element offset inside the source image
  int doff[CHM];   // element offset inside the LDS image slot
  int split[CHM];  // elements of the chunk before the next pixel (a chunk spans at most 2 pixels)
};

template <int CHM>
__device__ __forceinline__ void make_img_plan(ImgPlan<CHM>& pl, const CPGeom& g, int row_stride, int cp) {
  const int WC = g.W * g.C, cpr = WC / 4, cpi = g.H * cpr;
  const FDiv dcpi(cpi), dcpr(cpr), dC(g.C);
#pragma unroll
  for (int j = 0; j < CHM; ++j) {
    const int c = threadIdx.x + 256 * j;
    const int i = dcpi.div(c), r = c - i * cpi;
    const int y = dcpr.div(r), x4 = 4 * (r - y * cpr);
    const int px = dC.div(x4), ch = x4 - px * g.C;
    pl.img[j] = c < g.imgs * cpi ? i : (1 << 20);
    pl.soff[j] = y * WC + x4;
    pl.doff[j] = (y + g.pad) * row_stride + (g.pad + px) * cp + ch;
    pl.split[j] = cp == g.C ? 4 : g.C - ch;
  }
}

template <int CHM>
__device__ __forceinline__ void stage_plan(bf16* xs, int img_stride, const ImgPlan<CHM>& pl, const CPGeom& g,
                                           const void* x, int x_u8, const long long* idx, long long nrows,
                                           float scale, int b0, int nimg, int cp) {
  const long long HWC = (long long)g.H * g.W * g.C;
  const int gap = cp - g.C;
  // loads are unconditional (clamped image slot): a load under a branch makes hipcc wait vmcnt(0)
  // right after it, serialising the group's loads
  if (x_u8) {
    long long r[CHM];
#pragma unroll
    for (int j = 0; j < CHM; ++j) r[j] = idx[b0 + min(pl.img[j], nimg - 1)];
    uint32_t v[CHM];
#pragma unroll
    for (int j = 0; j < CHM; ++j)
      v[j] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(x) + cp_clamp(r[j], nrows) * HWC +
                                                pl.soff[j]);
#pragma unroll
    for (int j = 0; j < CHM; ++j)
      if (pl.img[j] < nimg) {
        bf16* d = xs + pl.img[j] * img_stride + pl.doff[j];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          d[k + (((pl.split[j] - k - 1) >> 31) & gap)] = f2bf((float)((v[j] >> (8 * k)) & 255u) * scale);
      }
  } else {
    uint2 v[CHM];
#pragma unroll
    for (int j = 0; j < CHM; ++j)
      v[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(x) + (b0 + min(pl.img[j], nimg - 1)) * HWC +
                                             pl.soff[j]);
#pragma unroll
    for (int j = 0; j < CHM; ++j)
      if (pl.img[j] < nimg) {
        uint16_t* d = reinterpret_cast<uint16_t*>(xs + pl.img[j] * img_stride + pl.doff[j]);
        const int sp = pl.split[j];
        d[0] = (uint16_t)(v[j].x & 0xffffu);
        d[1 + (((sp - 2) >> 31) & gap)] = (uint16_t)(v[j].x >> 16);
        d[2 + (((sp - 3) >> 31) & gap)] = (uint16_t)(v[j].y & 0xffffu);
        d[3 + (((sp - 4) >> 31) & gap)] = (uint16_t)(v[j].y >> 16);
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
// Forward.  LDS image layout per row y: S copies of the padded row, copy ci shifted left by sh = ci*G
// elements (copy[i] = row[i + sh]).  The 8 k-slots (kx*C + c = 8j..8j+7 of kernel row ky) of output
// pixel (oy, ox) are row[oy+ky][ox*C + 8j + e], e < 8 = copy_sh[(ox*C - sh) + 8j + e] with
// sh = (ox*C) & 7: 16-byte aligned, so each A fragment is ONE ds_read_b128 at
// pixel_base(tile, row) + koff(ky, j) — both table lookups.
//
// Latency, not issue, bounds these small convolutions, so every wave keeps U tiles in flight: all
// U*NK fragment loads are issued back to back (no data-dependent branches between them: NK is the
// exact k-step count or zero-padded), then the U*NK MFMAs, then the U epilogues.
template <int NK>
struct FwdU {
  static constexpr int value = NK <= 2 ? 4 : (NK <= 5 ? 2 : 1);
};

// PAIR (N <= 8): columns 0-7 = channels at pixel (oy, 2px), columns 8-15 = the same channels at
// (oy, 2px+1), through weights shifted by one kernel column; 16 rows = 8 windows x 2 rows, so one
// MFMA tile covers 8 pool windows and only even-x pixels are read.  The two halves of each window
// meet with one DPP row rotation by 8 lanes.
template <int NT, int NK, int CHM, bool PAIR>
__global__ void __launch_bounds__(256) convpool_fwd_kernel(CPGeom g, int vec, const void* x, int x_u8,
                                                           const long long* idx, long long nrows, float scale,
                                                           const bf16* __restrict__ w, const float* __restrict__ bias,
                                                           bf16* __restrict__ p, uint8_t* __restrict__ code) {
  constexpr int U = FwdU<NK>::value;
  constexpr int BT = 8;  // shifted-copy build tasks per thread held in registers
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int npool = g.PH * g.PW;
  constexpr int WPT = PAIR ? 8 : 4;           // pool windows per MFMA tile
  const int tpi = (npool + WPT - 1) / WPT;    // MFMA tiles per image
  const int gtiles = g.imgs * tpi;  // tiles per group
  int* ttab = reinterpret_cast<int*>(smem);                      // [gtiles*16] LDS offset of each tile row
  int2* wtab = reinterpret_cast<int2*>(ttab + gtiles * 16);      // [gtiles] (first pooled index, valid windows)
  bf16* xs = reinterpret_cast<bf16*>(smem + round_up(gtiles * 16 * 4 + gtiles * 8, 16));  // [imgs][Hp][S][RowP]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  CP_STAMP(0);

  // ---- once per workgroup: tables, zero-bordered image slots, register-resident weights
  const FDiv dtpi(tpi), dPW(g.PW), dG(g.G);
  for (int e = tid; e < gtiles * 16; e += 256) {
    const int T = e >> 4, row = e & 15;
    const int i = dtpi.div(T), tw = T - i * tpi;
    // plain: row = 4 windows x (dy, dx);  pair: row = 8 windows x dy at even x
    const int wg = PAIR ? tw * 8 + 2 * (row >> 2) + ((row & 3) >> 1) : tw * 4 + (row >> 2);
    const int dy = PAIR ? (row & 1) : ((row & 3) >> 1), dx = PAIR ? 0 : (row & 1);
    int v = i * g.xs_img;
    if (wg < npool) {
      const int py = dPW.div(wg), px = wg - py * g.PW;
      const int oy = 2 * py + dy, ox = 2 * px + dx;
      const int t0 = ox * g.Cp, sh = t0 & 7;
      v += oy * g.ystr + dG.div(sh) * g.RowP + (t0 - sh);
    }
    ttab[e] = v;
    if (row == 0) wtab[T] = make_int2(i * npool + tw * WPT, npool - tw * WPT);
  }
  lds_zero(xs, g.imgs * g.xs_img);
  const int nk = g.Kpad2 / 32;
  const int Npad = round_up(g.N, 16);
  bf16x8 bfr[NK][NT];
#pragma unroll
  for (int s = 0; s < NK; ++s)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = 16 * t + (lane & 15);
      if (s < nk && n < Npad)
        bfr[s][t] = *reinterpret_cast<const bf16x8*>(w + (long long)n * g.wKpad2 + 32 * s + 8 * (lane >> 4));
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) bfr[s][t][e] = (bf16)0.f;
    }
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = PAIR ? (lane & 7) : 16 * t + (lane & 15);
    bv[t] = (bias && n < g.N) ? bias[n] : 0.f;
  }
  int koff[NK];
  const FDiv dchunks(g.chunks);
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    const int q = 4 * s + (lane >> 4);  // 8-slot group of this lane in k-step s
    int v = 0;
    if (s < nk && q < g.KH * g.chunks) {
      const int ky = dchunks.div(q);
      v = ky * g.ystr + 8 * (q - ky * g.chunks);
    }
    koff[s] = v;
  }
  // shifted-copy build plan: task = (image, interior row, copy ci >= 1, 16-byte chunk); all offsets
  // are fixed per thread, so the per-group build is loads + stores only
  const int WC = g.Wp * g.Cp;
  const int cpr = g.RowP / 8;
  const int per_img = g.H * (g.S - 1) * cpr;
  int bsrc[BT], bdst[BT], blim[BT];
  const FDiv dpimg(max(per_img, 1)), dprow(max((g.S - 1) * cpr, 1)), dcpr(cpr);
#pragma unroll
  for (int j = 0; j < BT; ++j) {
    const int e = tid + 256 * j;
    const int i = dpimg.div(e);
    int r = e - i * per_img;
    const int y = dprow.div(r);
    r -= y * ((g.S - 1) * cpr);
    const int q8 = dcpr.div(r);
    const int ci = 1 + q8, c8 = 8 * (r - q8 * cpr), sh = ci * g.G;
    const int row = i * g.xs_img + (y + g.pad) * g.ystr;
    bsrc[j] = row + c8 + sh;
    bdst[j] = row + ci * g.RowP + c8;
    // chunks whose source starts past the row stay zero from lds_zero (never written); the others
    // read 8 elements unguarded (copy 0 has >= 8 zero elements of slack after the row)
    blim[j] = per_img > 0 && i < g.imgs && c8 + sh < WC ? e : (1 << 30);
  }
  __syncthreads();

  ImgPlan<CHM> plan;
  make_img_plan(plan, g, g.ystr, g.Cp);
  CP_STAMP(1);
  int grp = 0;
  // ---- persistent loop over groups of images
  for (int b0 = blockIdx.x * g.imgs; b0 < g.B; b0 += gridDim.x * g.imgs, ++grp) {
    const int nimg = min(g.imgs, g.B - b0);
    if (vec) {  // -> copy 0 of each row
      stage_plan(xs, g.xs_img, plan, g, x, x_u8, idx, nrows, scale, b0, nimg, g.Cp);
    } else {
      stage_images(xs, g, x, x_u8, idx, nrows, scale, b0, nimg, g.xs_img, g.ystr, g.Cp);
    }
    __syncthreads();
    CP_STAMP(2 + 3 * grp);
    if (g.S > 1) {  // shifted copies of the interior rows (border rows stay zero in every copy)
      const int lim_img = nimg * per_img;
#pragma unroll
      for (int j = 0; j < BT; ++j) {
        if (blim[j] < lim_img) {
          bf16x8 v;
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = xs[bsrc[j] + k];
          *reinterpret_cast<bf16x8*>(xs + bdst[j]) = v;
        }
      }
      for (int e = tid + 256 * BT; e < lim_img; e += 256) {  // beyond the register plan
        const int i = e / per_img;
        int r = e - i * per_img;
        const int y = r / ((g.S - 1) * cpr);
        r -= y * ((g.S - 1) * cpr);
        const int ci = 1 + r / cpr, c8 = 8 * (r - (r / cpr) * cpr), sh = ci * g.G;
        const bf16* src = xs + i * g.xs_img + (y + g.pad) * g.ystr;
        if (c8 + sh >= WC) continue;
        bf16x8 v;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = src[c8 + k + sh];
        *reinterpret_cast<bf16x8*>(xs + i * g.xs_img + (y + g.pad) * g.ystr + ci * g.RowP + c8) = v;
      }
      __syncthreads();
    }
    CP_STAMP(3 + 3 * grp);
    const int ntiles = nimg * tpi;
    bf16* pg = p + (long long)b0 * npool * g.N;
    uint8_t* cg = code ? code + (long long)b0 * npool * g.N : nullptr;
    for (int T0 = wid * U; T0 < ntiles; T0 += 4 * U) {
      int offs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) offs[u] = ttab[min(T0 + u, ntiles - 1) * 16 + (lane & 15)];
      bf16x8 a[U][NK];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int s = 0; s < NK; ++s) a[u][s] = *reinterpret_cast<const bf16x8*>(xs + offs[u] + koff[s]);
      f32x4 acc[U][NT];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < NK; ++s) acc[u][t] = mfma16x16x32(a[u][s], bfr[s][t], acc[u][t]);
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (T0 + u >= ntiles) break;
        const int2 wt = wtab[T0 + u];
        if (PAIR) {
          // lane (row group gq, column n): acc rows = windows 2gq, 2gq+1 x dy, at dx = set = n >> 3.
          // Each lane finishes window 2gq+set: own dx half + the partner's (lane ^ 8) half.
          const int n = lane & 15, set = n >> 3, ch = n & 7, gq = lane >> 4;
          const f32x4 a4 = acc[u][0];
          const float m0 = fmaxf(a4[0], a4[1]), m1 = fmaxf(a4[2], a4[3]);
          const int d0 = a4[1] > a4[0] ? 1 : 0, d1 = a4[3] > a4[2] ? 1 : 0;
          // send the half the partner needs (its window 2gq + (1-set)), receive ours
          const float sendm = set ? m0 : m1;
          const int sendd = set ? d0 : d1;
          const float pm = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(sendm), 0x128, 0xf, 0xf, false));
          const int pd = __builtin_amdgcn_mov_dpp(sendd, 0x128, 0xf, 0xf, false);
          const float mo = set ? m1 : m0;
          const int dd = set ? d1 : d0;
          // window max over (dy, dx); ties resolve to the lower (dy*2 + dx) like the plain kernel
          const int jo = dd * 2 + set, jp = pd * 2 + (1 - set);
          const bool take_p = pm > mo || (pm == mo && jp < jo);
          float m = take_p ? pm : mo;
          const int am = take_p ? jp : jo;
          const int wloc = 2 * gq + set;
          if (ch < g.N && wloc < wt.y) {
            m += bv[0];
            const int o = (wt.x + wloc) * g.N + ch;
            pg[o] = f2bf(fmaxf(m, 0.f));
            if (cg) cg[o] = (uint8_t)(am | (m > 0.f ? 4 : 0));
          }
          continue;
        }
        const int wl = lane >> 4;  // window of this lane's accumulator rows
        if (wl >= wt.y) continue;
        const int o = (wt.x + wl) * g.N;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int n = 16 * t + (lane & 15);
          if (n < g.N) {
            float m = acc[u][t][0];
            int am = 0;
#pragma unroll
            for (int r = 1; r < 4; ++r)
              if (acc[u][t][r] > m) { m = acc[u][t][r]; am = r; }
            m += bv[t];
            pg[o + n] = f2bf(fmaxf(m, 0.f));
            if (cg) cg[o + n] = (uint8_t)(am | (m > 0.f ? 4 : 0));
          }
        }
      }
    }
    CP_STAMP(4 + 3 * grp);
    __syncthreads();  // image slots are restaged by the next group
  }
  CP_STAMP(31);
}

// ------------------------------------------------------------------------------------------------
// Weight gradient through the pool: partial[block][n][k] (k < K), partial[block][n][K] = bias grad.
//   dW[n][k] = sum_pixels dConv[pixel][n] * im2col(X)[pixel][k]      (bias: column K of ones)
// Reduction slots of one lane are 8 CONSECUTIVE conv-output pixels of one row, so both MFMA operands
// are single aligned 16-byte LDS reads:
//   A = dConv^T: channel-planar LDS image [N][OHc][DWc], scattered from (dPooled, code) once per
//       group (the full-resolution gradient never reaches HBM);
//   B = im2col(X): channel-planar LDS image with KW x-shifted copies of every row,
//       [C][Hq][KW][RowQ], copy s = row shifted left by s, so column k = (ky, kx, c) of pixels
//       ox0..ox0+7 is copy kx of row oy+ky at ox0 (ox0 a multiple of 8).
// A chunk = (4/G) output rows x 8G columns (one row / 8 columns per 16-lane group).
struct CPWg {
  int G, R;                          // lane-group split: chunk = R = 4/G rows x 8G cols
  int OHc, OWc, cpr, cpc, cpi;       // chunk-aligned output extent, chunk rows/cols, chunks per image
  int Hq, RowQ, ystr, cstr, xs_img;  // X image [C][Hq][KW][RowQ] (+pads)
  int DWc, dcs, dc_img;              // dConv image [N+1][OHc][DWc] (+pad; plane N stays zero), dc_img = (N+1)*dcs
  int build_per_img;                 // shifted-copy build tasks per image
};

template <int KT>
struct WgU {
  static constexpr int value = KT <= 2 ? 4 : (KT <= 5 ? 2 : 1);
};

template <int NT, int KTMAX, int CHM>
__global__ void __launch_bounds__(256) convpool_wgrad_kernel(CPGeom g, CPWg q, int vec, const void* x, int x_u8,
                                                             const long long* idx, long long nrows, float scale,
                                                             const bf16* __restrict__ dp,
                                                             const uint8_t* __restrict__ code,
                                                             float* __restrict__ partial) {
  constexpr int U = WgU<KTMAX>::value;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Kt = g.K + 1;
  const int KT = (Kt + 15) / 16;  // k-tiles incl. the bias column
  const int npool = g.PH * g.PW;
  const int wn = npool * g.N;      // pooled elements per image
  const int gch = g.imgs * q.cpi;  // chunks per group
  int2* ctab = reinterpret_cast<int2*>(smem);                                   // [gch] (X base, dConv base)
  bf16* xs = reinterpret_cast<bf16*>(smem + round_up(gch * 8, 16));             // [imgs][xs_img]
  bf16* dc = xs + g.imgs * q.xs_img;                                            // [imgs][dc_img]
  float* red = reinterpret_cast<float*>(smem);  // aliases all of the above after the main loop

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  CP_STAMP(0);
  const FDiv dcpi(q.cpi), dcpc(q.cpc);
  for (int c = tid; c < gch; c += 256) {
    const int i = dcpi.div(c), r = c - i * q.cpi;
    const int rc = dcpc.div(r), cc = r - rc * q.cpc;
    ctab[c] = make_int2(i * q.xs_img + rc * q.R * q.ystr + cc * 8 * q.G,
                        i * q.dc_img + rc * q.R * q.DWc + cc * 8 * q.G);
  }
  lds_zero(xs, g.imgs * (q.xs_img + q.dc_img));
  // per-lane constants: 16-lane group h -> (row hr, 8-column block hx) inside a chunk
  const int h = lane >> 4, hr = h / q.G, hx = h - hr * q.G;
  const int xlane = hr * q.ystr + hx * 8;
  const int dlane = hr * q.DWc + hx * 8;
  int aoff[NT];  // channel plane of this lane's A row (rows >= N read the image's zero plane N)
#pragma unroll
  for (int t = 0; t < NT; ++t) aoff[t] = min(16 * t + (lane & 15), g.N) * q.dcs + dlane;
  int koff[KTMAX];  // B column k = (ky*KW + kx)*C + c -> copy kx of channel c, row +ky
  bool bias_col = false, zero_col = false;
  const FDiv dC(g.C), dKW(g.KW);
#pragma unroll
  for (int t = 0; t < KTMAX; ++t) {
    const int k = 16 * t + (lane & 15);
    int v = 0;
    if (t < KT && k < g.K) {
      const int tt = dC.div(k), c = k - tt * g.C, ky = dKW.div(tt), kx = tt - ky * g.KW;
      v = c * q.cstr + ky * q.ystr + kx * q.RowQ;
    }
    koff[t] = v;
    if (t == KT - 1) {
      bias_col = k == g.K;
      zero_col = k > g.K;
    }
  }
  // X staging plan: NHWC source chunk of 4 elements -> channel-planar copy-0 positions.  dst of
  // element k = sbase + k*cstr (channel steps), minus (C*cstr - 1) once the chunk crosses into the
  // next pixel (k >= split); C == 1 chunks are 4 consecutive pixels.
  const int WC = g.W * g.C, cprw = WC / 4, cpimg = g.H * cprw;
  int sdst[CHM], ssplit[CHM], simg[CHM], ssrc[CHM];
  const FDiv dcpimg(cpimg), dcprw(cprw);
#pragma unroll
  for (int j = 0; j < CHM; ++j) {
    const int c = tid + 256 * j;
    const int i = dcpimg.div(c), r = c - i * cpimg;
    const int y = dcprw.div(r), e0 = 4 * (r - y * cprw);
    const int px = dC.div(e0), ch = e0 - px * g.C;
    simg[j] = c < g.imgs * cpimg ? i : (1 << 20);
    ssrc[j] = y * WC + e0;
    sdst[j] = i * q.xs_img + ch * q.cstr + (y + g.pad) * q.ystr + px + g.pad;
    ssplit[j] = g.C - ch;
  }
  const int cstep = g.C == 1 ? 1 : q.cstr;
  const int cwrap = g.C == 1 ? 0 : g.C * q.cstr - 1;
  // dConv scatter plan: 4-element chunks of a group's pooled gradient (wn % 4 == 0), offsets of
  // the windows' top-left pixel packed as 16-bit pairs (the dConv images of a group are < 64K elems)
  constexpr int PC = CHM;
  uint32_t sbase[PC][2];
  const FDiv dwn(wn), dN(g.N), dPW(g.PW);
#pragma unroll
  for (int j = 0; j < PC; ++j)
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      uint32_t v = 0;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int e = 4 * (tid + 256 * j) + 2 * k2 + hh;
        const int i = dwn.div(e), r = e - i * wn;
        const int wg = dN.div(r), n = r - wg * g.N;
        const int py = dPW.div(wg), px = wg - py * g.PW;
        // elements past the group's images point at image 0's zero plane (their writes are zeros)
        const uint32_t off = i < g.imgs ? (uint32_t)(i * q.dc_img + n * q.dcs + 2 * py * q.DWc + 2 * px)
                                        : (uint32_t)(g.N * q.dcs);
        v |= (off & 0xffffu) << (16 * hh);
      }
      sbase[j][k2] = v;
    }
  uint32_t cvr[PC];
  __syncthreads();

  f32x4 acc[NT][KTMAX];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int u = 0; u < KTMAX; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones, zeros;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ones[e] = (bf16)1.f;
    zeros[e] = (bf16)0.f;
  }
  CP_STAMP(1);
  // ---- software pipeline over groups: group g+1's global loads are issued right after group g's
  // data has been written to LDS, so their latency overlaps g's copy build and MFMA phase.  The
  // dataset row indices run one more group ahead (index -> row is a dependent load).
  const long long HWC = (long long)g.H * WC;
  const int gstride = gridDim.x * g.imgs;
  uint32_t cvn[PC];
  uint2 dvn[PC], xbn[CHM];
  uint32_t xvn[CHM];
  long long rown[CHM];
  // All loads below are UNconditional (clamped addresses): a load under a branch makes hipcc wait
  // vmcnt(0) right after it, serialising the whole group's loads.  Validity is applied at use.
  auto load_rows = [&](int b0n) {  // raw dataset row index per staging chunk of group b0n
    const int bl = min(b0n, g.B - 1);
    const int nl = min(g.imgs, g.B - bl);
#pragma unroll
    for (int j = 0; j < CHM; ++j) rown[j] = x_u8 ? idx[bl + min(simg[j], nl - 1)] : 0;
  };
  auto issue_loads = [&](int b0n) {
    const int nimg_n = min(g.imgs, g.B - b0n);
    const long long o0n = (long long)b0n * wn;
    const int nch_n = nimg_n * wn / 4;
#pragma unroll
    for (int j = 0; j < PC; ++j) {
      const int c = min(tid + 256 * j, nch_n - 1);
      cvn[j] = *reinterpret_cast<const uint32_t*>(code + o0n + 4 * c);
      dvn[j] = *reinterpret_cast<const uint2*>(dp + o0n + 4 * c);
    }
    if (vec) {
#pragma unroll
      for (int j = 0; j < CHM; ++j) {
        const int im = min(simg[j], nimg_n - 1);
        if (x_u8)
          xvn[j] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(x) +
                                                       cp_clamp(rown[j], nrows) * HWC + ssrc[j]);
        else
          xbn[j] = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(x) + (b0n + im) * HWC + ssrc[j]);
      }
    }
  };
  int grp = 0;
  {
    const int b0s = blockIdx.x * g.imgs;
    load_rows(b0s);
    if (b0s < g.B) issue_loads(b0s);
    load_rows(b0s + gstride);
  }
  for (int b0 = blockIdx.x * g.imgs; b0 < g.B; b0 += gstride, ++grp) {
    const int nimg = min(g.imgs, g.B - b0);
    const int nch = nimg * wn / 4;
    uint2 dv[PC];
#pragma unroll
    for (int j = 0; j < PC; ++j) {  // chunks past the group carry no gradient (code 0)
      cvr[j] = tid + 256 * j < nch ? cvn[j] : 0u;
      dv[j] = dvn[j];
    }
    if (vec) {
#pragma unroll
      for (int j = 0; j < CHM; ++j)
        if (simg[j] < nimg) {
          uint16_t* xs16 = reinterpret_cast<uint16_t*>(xs);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int d = sdst[j] + k * cstep - (((ssplit[j] - k - 1) >> 31) & cwrap);
            if (x_u8)
              xs[d] = f2bf((float)((xvn[j] >> (8 * k)) & 255u) * scale);
            else
              xs16[d] = (uint16_t)(((k < 2 ? xbn[j].x : xbn[j].y) >> (16 * (k & 1))) & 0xffffu);
          }
        }
    } else {
      // generic element path (unaligned sources)
      for (int e = tid; e < nimg * (int)HWC; e += 256) {
        const int i = e / (int)HWC, r = e - i * (int)HWC;
        const int y = r / WC, rr = r - y * WC, px = rr / g.C, ch = rr - px * g.C;
        float v;
        if (x_u8) {
          const long long row = cp_clamp(idx[b0 + i], nrows);
          v = (float)reinterpret_cast<const uint8_t*>(x)[row * HWC + r] * scale;
        } else {
          v = (float)reinterpret_cast<const bf16*>(x)[(long long)(b0 + i) * HWC + r];
        }
        xs[i * q.xs_img + ch * q.cstr + (y + g.pad) * q.ystr + px + g.pad] = f2bf(v);
      }
    }
    // ---- scatter the routed pooled gradient into the zero dConv image.  Branch-free: an element
    // whose window max was <= 0 (code bit 2 clear) writes 0 to its own window's pixel.
#pragma unroll
    for (int j = 0; j < PC; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t cd = (cvr[j] >> (8 * k)) & 255u;
        const uint32_t bits = ((k < 2 ? dv[j].x : dv[j].y) >> (16 * (k & 1))) & (0u - ((cd >> 2) & 1u));
        const uint32_t base = (sbase[j][k >> 1] >> (16 * (k & 1))) & 0xffffu;
        reinterpret_cast<uint16_t*>(dc)[base + ((cd >> 1) & 1) * q.DWc + (cd & 1)] = (uint16_t)(bits & 0xffffu);
      }
    if (grp == 1) CP_STAMP(20);
    // ---- prefetch: next group's loads (rows already known), then the row indices one further
    if (b0 + gstride < g.B) issue_loads(b0 + gstride);
    load_rows(b0 + 2 * gstride);
    if (grp == 1) CP_STAMP(21);
    __syncthreads();
    if (grp == 1) CP_STAMP(22);
    // ---- shifted copies of the staged rows (copy s = row shifted left by s elements)
    {
      auto build_chunk = [&](int src) {
        const uint4 lo = *reinterpret_cast<const uint4*>(xs + src);
        const uint4 hi = *reinterpret_cast<const uint4*>(xs + src + 8);
        const uint32_t d[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
        for (int sc = 1; sc < 8; ++sc) {
          if (sc < g.KW) {
            uint4 o;
            uint32_t* op = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
              const int w0 = m + sc / 2;
              op[m] = (sc & 1) ? __builtin_amdgcn_alignbyte(d[w0 + 1], d[w0], 2) : d[w0];
            }
            *reinterpret_cast<uint4*>(xs + src + sc * q.RowQ) = o;
          }
        }
      };
      // task = (image, channel, interior row, 8-column chunk c8): reads row[c8, c8+16) and writes
      // chunk c8 of every copy s = 1..KW-1
      const int lim = nimg * q.build_per_img;
      const int per_row = q.RowQ / 8, per_ch = g.H * per_row;
      const FDiv dimg(max(q.build_per_img, 1)), dch(per_ch), drow(per_row);
#pragma unroll 1
      for (int e = tid; e < lim; e += 256) {
        const int i = dimg.div(e);
        int r = e - i * q.build_per_img;
        const int ch = dch.div(r);
        r -= ch * per_ch;
        const int y = drow.div(r), c8 = 8 * (r - y * per_row);
        if (c8 < g.Wp) build_chunk(i * q.xs_img + ch * q.cstr + (y + g.pad) * q.ystr + c8);
      }
    }
    if (grp == 1) CP_STAMP(23);
    __syncthreads();
    CP_STAMP(2 + 2 * grp);
    // ---- MFMA: U chunks per wave iteration, every LDS read issued before the MFMAs
    const int nchunks = nimg * q.cpi;
    for (int C0 = wid * U; C0 < nchunks; C0 += 4 * U) {
      int2 cb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) cb[u] = ctab[min(C0 + u, nchunks - 1)];
      bf16x8 af[U][NT], bfv[U][KTMAX];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool live = C0 + u < nchunks;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(dc + cb[u].y + aoff[t]);
          af[u][t] = live ? v : zeros;
        }
#pragma unroll
        for (int t = 0; t < KTMAX; ++t) bfv[u][t] = *reinterpret_cast<const bf16x8*>(xs + cb[u].x + xlane + koff[t]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < KTMAX; ++t) {
          bf16x8 bb = bfv[u][t];
          if (t == KT - 1) bb = bias_col ? ones : (zero_col ? zeros : bb);
#pragma unroll
          for (int n = 0; n < NT; ++n) acc[n][t] = mfma16x16x32(af[u][n], bb, acc[n][t]);
        }
    }
    __syncthreads();
    // ---- restore the zero dConv image (same positions as the scatter)
#pragma unroll
    for (int j = 0; j < PC; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t cd = (cvr[j] >> (8 * k)) & 255u;
        dc[((sbase[j][k >> 1] >> (16 * (k & 1))) & 0xffffu) + ((cd >> 1) & 1) * q.DWc + (cd & 1)] = (bf16)0.f;
      }
    __syncthreads();  // clean dConv image before the next group's scatter
    CP_STAMP(3 + 2 * grp);
  }
  CP_STAMP(30);
  __syncthreads();  // everything staged is dead now; reuse LDS for the cross-wave reduction
  const int RW = KT * 16;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int u = 0; u < KTMAX; ++u) {
      if (u < KT) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * t + 4 * (lane >> 4) + r;
          const int k = 16 * u + (lane & 15);
          red[(wid * NT * 16 + n) * RW + k] = acc[t][u][r];
        }
      }
    }
  __syncthreads();
  float* out = partial + (long long)blockIdx.x * g.N * Kt;
  for (int e = tid; e < g.N * Kt; e += 256) {
    const int n = e / Kt, k = e - (e / Kt) * Kt;
    float sum = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) sum += red[(ww * NT * 16 + n) * RW + k];
    out[e] = sum;
  }
  CP_STAMP(31);
}

// ------------------------------------------------------------------------------------------------
// Data gradient through the pool: dx[b][iy][ix][c] = sum_{ky,kx,n} dConv[iy+pad-ky][ix+pad-kx][n] W[n][ky][kx][c]
struct CPDgrad {
  int Hq, Wq, q_elems, P;  // padded dConv image in LDS, P = KH-1-pad
  int K2, K2pad;           // K2 = KH*KW*N  (pair: KH*(KW+1)*N)
  int Nq;                  // LDS pixel stride (>= N): 16-byte reads of 8 consecutive pixels hit distinct banks
  int pair;                // C <= 8, W even: MFMA rows = pixel pairs, columns 8-15 = pixel x+1 (shifted weights)
};

// dgrad weight layouts (emitted by the optimizer, csrc/optim.hip):
//  plain: [Cpad16][round32(KH*KW*N)],   element (c, (ky*KW+kx)*N + n) = W[n][ky][kx][c]
//  pair:  [16][round32(KH*(KW+1)*N)],  patch tap (a, b) = (row, col) of the flipped kernel window:
//         row c   : col (a*(KW+1) + b)*N + n = W[n][KH-1-a][KW-1-b][c]    (b < KW)
//         row 8+c : col (a*(KW+1) + b)*N + n = W[n][KH-1-a][KW-b][c]      (b >= 1)
static CPGeom make_geom(int B, int H, int W, int C, int KH, int KW, int pad, int N);

static CPDgrad make_dgrad(const CPGeom& g) {
  CPDgrad d{};
  d.P = g.KH - 1 - g.pad;
  d.Hq = g.OH + 2 * d.P;
  d.Wq = g.OW + 2 * d.P;
  // pixel stride: a multiple of 8 elements with an odd number of 16-byte chunks, so 8 consecutive
  // pixels start in 8 different 16-byte bank groups
  d.Nq = g.N % 8 == 0 ? ((g.N / 8) % 2 == 1 ? g.N : g.N + 8) : g.N;
  d.q_elems = round_up(d.Hq * d.Wq * d.Nq + 8, 8);
  d.pair = (g.C <= 8 && g.W % 2 == 0 && g.N % 8 == 0) ? 1 : 0;
  d.K2 = g.KH * (g.KW + d.pair) * g.N;
  d.K2pad = round_up(d.K2, 32);
  return d;
}

void convpool_dgrad_layout(int H, int W, int C, int KH, int KW, int pad, int N, int* pair, int* K2pad) {
  CPGeom g = make_geom(1, H, W, C, KH, KW, pad, N);
  const CPDgrad d = make_dgrad(g);
  *pair = d.pair;
  *K2pad = d.K2pad;
}

template <int NT, int NKMAX, bool VEC, int CHM, bool PAIR>
__global__ void __launch_bounds__(256) convpool_dgrad_kernel(CPGeom g, CPDgrad d, const bf16* __restrict__ dp,
                                                             const uint8_t* __restrict__ code,
                                                             const bf16* __restrict__ wt, bf16* __restrict__ dx) {
  constexpr int U = NKMAX <= 4 ? 4 : (NKMAX <= 8 ? 2 : 1);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int HW = g.H * g.W;
  const int nrow = PAIR ? HW / 2 : HW;  // MFMA rows per image: pixels, or pixel pairs (x even, x+1)
  const int tpi = (nrow + 15) / 16;
  const int gtiles = g.imgs * tpi;
  int* ttab = reinterpret_cast<int*>(smem);             // [gtiles*16] input pixel -> qs offset
  int2* otab = reinterpret_cast<int2*>(ttab + gtiles * 16);  // [gtiles] (first output pixel, valid pixels)
  int* klut = reinterpret_cast<int*>(otab + gtiles);    // [K2pad]
  bf16* qs = reinterpret_cast<bf16*>(smem + round_up((gtiles * 18 + d.K2pad) * 4, 16));  // [imgs][Hq][Wq][N]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  CP_STAMP(0);
  const int npool = g.PH * g.PW;
  const FDiv dtpi(tpi), dW(PAIR ? g.W / 2 : g.W);
  for (int e = tid; e < gtiles * 16; e += 256) {
    const int T = e >> 4, i = dtpi.div(T), tw = T - i * tpi;
    const int px = tw * 16 + (e & 15);
    int v = i * d.q_elems;
    if (px < nrow) {
      const int iy = dW.div(px), ix = (px - iy * (PAIR ? g.W / 2 : g.W)) * (PAIR ? 2 : 1);
      v += (iy * d.Wq + ix) * d.Nq;
    }
    ttab[e] = v;
    if ((e & 15) == 0) otab[T] = make_int2(i * nrow + tw * 16, nrow - tw * 16);
  }
  const FDiv dNk(g.N), dKWk(PAIR ? g.KW + 1 : g.KW);
  for (int k = tid; k < d.K2pad; k += 256) {
    int v = 0;
    if (k < d.K2) {
      const int t = dNk.div(k), n = k - t * g.N, ky = dKWk.div(t), kx = t - ky * (PAIR ? g.KW + 1 : g.KW);
      // pair: k = (patch row a, patch col b, n) in patch order (the flip lives in the weights)
      v = PAIR ? (ky * d.Wq + kx) * d.Nq + n : ((g.KH - 1 - ky) * d.Wq + (g.KW - 1 - kx)) * d.Nq + n;
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
  // scatter plan (CHM > 0, wn % 4 == 0): this thread's fixed 4-element chunks of a group's pooled
  // gradient and the LDS position of each element's window origin; codes stay in registers so the
  // same positions are cleared again after the group
  constexpr int PC = CHM > 0 ? CHM : 1;
  int sbase[PC][4];
  if (CHM > 0) {
    const FDiv dwn(wn), dN(g.N), dPW(g.PW);
#pragma unroll
    for (int j = 0; j < PC; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = 4 * (tid + 256 * j) + k;
        const int i = dwn.div(e), r = e - i * wn;
        const int wg = dN.div(r), c = r - wg * g.N;
        const int py = dPW.div(wg), px = wg - py * g.PW;
        sbase[j][k] = i * d.q_elems + ((2 * py + d.P) * d.Wq + 2 * px + d.P) * d.Nq + c;
      }
  }
  const int rowq = d.Wq * d.Nq;
  uint32_t cv[PC];
  CP_STAMP(1);
  int grp = 0;
  for (int b0 = blockIdx.x * g.imgs; b0 < g.B; b0 += gridDim.x * g.imgs, ++grp) {
    const int nimg = min(g.imgs, g.B - b0);
    const long long o0 = (long long)b0 * wn;
    const int ntot = nimg * wn;
    if (CHM > 0) {
      const int nch = ntot / 4;
      uint2 dv[PC];
#pragma unroll
      for (int j = 0; j < PC; ++j) {  // unconditional (clamped) loads; validity applied at use
        const int c = min(tid + 256 * j, nch - 1);
        cv[j] = *reinterpret_cast<const uint32_t*>(code + o0 + 4 * c);
        dv[j] = *reinterpret_cast<const uint2*>(dp + o0 + 4 * c);
      }
#pragma unroll
      for (int j = 0; j < PC; ++j)
        if (tid + 256 * j >= nch) cv[j] = 0;
#pragma unroll
      for (int j = 0; j < PC; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t cd = (cv[j] >> (8 * k)) & 255u;
          if (cd & 4) {
            const uint32_t bits = (k < 2 ? dv[j].x : dv[j].y) >> (16 * (k & 1));
            reinterpret_cast<uint16_t*>(qs)[sbase[j][k] + ((cd >> 1) & 1) * rowq + (cd & 1) * d.Nq] =
                (uint16_t)(bits & 0xffffu);
          }
        }
    } else {
      // scatter the routed pooled gradient into the zero full-resolution dConv image
      for (int e = tid; e < ntot; e += 256) {
        const int cd = code[o0 + e];
        if (cd & 4) {
          const int i = e / wn;
          const int r = e - i * wn;
          const int wg = r / g.N, c = r - (r / g.N) * g.N;
          const int py = wg / g.PW, px = wg - (wg / g.PW) * g.PW;
          const int oy = 2 * py + ((cd & 3) >> 1), ox = 2 * px + (cd & 1);
          qs[i * d.q_elems + ((oy + d.P) * d.Wq + ox + d.P) * d.Nq + c] = dp[o0 + e];
        }
      }
    }
    __syncthreads();
    CP_STAMP(2 + 3 * grp);
    const int ntiles = nimg * tpi;
    bf16* xg = dx + (long long)b0 * HW * g.C;
    for (int T0 = wid * U; T0 < ntiles; T0 += 4 * U) {
      int offs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) offs[u] = ttab[min(T0 + u, ntiles - 1) * 16 + (lane & 15)];
      bf16x8 a[U][NKMAX];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int s = 0; s < NKMAX; ++s) {
          if (VEC) {
            a[u][s] = *reinterpret_cast<const bf16x8*>(qs + offs[u] + koff[s][0]);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) a[u][s][e] = qs[offs[u] + koff[s][VEC ? 0 : e]];
          }
        }
      f32x4 acc[U][NT];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < NKMAX; ++s) acc[u][t] = mfma16x16x32(a[u][s], bfr[s][t], acc[u][t]);
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (T0 + u >= ntiles) break;
        const int2 ot = otab[T0 + u];
        if (PAIR) {  // column n: pixel 2*pair + (n >> 3), channel n & 7
          const int c = lane & 7, set = (lane >> 3) & 1;
          if (c < g.C) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int mm = 4 * (lane >> 4) + r;
              if (mm < ot.y) xg[(long long)(2 * (ot.x + mm) + set) * g.C + c] = f2bf(acc[u][0][r]);
            }
          }
          continue;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int c = 16 * t + (lane & 15);
          if (c >= g.C) continue;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int mm = 4 * (lane >> 4) + r;
            if (mm < ot.y) xg[(long long)(ot.x + mm) * g.C + c] = f2bf(acc[u][t][r]);
          }
        }
      }
    }
    __syncthreads();
    CP_STAMP(3 + 3 * grp);
    // restore the zero image: clear exactly the positions scattered above
    if (CHM > 0) {
#pragma unroll
      for (int j = 0; j < PC; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t cd = (cv[j] >> (8 * k)) & 255u;
          if (cd & 4) qs[sbase[j][k] + ((cd >> 1) & 1) * rowq + (cd & 1) * d.Nq] = (bf16)0.f;
        }
    } else {
      for (int e = tid; e < ntot; e += 256) {
        const int cd = code[o0 + e];
        if (cd & 4) {
          const int i = e / wn;
          const int r = e - i * wn;
          const int wg = r / g.N, c = r - (r / g.N) * g.N;
          const int py = wg / g.PW, px = wg - (wg / g.PW) * g.PW;
          const int oy = 2 * py + ((cd & 3) >> 1), ox = 2 * px + (cd & 1);
          qs[i * d.q_elems + ((oy + d.P) * d.Wq + ox + d.P) * d.Nq + c] = (bf16)0.f;
        }
      }
    }
    __syncthreads();
    CP_STAMP(4 + 3 * grp);
  }
  CP_STAMP(31);
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

// Many slabs: a 1024-thread block owns 64 consecutive outputs (one per lane, so every slab row is a
// coalesced 256-byte read) and its 16 waves split the slabs, 8 loads in flight per lane; the 16 wave
// partials are combined in LDS in a fixed order.
__global__ void __launch_bounds__(1024) slab_reduce_wave_kernel(const float* __restrict__ partial,
                                                                float* __restrict__ gw, float* __restrict__ gb, int N,
                                                                int K, int Kt, int S, float scale) {
  __shared__ float red[16][64];
  const int total = N * Kt;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + lane;
  const int oc = min(o, total - 1);
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
  int p = wv;
  for (; p + 7 * 16 < S; p += 8 * 16) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += partial[(long long)(p + 16 * j) * total + oc];
  }
  for (; p < S; p += 16) a[0] += partial[(long long)p * total + oc];
  red[wv][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (wv == 0 && o < total) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) v += red[w][lane];
    slab_store(gw, gb, o, K, Kt, v * scale);
  }
}

__global__ void __launch_bounds__(256) slab_reduce_thread_kernel(const float* __restrict__ partial,
                                                                 float* __restrict__ gw, float* __restrict__ gb,
                                                                 int N, int K, int Kt, int S, float scale) {
  const int total = N * Kt;
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= total) return;
  // 16 slab loads in flight per thread (issued before any add; a launch of one workgroup per CU is
  // latency bound otherwise), summed into 4 accumulators in a fixed order: deterministic
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int p = 0;
  for (; p + 15 < S; p += 16) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = partial[(long long)(p + j) * total + o];
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      a0 += v[j];
      a1 += v[j + 1];
      a2 += v[j + 2];
      a3 += v[j + 3];
    }
  }
  for (; p + 3 < S; p += 4) {
    a0 += partial[(long long)p * total + o];
    a1 += partial[(long long)(p + 1) * total + o];
    a2 += partial[(long long)(p + 2) * total + o];
    a3 += partial[(long long)(p + 3) * total + o];
  }
  for (; p < S; ++p) a0 += partial[(long long)p * total + o];
  slab_store(gw, gb, o, K, Kt, ((a0 + a1) + (a2 + a3)) * scale);
}

// Several layers' slab reductions in ONE launch (deferred convpool weight gradients): workgroup b
// serves segment i for b in [block0_i, block0_{i+1}); same per-output fixed summation order as
// slab_reduce_wave_kernel, so the result is bit-identical to separate launches.
__global__ void __launch_bounds__(1024) slab_reduce_multi_kernel(SlabSegs segs) {
  __shared__ float red[16][64];
  int si = 0;
#pragma unroll
  for (int i = 1; i < kMaxSlabSegs; ++i)
    if (i < segs.n && (int)blockIdx.x >= segs.s[i].block0) si = i;
  const SlabSeg sg = segs.s[si];
  const int total = sg.N * sg.Kt;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int o = ((int)blockIdx.x - sg.block0) * 64 + lane;
  const int oc = min(o, total - 1);
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
  int p = wv;
  for (; p + 7 * 16 < sg.S; p += 8 * 16) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += sg.partial[(long long)(p + 16 * j) * total + oc];
  }
  for (; p < sg.S; p += 16) a[0] += sg.partial[(long long)p * total + oc];
  red[wv][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (wv == 0 && o < total) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) v += red[w][lane];
    slab_store(sg.gw, sg.gb, o, sg.K, sg.Kt, v * sg.scale);
  }
}

hipError_t slab_reduce_multi(SlabSegs segs, hipStream_t st) {
  if (segs.n <= 0 || segs.n > kMaxSlabSegs) return hipErrorInvalidValue;
  int blocks = 0;
  for (int i = 0; i < segs.n; ++i) {
    segs.s[i].block0 = blocks;
    blocks += cdiv(segs.s[i].N * segs.s[i].Kt, 64);
  }
  hipLaunchKernelGGL(slab_reduce_multi_kernel, dim3(blocks), dim3(1024), 0, st, segs);
  return hipGetLastError();
}

hipError_t slab_reduce(const float* partial, float* gw, float* gb, int N, int K, int Kt, int S, float scale,
                       hipStream_t st) {
  const int total = N * Kt;
  if (S >= 64 && total <= (1 << 16))
    hipLaunchKernelGGL(slab_reduce_wave_kernel, dim3(cdiv(total, 64)), dim3(1024), 0, st, partial, gw, gb, N, K, Kt,
                       S, scale);
  else
    hipLaunchKernelGGL(slab_reduce_thread_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, partial, gw, gb, N, K, Kt,
                       S, scale);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// host side
// ---- forward LDS layout choice.  Every A fragment is one ds_read_b128; 8 lanes (8 MFMA rows = two
// pool windows) issue together, so their 16-byte chunks should fall in distinct 128-byte bank
// windows.  The channel stride Cp (>= C), the row-copy length RowP and a per-row pad are chosen by
// simulating that bank mapping over all tiles of the image, scored by k-steps x conflict degree
// (x a small charge per shifted copy, which must be built per group).
struct FwdLayout {
  int Cp, RowP, ypad;
};

static void set_fwd_layout(CPGeom& g, int Cp, int RowP, int ypad) {
  g.Cp = Cp;
  g.RLp = round_up(g.KW * Cp, 8);
  g.chunks = g.RLp / 8;
  g.Kpad2 = round_up(g.KH * g.RLp, 32);
  g.G = std::gcd(Cp, 8);
  g.S = 8 / g.G;
  // furthest element a fragment read touches in a row copy: floor8((OW-1)*Cp) + RLp - 1
  const int maxel = ((g.OW - 1) * Cp) / 8 * 8 + g.RLp;
  // + 8: zero slack after the row so shifted-copy builds read whole 8-element windows unguarded
  const int minrow = round_up(max(g.Wp * Cp + 8, maxel), 8);
  g.RowP = max(RowP, minrow);
  g.ystr = g.S * g.RowP + ypad;
  g.xs_img = g.Hp * g.ystr;
}

// Pixel (padded-image origin) of MFMA row m of forward tile tw; false when the row is padding.
//  plain: rows = 4 windows x 4 pixels;  pair: rows = 8 windows x 2 dy at even x (odd x in cols 8-15)
static bool fwd_row_pixel(const CPGeom& g, bool pair, int tw, int m, int* oy, int* ox) {
  const int npool = g.PH * g.PW;
  int wg, dy, dx;
  if (pair) {
    wg = tw * 8 + 2 * (m >> 2) + ((m & 3) >> 1);
    dy = m & 1;
    dx = 0;
  } else {
    wg = tw * 4 + (m >> 2);
    dy = (m & 3) >> 1;
    dx = m & 1;
  }
  if (wg >= npool) return false;
  *oy = 2 * (wg / g.PW) + dy;
  *ox = 2 * (wg % g.PW) + dx;
  return true;
}

// Mean LDS cycles per A-fragment ds_read_b128 (1.0 = conflict free), from the ISA's lane grouping:
// 4 groups of 16 lanes {0-3,12-15,20-27} {4-11,16-19,28-31} {32-35,44-47,52-59} {36-43,48-51,60-63},
// bank = (addr/4) mod 64; each extra distinct 16-byte address on a busy slot adds a cycle.
static double fwd_conflicts(const CPGeom& g, bool pair) {
  static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                 {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                 {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  const int npool = g.PH * g.PW, wpt = pair ? 8 : 4, tpi = cdiv(npool, wpt);
  const int nk = g.Kpad2 / 32;
  double tot = 0.0;
  int cnt = 0;
  for (int tw = 0; tw < tpi; ++tw) {
    int base[16];
    for (int m = 0; m < 16; ++m) {
      int oy, ox;
      base[m] = 0;
      if (fwd_row_pixel(g, pair, tw, m, &oy, &ox)) {
        const int t0 = ox * g.Cp, sh = t0 & 7;
        base[m] = oy * g.ystr + (sh / g.G) * g.RowP + (t0 - sh);
      }
    }
    for (int sk = 0; sk < nk; ++sk) {
      for (int q = 0; q < 4; ++q) {
        int addr[16];
        for (int i = 0; i < 16; ++i) {
          const int l = grp[q][i], kq = 4 * sk + (l >> 4);
          int koff = 0;
          if (kq < g.KH * g.chunks) koff = (kq / g.chunks) * g.ystr + 8 * (kq % g.chunks);
          addr[i] = base[l & 15] + koff;  // element offset (16-byte aligned)
        }
        int worst = 1;
        for (int i = 0; i < 16; ++i) {
          int distinct = 0;
          for (int j = 0; j < 16; ++j) {
            if (((addr[j] / 8) & 15) != ((addr[i] / 8) & 15)) continue;
            bool seen = false;
            for (int k2 = 0; k2 < j; ++k2)
              if (addr[k2] == addr[j]) seen = true;
            if (!seen) ++distinct;
          }
          worst = max(worst, distinct);
        }
        tot += worst;
        ++cnt;
      }
    }
  }
  return cnt ? tot / cnt : 1.0;
}

// pair mode (N <= 8): row segments cover KW+1 columns, only even-x pixels are read
static void set_fwd_pair_layout(CPGeom& g) {
  g.pair = 1;
  g.RLp = round_up((g.KW + 1) * g.Cp, 8);
  g.chunks = g.RLp / 8;
  g.Kpad2 = round_up(g.KH * g.RLp, 32);
  g.G = std::gcd(2 * g.Cp, 8);
  g.S = 8 / g.G;
  const int maxel = ((g.OW - 2) * g.Cp) / 8 * 8 + g.RLp;
  const int minrow = round_up(max(g.Wp * g.Cp + 8, maxel), 8);
  const int ypad = g.ystr - g.S * g.RowP;  // keep the row pad chosen for this layout
  g.RowP = max(g.RowP, minrow);
  g.ystr = g.S * g.RowP + max(ypad, 0);
  g.xs_img = g.Hp * g.ystr;
}

static const FwdLayout& choose_fwd_layout(const CPGeom& g0, bool pair) {
  static std::mutex mu;
  static std::map<std::array<int, 7>, FwdLayout> cache;
  const std::array<int, 7> key{g0.H, g0.W, g0.C, g0.KH, g0.KW, g0.pad, pair ? 1 : 0};
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  FwdLayout best{g0.C, 0, 0};
  double best_score = 1e30;
  for (int Cp : {g0.C, round_up(g0.C, 2), round_up(g0.C, 4), round_up(g0.C, 8)}) {
    CPGeom g = g0;
    set_fwd_layout(g, Cp, 0, 0);
    if (pair) set_fwd_pair_layout(g);
    if (g.Kpad2 / 32 > 16) continue;
    const int minrow = g.RowP;
    for (int rp = minrow; rp < minrow + 64; rp += 8)
      for (int yp = 0; yp < 64; yp += 8) {
        set_fwd_layout(g, Cp, rp, yp);
        if (pair) set_fwd_pair_layout(g);
        const double score =
            (g.Kpad2 / 32) * fwd_conflicts(g, pair) * (1.0 + 0.1 * (g.S - 1)) * (1.0 + 0.002 * g.xs_img / 64);
        if (score < best_score - 1e-9) {
          best_score = score;
          best = FwdLayout{Cp, rp, yp};
        }
      }
  }
  return cache.emplace(key, best).first->second;
}

static CPGeom make_geom(int B, int H, int W, int C, int KH, int KW, int pad, int N) {
  CPGeom g{};
  g.stamps = g_cp_stamps;
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
  set_fwd_layout(g, C, 0, 0);
  const bool pair = N <= 8 && g.OW >= 2;
  const FwdLayout& L = choose_fwd_layout(g, pair);
  set_fwd_layout(g, L.Cp, L.RowP, L.ypad);
  if (pair) set_fwd_pair_layout(g);
  g.wRLp = g.RLp;  // the compute copy is emitted by the optimizer in exactly the kernel's layout
  g.wKpad2 = g.Kpad2;
  return g;
}

static const size_t kLdsBudget = 64 * 1024;  // keeps >= 2 workgroups per CU (160 KiB LDS)
constexpr int kStageChunks = 4;              // register-staged 4-element chunks per thread and group

void convpool_fwd_layout(int H, int W, int C, int KH, int KW, int pad, int N, int* Cp, int* Kpad2, int* pair) {
  CPGeom g = make_geom(1, H, W, C, KH, KW, pad, N);
  *Cp = g.Cp;
  *Kpad2 = g.wKpad2;
  *pair = g.pair;
}

bool convpool_supported(int H, int W, int C, int KH, int KW, int pad, int N) {
  CPGeom g = make_geom(1, H, W, C, KH, KW, pad, N);
  if (g.OH <= 0 || g.OW <= 0 || (g.OH & 1) || (g.OW & 1)) return false;
  if ((g.PH * g.PW * N) % 4 != 0) return false;  // 4-element pooled-gradient chunks (wgrad scatter plan)
  if (g.PH * g.PW * N > kStageChunks * 1024) return false;  // one image's pooled gradient fits the plan
  if (C > 16 || N > 32 || KH > 7 || KW > 7) return false;
  if (g.Kpad2 / 32 > 16 || g.wKpad2 / 32 > 16) return false;  // fwd weight fragments in registers
  if ((g.K + 16) / 16 > 13) return false;                 // wgrad accumulators (incl. bias column)
  if (KH != KW) return false;  // dConv padding P = KH-1-pad is shared by both axes
  {
    const CPDgrad d = make_dgrad(g);
    if (d.K2pad / 32 > (d.pair ? 18 : 16)) return false;  // dgrad weight fragments in registers
  }
  const int P = KH - 1 - pad;
  if (P < 0) return false;
  const int Nq = N % 8 == 0 ? ((N / 8) % 2 == 1 ? N : N + 8) : N;
  const size_t q_elems = (size_t)(g.OH + 2 * P) * (g.OW + 2 * P) * Nq;
  if ((size_t)g.img_elems * 2 > kLdsBudget / 2 || q_elems * 2 > kLdsBudget / 2) return false;
  if ((size_t)g.xs_img * 2 > kLdsBudget / 2) return false;
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
// Persistent-grid sizing from the kernel's real occupancy: blocks/CU allowed by its registers picks
// the LDS budget per block (-> images per group), then the grid is exactly the resident block count
// at that LDS size, so every block starts in the first (and only) dispatch round.
static int blocks_per_cu(const void* kern, size_t lds) {
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_pair(kern, lds);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, lds) != hipSuccess || nb < 1) nb = 1;
  cache[key] = nb;
  return nb;
}

struct Sizing {
  int imgs, grid;
  size_t lds;
};

// Tuning overrides (measurement only, csrc/diag.h): cp_wpc caps workgroups per CU, cp_minimgs raises
// the images per group (fewer, longer-lived workgroups amortise the per-workgroup setup).

static Sizing size_persistent(const void* kern, int B, size_t fixed, size_t per_img, size_t min_lds, int cap) {
  static const int wpc_cap = max(1, diag_int("cp_wpc", 8));
  static const int min_imgs = max(1, diag_int("cp_minimgs", 1));
  const int wpc = min(wpc_cap, blocks_per_cu(kern, 0));
  const size_t budget = (160 * 1024) / wpc;
  int fit = (int)max((size_t)1, (budget > fixed ? budget - fixed : 0) / per_img);
  fit = max(1, min(fit, min(cap, 32)));
  Sizing z{};
  z.imgs = min(fit, max(min_imgs, cdiv(B, num_cus() * wpc)));
  z.lds = max(fixed + (size_t)z.imgs * per_img, min_lds);
  const int nb = blocks_per_cu(kern, z.lds);
  z.grid = min(num_cus() * nb, cdiv(B, z.imgs));
  return z;
}

template <int NT, int NK, bool PAIR = false>
static hipError_t launch_cp_fwd(CPGeom g, bool vec, const void* x, int x_u8, const long long* idx, long long nrows,
                                float scale, const bf16* w, const float* bias, bf16* p, uint8_t* code,
                                hipStream_t st) {
  auto kern = convpool_fwd_kernel<NT, NK, kStageChunks, PAIR>;
  const int tpi = cdiv(g.PH * g.PW, PAIR ? 8 : 4);
  const Sizing z = size_persistent(reinterpret_cast<const void*>(kern), g.B, 32,
                                   (size_t)tpi * (16 * 4 + 8) + (size_t)g.xs_img * 2, 0,
                                   kStageChunks * 256 * 4 / (g.H * g.W * g.C));
  g.imgs = z.imgs;
  hipLaunchKernelGGL(kern, dim3(z.grid), dim3(256), z.lds, st, g, (int)vec, x, x_u8, idx, nrows, scale, w, bias, p,
                     code);
  return hipGetLastError();
}

// 4-element vector staging applies when image rows are whole 4-element chunks and the source is aligned
static bool stage_vec_ok(const CPGeom& g, const void* x, int x_u8) {
  return (g.W * g.C) % 4 == 0 && g.H * g.W * g.C <= kStageChunks * 1024 && (g.Cp == g.C || g.C >= 2) &&
         (reinterpret_cast<uintptr_t>(x) % (x_u8 ? 4 : 8)) == 0;
}

hipError_t convpool_fwd(const void* x, int x_u8, const long long* idx, long long nrows, float scale, int B, int H,
                        int W, int C, int KH, int KW, int pad, int N, const bf16* w, const float* bias, bf16* p,
                        uint8_t* code, hipStream_t st) {
  if (!convpool_supported(H, W, C, KH, KW, pad, N)) return hipErrorInvalidValue;
  CPGeom g = make_geom(B, H, W, C, KH, KW, pad, N);
  const bool vec = stage_vec_ok(g, x, x_u8);
  const int nk = g.Kpad2 / 32;
  const int nt = cdiv(N, 16);
#define CP_FWD(NT_, NK_) return launch_cp_fwd<NT_, NK_>(g, vec, x, x_u8, idx, nrows, scale, w, bias, p, code, st)
#define CP_FWDP(NK_) return launch_cp_fwd<1, NK_, true>(g, vec, x, x_u8, idx, nrows, scale, w, bias, p, code, st)
  if (g.pair) {
    if (nk <= 1) CP_FWDP(1);
    if (nk <= 2) CP_FWDP(2);
    if (nk <= 3) CP_FWDP(3);
    if (nk <= 4) CP_FWDP(4);
    if (nk <= 5) CP_FWDP(5);
    if (nk <= 7) CP_FWDP(7);
    if (nk <= 10) CP_FWDP(10);
    CP_FWDP(16);
  }
  if (nt == 1) {
    if (nk <= 1) CP_FWD(1, 1);
    if (nk <= 2) CP_FWD(1, 2);
    if (nk <= 3) CP_FWD(1, 3);
    if (nk <= 4) CP_FWD(1, 4);
    if (nk <= 5) CP_FWD(1, 5);
    if (nk <= 6) CP_FWD(1, 6);
    if (nk <= 7) CP_FWD(1, 7);
    if (nk <= 8) CP_FWD(1, 8);
    if (nk <= 10) CP_FWD(1, 10);
    if (nk <= 13) CP_FWD(1, 13);
    CP_FWD(1, 16);
  }
  if (nk <= 2) CP_FWD(2, 2);
  if (nk <= 4) CP_FWD(2, 4);
  if (nk <= 5) CP_FWD(2, 5);
  if (nk <= 7) CP_FWD(2, 7);
  if (nk <= 8) CP_FWD(2, 8);
  if (nk <= 13) CP_FWD(2, 13);
  CP_FWD(2, 16);
#undef CP_FWD
#undef CP_FWDP
}

static CPWg make_wg(const CPGeom& g) {
  CPWg q{};
  // lane-group split G (chunk = 4/G rows x 8G columns) minimising the padded pixel count
  int best = 1 << 30;
  for (int G : {1, 2, 4}) {
    const int R = 4 / G;
    const int n = cdiv(g.OH, R) * cdiv(g.OW, 8 * G);
    if (n < best) {
      best = n;
      q.G = G;
    }
  }
  q.R = 4 / q.G;
  q.OHc = round_up(g.OH, q.R);
  q.OWc = round_up(g.OW, 8 * q.G);
  q.cpr = q.OHc / q.R;
  q.cpc = q.OWc / (8 * q.G);
  q.cpi = q.cpr * q.cpc;
  // X copies: rows oy+ky < OHc+KH-1; reads ox0..ox0+7 < OWc; build slack: copy 0 keeps >= 8 zero
  // elements after the padded row.  Odd 16-byte counts spread copies / rows / channels over banks.
  auto odd16 = [](int elems) { return ((elems / 8) % 2 == 0) ? elems + 8 : elems; };
  q.Hq = max(q.OHc + g.KH - 1, g.Hp);
  q.RowQ = odd16(round_up(max(q.OWc, g.Wp + 8), 8));
  q.ystr = odd16(g.KW * q.RowQ);
  q.cstr = odd16(q.Hq * q.ystr);
  q.xs_img = g.C * q.cstr;
  q.DWc = odd16(q.OWc);
  q.dcs = odd16(q.OHc * q.DWc);
  q.dc_img = (g.N + 1) * q.dcs;
  q.build_per_img = g.KW > 1 ? g.C * g.H * (q.RowQ / 8) : 0;
  return q;
}

template <int NT, int KTMAX>
static hipError_t launch_cp_wgrad(CPGeom g, bool vec, const void* x, int x_u8, const long long* idx, long long nrows,
                                  float scale, const bf16* dp, const uint8_t* code, float* gw, float* gb,
                                  float* workspace, size_t ws_floats, hipStream_t st, int* deferred) {
  auto kern = convpool_wgrad_kernel<NT, KTMAX, kStageChunks>;
  const CPWg q = make_wg(g);
  const int Kt = g.K + 1;
  const int KT = cdiv(Kt, 16);
  const int wn = g.PH * g.PW * g.N;
  const size_t red_bytes = (size_t)4 * NT * 16 * KT * 16 * 4;
  // caps: register staging plans (image chunks, 2x pooled chunks per thread)
  int cap = min(kStageChunks * 256 * 4 / (g.H * g.W * g.C), kStageChunks * 256 * 4 / wn);
  cap = min(cap, 65535 / q.dc_img);  // scatter offsets are packed as 16 bits
  Sizing z = size_persistent(reinterpret_cast<const void*>(kern), g.B, 64,
                             (size_t)q.cpi * 8 + ((size_t)q.xs_img + q.dc_img) * 2 + 16, red_bytes, max(cap, 1));
  while ((size_t)z.grid * g.N * Kt > ws_floats && z.grid > 1) z.grid /= 2;
  if ((size_t)z.grid * g.N * Kt > ws_floats || z.lds > 160 * 1024) return hipErrorInvalidValue;
  g.imgs = z.imgs;
  hipLaunchKernelGGL(kern, dim3(z.grid), dim3(256), z.lds, st, g, q, (int)vec, x, x_u8, idx, nrows, scale, dp, code,
                     workspace);
  DFA_HIP_CHECK(hipGetLastError());
  if (deferred) {  // the caller batches this slab reduction with others (slab_reduce_multi)
    *deferred = z.grid;
    return hipSuccess;
  }
  return slab_reduce(workspace, gw, gb, g.N, g.K, Kt, z.grid, 1.f, st);
}

hipError_t convpool_wgrad(const void* x, int x_u8, const long long* idx, long long nrows, float scale, int B, int H,
                          int W, int C, int KH, int KW, int pad, int N, const bf16* dp, const uint8_t* code,
                          float* gw, float* gb, float* workspace, size_t ws_floats, hipStream_t st, int* deferred) {
  if (!convpool_supported(H, W, C, KH, KW, pad, N)) return hipErrorInvalidValue;
  CPGeom g = make_geom(B, H, W, C, KH, KW, pad, N);
  const int KT = cdiv(g.K + 1, 16);
  const int NT = cdiv(N, 16);
  const int npool = g.PH * g.PW;
  if (reinterpret_cast<uintptr_t>(dp) % 8 != 0 || reinterpret_cast<uintptr_t>(code) % 4 != 0)
    return hipErrorInvalidValue;  // pooled gradient / codes are read as 4-element chunks
  (void)npool;
  const bool vec = stage_vec_ok(g, x, x_u8);
#define CP_WG(NT_, KT_) \
  return launch_cp_wgrad<NT_, KT_>(g, vec, x, x_u8, idx, nrows, scale, dp, code, gw, gb, workspace, ws_floats, st, deferred)
  if (NT == 1) {
    if (KT <= 2) CP_WG(1, 2);
    if (KT <= 4) CP_WG(1, 4);
    if (KT <= 10) CP_WG(1, 10);
    CP_WG(1, 13);
  }
  if (KT <= 2) CP_WG(2, 2);
  if (KT <= 4) CP_WG(2, 4);
  CP_WG(2, 13);
#undef CP_WG
}

template <int NT, int NKMAX, bool VEC, bool PAIR = false>
static hipError_t launch_cp_dgrad(CPGeom g, const CPDgrad& d, bool plan, const bf16* dp, const uint8_t* code,
                                  const bf16* wt, bf16* dx, hipStream_t st) {
  auto kern = plan ? convpool_dgrad_kernel<NT, NKMAX, VEC, kStageChunks, PAIR>
                   : convpool_dgrad_kernel<NT, NKMAX, VEC, 0, PAIR>;
  const int tpi = cdiv(PAIR ? g.H * g.W / 2 : g.H * g.W, 16);
  const int wn = g.PH * g.PW * g.N;
  const Sizing z = size_persistent(reinterpret_cast<const void*>(kern), g.B, (size_t)d.K2pad * 4 + 32,
                                   (size_t)tpi * 72 + (size_t)d.q_elems * 2, 0, plan ? kStageChunks * 256 * 4 / wn : 32);
  g.imgs = z.imgs;
  hipLaunchKernelGGL(kern, dim3(z.grid), dim3(256), z.lds, st, g, d, dp, code, wt, dx);
  return hipGetLastError();
}

hipError_t convpool_dgrad(const bf16* dp, const uint8_t* code, const bf16* wt, bf16* dx, int B, int H, int W, int C,
                          int KH, int KW, int pad, int N, hipStream_t st) {
  if (!convpool_supported(H, W, C, KH, KW, pad, N)) return hipErrorInvalidValue;
  CPGeom g = make_geom(B, H, W, C, KH, KW, pad, N);
  const CPDgrad d = make_dgrad(g);
  const int wn = g.PH * g.PW * N;
  const bool plan = wn % 4 == 0 && wn <= kStageChunks * 1024 && reinterpret_cast<uintptr_t>(dp) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(code) % 4 == 0;
  const int nk = d.K2pad / 32;
  if (cdiv(C, 16) != 1) return hipErrorInvalidValue;
  if (d.pair) {
    if (nk <= 4) return launch_cp_dgrad<1, 4, true, true>(g, d, plan, dp, code, wt, dx, st);
    if (nk <= 8) return launch_cp_dgrad<1, 8, true, true>(g, d, plan, dp, code, wt, dx, st);
    if (nk <= 12) return launch_cp_dgrad<1, 12, true, true>(g, d, plan, dp, code, wt, dx, st);
    if (nk <= 15) return launch_cp_dgrad<1, 15, true, true>(g, d, plan, dp, code, wt, dx, st);
    return launch_cp_dgrad<1, 18, true, true>(g, d, plan, dp, code, wt, dx, st);
  }
  if (N % 8 == 0) {
    if (nk <= 2) return launch_cp_dgrad<1, 2, true>(g, d, plan, dp, code, wt, dx, st);
    if (nk <= 4) return launch_cp_dgrad<1, 4, true>(g, d, plan, dp, code, wt, dx, st);
    if (nk <= 5) return launch_cp_dgrad<1, 5, true>(g, d, plan, dp, code, wt, dx, st);
    if (nk <= 8) return launch_cp_dgrad<1, 8, true>(g, d, plan, dp, code, wt, dx, st);
    if (nk <= 10) return launch_cp_dgrad<1, 10, true>(g, d, plan, dp, code, wt, dx, st);
    if (nk <= 13) return launch_cp_dgrad<1, 13, true>(g, d, plan, dp, code, wt, dx, st);
    return launch_cp_dgrad<1, 16, true>(g, d, plan, dp, code, wt, dx, st);
  }
  if (nk <= 4) return launch_cp_dgrad<1, 4, false>(g, d, plan, dp, code, wt, dx, st);
  if (nk <= 8) return launch_cp_dgrad<1, 8, false>(g, d, plan, dp, code, wt, dx, st);
  return launch_cp_dgrad<1, 16, false>(g, d, plan, dp, code, wt, dx, st);
}

}  // namespace dfa
