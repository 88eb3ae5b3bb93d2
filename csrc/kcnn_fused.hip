// The reference CNN's convolution block in two launches per direction (gfx950 / MI355X).
//
// /root/reference/experiment/mnist/model.json: conv2d_1 (3x3x1 -> 32, ReLU) -> conv2d_2 (3x3x32 -> 32,
// ReLU) -> max_pooling2d_1 (2x2) [-> dropout_1, folded in].  Per-layer kernels move every activation
// through HBM (conv1's 26x26x32 output is 44 MB per 1024 images, written once and read three times) and
// run conv2 as short implicit GEMMs (K = 288) whose per-workgroup prologue/epilogue dominate.  Here a
// workgroup keeps one image at a time entirely in LDS:
//
//   kcnn_fwd  (persistent, 768 workgroups: 3 per CU)
//     x0 (uint8 dataset row through the batch index, or bf16)  -> LDS
//     conv1 + bias + ReLU on MFMA (9 taps zero-padded to k = 32)  -> X1 [676][32] bf16 in LDS (never in HBM)
//     conv2 on MFMA 16x16x32: one k-step per tap (32 channels), the 18 B fragments (9 taps x 2 channel
//     halves) stay in registers, A fragments are 16-byte LDS reads of X1.  Output pixels are taken
//     pool-window-major, so the four pixels of a 2x2 window are the four accumulator rows of one lane:
//     max-pool, argmax code, ReLU and the folded dropout happen in registers and only the pooled map
//     [144][32] and a 1-byte code per pooled element are written.
//   kcnn_bwd  (persistent)
//     x0 -> LDS, conv1 recomputed into X1 (cheaper than storing and re-reading it), the conv2 output
//     gradient dY2 [576][32] expanded in LDS from the pooled gradient and the codes (conv2 bias
//     gradient summed on the way), then
//       conv2 weight gradient  MFMA, D[n][(tap, ci)] over 18 pixel blocks of 32 per image; both operands
//                              come from ds_read_b64_tr_b16 (transposing 4-row blocks in the read);
//                              accumulators stay in registers across the workgroup's images
//       conv2 data gradient    MFMA, one k-step per tap (32 output channels) against the dgrad weight
//                              copy, x relu'(X1), rounded to bf16 as the per-layer path stores it, and
//       conv1 weight gradient  consumed in registers: 10 FMAs (9 taps + bias) per element against x0,
//                              so dX1 never exists in HBM either
//     each workgroup writes one slab of conv2 [32][289] and conv1 [32][10] partial sums
//   kcnn_reduce  sums the slabs in a fixed order (deterministic), writes the four gradients and
//     advances the dropout step counter (the last reader of the step's masks has run).
//
// The forward matches the per-layer path to bf16 rounding: conv1's 9-tap fp32 sums run in the MFMA's order
// (the per-layer kernel: a VALU FMA chain), conv2 has the same k order and the conv output is rounded to
// bf16 before the max exactly as it was stored; the weight gradients are the same sums in a different fp32
// order.  LDS in kcnn_bwd: 1.5 + 42.3 + 36 KB = 80 KB, two workgroups per CU.
#include "common.h"
#include "diag.h"
#include "kernels.h"

#include <algorithm>

namespace dfa {

namespace {

constexpr int KT = 256;
constexpr int H0 = 28, H1 = 26, H2 = 24, PW = 12, C = 32;
constexpr int NP0 = H0 * H0, NP1 = H1 * H1, NP2 = H2 * H2, NPP = PW * PW;  // 784, 676, 576, 144
constexpr int K2 = 9 * C;                                                   // 288
constexpr int S2 = K2 + 1, S1 = 10;  // slab row lengths: conv2 (288 + bias), conv1 (9 + bias)


typedef __bf16 bf16x4_vs __attribute__((__vector_size__(8)));

__device__ __forceinline__ bf16x4 tr_read(const bf16* p) {
  auto* lp = (__attribute__((address_space(3))) bf16*)(const_cast<bf16*>(p));
  const bf16x4_vs v =
      __builtin_amdgcn_ds_read_tr16_b64_v4bf16(reinterpret_cast<__attribute__((address_space(3))) bf16x4_vs*>(lp));
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    r[e] = a[e];
    r[e + 4] = b[e];
  }
  return r;
}
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// [pixel][32] bf16 LDS maps (X1 26x26, dY2 24x24) with the 16-byte chunk index XOR-swizzled by the
// pixel's image row: f(row) = 2 (row & 1) + ((row >> 1) & 1).  The transposed 4-row reads of the weight
// gradient (4 consecutive pixels of one row per 16-lane group, adjacent rows in the two groups of a
// half-wave) then hit disjoint bank halves, and the 16-byte reads of a 4x4 pixel tile spread over all
// 64 banks.  Since f depends on row & 3 only, the swizzle of a lane's pixel folds into constants when
// the tile origin row is a multiple of 4.
__device__ __forceinline__ int swf(int row) { return ((row & 1) << 1) | ((row >> 1) & 1); }
__device__ __forceinline__ int xsr(int pix, int row, int ch) {
  return pix * C + ((((ch >> 3) ^ swf(row))) << 3) + (ch & 7);
}

__device__ __forceinline__ long long src_row(const KcnnArgs& a, int b) {
  if (!a.idx) return b;
  long long r = a.idx[b];
  return r < 0 ? 0 : (r >= a.nrows ? a.nrows - 1 : r);
}

// x0 of image b as bf16 (the gather kernel's rounding: bf16(u8 * scale)), loaded one image ahead: the
// raw bytes / bf16 bits stay in registers and are converted only when stored (converting at load time
// made every load wait for its data right away, one memory latency per element, and the prefetch of
// the next image was no prefetch at all)
constexpr int X0_PER = (NP0 + KT - 1) / KT;  // 4 elements per thread
struct X0Regs {
  unsigned v[X0_PER];
};
__device__ __forceinline__ X0Regs load_x0(const KcnnArgs& a, int b) {
  X0Regs r;
  if (b >= a.B) return r;
  const long long row = src_row(a, b);
  if (a.x_u8) {
#pragma unroll
    for (int u = 0; u < X0_PER; ++u) r.v[u] = a.x_u8[row * NP0 + min((int)threadIdx.x + KT * u, NP0 - 1)];
  } else {
    const unsigned short* xb = reinterpret_cast<const unsigned short*>(a.x_bf);
#pragma unroll
    for (int u = 0; u < X0_PER; ++u) r.v[u] = xb[row * NP0 + min((int)threadIdx.x + KT * u, NP0 - 1)];
  }
  return r;
}
__device__ __forceinline__ void store_x0(const KcnnArgs& a, const X0Regs& r, bf16* x0) {
#pragma unroll
  for (int u = 0; u < X0_PER; ++u) {
    const int e = threadIdx.x + KT * u;
    float f;
    if (a.x_u8) f = (float)r.v[u] * a.scale;
    else {
      f = __builtin_bit_cast(float, r.v[u] << 16);  // bf16 bits -> fp32
      if (a.idx) f *= a.scale;
    }
    if (e < NP0) x0[e] = f2bf(f);
  }
}

// conv1 + bias + ReLU -> X1 (LDS) on MFMA: D[channel][pixel] = W1[channel][k] x0col[k][pixel] over 16-pixel
// tiles, k = the 9 taps (zero-padded to 32), two 16-channel tiles per pixel tile.  A (the weights) stays in
// registers; lane (G, i) supplies the taps 8G..8G+7 of pixel i as B; its D rows are channels 4G..4G+3 of
// pixel i, so the epilogue (fp32 bias, ReLU, bf16) ends in one 8-byte store per channel tile.  ~3x fewer
// instructions than the VALU FMA chains (the phase was VALU-bound); the products are exact in fp32 either
// way, only the order of the fp32 sum of the 9 taps differs (forward and backward recompute use this same
// code, so they agree bit for bit).
__device__ __forceinline__ void conv1_mfma_to_lds(const KcnnArgs& a, const bf16* x0, bf16* x1) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, G = lane >> 4, i = lane & 15;
  const unsigned short* x0u = reinterpret_cast<const unsigned short*>(x0);
  bf16x8 wa[2];
  float bias[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * G + e;
      wa[h][e] = k < 9 ? a.w1[(16 * h + i) * a.kpad1 + k] : (bf16)0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[h][r] = a.b1[16 * h + 4 * G + r];
  }
  // this lane's taps k = 8G + e as x0 offsets (clamped to tap 8 past the ninth; masked below)
  int toff[8];
  unsigned short keep[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = min(8 * G + e, 8);
    toff[e] = (k / 3) * H0 + (k - 3 * (k / 3));
    keep[e] = 8 * G + e < 9 ? 0xffffu : 0u;
  }
  // two pixel tiles per iteration (t, t + 4): all 16 tap reads go out before the first MFMA
  constexpr int NT = (NP1 + 15) / 16;  // 43
  for (int t0 = wid; t0 < NT; t0 += 8) {
    int pp[2], py[2];
    bf16x8 bx[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = 16 * (t0 + 4 * u) + i, pc = min(p, NP1 - 1);
      const int oy = pc / H1, ox = pc - oy * H1;
      pp[u] = p;
      py[u] = oy;
      const int base = oy * H0 + ox;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        bx[u][e] = __builtin_bit_cast(bf16, (unsigned short)(x0u[base + toff[e]] & keep[e]));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 d0 = mfma16x16x32(wa[0], bx[u], z);
      const f32x4 d1 = mfma16x16x32(wa[1], bx[u], z);
      if (pp[u] < NP1) {
        bf16x4 o0, o1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o0[r] = f2bf(fmaxf(d0[r] * 1.f + bias[0][r], 0.f));
          o1[r] = f2bf(fmaxf(d1[r] * 1.f + bias[1][r], 0.f));
        }
        *reinterpret_cast<bf16x4*>(x1 + xsr(pp[u], py[u], 4 * G)) = o0;
        *reinterpret_cast<bf16x4*>(x1 + xsr(pp[u], py[u], 16 + 4 * G)) = o1;
      }
    }
  }
}

__global__ void __launch_bounds__(KT, 3) kcnn_fwd_kernel(KcnnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 x0[NP0];
  __shared__ __attribute__((aligned(16))) bf16 x1[NP1 * C];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, G = lane >> 4, i = lane & 15;
  // conv2 B fragments: tap t, channel half h -> B[k = 8G..8G+7 of tap t][n = 16h + i]
  bf16x8 bw[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h) bw[t][h] = ld8(a.w2 + (16 * h + i) * K2 + t * C + 8 * G);
  const float bias2[2] = {a.b2[i], a.b2[16 + i]};
  const unsigned long long dseed = a.drop.on ? drop_seed(a.drop.seed, a.drop.step, a.drop.step_add) : 0ull;
  // this lane's A row in a tile of 4 windows: window j = i >> 2, position r = i & 3
  const int jw = i >> 2, rp = i & 3;
  X0Regs xr = load_x0(a, blockIdx.x);
  for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
    store_x0(a, xr, x0);
    xr = load_x0(a, b + gridDim.x);  // next image: in flight during this one
    __syncthreads();
    conv1_mfma_to_lds(a, x0, x1);
    __syncthreads();
    for (int t = wid; t < NPP / 4; t += 4) {
      const int q0 = 4 * t, ph = q0 / PW, pw0 = q0 - ph * PW;
      const int oy = 2 * ph + (rp >> 1), ox = 2 * (pw0 + jw) + (rp & 1);
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const bf16x8 af = ld8(x1 + xsr((oy + ky) * H1 + ox + kx, oy + ky, 8 * G));
          acc[0] = mfma16x16x32(af, bw[3 * ky + kx][0], acc[0]);
          acc[1] = mfma16x16x32(af, bw[3 * ky + kx][1], acc[1]);
        }
      // lane holds rows 4G..4G+3 = the four positions of window q0 + G, channel 16h + i
      const long long prow = (long long)b * NPP + q0 + G;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float m = -INFINITY;
        int cd = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = (float)f2bf(acc[h][r] * 1.f + bias2[h]);
          if (v > m) {
            m = v;
            cd = r;
          }
        }
        if (!(m > 0.f)) cd = 4;  // ReLU'd max is 0: no gradient
        float o = fmaxf(m, 0.f);
        const int n = 16 * h + i;
        if (a.drop.on) o = drop_keep(dseed, a.drop.thresh, prow * C + n) ? (float)f2bf(o) * a.drop.scale : 0.f;
        a.pooled[prow * C + n] = f2bf(o);
        a.code[prow * C + n] = (uint8_t)cd;
      }
    }
    __syncthreads();  // x0 / x1 are rewritten for the next image
  }
}

unsigned long long* g_kcnn_stamps = nullptr;

// per-phase clocks of the first two images of every workgroup (diagnostic; scripts/kcnnstamps.py)
#define KC_STAMP(slot)                                                               \
  do {                                                                               \
    if (a.stamps) {                                                                  \
      __builtin_amdgcn_sched_barrier(0);                                             \
      unsigned long long t_;                                                         \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");   \
      __builtin_amdgcn_sched_barrier(0);                                             \
      const int im_ = (b - (int)blockIdx.x) / (int)gridDim.x;                        \
      if (threadIdx.x == 0 && im_ < 2) a.stamps[(blockIdx.x * 2 + im_) * 16 + (slot)] = t_; \
    }                                                                                \
  } while (0)

__global__ void __launch_bounds__(KT, 2) kcnn_bwd_kernel(KcnnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 x0[NP0];
  __shared__ __attribute__((aligned(16))) bf16 x1[NP1 * C];
  __shared__ __attribute__((aligned(16))) bf16 dy2[NP2 * C];
  __shared__ __attribute__((aligned(16))) bf16 zc[8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, G = lane >> 4, i = lane & 15;
  if (tid < 8) zc[tid] = (bf16)0.f;
  // conv2 weight gradient: this wave's output channel half hn and input channel half hc, all 9 taps.  Its
  // accumulators live in registers only from the conv1 recompute of an image to the end of that image's
  // weight-gradient phase: stored into the workgroup's slab after it and reloaded (issued before the next
  // image's conv1 recompute) -- the same fp32 sums in the same order, and 36 registers free in the data
  // gradient phase, which holds its 72-register B operand (with them live there the dY2 reads of a tile
  // were serialised, one LDS round trip per tap)
  const int hn = wid & 1, hc = wid >> 1;
  float* s2 = a.slab2 + (long long)blockIdx.x * C * S2;
  float db2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) db2[j] = 0.f;
  f32x4 acc1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};  // conv1 D[ci = 16h + 4G + r][tap1 = i]
  const int c8 = tid & 3;  // this thread's 8-channel group in the dY2 expansion (256 % 4 == 0)

  X0Regs xr = load_x0(a, blockIdx.x);
  for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
    // ---- stage x0; expand dY2 from the pooled gradient and the codes (conv2 bias gradient on the way)
    KC_STAMP(0);
    store_x0(a, xr, x0);
    xr = load_x0(a, b + gridDim.x);
    for (int e = tid; e < NPP * 4; e += KT) {
      const int q = e >> 2;
      const long long o = ((long long)b * NPP + q) * C + 8 * c8;
      const bf16x8 gv = ld8(a.dyp + o);
      const uint2 cw = *reinterpret_cast<const uint2*>(a.code + o);
      const int ph = q / PW, pw = q - ph * PW;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        bf16x8 ov;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned cd = ((j < 4 ? cw.x : cw.y) >> (8 * (j & 3))) & 0xffu;
          ov[j] = cd == (unsigned)p ? gv[j] : (bf16)0.f;
          if (cd == (unsigned)p) db2[j] += (float)gv[j];
        }
        const int py = 2 * ph + (p >> 1);
        *reinterpret_cast<bf16x8*>(dy2 + xsr(py * H2 + 2 * pw + (p & 1), py, 8 * c8)) = ov;
      }
    }
    KC_STAMP(1);
    __syncthreads();
    KC_STAMP(2);
    f32x4 acc2[9];
    if (b == (int)blockIdx.x) {
#pragma unroll
      for (int t = 0; t < 9; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc2[t][r] = s2[(16 * hn + 4 * G + r) * S2 + t * C + 16 * hc + i];
    }
    conv1_mfma_to_lds(a, x0, x1);
    KC_STAMP(3);
    __syncthreads();
    KC_STAMP(4);

    // ---- conv2 weight gradient: D[n][(tap, ci)] += dY2^T[n][p] X1[p + tap][ci] over 18 blocks of 32 output
    // pixels, block = 4 rows x 8 columns: k slot 8G + 4hf + r is pixel (oy0 + G, ox0 + 4hf + r), so the
    // lane's addresses are a per-block uniform offset plus lane / tap constants
    {
      const int q = i >> 2, cq = 4 * (i & 3);
#pragma unroll 1
      for (int k0 = 0; k0 < NP2 / 32; ++k0) {
        const int oy0 = 4 * (k0 / 3), ox0 = 8 * (k0 % 3);
        bf16x8 af;
        {
          const int row = oy0 + G;
          const bf16x4 lo = tr_read(dy2 + xsr(row * H2 + ox0 + q, row, 16 * hn + cq));
          const bf16x4 hi = tr_read(dy2 + xsr(row * H2 + ox0 + 4 + q, row, 16 * hn + cq));
          af = cat8(lo, hi);
        }
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int row = oy0 + G + ky;
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const bf16x4 lo = tr_read(x1 + xsr(row * H1 + ox0 + q + kx, row, 16 * hc + cq));
            const bf16x4 hi = tr_read(x1 + xsr(row * H1 + ox0 + 4 + q + kx, row, 16 * hc + cq));
            acc2[3 * ky + kx] = mfma16x16x32(af, cat8(lo, hi), acc2[3 * ky + kx]);
          }
        }
      }
    }
    KC_STAMP(5);

    // ---- conv2 data gradient x relu'(X1) over 4x4 pixel tiles of X1 (7 x 7 tiles cover 26 x 26), and the
    // conv1 weight gradient on MFMA from pairs of tiles: D1[ci][tap1] += g[ci][pixel] x0[pixel + tap1]
    // (tap1 = 9 is the bias: a ones column).  A row i = pixel (4ty + i/4, 4tx + i%4); the dgrad D layout
    // puts pixels (4ty + G, 4tx + r) of channel 16h + i in lane (G, i), which is already the conv1 A
    // fragment of two tiles (k slot 8G + e: tile e / 4, column e % 4).
    {
      bf16x8 bt[9][2];  // B[k = (tap, n = 8G..8G+7)][ci = 16h + i] from the dgrad copy [ci][tap * 32 + n]
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h) bt[t][h] = ld8(a.w2t + (16 * h + i) * K2 + t * C + 8 * G);
      // (after the B loads: vmcnt counts stores too, and the first MFMA waits for the B operand)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) s2[(16 * hn + 4 * G + r) * S2 + t * C + 16 * hc + i] = acc2[t][r];
      KC_STAMP(6);
      // this lane's conv1 tap (column of the conv1 B operand; lanes i >= 9 read tap 0 and drop it)
      const int ty1 = i < 9 ? i / 3 : 0, tx1 = i < 9 ? i - 3 * (i / 3) : 0;
#pragma unroll 1
      for (int T0 = wid; T0 < 49; T0 += 8) {
        bf16x8 ag[2];  // conv1 A operand per channel half h: element 4u + r = the gradient of tile u, column r
        // the relu' mask and conv1 B operand reads are unconditional, at clamped (valid) addresses, and selected
        // afterwards: with the reads under their validity conditions (a short-circuit &&) the compiler built one
        // exec-mask branch per read, each waiting for its read -- 24 serialised LDS round trips per pair, half
        // of the kernel's time (scripts/kcnnstamps.py)
        // both tiles of the pair unconditionally (the second clamped to tile 48 and dropped when past the
        // last): their four MFMA accumulation chains interleave (a per-tile branch kept them apart)
        int py[2], px0[2], Tt[2], iy[2], ix[2];
        bool tl[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          tl[u] = T0 + 4 * u < 49;
          Tt[u] = min(T0 + 4 * u, 48);
          const int ty = Tt[u] / 7, tx = Tt[u] - 7 * (Tt[u] / 7);
          iy[u] = 4 * ty + (i >> 2);
          ix[u] = 4 * tx + (i & 3);
        }
        f32x4 acc[2][2];
        bf16x8 af[2][9];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          acc[u][0] = acc[u][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const int sy = iy[u] - ky, sx = ix[u] - kx;
              const bool ok = iy[u] < H1 && ix[u] < H1 && (unsigned)sy < (unsigned)H2 && (unsigned)sx < (unsigned)H2;
              af[u][3 * ky + kx] = ld8(ok ? dy2 + xsr(sy * H2 + sx, sy, 8 * G) : zc);
            }
        }
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            acc[u][0] = mfma16x16x32(af[u][t], bt[t][0], acc[u][0]);
            acc[u][1] = mfma16x16x32(af[u][t], bt[t][1], acc[u][1]);
          }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int ty = Tt[u] / 7, tx = Tt[u] - 7 * (Tt[u] / 7);
          const int ry = 4 * ty + G, cy = min(ry, H1 - 1);
          py[u] = cy;
          px0[u] = 4 * tx;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rx = 4 * tx + r, cx = min(rx, H1 - 1);
            const bool valid = tl[u] && ry < H1 && rx < H1;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float mv = (float)x1[xsr(cy * H1 + cx, cy, 16 * h + i)];
              const bool live = valid & (mv > 0.f);
              ag[h][4 * u + r] = live ? f2bf(acc[u][h][r]) : (bf16)0.f;
            }
          }
        }
        // conv1 B operand: B[8G + e][tap1 = i] = x0 at (pixel e) + tap1, 1 for the bias column
        bf16x8 bx;
        {
          // lanes i >= 9 read tap 0 too and mask it out with bit operations (a select let the compiler sink
          // the read into an exec-mask branch of the i < 9 lanes)
          const unsigned short keep = i < 9 ? 0xffffu : 0u, one = i == 9 ? 0x3f80u : 0u;  // bf16 1.0
          const unsigned short* x0u = reinterpret_cast<const unsigned short*>(x0);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int u = e >> 2;
            const int cx = min(px0[u] + (e & 3), H1 - 1);
            const unsigned short v = x0u[(py[u] + ty1) * H0 + cx + tx1];
            bx[e] = __builtin_bit_cast(bf16, (unsigned short)((v & keep) | one));
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) acc1[h] = mfma16x16x32(ag[h], bx, acc1[h]);
      }
    }
    KC_STAMP(7);
    __syncthreads();  // LDS is rewritten for the next image
    KC_STAMP(8);
  }

  // ---- per-workgroup slabs (conv2's weights: stored after every image's weight-gradient phase)
  float* s1 = a.slab1 + (long long)blockIdx.x * C * S1;
  // conv2 bias: threads sharing c8 (lane bits 0-1) -> xor over lane bits 2-5, then the 4 waves
  float* red = reinterpret_cast<float*>(x1);  // LDS reuse (after the final barrier)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = db2[j];
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane < 4) red[(wid * 4 + lane) * 8 + j] = v;
  }
  // conv1: lane (G, i) owns ci = 16h + 4G + r, tap1 = i (< 10); the 4 waves are summed below
  if (i < S1) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[128 + (wid * 32 + 16 * h + 4 * G + r) * 10 + i] = acc1[h][r];
  }
  __syncthreads();
  if (tid < C) {
    const int grp = tid >> 3, j = tid & 7;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * 4 + grp) * 8 + j];
    s2[tid * S2 + K2] = v;
  }
  for (int e = tid; e < C * S1; e += KT) {
    const int ci = e / S1, k = e - ci * S1;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[128 + (w * 32 + ci) * 10 + k];
    s1[e] = v;
  }
}

// Slabs -> gradients.  64 outputs per workgroup, the 16 waves each sum slabs w, w + 16, ... (fixed
// order), then a fixed-order combine in LDS.
__global__ void __launch_bounds__(1024) kcnn_reduce_kernel(const float* __restrict__ slab2,
                                                           const float* __restrict__ slab1, int nslab, float* g_w2,
                                                           float* g_b2, float* g_w1, float* g_b1,
                                                           long long* step_inc) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + lane;  // output index over [conv2 32 x 289][conv1 32 x 10]
  const int n2 = C * S2, n1 = C * S1;
  float s = 0.f;
  if (o < n2 + n1) {
    const float* src = o < n2 ? slab2 + o : slab1 + (o - n2);
    const long long stride = o < n2 ? n2 : n1;
    for (int q0 = wid; q0 < nslab; q0 += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = q0 + 16 * u;
        v[u] = q < nslab ? src[(long long)q * stride] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
  }
  part[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && o < n2 + n1) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) v += part[w][lane];
    if (o < n2) {
      const int n = o / S2, k = o - n * S2;
      if (k < K2) g_w2[n * K2 + k] = v;
      else g_b2[n] = v;
    } else {
      const int n = (o - n2) / S1, k = (o - n2) - n * S1;
      if (k < 9) g_w1[n * 9 + k] = v;
      else g_b1[n] = v;
    }
  }
  if (step_inc && blockIdx.x == 0 && threadIdx.x == 0) step_inc[0] += 1;
}

}  // namespace

void kcnn_set_stamps(void* buf) { g_kcnn_stamps = reinterpret_cast<unsigned long long*>(buf); }
int kcnn_blocks(int B) { return B < 512 ? B : 512; }
size_t kcnn_slab_floats(int B) { return (size_t)kcnn_blocks(B) * C * (S2 + S1); }

hipError_t kcnn_fwd(const KcnnArgs& a, hipStream_t st) {
  if (a.B <= 0 || (!a.x_u8 && !a.x_bf) || !a.w1 || !a.b1 || !a.w2 || !a.b2 || !a.pooled || !a.code || a.kpad1 < 9)
    return hipErrorInvalidValue;
  // 3 workgroups per CU fit (163 VGPRs, 44 KB of LDS): the forward is not reduced through per-workgroup slabs,
  // so its grid is free; DISTRIFLOW_DIAG=kcnn_fwd_wg=<n> sets it (default 768)
  static const int fwd_wg = diag_int("kcnn_fwd_wg", 768);
  hipLaunchKernelGGL(kcnn_fwd_kernel, dim3(std::min(a.B, std::max(1, fwd_wg))), dim3(KT), 0, st, a);
  return hipGetLastError();
}

hipError_t kcnn_bwd(const KcnnArgs& a, float* g_w1, float* g_b1, float* g_w2, float* g_b2, long long* step_inc,
                    hipStream_t st) {
  if (a.B <= 0 || (!a.x_u8 && !a.x_bf) || !a.w1 || !a.b1 || !a.w2t || !a.dyp || !a.code || !a.slab2 || !a.slab1 ||
      !g_w1 || !g_b1 || !g_w2 || !g_b2)
    return hipErrorInvalidValue;
  const int nb = kcnn_blocks(a.B);
  KcnnArgs ab = a;
  ab.stamps = g_kcnn_stamps;
  hipLaunchKernelGGL(kcnn_bwd_kernel, dim3(nb), dim3(KT), 0, st, ab);
  DFA_HIP_CHECK(hipGetLastError());
  const int outs = C * (S2 + S1);
  hipLaunchKernelGGL(kcnn_reduce_kernel, dim3(cdiv(outs, 64)), dim3(1024), 0, st, a.slab2, a.slab1, nb, g_w2, g_b2,
                     g_w1, g_b1, step_inc);
  return hipGetLastError();
}

}  // namespace dfa
