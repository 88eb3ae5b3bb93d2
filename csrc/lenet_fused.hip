// Whole-network LeNet-5 training step in three launches (gfx950 / MI355X).
//
// The reference trains its MNIST CNNs with one tf.js op per layer and per direction
// (DistributedTfModel.fit, /root/reference/src/common/models.ts:137-142).  The
// per-layer design of this repo (convpool.hip + mlphead.hip: 9 launches per step) left LeNet-5 at
// 0.174 ms per 4096-image step, ~60 us of it fixed per-launch cost and the rest VALU-bound im2col.
// LeNet-5 is small enough that a workgroup can keep EVERYTHING of its images on chip, so here:
//
//   lenet_prep_kernel    the conv weights of this step as ready-made MFMA B fragments (banded conv1,
//                        conv2 forward, pair-banded conv2 data gradient): 37 x 1 KB, read by every
//                        workgroup with one 16-byte load per lane and fragment
//   lenet_train_kernel   one workgroup = 8 images, 4 waves, ~78 KB of LDS (two workgroups per CU):
//     conv1 5x5 'same' + bias + ReLU + 2x2 max-pool   MFMA with a banded (Toeplitz) weight operand:
//                          A = 32 consecutive input pixels of a row (one aligned ds_read_b128; odd
//                          output columns read a copy of the image shifted by one pixel), so the
//                          4 accumulator rows of a lane are one 2x2 pool window: the pool is in-lane
//     conv2 5x5 + bias + ReLU + pool                  implicit GEMM, output rows in pool-window order
//     dense 400-120-84-10 + softmax-CE + backward     MFMA, weights streamed from L2
//     conv2 weight gradient                           ds_read_b64_tr_b16 transposed reads of both
//                          operands from their natural NHWC images; bias = a column of ones
//     conv2 data gradient                             pair-banded MFMA (two output columns per row)
//     conv1 weight gradient                           A fragments unpooled in registers from the pool
//                          gradient + argmax codes, B = 4 dword reads of the (shifted) input image
//   and writes per-workgroup conv gradient partials plus transposed dense activations/gradients;
//   lenet_reduce_kernel  deterministic reductions: conv partials (one wave per parameter over all
//                        workgroups), dense weight gradients over the batch (MFMA, K = batch), loss.
#include "common.h"
#include "diag.h"
#include "kernels.h"
#include "lenet_frag.h"
#include "ll_exchange.h"
#include "optim_device.h"
#include "ps_device.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace dfa {
namespace {

constexpr int IMG = 8;     // images per workgroup
constexpr int NT = 512;    // threads per workgroup: 8 waves, 2 workgroups per CU = 4 waves per SIMD
constexpr int NW = NT / 64;
constexpr int ccdiv(int a, int b) { return (a + b - 1) / b; }
// LDS carve (bytes), every offset 16-byte aligned
constexpr int XS_ELEMS = IMG * 1024 + 32;           // [8][32][32] padded input (+ tail pad)
constexpr int OFF_XS = 0;
constexpr int OFF_P1 = OFF_XS + XS_ELEMS * 2;       // [8][196][8] bf16 pool1 output, later its gradient
constexpr int OFF_C1 = OFF_P1 + IMG * 196 * 16;     // [8][196] u32 pool1 codes (3 bits per channel)
constexpr int OFF_K = OFF_C1 + IMG * 196 * 4;       // 64 B zeros, 32 B ones (bf16)
constexpr int OFF_FT = OFF_K + 128;                 // conv2 dgrad table [98][2][16] u8 (host-built)
constexpr int OFF_PX = OFF_FT + 98 * 2 * 16;        // conv2 output row -> P1 pixel [800] u16 (host-built)
constexpr int OFF_W = OFF_PX + 800 * 2;             // f32: b1 [6], b2 [16]
constexpr int OFF_U = OFF_W + 128;                  // phase-dependent union
constexpr int OFF_XS1 = OFF_U;                      // phases A and G: input shifted left by one pixel
constexpr int LD0 = 424, LD1 = 136, LD2 = 104, LD3 = 40;  // dense row strides (elements)
constexpr int OFF_H0 = OFF_U;
constexpr int OFF_H1 = OFF_H0 + IMG * LD0 * 2;
constexpr int OFF_H2 = OFF_H1 + IMG * LD1 * 2;
constexpr int OFF_Z3 = OFF_H2 + IMG * LD2 * 2;
constexpr int OFF_Z2 = OFF_Z3 + IMG * LD3 * 2;
constexpr int OFF_Z1 = OFF_Z2 + IMG * LD2 * 2;
constexpr int OFF_ZR = OFF_Z1 + IMG * LD1 * 2;      // zero row [LD0] (A rows 8..15 of every dense GEMM)
constexpr int OFF_LG = OFF_ZR + LD0 * 2;            // [8][16] f32 logits
constexpr int OFF_C2 = OFF_LG + IMG * 16 * 4;       // [8][25][16] u8 pool2 codes
constexpr int U_DENSE = OFF_C2 + IMG * 25 * 16 - OFF_U;
constexpr int OFF_DC2 = OFF_U;                      // [800][16] bf16 conv2 output gradient
constexpr int U_DC2 = 800 * 16 * 2;
constexpr int OFF_RED = OFF_U + XS_ELEMS * 2;       // [4][16][32] f32 cross-wave conv1 wgrad sums
constexpr int U_G = XS_ELEMS * 2 + 4 * 16 * 32 * 4;
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int LDS_BYTES = OFF_U + cmax(cmax(U_DENSE, U_DC2), U_G);
static_assert(OFF_U % 16 == 0 && OFF_H1 % 16 == 0 && OFF_ZR % 16 == 0 && OFF_C2 % 16 == 0 && OFF_RED % 16 == 0 &&
                  OFF_PX % 16 == 0 && OFF_W % 16 == 0,
              "LDS carve must stay 16-byte aligned");
static_assert(2 * LDS_BYTES <= 160 * 1024, "two workgroups per CU");

typedef __bf16 bf16x4_vs __attribute__((__vector_size__(8)));

// diagnostic per-phase clocks (scripts/lenetstamps.py): [grid][16] s_memtime after each phase's barrier
#define LN_STAMP(slot)                                                            \
  do {                                                                            \
    if (stamps) {                                                                 \
      __builtin_amdgcn_sched_barrier(0);                                          \
      unsigned long long t_;                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                          \
      if (threadIdx.x == 0) stamps[blockIdx.x * 16 + (slot)] = t_;                \
    }                                                                             \
  } while (0)

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
__device__ __forceinline__ void st8(bf16* p, const bf16x8& v) { *reinterpret_cast<bf16x8*>(p) = v; }
__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int e = 0; e < 8; ++e) z[e] = (bf16)0.f;
  return z;
}

// Xs1[e] = Xs[e + 1]: the padded images shifted left by one pixel (dword-aligned funnel shift)
__device__ __forceinline__ void build_shift1(const bf16* Xs, bf16* Xs1) {
  for (int t = threadIdx.x; t < XS_ELEMS / 8 - 1; t += NT) {
    const uint4 lo = *reinterpret_cast<const uint4*>(Xs + 8 * t);
    const unsigned nx = *reinterpret_cast<const unsigned*>(Xs + 8 * t + 8);
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(lo.y, lo.x, 2);
    o.y = __builtin_amdgcn_alignbyte(lo.z, lo.y, 2);
    o.z = __builtin_amdgcn_alignbyte(lo.w, lo.z, 2);
    o.w = __builtin_amdgcn_alignbyte(nx, lo.w, 2);
    *reinterpret_cast<uint4*>(Xs1 + 8 * t) = o;
  }
}

// 2x2 max-pool of one window (elements in (dy, dx) row-major order) + ReLU; code = argmax position
// (first maximum), 4 = inactive (no gradient flows: pooled value <= 0).
__device__ __forceinline__ void pool4(float a00, float a01, float a10, float a11, float& best, unsigned& code) {
  best = a00;
  code = 0;
  if (a01 > best) { best = a01; code = 1; }
  if (a10 > best) { best = a10; code = 2; }
  if (a11 > best) { best = a11; code = 3; }
  if (!(best > 0.f)) { best = 0.f; code = 4; }
}

// Weight fragments of one dense GEMM for the tiles t = w + NW tt this wave owns, loaded ahead of use so
// that the L2 latency of layer l + 1's weights hides behind layer l (W rows of 32 * KS elements).
template <int KS, int NTW>
struct DenseFrags {
  bf16x8 b[NTW][KS];
};
template <int KS, int NTW>
__device__ __forceinline__ void dense_load(DenseFrags<KS, NTW>& f, const bf16* __restrict__ W, int ntiles) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    const int t = w + NW * tt;
    if (t < ntiles) {
      const bf16* wrow = W + (long long)(16 * t + i) * (32 * KS) + 8 * g;
#pragma unroll
      for (int s = 0; s < KS; ++s) f.b[tt][s] = ld8(wrow + 32 * s);
    }
  }
}

// Z[8 rows][N] = A[8][Kpad] W^T (+bias, ReLU); A rows 8..15 of the MFMA tile read the zero row.
template <int KS, int NTW>
__device__ __forceinline__ void dense_fwd(const DenseFrags<KS, NTW>& f, const bf16* A, int lda, const bf16* zr,
                                          const float* __restrict__ bias, int N, bool relu, bf16* out, int ldo,
                                          float* out32, bf16* __restrict__ hT, int ldt, int r0, int rows) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  const int ntiles = (N + 15) / 16;
  const bf16* arow = (i < IMG ? A + i * lda : zr) + 8 * g;
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    const int t = w + NW * tt;
    if (t >= ntiles) break;
    const int n = 16 * t + i;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = mfma16x16x32(ld8(arow + 32 * s), f.b[tt][s], acc);
    if (g >= 2) continue;  // output rows 8..15 are padding
    const float bv = (bias != nullptr && n < N) ? bias[n] : 0.f;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = acc[r] + bv;
      if (relu) v[r] = fmaxf(v[r], 0.f);
      if (n >= N) v[r] = 0.f;
      const int row = 4 * g + r;
      if (out) out[row * ldo + n] = f2bf(v[r]);
      if (out32) out32[row * 16 + (n & 15)] = v[r];
    }
    if (hT != nullptr && n < N) {
      bf16* dst = hT + (long long)n * ldt + r0 + 4 * g;
      if (4 * g + 4 <= rows) {
        bf16x4 pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk[r] = f2bf(v[r]);
        *reinterpret_cast<bf16x4*>(dst) = pk;
      } else {
        for (int r = 0; r < 4; ++r)
          if (4 * g + r < rows) dst[r] = f2bf(v[r]);
      }
    }
  }
}

// dA[8][K] = dZ[8][32*KS] Wt^T, masked by (mask > 0); also dZ^T rows for the weight gradient.
template <int KS, int NTW>
__device__ __forceinline__ void dense_bwd(const DenseFrags<KS, NTW>& f, const bf16* dZ, int ldz, const bf16* zr,
                                          int K, const bf16* mask, int ldm, bf16* out, int ldo,
                                          bf16* __restrict__ gT, int ldt, int r0, int rows) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  const int ktiles = (K + 15) / 16;
  const bf16* zrow = (i < IMG ? dZ + i * ldz : zr) + 8 * g;
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    const int t = w + NW * tt;
    if (t >= ktiles) break;
    const int j = 16 * t + i;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = mfma16x16x32(ld8(zrow + 32 * s), f.b[tt][s], acc);
    if (g >= 2) continue;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * g + r;
      v[r] = acc[r];
      if (mask != nullptr && !((float)mask[row * ldm + j] > 0.f)) v[r] = 0.f;
      if (j >= K) v[r] = 0.f;
      out[row * ldo + j] = f2bf(v[r]);
    }
    if (gT != nullptr && j < K) {
      bf16* dst = gT + (long long)j * ldt + r0 + 4 * g;
      if (4 * g + 4 <= rows) {
        bf16x4 pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk[r] = f2bf(v[r]);
        *reinterpret_cast<bf16x4*>(dst) = pk;
      } else {
        for (int r = 0; r < 4; ++r)
          if (4 * g + r < rows) dst[r] = f2bf(v[r]);
      }
    }
  }
}

__global__ void __launch_bounds__(NT, 2 * NT / 256) lenet_train_kernel(LeNetArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Xs = reinterpret_cast<bf16*>(smem + OFF_XS);
  bf16* Xs1 = reinterpret_cast<bf16*>(smem + OFF_XS1);
  bf16* P1 = reinterpret_cast<bf16*>(smem + OFF_P1);
  unsigned* C1 = reinterpret_cast<unsigned*>(smem + OFF_C1);
  bf16* KZ = reinterpret_cast<bf16*>(smem + OFF_K);       // 32 zeros
  bf16* KO = KZ + 32;                                       // 16 ones
  unsigned char* FT = reinterpret_cast<unsigned char*>(smem + OFF_FT);
  unsigned short* PX = reinterpret_cast<unsigned short*>(smem + OFF_PX);
  float* WS = reinterpret_cast<float*>(smem + OFF_W);       // b1[6] b2[16]
  bf16* H0 = reinterpret_cast<bf16*>(smem + OFF_H0);
  bf16* H1 = reinterpret_cast<bf16*>(smem + OFF_H1);
  bf16* H2 = reinterpret_cast<bf16*>(smem + OFF_H2);
  bf16* Z3 = reinterpret_cast<bf16*>(smem + OFF_Z3);
  bf16* Z2 = reinterpret_cast<bf16*>(smem + OFF_Z2);
  bf16* Z1 = reinterpret_cast<bf16*>(smem + OFF_Z1);
  bf16* ZR = reinterpret_cast<bf16*>(smem + OFF_ZR);
  float* LG = reinterpret_cast<float*>(smem + OFF_LG);
  unsigned char* C2 = reinterpret_cast<unsigned char*>(smem + OFF_C2);
  bf16* DC2 = reinterpret_cast<bf16*>(smem + OFF_DC2);
  float* RED = reinterpret_cast<float*>(smem + OFF_RED);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * IMG;
  const int rows = min(IMG, a.B - r0);
  const long long nb = gridDim.x;
  const bf16x8* __restrict__ frag = reinterpret_cast<const bf16x8*>(a.frag);
  float* part = a.conv_part + blockIdx.x;  // this workgroup's partials: parameter p at part[p * part_ld]
  const long long pld = a.part_ld;
  unsigned long long* const stamps = a.stamps;
  LN_STAMP(0);

  // ---------------------------------------------------------------- phase 0: zero fills, staging
  // conv1 B fragments of this step (lenet_prep_kernel): in flight while the images load
  bf16x8 bc[15];
#pragma unroll
  for (int f = 0; f < 15; ++f) bc[f] = frag[(FR_C1 + f) * 64 + lane];
  const bf16x8 z8 = zero8();
  for (int e = tid; e < (OFF_K - OFF_XS) / 16; e += NT) st8(Xs + 8 * e, z8);  // Xs, P1 (pad channels), C1
  for (int e = tid; e < (LDS_BYTES - OFF_U) / 16; e += NT) st8(reinterpret_cast<bf16*>(smem + OFF_U) + 8 * e, z8);
  if (tid < 4) st8(KZ + 8 * tid, z8);
  if (tid < 2) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)1.f;
    st8(KO + 8 * tid, o);
  }
  if (tid < 6) WS[tid] = a.b1[tid];
  if (tid < 16) WS[6 + tid] = a.b2[tid];
  if (tid < 98 * 2) reinterpret_cast<uint4*>(FT)[tid] = reinterpret_cast<const uint4*>(a.ftab)[tid];
  if (tid < 100) reinterpret_cast<uint4*>(PX)[tid] = reinterpret_cast<const uint4*>(a.pxtab)[tid];
  __syncthreads();
  // input rows -> bf16, 2-pixel zero border ('same' padding)
  if (tid < IMG * 28) {
    const int img = tid / 28, y = tid - 28 * (tid / 28);
    if (img < rows) {
      long long src = a.idx ? a.idx[r0 + img] : (long long)(r0 + img);
      src = src < 0 ? 0 : (src >= a.nrows ? a.nrows - 1 : src);
      unsigned* dst = reinterpret_cast<unsigned*>(Xs + img * 1024 + (y + 2) * 32 + 2);
      if (a.x_u8 != nullptr) {
        const unsigned* p = reinterpret_cast<const unsigned*>(a.x_u8 + src * 784 + y * 28);
        unsigned v[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < 7; ++k)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const float f0 = (float)((v[k] >> (16 * h)) & 255u) * a.scale;
            const float f1 = (float)((v[k] >> (16 * h + 8)) & 255u) * a.scale;
            const unsigned lo = __builtin_bit_cast(unsigned short, f2bf(f0));
            const unsigned hi = __builtin_bit_cast(unsigned short, f2bf(f1));
            dst[2 * k + h] = lo | (hi << 16);
          }
      } else {
        const uint2* p = reinterpret_cast<const uint2*>(a.x_bf + src * 784 + y * 28);
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          const uint2 v = p[k];
          dst[2 * k] = v.x;
          dst[2 * k + 1] = v.y;
        }
      }
    }
  }
  __syncthreads();
  build_shift1(Xs, Xs1);
  __syncthreads();
  LN_STAMP(1);

  // ---------------------------------------------------------------- phase A: conv1 + ReLU + pool
  // rows m = (image, y, parity): A = row y of the image (parity 1: shifted by one pixel) from column
  // x0; column j of channel-pair tile T = output x = x0 + 2 (j & 7) + parity, channel 2T + (j >> 3).
  // A lane's 4 accumulator rows (y, y+1) x (parity 0, 1) are one 2x2 pool window.
  {
    const float b1c[3] = {WS[(i >> 3)], WS[2 + (i >> 3)], WS[4 + (i >> 3)]};
#pragma unroll 2
    for (int u = w; u < 56; u += NT / 64) {
      const int mt = u >> 1, x0 = (u & 1) * 16;
      const int m = 16 * mt + i;
      const int img = m / 56, rem = m - 56 * (m / 56);
      const bf16* abase = ((rem & 1) ? Xs1 : Xs) + img * 1024 + (rem >> 1) * 32 + x0 + 8 * g;
      f32x4 acc[3];
#pragma unroll
      for (int T = 0; T < 3; ++T) acc[T] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        const bf16x8 av = ld8(abase + ky * 32);
#pragma unroll
        for (int T = 0; T < 3; ++T) acc[T] = mfma16x16x32(av, bc[ky * 3 + T], acc[T]);
      }
      const int m0 = 16 * mt + 4 * g;
      const int imgo = m0 / 56, py = (m0 - 56 * (m0 / 56)) >> 2;
      const int px = (x0 >> 1) + (i & 7);
      unsigned cw = 0;
#pragma unroll
      for (int T = 0; T < 3; ++T) {
        float best;
        unsigned code;
        pool4(acc[T][0] + b1c[T], acc[T][1] + b1c[T], acc[T][2] + b1c[T], acc[T][3] + b1c[T], best, code);
        const int c = 2 * T + (i >> 3);
        if (px < 14) P1[((imgo * 14 + py) * 14 + px) * 8 + c] = f2bf(best);
        cw |= code << (3 * c);
      }
      cw |= __shfl_xor(cw, 8, 64);
      if (i < 8 && px < 14) C1[(imgo * 14 + py) * 14 + px] = cw;
    }
  }
  __syncthreads();
  LN_STAMP(2);

  // ---------------------------------------------------------------- phase B: conv2 + ReLU + pool
  DenseFrags<13, ccdiv(8, NW)> f1;  // dense-1 weights: L2 latency hidden behind conv2
  dense_load(f1, a.d1w, 8);
  {
    bf16x8 bw[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) bw[s] = frag[(FR_C2 + s) * 64 + lane];
    int toff[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int tap = 4 * s + g;
      toff[s] = tap < 25 ? ((tap / 5) * 14 + (tap - 5 * (tap / 5))) * 8 : 0;
    }
    const float b2 = WS[6 + i];
#pragma unroll 2
    for (int mt = w; mt < 50; mt += NT / 64) {
      const bf16* abase = P1 + (int)PX[16 * mt + i] * 8;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 7; ++s) acc = mfma16x16x32(ld8(abase + toff[s]), bw[s], acc);
      const int m0 = 16 * mt + 4 * g;
      const int img0 = m0 / 100, win0 = (m0 - 100 * (m0 / 100)) >> 2;
      float best;
      unsigned code;
      pool4(acc[0] + b2, acc[1] + b2, acc[2] + b2, acc[3] + b2, best, code);
      H0[img0 * LD0 + win0 * 16 + i] = f2bf(best);
      C2[(img0 * 25 + win0) * 16 + i] = (unsigned char)code;
    }
  }
  __syncthreads();
  LN_STAMP(3);

  // ---------------------------------------------------------------- phase C: dense head, CE, backward
  // H0^T for the dense-1 weight gradient (before H0 is overwritten by its gradient)
  for (int k = tid; k < 400; k += NT) {
    bf16* dst = a.h0T + (long long)k * a.ldt + r0;
    if (rows == IMG) {
      bf16x8 v;
#pragma unroll
      for (int r = 0; r < IMG; ++r) v[r] = H0[r * LD0 + k];
      st8(dst, v);
    } else {
      for (int r = 0; r < rows; ++r) dst[r] = H0[r * LD0 + k];
    }
  }
  DenseFrags<4, ccdiv(6, NW)> f2;
  DenseFrags<3, 1> f3;
  dense_load(f2, a.d2w, 6);
  dense_load(f3, a.d3w, 1);
  dense_fwd(f1, H0, LD0, ZR, a.d1b, 120, true, H1, LD1, nullptr, a.h1T, a.ldt, r0, rows);
  __syncthreads();
  DenseFrags<1, ccdiv(6, NW)> g3;
  DenseFrags<3, ccdiv(8, NW)> g2;
  dense_load(g3, a.d3wt, 6);
  dense_load(g2, a.d2wt, 8);
  dense_fwd(f2, H1, LD1, ZR, a.d2b, 84, true, H2, LD2, nullptr, a.h2T, a.ldt, r0, rows);
  __syncthreads();
  DenseFrags<4, ccdiv(25, NW)> g1;  // dense-1 data-gradient weights: loads overlap dense-3 and the loss
  dense_load(g1, a.d1wt, 25);
  dense_fwd(f3, H2, LD2, ZR, a.d3b, 10, false, nullptr, 0, LG, nullptr, a.ldt, r0, rows);
  __syncthreads();
  LN_STAMP(4);
  if (tid < IMG) {
    const int r = tid;
    float lsum = 0.f, corr = 0.f;
    if (r < rows) {
      const long long src = a.idx ? a.idx[r0 + r] : (long long)(r0 + r);
      int y = a.labels[src < 0 ? 0 : (src >= a.nrows ? a.nrows - 1 : src)];
      y = y < 0 ? 0 : (y > 9 ? 9 : y);
      float mx = -INFINITY;
      int am = 0;
      for (int c = 0; c < 10; ++c) {
        const float z = LG[r * 16 + c];
        if (a.logits) a.logits[(long long)(r0 + r) * 10 + c] = z;
        if (z > mx) { mx = z; am = c; }
      }
      float pr[10], s = 0.f;
      for (int c = 0; c < 10; ++c) {
        pr[c] = __expf(LG[r * 16 + c] - mx);
        s += pr[c];
      }
      const float inv = 1.f / s;
      lsum = -(LG[r * 16 + y] - mx - __logf(s));
      corr = am == y ? 1.f : 0.f;
      for (int c = 0; c < 10; ++c) {
        const float gv = (pr[c] * inv - (c == y ? 1.f : 0.f)) * a.grad_scale;
        Z3[r * LD3 + c] = f2bf(gv);
        a.dz3T[(long long)c * a.ldt + r0 + r] = f2bf(gv);
      }
    }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) {
      lsum += __shfl_xor(lsum, o, 8);
      corr += __shfl_xor(corr, o, 8);
    }
    if (tid == 0) {
      a.loss_part[2 * blockIdx.x] = lsum;
      a.loss_part[2 * blockIdx.x + 1] = corr;
    }
  }
  __syncthreads();
  LN_STAMP(5);
  dense_bwd(g3, Z3, LD3, ZR, 84, H2, LD2, Z2, LD2, a.dz2T, a.ldt, r0, rows);
  __syncthreads();
  dense_bwd(g2, Z2, LD2, ZR, 120, H1, LD1, Z1, LD1, a.dz1T, a.ldt, r0, rows);
  __syncthreads();
  dense_bwd(g1, Z1, LD1, ZR, 400, H0, LD0, H0, LD0, nullptr, 0, r0, rows);  // in place: dP2
  __syncthreads();
  LN_STAMP(6);

  // ---------------------------------------------------------------- phase D: unpool dP2 -> dC2
  {
    bf16x8 dp[2];
    unsigned long long cd[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int it = tid + k * NT;
      if (it < IMG * 50) {
        const int img = it / 50, rem = it - 50 * (it / 50), win = rem >> 1, nh = rem & 1;
        dp[k] = ld8(H0 + img * LD0 + win * 16 + 8 * nh);
        cd[k] = *reinterpret_cast<const unsigned long long*>(C2 + (img * 25 + win) * 16 + 8 * nh);
      }
    }
    __syncthreads();  // dC2 overlays H0 / codes2
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int it = tid + k * NT;
      if (it < IMG * 50) {
        const int img = it / 50, rem = it - 50 * (it / 50), win = rem >> 1, nh = rem & 1;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = ((cd[k] >> (8 * e)) & 255u) == (unsigned)d ? dp[k][e] : (bf16)0.f;
          st8(DC2 + ((img * 100 + win * 4 + d) * 16 + 8 * nh), o);
        }
      }
    }
  }
  __syncthreads();
  LN_STAMP(7);

  // ---------------------------------------------------------------- phase E: conv2 weight gradient
  // dW2[n][(tap, c)] = sum_m dC2[m][n] im2col(P1)[m][(tap, c)]: both operands by transposed reads;
  // wave w owns the 16-column tiles T = w + NW k (taps 2T, 2T + 1); tap 25 is the bias column of ones.
  bf16x8 bd[15];  // conv2 data-gradient fragments for phase F, in flight during this phase
#pragma unroll
  for (int s = 0; s < 15; ++s) bd[s] = frag[(FR_DG + s) * 64 + lane];
  {
    const int q = (lane & 15) >> 2, p = lane & 3;
    constexpr int KT = ccdiv(13, NW);  // column tiles per wave (13 tiles: taps 0..24 + the bias column)
    int toff[KT];
    bool ones[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int tap = 2 * (w + NW * k) + (p >> 1);
      ones[k] = tap >= 25;
      toff[k] = tap < 25 ? ((tap / 5) * 14 + (tap - 5 * (tap / 5))) * 8 + 4 * (p & 1) : 0;
    }
    const int ntile = (13 - w + NW - 1) / NW;
    f32x4 acc[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) acc[k] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 5
    for (int s = 0; s < 25; ++s) {
      const int mA = 32 * s + 8 * g + q;
      const bf16x8 av = cat8(tr_read(DC2 + mA * 16 + 4 * p), tr_read(DC2 + (mA + 4) * 16 + 4 * p));
      const bf16* pb0 = P1 + (int)PX[mA] * 8;
      const bf16* pb1 = P1 + (int)PX[mA + 4] * 8;
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        if (k < ntile) {
          const bf16x4 t0 = tr_read(ones[k] ? KO : pb0 + toff[k]);
          const bf16x4 t1 = tr_read(ones[k] ? KO : pb1 + toff[k]);
          acc[k] = mfma16x16x32(av, cat8(t0, t1), acc[k]);
        }
      }
    }
    // D[row = output channel 4g + r][col i = (tap 2T + (i >> 3), channel i & 7)]
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      if (k < ntile) {
        const int T = w + NW * k;
        const int tap = 2 * T + (i >> 3), c = i & 7;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 4 * g + r;
          if (tap < 25 && c < 6) part[(long long)(kLeNetPW2 + n * 150 + tap * 6 + c) * pld] = acc[k][r];
          else if (tap == 25 && c == 0) part[(long long)(kLeNetPB2 + n) * pld] = acc[k][r];
        }
      }
    }
  }
  __syncthreads();  // phase E finished reading P1: it now receives dP1
  LN_STAMP(8);

  // ---------------------------------------------------------------- phase F: conv2 data gradient
  {
    const int bcol = i >> 3, c = i & 7;
#pragma unroll 2
    for (int mt = w; mt < 49; mt += NT / 64) {
      const int m = 16 * mt + i;
      const int img = m / 98, rem = m - 98 * (m / 98);
      const uint4 tv = *reinterpret_cast<const uint4*>(FT + (rem * 2 + (g >> 1)) * 16);
      const unsigned tw[4] = {tv.x, tv.y, tv.z, tv.w};
      const bf16* dbase = DC2 + img * 1600 + 8 * (g & 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 15; ++s) {
        const unsigned t = (tw[s >> 2] >> (8 * (s & 3))) & 255u;
        acc = mfma16x16x32(ld8(t == 255u ? KZ : dbase + t * 16), bd[s], acc);
      }
      if (c < 6) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mm = 16 * mt + 4 * g + r;
          const int im = mm / 98, rm = mm - 98 * (mm / 98);
          const int y = rm / 7, X2 = rm - 7 * (rm / 7);
          P1[((im * 14 + y) * 14 + 2 * X2 + bcol) * 8 + c] = f2bf(acc[r]);
        }
      }
    }
  }
  __syncthreads();
  build_shift1(Xs, Xs1);  // dC2 is no longer needed: the union takes the shifted input again
  __syncthreads();
  LN_STAMP(9);

  // ---------------------------------------------------------------- phase G: conv1 weight gradient
  // D[c][tap] = sum over (image, y, x) of dC1[c][y][x] X[y + ky][x + kx].  A fragment of lane
  // (c = i, g) = dC1[c][y][8g .. 8g + 8) unpooled in registers from dP1 + codes (4 windows); B of lane
  // (tap = 16T + i, g) = 4 dword reads of the input row y + ky at column 8g + kx (odd kx: the shifted
  // copy).  No per-image staging, no barrier inside the loop.
  {
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int ca = i < 6 ? i : 5;
    int boff[2];
    const bf16* bsrc[2];
#pragma unroll
    for (int T = 0; T < 2; ++T) {
      const int tap = 16 * T + i;
      if (tap < 25) {
        const int ky = tap / 5, kx = tap - 5 * (tap / 5);
        bsrc[T] = (kx & 1) ? Xs1 : Xs;
        boff[T] = ky * 32 + 8 * g + (kx & ~1);
      } else {
        bsrc[T] = tap == 25 ? KO : KZ;
        boff[T] = -1;
      }
    }
#pragma unroll 2
    for (int rp = w; rp < IMG * 14; rp += NT / 64) {
      const int img = rp / 14, py = rp - 14 * (rp / 14);
      // A rows y = 2 py (dy = 0) and 2 py + 1 (dy = 1) from the same 4 pool windows px = 4g .. 4g + 3
      const int p0 = (img * 14 + py) * 14 + 4 * g;
      const uint2 cA = *reinterpret_cast<const uint2*>(C1 + p0);
      const uint2 cB = *reinterpret_cast<const uint2*>(C1 + p0 + 2);
      const unsigned cw[4] = {cA.x, cA.y, cB.x, cB.y};
      bf16x8 a0, a1;
#pragma unroll
      for (int wd = 0; wd < 4; ++wd) {
        const bool ok = 4 * g + wd < 14 && i < 6;
        const unsigned code = (cw[wd] >> (3 * ca)) & 7u;
        const bf16 v = ok ? P1[(p0 + wd) * 8 + ca] : (bf16)0.f;
        a0[2 * wd] = code == 0u ? v : (bf16)0.f;
        a0[2 * wd + 1] = code == 1u ? v : (bf16)0.f;
        a1[2 * wd] = code == 2u ? v : (bf16)0.f;
        a1[2 * wd + 1] = code == 3u ? v : (bf16)0.f;
      }
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const int y = 2 * py + dy;
#pragma unroll
        for (int T = 0; T < 2; ++T) {
          bf16x8 bv;
          if (boff[T] >= 0) {
            const unsigned* bp = reinterpret_cast<const unsigned*>(bsrc[T] + img * 1024 + y * 32 + boff[T]);
            uint4 u;
            u.x = bp[0];
            u.y = bp[1];
            u.z = bp[2];
            u.w = bp[3];
            bv = __builtin_bit_cast(bf16x8, u);
          } else {
            bv = ld8(bsrc[T]);
          }
          acc[T] = mfma16x16x32(dy ? a1 : a0, bv, acc[T]);
        }
      }
    }
    // cross-wave sum: D[row = channel 4g + r][col = tap 16T + i]; waves w and w + 4 share slot w & 3
    // (the upper half writes, then the lower half adds in place: a [4][16][32] buffer for 8 waves)
    if (w >= 4) {
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) RED[((w & 3) * 16 + 4 * g + r) * 32 + 16 * T + i] = acc[T][r];
    }
    __syncthreads();
    if (w < 4) {
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* q = RED + (w * 16 + 4 * g + r) * 32 + 16 * T + i;
          *q = (NW > 4 ? *q : 0.f) + acc[T][r];
        }
    }
    __syncthreads();
    for (int e = tid; e < 6 * 32; e += NT) {
      const int c = e >> 5, col = e & 31;
      const float v = RED[(0 * 16 + c) * 32 + col] + RED[(1 * 16 + c) * 32 + col] + RED[(2 * 16 + c) * 32 + col] +
                      RED[(3 * 16 + c) * 32 + col];
      if (col < 25) part[(long long)(kLeNetPW1 + c * 25 + col) * pld] = v;
      else if (col == 25) part[(long long)(kLeNetPB1 + c) * pld] = v;
    }
  }
  LN_STAMP(10);
}

// Conv weights of this step as MFMA B fragments: one block (csrc/lenet_frag.h).  Only launched when
// the optimizer does not rebuild them (the fused step's SGD launch normally does, see optim.hip).
constexpr int PT = 1024;
__global__ void __launch_bounds__(PT) lenet_prep_kernel(const float* __restrict__ w1g, const float* __restrict__ w2g,
                                                        bf16x8* __restrict__ frag) {
  __shared__ float w[kLeNetConvW];
  for (int e = threadIdx.x; e < 150; e += PT) w[e] = w1g[e];
  for (int e = threadIdx.x; e < 2400; e += PT) w[150 + e] = w2g[e];
  __syncthreads();
  lenet_build_frags(w, frag, threadIdx.x, PT);
}

// ------------------------------------------------------------------------------------------------
// Reductions in one launch, deterministic (fixed summation order everywhere):
//   blocks [0, dense_tiles)  one 16x16 tile of a dense weight gradient each (K = batch split over 16
//                 waves, LDS combine; bias = a column of ones).  Tiles are placed by a host table so
//                 that all tiles reading the same 16 activation rows run on one XCD: every XCD then
//                 fetches its share of H^T once and dZ^T once into its own L2 and re-reads them there.
//   next nconv_blocks        64 conv parameters each: wave w sums the contiguous partial rows of
//                 parameters 4w .. 4w + 3 (parameter-major partial layout), butterfly combine.
//   last block               loss partials -> stats.
constexpr int RT = 1024;


// ---- one exchange slot = one dense weight-gradient tile (16 x 16, threads t < 256 own an element each) or
// one conv block (64 parameters, lanes of wave 0).  The value functions return this thread's local sum.

// dense tile `slot`: K = batch split over the 16 waves, LDS combine (bias = a column of ones)
__device__ __forceinline__ float dense_tile_value(const LeNetRedArgs& a, int slot, float (*red)[16][17]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int tile = a.tile_of_block[slot];
  int l = 0;
  if (tile >= a.L[0].tiles) {
    tile -= a.L[0].tiles;
    l = 1;
    if (tile >= a.L[1].tiles) {
      tile -= a.L[1].tiles;
      l = 2;
    }
  }
  const LeNetDense& L = a.L[l];
  const int tk = tile / ((L.N + 15) / 16), tn = tile - ((L.N + 15) / 16) * tk;  // tn fastest
  const int n = 16 * tn + (lane & 15), k = 16 * tk + (lane & 15);
  const bf16* arow = L.dzT + (long long)min(n, L.N - 1) * a.ldt + 8 * (lane >> 4);
  const bf16* brow = L.hT + (long long)min(k, L.K - 1) * a.ldt + 8 * (lane >> 4);
  const bool a_ok = n < L.N, b_ones = k == L.K, b_ok = k < L.K;
  bf16x8 ones, zeros = zero8();
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.f;
  const int steps = a.ldt / 32;
  const int per = (steps + 15) / 16;
  const int s0 = wid * per, s1 = min(steps, s0 + per);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < (a.probe == 1 ? s0 : s1); s += 8) {
    bf16x8 av[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int ss = min(s + u, s1 - 1);
      av[u] = ld8(arow + 32 * ss);
      bv[u] = ld8(brow + 32 * ss);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool live = s + u < s1;
      acc = mfma16x16x32((a_ok && live) ? av[u] : zeros, b_ok ? bv[u] : (b_ones ? ones : zeros), acc);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wid][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  float v = 0.f;
  if (threadIdx.x < 256) {
    const int rn = threadIdx.x >> 4, ck = threadIdx.x & 15;
#pragma unroll
    for (int ww = 0; ww < 16; ++ww) v += red[ww][rn][ck];
  }
  return v;
}

__device__ __forceinline__ void dense_tile_apply(const LeNetRedArgs& a, int slot, float v) {
  int tile = a.tile_of_block[slot];
  int l = 0;
  if (tile >= a.L[0].tiles) {
    tile -= a.L[0].tiles;
    l = 1;
    if (tile >= a.L[1].tiles) {
      tile -= a.L[1].tiles;
      l = 2;
    }
  }
  const LeNetDense& L = a.L[l];
  const int tk = tile / ((L.N + 15) / 16), tn = tile - ((L.N + 15) / 16) * tk;
  const int on = 16 * tn + (threadIdx.x >> 4), ok = 16 * tk + (threadIdx.x & 15);
  if (on < L.N) {
    if (ok < L.K) L.gw[(long long)on * L.K + ok] = v;
    else if (ok == L.K) L.gb[on] = v;
    if (a.sgd_on && ok <= L.K)  // fused update of this element
      sgd_apply_one(a.sgd.d[4 + 2 * l + (ok == L.K ? 1 : 0)], ok < L.K ? on * L.K + ok : on, v, a.sgd.master,
                    a.sgd.mom, a.sgd.wbf, a.sgd.hyper);
  }
}

// conv block `cb`: 64 parameters; wave w sums parameters 4w .. 4w + 3, each over its contiguous row of
// workgroup partials (16-byte loads, all in flight, fixed-order lane sums + butterfly: deterministic)
__device__ __forceinline__ float conv_value(const LeNetRedArgs& a, int cb, float (*red)[16][17]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* sred = &red[0][0][0];
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int q0 = 0; q0 < (a.probe == 2 ? 0 : a.part_ld); q0 += 512) {
    f32x4 x[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = min(cb * 64 + 4 * wid + j, kLeNetConvParams - 1);
      const f32x4* row = reinterpret_cast<const f32x4*>(a.conv_part + (long long)p * a.part_ld + q0 + lane * 8);
      x[j][0] = row[0];
      x[j][1] = row[1];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      s[j] += ((x[j][0][0] + x[j][0][1]) + (x[j][0][2] + x[j][0][3])) +
              ((x[j][1][0] + x[j][1][1]) + (x[j][1][2] + x[j][1][3]));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float t = wave_sum(s[j]);
    if (lane == 0) sred[4 * wid + j] = t;
  }
  __syncthreads();
  return wid == 0 ? sred[lane] : 0.f;
}

__device__ __forceinline__ void conv_apply(const LeNetRedArgs& a, int cb, float v) {
  const int p = cb * 64 + (threadIdx.x & 63);
  if (p >= kLeNetConvParams) return;
  float* dst = p < kLeNetPB1 ? a.g_w1 + p
               : p < kLeNetPW2 ? a.g_b1 + (p - kLeNetPB1)
               : p < kLeNetPB2 ? a.g_w2 + (p - kLeNetPW2)
                               : a.g_b2 + (p - kLeNetPB2);
  *dst = v;
  const int wj = p < kLeNetPB1 ? p : (p >= kLeNetPW2 && p < kLeNetPB2) ? 150 + (p - kLeNetPW2) : -1;
  if (a.sgd_on) {
    const int di = p < kLeNetPB1 ? 0 : p < kLeNetPW2 ? 1 : p < kLeNetPB2 ? 2 : 3;
    const int i = p - (di == 0 ? 0 : di == 1 ? kLeNetPB1 : di == 2 ? kLeNetPW2 : kLeNetPB2);
    const float nw = sgd_apply_one(a.sgd.d[di], i, v, a.sgd.master, a.sgd.mom, a.sgd.wbf, a.sgd.hyper);
    // the new conv weight goes straight into the next step's MFMA fragments
    if (wj >= 0) lenet_frag_scatter(a.sgd.frag, wj, nw);
  } else if (a.snap != nullptr && wj >= 0) {
    // the conv kernels' weights and momentum as this gradient saw them: the optimizer launch rebuilds
    // the next step's fragments from these (no read of state it is overwriting)
    const long long o = wj < 150 ? wj : wj - 150;
    a.snap[wj] = wj < 150 ? a.w1[o] : a.w2[o];
    a.snap[kLeNetConvW + wj] = a.m1 == nullptr ? 0.f : (wj < 150 ? a.m1[o] : a.m2[o]);
  }
}

// ---- asynchronous SGD against the device parameter server (LeNetRedArgs::ps_on) ------------------------
// Decision codes: the gradient is admitted (apply + refresh from the new version), rejected as too stale
// (refresh from the current version; the writer lock is held while the copies are read), the schedule
// is finished (no-op), or a wait timed out (no-op, error bits set).
constexpr unsigned kPSAccept = 1, kPSReject = 2, kPSFailed = 3, kPSFinished = 4;

// Every exchanging workgroup (and the staging workgroup) learns this launch's decision.  Workgroup 0
// takes the writer lock (seqlock CAS on the server's word), checks staleness = version_now -
// version_pulled against the bound and completes the microbatch under the lock; the others wait for
// the decision word tagged with this launch's epoch (local, agent scope: all of them are resident).
__device__ void lenet_ps_decide(const LeNetRedArgs& a, unsigned* s_dec, unsigned* s_seq, bool after_completion = false) {
  const PSArgs& p = a.ps;
  if (threadIdx.x == 0) {
    const unsigned ep = __hip_atomic_load(p.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const unsigned long long t0 = wall_clock64();
    unsigned dec = kPSFailed, s = 0;
    if (blockIdx.x == 0) {
      const long long bid = *p.bid_out;
      if (p.done_epoch != nullptr && bid < 0) {  // dataset finished: a no-op step (no lock taken)
        dec = kPSFinished;
        p.stats[6] += 1;
      } else {
        for (;;) {
          s = ps_ld_acq(p.seq);
          if (!(s & 1u)) {
            unsigned expected = s;
            if (__hip_atomic_compare_exchange_strong(p.seq, &expected, s + 1u, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM)) {
              const unsigned stale = (s >> 1) - *p.vpulled;
              dec = ((int)stale <= p.max_stale || p.max_stale < 0) ? kPSAccept : kPSReject;
              // the appliers need only the decision: publish it first, then do the bookkeeping
              __hip_atomic_store(p.scratch + kPSLockedSeq, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(p.scratch + kPSDecision, (ep << 3) | dec, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
              if (dec == kPSAccept) {
                p.stats[0] += 1;
                p.stats[2] += stale;
                if (stale > p.stats[3]) p.stats[3] = stale;
                if (p.done_epoch != nullptr) complete_microbatch(p, bid);  // under the writer lock
              } else {
                p.stats[1] += 1;  // rejected: the lock is held until every workgroup copied version s / 2
              }
              break;
            }
          }
          if (wall_clock64() - t0 > (unsigned long long)p.timeout_ticks) {
            atomicOr(p.stats + 5, 4ull);
            if (p.herr) __hip_atomic_store(p.herr, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (dec != kPSAccept && dec != kPSReject) {  // no lock taken: finished schedule or timeout
        __hip_atomic_store(p.scratch + kPSLockedSeq, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p.scratch + kPSDecision, (ep << 3) | dec, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      // the microbatch bookkeeping is done: the staging workgroup may claim the next one
      __hip_atomic_store(p.scratch + kPSCompleted, ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const unsigned* word = p.scratch + (after_completion ? kPSCompleted : kPSDecision);
      for (;;) {  // relaxed polls, one acquire once the word matches (acquire polls cost every poller an
                  // L1 invalidate per iteration)
        const unsigned w = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned d = after_completion
                               ? (w == ep ? __hip_atomic_load(p.scratch + kPSDecision, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT)
                                          : 0u)
                               : w;
        if ((d >> 3) == ep) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          dec = d & 7u;
          break;
        }
        if (wall_clock64() - t0 > 2ull * (unsigned long long)p.timeout_ticks) {
          atomicOr(p.stats + 5, 8ull);
          if (p.herr) __hip_atomic_store(p.herr, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s = __hip_atomic_load(p.scratch + kPSLockedSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *s_dec = dec;
    *s_seq = s;
  }
  __syncthreads();
}

// One parameter element on the PS: w_new = w[v] - lr * g into buffer (v + 1) % 3 of the shared master
// (admitted) or the current w[v] (rejected); either way the local master and its bf16 compute copies
// become that version.  Returns the local weight.
__device__ __forceinline__ float lenet_ps_elem(const LeNetRedArgs& a, const ParamDesc& d, int i, float g,
                                               unsigned dec, unsigned seq) {
  const PSArgs& p = a.ps;
  const unsigned v = seq >> 1;
  const long long off = d.off + i;
  const float w = p.ps_w[(long long)(v % 3u) * p.nstride + off];
  float wn = w;
  if (dec == kPSAccept) {
    wn = w - p.lr * g;
    p.ps_w[(long long)((v + 1u) % 3u) * p.nstride + off] = wn;
  }
  a.sgd.master[off] = wn;
  emit_copies(d, i, wn, a.sgd.wbf);
  return wn;
}

__device__ __forceinline__ void dense_tile_ps(const LeNetRedArgs& a, int slot, float g, unsigned dec, unsigned seq) {
  int tile = a.tile_of_block[slot];
  int l = 0;
  if (tile >= a.L[0].tiles) {
    tile -= a.L[0].tiles;
    l = 1;
    if (tile >= a.L[1].tiles) {
      tile -= a.L[1].tiles;
      l = 2;
    }
  }
  const LeNetDense& L = a.L[l];
  const int tk = tile / ((L.N + 15) / 16), tn = tile - ((L.N + 15) / 16) * tk;
  const int on = 16 * tn + (threadIdx.x >> 4), ok = 16 * tk + (threadIdx.x & 15);
  if (on >= L.N || ok > L.K) return;
  if (ok < L.K) L.gw[(long long)on * L.K + ok] = g;
  else L.gb[on] = g;
  lenet_ps_elem(a, a.sgd.d[4 + 2 * l + (ok == L.K ? 1 : 0)], ok < L.K ? on * L.K + ok : on, g, dec, seq);
}

__device__ __forceinline__ void conv_ps(const LeNetRedArgs& a, int cb, float g, unsigned dec, unsigned seq) {
  const int p = cb * 64 + (threadIdx.x & 63);
  if (p >= kLeNetConvParams) return;
  float* dst = p < kLeNetPB1 ? a.g_w1 + p
               : p < kLeNetPW2 ? a.g_b1 + (p - kLeNetPB1)
               : p < kLeNetPB2 ? a.g_w2 + (p - kLeNetPW2)
                               : a.g_b2 + (p - kLeNetPB2);
  *dst = g;
  const int di = p < kLeNetPB1 ? 0 : p < kLeNetPW2 ? 1 : p < kLeNetPB2 ? 2 : 3;
  const int i = p - (di == 0 ? 0 : di == 1 ? kLeNetPB1 : di == 2 ? kLeNetPW2 : kLeNetPB2);
  const float w = lenet_ps_elem(a, a.sgd.d[di], i, g, dec, seq);
  const int wj = p < kLeNetPB1 ? p : (p >= kLeNetPW2 && p < kLeNetPB2) ? 150 + (p - kLeNetPW2) : -1;
  if (wj >= 0) lenet_frag_scatter(a.sgd.frag, wj, w);  // the next step's conv fragments
}

// Arrival of one of the nexch + 1 protocol workgroups (exchanging + staging): the last one publishes
// version v + 1 (admitted) or releases the lock (rejected) and records the pulled version.
__device__ void lenet_ps_arrive(const LeNetRedArgs& a, int arrivals, unsigned dec, unsigned seq) {
  const PSArgs& p = a.ps;
  // every storing wave drains its shared-master stores (uncached / fine-grained memory: complete at the
  // server's HBM once acknowledged), then the arrival ticket; the last arriver's system-scope release
  // store of the version word orders all of them before the publish (no per-workgroup L2 write-back)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(p.scratch + kPSApplyDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned)arrivals - 1) {
      __hip_atomic_store(p.scratch + kPSApplyDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.scratch + kPSEpoch, __hip_atomic_load(p.scratch + kPSEpoch, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT) + 1u,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every workgroup's arrival happened before the unlock
      if (dec == kPSAccept) {
        *p.vpulled = (seq >> 1) + 1u;
        __hip_atomic_store(p.seq, seq + 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      } else if (dec == kPSReject) {
        *p.vpulled = seq >> 1;
        __hip_atomic_store(p.seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

constexpr int kMaxSlotsPerBlock = 8;

// Exchange workgroups [0, exch_blocks) own slots blockIdx.x + k * exch_blocks: all their slots' local
// sums are computed and pushed to the peers first, then each is waited for, summed over the ranks and
// applied (one round trip per workgroup, not per slot).  On a node with one rank per GPU exch_blocks ==
// slots (one each, every workgroup resident); ranks that time-share one GPU use fewer, so that the
// waiting workgroups of all ranks fit on the chip beside the peers' train kernels.
// Then one workgroup: loss partials -> stats; one more (index stream bound): stage the next batch.
// diagnostic phase clocks of the reduce launch: stamps[block][slot] (0 start, 1 local sums pushed,
// 2 decision / exchange done, 3 applied, 4 end, 5 all waves started, 6 first slot summed)
#define LR_STAMP(slot)                                                            \
  do {                                                                            \
    if (a.stamps) {                                                               \
      __builtin_amdgcn_sched_barrier(0);                                          \
      unsigned long long t_;                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                          \
      if (threadIdx.x == 0) a.stamps[blockIdx.x * 8 + (slot)] = t_;               \
    }                                                                             \
  } while (0)

__global__ void __launch_bounds__(RT, 8) lenet_reduce_kernel(LeNetRedArgs a) {
  __shared__ float red[16][16][17];
  __shared__ unsigned s_e;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  LR_STAMP(0);
  if (a.stamps) {
    __syncthreads();
    LR_STAMP(5);  // every wave of the workgroup has started
  }
  const int nslot = a.dense_tiles + a.nconv_blocks;
  const int nexch = a.exch_blocks;
  if ((int)blockIdx.x < nexch) {
    __shared__ float keep[kMaxSlotsPerBlock][256];  // this workgroup's local sums, per slot and position
    __shared__ unsigned ep[kMaxSlotsPerBlock];
#pragma unroll 1
    for (int k = 0; k < kMaxSlotsPerBlock; ++k) {
      const int slot = blockIdx.x + k * nexch;
      if (slot >= nslot) break;  // uniform over the workgroup
      __syncthreads();           // the previous slot's readers of red are done
      const bool dense = slot < a.dense_tiles;
      const float v = dense ? dense_tile_value(a, slot, red) : conv_value(a, slot - a.dense_tiles, red);
      if (k == 0) LR_STAMP(6);  // the first slot's partial sums are in
      const bool owner = dense ? threadIdx.x < 256 : wid == 0;
      if (owner) keep[k][threadIdx.x] = v;
      if (a.ll_on) {
        const unsigned e = ll_epoch(a.ll, slot, &s_e);
        if (threadIdx.x == 0) ep[k] = e;
        if (owner) ll_push(a.ll, slot, threadIdx.x, e, v);
      }
    }
    __syncthreads();
    LR_STAMP(1);
    __shared__ unsigned s_dec, s_seq;
    if (a.ps_on) lenet_ps_decide(a, &s_dec, &s_seq);
    LR_STAMP(2);
    const unsigned dec = a.ps_on ? s_dec : 0u, seq = a.ps_on ? s_seq : 0u;
#pragma unroll 1
    for (int k = 0; k < kMaxSlotsPerBlock; ++k) {
      const int slot = blockIdx.x + k * nexch;
      if (slot >= nslot) break;
      const bool dense = slot < a.dense_tiles;
      if (a.ps_on) {
        if ((dense ? threadIdx.x < 256 : wid == 0) && (dec == kPSAccept || dec == kPSReject)) {
          if (dense) dense_tile_ps(a, slot, keep[k][threadIdx.x], dec, seq);
          else conv_ps(a, slot - a.dense_tiles, keep[k][threadIdx.x], dec, seq);
        }
        continue;
      }
      if (dense ? threadIdx.x < 256 : wid == 0) {
        float v = keep[k][threadIdx.x];
        bool ok = true;
        if (a.ll_on) {  // the rank-order sum over the ranks (no all-reduce launch)
          ok = ll_wait_sum(a.ll, slot, threadIdx.x, ep[k], v, v);
          if (ok && threadIdx.x == 0) ll_commit(a.ll, slot, ep[k]);
        }
        if (ok) {
          if (dense) dense_tile_apply(a, slot, v);
          else conv_apply(a, slot - a.dense_tiles, v);
        }
      }
    }
    LR_STAMP(3);
    if (a.ps_on) lenet_ps_arrive(a, nexch + 1, dec, seq);
    LR_STAMP(4);
    return;
  }
  const int blk = blockIdx.x - nexch;
  if (blk == 1 && a.ps_on) {
    // async: once this launch's decision is known (the current microbatch is completed under the lock),
    // claim the next microbatch FCFS on the server and stage its example indices
    __shared__ unsigned s_dec, s_seq;
    __shared__ long long s_bid;
    lenet_ps_decide(a, &s_dec, &s_seq, /*after_completion=*/true);
    if (a.ps.done_epoch != nullptr) {
      claim_microbatch(a.ps, threadIdx.x, &s_bid);
    } else if (threadIdx.x == 0) {
      s_bid = (long long)(__hip_atomic_fetch_add(a.ps.batch_ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) %
                          (unsigned long long)(a.ps.nbatches > 0 ? a.ps.nbatches : 1));
    }
    __syncthreads();
    if (threadIdx.x == 0) *a.ps.bid_out = s_bid;
    ps_stage_indices(a.ps, s_bid, threadIdx.x, RT);
    lenet_ps_arrive(a, nexch + 1, s_dec, s_seq);
    return;
  }
  if (blk == 1) {  // fused update: stage the next step's batch indices, advance the cursor
    __shared__ long long nxt;
    if (threadIdx.x == 0) nxt = (*a.sgd.cursor + 1) % a.sgd.nsteps;
    __syncthreads();
    const long long* src = a.sgd.src + nxt * a.sgd.B;
    for (int i = threadIdx.x; i < a.sgd.B; i += RT) a.sgd.dst[i] = src[i];
    if (threadIdx.x == 0) *a.sgd.cursor = nxt;
    return;
  }
  if (wid == 0) {  // loss partials -> stats
    float l = 0.f, c = 0.f;
    for (int k = lane; k < a.nblk; k += 64) {
      l += a.loss_part[2 * k];
      c += a.loss_part[2 * k + 1];
    }
    l = wave_sum(l);
    c = wave_sum(c);
    if (lane == 0) {
      a.stats[0] = l;
      a.stats[1] = c;
      if (a.sgd_on && a.sgd.run_stats != nullptr) {  // device run statistics (trainer callbacks)
        a.sgd.run_stats[0] += l;
        a.sgd.run_stats[1] += c;
        a.sgd.run_stats[2] += 1.f;
      }
    }
  }
}

}  // namespace

size_t lenet_train_lds() { return LDS_BYTES; }
int lenet_blocks(int B) { return (B + IMG - 1) / IMG; }

static unsigned long long* g_lenet_stamps_host = nullptr;
void lenet_set_stamps(void* buf) { g_lenet_stamps_host = reinterpret_cast<unsigned long long*>(buf); }

size_t lenet_frag_bytes() { return (size_t)NFRAG * 64 * 16; }
int lenet_dense_part_floats(int B) { (void)B; return 0; }

hipError_t lenet_train(const LeNetArgs& a_in, LeNetRedArgs r, hipStream_t st) {
  LeNetArgs a = a_in;
  a.stamps = g_lenet_stamps_host;
  // the reduce launch's clocks follow the train kernel's [4096][16] region
  r.stamps = g_lenet_stamps_host ? g_lenet_stamps_host + 4096 * 16 : nullptr;
  r.probe = diag_int("lenet_red_probe", 0);
  if (a.B <= 0 || a.ldt % 32 || a.ldt < a.B || !a.frag || !a.ftab || !a.pxtab) return hipErrorInvalidValue;
  const int nblk = (a.B + IMG - 1) / IMG;
  if (a.prep) {
    hipLaunchKernelGGL(lenet_prep_kernel, dim3(1), dim3(PT), 0, st, a.w1, a.w2,
                       reinterpret_cast<bf16x8*>(const_cast<void*>(a.frag)));
    DFA_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(lenet_train_kernel, dim3(nblk), dim3(NT), LDS_BYTES, st, a);
  DFA_HIP_CHECK(hipGetLastError());
  r.nblk = nblk;
  r.ldt = a.ldt;
  r.nconv_blocks = (kLeNetConvParams + 63) / 64;
  // dense tiles in (layer, tk, tn) order, tn fastest; XCD x (= block id mod 8) takes the tiles with
  // tk = x (mod 8) of every layer, so all 16-row groups of H^T stay in one L2
  int tiles_per_layer[3], base = 0;
  std::vector<int> by_xcd[8];
  for (int l = 0; l < 3; ++l) {
    const int nt = (r.L[l].N + 15) / 16, kt = (r.L[l].K + 1 + 15) / 16;
    r.L[l].tiles = nt * kt;
    tiles_per_layer[l] = nt * kt;
    for (int tk = 0; tk < kt; ++tk)
      for (int tn = 0; tn < nt; ++tn) by_xcd[tk % 8].push_back(base + tk * nt + tn);
    base += nt * kt;
  }
  (void)tiles_per_layer;
  r.dense_tiles = base;
  if (r.dense_tiles > kLeNetMaxTiles) return hipErrorInvalidValue;
  size_t maxq = 0;
  for (auto& v : by_xcd) maxq = std::max(maxq, v.size());
  int b = 0;
  std::vector<int> order;
  for (size_t slot = 0; slot < maxq; ++slot)
    for (int x = 0; x < 8; ++x)
      if (slot < by_xcd[x].size()) order.push_back(by_xcd[x][slot]);
  for (int t : order) r.tile_of_block[b++] = t;
  if (r.sgd_on && (!r.sgd.master || !r.sgd.wbf || !r.sgd.hyper || !r.sgd.frag))
    return hipErrorInvalidValue;
  const int nslot = r.dense_tiles + r.nconv_blocks;
  if (r.exch_blocks <= 0 || r.exch_blocks > nslot) r.exch_blocks = nslot;
  if (r.exch_blocks * kMaxSlotsPerBlock < nslot) return hipErrorInvalidValue;
  if (r.ll_on) {
    // slot s is LL slot s.  Every exchanging workgroup must be resident at once on every rank (a waiting
    // workgroup must never keep a peer's from being dispatched): 1024-thread workgroups at 64 VGPRs and
    // 28 KB LDS run 2 per CU, so <= 512 on 256 CUs with one rank per GPU
    if (!r.sgd_on || r.ll.world < 2 || r.ll.world > kP2PMaxRanks || r.ll.rank < 0 || r.ll.rank >= r.ll.world ||
        !r.ll.epochs || !r.ll.err || nslot > r.ll.nslots || r.exch_blocks > 512)
      return hipErrorInvalidValue;
    for (int k = 0; k < r.ll.world; ++k)
      if (!r.ll.bases[k]) return hipErrorInvalidValue;
  }
  if (r.ps_on) {
    // async PS: every protocol workgroup must be resident at once (workgroup 0's decision is awaited)
    if (!r.sgd_on || r.ll_on || r.sgd.src || !r.ps.seq || !r.ps.ps_w || !r.ps.vpulled || !r.ps.bid_out ||
        !r.ps.stats || !r.ps.scratch || r.exch_blocks + 1 > 512 || r.sgd.mom)
      return hipErrorInvalidValue;
  }
  const int extra = ((r.sgd_on && r.sgd.src) || r.ps_on) ? 1 : 0;  // the index-staging workgroup
  hipLaunchKernelGGL(lenet_reduce_kernel, dim3(r.exch_blocks + 1 + extra), dim3(RT), 0, st, r);
  return hipGetLastError();
}

}  // namespace dfa
