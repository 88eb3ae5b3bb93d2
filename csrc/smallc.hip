// Direct convolution for single-channel inputs: the Keras CNN's first conv (3x3x1 -> 32,
// /root/reference/experiment/mnist/model.json).  (Measured on the ResNet-18 stem, 3x3x3 -> 64, the
// generic implicit GEMM stays faster, so dispatch is limited to C_in = 1.)
// SURVEY §2.4 O3 asks for "direct VALU conv for C_in=1 first layer (K=9)": with K = KH*KW*C_in <= 64
// an implicit GEMM wastes most of every 32-deep MFMA step and still pays the im2col gather, while the
// layer is bound by writing (forward) or reading (weight gradient) its wide output.
//
//   forward : one thread = one output pixel x 8 output channels; the weights sit in LDS as fp32
//             [K][N]; bias + alpha + ReLU in registers; one 16-byte store per thread
//   wgrad   : persistent workgroups walk 64-pixel tiles; each tile stages dY [64][N] and the im2col
//             rows X [64][K+1] (a ones column at k = K for the bias gradient) in LDS as fp32, and
//             every thread accumulates its (n, k) pairs over the tile; one fp32 slab [N][K+1] per
//             workgroup, summed in a fixed order by slab_reduce (deterministic)
#include "common.h"
#include "kernels.h"

namespace dfa {

namespace {

constexpr int kSmallMaxK = 64, kSmallMaxN = 64;

__global__ void __launch_bounds__(256) smallc_fwd_kernel(IGemmArgs a, FastDiv d_ow, FastDiv d_ohw) {
  __shared__ float wl[kSmallMaxK * kSmallMaxN];
  __shared__ float bl[kSmallMaxN];
  const int N = a.N, K = a.K;
  for (int i = threadIdx.x; i < K * N; i += 256) {
    const int k = i / N, n = i - k * N;
    wl[i] = (float)a.w[(long long)n * a.Kpad + k];
  }
  for (int i = threadIdx.x; i < N; i += 256) bl[i] = a.bias ? a.bias[i] : 0.f;
  __syncthreads();
  const int ng = N >> 3;
  const long long total = (long long)a.M * ng;
  const unsigned ohw = (unsigned)(a.OH * a.OW);
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const unsigned m = (unsigned)(idx / ng);
    const int g = (int)(idx - (long long)m * ng);
    const unsigned b = fdiv(m, d_ohw);
    const unsigned rem = m - b * ohw;
    const unsigned oh = fdiv(rem, d_ow);
    const int ow = (int)(rem - oh * (unsigned)a.OW);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const bf16* xb = a.src + (long long)b * a.SH * a.SW * a.SC;
    int k = 0;
    for (int kh = 0; kh < a.KH; ++kh) {
      const int ih = (int)oh * a.stride - a.pad + kh;
      const bool hv = (unsigned)ih < (unsigned)a.SH;
      for (int kw = 0; kw < a.KW; ++kw) {
        const int iw = ow * a.stride - a.pad + kw;
        const bool v = hv && (unsigned)iw < (unsigned)a.SW;
        const bf16* xp = xb + ((long long)(v ? ih : 0) * a.SW + (v ? iw : 0)) * a.SC;
        for (int c = 0; c < a.SC; ++c, ++k) {
          const float xv = v ? (float)xp[c] : 0.f;
          const float* wr = wl + k * N + g * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += xv * wr[j];
        }
      }
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = acc[j] * a.alpha + bl[g * 8 + j];
      if (a.relu) o[j] = fmaxf(o[j], 0.f);
    }
    const long long off = (long long)m * a.ldc + g * 8;
    if (a.out_f32) {
      float* op = reinterpret_cast<float*>(a.out) + off;
      *reinterpret_cast<f32x4*>(op) = f32x4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<f32x4*>(op + 4) = f32x4{o[4], o[5], o[6], o[7]};
    } else {
      bf16x8 ov;
#pragma unroll
      for (int j = 0; j < 8; ++j) ov[j] = f2bf(o[j]);
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.out) + off) = ov;
    }
  }
}

__global__ void __launch_bounds__(256) smallc_wgrad_kernel(WgradArgs a, FastDiv d_ow, FastDiv d_ohw, float* slabs) {
  constexpr int TM = 64;
  __shared__ float dl[TM * (kSmallMaxN + 1)];
  __shared__ float xl[TM * (kSmallMaxK + 1)];
  const int N = a.N, K = a.K, Kt = K + (a.with_bias ? 1 : 0);
  const int P = N * Kt;  // (n, k) pairs; thread t owns pairs t, t + 256, ...
  const int DS = N + 1, XS = Kt + 1;  // padded LDS rows
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const unsigned ohw = (unsigned)(a.OH * a.OW);
  const int ntiles = cdiv(a.M, TM);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int m0 = tile * TM;
    __syncthreads();  // previous tile's reads are done
    // dY tile [TM][N] (8 channels per thread-load)
    const int ng = N >> 3;
    for (int i = threadIdx.x; i < TM * ng; i += 256) {
      const int r = i / ng, g = i - r * ng;
      const int m = m0 + r;
      bf16x8 v = {};
      if (m < a.M) v = *reinterpret_cast<const bf16x8*>(a.dy + (long long)m * a.ldd + g * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) dl[r * DS + g * 8 + j] = (float)v[j];
    }
    // im2col rows [TM][Kt]
    for (int i = threadIdx.x; i < TM * Kt; i += 256) {
      const int r = i / Kt, k = i - r * Kt;
      const unsigned m = (unsigned)(m0 + r);
      float xv = 0.f;
      if ((int)m < a.M) {
        if (k == K) {
          xv = 1.f;
        } else {
          const unsigned b = fdiv(m, d_ohw);
          const unsigned rem = m - b * ohw;
          const unsigned oh = fdiv(rem, d_ow);
          const int ow = (int)(rem - oh * (unsigned)a.OW);
          const int c = k % a.SC, t = k / a.SC;
          const int kh = t / a.KW, kw = t - kh * a.KW;
          const int ih = (int)oh * a.stride - a.pad + kh, iw = ow * a.stride - a.pad + kw;
          if ((unsigned)ih < (unsigned)a.SH && (unsigned)iw < (unsigned)a.SW)
            xv = (float)a.src[(((long long)b * a.SH + ih) * a.SW + iw) * a.SC + c];
        }
      }
      xl[r * XS + k] = xv;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int p = threadIdx.x + j * 256;
      if (p < P) {
        const int n = p / Kt, k = p - n * Kt;
        float s = 0.f;
#pragma unroll 8
        for (int r = 0; r < TM; ++r) s += dl[r * DS + n] * xl[r * XS + k];
        acc[j] += s;
      }
    }
  }
  float* slab = slabs + (long long)blockIdx.x * P;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int p = threadIdx.x + j * 256;
    if (p < P) slab[p] = acc[j];
  }
}

}  // namespace

bool smallc_fwd_supported(const IGemmArgs& a, int mode) {
  return mode == MODE_FWD && a.SC == 1 && a.K <= kSmallMaxK && a.N % 8 == 0 && a.N <= kSmallMaxN && !a.mask &&
         !a.res && a.ldc % 8 == 0 && ((uintptr_t)a.out & 15) == 0 && a.OH > 0 && a.OW > 0;
}

hipError_t smallc_fwd(const IGemmArgs& a, hipStream_t st) {
  const FastDiv d_ow = make_fastdiv((unsigned)a.OW), d_ohw = make_fastdiv((unsigned)(a.OH * a.OW));
  const long long total = (long long)a.M * (a.N / 8);
  const int grid = (int)min((total + 255) / 256, 8192LL);
  hipLaunchKernelGGL(smallc_fwd_kernel, dim3(grid), dim3(256), 0, st, a, d_ow, d_ohw);
  return hipGetLastError();
}

bool smallc_wgrad_supported(const WgradArgs& a, int mode) {
  return mode == MODE_FWD && a.SC == 1 && a.K < kSmallMaxK && a.N % 8 == 0 && a.N <= kSmallMaxN &&
         a.N * (a.K + 1) <= 8 * 256 && a.ldd % 8 == 0 && ((uintptr_t)a.dy & 15) == 0 && a.OH > 0 && a.OW > 0 &&
         (!a.with_bias || a.gb != nullptr);
}

hipError_t smallc_wgrad(const WgradArgs& a, float* ws, size_t ws_floats, hipStream_t st) {
  const int Kt = a.K + (a.with_bias ? 1 : 0);
  const int P = a.N * Kt;
  int grid = min(cdiv(a.M, 64), 1024);
  while (grid > 1 && (size_t)grid * P > ws_floats) grid /= 2;
  const FastDiv d_ow = make_fastdiv((unsigned)a.OW), d_ohw = make_fastdiv((unsigned)(a.OH * a.OW));
  hipLaunchKernelGGL(smallc_wgrad_kernel, dim3(grid), dim3(256), 0, st, a, d_ow, d_ohw, ws);
  DFA_HIP_CHECK(hipGetLastError());
  return slab_reduce(ws, a.gw, a.with_bias ? a.gb : nullptr, a.N, a.K, Kt, grid, a.scale, st);
}

}  // namespace dfa
