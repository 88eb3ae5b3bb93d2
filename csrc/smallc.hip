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

// ---- 3x3 single-channel conv, 32 output channels (the Keras CNN's conv1): image-resident variants.
// A workgroup owns C1_IMGS whole images, staged once into LDS as fp32 with a zero border, so every
// tap is an unchecked LDS read (4 threads of a pixel read the same word: broadcast; neighbouring
// pixels read neighbouring words: conflict free).  Thread (ps = t >> 2, g = t & 3) owns output
// channels 8g..8g+7 of pixels ps, ps + 64, ...: its 72 weights live in registers.
//   forward: 72 FMA + one 16-byte store per (pixel, g); a wave writes 16 whole 64-byte pixel rows
//   wgrad  : 80 fp32 accumulators (8 channels x (9 taps + bias)) per thread over the workgroup's
//            pixels, four dY rows in flight per thread; wave reduction by lane shuffles, workgroup
//            reduction in LDS, one slab [32][10] per workgroup for slab_reduce (fixed order)
constexpr int C1_IMGS = 2, C1_N = 32, C1_MAXP = 34 * 34;

__device__ __forceinline__ void c1_stage(const bf16* __restrict__ src, int b0, int nimg, int SH, int SW, int pad,
                                         float* xs) {
  const int SWp = SW + 2 * pad, HWp = (SH + 2 * pad) * SWp;
  for (int i = threadIdx.x; i < C1_IMGS * HWp; i += 256) {
    const int im = i / HWp, r = i - im * HWp;
    const int y = r / SWp - pad, x = r - (r / SWp) * SWp - pad;
    float v = 0.f;
    if (im < nimg && (unsigned)y < (unsigned)SH && (unsigned)x < (unsigned)SW)
      v = (float)src[((long long)(b0 + im) * SH + y) * SW + x];
    xs[im * C1_MAXP + r] = v;
  }
}

__global__ void __launch_bounds__(256) c1_fwd_kernel(IGemmArgs a, int B, FastDiv d_ow) {
  __shared__ float xs[C1_IMGS * C1_MAXP];
  const int b0 = blockIdx.x * C1_IMGS, nimg = min(C1_IMGS, B - b0);
  const int g = threadIdx.x & 3, ps = threadIdx.x >> 2;
  float w[8][9], bias[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int k = 0; k < 9; ++k) w[j][k] = (float)a.w[(long long)(8 * g + j) * a.Kpad + k];
    bias[j] = a.bias ? a.bias[8 * g + j] : 0.f;
  }
  c1_stage(a.src, b0, nimg, a.SH, a.SW, a.pad, xs);
  __syncthreads();
  const int SWp = a.SW + 2 * a.pad, P = a.OH * a.OW;
  for (int im = 0; im < nimg; ++im) {
    const float* xi = xs + im * C1_MAXP;
    bf16* ob = reinterpret_cast<bf16*>(a.out) + (long long)(b0 + im) * P * a.ldc + 8 * g;
    for (int p = ps; p < P; p += 64) {
      const int oh = (int)fdiv((unsigned)p, d_ow), ow = p - oh * a.OW;
      const float* x0 = xi + oh * SWp + ow;
      float xv[9];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) xv[3 * ky + kx] = x0[ky * SWp + kx];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) acc = fmaf(xv[k], w[j][k], acc);
        float v = acc * a.alpha + bias[j];
        if (a.relu) v = fmaxf(v, 0.f);
        o[j] = f2bf(v);
      }
      *reinterpret_cast<bf16x8*>(ob + (long long)p * a.ldc) = o;
    }
  }
}

__global__ void __launch_bounds__(256) c1_wgrad_kernel(WgradArgs a, int B, FastDiv d_ow, float* slabs) {
  __shared__ float xs[C1_IMGS * C1_MAXP];
  __shared__ float red[4][4][80];
  const int b0 = blockIdx.x * C1_IMGS, nimg = min(C1_IMGS, B - b0);
  const int g = threadIdx.x & 3, ps = threadIdx.x >> 2;
  c1_stage(a.src, b0, nimg, a.SH, a.SW, a.pad, xs);
  __syncthreads();
  float acc[8][10];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[j][k] = 0.f;
  const int SWp = a.SW + 2 * a.pad, P = a.OH * a.OW;
  constexpr int U = 4;
  for (int im = 0; im < nimg; ++im) {
    const float* xi = xs + im * C1_MAXP;
    const bf16* db = a.dy + (long long)(b0 + im) * P * a.ldd + 8 * g;
    for (int p0 = ps; p0 < P; p0 += 64 * U) {
      bf16x8 dv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = min(p0 + 64 * u, P - 1);
        dv[u] = *reinterpret_cast<const bf16x8*>(db + (long long)p * a.ldd);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + 64 * u;
        if (p >= P) break;
        const int oh = (int)fdiv((unsigned)p, d_ow), ow = p - oh * a.OW;
        const float* x0 = xi + oh * SWp + ow;
        float xv[9];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) xv[3 * ky + kx] = x0[ky * SWp + kx];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (float)dv[u][j];
#pragma unroll
          for (int k = 0; k < 9; ++k) acc[j][k] = fmaf(d, xv[k], acc[j][k]);
          acc[j][9] += d;
        }
      }
    }
  }
  // lanes sharing g: xor over lane bits 2..5
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      float v = acc[j][k];
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      acc[j][k] = v;
    }
  if (lane < 4) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int k = 0; k < 10; ++k) red[wid][lane][j * 10 + k] = acc[j][k];
  }
  __syncthreads();
  const int Kt = a.with_bias ? 10 : 9;
  for (int t = threadIdx.x; t < C1_N * Kt; t += 256) {
    const int n = t / Kt, k = t - n * Kt;
    const int gg = n >> 3, j = n & 7;
    const float v = red[0][gg][j * 10 + k] + red[1][gg][j * 10 + k] + red[2][gg][j * 10 + k] + red[3][gg][j * 10 + k];
    slabs[(long long)blockIdx.x * C1_N * Kt + t] = v;
  }
}

bool c1_ok(int SC, int KH, int KW, int stride, int pad, int N, int SH, int SW) {
  return SC == 1 && KH == 3 && KW == 3 && stride == 1 && N == C1_N && pad >= 0 && pad <= 1 &&
         (SH + 2 * pad) <= 34 && (SW + 2 * pad) <= 34;
}

}  // namespace

bool smallc_fwd_supported(const IGemmArgs& a, int mode) {
  return mode == MODE_FWD && a.SC == 1 && a.K <= kSmallMaxK && a.N % 8 == 0 && a.N <= kSmallMaxN && !a.mask &&
         !a.res && a.ldc % 8 == 0 && ((uintptr_t)a.out & 15) == 0 && a.OH > 0 && a.OW > 0;
}

hipError_t smallc_fwd(const IGemmArgs& a, hipStream_t st) {
  const FastDiv d_ow = make_fastdiv((unsigned)a.OW), d_ohw = make_fastdiv((unsigned)(a.OH * a.OW));
  if (c1_ok(a.SC, a.KH, a.KW, a.stride, a.pad, a.N, a.SH, a.SW) && !a.out_f32 && a.K == 9) {
    const int B = a.M / (a.OH * a.OW);
    hipLaunchKernelGGL(c1_fwd_kernel, dim3(cdiv(B, C1_IMGS)), dim3(256), 0, st, a, B, d_ow);
    return hipGetLastError();
  }
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
  if (c1_ok(a.SC, a.KH, a.KW, a.stride, a.pad, a.N, a.SH, a.SW) && a.K == 9) {
    const int B = a.M / (a.OH * a.OW);
    const int nb = cdiv(B, C1_IMGS);
    if ((size_t)nb * P <= ws_floats) {
      hipLaunchKernelGGL(c1_wgrad_kernel, dim3(nb), dim3(256), 0, st, a, B, make_fastdiv((unsigned)a.OW), ws);
      DFA_HIP_CHECK(hipGetLastError());
      return slab_reduce(ws, a.gw, a.with_bias ? a.gb : nullptr, a.N, a.K, Kt, nb, a.scale, st);
    }
  }
  int grid = min(cdiv(a.M, 64), 1024);
  while (grid > 1 && (size_t)grid * P > ws_floats) grid /= 2;
  const FastDiv d_ow = make_fastdiv((unsigned)a.OW), d_ohw = make_fastdiv((unsigned)(a.OH * a.OW));
  hipLaunchKernelGGL(smallc_wgrad_kernel, dim3(grid), dim3(256), 0, st, a, d_ow, d_ohw, ws);
  DFA_HIP_CHECK(hipGetLastError());
  return slab_reduce(ws, a.gw, a.with_bias ? a.gb : nullptr, a.N, a.K, Kt, grid, a.scale, st);
}

}  // namespace dfa
