// BatchNorm (NHWC, per-channel over M = B*H*W rows) for the CIFAR-10 ResNet-18 config
// (BASELINE.json configs[3]; not present in the reference).
//
// Train forward = 3 launches: per-block partial sums (fp32, 16-byte vector loads) ->
// single-block finalize in fp64 (mean, invstd, running-stat update) -> normalize(+ReLU).
// Backward = 3 launches: partial (sum g, sum g*xhat) with relu' fused -> finalize (writes dgamma,
// dbeta straight into the flat gradient buffer) -> dx.  Partial slabs keep the reduction
// deterministic (no float atomics).
#include "common.h"
#include "kernels.h"

namespace dfa {

constexpr int BN_MAX_G = 255;

static int bn_grid(int M, int rpp) {
  int g = cdiv(M, rpp * 16);
  if (g > BN_MAX_G) g = BN_MAX_G;
  if (g < 1) g = 1;
  return g;
}

// mode 0: s += x, q += x*x ; mode 1: g = dy*relu'(y), xh = (x-mean)*invstd ; s += g, q += g*xh
template <int MODE, bool VEC>
__global__ void __launch_bounds__(256) bn_partial_kernel(const bf16* __restrict__ x, const bf16* __restrict__ y,
                                                         const bf16* __restrict__ dy, const float* __restrict__ mean,
                                                         const float* __restrict__ invstd, float* __restrict__ ws,
                                                         int M, int C, int relu) {
  __shared__ float ls[2048], lq[2048];
  constexpr int W = VEC ? 8 : 1;
  const int cpr = C / W;
  const int rpp = 256 / cpr;
  const int t = threadIdx.x;
  const int chunk = t % cpr, rsub = t / cpr;
  float s[W], q[W], mu[W], is[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    s[j] = 0.f; q[j] = 0.f;
    if (MODE == 1) { mu[j] = mean[chunk * W + j]; is[j] = invstd[chunk * W + j]; }
  }
  if (rsub < rpp) {
    for (long long r = (long long)blockIdx.x * rpp + rsub; r < M; r += (long long)gridDim.x * rpp) {
      const long long o = r * C + chunk * W;
      float xv[W], gv[W];
      if (VEC) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + o);
#pragma unroll
        for (int j = 0; j < W; ++j) xv[j] = (float)v[j];
        if (MODE == 1) {
          const bf16x8 g = *reinterpret_cast<const bf16x8*>(dy + o);
          const bf16x8 yy = *reinterpret_cast<const bf16x8*>(y + o);
#pragma unroll
          for (int j = 0; j < W; ++j) gv[j] = (relu && !((float)yy[j] > 0.f)) ? 0.f : (float)g[j];
        }
      } else {
        xv[0] = (float)x[o];
        if (MODE == 1) gv[0] = (relu && !((float)y[o] > 0.f)) ? 0.f : (float)dy[o];
      }
#pragma unroll
      for (int j = 0; j < W; ++j) {
        if (MODE == 0) {
          s[j] += xv[j];
          q[j] += xv[j] * xv[j];
        } else {
          const float xh = (xv[j] - mu[j]) * is[j];
          s[j] += gv[j];
          q[j] += gv[j] * xh;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
      ls[rsub * C + chunk * W + j] = s[j];
      lq[rsub * C + chunk * W + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rpp; ++r) { a += ls[r * C + c]; b += lq[r * C + c]; }
    ws[(long long)blockIdx.x * 2 * C + c] = a;
    ws[(long long)blockIdx.x * 2 * C + C + c] = b;
  }
}

__global__ void bn_fwd_finalize_kernel(const float* __restrict__ ws, int G, int M, int C, float momentum, float eps,
                                       float* __restrict__ mean, float* __restrict__ invstd,
                                       float* __restrict__ run_mean, float* __restrict__ run_var) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s = 0.0, q = 0.0;
    for (int g = 0; g < G; ++g) { s += ws[(long long)g * 2 * C + c]; q += ws[(long long)g * 2 * C + C + c]; }
    const double mu = s / M;
    double var = q / M - mu * mu;
    if (var < 0.0) var = 0.0;
    mean[c] = (float)mu;
    invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
      const double unb = M > 1 ? var * M / (M - 1) : var;
      run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mu);
      run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
    }
  }
}

__global__ void bn_bwd_finalize_kernel(float* __restrict__ ws, int G, int C, float gscale, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s = 0.0, q = 0.0;
    for (int g = 0; g < G; ++g) { s += ws[(long long)g * 2 * C + c]; q += ws[(long long)g * 2 * C + C + c]; }
    ws[(long long)G * 2 * C + c] = (float)s;       // raw sums for the dx pass
    ws[(long long)G * 2 * C + C + c] = (float)q;
    dbeta[c] = (float)s * gscale;
    dgamma[c] = (float)q * gscale;
  }
}

// mode 0 (train/eval fwd): y = (x - a) * b * gamma + beta (+relu), with (a, b) = (mean, invstd)
template <bool VEC>
__global__ void bn_apply_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const float* __restrict__ mean,
                                const float* __restrict__ invstd, int eval_var, float eps, long long M, int C,
                                int relu) {
  constexpr int W = VEC ? 8 : 1;
  const long long total = M * C / W;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c0 = (int)((i * W) % C);
    float xv[W];
    if (VEC) {
      const bf16x8 v = reinterpret_cast<const bf16x8*>(x)[i];
#pragma unroll
      for (int j = 0; j < W; ++j) xv[j] = (float)v[j];
    } else {
      xv[0] = (float)x[i];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const int c = c0 + j;
      const float is = eval_var ? rsqrtf(invstd[c] + eps) : invstd[c];
      float v = (xv[j] - mean[c]) * is * gamma[c] + beta[c];
      if (relu) v = fmaxf(v, 0.f);
      o[j] = f2bf(v);
    }
    if (VEC)
      reinterpret_cast<bf16x8*>(y)[i] = o;
    else
      y[i] = o[0];
  }
}

template <bool VEC>
__global__ void bn_dx_kernel(const bf16* __restrict__ x, const bf16* __restrict__ y, const bf16* __restrict__ dy,
                             bf16* __restrict__ dx, const float* __restrict__ gamma, const float* __restrict__ mean,
                             const float* __restrict__ invstd, const float* __restrict__ sums, long long M, int C,
                             int relu) {
  constexpr int W = VEC ? 8 : 1;
  const long long total = M * C / W;
  const float invM = 1.f / (float)M;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c0 = (int)((i * W) % C);
    float xv[W], gv[W];
    if (VEC) {
      const bf16x8 v = reinterpret_cast<const bf16x8*>(x)[i];
      const bf16x8 g = reinterpret_cast<const bf16x8*>(dy)[i];
      const bf16x8 yy = reinterpret_cast<const bf16x8*>(y)[i];
#pragma unroll
      for (int j = 0; j < W; ++j) {
        xv[j] = (float)v[j];
        gv[j] = (relu && !((float)yy[j] > 0.f)) ? 0.f : (float)g[j];
      }
    } else {
      xv[0] = (float)x[i];
      gv[0] = (relu && !((float)y[i] > 0.f)) ? 0.f : (float)dy[i];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const int c = c0 + j;
      const float is = invstd[c];
      const float xh = (xv[j] - mean[c]) * is;
      const float v = gamma[c] * is * (gv[j] - sums[c] * invM - xh * sums[C + c] * invM);
      o[j] = f2bf(v);
    }
    if (VEC)
      reinterpret_cast<bf16x8*>(dx)[i] = o;
    else
      dx[i] = o[0];
  }
}

static int ew_grid(long long n) {
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

hipError_t bn_fwd_train(const bf16* x, bf16* y, const float* gamma, const float* beta, float* mean, float* invstd,
                        float* run_mean, float* run_var, float* ws, int M, int C, float momentum, float eps, int relu,
                        hipStream_t st) {
  if (C > 2048 || M <= 0) return hipErrorInvalidValue;
  const bool vec = C % 8 == 0 && C / 8 <= 256;
  if (!vec && C > 256) return hipErrorInvalidValue;
  const int rpp = 256 / (vec ? C / 8 : C);
  const int G = bn_grid(M, rpp);
  if (vec)
    hipLaunchKernelGGL((bn_partial_kernel<0, true>), dim3(G), dim3(256), 0, st, x, nullptr, nullptr, nullptr, nullptr,
                       ws, M, C, 0);
  else
    hipLaunchKernelGGL((bn_partial_kernel<0, false>), dim3(G), dim3(256), 0, st, x, nullptr, nullptr, nullptr, nullptr,
                       ws, M, C, 0);
  DFA_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(1), dim3(256), 0, st, ws, G, M, C, momentum, eps, mean, invstd,
                     run_mean, run_var);
  DFA_HIP_CHECK(hipGetLastError());
  const long long n = (long long)M * C / (vec ? 8 : 1);
  if (vec)
    hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(ew_grid(n)), dim3(256), 0, st, x, y, gamma, beta, mean, invstd, 0,
                       eps, (long long)M, C, relu);
  else
    hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(ew_grid(n)), dim3(256), 0, st, x, y, gamma, beta, mean, invstd, 0,
                       eps, (long long)M, C, relu);
  return hipGetLastError();
}

hipError_t bn_fwd_eval(const bf16* x, bf16* y, const float* gamma, const float* beta, const float* run_mean,
                       const float* run_var, int M, int C, float eps, int relu, hipStream_t st) {
  const bool vec = C % 8 == 0;
  const long long n = (long long)M * C / (vec ? 8 : 1);
  if (vec)
    hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(ew_grid(n)), dim3(256), 0, st, x, y, gamma, beta, run_mean, run_var,
                       1, eps, (long long)M, C, relu);
  else
    hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(ew_grid(n)), dim3(256), 0, st, x, y, gamma, beta, run_mean,
                       run_var, 1, eps, (long long)M, C, relu);
  return hipGetLastError();
}

hipError_t bn_bwd(const bf16* x, const bf16* y, const bf16* dy, bf16* dx, const float* gamma, const float* beta,
                  const float* mean, const float* invstd, float* dgamma, float* dbeta, float* ws, int M, int C,
                  int relu, float gscale, hipStream_t st) {
  (void)beta;
  if (C > 2048 || M <= 0) return hipErrorInvalidValue;
  const bool vec = C % 8 == 0 && C / 8 <= 256;
  if (!vec && C > 256) return hipErrorInvalidValue;
  const int rpp = 256 / (vec ? C / 8 : C);
  const int G = bn_grid(M, rpp);
  if (vec)
    hipLaunchKernelGGL((bn_partial_kernel<1, true>), dim3(G), dim3(256), 0, st, x, y, dy, mean, invstd, ws, M, C, relu);
  else
    hipLaunchKernelGGL((bn_partial_kernel<1, false>), dim3(G), dim3(256), 0, st, x, y, dy, mean, invstd, ws, M, C,
                       relu);
  DFA_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(1), dim3(256), 0, st, ws, G, C, gscale, dgamma, dbeta);
  DFA_HIP_CHECK(hipGetLastError());
  const float* sums = ws + (long long)G * 2 * C;
  const long long n = (long long)M * C / (vec ? 8 : 1);
  if (vec)
    hipLaunchKernelGGL(bn_dx_kernel<true>, dim3(ew_grid(n)), dim3(256), 0, st, x, y, dy, dx, gamma, mean, invstd, sums,
                       (long long)M, C, relu);
  else
    hipLaunchKernelGGL(bn_dx_kernel<false>, dim3(ew_grid(n)), dim3(256), 0, st, x, y, dy, dx, gamma, mean, invstd,
                       sums, (long long)M, C, relu);
  return hipGetLastError();
}

}  // namespace dfa
