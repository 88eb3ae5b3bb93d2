// Generic Keras layer kernels (gfx950): elementwise activations that cannot fold into a producer's
// epilogue, sigmoid cross-entropy on logits, and general 2-D pooling (max / average, any window and
// stride, 'valid' or 'same' padding).
//
// The reference accepts any tf.LayersModel fetched by URL (/root/reference/src/common/utils.ts:236-244,
// src/common/models.ts:92-100) and its loss registry includes sigmoidCrossEntropy (utils.ts:19-30), so
// the engine must train models beyond the MNIST CNN's relu/softmax/2x2-max-pool set.  These kernels are
// the general path; the fused kernels (lenet_fused, kcnn_fused, igemm64 pooled epilogues) keep the hot
// shapes.  All of them are memory-bound streaming passes: 16-byte (8 x bf16) accesses where the
// element count allows, grid-stride loops sized for 256 CUs.
#include "common.h"
#include "kernels.h"

namespace dfa {
namespace {

__device__ __forceinline__ float act_f(int kind, float x) {
  switch (kind) {
    case kActRelu: return fmaxf(x, 0.f);
    case kActRelu6: return fminf(fmaxf(x, 0.f), 6.f);
    case kActSigmoid: return 1.f / (1.f + __expf(-x));
    case kActTanh: return tanhf(x);
    case kActElu: return x > 0.f ? x : __expf(x) - 1.f;
    case kActSelu: {
      const float a = 1.6732632423543772f, s = 1.0507009873554805f;
      return s * (x > 0.f ? x : a * (__expf(x) - 1.f));
    }
    case kActSoftplus: return x > 20.f ? x : log1pf(__expf(x));
    case kActSoftsign: return x / (1.f + fabsf(x));
    case kActHardSigmoid: return fminf(fmaxf(0.2f * x + 0.5f, 0.f), 1.f);
    case kActSwish: return x / (1.f + __expf(-x));
    case kActExp: return __expf(x);
    default: return x;  // linear
  }
}

// d act / dx at the activation's input x
__device__ __forceinline__ float act_df(int kind, float x) {
  switch (kind) {
    case kActRelu: return x > 0.f ? 1.f : 0.f;
    case kActRelu6: return (x > 0.f && x < 6.f) ? 1.f : 0.f;
    case kActSigmoid: {
      const float s = 1.f / (1.f + __expf(-x));
      return s * (1.f - s);
    }
    case kActTanh: {
      const float t = tanhf(x);
      return 1.f - t * t;
    }
    case kActElu: return x > 0.f ? 1.f : __expf(x);
    case kActSelu: {
      const float a = 1.6732632423543772f, s = 1.0507009873554805f;
      return x > 0.f ? s : s * a * __expf(x);
    }
    case kActSoftplus: return 1.f / (1.f + __expf(-x));
    case kActSoftsign: {
      const float d = 1.f + fabsf(x);
      return 1.f / (d * d);
    }
    case kActHardSigmoid: return (x > -2.5f && x < 2.5f) ? 0.2f : 0.f;
    case kActSwish: {
      const float s = 1.f / (1.f + __expf(-x));
      return s + x * s * (1.f - s);
    }
    case kActExp: return __expf(x);
    default: return 1.f;
  }
}

// y = act(x); 8 elements per thread (n % 8 == 0) or 1
template <bool VEC>
__global__ void act_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long long n, int kind) {
  const long long m = VEC ? n / 8 : n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < m; i += (long long)gridDim.x * blockDim.x) {
    if (VEC) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + 8 * i);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(act_f(kind, (float)v[j]));
      *reinterpret_cast<bf16x8*>(y + 8 * i) = o;
    } else {
      y[i] = f2bf(act_f(kind, (float)x[i]));
    }
  }
}

// dx = dy * act'(x) [* relu'(x): the activation's input is itself a fused-ReLU output]
template <bool VEC>
__global__ void act_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy, bf16* __restrict__ dx,
                               long long n, int kind, int in_relu) {
  const long long m = VEC ? n / 8 : n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < m; i += (long long)gridDim.x * blockDim.x) {
    if (VEC) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + 8 * i);
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(dy + 8 * i);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = (float)v[j];
        float d = (float)g[j] * act_df(kind, xv);
        if (in_relu && !(xv > 0.f)) d = 0.f;
        o[j] = f2bf(d);
      }
      *reinterpret_cast<bf16x8*>(dx + 8 * i) = o;
    } else {
      const float xv = (float)x[i];
      float d = (float)dy[i] * act_df(kind, xv);
      if (in_relu && !(xv > 0.f)) d = 0.f;
      dx[i] = f2bf(d);
    }
  }
}

// Sigmoid cross-entropy on fp32 logits against one-hot(label) targets, summed over classes:
//   loss_b = sum_c max(z,0) - z t + log(1 + exp(-|z|)),  dlogits = (sigmoid(z) - t) * grad_scale.
// One row per thread; stats[0] += loss, stats[1] += (argmax == label) with one atomic per workgroup.
__global__ void sigmoid_ce_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                                  bf16* __restrict__ dlogits, float* __restrict__ stats, int B, int C, int ldl,
                                  int ldg, float grad_scale) {
  __shared__ float s_loss[4], s_corr[4];
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  float loss = 0.f, corr = 0.f;
  if (b < B) {
    const float* z = logits + (long long)b * ldl;
    const int y = min(max(labels[b], 0), C - 1);
    float mx = -INFINITY;
    int am = 0;
    for (int c = 0; c < C; ++c) {
      const float v = z[c];
      if (v > mx) { mx = v; am = c; }
      const float t = c == y ? 1.f : 0.f;
      loss += fmaxf(v, 0.f) - v * t + log1pf(__expf(-fabsf(v)));
      if (dlogits) dlogits[(long long)b * ldg + c] = f2bf((1.f / (1.f + __expf(-v)) - t) * grad_scale);
    }
    corr = am == y ? 1.f : 0.f;
  }
  loss = wave_sum(loss);
  corr = wave_sum(corr);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { s_loss[wid] = loss; s_corr[wid] = corr; }
  __syncthreads();
  if (threadIdx.x == 0 && stats) {
    float l = 0.f, c = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { l += s_loss[w]; c += s_corr[w]; }
    atomicAdd(&stats[0], l);
    atomicAdd(&stats[1], c);
  }
}

// General 2-D pooling, NHWC bf16, one thread per output element (8 channels when C % 8 == 0).
// Window of output (oh, ow): rows oh*sh - pt .. + ph - 1, cols ow*sw - pl .. + pw - 1, clipped to the
// image ('same' padding never contributes: max ignores it, average divides by the in-image count, as
// TensorFlow / tf.js do).
template <bool VEC, bool AVG>
__global__ void pool2d_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, Pool2DGeom g) {
  const int CC = VEC ? g.C / 8 : g.C;
  const long long total = (long long)g.B * g.OH * g.OW * CC;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    long long t = i / CC;
    const int ow = (int)(t % g.OW);
    t /= g.OW;
    const int oh = (int)(t % g.OH);
    const long long b = t / g.OH;
    const int h0 = max(oh * g.sh - g.pt, 0), h1 = min(oh * g.sh - g.pt + g.ph, g.H);
    const int w0 = max(ow * g.sw - g.pl, 0), w1 = min(ow * g.sw - g.pl + g.pw, g.W);
    const float inv = (h1 > h0 && w1 > w0) ? 1.f / (float)((h1 - h0) * (w1 - w0)) : 0.f;
    float m[VEC ? 8 : 1];
#pragma unroll
    for (int j = 0; j < (VEC ? 8 : 1); ++j) m[j] = AVG ? 0.f : -INFINITY;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) {
        const bf16* p = x + ((b * g.H + h) * g.W + w) * g.C;
        if (VEC) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(p + 8 * cc);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = AVG ? m[j] + (float)v[j] : fmaxf(m[j], (float)v[j]);
        } else {
          const float v = (float)p[cc];
          m[0] = AVG ? m[0] + v : fmaxf(m[0], v);
        }
      }
    if (VEC) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(AVG ? m[j] * inv : (h1 > h0 && w1 > w0 ? m[j] : 0.f));
      *reinterpret_cast<bf16x8*>(y + 8 * i) = o;
    } else {
      y[i] = f2bf(AVG ? m[0] * inv : (h1 > h0 && w1 > w0 ? m[0] : 0.f));
    }
  }
}

// Backward, input-centric (no atomics, overlapping windows allowed): dx(h, w) sums the windows that
// contain (h, w); a max window passes its gradient to its FIRST maximum only (row-major scan), as the
// forward's comparison order defines.  ``in_relu``: the pooled input is a fused-ReLU output, so a
// window whose max is not positive passes nothing.
template <bool AVG>
__global__ void pool2d_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                  Pool2DGeom g, int in_relu) {
  const long long total = (long long)g.B * g.H * g.W * g.C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    long long t = i / g.C;
    const int w = (int)(t % g.W);
    t /= g.W;
    const int h = (int)(t % g.H);
    const long long b = t / g.H;
    // output windows containing row h: oh*sh - pt <= h < oh*sh - pt + ph
    const int oh_lo = max(0, (h + g.pt - g.ph + g.sh) / g.sh), oh_hi = min(g.OH - 1, (h + g.pt) / g.sh);
    const int ow_lo = max(0, (w + g.pl - g.pw + g.sw) / g.sw), ow_hi = min(g.OW - 1, (w + g.pl) / g.sw);
    const float xv = (float)x[i];
    float acc = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int h0 = max(oh * g.sh - g.pt, 0), h1 = min(oh * g.sh - g.pt + g.ph, g.H);
      if (h < h0 || h >= h1) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int w0 = max(ow * g.sw - g.pl, 0), w1 = min(ow * g.sw - g.pl + g.pw, g.W);
        if (w < w0 || w >= w1) continue;
        const float gy = (float)dy[((b * g.OH + oh) * g.OW + ow) * g.C + c];
        if (AVG) {
          acc += gy / (float)((h1 - h0) * (w1 - w0));
        } else {
          // first maximum of the window
          float mx = -INFINITY;
          int ah = -1, aw = -1;
          for (int hh = h0; hh < h1; ++hh)
            for (int ww = w0; ww < w1; ++ww) {
              const float v = (float)x[((b * g.H + hh) * g.W + ww) * g.C + c];
              if (v > mx) { mx = v; ah = hh; aw = ww; }
            }
          if (ah == h && aw == w && (!in_relu || mx > 0.f)) acc += gy;
        }
      }
    }
    if (AVG && in_relu && !(xv > 0.f)) acc = 0.f;
    dx[i] = f2bf(acc);
  }
}

int grid_of(long long total) {
  long long g = (total + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace

hipError_t act_fwd(const bf16* x, bf16* y, long long n, int kind, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n % 8 == 0)
    hipLaunchKernelGGL(act_fwd_kernel<true>, dim3(grid_of(n / 8)), dim3(256), 0, st, x, y, n, kind);
  else
    hipLaunchKernelGGL(act_fwd_kernel<false>, dim3(grid_of(n)), dim3(256), 0, st, x, y, n, kind);
  return hipGetLastError();
}

hipError_t act_bwd(const bf16* x, const bf16* dy, bf16* dx, long long n, int kind, int in_relu, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n % 8 == 0)
    hipLaunchKernelGGL(act_bwd_kernel<true>, dim3(grid_of(n / 8)), dim3(256), 0, st, x, dy, dx, n, kind, in_relu);
  else
    hipLaunchKernelGGL(act_bwd_kernel<false>, dim3(grid_of(n)), dim3(256), 0, st, x, dy, dx, n, kind, in_relu);
  return hipGetLastError();
}

hipError_t sigmoid_ce(const float* logits, const int* labels, bf16* dlogits, float* stats, int B, int C, int ldl,
                      int ldg, float grad_scale, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(sigmoid_ce_kernel, dim3(cdiv(B, 256)), dim3(256), 0, st, logits, labels, dlogits, stats, B, C,
                     ldl, ldg, grad_scale);
  return hipGetLastError();
}

hipError_t pool2d_fwd(const bf16* x, bf16* y, const Pool2DGeom& g, int avg, hipStream_t st) {
  if (g.ph < 1 || g.pw < 1 || g.sh < 1 || g.sw < 1 || g.OH < 1 || g.OW < 1) return hipErrorInvalidValue;
  const bool vec = g.C % 8 == 0;
  const long long total = (long long)g.B * g.OH * g.OW * (vec ? g.C / 8 : g.C);
  if (total == 0) return hipSuccess;
  const dim3 grid(grid_of(total)), block(256);
  if (vec && avg) hipLaunchKernelGGL((pool2d_fwd_kernel<true, true>), grid, block, 0, st, x, y, g);
  else if (vec) hipLaunchKernelGGL((pool2d_fwd_kernel<true, false>), grid, block, 0, st, x, y, g);
  else if (avg) hipLaunchKernelGGL((pool2d_fwd_kernel<false, true>), grid, block, 0, st, x, y, g);
  else hipLaunchKernelGGL((pool2d_fwd_kernel<false, false>), grid, block, 0, st, x, y, g);
  return hipGetLastError();
}

hipError_t pool2d_bwd(const bf16* x, const bf16* dy, bf16* dx, const Pool2DGeom& g, int avg, int in_relu,
                      hipStream_t st) {
  if (g.ph < 1 || g.pw < 1 || g.sh < 1 || g.sw < 1) return hipErrorInvalidValue;
  const long long total = (long long)g.B * g.H * g.W * g.C;
  if (total == 0) return hipSuccess;
  if (avg)
    hipLaunchKernelGGL(pool2d_bwd_kernel<true>, dim3(grid_of(total)), dim3(256), 0, st, x, dy, dx, g, in_relu);
  else
    hipLaunchKernelGGL(pool2d_bwd_kernel<false>, dim3(grid_of(total)), dim3(256), 0, st, x, dy, dx, g, in_relu);
  return hipGetLastError();
}

}  // namespace dfa
