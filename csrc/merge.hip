// Keras merge layers of functional (branching) graphs, gfx950: Add, Subtract, Multiply, Average,
// Maximum, Minimum and Concatenate (channels, the last axis), forward and the per-input gradients.
//
// The reference loads any tf.LayersModel (/root/reference/src/common/utils.ts:236-244,
// src/common/models.ts:92-100); Keras functional models join branches with these layers.  They are
// memory-bound streaming passes over bf16 NHWC tensors: one launch per merge node and direction, every
// input / gradient pointer in the kernel argument (up to kMergeMaxIn), grid-stride over the output
// elements.  Numerics follow the per-element fp32 formula with one bf16 rounding of the result (the
// product and the average in the written input order), like the elementwise kernels of csrc/act.hip.
#include "common.h"
#include "kernels.h"

namespace dfa {
namespace {

constexpr int kMT = 256;

__device__ __forceinline__ float ldf(const bf16* p, long long i) { return (float)p[i]; }

__global__ void __launch_bounds__(kMT) merge_fwd_kernel(MergeArgs a) {
  const long long total = a.rows * (long long)a.cout;
  for (long long e = blockIdx.x * (long long)kMT + threadIdx.x; e < total; e += (long long)gridDim.x * kMT) {
    float v = 0.f;
    if (a.kind == kMergeConcat) {
      const long long r = e / a.cout;
      const int c = (int)(e - r * a.cout);
#pragma unroll
      for (int i = 0, b = 0; i < kMergeMaxIn; ++i) {  // input i holds channels [b, b + w[i])
        if (i < a.n) {
          if (c >= b && c < b + a.w[i]) v = ldf(a.in[i], r * a.w[i] + (c - b));
          b += a.w[i];
        }
      }
    } else {
      v = ldf(a.in[0], e);
#pragma unroll
      for (int i = 1; i < kMergeMaxIn; ++i) {
        if (i >= a.n) break;
        const float x = ldf(a.in[i], e);
        switch (a.kind) {
          case kMergeAdd: case kMergeAverage: v += x; break;
          case kMergeSubtract: v -= x; break;
          case kMergeMultiply: v *= x; break;
          case kMergeMaximum: v = fmaxf(v, x); break;
          case kMergeMinimum: v = fminf(v, x); break;
          default: break;
        }
      }
      if (a.kind == kMergeAverage) v *= 1.f / (float)a.n;
    }
    a.out[e] = f2bf(v);
  }
}

// gradient of input j = blockIdx.y: d out / d in_j * dy
__global__ void __launch_bounds__(kMT) merge_bwd_kernel(MergeArgs a) {
  const int j = blockIdx.y;
  bf16* gj = nullptr;
  int wj = 0, off = 0;
#pragma unroll
  for (int i = 0; i < kMergeMaxIn; ++i)
    if (i < a.n) {
      if (i == j) {
        gj = a.grad[i];
        wj = a.w[i];
      } else if (i < j) {
        off += a.w[i];
      }
    }
  if (gj == nullptr) return;
  const long long total = a.kind == kMergeConcat ? a.rows * (long long)wj : a.rows * (long long)a.cout;
  for (long long e = blockIdx.x * (long long)kMT + threadIdx.x; e < total; e += (long long)gridDim.x * kMT) {
    float g;
    if (a.kind == kMergeConcat) {
      const long long r = e / wj;
      g = ldf(a.dy, r * a.cout + off + (e - r * wj));
    } else {
      const float dy = ldf(a.dy, e);
      switch (a.kind) {
        case kMergeAdd: g = dy; break;
        case kMergeAverage: g = dy * (1.f / (float)a.n); break;
        case kMergeSubtract: g = j == 0 ? dy : -dy; break;
        case kMergeMultiply: {
          float p = 1.f;
#pragma unroll
          for (int i = 0; i < kMergeMaxIn; ++i)
            if (i < a.n && i != j) p *= ldf(a.in[i], e);
          g = dy * p;
          break;
        }
        default: {  // maximum / minimum: the gradient goes to the first input holding the extreme value
          const float xj = ldf(a.in[j], e);
          bool first = true;
#pragma unroll
          for (int i = 0; i < kMergeMaxIn; ++i) {
            if (i >= a.n) break;
            const float x = ldf(a.in[i], e);
            const bool better = a.kind == kMergeMaximum ? x > xj : x < xj;
            if (better || (i < j && x == xj)) first = false;
          }
          g = first ? dy : 0.f;
          break;
        }
      }
    }
    gj[e] = f2bf(g);
  }
}

int merge_grid(long long total) {
  long long g = (total + kMT - 1) / kMT;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

}  // namespace

hipError_t merge_fwd(const MergeArgs& a, hipStream_t st) {
  if (a.n < 1 || a.n > kMergeMaxIn || a.rows <= 0 || a.cout <= 0 || !a.out) return hipErrorInvalidValue;
  if (a.kind == kMergeSubtract && a.n != 2) return hipErrorInvalidValue;
  long long wsum = 0;
  for (int i = 0; i < a.n; ++i) {
    if (!a.in[i] || a.w[i] <= 0 || (a.kind != kMergeConcat && a.w[i] != a.cout)) return hipErrorInvalidValue;
    wsum += a.w[i];
  }
  if (a.kind == kMergeConcat ? wsum != a.cout : false) return hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_fwd_kernel, dim3(merge_grid(a.rows * (long long)a.cout)), dim3(kMT), 0, st, a);
  return hipGetLastError();
}

hipError_t merge_bwd(const MergeArgs& a, hipStream_t st) {
  if (a.n < 1 || a.n > kMergeMaxIn || a.rows <= 0 || a.cout <= 0 || !a.dy) return hipErrorInvalidValue;
  for (int i = 0; i < a.n; ++i)
    if (!a.in[i] || !a.grad[i] || a.w[i] <= 0 || (a.kind != kMergeConcat && a.w[i] != a.cout))
      return hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_bwd_kernel, dim3(merge_grid(a.rows * (long long)a.cout), a.n), dim3(kMT), 0, st, a);
  return hipGetLastError();
}

}  // namespace dfa
