// Device-side evaluation metrics of a classifier: [sum of the compiled loss, number
// correct] of a batch in one launch, so DistriModel.evaluate / sendMetrics run no framework ops.
//
// Reference: DistributedTfModel.evaluate = model.evaluate(x, y) with the compile args' loss and the
// 'accuracy' metric (/root/reference/src/common/models.ts:106-115), called before every upload when
// sendMetrics is set (/root/reference/src/client/federated_client.ts:89-92).  The loss kinds are the
// lossesMap entries (/root/reference/src/common/utils.ts:19-30), each as the per-example mean over
// classes of the one-hot label vs the model output (probabilities when the model ends in softmax).
//
// One workgroup of 1024 threads: a thread owns rows t, t + 1024, ... (one pass over the logits,
// softmax in registers for C <= 64), then a fixed-order tree over the workgroup: deterministic.
#include "common.h"
#include "kernels.h"

namespace dfa {
namespace {

constexpr int MT = 1024;
constexpr int kMaxC = 64;

__device__ __forceinline__ float row_loss(int kind, float p, float y) {
  switch (kind) {
    case kMetricMSE: return (y - p) * (y - p);
    case kMetricAbs: return fabsf(y - p);
    case kMetricHinge: return fmaxf(0.f, 1.f - (2.f * y - 1.f) * p);
    case kMetricHuber: {
      const float d = fabsf(p - y);
      return d <= 1.f ? 0.5f * d * d : d - 0.5f;
    }
    case kMetricLog: return -(y * __logf(p + 1e-7f) + (1.f - y) * __logf(1.f - p + 1e-7f));
    case kMetricSigmoidCE: return fmaxf(p, 0.f) - p * y + __logf(1.f + __expf(-fabsf(p)));
    default: return 0.f;
  }
}

__global__ void __launch_bounds__(MT) classifier_metrics_kernel(const float* __restrict__ z, const int* __restrict__ labels,
                                                                int B, int C, int kind, int softmax,
                                                                float* __restrict__ out) {
  __shared__ float sl[MT / 64], sc[MT / 64];
  float lsum = 0.f, corr = 0.f;
  for (int r = threadIdx.x; r < B; r += MT) {
    float p[kMaxC];
    const float* zr = z + (long long)r * C;
    float mx = -INFINITY;
    int am = 0;
    for (int c = 0; c < C; ++c) {
      p[c] = zr[c];
      if (p[c] > mx) { mx = p[c]; am = c; }
    }
    int y = labels[r];
    y = y < 0 ? 0 : (y >= C ? C - 1 : y);
    corr += am == y ? 1.f : 0.f;  // argmax is invariant under the softmax / sigmoid
    if (softmax == 2) {  // the model ends in sigmoid: metrics of its probabilities
      for (int c = 0; c < C; ++c) p[c] = 1.f / (1.f + __expf(-p[c]));
    } else if (softmax || kind == kMetricSoftmaxCE) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += __expf(p[c] - mx);
      if (kind == kMetricSoftmaxCE && !softmax) {  // logits in: -log softmax(z)_y
        lsum += -(p[y] - mx - __logf(s));
        continue;
      }
      const float inv = 1.f / s;
      for (int c = 0; c < C; ++c) p[c] = __expf(p[c] - mx) * inv;
    }
    if (kind == kMetricSoftmaxCE) {  // applied to probabilities (the reference's swapped-argument use)
      float m2 = -INFINITY, s2 = 0.f;
      for (int c = 0; c < C; ++c) m2 = fmaxf(m2, p[c]);
      for (int c = 0; c < C; ++c) s2 += __expf(p[c] - m2);
      lsum += -(p[y] - m2 - __logf(s2));
    } else if (kind == kMetricCategoricalCE) {
      lsum += -__logf(fminf(fmaxf(p[y], 1e-7f), 1.f));
    } else {
      float v = 0.f;
      for (int c = 0; c < C; ++c) v += row_loss(kind, p[c], c == y ? 1.f : 0.f);
      lsum += v / C;
    }
  }
  lsum = wave_sum(lsum);
  corr = wave_sum(corr);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sl[wid] = lsum;
    sc[wid] = corr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int w = 0; w < MT / 64; ++w) {
      a += sl[w];
      b += sc[w];
    }
    out[0] = a;
    out[1] = b;
  }
}

}  // namespace

hipError_t classifier_metrics(const float* z, const int* labels, int B, int C, int kind, int softmax, float* out,
                              hipStream_t st) {
  if (B <= 0 || C <= 0 || C > kMaxC || kind < 0 || kind > kMetricCategoricalCE) return hipErrorInvalidValue;
  hipLaunchKernelGGL(classifier_metrics_kernel, dim3(1), dim3(MT), 0, st, z, labels, B, C, kind, softmax, out);
  return hipGetLastError();
}

}  // namespace dfa
