// Memory-bound layer kernels (gfx950): max-pool fwd/bwd, fused softmax-cross-entropy,
// dropout (counter-based mask, regenerated in backward), batch gather from the HBM-resident
// dataset, elementwise add / relu-backward, global average pool.
//
// Reference ops they replace (tf.js): O5 MaxPooling2D (model.json layer 5),
// O6 Dropout (model.json layers 6/10), O7 softmax + tf.losses.softmaxCrossEntropy + mean
// (/root/reference/src/common/models.ts:139), O11 DistributedDataset.getBatch slice
// (/root/reference/src/server/dataset.ts:69-85), O12 uint8->float cast + oneHot
// (/root/reference/experiment/mnist/mnist_data.ts:43-44,70), O15 evaluate's accuracy metric.
// All kernels use 16-byte (8 x bf16) vector accesses when the channel count allows it.
#include "common.h"
#include "kernels.h"

namespace dfa {

// ------------------------------------------------------------------------------------------
// MaxPool (pool == stride, 'valid'), NHWC bf16.  One thread per (output pixel, 8-channel chunk).
template <bool VEC>
__global__ void maxpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int H, int W,
                                   int C, int OH, int OW, int P, DropSpec drop) {
  const unsigned long long ds = drop.on ? drop_seed(drop.seed, drop.step, drop.step_add) : 0ull;
  const int CC = VEC ? C / 8 : C;
  const long long total = (long long)B * OH * OW * CC;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cc = i % CC;
    long long t = i / CC;
    const int ow = t % OW; t /= OW;
    const int oh = t % OH;
    const int b = t / OH;
    const bf16* base = x + (((long long)b * H + oh * P) * W + ow * P) * C;
    if (VEC) {
      float m[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
      for (int ph = 0; ph < P; ++ph)
        for (int pw = 0; pw < P; ++pw) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(base + ((long long)ph * W + pw) * C + cc * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], (float)v[j]);
        }
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // folded dropout: the pooled value rounds to bf16 first, as the standalone dropout saw it
        if (drop.on) m[j] = drop_keep(ds, drop.thresh, i * 8 + j) ? (float)f2bf(m[j]) * drop.scale : 0.f;
        o[j] = f2bf(m[j]);
      }
      *reinterpret_cast<bf16x8*>(y + i * 8) = o;
    } else {
      float m = -INFINITY;
      for (int ph = 0; ph < P; ++ph)
        for (int pw = 0; pw < P; ++pw) m = fmaxf(m, (float)base[((long long)ph * W + pw) * C + cc]);
      if (drop.on) m = drop_keep(ds, drop.thresh, i) ? (float)f2bf(m) * drop.scale : 0.f;
      y[i] = f2bf(m);
    }
  }
}

// Backward: dX = dY at the first arg-max of each window, 0 elsewhere.  With relu_fused the
// producer was conv+ReLU, so relu' is applied too (a window whose max is 0 passes no gradient).
// Rows/cols outside every window (H % P != 0) are zeroed by the caller.
template <bool VEC>
__global__ void maxpool_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                   bf16* __restrict__ dx, int B, int H, int W, int C, int OH, int OW, int P,
                                   int relu_fused) {
  const int CC = VEC ? C / 8 : C;
  const long long total = (long long)B * OH * OW * CC;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cc = i % CC;
    long long t = i / CC;
    const int ow = t % OW; t /= OW;
    const int oh = t % OH;
    const int b = t / OH;
    const long long base = (((long long)b * H + oh * P) * W + ow * P) * C;
    if (VEC) {
      float m[8];
      int am[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { m[j] = -INFINITY; am[j] = 0; }
      for (int ph = 0; ph < P; ++ph)
        for (int pw = 0; pw < P; ++pw) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + base + ((long long)ph * W + pw) * C + cc * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float f = (float)v[j];
            if (f > m[j]) { m[j] = f; am[j] = ph * P + pw; }
          }
        }
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(dy + i * 8);
      for (int ph = 0; ph < P; ++ph)
        for (int pw = 0; pw < P; ++pw) {
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const bool take = am[j] == ph * P + pw && (!relu_fused || m[j] > 0.f);
            o[j] = take ? g[j] : (bf16)0.f;
          }
          *reinterpret_cast<bf16x8*>(dx + base + ((long long)ph * W + pw) * C + cc * 8) = o;
        }
    } else {
      float m = -INFINITY;
      int am = 0;
      for (int ph = 0; ph < P; ++ph)
        for (int pw = 0; pw < P; ++pw) {
          const float f = (float)x[base + ((long long)ph * W + pw) * C + cc];
          if (f > m) { m = f; am = ph * P + pw; }
        }
      const bf16 g = dy[i];
      for (int ph = 0; ph < P; ++ph)
        for (int pw = 0; pw < P; ++pw) {
          const bool take = am == ph * P + pw && (!relu_fused || m > 0.f);
          dx[base + ((long long)ph * W + pw) * C + cc] = take ? g : (bf16)0.f;
        }
    }
  }
}

// dY of a conv whose 2x2 max-pool was fused into its forward epilogue (igemm64 POOL): every pooled
// gradient goes to the window position its code names (code 4 = none: the ReLU'd max was 0).
// One thread per (pooled pixel, 8 channels): a 16-byte gradient load, an 8-byte code load, four
// 16-byte stores.
__global__ void unpool2_kernel(const bf16* __restrict__ dyp, const uint8_t* __restrict__ code, bf16* __restrict__ dy,
                               int B, int OH, int OW, int N) {
  const int PH = OH / 2, PW = OW / 2, NC = N / 8;
  const long long total = (long long)B * PH * PW * NC;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % NC);
    const long long prow = i / NC;
    const int pw = (int)(prow % PW);
    const long long t = prow / PW;
    const int ph = (int)(t % PH);
    const long long b = t / PH;
    const bf16x8 g = *reinterpret_cast<const bf16x8*>(dyp + prow * N + cc * 8);
    const uint2 cw = *reinterpret_cast<const uint2*>(code + prow * N + cc * 8);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned cd = ((j < 4 ? cw.x : cw.y) >> (8 * (j & 3))) & 0xff;
        o[j] = cd == (unsigned)p ? g[j] : (bf16)0.f;
      }
      const long long px = (b * OH + 2 * ph + (p >> 1)) * OW + 2 * pw + (p & 1);
      *reinterpret_cast<bf16x8*>(dy + px * N + cc * 8) = o;
    }
  }
}

static int grid_for(long long total, int block = 256) {
  long long g = (total + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

hipError_t maxpool_fwd(const bf16* x, bf16* y, int B, int H, int W, int C, int P, hipStream_t st, DropSpec drop) {
  const int OH = H / P, OW = W / P;
  const bool vec = C % 8 == 0;
  const long long total = (long long)B * OH * OW * (vec ? C / 8 : C);
  if (total == 0) return hipSuccess;
  if (vec)
    hipLaunchKernelGGL(maxpool_fwd_kernel<true>, dim3(grid_for(total)), dim3(256), 0, st, x, y, B, H, W, C, OH, OW, P,
                       drop);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<false>, dim3(grid_for(total)), dim3(256), 0, st, x, y, B, H, W, C, OH, OW,
                       P, drop);
  return hipGetLastError();
}

hipError_t unpool2(const bf16* dyp, const uint8_t* code, bf16* dy, int B, int OH, int OW, int N, hipStream_t st) {
  if (OH % 2 || OW % 2 || N % 8) return hipErrorInvalidValue;
  const long long total = (long long)B * (OH / 2) * (OW / 2) * (N / 8);
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(unpool2_kernel, dim3(grid_for(total)), dim3(256), 0, st, dyp, code, dy, B, OH, OW, N);
  return hipGetLastError();
}

hipError_t maxpool_bwd(const bf16* x, const bf16* dy, bf16* dx, int B, int H, int W, int C, int P, int relu_fused,
                       hipStream_t st) {
  const int OH = H / P, OW = W / P;
  if (OH * P != H || OW * P != W) DFA_HIP_CHECK(hipMemsetAsync(dx, 0, (size_t)B * H * W * C * sizeof(bf16), st));
  const bool vec = C % 8 == 0;
  const long long total = (long long)B * OH * OW * (vec ? C / 8 : C);
  if (total == 0) return hipSuccess;
  if (vec)
    hipLaunchKernelGGL(maxpool_bwd_kernel<true>, dim3(grid_for(total)), dim3(256), 0, st, x, dy, dx, B, H, W, C, OH,
                       OW, P, relu_fused);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<false>, dim3(grid_for(total)), dim3(256), 0, st, x, dy, dx, B, H, W, C, OH,
                       OW, P, relu_fused);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Fused softmax cross-entropy on fp32 logits [B][ldl] (C classes), int32 labels.
//   dlogits[b][c] = (softmax(z_b)[c] - [c == y_b]) * grad_scale      (bf16, ld = ldg)
//   stats[0] += sum_b loss_b ; stats[1] += #correct (argmax == label)  (fp32 atomics)
// Row-per-thread for C <= 32 (MNIST / CIFAR heads), wave-per-row otherwise.
__global__ void softmax_ce_small_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                                        bf16* __restrict__ dlogits, float* __restrict__ stats, int B, int C,
                                        int ldl, int ldg, float grad_scale) {
  __shared__ float s_loss[4], s_corr[4];
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  float loss = 0.f, corr = 0.f;
  if (b < B) {
    const float* z = logits + (long long)b * ldl;
    float mx = -INFINITY;
    int am = 0;
    for (int c = 0; c < C; ++c) {
      const float v = z[c];
      if (v > mx) { mx = v; am = c; }
    }
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(z[c] - mx);
    const int y = min(max(labels[b], 0), C - 1);  // never index outside the row
    const float lse = mx + __logf(se);
    loss = lse - z[y];
    corr = (am == y) ? 1.f : 0.f;
    if (dlogits) {
      const float inv = 1.f / se;
      for (int c = 0; c < C; ++c) {
        const float p = __expf(z[c] - mx) * inv;
        dlogits[(long long)b * ldg + c] = f2bf((p - (c == y ? 1.f : 0.f)) * grad_scale);
      }
    }
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

__global__ void softmax_ce_wave_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                                       bf16* __restrict__ dlogits, float* __restrict__ stats, int B, int C, int ldl,
                                       int ldg, float grad_scale) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* z = logits + (long long)b * ldl;
  float mx = -INFINITY;
  int am = 0x7fffffff;
  for (int c = lane; c < C; c += 64) {
    const float v = z[c];
    if (v > mx) { mx = v; am = c; }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(mx, off, 64);
    const int oa = __shfl_xor(am, off, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += __expf(z[c] - mx);
  se = wave_sum(se);
  const int y = min(max(labels[b], 0), C - 1);
  if (dlogits) {
    const float inv = 1.f / se;
    for (int c = lane; c < C; c += 64) {
      const float p = __expf(z[c] - mx) * inv;
      dlogits[(long long)b * ldg + c] = f2bf((p - (c == y ? 1.f : 0.f)) * grad_scale);
    }
  }
  if (lane == 0 && stats) {
    atomicAdd(&stats[0], mx + __logf(se) - z[y]);
    atomicAdd(&stats[1], am == y ? 1.f : 0.f);
  }
}

hipError_t softmax_ce(const float* logits, const int* labels, bf16* dlogits, float* stats, int B, int C, int ldl,
                      int ldg, float grad_scale, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (C <= 32)
    hipLaunchKernelGGL(softmax_ce_small_kernel, dim3(cdiv(B, 256)), dim3(256), 0, st, logits, labels, dlogits, stats,
                       B, C, ldl, ldg, grad_scale);
  else
    hipLaunchKernelGGL(softmax_ce_wave_kernel, dim3(cdiv(B, 4)), dim3(256), 0, st, logits, labels, dlogits, stats, B,
                       C, ldl, ldg, grad_scale);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Dropout: y = x * keep(seed, i) / (1 - p) [* relu'(mask)].  The same call on dY is the backward
// (the mask is regenerated from (seed, i)); `mask` fuses the producer's relu' into that pass.
__global__ void dropout_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, const bf16* __restrict__ mask,
                               long long n, float p, unsigned long long seed0, const long long* __restrict__ step) {
  const unsigned long long seed = seed0 ^ (step ? (unsigned long long)step[0] * 0x9E3779B1ull : 0ull);
  const uint32_t thresh = (uint32_t)((double)p * 4294967296.0);
  const float scale = 1.f / (1.f - p);
  const long long n8 = n / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i * 8);
    bf16x8 mk;
    if (mask) mk = *reinterpret_cast<const bf16x8*>(mask + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bool keep = hash_u32(seed, (uint64_t)(i * 8 + j)) >= thresh;
      if (mask) keep = keep && ((float)mk[j] > 0.f);
      v[j] = keep ? f2bf((float)v[j] * scale) : (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(y + i * 8) = v;
  }
  for (long long i = n8 * 8 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    bool keep = hash_u32(seed, (uint64_t)i) >= thresh;
    if (mask) keep = keep && ((float)mask[i] > 0.f);
    y[i] = keep ? f2bf((float)x[i] * scale) : (bf16)0.f;
  }
}

hipError_t dropout(const bf16* x, bf16* y, const bf16* mask, long long n, float p, unsigned long long seed,
                   const long long* step, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for((n + 7) / 8)), dim3(256), 0, st, x, y, mask, n, p, seed, step);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Batch gather from the HBM-resident dataset: out[b] = data[idx[b]] (row = `row` elements).
// u8 sources are cast to bf16 with `scale` (the one-time preprocessing of O12 done on the fly).
__device__ __forceinline__ long long clamp_row(long long r, long long nrows) {
  return r < 0 ? 0 : (r >= nrows ? nrows - 1 : r);
}

template <typename T>
__global__ void gather_rows_kernel(const T* __restrict__ data, const long long* __restrict__ idx,
                                   bf16* __restrict__ out, int B, int row, float scale, long long nrows,
                                   long long* __restrict__ step_inc) {
  // the step's first launch advances the device step counter (dropout masks of the step read it)
  if (step_inc && blockIdx.x == 0 && threadIdx.x == 0) step_inc[0] += 1;
  const int per = row;  // elements per row
  const long long total = (long long)B * per;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = i / per;
    const int e = i - (long long)b * per;
    out[i] = f2bf((float)data[clamp_row(idx[b], nrows) * per + e] * scale);
  }
}

__global__ void gather_rows_bf16_vec_kernel(const bf16* __restrict__ data, const long long* __restrict__ idx,
                                            bf16* __restrict__ out, int B, int row8, long long nrows,
                                            long long* __restrict__ step_inc) {
  if (step_inc && blockIdx.x == 0 && threadIdx.x == 0) step_inc[0] += 1;
  const long long total = (long long)B * row8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = i / row8;
    const int e = i - (long long)b * row8;
    reinterpret_cast<bf16x8*>(out)[i] = reinterpret_cast<const bf16x8*>(data)[clamp_row(idx[b], nrows) * row8 + e];
  }
}

__global__ void gather_labels_kernel(const int* __restrict__ labels, const long long* __restrict__ idx,
                                     int* __restrict__ out, int B, long long nrows) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) out[b] = labels[clamp_row(idx[b], nrows)];
}

hipError_t gather_batch(const void* data, int data_is_u8, const int* labels, const long long* idx, bf16* out,
                        int* out_labels, int B, int row, float scale, long long nrows, hipStream_t st,
                        long long* step_inc) {
  if (B <= 0) return hipSuccess;
  const long long total = (long long)B * row;
  if (data_is_u8) {
    hipLaunchKernelGGL(gather_rows_kernel<uint8_t>, dim3(grid_for(total)), dim3(256), 0, st,
                       (const uint8_t*)data, idx, out, B, row, scale, nrows, step_inc);
  } else if (row % 8 == 0 && scale == 1.f) {
    hipLaunchKernelGGL(gather_rows_bf16_vec_kernel, dim3(grid_for(total / 8)), dim3(256), 0, st, (const bf16*)data,
                       idx, out, B, row / 8, nrows, step_inc);
  } else {
    hipLaunchKernelGGL(gather_rows_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, (const bf16*)data, idx,
                       out, B, row, scale, nrows, step_inc);
  }
  DFA_HIP_CHECK(hipGetLastError());
  if (labels && out_labels) {
    hipLaunchKernelGGL(gather_labels_kernel, dim3(cdiv(B, 256)), dim3(256), 0, st, labels, idx, out_labels, B, nrows);
    DFA_HIP_CHECK(hipGetLastError());
  }
  return hipSuccess;
}

hipError_t gather_labels(const int* labels, const long long* idx, int* out, int B, long long nrows, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_labels_kernel, dim3(cdiv(B, 256)), dim3(256), 0, st, labels, idx, out, B, nrows);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Elementwise: out = a + b (+ optional relu), and relu backward dx = dy * (y > 0).
__global__ void add_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b, bf16* __restrict__ out, long long n8,
                           int relu) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const bf16x8 x = reinterpret_cast<const bf16x8*>(a)[i];
    const bf16x8 y = reinterpret_cast<const bf16x8*>(b)[i];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = (float)x[j] + (float)y[j];
      if (relu) v = fmaxf(v, 0.f);
      o[j] = f2bf(v);
    }
    reinterpret_cast<bf16x8*>(out)[i] = o;
  }
}

__global__ void relu_bwd_kernel(const bf16* __restrict__ y, const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const bf16x8 v = reinterpret_cast<const bf16x8*>(y)[i];
    const bf16x8 g = reinterpret_cast<const bf16x8*>(dy)[i];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = ((float)v[j] > 0.f) ? g[j] : (bf16)0.f;
    reinterpret_cast<bf16x8*>(dx)[i] = o;
  }
}

hipError_t add_act(const bf16* a, const bf16* b, bf16* out, long long n, int relu, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(add_kernel, dim3(grid_for(n / 8)), dim3(256), 0, st, a, b, out, n / 8, relu);
  return hipGetLastError();
}

hipError_t relu_bwd(const bf16* y, const bf16* dy, bf16* dx, long long n, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(n / 8)), dim3(256), 0, st, y, dy, dx, n / 8);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Global average pool NHWC [B][HW][C] -> [B][C] and its backward (broadcast / HW).
__global__ void gap_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int HW, int C) {
  const long long total = (long long)B * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = i % C;
    const int b = i / C;
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += (float)x[((long long)b * HW + p) * C + c];
    y[i] = f2bf(s / HW);
  }
}

__global__ void gap_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx, int B, int HW, int C) {
  const long long total = (long long)B * HW * C;
  const float inv = 1.f / HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = i % C;
    const int b = i / ((long long)HW * C);
    dx[i] = f2bf((float)dy[(long long)b * C + c] * inv);
  }
}

hipError_t gap_fwd(const bf16* x, bf16* y, int B, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(grid_for((long long)B * C)), dim3(256), 0, st, x, y, B, HW, C);
  return hipGetLastError();
}
hipError_t gap_bwd(const bf16* dy, bf16* dx, int B, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(grid_for((long long)B * HW * C)), dim3(256), 0, st, dy, dx, B, HW, C);
  return hipGetLastError();
}

}  // namespace dfa
