// Fused multi-tensor SGD (gfx950): one launch updates every parameter of the model.
//
// Replaces DistributedTfModel.update (w <- w - lr * g per weight, one tf.js op chain per tensor,
// /root/reference/src/common/models.ts:128-135) and the server-side mean aggregation
// (/root/reference/src/server/federated_server.ts:98-106):
//   * the 1/world (or 1/K) gradient-mean scale is folded in (grad_scale), so the all-reduce is a
//     plain SUM and no separate "mean" pass exists,
//   * optional momentum / weight decay (not in the reference; used by the ResNet config),
//   * the same pass re-emits the bf16 compute copies of each weight matrix in the two layouts the
//     MFMA kernels read: [N][K] (fwd, K = KH*KW*Cin) and the dgrad layout [Cin][KH*KW*N], both
//     zero padded to 16 x 32 tiles (or the row-segment layout of the fused conv+pool forward).  Hyper-parameters live in device memory so a captured hipGraph
//     sees learning-rate changes without re-capture.
#include "common.h"
#include "kernels.h"
#include "lenet_frag.h"
#include "optim_device.h"

namespace dfa {

constexpr int SGD_ELEMS_PER_BLOCK = 1024;

template <typename DT>
__device__ __forceinline__ int find_desc(const DT& d, int n, int bid) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].block_start <= bid) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// hyper = [lr, momentum, weight_decay, grad_scale, nesterov]
template <typename DT>
__device__ __forceinline__ void sgd_multi_body(const DT& descs, int ndesc,
                                               float* __restrict__ master, const float* __restrict__ grad,
                                               float* __restrict__ mom_buf, bf16* __restrict__ wbf,
                                               const float* __restrict__ hyper, int apply_update, int bid,
                                               float* __restrict__ mirror = nullptr) {
  const int di = find_desc(descs, ndesc, bid);
  const ParamDesc d = descs[di];
  const int base = (bid - d.block_start) * SGD_ELEMS_PER_BLOCK;
  float lr = 0.f, mom = 0.f, wd = 0.f, gs = 1.f;
  bool nesterov = false;
  if (apply_update) {
    lr = hyper[0]; mom = hyper[1]; wd = hyper[2]; gs = hyper[3]; nesterov = hyper[4] != 0.f;
  }
  const int K = d.T * d.Ci;
  auto update = [&](int i) -> float {
    float w = master[d.off + i];
    if (apply_update) {
      float v = 0.f;
      w = sgd_new_weight(w, grad[d.off + i], mom != 0.f ? mom_buf[d.off + i] : 0.f, lr, mom, wd, gs, nesterov, &v);
      if (mom != 0.f) mom_buf[d.off + i] = v;
      master[d.off + i] = w;
      if (mirror != nullptr) mirror[d.off + i] = w;
    }
    return w;
  };
  // d.pad_ bit 28: tile mode for a plain [N][K] matrix with a plain dgrad copy [Ci][T*N]: the workgroup
  // owns a 32 (n) x 32 (k) tile; the update and the primary copy run along k (coalesced), and the
  // dgrad copy is written through an LDS transpose as 64-byte runs along n (instead of 2-byte
  // scatters one KpadT row apart)
  if ((d.pad_ >> 28) & 1) {
    __shared__ bf16 tt[32][34];
    const int ntk = cdiv(K, 32);
    const int tl = bid - d.block_start;
    const int n0 = (tl / ntk) * 32, k0 = (tl % ntk) * 32;
    const int Kp = round_up(K, 32);
    const int KpT = round_up(d.T * d.N, 32);
    const int cc = threadIdx.x & 31, r0 = threadIdx.x >> 5;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int n = n0 + r0 + 8 * rr, k = k0 + cc;
      if (n < d.N && k < K) {
        const bf16 wb = f2bf(update(n * K + k));
        wbf[d.bf_off + (long long)n * Kp + k] = wb;
        tt[cc][r0 + 8 * rr] = wb;
      }
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int k = k0 + r0 + 8 * rr, n = n0 + cc;
      if (n < d.N && k < K) {
        const int t = k / d.Ci, ci = k - t * d.Ci;
        wbf[d.bft_off + (long long)ci * KpT + t * d.N + n] = tt[r0 + 8 * rr][cc];
      }
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < SGD_ELEMS_PER_BLOCK / 256; ++r) {
    const int i = base + r * 256 + threadIdx.x;
    if (i >= d.numel) break;
    emit_copies(d, i, update(i), wbf);
  }
}

// Device-resident index stream: the optimizer is the last kernel of a training step, so one extra
// workgroup of the same launch stages the NEXT step's batch indices (src[(cursor+1) % nsteps]) into
// the static index buffer the step's first kernels read, then advances the cursor.  A replayed step
// graph then needs no host-side copy (and no extra launch) to move to the next batch.
__device__ __forceinline__ void index_stream_body(const IndexStream& is) {
  if (is.src == nullptr) {  // run statistics only (no index stream bound)
    if (threadIdx.x == 0 && is.run_stats != nullptr) {
      is.run_stats[0] += is.step_stats[0];
      is.run_stats[1] += is.step_stats[1];
      is.run_stats[2] += 1.f;
    }
    return;
  }
  __shared__ long long next;
  // thread 0 loads the cursor and, with it, the running / step statistics it updates at the end: one round
  // trip for all of them (the statistics used to be read after the index copy, a third round trip on the
  // launch's critical path)
  float rs[3] = {0.f, 0.f, 0.f}, ss[2] = {0.f, 0.f};
  if (threadIdx.x == 0) {
    const long long c = *is.cursor;
    if (is.run_stats != nullptr) {
      rs[0] = is.run_stats[0], rs[1] = is.run_stats[1], rs[2] = is.run_stats[2];
      ss[0] = is.step_stats[0], ss[1] = is.step_stats[1];
    }
    next = (c + 1) % is.nsteps;
  }
  __syncthreads();
  const long long* src = is.src + next * is.B;
  // all loads of a thread are issued before its stores (one memory round trip for B <= 8192)
  constexpr int R = 16;
  long long v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = threadIdx.x + 256 * r;
    v[r] = src[min(i, is.B - 1)];
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = threadIdx.x + 256 * r;
    if (i < is.B) is.dst[i] = v[r];
  }
  for (int i = threadIdx.x + 256 * R; i < is.B; i += 256) is.dst[i] = src[i];
  if (threadIdx.x == 0) {
    *is.cursor = next;
    if (is.run_stats != nullptr) {  // this step's stats are final: every step kernel precedes this launch
      is.run_stats[0] = rs[0] + ss[0];
      is.run_stats[1] = rs[1] + ss[1];
      is.run_stats[2] = rs[2] + 1.f;
    }
  }
}

// Fused LeNet-5: the conv-weight MFMA fragments of the next step, kLeNetFragBlocks extra workgroups,
// one fragment lane per thread.  Each new weight is recomputed with the owning workgroup's exact
// (non-contracted) update from the pre-update snapshot the reduce kernel took: nothing here reads
// master / momentum, which the owners overwrite in this same launch.  apply_update == 0 (compute
// copy refresh, master not written) reads master directly.
constexpr int kLeNetFragBlocks = (kLeNetFragLanes + 255) / 256;

__device__ __forceinline__ void lenet_frag_body(const IndexStream& is, int fb, const float* __restrict__ master,
                                                const float* __restrict__ grad, const float* __restrict__ hyper,
                                                int apply_update) {
  const int fl = fb * 256 + threadIdx.x;
  if (fl >= kLeNetFragLanes) return;
  bf16x8* frag = reinterpret_cast<bf16x8*>(is.frag);
  if (!apply_update) {
    frag[fl] = lenet_frag_lane(fl, [&](int j) { return master[j < 150 ? is.frag_w1 + j : is.frag_w2 + (j - 150)]; });
    return;
  }
  const float lr = hyper[0], mom = hyper[1], wd = hyper[2], gs = hyper[3];
  const bool nesterov = hyper[4] != 0.f;
  frag[fl] = lenet_frag_lane(fl, [&](int j) {
    const float g = grad[j < 150 ? is.frag_w1 + j : is.frag_w2 + (j - 150)];
    return sgd_new_weight(is.snap[j], g, mom != 0.f ? is.snap[kLeNetConvW + j] : 0.f, lr, mom, wd, gs, nesterov,
                          nullptr);
  });
}

template <bool INL>
__global__ void __launch_bounds__(256) sgd_multi_stream_kernel(const ParamDesc* __restrict__ descs,
                                                               const ParamDescTable tab, int ndesc,
                                                               float* __restrict__ master,
                                                               const float* __restrict__ grad,
                                                               float* __restrict__ mom_buf, bf16* __restrict__ wbf,
                                                               const float* __restrict__ hyper, int apply_update,
                                                               int total_blocks, IndexStream is) {
  if ((int)blockIdx.x < total_blocks) {
    // async PS exclusive writer: a rejected / finished step leaves the weights (and their copies) as they are
    if (is.gate != nullptr && (__hip_atomic_load(is.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 7u) != 1u)
      return;
    if (INL)
      sgd_multi_body(tab.d, ndesc, master, grad, mom_buf, wbf, hyper, apply_update, blockIdx.x, is.mirror);
    else
      sgd_multi_body(descs, ndesc, master, grad, mom_buf, wbf, hyper, apply_update, blockIdx.x, is.mirror);
    return;
  }
  int fb = blockIdx.x - total_blocks;
  if (is.src != nullptr || is.run_stats != nullptr) {
    if (fb == 0) {
      index_stream_body(is);  // the single index-stream workgroup
      return;
    }
    --fb;
  }
  if (is.frag != nullptr) lenet_frag_body(is, fb, master, grad, hyper, apply_update);
}

hipError_t sgd_multi(const ParamDesc* descs, int ndesc, int total_blocks, float* master, const float* grad,
                     float* mom_buf, bf16* wbf, const float* hyper, int apply_update, hipStream_t st,
                     const IndexStream* is, const ParamDesc* host_descs) {
  // the extra workgroup: index staging and / or the run statistics
  const bool stream = is != nullptr && (is->src != nullptr || is->run_stats != nullptr);
  const bool frag = is != nullptr && is->frag != nullptr;
  total_blocks = max(total_blocks, 0);
  if ((ndesc <= 0 || total_blocks <= 0) && !stream && !frag) return hipSuccess;
  IndexStream isv{};
  if (is != nullptr) isv = *is;
  if (!stream) isv.src = nullptr, isv.run_stats = nullptr;
  if ((isv.gate != nullptr || isv.mirror != nullptr) && (frag || !apply_update)) return hipErrorInvalidValue;
  if (frag && apply_update && is->snap == nullptr) return hipErrorInvalidValue;
  const int grid = total_blocks + (stream ? 1 : 0) + (frag ? kLeNetFragBlocks : 0);
  if (host_descs != nullptr && ndesc <= kInlineDescs) {
    ParamDescTable tab{};
    for (int i = 0; i < ndesc; ++i) tab.d[i] = host_descs[i];
    hipLaunchKernelGGL(sgd_multi_stream_kernel<true>, dim3(grid), dim3(256), 0, st, descs, tab, ndesc, master, grad,
                       mom_buf, wbf, hyper, apply_update, total_blocks, isv);
  } else {
    ParamDescTable tab{};
    hipLaunchKernelGGL(sgd_multi_stream_kernel<false>, dim3(grid), dim3(256), 0, st, descs, tab, ndesc, master,
                       grad, mom_buf, wbf, hyper, apply_update, total_blocks, isv);
  }
  return hipGetLastError();
}

// out = scale * sum_j in_j   (server-side aggregation of K uploaded gradient buffers)
__global__ void sum_buffers_kernel(const float* const* __restrict__ ins, int nin, float* __restrict__ out,
                                   long long n, float scale) {
  const long long n4 = n / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = 0; j < nin; ++j) {
      const float4 v = reinterpret_cast<const float4*>(ins[j])[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
    reinterpret_cast<float4*>(out)[i] = s;
  }
  for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < nin; ++j) s += ins[j][i];
    out[i] = s * scale;
  }
}

hipError_t sum_buffers(const float* const* ins, int nin, float* out, long long n, float scale, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  long long g = (n / 4 + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(sum_buffers_kernel, dim3((int)g), dim3(256), 0, st, ins, nin, out, n, scale);
  return hipGetLastError();
}

// out = a + alpha * (b - a)  — FedAvg-style weight interpolation / delta application on flat buffers
__global__ void axpby_kernel(float* __restrict__ out, const float* __restrict__ a, const float* __restrict__ b,
                             float alpha, float beta, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = alpha * a[i] + beta * b[i];
}

hipError_t axpby(float* out, const float* a, const float* b, float alpha, float beta, long long n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  long long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(axpby_kernel, dim3((int)g), dim3(256), 0, st, out, a, b, alpha, beta, n);
  return hipGetLastError();
}

}  // namespace dfa
