// Device-resident bounded-staleness parameter server for asynchronous SGD (BASELINE.json configs[2]).
//
// Reference semantics (/root/reference/src/server/asynchronousSGD_server.ts:45-108, client side
// /root/reference/src/client/asynchronousSGD_client.ts:16-84): the server dispenses microbatches
// first-come-first-serve, every worker computes a gradient on the weights it last downloaded, and the
// server applies each gradient on arrival.  The README's intended `maximumStaleness` bound
// (/root/reference/README.md:27) is enforced here.
//
// MI355X design: the server state lives in rank 0's HBM, in one IPC-exported uncached buffer that every
// rank maps over xGMI.  There is no server thread and no message loop.  A worker's whole step is
// device work that it replays from its own hipGraph at its own pace:
//   ps_fetch_pull  claim the next microbatch id with a remote atomic (the FCFS dispenser), stage its
//                  example indices, and copy the current weights out under a seqlock (a consistent
//                  snapshot plus the version it belongs to);
//   (forward / backward kernels of the model)
//   ps_apply       take the writer lock (seq odd), check staleness = version_now - version_pulled
//                  against the bound, apply w -= lr * g to the shared master, publish version + 1.
// Every wait is bounded by a wall-clock timeout that sets a sticky error word instead of spinning
// forever.  Both kernels run as one 1024-thread workgroup: the MNIST-sized payloads (247 KB for LeNet-5,
// 2.4 MB for the Keras CNN) are latency bound, and a single workgroup makes the seqlock check exact.
//
// Shared buffer layout (rank 0): [0] u32 seq (version = seq / 2), [16] u64 batch counter,
// [256] fp32 master[n].
#include "common.h"
#include "kernels.h"

namespace dfa {
namespace {

constexpr int kPSThreads = 1024;
constexpr int kPSUnroll = 8;  // float4 loads in flight per thread per round

__device__ __forceinline__ unsigned ld_acq(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kPSThreads) void ps_fetch_pull_kernel(PSArgs a) {
  const int t = threadIdx.x;
  __shared__ long long s_bid;
  __shared__ unsigned s_seq;
  __shared__ int s_state;  // 0 = copy, 1 = done, 2 = error
  // 1. FCFS microbatch id + its example indices
  if (t == 0) {
    s_bid = (long long)__hip_atomic_fetch_add(a.batch_ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *a.bid_out = s_bid;
  }
  __syncthreads();
  if (a.perm != nullptr) {
    const long long row = s_bid % a.nbatches;
    for (int i = t; i < a.B; i += kPSThreads) a.idx[i] = a.perm[row * a.B + i];
  }
  // 2. seqlock snapshot of the shared master
  const unsigned long long t0 = wall_clock64();
  const long long n4 = a.n >> 2;
  for (int attempt = 0;; ++attempt) {
    if (t == 0) {
      unsigned s = ld_acq(a.seq);
      while (s & 1u) {  // a writer holds the lock
        if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) break;
        __builtin_amdgcn_s_sleep(2);
        s = ld_acq(a.seq);
      }
      s_seq = s;
      s_state = (s & 1u) ? 2 : 0;
    }
    __syncthreads();
    if (s_state == 2) {
      if (t == 0) atomicOr(reinterpret_cast<unsigned long long*>(a.stats) + 5, 1ull);
      return;
    }
    const f32x4* src = reinterpret_cast<const f32x4*>(a.ps_w);
    f32x4* dst = reinterpret_cast<f32x4*>(a.w);
    for (long long base = t; base < n4; base += (long long)kPSThreads * kPSUnroll) {
      f32x4 v[kPSUnroll];
#pragma unroll
      for (int u = 0; u < kPSUnroll; ++u) {
        const long long i = base + (long long)u * kPSThreads;
        if (i < n4) v[u] = src[i];
      }
#pragma unroll
      for (int u = 0; u < kPSUnroll; ++u) {
        const long long i = base + (long long)u * kPSThreads;
        if (i < n4) dst[i] = v[u];
      }
    }
    for (long long i = (n4 << 2) + t; i < a.n; i += kPSThreads) a.w[i] = a.ps_w[i];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // data loads complete before the re-check
    __syncthreads();
    if (t == 0) {
      const unsigned s2 = ld_acq(a.seq);
      if (s2 == s_seq) {
        s_state = 1;
        *a.vpulled = s_seq >> 1;
      } else {
        a.stats[4] += 1;  // torn snapshot: retry
        if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) {
          atomicOr(reinterpret_cast<unsigned long long*>(a.stats) + 5, 2ull);
          s_state = 1;
          *a.vpulled = s_seq >> 1;
        }
      }
    }
    __syncthreads();
    if (s_state == 1) return;
    __syncthreads();  // every thread has read s_state before thread 0 rewrites it
  }
}

__global__ __launch_bounds__(kPSThreads) void ps_apply_kernel(PSArgs a) {
  const int t = threadIdx.x;
  __shared__ unsigned s_seq;
  __shared__ int s_go;  // 1 = apply, 0 = stale (rejected), -1 = lock timeout
  if (t == 0) {
    const unsigned long long t0 = wall_clock64();
    int go = -1;
    for (;;) {
      unsigned s = ld_acq(a.seq);
      if (!(s & 1u)) {
        unsigned expected = s;
        if (__hip_atomic_compare_exchange_strong(a.seq, &expected, s + 1u, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM)) {
          s_seq = s;
          const unsigned stale = (s >> 1) - *a.vpulled;
          go = ((int)stale <= a.max_stale || a.max_stale < 0) ? 1 : 0;
          if (go) {
            a.stats[0] += 1;
            a.stats[2] += stale;
            if (stale > a.stats[3]) a.stats[3] = stale;
          } else {
            a.stats[1] += 1;
            __hip_atomic_store(a.seq, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // unlock, no new version
          }
          break;
        }
      }
      if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) {
        atomicOr(reinterpret_cast<unsigned long long*>(a.stats) + 5, 4ull);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    s_go = go;
  }
  __syncthreads();
  if (s_go != 1) return;
  const float lr = a.lr;
  const long long n4 = a.n >> 2;
  f32x4* w = reinterpret_cast<f32x4*>(a.ps_w);
  const f32x4* g = reinterpret_cast<const f32x4*>(a.g);
  for (long long base = t; base < n4; base += (long long)kPSThreads * kPSUnroll) {
    f32x4 v[kPSUnroll], gv[kPSUnroll];
#pragma unroll
    for (int u = 0; u < kPSUnroll; ++u) {
      const long long i = base + (long long)u * kPSThreads;
      if (i < n4) {
        v[u] = w[i];
        gv[u] = g[i];
      }
    }
#pragma unroll
    for (int u = 0; u < kPSUnroll; ++u) {
      const long long i = base + (long long)u * kPSThreads;
      if (i < n4) w[i] = v[u] - lr * gv[u];
    }
  }
  for (long long i = (n4 << 2) + t; i < a.n; i += kPSThreads) a.ps_w[i] = a.ps_w[i] - lr * a.g[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // all weight stores visible before the new version
  __syncthreads();
  if (t == 0) __hip_atomic_store(a.seq, s_seq + 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t ps_fetch_pull(const PSArgs& a, hipStream_t st) {
  if (a.n <= 0 || (a.perm != nullptr && (a.B <= 0 || a.nbatches <= 0))) return hipErrorInvalidValue;
  ps_fetch_pull_kernel<<<1, kPSThreads, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t ps_apply(const PSArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipErrorInvalidValue;
  ps_apply_kernel<<<1, kPSThreads, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace dfa
