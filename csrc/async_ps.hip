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
//                  example indices, and copy the current weights out (a consistent snapshot plus the
//                  version it belongs to).  The master is triple buffered (version v in buffer v % 3):
//                  readers never wait for the writer lock and a snapshot is torn only if three new
//                  versions are published while it is being copied;
//   (forward / backward kernels of the model)
//   ps_apply       take the writer lock (seq odd), check staleness = version_now - version_pulled
//                  against the bound, write w[v+1] = w[v] - lr * g into the next buffer, publish v + 1.
// Every wait is bounded by a wall-clock timeout that sets a sticky error word instead of spinning
// forever.  Both kernels spread the weights over up to 64 workgroups (one workgroup moves only
// ~60 GB/s of uncached / remote traffic; a single-workgroup version spent ~11 us per kernel on
// LeNet-5's 247 KB).  The last-arriving workgroup finishes the protocol (seqlock check, unlock).
//
// Microbatch dispatch is at-least-once and epoch scoped (claim_microbatch / complete_microbatch):
// a batch is complete only once a gradient for it is admitted; rejected ones are dispatched again.
//
// Shared buffer layout (rank 0): [0] u32 seq (version = seq / 2, odd = writer active), [16] u64 batch
// cursor, [32] u32 dataset epoch, [36] u32 batches completed in it, [48] u64 completed / redispatched /
// skipped / duplicate counters, [256] fp32 master[3][nstride], then u32 done_epoch[kPSMaxBatches] and
// u32 claimed_epoch[kPSMaxBatches].
#include "common.h"
#include "kernels.h"
#include "ps_device.h"

namespace dfa {
namespace {

constexpr int kPSBlock = 256;
constexpr int kPSUnroll = 4;  // float4 loads in flight per thread per round
__device__ __forceinline__ unsigned ld_acq(const unsigned* p) { return ps_ld_acq(p); }

// Multi-workgroup snapshot.  Every workgroup copies its slice of the committed version's buffer between
// two reads of the version word and records the version; the last workgroup to finish checks that all
// slices copied the same version.  A version published in between (a worker commits every few
// microseconds at 8 ranks) makes the last workgroup redo the whole copy of one version alone.
__device__ void copy_slice(const float* __restrict__ src, float* __restrict__ dst, long long lo, long long hi,
                           int t, int nt) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
  f32x4* d4 = reinterpret_cast<f32x4*>(dst);
  const long long lo4 = lo >> 2, hi4 = hi >> 2;  // lo, hi multiples of 4
  for (long long base = lo4 + t; base < hi4; base += (long long)nt * kPSUnroll) {
    f32x4 v[kPSUnroll];
#pragma unroll
    for (int u = 0; u < kPSUnroll; ++u) {
      const long long i = base + (long long)u * nt;
      if (i < hi4) v[u] = s4[i];
    }
#pragma unroll
    for (int u = 0; u < kPSUnroll; ++u) {
      const long long i = base + (long long)u * nt;
      if (i < hi4) d4[i] = v[u];
    }
  }
}

__global__ __launch_bounds__(kPSBlock) void ps_fetch_pull_kernel(PSArgs a) {
  const int t = threadIdx.x, b = blockIdx.x, G = gridDim.x;
  __shared__ unsigned s_seq;
  __shared__ int s_state;  // 0 = copy, 1 = consistent, 2 = error
  __shared__ int s_last;
  if (b == 0) {
    // FCFS microbatch id (remote atomic on the server's cursor) + its example indices
    __shared__ long long s_bid;
    if (a.done_epoch != nullptr) {
      claim_microbatch(a, t, &s_bid);
    } else if (t == 0) {
      s_bid = (long long)(__hip_atomic_fetch_add(a.batch_ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) %
                          (unsigned long long)(a.nbatches > 0 ? a.nbatches : 1));
    }
    __syncthreads();
    if (t == 0) *a.bid_out = s_bid;
    if (a.perm != nullptr && s_bid >= 0) {
      // 16-byte copies, all loads of a thread in flight before its stores (B is even, rows 16B aligned)
      typedef long long i64x2 __attribute__((ext_vector_type(2)));
      const i64x2* src = reinterpret_cast<const i64x2*>(a.perm + (s_bid & 0xffffffffLL) * a.B);
      i64x2* dst = reinterpret_cast<i64x2*>(a.idx);
      const int nv = a.B >> 1;
      for (int base = t; base < nv; base += kPSBlock * 8) {
        i64x2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (base + u * kPSBlock < nv) v[u] = src[base + u * kPSBlock];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (base + u * kPSBlock < nv) dst[base + u * kPSBlock] = v[u];
      }
    }
  }
  const long long per = ((a.n + 4LL * G - 1) / (4LL * G)) * 4;  // slice length, multiple of 4
  const long long lo = b * per, hi = lo + per < a.n ? lo + per : a.n;
  const unsigned long long t0 = wall_clock64();
  // Version v lives in buffer v % 3; the writer of v + 1 writes buffer (v + 1) % 3, so a copy of
  // version v stays valid until a writer of v + 3 starts, i.e. while seq <= 2v + 4.  A reader never
  // waits for the writer lock.
  for (;;) {
    if (t == 0) {
      const unsigned s = ld_acq(a.seq);
      s_seq = s >> 1;  // committed version
    }
    __syncthreads();
    const unsigned v = s_seq;
    if (lo < hi) copy_slice(a.ps_w + (long long)(v % 3u) * a.nstride, a.w, lo, hi, t, kPSBlock);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // slice loads complete before the re-check
    __syncthreads();
    if (t == 0) {
      if (ld_acq(a.seq) <= 2u * v + 4u) s_state = 1;
      else if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) s_state = 2;
      else s_state = 0;
    }
    __syncthreads();
    if (s_state != 0) break;
    __syncthreads();  // every thread has read s_state / s_seq before thread 0 rewrites them
  }
  // publish this slice's version (or a "failed" marker) and elect the last workgroup
  if (t == 0) {
    a.scratch[kPSSlots + b] = s_state == 1 ? s_seq : 0xffffffffu;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned prev = __hip_atomic_fetch_add(a.scratch + kPSPullDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (unsigned)G - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (t == 0) {
    const unsigned v0 = __hip_atomic_load(a.scratch + kPSSlots, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int same = v0 != 0xffffffffu;
    for (int i = 1; i < G && same; ++i)
      same = __hip_atomic_load(a.scratch + kPSSlots + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == v0;
    s_state = same ? 1 : 0;
    s_seq = v0;
    a.scratch[kPSPullDone] = 0;  // reset for the next launch (kernel boundary orders it)
  }
  __syncthreads();
  if (s_state == 1) {
    if (t == 0) *a.vpulled = s_seq;
    return;
  }
  // slices of different versions: redo the whole copy of one version in this workgroup
  if (t == 0) a.stats[4] += 1;
  for (;;) {
    if (t == 0) s_seq = ld_acq(a.seq) >> 1;
    __syncthreads();
    const unsigned v = s_seq;
    copy_slice(a.ps_w + (long long)(v % 3u) * a.nstride, a.w, 0, a.n, t, kPSBlock);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __syncthreads();
    if (t == 0) {
      s_state = 0;
      if (ld_acq(a.seq) <= 2u * v + 4u) {
        s_state = 1;
        *a.vpulled = v;
      } else if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) {
        atomicOr(a.stats + 5, 2ull);
        if (a.herr) __hip_atomic_store(a.herr, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_state = 1;
        *a.vpulled = v;
      }
    }
    __syncthreads();
    if (s_state == 1) return;
    __syncthreads();
  }
}

// Multi-workgroup locked apply.  Workgroup 0 takes the writer lock and decides (staleness check); the
// others wait for that decision on a local word tagged with this launch's epoch, apply their slice, and
// the last workgroup to finish publishes version + 1 (releases the lock).  The grid is small (<= 64
// workgroups), so all of it is resident and the decision wait cannot starve workgroup 0.
__global__ __launch_bounds__(kPSBlock) void ps_apply_kernel(PSArgs a) {
  const int t = threadIdx.x, b = blockIdx.x, G = gridDim.x;
  __shared__ unsigned s_dec;  // 1 = apply, 2 = stale (rejected), 3 = error
  __shared__ unsigned s_seq;
  __shared__ int s_last;
  if (t == 0) {
    const unsigned ep = __hip_atomic_load(a.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const unsigned long long t0 = wall_clock64();
    if (b == 0) {
      unsigned dec = 3, s = 0;
      const long long bid = *a.bid_out;
      if (a.done_epoch != nullptr && bid < 0) {  // dataset finished: this step is a no-op (no lock taken)
        dec = 2;
        a.stats[6] += 1;
      } else for (;;) {
        s = ld_acq(a.seq);
        if (!(s & 1u)) {
          unsigned expected = s;
          if (__hip_atomic_compare_exchange_strong(a.seq, &expected, s + 1u, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_SYSTEM)) {
            const unsigned stale = (s >> 1) - *a.vpulled;
            if ((int)stale <= a.max_stale || a.max_stale < 0) {
              dec = 1;
              a.stats[0] += 1;
              a.stats[2] += stale;
              if (stale > a.stats[3]) a.stats[3] = stale;
              if (a.done_epoch != nullptr) complete_microbatch(a, bid);  // under the writer lock
            } else {
              dec = 2;
              a.stats[1] += 1;
              __hip_atomic_store(a.seq, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // unlock, no new version
            }
            break;
          }
        }
        if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) {
          atomicOr(a.stats + 5, 4ull);
        if (a.herr) __hip_atomic_store(a.herr, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      a.scratch[kPSLockedSeq] = s;
      __hip_atomic_store(a.scratch + kPSDecision, (ep << 2) | dec, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      s_dec = dec;
    } else {
      unsigned d = 0;
      for (;;) {
        d = __hip_atomic_load(a.scratch + kPSDecision, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if ((d >> 2) == ep) break;
        if (wall_clock64() - t0 > 2ull * (unsigned long long)a.timeout_ticks) {
          atomicOr(a.stats + 5, 8ull);
        if (a.herr) __hip_atomic_store(a.herr, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          d = 3;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_dec = d & 3u;
    }
    s_seq = a.scratch[kPSLockedSeq];
  }
  __syncthreads();
  if (s_dec == 1) {
    const long long per = ((a.n + 4LL * G - 1) / (4LL * G)) * 4;
    const long long lo = b * per, hi = lo + per < a.n ? lo + per : a.n;
    const float lr = a.lr;
    const unsigned v = s_seq >> 1;  // version being replaced: buffer v % 3 -> buffer (v + 1) % 3
    const f32x4* w = reinterpret_cast<const f32x4*>(a.ps_w + (long long)(v % 3u) * a.nstride);
    f32x4* wn = reinterpret_cast<f32x4*>(a.ps_w + (long long)((v + 1u) % 3u) * a.nstride);
    const f32x4* g = reinterpret_cast<const f32x4*>(a.g);
    for (long long base = (lo >> 2) + t; base < (hi >> 2); base += (long long)kPSBlock * kPSUnroll) {
      f32x4 v[kPSUnroll], gv[kPSUnroll];
#pragma unroll
      for (int u = 0; u < kPSUnroll; ++u) {
        const long long i = base + (long long)u * kPSBlock;
        if (i < (hi >> 2)) {
          v[u] = w[i];
          gv[u] = g[i];
        }
      }
#pragma unroll
      for (int u = 0; u < kPSUnroll; ++u) {
#pragma clang fp contract(off)  // the same rounding as the fused reduce launch's ps_new_weight
        const long long i = base + (long long)u * kPSBlock;
        if (i < (hi >> 2)) wn[i] = v[u] - lr * gv[u];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // this slice's weight stores visible system-wide
  }
  __syncthreads();
  if (t == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.scratch + kPSApplyDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (unsigned)G - 1;
    if (s_last) {
      a.scratch[kPSApplyDone] = 0;
      a.scratch[kPSEpoch] += 1u;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // every slice's release happened before the unlock
      if (s_dec == 1) __hip_atomic_store(a.seq, s_seq + 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace

// ~16 KB of weights per workgroup, at most kPSMaxGrid workgroups (all resident: the apply kernel's
// decision wait relies on it)
static int ps_grid(long long n) {
  long long g = (n + 4095) / 4096;
  return (int)(g < 1 ? 1 : (g > kPSMaxGrid ? kPSMaxGrid : g));
}

hipError_t ps_fetch_pull(const PSArgs& a, hipStream_t st) {
  if (a.n <= 0 || (a.n & 3) || (a.perm != nullptr && (a.B <= 0 || (a.B & 1) || a.nbatches <= 0)))
    return hipErrorInvalidValue;
  ps_fetch_pull_kernel<<<ps_grid(a.n), kPSBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t ps_apply(const PSArgs& a, hipStream_t st) {
  if (a.n <= 0 || (a.n & 3)) return hipErrorInvalidValue;
  ps_apply_kernel<<<ps_grid(a.n), kPSBlock, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace dfa
