// Device-side protocol pieces of the parameter server shared by csrc/async_ps.hip (pull / apply
// launches) and the fused LeNet-5 reduce kernel, which applies an admitted gradient to the shared
// master itself (csrc/lenet_fused.hip): microbatch claims and completion accounting.
#pragma once
#include "common.h"
#include "kernels.h"

namespace dfa {

// local scratch words (PSArgs::scratch, u32 index)
constexpr int kPSPullDone = 0, kPSApplyDone = 1, kPSEpoch = 2, kPSDecision = 3, kPSLockedSeq = 4, kPSCompleted = 5,
              kPSSlots = 64;

__device__ __forceinline__ unsigned ps_ld_acq(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// At-least-once FCFS dispatch (/root/reference/src/server/dataset.ts:47-67).  The shared cursor
// (batch_ctr) walks the batch ids of the current dataset epoch round and round; a batch stays
// incomplete until ps_apply ADMITS a gradient for it, so batches whose gradient was rejected as too
// stale (or is still in flight) come round again on the next lap, and the epoch only advances
// once every batch is complete.  Wave 0 of the block reads 64 completion words per remote round
// trip, claims the first incomplete batch after the cursor and moves the cursor past the completed
// ones it skipped.  Two claimers can land on the same incomplete batch near the end of an epoch;
// the second gradient then counts as a duplicate (applied, not re-completed).
__device__ inline void claim_microbatch(const PSArgs& a, int t, long long* s_bid) {
  __shared__ unsigned long long s_c;
  __shared__ unsigned s_e;
  __shared__ int s_k;  // >= 0: claimed offset from the cursor; -1: chunk all complete; -2: finished
  const long long nb = a.nbatches;
  const int rounds = (int)((nb + 63) / 64) + 2;
  for (int r = 0;; ++r) {
    if (t == 0) {
      s_c = __hip_atomic_fetch_add(a.batch_ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      s_e = __hip_atomic_load(a.sched, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    const unsigned e = s_e;
    const unsigned long long c = s_c;
    if (t < 64) {
      int k;
      if (a.max_epochs > 0 && e >= (unsigned)a.max_epochs) {
        k = -2;
      } else {
        const long long j = (long long)((c + (unsigned long long)t) % (unsigned long long)nb);
        const unsigned d = t < nb ? ps_ld_acq(a.done_epoch + j) : 0xffffffffu;
        const unsigned long long inc = __ballot(d < e + 1u);  // incomplete in epoch e
        k = inc ? (int)__builtin_ctzll(inc) : (r + 1 >= rounds ? 0 : -1);
      }
      if (t == 0) s_k = k;
    }
    __syncthreads();
    const int k = s_k;
    if (k == -2) {
      if (t == 0) *s_bid = -1;
      return;
    }
    if (k >= 0) {
      if (t == 0) {
        const long long bb = (long long)((c + (unsigned long long)k) % (unsigned long long)nb);
        if (k > 0) {  // move the shared cursor past the completed batches this claim stepped over
          __hip_atomic_fetch_add(a.batch_ctr, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_fetch_add(a.sched_ctr + 2, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const unsigned prev = __hip_atomic_exchange(a.claimed_epoch + bb, e + 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_SYSTEM);
        if (prev == e + 1u)  // dispatched before in this epoch and not complete: a re-dispatch
          __hip_atomic_fetch_add(a.sched_ctr + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *s_bid = ((long long)e << 32) | bb;
      }
      return;
    }
    if (t == 0) {  // the whole 64-batch chunk is complete: skip it
      __hip_atomic_fetch_add(a.batch_ctr, 63ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_fetch_add(a.sched_ctr + 2, 64ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();  // s_c / s_e / s_k are rewritten by the next round
  }
}

// Completion accounting for an admitted gradient; runs in one thread while it holds the writer lock,
// so every completion is serialised.  A gradient claimed in an older epoch, or for a batch another
// worker already completed, is applied but counted as a duplicate.
__device__ inline void complete_microbatch(const PSArgs& a, long long bid) {
  const unsigned e = (unsigned)(bid >> 32);
  const long long bb = bid & 0xffffffffLL;
  const unsigned cur = __hip_atomic_load(a.sched, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (e != cur || ps_ld_acq(a.done_epoch + bb) == e + 1u) {
    __hip_atomic_fetch_add(a.sched_ctr + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  __hip_atomic_store(a.done_epoch + bb, e + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_fetch_add(a.sched_ctr + 0, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned n = __hip_atomic_load(a.sched + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
  if ((long long)n >= a.nbatches) {  // every batch of epoch e applied: next epoch
    __hip_atomic_store(a.sched + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.sched, e + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    __hip_atomic_store(a.sched + 1, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Stage microbatch `bid`'s example indices (perm row) into the static index buffer: 16-byte copies, all
// loads of a thread in flight before its stores (B even, rows 16-byte aligned).  One workgroup.
// Block-wide copy of n int64 with every load of a pass in flight before its stores (a plain strided copy
// loop waits one memory round trip per iteration).  16-byte vectors when both ends are 16-byte aligned.
__device__ inline void copy_i64(long long* __restrict__ dst, const long long* __restrict__ src, int n, int t, int nt) {
  typedef long long i64x2 __attribute__((ext_vector_type(2)));
  int done = 0;
  if ((((unsigned long long)src | (unsigned long long)dst) & 15) == 0) {
    const int nv = n >> 1;
    const i64x2* s2 = reinterpret_cast<const i64x2*>(src);
    i64x2* d2 = reinterpret_cast<i64x2*>(dst);
    for (int base = t; base < nv; base += nt * 8) {
      i64x2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (base + u * nt < nv) v[u] = s2[base + u * nt];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (base + u * nt < nv) d2[base + u * nt] = v[u];
    }
    done = 2 * nv;
  }
  for (int base = done + t; base < n; base += nt * 8) {
    long long v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (base + u * nt < n) v[u] = src[base + u * nt];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (base + u * nt < n) dst[base + u * nt] = v[u];
  }
}

__device__ inline void ps_stage_indices(const PSArgs& a, long long bid, int t, int nt) {
  if (a.perm == nullptr || bid < 0) return;
  copy_i64(a.idx, a.perm + (bid & 0xffffffffLL) * a.B, a.B, t, nt);
}

}  // namespace dfa
