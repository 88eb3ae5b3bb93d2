// Device-side protocol pieces of the parameter server shared by csrc/async_ps.hip (pull / apply
// launches) and the fused LeNet-5 reduce kernel, which applies an admitted gradient to the sharded
// master itself (csrc/lenet_fused.hip): the lock-free admission decision, the per-element shard adds,
// microbatch claims and completion accounting.
//
// Reference: AsynchronousSGDServer applies every uploaded gradient on arrival and hands out the next
// batch (/root/reference/src/server/asynchronousSGD_server.ts:65-82,95-108): a version only ever names
// fully applied weights (updateModel applies, then save() bumps the version, :73-77,95-108).  The
// README's maximumStaleness bound (/root/reference/README.md:27) is the admission check here.  Nothing
// in the protocol holds a lock across an apply, so applies of different ranks proceed in parallel:
//   admission   one CAS on the shared version word `ver` (= gradients admitted so far): admitted iff
//               ver - vp <= max_stale, and then ver -> ver + 1 (a failed CAS re-reads and re-checks);
//   apply       per element, w += -(lr * g) on the owning shard: a plain read-modify-write when this
//               rank is the only writer (world 1), else a compare-and-swap loop on the element's bits
//               (no add is lost; adds of different ranks to one element serialise in memory only); when
//               every add of an admitted gradient has landed, its last workgroup bumps the shared
//               `applied` counter (the count of FULLY applied gradients);
//   refresh     every workgroup that copies weights out of the shards (a pull, or the refresh of the
//               fused reduce launch) first reads `applied` = A, then copies: the copy contains at least
//               those A updates on every element (plus its own, when the refresh is its own admitted
//               add).  vp = the minimum of A (+ own) over the refreshing workgroups (kPSVMin).
// So `ver - vp` at admission bounds from above the number of admitted updates missing from ANY element
// of the weights the gradient was computed on: the staleness bound holds exactly at every world size
// (conservatively: an add in flight but partly landed counts as missing).
#pragma once
#include "common.h"
#include "kernels.h"

namespace dfa {

// local scratch words (PSArgs::scratch, u32 index)
// kPSVMin: min over this step's refreshing workgroups of (applied read before the copy [+ 1 for its own
// admitted add]); reset to kPSNoVer by the admission that consumes it
constexpr int kPSPullDone = 0, kPSApplyDone = 1, kPSEpoch = 2, kPSDecision = kPSDecisionWord, kPSVMin = kPSVMinWord, kPSSlots = 64;
// owner-applies words: the admitted sequence number, the pull launches' epoch, the drain decision's epoch
// and, per shard, the first sequence number and the count this launch drains
constexpr int kPSSeq = 5, kPSPullEp = 6, kPSDrain = 7, kPSDrainP = 8, kPSDrainN = 16;  // (+ shard, < 8 each)
// exclusive-writer step (async_ps.hip ps_excl_step): its claim workgroup's step counter, and the admission
// workgroup's "microbatch id read" flag (= counter + 1) the claim waits for before overwriting the id
constexpr int kPSStepCtr = 24, kPSBidRead = 25;  // kPSBidRead: "id read and completed" flag
constexpr unsigned kPSNoVer = 0xffffffffu;
// the decision word is (launch epoch << 3) | code: compare epochs modulo 2^29
__device__ __forceinline__ bool ps_epoch_eq(unsigned word, unsigned ep) { return (word >> 3) == (ep & 0x1fffffffu); }
// decision codes: admitted (apply + refresh from the new values), rejected as too stale (refresh from the
// current values), the schedule is finished (no-op), or a wait timed out (no-op, error bits set)
constexpr unsigned kPSAccept = 1, kPSReject = 2, kPSFailed = 3, kPSFinished = 4;

__device__ __forceinline__ unsigned ps_ld_acq(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The exclusive writer (one rank: no other agent touches the server words) needs no acquire / release on
// them: each system-scope acquire invalidates and each release writes back the issuing XCD's L2, several
// microseconds on the async step's critical path.  These helpers drop the ordering when a.excl.
__device__ __forceinline__ unsigned ps_ld_acq_x(const PSArgs& a, const unsigned* p) {
  return a.excl ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : ps_ld_acq(p);
}

// The fully applied count, read by thread 0 of every workgroup that refreshes weights from the shards
// BEFORE any of its shard reads or adds (reading it earlier only makes the count more conservative, so the
// fused reduce launch reads it at its start, where the load's latency hides behind the jobs).
__device__ __forceinline__ unsigned ps_read_applied(const PSArgs& a) {
  if (a.owner_ring > 0) {  // owner-applies: every owner has drained at least the minimum
    unsigned m = 0xffffffffu;
    for (int k = 0; k < a.nshards; ++k) {
      const unsigned p = __hip_atomic_load(a.pref + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      m = p < m ? p : m;
    }
    return m;
  }
  return a.applied ? __hip_atomic_load(a.applied, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
}
// owner k's inbox flags (after its owner_ring slots)
__device__ __forceinline__ unsigned* ps_inbox_flags(const PSArgs& a, int k) {
  return reinterpret_cast<unsigned*>(a.inbox[k] + ((long long)a.owner_ring << a.shard_shift));
}
// owner-applies drain decisions of the fused LeNet-5 step (csrc/lenet_fused.hip mode 4): one u64 per shard in
// the local scratch (u32 words 32..47), (launch epoch & 0xffffff) << 40 | count << 32 | first sequence number
constexpr int kPSOwnerDrainWords = 32;
__device__ __forceinline__ unsigned long long* ps_owner_drain_words(const PSArgs& a) {
  return reinterpret_cast<unsigned long long*>(a.scratch + kPSOwnerDrainWords);
}
__device__ __forceinline__ unsigned long long ps_owner_word(unsigned ep, unsigned n, unsigned P) {
  return ((unsigned long long)(ep & 0xffffffu) << 40) | ((unsigned long long)(n & 0xffu) << 32) | P;
}
__device__ __forceinline__ unsigned ps_owner_word_ep(unsigned long long w) { return (unsigned)(w >> 40); }
// Records that this workgroup's refresh contains `count` fully applied gradients (the applied count it read
// + 1 when the refresh values are the results of this rank's own admitted adds): kPSVMin = the minimum.
__device__ __forceinline__ void ps_note_refresh(const PSArgs& a, unsigned count) {
  if (a.applied != nullptr)
    __hip_atomic_fetch_min(a.scratch + kPSVMin, count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The last workgroup of an ADMITTED apply, after every add of the gradient has landed: each workgroup drained
// its adds (CAS results returned / plain stores acknowledged, s_waitcnt vmcnt(0)) before its arrival, and
// the shards are uncached memory, so nothing remains to be written back: a relaxed add orders behind them
// (a system-scope release here would write back this XCD's L2, ~2-7 us on the critical path).
__device__ __forceinline__ void ps_publish_applied(const PSArgs& a) {
  if (a.owner_ring > 0) return;  // owner-applies: the owners' drains publish (pref)
  if (a.applied != nullptr) __hip_atomic_fetch_add(a.applied, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
      s_e = ps_ld_acq_x(a, a.sched);
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
        const unsigned d = t < nb ? ps_ld_acq_x(a, a.done_epoch + j) : 0xffffffffu;
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

// Completion accounting for an admitted gradient, lock-free (admissions of different ranks may run it
// concurrently).  The exchange on done_epoch[b] makes exactly one admitted gradient per (batch, epoch)
// the completing one; a gradient claimed in an older epoch, or for a batch another worker already
// completed, is applied but counted as a duplicate.  The completion that brings the epoch's count to
// nbatches resets the count and opens the next epoch (a completion of epoch e + 1 needs a claim made
// after that release, so no completion of the new epoch is counted before the reset).
__device__ inline void complete_microbatch(const PSArgs& a, long long bid) {
  const unsigned e = (unsigned)(bid >> 32);
  const long long bb = bid & 0xffffffffLL;
  const unsigned cur = __hip_atomic_load(a.sched, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned prev_done;
  if (a.excl)
    prev_done = e != cur ? 0u : __hip_atomic_exchange(a.done_epoch + bb, e + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else
    prev_done = e != cur ? 0u : __hip_atomic_exchange(a.done_epoch + bb, e + 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
  if (e != cur || prev_done == e + 1u) {
    __hip_atomic_fetch_add(a.sched_ctr + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  __hip_atomic_fetch_add(a.sched_ctr + 0, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned n = (a.excl ? __hip_atomic_fetch_add(a.sched + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                             : __hip_atomic_fetch_add(a.sched + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM)) + 1u;
  if ((long long)n >= a.nbatches) {  // every batch of epoch e applied: next epoch
    __hip_atomic_store(a.sched + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (a.excl) __hip_atomic_store(a.sched, e + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_store(a.sched, e + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The admission decision for the gradient of microbatch *bid_out (one thread).  Lock-free: read the
// version, check the staleness bound against vp (kPSVMin, see the header), CAS version -> version + 1; a
// CAS lost to another rank's admission re-reads and re-checks.  Records vp in *vpulled, the counters, the
// optional audit row and the microbatch completion.  Returns the decision code.
__device__ inline unsigned ps_admit(const PSArgs& a, bool complete_now = true, const long long* bid_pre = nullptr) {
  // every independent load first (one memory round trip, not one per load: the admission is the async
  // step's critical path), then the CAS.  bid_pre: the microbatch id as the caller read it (the id word
  // may be rewritten by a concurrent claim once the caller has read it)
  const long long bid = bid_pre ? *bid_pre : *a.bid_out;
  const unsigned long long s0 = a.stats[0], s1 = a.stats[1], s2 = a.stats[2], s3 = a.stats[3];
  unsigned vp = __hip_atomic_load(a.scratch + kPSVMin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned v = __hip_atomic_load(a.ver, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long k = s0 + s1;  // this rank's decision index
  if (a.done_epoch != nullptr && bid < 0) {  // dataset finished: a no-op step (no refresh follows)
    a.stats[6] += 1;
    return kPSFinished;
  }
  const unsigned long long t0 = wall_clock64();
  if (vp == kPSNoVer) vp = 0;  // no refresh recorded (never on a well-formed step): count from version 0
  // consumed: this step's refreshers record afresh (they run after the decision, which is published
  // with release semantics behind this store)
  __hip_atomic_store(a.scratch + kPSVMin, kPSNoVer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *a.vpulled = vp;
  auto audit = [&](unsigned dec) {
    if (a.audit != nullptr && k < (unsigned long long)a.audit_cap) {
      a.audit[3 * k] = v;
      a.audit[3 * k + 1] = vp;
      a.audit[3 * k + 2] = dec;
    }
  };
  unsigned long long retries = 0;
  for (;;) {
    const unsigned stale = v - vp;
    if (a.max_stale >= 0 && (int)stale > a.max_stale) {
      a.stats[1] = s1 + 1;
      if (retries) a.stats[4] += retries;
      audit(kPSReject);
      return kPSReject;
    }
    unsigned expected = v;
    const bool won = a.excl ? __hip_atomic_compare_exchange_strong(a.ver, &expected, v + 1u, __ATOMIC_RELAXED,
                                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                            : __hip_atomic_compare_exchange_strong(a.ver, &expected, v + 1u, __ATOMIC_ACQ_REL,
                                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (won) {
      a.scratch[kPSSeq] = v;  // this gradient's sequence number (owner-applies: its ring slot)
      a.stats[0] = s0 + 1;
      a.stats[2] = s2 + stale;
      if (stale > s3) a.stats[3] = stale;
      if (retries) a.stats[4] += retries;
      audit(kPSAccept);
      // (complete_now false: the caller completes the microbatch after publishing the decision)
      if (a.done_epoch != nullptr && complete_now) complete_microbatch(a, bid);
      return kPSAccept;
    }
    v = expected;  // another rank admitted in between: re-check against its version
    ++retries;
    if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) {
      a.stats[4] += retries;
      atomicOr(a.stats + 5, 4ull);
      if (a.herr) __hip_atomic_store(a.herr, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return kPSFailed;
    }
  }
}

// The shard bases into LDS (indexing the by-value kernel argument with a run-time shard number would
// copy the whole argument block to scratch per thread).  Every thread of the workgroup calls it.
__device__ __forceinline__ void ps_stage_shards(const PSArgs& a, float** tab, bool barrier = true) {
  if (threadIdx.x < kP2PMaxRanks) {
    float* v = nullptr;
#pragma unroll
    for (int k = 0; k < kP2PMaxRanks; ++k)
      if ((int)threadIdx.x == k) v = a.shard[k];
    tab[threadIdx.x] = v;
  }
  if (barrier) __syncthreads();  // (false: the caller's next barrier publishes the table)
}

// Address of master element i (tab: the shard bases, staged in LDS by the caller)
__device__ __forceinline__ float* ps_elem(float* const* tab, int shift, long long i) {
  return tab[i >> shift] + (i & ((1LL << shift) - 1));
}

// w += d for N elements (p[e] null: skip), returning the new values.  Exclusive writer: plain loads, then
// stores.  Shared: every element's load in flight, then every CAS in flight, re-trying the ones another
// rank's add beat (bounded by the timeout; a timed-out element keeps its loaded value).
template <int N>
__device__ __forceinline__ void ps_add(float* const (&p)[N], const float (&d)[N], float (&out)[N], bool excl,
                                       const PSArgs& a) {
  unsigned cur[N];
#pragma unroll
  for (int e = 0; e < N; ++e)
    cur[e] = p[e] ? __hip_atomic_load(reinterpret_cast<unsigned*>(p[e]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
  if (excl) {
#pragma unroll
    for (int e = 0; e < N; ++e) {
#pragma clang fp contract(off)
      out[e] = __uint_as_float(cur[e]) + d[e];
      if (p[e]) __hip_atomic_store(reinterpret_cast<unsigned*>(p[e]), __float_as_uint(out[e]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  unsigned pending = 0;
#pragma unroll
  for (int e = 0; e < N; ++e)
    if (p[e]) pending |= 1u << e;
  const unsigned long long t0 = wall_clock64();
  while (pending) {
#pragma unroll
    for (int e = 0; e < N; ++e) {
      if (!((pending >> e) & 1u)) continue;
      float nw;
      {
#pragma clang fp contract(off)
        nw = __uint_as_float(cur[e]) + d[e];
      }
      unsigned expected = cur[e];
      if (__hip_atomic_compare_exchange_strong(reinterpret_cast<unsigned*>(p[e]), &expected, __float_as_uint(nw),
                                               __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
        out[e] = nw;
        pending &= ~(1u << e);
      } else {
        cur[e] = expected;
      }
    }
    if (pending && wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) {
      atomicOr(a.stats + 5, 16ull);
      if (a.herr) __hip_atomic_store(a.herr, 16u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
      for (int e = 0; e < N; ++e)
        if ((pending >> e) & 1u) out[e] = __uint_as_float(cur[e]);
      break;
    }
  }
#pragma unroll
  for (int e = 0; e < N; ++e)
    if (!p[e]) out[e] = 0.f;
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
