// Device-resident bounded-staleness parameter server for asynchronous SGD (BASELINE.json configs[2]).
//
// Reference semantics (/root/reference/src/server/asynchronousSGD_server.ts:45-108, client side
// /root/reference/src/client/asynchronousSGD_client.ts:16-84): the server dispenses microbatches
// first-come-first-serve, every worker computes a gradient on the weights it last downloaded, and the
// server applies each gradient on arrival.  The README's intended `maximumStaleness` bound
// (/root/reference/README.md:27) is enforced here.
//
// MI355X design: there is no server thread and no message loop.  The fp32 master is sharded by contiguous
// parameter range over the ranks' HBM (each shard IPC-mapped into every rank); the version counter, the
// FCFS cursor and the completion arrays sit in the server rank's control buffer.  A worker's whole step
// is device work that it replays from its own hipGraph at its own pace:
//   ps_fetch_pull  claim the next microbatch id with a remote atomic (the FCFS dispenser), stage its
//                  example indices; every workgroup reads the fully-applied count, then copies its slice
//                  of the current master out of the shards (vp = the minimum count, ps_device.h);
//   (forward / backward kernels of the model)
//   ps_apply       admit the gradient with one lock-free CAS on the version word (staleness bound
//                  ver - vp), then every workgroup adds -lr * g to its slice of the shards, element by
//                  element (csrc/ps_device.h: plain RMW at world 1, CAS adds otherwise); the last one to
//                  finish publishes the gradient as fully applied.
// No lock is held across an apply, so ranks never serialise behind one another.  Every wait is bounded
// by a wall-clock timeout that sets a sticky error word instead of spinning forever.  Both kernels spread
// the weights over up to 64 workgroups (one workgroup moves only ~60 GB/s of uncached / remote traffic).
//
// Microbatch dispatch is at-least-once and epoch scoped (claim_microbatch / complete_microbatch):
// a batch is complete only once a gradient for it is admitted; rejected ones are dispatched again.
//
// Control buffer layout (server rank): [0] u32 version, [8] u32 fully applied, [16] u64 batch cursor, [32] u32 dataset epoch,
// [36] u32 batches completed in it, [48] u64 completed / redispatched / skipped / duplicate counters,
// [256] u32 done_epoch[kPSMaxBatches], then u32 claimed_epoch[kPSMaxBatches].
#include "common.h"
#include "kernels.h"
#include "ps_device.h"

namespace dfa {
namespace {

constexpr int kPSBlock = 256;
constexpr int kPSUnroll = 4;  // float4 loads in flight per thread per round
constexpr int kPSExclGroups = 2;  // exclusive writer: float4 groups per thread issued at the kernel's start
// Multi-workgroup pull: workgroup 0 claims the microbatch and records the version; every workgroup copies
// its slice of the master out of the shards (4 float4 loads per thread in flight; a slice of 4-aligned
// elements never crosses a shard boundary, shards being multiples of 64 elements).
__global__ __launch_bounds__(kPSBlock) void ps_fetch_pull_kernel(PSArgs a) {
  const int t = threadIdx.x, b = blockIdx.x, G = gridDim.x;
  __shared__ float* tab[kP2PMaxRanks];
  ps_stage_shards(a, tab);
  // the exclusive writer (one rank): no add can land during this copy (the last apply ended with its
  // launch), so the shard loads go out at once, over a wide grid, beside the claim and the version record
  const bool vexcl = a.excl != 0 && a.owner_ring <= 0;
  const long long gstride = (long long)G * kPSBlock;
  f32x4 xv[kPSExclGroups];
  if (vexcl)
#pragma unroll
    for (int k = 0; k < kPSExclGroups; ++k) {
      const long long i = 4 * ((long long)b * kPSBlock + t + k * gstride);
      if (i < a.n) xv[k] = *reinterpret_cast<const f32x4*>(ps_elem(tab, a.shard_shift, i));
    }
  // every workgroup: the fully applied count BEFORE its own slice copy (ps_device.h: vp = the minimum)
  if (t == 0) ps_note_refresh(a, ps_read_applied(a));
  // owner-applies: workgroup 0 takes the drain lock of every shard no other rank is draining (one CAS per
  // shard) and decides, for each shard it holds, how many flagged sequence numbers (in order, from the
  // first one not yet drained) this launch adds into it; the other workgroups take its decision.  Any
  // stepping rank drains, so a rank that stops does not stall the others.
  __shared__ unsigned s_P[kP2PMaxRanks], s_n[kP2PMaxRanks], s_pep;
  if (a.owner_ring > 0 && t == 0) {
    const unsigned R = (unsigned)a.owner_ring;
    const unsigned pep = __hip_atomic_load(a.scratch + kPSPullEp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_pep = pep;
    if (b == 0) {
      for (int k = 0; k < a.nshards; ++k) {
        unsigned P = 0, n = 0, free_ = 0;
        if (__hip_atomic_compare_exchange_strong(a.dlock + k, &free_, (unsigned)a.rank + 1u, __ATOMIC_ACQUIRE,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          P = __hip_atomic_load(a.pref + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const unsigned* fl = ps_inbox_flags(a, k);
          while (n < R && __hip_atomic_load(const_cast<unsigned*>(fl) + (P + n) % R, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_SYSTEM) == P + n + 1u)
            ++n;
          if (n == 0) __hip_atomic_store(a.dlock + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        a.scratch[kPSDrainP + k] = P;
        a.scratch[kPSDrainN + k] = n;
        s_P[k] = P, s_n[k] = n;
      }
      __hip_atomic_store(a.scratch + kPSDrain, pep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const unsigned long long t0 = wall_clock64();
      bool ok = true;
      for (;;) {
        if (__hip_atomic_load(a.scratch + kPSDrain, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pep) break;
        if (wall_clock64() - t0 > 2ull * (unsigned long long)a.timeout_ticks) {
          atomicOr(a.stats + 5, 32ull);
          if (a.herr) __hip_atomic_store(a.herr, 32u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      for (int k = 0; k < a.nshards; ++k) {
        s_P[k] = a.scratch[kPSDrainP + k];
        s_n[k] = ok ? a.scratch[kPSDrainN + k] : 0u;  // (a timed-out workgroup only copies)
      }
    }
  }
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
    ps_stage_indices(a, s_bid, t, kPSBlock);
  }
  if (vexcl) {
#pragma unroll
    for (int k = 0; k < kPSExclGroups; ++k) {
      const long long i = 4 * ((long long)b * kPSBlock + t + k * gstride);
      if (i < a.n) *reinterpret_cast<f32x4*>(a.w + i) = xv[k];
    }
    for (long long i = 4 * ((long long)b * kPSBlock + t + kPSExclGroups * gstride); i < a.n; i += 4 * gstride)
      *reinterpret_cast<f32x4*>(a.w + i) = *reinterpret_cast<const f32x4*>(ps_elem(tab, a.shard_shift, i));
    return;
  }
  __syncthreads();
  const long long per = ((a.n + 4LL * G - 1) / (4LL * G)) * 4;  // slice length, multiple of 4
  const long long lo = b * per, hi = lo + per < a.n ? lo + per : a.n;
  if (a.owner_ring > 0) {
    // the shards this launch drains: add the flagged slots in sequence order (the lock holder is the
    // shard's only writer), store them write-through for the peers' pulls; other shards: copy
    const unsigned R = (unsigned)a.owner_ring;
    const long long mask = (1LL << a.shard_shift) - 1;
    for (long long i = lo + t; i < hi; i += kPSBlock) {
      const int k = (int)(i >> a.shard_shift);
      float* src = tab[k] + (i & mask);
      float v = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(src), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM));
      const unsigned nd = s_n[k];
      if (nd > 0) {
        const unsigned P = s_P[k];
        for (unsigned j = 0; j < nd; ++j)
          v += __uint_as_float(__hip_atomic_load(
              reinterpret_cast<unsigned*>(a.inbox[k] + ((long long)((P + j) % R) << a.shard_shift) + (i & mask)),
              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        __hip_atomic_store(reinterpret_cast<unsigned*>(src), __float_as_uint(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      a.w[i] = v;
    }
    // every shard store has landed before the drained counts are published and the locks released (a
    // sender reuses a slot only once every shard has drained it: ring = max staleness + 2)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      const unsigned prev = __hip_atomic_fetch_add(a.scratch + kPSPullDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (unsigned)G - 1) {
        a.scratch[kPSPullDone] = 0;
        for (int k = 0; k < a.nshards; ++k)
          if (s_n[k] > 0) {
            __hip_atomic_store(a.pref + k, s_P[k] + s_n[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.dlock + k, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        __hip_atomic_store(a.scratch + kPSPullEp, s_pep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  f32x4* d4 = reinterpret_cast<f32x4*>(a.w);
  for (long long base = (lo >> 2) + t; base < (hi >> 2); base += (long long)kPSBlock * kPSUnroll) {
    f32x4 v[kPSUnroll];
#pragma unroll
    for (int u = 0; u < kPSUnroll; ++u) {
      const long long i = base + (long long)u * kPSBlock;
      if (i < (hi >> 2)) v[u] = *reinterpret_cast<const f32x4*>(ps_elem(tab, a.shard_shift, 4 * i));
    }
#pragma unroll
    for (int u = 0; u < kPSUnroll; ++u) {
      const long long i = base + (long long)u * kPSBlock;
      if (i < (hi >> 2)) d4[i] = v[u];
    }
  }
}

// Multi-workgroup apply.  Workgroup 0 admits or rejects (ps_admit: one CAS on the version word, no lock);
// the others wait for that decision on a local word tagged with this launch's epoch and then add their
// slice; the last workgroup to finish advances the epoch.  The grid is small (<= 64 workgroups), so all of
// it is resident and the decision wait cannot starve workgroup 0.
__global__ __launch_bounds__(kPSBlock) void ps_apply_kernel(PSArgs a) {
  const int t = threadIdx.x, b = blockIdx.x, G = gridDim.x;
  __shared__ float* tab[kP2PMaxRanks];
  __shared__ unsigned s_dec;
  __shared__ int s_last;
  ps_stage_shards(a, tab);
  // the exclusive writer (one rank, cached shard memory, no concurrent reader): plain 16-byte read-modify-
  // writes over a wide grid, this thread's first groups of gradient and shard values loaded while
  // workgroup 0 decides (the per-element system-scope path took ~21 us for 600 k parameters)
  const bool vexcl = a.excl != 0 && a.owner_ring <= 0;
  const long long gstride = (long long)G * kPSBlock;
  f32x4 gv[kPSExclGroups], wv[kPSExclGroups];
  if (vexcl)
#pragma unroll
    for (int k = 0; k < kPSExclGroups; ++k) {
      const long long i = 4 * ((long long)b * kPSBlock + t + k * gstride);
      if (i < a.n) {
        gv[k] = *reinterpret_cast<const f32x4*>(a.g + i);
        wv[k] = *reinterpret_cast<const f32x4*>(ps_elem(tab, a.shard_shift, i));
      }
    }
  if (t == 0) {
    const unsigned ep = __hip_atomic_load(a.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (b == 0) {
      const long long bid = *a.bid_out;
      const unsigned dec = ps_admit(a, false);
      // owner-applies: the other workgroups read kPSSeq behind the decision (release); otherwise the word
      // alone is consumed.  The microbatch completion follows the decision, off the critical path.
      if (a.owner_ring > 0)
        __hip_atomic_store(a.scratch + kPSDecision, (ep << 3) | dec, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      else
        __hip_atomic_store(a.scratch + kPSDecision, (ep << 3) | dec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_dec = dec;
      if (dec == kPSAccept && a.done_epoch != nullptr) complete_microbatch(a, bid);
    } else {
      const unsigned long long t0 = wall_clock64();
      unsigned d = 0;
      for (;;) {
        d = __hip_atomic_load(a.scratch + kPSDecision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ps_epoch_eq(d, ep)) break;
        if (wall_clock64() - t0 > 2ull * (unsigned long long)a.timeout_ticks) {
          atomicOr(a.stats + 5, 8ull);
          if (a.herr) __hip_atomic_store(a.herr, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          d = kPSFailed;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_dec = d & 7u;
    }
  }
  __syncthreads();
  __shared__ unsigned s_q;
  if (s_dec == kPSAccept && a.owner_ring > 0) {
    // owner-applies: -lr * g into ring slot q % R of every owner's inbox (plain system-scope stores, no
    // atomics); the last workgroup flags the slot at every owner once all of them have landed
    if (t == 0) {
      if (b != 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (kPSSeq is behind the decision)
      s_q = a.scratch[kPSSeq];
    }
    __syncthreads();
    const long long per = ((a.n + 4LL * G - 1) / (4LL * G)) * 4;
    const long long lo = b * per, hi = lo + per < a.n ? lo + per : a.n;
    const float lr = a.lr_dev ? *a.lr_dev : a.lr;
    const long long soff = (long long)(s_q % (unsigned)a.owner_ring) << a.shard_shift;
    const long long mask = (1LL << a.shard_shift) - 1;
    for (long long i = lo + t; i < hi; i += kPSBlock) {
      float d;
      {
#pragma clang fp contract(off)  // the same rounding as the CAS path
        d = -(lr * a.g[i]);
      }
      __hip_atomic_store(reinterpret_cast<unsigned*>(a.inbox[i >> a.shard_shift] + soff + (i & mask)),
                         __float_as_uint(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  } else if (s_dec == kPSAccept && vexcl) {
    const float lr = a.lr_dev ? *a.lr_dev : a.lr;
#pragma unroll
    for (int k = 0; k < kPSExclGroups; ++k) {
      const long long i = 4 * ((long long)b * kPSBlock + t + k * gstride);
      if (i < a.n) {
        f32x4 nw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma clang fp contract(off)  // the same rounding as the CAS path
          nw[e] = wv[k][e] + -(lr * gv[k][e]);
        }
        *reinterpret_cast<f32x4*>(ps_elem(tab, a.shard_shift, i)) = nw;
      }
    }
    for (long long i = 4 * ((long long)b * kPSBlock + t + kPSExclGroups * gstride); i < a.n; i += 4 * gstride) {
      const f32x4 g4 = *reinterpret_cast<const f32x4*>(a.g + i);
      float* wp = ps_elem(tab, a.shard_shift, i);
      f32x4 w4 = *reinterpret_cast<const f32x4*>(wp);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma clang fp contract(off)
        w4[e] = w4[e] + -(lr * g4[e]);
      }
      *reinterpret_cast<f32x4*>(wp) = w4;
    }
  } else if (s_dec == kPSAccept) {
    const long long per = ((a.n + 4LL * G - 1) / (4LL * G)) * 4;
    const long long lo = b * per, hi = lo + per < a.n ? lo + per : a.n;
    const float lr = a.lr_dev ? *a.lr_dev : a.lr;
    for (long long i0 = lo + t; i0 < hi; i0 += (long long)kPSBlock * kPSUnroll) {
      float* p[kPSUnroll];
      float d[kPSUnroll], nw[kPSUnroll];
#pragma unroll
      for (int u = 0; u < kPSUnroll; ++u) {
        const long long i = i0 + (long long)u * kPSBlock;
        p[u] = i < hi ? ps_elem(tab, a.shard_shift, i) : nullptr;
        d[u] = 0.f;
        if (i < hi) {
#pragma clang fp contract(off)  // the same rounding as the fused reduce launch
          d[u] = -(lr * a.g[i]);
        }
      }
      ps_add<kPSUnroll>(p, d, nw, a.excl != 0, a);
    }
  }
  // every add of this workgroup has landed (results returned / stores acknowledged) before its arrival; the
  // exclusive writer's adds have no reader before the next launch
  if (!vexcl) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.scratch + kPSApplyDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (unsigned)G - 1;
    if (s_last) {
      a.scratch[kPSApplyDone] = 0;
      a.scratch[kPSEpoch] += 1u;
      // every workgroup drained its adds before arriving: the gradient is now fully applied
      if (s_dec == kPSAccept) ps_publish_applied(a);
      if (s_dec == kPSAccept && a.owner_ring > 0)  // every slot store has landed: flag it at every owner
        for (int k = 0; k < a.nshards; ++k)
          __hip_atomic_store(ps_inbox_flags(a, k) + s_q % (unsigned)a.owner_ring, s_q + 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// The exclusive writer's step (one rank; csrc/kernels.h ps_excl_step): the admission of this step's gradient
// (vp: the applied count its weights contain, noted by the previous step's launch or the prologue's pull),
// the refresh record of the NEXT step's weights (the optimizer launch that follows applies this gradient
// when admitted: applied0 + 1 updates), the decision word the optimizer launch is gated on, the completion
// and the next microbatch's claim and index staging.  Two workgroups; no shard access (the gated optimizer
// launch writes the new weights to the local master, its compute copies and the shard, in one pass).
// The claim waits for the admission's completion flag (kPSBidRead = step counter + 1, stored AFTER
// complete_microbatch): a claim that ran beside the completion saw the epoch's last in-flight batch still
// incomplete and dispatched it a second time (one extra "duplicate" update per epoch).
__global__ __launch_bounds__(kPSBlock) void ps_excl_step_kernel(PSArgs a) {
  const int t = threadIdx.x;
  if (blockIdx.x == 0) {  // the admission (one thread)
    if (t != 0) return;
    const unsigned c = __hip_atomic_load(a.scratch + kPSStepCtr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long bid = *a.bid_out;
    const unsigned applied0 = ps_read_applied(a);
    const unsigned ep = __hip_atomic_load(a.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const unsigned dec = ps_admit(a, false, &bid);
    if (dec == kPSAccept || dec == kPSReject) ps_note_refresh(a, applied0 + (dec == kPSAccept ? 1u : 0u));
    // (relaxed: the next launch reads it, behind the kernel boundary)
    __hip_atomic_store(a.scratch + kPSDecision, (ep << 3) | dec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.scratch + kPSEpoch, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dec == kPSAccept) {
      if (a.done_epoch != nullptr) complete_microbatch(a, bid);
      // the gated update lands before anyone can read the count: this rank's next launch
      ps_publish_applied(a);
    }
    // the completion's system-scope writes (done_epoch, the epoch words: write-through, read by the claim
    // with system-scope loads that bypass the caches) are acknowledged before the flag goes out (an agent-
    // scope release would write back this XCD's L2 on the step's critical path)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.scratch + kPSBidRead, c + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // the next microbatch's claim and index staging, once workgroup 0 has read the current id AND completed it
  if (a.perm == nullptr) return;
  __shared__ long long s_bid;
  __shared__ unsigned s_c;
  if (t == 0) {
    const unsigned c = __hip_atomic_load(a.scratch + kPSStepCtr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_c = c;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(a.scratch + kPSBidRead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != c + 1u) {
      if (wall_clock64() - t0 > 2ull * (unsigned long long)a.timeout_ticks) {  // never expected
        atomicOr(a.stats + 5, 8ull);
        if (a.herr) __hip_atomic_store(a.herr, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (a.done_epoch != nullptr) {
    claim_microbatch(a, t, &s_bid);
  } else if (t == 0) {
    s_bid = (long long)(__hip_atomic_fetch_add(a.batch_ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) %
                        (unsigned long long)(a.nbatches > 0 ? a.nbatches : 1));
  }
  __syncthreads();
  if (t == 0) {
    *a.bid_out = s_bid;
    __hip_atomic_store(a.scratch + kPSStepCtr, s_c + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  ps_stage_indices(a, s_bid, t, kPSBlock);
}

// Shard self-test: thread j < n of workgroup k adds (rank + 1) * (j + 1) to word j of shard k's test area
// through the same element add as the apply.
__global__ void ps_selftest_kernel(PSArgs a, float* const* words, int n, float rank1) {
  const int k = blockIdx.x, j = threadIdx.x;
  if (j >= n) return;
  float* p[1] = {words[k] + j};
  const float d[1] = {rank1 * (float)(j + 1)};
  float o[1];
  ps_add<1>(p, d, o, a.excl != 0, a);
}

// Apply-path calibration (AsyncPSTrainer setup, every rank at once, before the master is seeded): the two ways
// an admitted gradient reaches the sharded master, over this model's n elements with a zero update (no value
// changes), on the real topology:
//   mode 0  the CAS path's per-element compare-and-swap adds on the owning shards (ps_add, shared form);
//   mode 1  owner-applies: the plain store into the element's inbox ring slot R - 1, the shard load of the
//           refresh and one inbox-slot load of the drain (each admitted gradient is drained once per element).
__global__ __launch_bounds__(kPSBlock) void ps_calib_kernel(PSArgs a, int mode) {
  __shared__ float* tab[kP2PMaxRanks];
  __shared__ float* itab[kP2PMaxRanks];
  if (mode == 1 && threadIdx.x < kP2PMaxRanks) {
    float* v = nullptr;
#pragma unroll
    for (int k = 0; k < kP2PMaxRanks; ++k)
      if ((int)threadIdx.x == k) v = a.inbox[k];
    itab[threadIdx.x] = v;
  }
  ps_stage_shards(a, tab);
  const int t = threadIdx.x, b = blockIdx.x, G = gridDim.x;
  const long long per = ((a.n + 4LL * G - 1) / (4LL * G)) * 4;
  const long long lo = b * per, hi = lo + per < a.n ? lo + per : a.n;
  if (mode == 0) {
    for (long long i0 = lo + t; i0 < hi; i0 += (long long)kPSBlock * kPSUnroll) {
      float* p[kPSUnroll];
      float d[kPSUnroll], nw[kPSUnroll];
#pragma unroll
      for (int u = 0; u < kPSUnroll; ++u) {
        const long long i = i0 + (long long)u * kPSBlock;
        p[u] = i < hi ? ps_elem(tab, a.shard_shift, i) : nullptr;
        d[u] = 0.f;
      }
      ps_add<kPSUnroll>(p, d, nw, false, a);
    }
    return;
  }
  const long long mask = (1LL << a.shard_shift) - 1;
  const unsigned R = (unsigned)a.owner_ring;
  float acc = 0.f;
  for (long long i = lo + t; i < hi; i += kPSBlock) {
    const int k = (int)(i >> a.shard_shift);
    __hip_atomic_store(reinterpret_cast<unsigned*>(itab[k] + ((long long)(R - 1) << a.shard_shift) + (i & mask)), 0u,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    acc += __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(tab[k] + (i & mask)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM));
    acc += __uint_as_float(__hip_atomic_load(
        reinterpret_cast<unsigned*>(itab[k] + ((long long)(R - 2) << a.shard_shift) + (i & mask)), __ATOMIC_RELAXED,
        __HIP_MEMORY_SCOPE_SYSTEM));
  }
  asm volatile("" ::"v"(acc));
}

}  // namespace

// ~16 KB of weights per workgroup, at most kPSMaxGrid workgroups (all resident: the apply kernel's
// decision wait relies on it)
static int ps_grid(long long n) {
  long long g = (n + 4095) / 4096;
  return (int)(g < 1 ? 1 : (g > kPSMaxGrid ? kPSMaxGrid : g));
}

// exclusive writer: one workgroup per 2 K elements (kPSExclGroups float4 per thread), at most 2048;
// otherwise ps_grid
static int ps_excl_grid(const PSArgs& a) {
  if (a.excl == 0 || a.owner_ring > 0) return ps_grid(a.n);
  const long long g = (a.n + 4LL * kPSBlock * kPSExclGroups - 1) / (4LL * kPSBlock * kPSExclGroups);
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

static bool ps_shards_ok(const PSArgs& a) {
  if (a.nshards < 1 || a.nshards > kP2PMaxRanks || a.shard_shift < 6 || a.shard_shift > 30 || !a.ver) return false;
  if (((a.n - 1) >> a.shard_shift) >= a.nshards) return false;
  for (int k = 0; k < a.nshards; ++k)
    if (!a.shard[k]) return false;
  return true;
}

// owner-applies arguments: every owner's inbox, the drained counts, this rank, a ring of <= 255 slots (the
// drain decision packs the count in 8 bits)
static bool ps_owner_ok(const PSArgs& a) {
  if (a.owner_ring <= 0) return true;
  if (!a.pref || !a.dlock || a.rank < 0 || a.owner_ring > 255) return false;  // (a joiner's id is >= nshards)
  for (int k = 0; k < a.nshards; ++k)
    if (!a.inbox[k]) return false;
  return true;
}

hipError_t ps_fetch_pull(const PSArgs& a, hipStream_t st) {
  if (a.n <= 0 || (a.n & 3) || !ps_shards_ok(a) || !ps_owner_ok(a) ||
      (a.perm != nullptr && (a.B <= 0 || (a.B & 1) || a.nbatches <= 0)))
    return hipErrorInvalidValue;
  ps_fetch_pull_kernel<<<ps_excl_grid(a), kPSBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t ps_apply(const PSArgs& a, hipStream_t st) {
  if (a.n <= 0 || (a.n & 3) || !ps_shards_ok(a) || !ps_owner_ok(a)) return hipErrorInvalidValue;
  // a slot is rewritten R sequence numbers later; every owner has drained it by then only if an admitted
  // gradient is at most R - 2 behind (its pull saw min_k pref[k] >= q - max_stale)
  if (a.owner_ring > 0 && (a.max_stale < 0 || a.owner_ring < a.max_stale + 2)) return hipErrorInvalidValue;
  ps_apply_kernel<<<ps_excl_grid(a), kPSBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t ps_excl_step(const PSArgs& a, hipStream_t st) {
  if (a.excl == 0 || a.owner_ring > 0 || a.nshards != 1 || !ps_shards_ok(a) ||
      (a.perm != nullptr && (a.B <= 0 || (a.B & 1) || a.nbatches <= 0)))
    return hipErrorInvalidValue;
  ps_excl_step_kernel<<<2, kPSBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t ps_calibrate(const PSArgs& a, int mode, hipStream_t st) {
  if (a.n <= 0 || (a.n & 3) || !ps_shards_ok(a) || (mode != 0 && mode != 1) ||
      (mode == 1 && (a.owner_ring < 2 || !ps_owner_ok(a))))
    return hipErrorInvalidValue;
  // the fused LeNet-5 reduce applies from ~600 workgroups at once: a wide grid (one float4 group per thread)
  const long long g = (a.n + 4LL * kPSBlock - 1) / (4LL * kPSBlock);
  ps_calib_kernel<<<(int)(g < 1 ? 1 : (g > 1024 ? 1024 : g)), kPSBlock, 0, st>>>(a, mode);
  return hipGetLastError();
}

hipError_t ps_selftest_add(const PSArgs& a, float* const* words, int n, float rank1, hipStream_t st) {
  if (n <= 0 || n > kPSBlock || a.nshards < 1 || a.nshards > kP2PMaxRanks || !words) return hipErrorInvalidValue;
  ps_selftest_kernel<<<a.nshards, kPSBlock, 0, st>>>(a, words, n, rank1);
  return hipGetLastError();
}

}  // namespace dfa
