// Device FedSGD with a count barrier of K < W: the reference FederatedServer on the device parameter
// server's memory (BASELINE.json configs[1] FedSGD semantics).
//
// Reference (/root/reference/src/server/federated_server.ts:71-117): an upload is accepted only when its
// gradient was computed on the CURRENT model version and no update is in progress; after
// minUpdatesPerVersion (K) accepted uploads the server averages them, applies w -= lr * mean, bumps the
// version and broadcasts it.  Late uploads of an old version are dropped, so the barrier counts updates,
// not workers: a slow or lost worker never blocks a version.
//
// MI355X design: no server process.  The fp32 master is sharded over the ranks' HBM (PSComm, the async
// engine's shards); the version is a seqlock word in the control buffer (even 2v: version v stable, odd:
// being applied).  Per step a rank
//   fed_pull    copies the master with the seqlock (a copy that saw the word change is retried) and records
//               the even word it copied under (every workgroup; a step whose workgroups saw different
//               versions is dropped at upload);
//   (the model's forward / backward on its own microbatch)
//   fed_upload  takes a ticket for that version: one CAS on a (version << 32 | count) word -- stale
//               version, update in progress or count >= K: dropped; else slot t = the count.  The admitted
//               gradient is stored into slot t (sharded like the master, plain stores) and, once every
//               workgroup's slice has landed, its bit is set on the (version << 32 | landed-slot mask) word;
//               the lander that completes the mask is this version's applier;
//   fed_apply   (a no-op unless this rank is an applier) takes the version by one CAS of the seqlock word
//               v -> v + 1 (odd; the one winner applies, so a second applier -- a recovering rank -- never
//               applies twice), adds -lr * mean of the version's good slots (fixed slot order: every element
//               gets the same arithmetic whoever applies) into the master shards and publishes v + 1 (even).
// Liveness: a version must close even when a ticket holder never lands or the applier never
// applies.  (1) A landing counts as good only if every workgroup of the upload stored its slice; a torn
// upload (a workgroup's decision wait timed out) lands its slot as BAD (the version's bad-slot mask, so
// the apply excludes it) instead of not landing.  (2) A rank whose uploads see the same version full for
// longer than the timeout recovers it: the slots that never landed are landed as bad, and it becomes an
// applier itself (a dead applier never takes the seqlock); a won recovery apply is counted (stats[5]), and
// a version still stuck a second timeout later sets a sticky error bit.
// Every wait is bounded by a wall-clock timeout that sets a sticky error bit instead of spinning forever.
#include "common.h"
#include "kernels.h"
#include "ps_device.h"

namespace dfa {
namespace {

constexpr int kFedBlock = 256;
constexpr unsigned kFedAdmit = 1, kFedStale = 2, kFedFull = 3, kFedFailed = 4;
// local scratch words (FedArgs::scratch): decision word (epoch << 3 | code), the admitted slot, launch epoch,
// arrivals of the upload / apply launches, the applier flag (version seqlock word + 1, 0 = not the applier),
// torn-upload count (workgroups of this launch that stored nothing), the version first seen full + 1 and
// that time (u64 in two words), the apply launches' epoch and decision (epoch << 1 | won) and whether the
// applier flag comes from a recovery, and per pull workgroup the seqlock word it copied under
constexpr int kFedDecision = 0, kFedSlot = 1, kFedEpoch = 2, kFedUpDone = 3, kFedApDone = 4, kFedApplier = 5,
              kFedTorn = 6, kFedFullV = 7, kFedFullT = 8, kFedApEp = 10, kFedApDec = 11, kFedRecov = 12,
              kFedPulled = 64;
// error bits (stats[7]): 1 pull timed out, 2 admission CAS timed out, 4 decision wait timed out, 8 torn upload
// landed as a bad slot, 16 a version stayed full past twice the timeout even after a recovery
constexpr unsigned kFedErrTorn = 8u, kFedErrStuck = 16u;

// OR `bits` into a (version << 32 | mask) word for version vp (a word of an older version restarts)
__device__ inline unsigned long long fed_or_tagged(unsigned long long* w, unsigned vp, unsigned bits) {
  unsigned long long cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    const unsigned long long nw = ((unsigned)(cur >> 32) == vp) ? (cur | bits) : (((unsigned long long)vp << 32) | bits);
    if (__hip_atomic_compare_exchange_strong(w, &cur, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
      return nw;
  }
}
__device__ __forceinline__ unsigned fed_full_mask(int K) { return K >= 32 ? 0xffffffffu : ((1u << K) - 1u); }
__device__ __forceinline__ unsigned fed_ld(const unsigned* p) {
  return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The master shards and the slots live in other ranks' memory (IPC-mapped; on a shared GPU the importing
// process may map them cacheable): every access to them is a system-scope one, so no XCD's L2 serves a
// stale line and no store waits in one (4-byte relaxed atomics: global_load / store with sc0 sc1).
__device__ __forceinline__ f32x4 fed_ld4(const float* p) {
  f32x4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    v[j] = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(const_cast<float*>(p)) + j, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM));
  return v;
}
__device__ __forceinline__ void fed_st4(float* p, const f32x4& v) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    __hip_atomic_store(reinterpret_cast<unsigned*>(p) + j, __float_as_uint(v[j]), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ float* fed_elem(float* const* tab, int shift, long long i, long long slot_off) {
  return tab[i >> shift] + slot_off + (i & ((1LL << shift) - 1));
}

__device__ __forceinline__ void fed_stage(const FedArgs& a, float** master, float** slots) {
  if (threadIdx.x < kP2PMaxRanks) {
    float *m = nullptr, *s = nullptr;
#pragma unroll
    for (int k = 0; k < kP2PMaxRanks; ++k)
      if ((int)threadIdx.x == k) m = a.shard[k], s = a.slot[k];
    master[threadIdx.x] = m;
    slots[threadIdx.x] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ void fed_fail(const FedArgs& a, unsigned bit) {
  atomicOr(a.stats + 7, (unsigned long long)bit);
  if (a.herr) __hip_atomic_store(a.herr, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the slice of workgroup b of G: 4-aligned, never crossing a shard (shards are multiples of 64 elements)
__device__ __forceinline__ void fed_slice(const FedArgs& a, int b, int G, long long& lo, long long& hi) {
  const long long per = ((a.n + 4LL * G - 1) / (4LL * G)) * 4;
  lo = b * per;
  hi = lo + per < a.n ? lo + per : a.n;
}

__global__ __launch_bounds__(kFedBlock) void fed_pull_kernel(FedArgs a) {
  __shared__ float* master[kP2PMaxRanks];
  __shared__ float* slots[kP2PMaxRanks];
  __shared__ unsigned s_seq;
  __shared__ int s_ok;
  fed_stage(a, master, slots);
  long long lo, hi;
  fed_slice(a, blockIdx.x, gridDim.x, lo, hi);
  const unsigned long long t0 = wall_clock64();
  for (int attempt = 0;; ++attempt) {
    if (threadIdx.x == 0) {
      unsigned s = fed_ld(a.seq);
      while (s & 1u) {  // a version is being applied: wait for it
        if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) break;
        __builtin_amdgcn_s_sleep(2);
        s = fed_ld(a.seq);
      }
      s_seq = s;
    }
    __syncthreads();
    const unsigned s0 = s_seq;
    for (long long i = lo + 4LL * threadIdx.x; i < hi; i += 4LL * kFedBlock) {
      const f32x4 v = fed_ld4(fed_elem(master, a.shard_shift, i, 0));
      *reinterpret_cast<f32x4*>(a.w + i) = v;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the copy's loads returned before the re-check
    __syncthreads();
    if (threadIdx.x == 0) s_ok = fed_ld(a.seq) == s0 && !(s0 & 1u);
    __syncthreads();
    if (s_ok) break;
    if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) {
      if (threadIdx.x == 0) {
        fed_fail(a, 1u);
        s_seq = 1u;  // odd: the upload drops this step
      }
      __syncthreads();
      break;
    }
  }
  if (threadIdx.x == 0) a.scratch[kFedPulled + blockIdx.x] = s_seq;
}

// admission (one thread): the ticket of version word s (even) on the (version << 32 | count) word
__device__ inline unsigned fed_admit(const FedArgs& a, int pull_blocks, unsigned* slot_out, unsigned* vp_out) {
  const unsigned vp = a.scratch[kFedPulled];
  *vp_out = vp;
  bool torn = (vp & 1u) != 0;
  for (int b = 1; b < pull_blocks; ++b) torn |= a.scratch[kFedPulled + b] != vp;
  if (torn || fed_ld(a.seq) != vp) return kFedStale;
  unsigned long long w = __hip_atomic_load(a.tick, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    const unsigned tag = (unsigned)(w >> 32), cnt = (unsigned)w;
    unsigned long long nw;
    unsigned t;
    if (tag == vp) {
      if (cnt >= (unsigned)a.K) return kFedFull;
      t = cnt;
      nw = w + 1ull;
    } else if ((int)(tag - vp) < 0) {  // the first upload of version vp
      t = 0;
      nw = ((unsigned long long)vp << 32) | 1ull;
    } else {
      return kFedStale;  // the word already names a newer version
    }
    if (__hip_atomic_compare_exchange_strong(a.tick, &w, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM)) {
      // (the version cannot close before this ticket lands: closing takes K landed tickets < K, and this
      // is one of them -- so an admitted gradient must always land, or the version never closes)
      *slot_out = t;
      return kFedAdmit;
    }
    if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) return kFedFailed;
  }
}

__global__ __launch_bounds__(kFedBlock) void fed_upload_kernel(FedArgs a, int pull_blocks) {
  __shared__ float* master[kP2PMaxRanks];
  __shared__ float* slots[kP2PMaxRanks];
  __shared__ unsigned s_dec, s_slot, s_vp;
  fed_stage(a, master, slots);
  const int G = gridDim.x;
  if (threadIdx.x == 0) {
    const unsigned ep = __hip_atomic_load(a.scratch + kFedEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (blockIdx.x == 0) {
      unsigned slot = 0, vp = 0;
      const unsigned dec = fed_admit(a, pull_blocks, &slot, &vp);
      unsigned applier = 0, recov = 0;
      if (dec == kFedFull) {
        // the version is full: note when this rank first saw it so; past the timeout, recover it
        const unsigned long long now = wall_clock64();
        if (a.scratch[kFedFullV] != vp + 1u) {
          a.scratch[kFedFullV] = vp + 1u;
          a.scratch[kFedFullT] = (unsigned)now;
          a.scratch[kFedFullT + 1] = (unsigned)(now >> 32);
        } else {
          const unsigned long long t1 =
              ((unsigned long long)a.scratch[kFedFullT + 1] << 32) | (unsigned long long)a.scratch[kFedFullT];
          if (now - t1 > (unsigned long long)a.timeout_ticks && fed_ld(a.seq) == vp) {
            // tickets taken but never landed (their rank died or stalled): landed as bad slots, then the
            // apply claimed if no lander or dead applier has claimed it
            const unsigned long long lw = __hip_atomic_load(a.land, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const unsigned landed = (unsigned)(lw >> 32) == vp ? (unsigned)lw : 0u;
            const unsigned missing = fed_full_mask(a.K) & ~landed;
            if (missing) {
              fed_or_tagged(a.bad, vp, missing);
              fed_or_tagged(a.land, vp, missing);
            }
            applier = vp + 1u, recov = 1u;  // (the apply's seqlock CAS picks one winner)
            if (now - t1 > 2ull * (unsigned long long)a.timeout_ticks)
              fed_fail(a, kFedErrStuck);  // a recovery already ran a timeout ago and the version did not move
          }
        }
      }
      const unsigned long long k = a.stats[0] + a.stats[1] + a.stats[2] + a.stats[3];
      a.stats[dec == kFedAdmit ? 0 : dec == kFedStale ? 1 : dec == kFedFull ? 2 : 3] += 1;
      if (dec == kFedFailed) fed_fail(a, 2u);
      if (a.audit && k < (unsigned long long)a.audit_cap) {
        a.audit[3 * k] = vp;
        a.audit[3 * k + 1] = dec;
        a.audit[3 * k + 2] = dec == kFedAdmit ? slot : 0xffffffffu;
      }
      a.scratch[kFedSlot] = slot;
      a.scratch[kFedApplier] = applier;
      a.scratch[kFedRecov] = recov;
      __hip_atomic_store(a.scratch + kFedDecision, ((ep & 0x1fffffffu) << 3) | dec, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
      s_dec = dec, s_slot = slot, s_vp = vp;
    } else {
      const unsigned long long t0 = wall_clock64();
      unsigned d = 0;
      for (;;) {
        d = __hip_atomic_load(a.scratch + kFedDecision, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if ((d >> 3) == (ep & 0x1fffffffu)) break;
        if (wall_clock64() - t0 > 2ull * (unsigned long long)a.timeout_ticks) {
          fed_fail(a, 4u);
          // this workgroup stores no slice: if workgroup 0 did admit, the landing must not count as good
          __hip_atomic_fetch_add(a.scratch + kFedTorn, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          d = kFedFailed;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_dec = d & 7u;
      s_slot = a.scratch[kFedSlot];
      s_vp = a.scratch[kFedPulled];
    }
  }
  __syncthreads();
  if (s_dec == kFedAdmit && !a.drop_land) {  // this workgroup's slice of the gradient into slot t
    long long lo, hi;
    fed_slice(a, blockIdx.x, G, lo, hi);
    const long long soff = (long long)s_slot << a.shard_shift;
    for (long long i = lo + 4LL * threadIdx.x; i < hi; i += 4LL * kFedBlock)
      fed_st4(fed_elem(slots, a.shard_shift, i, soff), *reinterpret_cast<const f32x4*>(a.g + i));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's slot stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.scratch + kFedUpDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned)G - 1) {  // the last workgroup: every workgroup's slice store has landed
      a.scratch[kFedUpDone] = 0;
      a.scratch[kFedEpoch] += 1u;
      // the launch's true decision (workgroup 0 published it before arriving; this workgroup may itself be
      // one whose wait timed out) and whether any workgroup stored nothing
      const unsigned dec = a.scratch[kFedDecision] & 7u;
      const unsigned torn = a.scratch[kFedTorn];
      a.scratch[kFedTorn] = 0;
      if (dec == kFedAdmit && !a.drop_land) {
        const unsigned vp = a.scratch[kFedPulled], bit = 1u << a.scratch[kFedSlot];
        if (torn) {  // a partly stored gradient: landed as a bad slot (the version still closes without it)
          fed_or_tagged(a.bad, vp, bit);
          fed_fail(a, kFedErrTorn);
        }
        const unsigned long long nw = fed_or_tagged(a.land, vp, bit);
        // the lander that completes the mask applies (against a recovering rank: the seqlock CAS decides)
        if ((unsigned)nw == fed_full_mask(a.K)) a.scratch[kFedApplier] = vp + 1u;
      }
    }
  }
}

__global__ __launch_bounds__(kFedBlock) void fed_apply_kernel(FedArgs a) {
  __shared__ float* master[kP2PMaxRanks];
  __shared__ float* slots[kP2PMaxRanks];
  __shared__ unsigned s_app;
  fed_stage(a, master, slots);
  if (threadIdx.x == 0) s_app = a.scratch[kFedApplier];
  __syncthreads();
  if (s_app == 0) return;  // not this rank's version to apply (every workgroup returns)
  const unsigned vp = s_app - 1u;
  // workgroup 0 takes the version (v -> v + 1, odd: pullers retry, uploads drop) -- or loses it to another
  // applier -- and the others take its decision (all <= kPSMaxGrid workgroups are resident)
  __shared__ unsigned s_go, s_ep;
  if (threadIdx.x == 0) {
    const unsigned ep = (a.scratch[kFedApEp] + 1u) & 0x7fffffffu;
    s_ep = ep;
    if (blockIdx.x == 0) {
      unsigned e = vp;
      const bool won = __hip_atomic_compare_exchange_strong(a.seq, &e, vp + 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.scratch + kFedApDec, (ep << 1) | (won ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_go = won;
    } else {
      const unsigned long long t0 = wall_clock64();
      unsigned d = 0;
      for (;;) {
        d = __hip_atomic_load(a.scratch + kFedApDec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((d >> 1) == ep) break;
        if (wall_clock64() - t0 > 2ull * (unsigned long long)a.timeout_ticks) {  // (workgroup 0 never decided)
          fed_fail(a, 4u);
          d = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_go = d & 1u;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const bool go = s_go != 0;
  long long lo, hi;
  fed_slice(a, blockIdx.x, gridDim.x, lo, hi);
  const float lr = a.lr_dev ? *a.lr_dev : a.lr;
  // the version's bad slots (torn or never landed) are left out of the mean; none good: no update
  __shared__ unsigned s_good;
  if (threadIdx.x == 0) {
    const unsigned long long bw = __hip_atomic_load(a.bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s_good = fed_full_mask(a.K) & ~((unsigned)(bw >> 32) == vp ? (unsigned)bw : 0u);
  }
  __syncthreads();
  const unsigned good = s_good;
  const int ngood = __builtin_popcount(good);
  const float invk = 1.f / (float)(ngood > 0 ? ngood : 1);
  for (long long i = lo + 4LL * threadIdx.x; go && i < hi && ngood > 0; i += 4LL * kFedBlock) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    bool first = true;
    for (int t = 0; t < a.K; ++t) {
      if (!((good >> t) & 1u)) continue;
      const f32x4 v = fed_ld4(fed_elem(slots, a.shard_shift, i, (long long)t << a.shard_shift));
      s = first ? v : s + v;
      first = false;
    }
    float* m = fed_elem(master, a.shard_shift, i, 0);
    f32x4 w = fed_ld4(m);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma clang fp contract(off)
      w[j] = w[j] - lr * (s[j] * invk);
    }
    fed_st4(m, w);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's master stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.scratch + kFedApDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {  // every element applied: publish version v + 1
      a.scratch[kFedApDone] = 0;
      a.scratch[kFedApplier] = 0;
      a.scratch[kFedApEp] = s_ep;
      if (go) {
        __hip_atomic_store(a.seq, vp + 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        a.stats[4] += 1;
        if (a.scratch[kFedRecov]) a.stats[5] += 1;  // a stuck version recovered by this rank
      }
    }
  }
}

int fed_grid(long long n) {
  long long g = (n + 4095) / 4096;
  return (int)(g < 1 ? 1 : (g > kPSMaxGrid ? kPSMaxGrid : g));
}

bool fed_ok(const FedArgs& a) {
  if (a.nshards < 1 || a.nshards > kP2PMaxRanks || a.shard_shift < 6 || a.shard_shift > 30 || !a.seq || !a.tick ||
      !a.land || !a.bad || a.K < 1 || a.K > kFedMaxK || a.n <= 0 || (a.n & 3) || ((a.n - 1) >> a.shard_shift) >= a.nshards)
    return false;
  for (int k = 0; k < a.nshards; ++k)
    if (!a.shard[k] || !a.slot[k]) return false;
  return true;
}

}  // namespace

hipError_t fed_pull(const FedArgs& a, hipStream_t st) {
  if (!fed_ok(a) || !a.w) return hipErrorInvalidValue;
  fed_pull_kernel<<<fed_grid(a.n), kFedBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t fed_upload(const FedArgs& a, hipStream_t st) {
  if (!fed_ok(a) || !a.g) return hipErrorInvalidValue;
  fed_upload_kernel<<<fed_grid(a.n), kFedBlock, 0, st>>>(a, fed_grid(a.n));
  return hipGetLastError();
}

hipError_t fed_apply(const FedArgs& a, hipStream_t st) {
  if (!fed_ok(a)) return hipErrorInvalidValue;
  fed_apply_kernel<<<fed_grid(a.n), kFedBlock, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace dfa
