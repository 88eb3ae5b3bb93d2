// In-kernel low-latency all-reduce of one "slot" of values (kernels.h LLComm).
//
// Used where a reduction epilogue already holds the final local value of each element it owns (the fused
// LeNet-5 reduce kernel: one dense weight-gradient tile or 64 conv parameters per workgroup): instead of
// storing the local gradient and running a separate all-reduce launch over xGMI, the workgroup PUSHES
// each value as an 8-byte {fp32 value, u32 epoch} granule into slot `slot` of every peer's IPC-mapped
// region and polls its own region until the W - 1 peer granules of that position carry the epoch.  The
// value and its tag travel in one naturally aligned 8-byte store, so no fence or separate flag is
// needed and one one-way xGMI trip (pipelined over all 7 links) is the whole synchronisation; the
// reads after it are local HBM.  Sums are taken in rank order, so every rank gets bit-identical results.
//
// Reuse of a slot: granules of epoch e go to parity e & 1.  A sender can only reach epoch e + 2 of a
// slot after it received every peer's e + 1 granules of that slot, which a peer sends only in a later
// launch than the one in which it consumed parity e & 1: no granule is overwritten before it is read.
// Epochs advance per call on the device, so hipGraph replays and multi-step graphs keep them in step.
// A peer missing for timeout_ticks (wall_clock64, 100 MHz) sets the sticky error word and the host
// mirror, and the call reports failure instead of spinning forever.
#pragma once
#include "common.h"
#include "kernels.h"

namespace dfa {

// Block-wide epoch of `slot` for this call; every thread of the workgroup must call it.
__device__ __forceinline__ unsigned ll_epoch(const LLComm& c, int slot, unsigned* s_e) {
  if (threadIdx.x == 0) *s_e = c.epochs[slot] + 1u;
  __syncthreads();
  return *s_e;
}

__device__ __forceinline__ void ll_commit(const LLComm& c, int slot, unsigned e) {
  if (threadIdx.x == 0) c.epochs[slot] = e;
}

__device__ __forceinline__ long long ll_off(const LLComm& c, int slot, int pos, unsigned e) {
  return ((long long)(e & 1u) * c.nslots + slot) * (kP2PMaxRanks * kLLSlot) + pos;
}

// Push value `v` of position `pos` (< kLLSlot) of `slot`, epoch e, into every peer's region.  Called by
// every lane that owns a position (the same lanes on every rank); never waits.
__device__ __forceinline__ void ll_push(const LLComm& c, int slot, int pos, unsigned e, float v) {
  // 32-bit byte offset (the region is < 4 GB): one SGPR base per peer + one VGPR offset, so the W - 1
  // stores need no per-peer 64-bit address registers
  const unsigned boff = (unsigned)(ll_off(c, slot, pos, e) + (long long)c.rank * kLLSlot) * 8u;
  const unsigned long long g = (unsigned long long)__float_as_uint(v) | ((unsigned long long)e << 32);
#pragma unroll
  for (int r = 0; r < kP2PMaxRanks; ++r)
    if (r < c.world && r != c.rank)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(c.bases[r]) + boff), g,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait for the W - 1 peer granules of (slot, pos, e) and return the rank-order sum with this rank's own
// value `v`.  Returns false on a peer timeout (error word + host mirror set).
__device__ __forceinline__ bool ll_wait_sum(const LLComm& c, int slot, int pos, unsigned e, float v, float& out) {
  unsigned pending = 0;
#pragma unroll
  for (int r = 0; r < kP2PMaxRanks; ++r)
    if (r < c.world && r != c.rank) pending |= 1u << r;
  float vals[kP2PMaxRanks];
#pragma unroll
  for (int r = 0; r < kP2PMaxRanks; ++r) vals[r] = v;
  const unsigned long long* mine = c.bases[c.rank] + ll_off(c, slot, pos, e);
  const unsigned long long t0 = wall_clock64();
  bool ok = true;
  while (pending) {
    unsigned long long x[kP2PMaxRanks];
#pragma unroll
    for (int r = 0; r < kP2PMaxRanks; ++r)
      if ((pending >> r) & 1u)
        x[r] = __hip_atomic_load(const_cast<unsigned long long*>(mine + (long long)r * kLLSlot), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
    for (int r = 0; r < kP2PMaxRanks; ++r)
      if (((pending >> r) & 1u) && (unsigned)(x[r] >> 32) == e) {
        vals[r] = __uint_as_float((unsigned)x[r]);
        pending &= ~(1u << r);
      }
    if (!pending) break;
    if (wall_clock64() - t0 > (unsigned long long)c.timeout_ticks) {
      atomicOr(c.err, 1);
      if (c.herr) __hip_atomic_store(c.herr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  float acc = vals[0];
#pragma unroll
  for (int r = 1; r < kP2PMaxRanks; ++r)
    if (r < c.world) acc += vals[r];
  out = acc;
  return ok;
}

// Push + wait in one call (a slot whose owner has nothing else to overlap with the round trip).
__device__ __forceinline__ bool ll_allreduce(const LLComm& c, int slot, int pos, unsigned e, float v, float& out) {
  ll_push(c, slot, pos, e, v);
  return ll_wait_sum(c, slot, pos, e, v, out);
}

}  // namespace dfa
