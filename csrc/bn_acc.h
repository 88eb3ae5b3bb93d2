// BatchNorm statistics accumulated by the PRODUCING kernel's epilogue (kernels.h BnAcc).
//
// Round 3/4 finalised the statistics inside the producing launch with two levels of last-arriver
// hand-offs (bn_epi.h) or in separate statistics launches (bn.hip): each workgroup waited for its
// write-through partials and a ticket, or the statistics pass re-read the whole tensor (ResNet-18 B=256:
// 40 launches, 592 us of a 2.86 ms step, profiles/r4/resnet18_b256_step_breakdown_r4_final.txt).  Here a
// workgroup reduces the values it STORED (bf16-rounded, masked) in registers, across the 16 lanes that
// share a channel (xor shuffles) and across its waves (LDS slots, fixed order), then adds one fp64 partial
// per channel and quantity into a replica of the accumulator with no-return atomics: no wait, no ticket,
// no re-read.  The replicas (blockIdx % nrep) spread the adds of many workgroups over several addresses
// (MI355X_MICROARCH.md 'Global float atomics': one address takes ~25 ns per add).  The consumer finalises.
#pragma once
#include "common.h"
#include "kernels.h"

namespace dfa {

typedef __bf16 bacc_bf16x4 __attribute__((ext_vector_type(4)));

// running sums of one lane for 4 consecutive channels: S, Q (and Q2 for the second BatchNorm)
struct BnAccLane {
  float s[4], q[4], q2[4];
};
// per-channel statistics of the lane's 4 channels (mode 1)
struct BnAccChan {
  float mu[4], is[4], mu2[4], is2[4];
};

__device__ __forceinline__ void bacc_zero(BnAccLane& l) {
#pragma unroll
  for (int r = 0; r < 4; ++r) l.s[r] = l.q[r] = l.q2[r] = 0.f;
}

__device__ __forceinline__ BnAccChan bacc_chan(const BnAcc& e, int col) {
  BnAccChan c;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    c.mu[r] = c.mu2[r] = 0.f;
    c.is[r] = c.is2[r] = 1.f;
  }
  if (e.mode == 1) {
    const float* m2 = e.acc2 ? e.mean2 : e.mean;
    const float* i2 = e.acc2 ? e.invstd2 : e.invstd;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      c.mu[r] = e.mean[col + r];
      c.is[r] = e.invstd[col + r];
      c.mu2[r] = m2[col + r];
      c.is2[r] = i2[col + r];
    }
  }
  return c;
}

// the BatchNorm inputs x (and x2) at element offset o (mode 1).  Epilogues load these for ALL their
// elements before their first store: a load issued behind a store waits for that store too (one vmcnt
// counter), so a load / compute / store sequence per element serialised a round trip per element (the
// ResNet-18 data-gradient convs ran at half their speed).
struct BnAccX {
  bacc_bf16x4 x, x2;
};
__device__ __forceinline__ BnAccX bacc_loadx(const BnAcc& e, long long o) {
  BnAccX r;
  if (e.mode == 1) {
    r.x = *reinterpret_cast<const bacc_bf16x4*>(e.x + o);
    // (one BatchNorm: the second factor is the first; no second read of the same tensor)
    r.x2 = e.acc2 ? *reinterpret_cast<const bacc_bf16x4*>(e.x2 + o) : r.x;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) r.x[k] = r.x2[k] = (__bf16)0.f;
  }
  return r;
}

// v: the 4 values as STORED (bf16-rounded, masked) at element offset o of [M][ldc] (o % 4 == 0), xs their
// bacc_loadx.  The sums are updated unconditionally (only the factor depends on the mode): a mode-dependent
// update made hipcc keep the accumulators in scratch with a dynamic index.
__device__ __forceinline__ void bacc_add4x(BnAccLane& l, const BnAcc& e, const BnAccChan& c, const BnAccX& xs,
                                           const float (&v)[4]) {
  float f[4], f2[4];
  if (e.mode == 1) {  // Q: g * xhat (of the first / the second BatchNorm's input)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      f[r] = ((float)xs.x[r] - c.mu[r]) * c.is[r];
      f2[r] = ((float)xs.x2[r] - c.mu2[r]) * c.is2[r];
    }
  } else {  // Q: y * y
#pragma unroll
    for (int r = 0; r < 4; ++r) f[r] = f2[r] = v[r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    l.s[r] += v[r];
    l.q[r] += v[r] * f[r];
    l.q2[r] += v[r] * f2[r];
  }
}
__device__ __forceinline__ void bacc_add4(BnAccLane& l, const BnAcc& e, const BnAccChan& c, long long o,
                                          const float (&v)[4]) {
  bacc_add4x(l, e, c, bacc_loadx(e, o), v);
}

// sum over the lanes l ^ m, m in {1, 2, 4, 8} (the 16 lanes of an MFMA 16x16 C/D row group that hold
// the same 4 channels for 16 different pixels); fixed order: deterministic
__device__ __forceinline__ float bacc_x16(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}
__device__ __forceinline__ void bacc_reduce16(BnAccLane& l, bool two) {
  (void)two;  // (Q2 reduced unconditionally: see bacc_add4)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    l.s[r] = bacc_x16(l.s[r]);
    l.q[r] = bacc_x16(l.q[r]);
    l.q2[r] = bacc_x16(l.q2[r]);
  }
}

// LDS slot layout: red[(slot * W + ch) * 3 + k], k = S, Q, Q2; W channels per slot
__device__ __forceinline__ void bacc_stash(float* red, int slot, int W, int ch, const BnAccLane& l) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float* p = red + ((long long)slot * W + ch + r) * 3;
    p[0] = l.s[r];
    p[1] = l.q[r];
    p[2] = l.q2[r];
  }
}

// Threads tid < W (of nthreads): sum the nslot slots of channel n0 + tid in slot order and add the fp64
// partials into this workgroup's replica.  Caller: a barrier between the last bacc_stash and this.
__device__ __forceinline__ void bacc_flush(const BnAcc& e, const float* red, int nslot, int W, int n0, int N,
                                           int tid, int nthreads) {
  const int rep = (int)(blockIdx.x % (unsigned)e.nrep);
  for (int c = tid; c < W; c += nthreads) {
    if (n0 + c >= N) continue;
    float s = 0.f, q = 0.f, q2 = 0.f;
    for (int k = 0; k < nslot; ++k) {
      const float* p = red + ((long long)k * W + c) * 3;
      s += p[0];
      q += p[1];
      q2 += p[2];
    }
    double* a = e.acc + (long long)rep * 2 * N + n0 + c;
    unsafeAtomicAdd(a, (double)s);
    unsafeAtomicAdd(a + N, (double)q);
    if (e.acc2) {
      double* a2 = e.acc2 + (long long)rep * 2 * N + n0 + c;
      unsafeAtomicAdd(a2, (double)s);
      unsafeAtomicAdd(a2 + N, (double)q2);
    }
  }
}

}  // namespace dfa
