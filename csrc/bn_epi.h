// In-launch BatchNorm statistics of a conv's stored output (kernels.h BnEpi), shared by the igemm64
// epilogue; and the fence-free last-arriver hand-off it (and csrc/bn.hip) uses.
//
// Hand-off (cdna_hip_programming.md Guideline 16, sc1 form): every slab word is stored write-through
// (relaxed agent-scope atomic store = sc1) and drained by every storing wave before the barrier; lane 0
// then draws a ticket.  The last of `n` arrivers reads the slabs with sc1 loads, so neither side pays an
// agent-scope release (L2 write-back) or acquire.  The last arriver re-arms the counter for the next
// launch.  Every sum runs in a fixed order (tile order, then group order): deterministic.
// Memory-model note: the ordering this relies on -- write-through (sc1) stores drained by
// s_waitcnt vmcnt(0) in every storing wave before a relaxed agent-scope ticket RMW, then sc1 loads in
// the last arriver -- is the gfx950 hand-off form of cdna_hip_programming.md Guideline 16 (R1, counter
// variant) and MI355X_MICROARCH.md's visibility rules, not a C++-memory-model happens-before: the
// vmcnt drain is what makes the stores globally performed before the ticket.  This header is gfx950
// only (the build targets nothing else); a port would put release / acquire on the ticket instead.
#pragma once
#include "common.h"
#include "kernels.h"

namespace dfa {

__device__ __forceinline__ void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool last_arriver(unsigned* counter, unsigned n, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned tk = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = (tk == n - 1) ? 1 : 0;
    if (*flag) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
  return *flag != 0;
}

constexpr int kBnEpiGroup = 16;

// Called by every thread of a row-tile workgroup (NT threads) after it stored the partial row
// part[tile_m][2][n0 .. n0 + ncols) write-through: the last of every 16 row tiles sums its group's
// partials into part[ntm + grp]; the last group reducer of this column range sums the groups in fp64 and
// finalises columns [n0, n0 + ncols).  `tile_n` picks this column range's tickets.
template <int NT>
__device__ __forceinline__ void bn_epi_finalize(const BnEpi& e, int N, long long M, int tile_m, int tile_n, int n0,
                                                int ncols, int* flag) {
  const int grp = tile_m / kBnEpiGroup, gbeg = grp * kBnEpiGroup, gn = min(kBnEpiGroup, e.ntm - gbeg);
  unsigned* tk = e.ticket + (long long)tile_n * (1 + e.ngrp);
  if (!last_arriver(tk + 1 + grp, (unsigned)gn, flag)) return;
  float* gpart = e.part + (long long)e.ntm * 2 * N;  // [ngrp][2][N]
  for (int t = threadIdx.x; t < 2 * ncols; t += NT) {
    const int which = t / ncols, col = n0 + t - which * ncols;
    float v[kBnEpiGroup];
#pragma unroll
    for (int j = 0; j < kBnEpiGroup; ++j) v[j] = ld_sc1(e.part + ((long long)(gbeg + min(j, gn - 1)) * 2 + which) * N + col);
    float u = 0.f;
#pragma unroll
    for (int j = 0; j < kBnEpiGroup; ++j) u += j < gn ? v[j] : 0.f;
    st_sc1(gpart + ((long long)grp * 2 + which) * N + col, u);
  }
  if (!last_arriver(tk, (unsigned)e.ngrp, flag)) return;
  for (int c = threadIdx.x; c < ncols; c += NT) {
    const int col = n0 + c;
    double S = 0.0, Q = 0.0;
    for (int g0 = 0; g0 < e.ngrp; g0 += kBnEpiGroup) {
      float su[kBnEpiGroup], qu[kBnEpiGroup];
#pragma unroll
      for (int j = 0; j < kBnEpiGroup; ++j) {
        const long long base = (long long)min(g0 + j, e.ngrp - 1) * 2 * N + col;
        su[j] = ld_sc1(gpart + base);
        qu[j] = ld_sc1(gpart + base + N);
      }
#pragma unroll
      for (int j = 0; j < kBnEpiGroup; ++j)
        if (g0 + j < e.ngrp) {
          S += (double)su[j];
          Q += (double)qu[j];
        }
    }
    if (e.mode == 0) {
      const double m = S / M;
      double var = Q / M - m * m;
      if (var < 0.0) var = 0.0;
      e.mean_out[col] = (float)m;
      e.invstd_out[col] = (float)(1.0 / sqrt(var + (double)e.eps));
      if (e.run_mean) {
        const double unb = M > 1 ? var * M / (M - 1) : var;
        e.run_mean[col] = (float)((1.0 - e.momentum) * e.run_mean[col] + e.momentum * m);
        e.run_var[col] = (float)((1.0 - e.momentum) * e.run_var[col] + e.momentum * unb);
      }
    } else {
      e.dbeta[col] = (float)S * e.gscale;
      e.dgamma[col] = (float)Q * e.gscale;
      const double isd = e.invstd[col], gam = e.gamma[col], m = e.mean[col];
      const double k1 = gam * isd;
      e.coef[col] = (float)k1;
      e.coef[N + col] = (float)(-k1 * isd * Q / M);
      e.coef[2 * N + col] = (float)(k1 * (m * isd * Q / M - S / M));
    }
  }
}

}  // namespace dfa
