// BatchNorm (NHWC, per-channel over M = B*H*W rows) for the CIFAR-10 ResNet-18 config
// (BASELINE.json configs[3]; not present in the reference).
//
// Two launches per direction:
//   stats  : every workgroup reduces a row range into an fp32 partial slab [2][C]; the slabs are
//            then combined inside the same launch by last-arriver hand-offs (write-through sc1 slab
//            stores, ticket counter, sc1 loads: no fences): the last of every 16 workgroups sums its
//            group's slabs, and the last group reducer sums the (<= 16) group slabs in fp64 and
//            finalises — forward: mean, invstd and the running statistics; backward: dgamma/dbeta
//            straight into the flat gradient buffer plus the per-channel coefficients of
//            dx = k1*g + k2*x + k3.  Every sum runs in a fixed order: deterministic, no atomics on
//            data.  Two levels keep each reducer at one round trip of independent loads.
//   apply  : a streaming pass with 16-byte loads whose channel chunk is constant per thread (the
//            grid stride is a multiple of C/8), so the per-channel affine coefficients live in
//            registers.  The forward apply optionally fuses the residual join of a ResNet block,
//            y = relu(bn(x) + r) or relu(bn(x) + bn_r(r)) (projection shortcut), and the backward
//            apply fuses relu' of a mask tensor into g = dy * (mask > 0).
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "diag.h"
#include "bn_epi.h"
#include "bn_acc.h"

namespace dfa {

constexpr int BN_MAX_G = 255;  // more workgroups cost more than they add: every one pays a release fence (L2 writeback)
constexpr int BN_GROUP = 16;

static bool bn_vec(int C) { return C % 8 == 0 && C / 8 <= 256 && 256 % (C / 8) == 0; }

static int bn_rows_per_pass(int C, bool vec) { return 256 / (vec ? C / 8 : C); }

// rows per thread of the statistics pass (default 16; diagnostic bn_rpt, csrc/diag.h)
static int bn_rows_per_thread() {
  static const int r = [] {
    const int v = diag_int("bn_rpt", 16);
    return v >= 1 && v <= 64 ? v : 16;
  }();
  return r;
}

// workgroup cap of a statistics launch (default BN_MAX_G; diagnostic bn_max_g <= 1008: 1 + 63 tickets)
static int bn_max_g() {
  static const int g = [] {
    const int v = diag_int("bn_max_g", BN_MAX_G);
    return v >= 16 && v <= 1008 ? v : BN_MAX_G;
  }();
  return g;
}

static int bn_grid(int M, int rpp) {
  int g = cdiv(M, rpp * bn_rows_per_thread());
  if (g > bn_max_g()) g = bn_max_g();
  if (g < 1) g = 1;
  return g;
}

// Hand-off without fences: st_sc1 / ld_sc1 / last_arriver (csrc/bn_epi.h).
__device__ __forceinline__ bool bn_last_arriver(unsigned* counter, unsigned n, int* flag) {
  return last_arriver(counter, n, flag);
}

// MODE 0: s += x, q += x*x.   MODE 1: g = dy * relu'(mask), xh = (x - mean) * invstd; s += g, q += g*xh.
// The statistics body; returns true in the one workgroup that finalised (the last arriver of the last
// group).  FUSED: every workgroup reaches the end (no early return), so that it can wait for the
// finalisation and run the apply pass of the same launch.
template <int MODE, bool VEC, bool FUSED>
__device__ __forceinline__ bool bn_stats_body(const BnStatsArgs& a, float* lsq) {
  __shared__ int last;
  float* ls = lsq;
  float* lq = lsq + 2048;
  constexpr int W = VEC ? 8 : 1;
  const int C = a.C, M = a.M;
  const int cpr = C / W;
  const int rpp = 256 / cpr;
  const int t = threadIdx.x;
  const int chunk = t % cpr, rsub = t / cpr;
  float s[W], q[W], mu[W], is[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    s[j] = 0.f;
    q[j] = 0.f;
    mu[j] = 0.f;
    is[j] = 1.f;
    if (MODE == 1 && rsub < rpp) {
      mu[j] = a.mean[chunk * W + j];
      is[j] = a.invstd[chunk * W + j];
    }
  }
  if (rsub < rpp) {
    // U rows per thread per round, every load of the round issued before the first use: a streaming
    // reduction needs ~16-32 KB in flight per CU to cover HBM latency
    constexpr int U = MODE == 0 ? 8 : 4;
    const long long step = (long long)gridDim.x * rpp;
    long long r = (long long)blockIdx.x * rpp + rsub;
    for (; r < M; r += U * step) {
      float xv[U][W], gv[U][W];
      if (VEC) {
        bf16x8 vx[U], vg[U], vm[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long rr = r + u * step;
          const long long o = (rr < M ? rr : r) * C + chunk * W;  // clamped, masked below
          vx[u] = *reinterpret_cast<const bf16x8*>(a.x + o);
          if (MODE == 1) {
            vg[u] = *reinterpret_cast<const bf16x8*>(a.dy + o);
            if (a.mask) vm[u] = *reinterpret_cast<const bf16x8*>(a.mask + o);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool ok = r + u * step < M;
#pragma unroll
          for (int j = 0; j < W; ++j) {
            xv[u][j] = ok ? (float)vx[u][j] : 0.f;
            if (MODE == 1) gv[u][j] = (ok && (!a.mask || (float)vm[u][j] > 0.f)) ? (float)vg[u][j] : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long rr = r + u * step;
          const bool ok = rr < M;
          const long long o = (ok ? rr : r) * C + chunk;
          xv[u][0] = ok ? (float)a.x[o] : 0.f;
          if (MODE == 1) gv[u][0] = (!ok || (a.mask && !((float)a.mask[o] > 0.f))) ? 0.f : (float)a.dy[o];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int j = 0; j < W; ++j) {
          if (MODE == 0) {
            s[j] += xv[u][j];
            q[j] += xv[u][j] * xv[u][j];
          } else {
            // rows past M contribute g = 0 (and their xh is multiplied by 0)
            const float xh = (xv[u][j] - mu[j]) * is[j];
            s[j] += gv[u][j];
            q[j] += gv[u][j] * xh;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
      ls[rsub * C + chunk * W + j] = s[j];
      lq[rsub * C + chunk * W + j] = q[j];
    }
  }
  __syncthreads();
  const int G = gridDim.x;
  const int ncol = 2 * C;
  float* slab = a.ws + (long long)blockIdx.x * ncol;
  for (int c = t; c < C; c += 256) {
    float u = 0.f, v = 0.f;
    for (int r = 0; r < rpp; ++r) {
      u += ls[r * C + c];
      v += lq[r * C + c];
    }
    st_sc1(slab + c, u);
    st_sc1(slab + C + c, v);
  }

  // ---- level 1: the last of each group of 16 workgroups sums the group's slabs
  const int grp = blockIdx.x / BN_GROUP;
  const int gbeg = grp * BN_GROUP, gn = min(BN_GROUP, G - gbeg);
  const int ngrp = cdiv(G, BN_GROUP);
  float* gslab = a.ws + (long long)G * ncol;  // [ngrp][2C]
  if (!bn_last_arriver(a.counter + 1 + grp, (unsigned)gn, &last)) return false;
  for (int col = t; col < ncol; col += 256) {
    float v[BN_GROUP];
#pragma unroll
    for (int j = 0; j < BN_GROUP; ++j) v[j] = ld_sc1(a.ws + (long long)(gbeg + min(j, gn - 1)) * ncol + col);
    float u = 0.f;
#pragma unroll
    for (int j = 0; j < BN_GROUP; ++j) u += j < gn ? v[j] : 0.f;
    st_sc1(gslab + (long long)grp * ncol + col, u);
  }

  // ---- level 2: the last group reducer sums the group slabs in fp64 and finalises
  if (!bn_last_arriver(a.counter, (unsigned)ngrp, &last)) return false;
  for (int c = t; c < C; c += 256) {
    double sv = 0.0, qv = 0.0;
    for (int g0 = 0; g0 < ngrp; g0 += BN_GROUP) {
      float su[BN_GROUP], qu[BN_GROUP];
#pragma unroll
      for (int j = 0; j < BN_GROUP; ++j) {
        const long long base = (long long)min(g0 + j, ngrp - 1) * ncol;
        su[j] = ld_sc1(gslab + base + c);
        qu[j] = ld_sc1(gslab + base + C + c);
      }
#pragma unroll
      for (int j = 0; j < BN_GROUP; ++j) {
        if (g0 + j < ngrp) {
          sv += (double)su[j];
          qv += (double)qu[j];
        }
      }
    }
    if (MODE == 0) {
      const double m = sv / M;
      double var = qv / M - m * m;
      if (var < 0.0) var = 0.0;
      st_sc1(a.mean_out + c, (float)m);  // write-through: a fused apply pass reads them in this launch
      st_sc1(a.invstd_out + c, (float)(1.0 / sqrt(var + (double)a.eps)));
      if (a.run_mean) {
        const double unb = M > 1 ? var * M / (M - 1) : var;
        a.run_mean[c] = (float)((1.0 - a.momentum) * a.run_mean[c] + a.momentum * m);
        a.run_var[c] = (float)((1.0 - a.momentum) * a.run_var[c] + a.momentum * unb);
      }
    } else {
      a.dbeta[c] = (float)sv * a.gscale;
      a.dgamma[c] = (float)qv * a.gscale;
      const double isd = a.invstd[c], gam = a.gamma[c], m = a.mean[c];
      const double k1 = gam * isd;
      st_sc1(a.coef + c, (float)k1);
      st_sc1(a.coef + C + c, (float)(-k1 * isd * qv / M));
      st_sc1(a.coef + 2 * C + c, (float)(k1 * (m * isd * qv / M - sv / M)));
    }
  }
  return true;
}

template <int MODE, bool VEC>
__global__ void __launch_bounds__(256) bn_stats_kernel(BnStatsArgs a) {
  __shared__ __attribute__((aligned(16))) float lsq[4096];
  bn_stats_body<MODE, VEC, false>(a, lsq);
}

// Statistics and the streaming pass in ONE launch (C % 8 == 0): every workgroup computes its partials,
// the last arriver finalises as above and bumps the generation word; the others wait for it (all
// workgroups of the launch are resident: G <= 1008 workgroups of 256 threads) and then stream over the
// same rows they reduced (mostly still in their XCD's L2).  Forward: y = act(bn(x) [+ r | + bn_r(r)]);
// backward: dx = k1 * g + k2 * x + k3.  The finalised per-channel values are read write-through.
// gen: a word that only ever increments (no reset between launches or graph replays).
template <int MODE, int RES>
__global__ void __launch_bounds__(256, 4) bn_fused_kernel(BnStatsArgs a, BnApplyArgs p, bf16* __restrict__ dx,
                                                       unsigned* gen) {
  __shared__ __attribute__((aligned(16))) float lsq[4096];
  __shared__ unsigned g0;
  if (threadIdx.x == 0) g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();  // the generation is read before this workgroup's arrival can complete the count
  const bool fin = bn_stats_body<MODE, true, true>(a, lsq);
  if (fin) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the finalised values are written through
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (threadIdx.x == 0) {
      // bounded: a launch that could not make every workgroup resident ends (wrong, not hung)
      for (unsigned it = 0; it < (1u << 24); ++it) {
        if (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != g0) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
  }
  const int C = a.C, M = a.M;
  const int cpr = C / 8, rpp = 256 / cpr;
  const int t = threadIdx.x, chunk = t % cpr, rsub = t / cpr;
  if (rsub >= rpp) return;
  const int c0 = chunk * 8;
  float k1[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (MODE == 0) {
      const float m = ld_sc1(a.mean_out + c0 + j), is = ld_sc1(a.invstd_out + c0 + j);
      k1[j] = p.gamma[c0 + j] * is;
      k2[j] = p.beta[c0 + j] - m * k1[j];
      k3[j] = 0.f;
      if (RES == 2) {
        const float ra = p.rgamma[c0 + j] * p.rinvstd[c0 + j];
        k3[j] = ra;
      }
    } else {
      k1[j] = ld_sc1(a.coef + c0 + j);
      k2[j] = ld_sc1(a.coef + C + c0 + j);
      k3[j] = ld_sc1(a.coef + 2 * C + c0 + j);
    }
  }
  float rb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) rb[j] = RES == 2 ? p.rbeta[c0 + j] - p.rmean[c0 + j] * k3[j] : 0.f;
  // the rows this thread reduced, U at a time: every load of a round in flight before the first store
  constexpr int U = MODE == 0 ? 8 : 4;  // backward: three tensors per row (x, dy, mask) within 128 VGPRs
  const long long step = (long long)gridDim.x * rpp;
  for (long long r = (long long)blockIdx.x * rpp + rsub; r < M; r += U * step) {
    bf16x8 xv[U], v1[U], v2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long rr = r + u * step;
      const long long o = (rr < M ? rr : r) * C + c0;
      xv[u] = *reinterpret_cast<const bf16x8*>(a.x + o);
      if (MODE == 0 && RES) v1[u] = *reinterpret_cast<const bf16x8*>(p.r + o);
      if (MODE == 1) {
        v1[u] = *reinterpret_cast<const bf16x8*>(a.dy + o);
        if (a.mask) v2[u] = *reinterpret_cast<const bf16x8*>(a.mask + o);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long rr = r + u * step;
      if (rr >= M) break;
      const long long o = rr * C + c0;
      bf16x8 out;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MODE == 0) {
          float v = (float)xv[u][j] * k1[j] + k2[j];
          if (RES == 1) v += (float)v1[u][j];
          if (RES == 2) v += (float)v1[u][j] * k3[j] + rb[j];
          if (p.relu) v = fmaxf(v, 0.f);
          out[j] = f2bf(v);
        } else {
          const float g = (a.mask && !((float)v2[u][j] > 0.f)) ? 0.f : (float)v1[u][j];
          out[j] = f2bf(k1[j] * g + k2[j] * (float)xv[u][j] + k3[j]);
        }
      }
      *reinterpret_cast<bf16x8*>((MODE == 0 ? p.y : dx) + o) = out;
    }
  }
}

// BatchNorm forward statistics from the partial sums the producing conv's epilogue emitted
// ([ntm][2][C] row-tile partials, e.g. a BnEpi buffer): per channel a fixed-order fp64 sum over the row tiles (16 waves
// of a workgroup take every 16th tile, 8 loads in flight each, combined in wave order), then the same
// finalisation as bn_stats_kernel<0>.  Replaces a full read of the conv output.
__global__ void __launch_bounds__(1024) bn_finalize_partials_kernel(const float* __restrict__ part, int ntm, int C,
                                                                    long long M, float* mean, float* invstd,
                                                                    float* run_mean, float* run_var, float momentum,
                                                                    float eps) {
  __shared__ double ps[16][64], pq[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double s = 0.0, q = 0.0;
  if (c < C) {
    for (int t0 = w; t0 < ntm; t0 += 16 * 8) {
      float u[8], v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int t = min(t0 + 16 * k, ntm - 1);
        u[k] = part[((long long)t * 2) * C + c];
        v[k] = part[((long long)t * 2 + 1) * C + c];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (t0 + 16 * k < ntm) {
          s += (double)u[k];
          q += (double)v[k];
        }
    }
  }
  ps[w][lane] = s;
  pq[w][lane] = q;
  __syncthreads();
  if (w == 0 && c < C) {
    double S = 0.0, Q = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      S += ps[k][lane];
      Q += pq[k][lane];
    }
    const double m = S / M;
    double var = Q / M - m * m;
    if (var < 0.0) var = 0.0;
    mean[c] = (float)m;
    invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
      const double unb = M > 1 ? var * M / (M - 1) : var;
      run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * m);
      run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
    }
  }
}

hipError_t bn_finalize_partials(const float* part, int ntm, int C, long long M, float* mean, float* invstd,
                                float* run_mean, float* run_var, float momentum, float eps, hipStream_t st) {
  if (ntm <= 0 || C <= 0 || M <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_finalize_partials_kernel, dim3(cdiv(C, 64)), dim3(1024), 0, st, part, ntm, C, M, mean, invstd,
                     run_mean, run_var, momentum, eps);
  return hipGetLastError();
}

__device__ __forceinline__ void bn_affine(const BnApplyArgs& a, const float* g, const float* b, const float* m,
                                          const float* v, int c, float& sa, float& sb) {
  const float is = a.eval ? rsqrtf(v[c] + a.eps) : v[c];
  sa = g[c] * is;
  sb = b[c] - m[c] * sa;
}

// Forward apply: y = act(x*sa + sb [+ r | + r*ra + rb]), (sa, sb) = (gamma*invstd, beta - mean*gamma*invstd);
// eval mode derives invstd from the running variance.
template <int RES, bool VEC>
__global__ void __launch_bounds__(256) bn_apply_kernel(BnApplyArgs a) {
  const int C = a.C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  if (VEC) {
    const long long total = (long long)a.M * C / 8;
    const int c0 = (int)(threadIdx.x % (C / 8)) * 8;  // constant: 256 and the grid stride are multiples of C/8
    float sa[8], sb[8], ra[8], rb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bn_affine(a, a.gamma, a.beta, a.mean, a.invstd, c0 + j, sa[j], sb[j]);
      ra[j] = 1.f;
      rb[j] = 0.f;
      if (RES == 2) bn_affine(a, a.rgamma, a.rbeta, a.rmean, a.rinvstd, c0 + j, ra[j], rb[j]);
    }
#pragma unroll 2
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += stride) {
      const bf16x8 xv = reinterpret_cast<const bf16x8*>(a.x)[i];
      bf16x8 rv;
      if (RES) rv = reinterpret_cast<const bf16x8*>(a.r)[i];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = (float)xv[j] * sa[j] + sb[j];
        if (RES) v += (float)rv[j] * ra[j] + rb[j];
        if (a.relu) v = fmaxf(v, 0.f);
        o[j] = f2bf(v);
      }
      reinterpret_cast<bf16x8*>(a.y)[i] = o;
    }
  } else {
    const long long total = (long long)a.M * C;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += stride) {
      const int c = (int)(i % C);
      float sa, sb, ra = 1.f, rb = 0.f;
      bn_affine(a, a.gamma, a.beta, a.mean, a.invstd, c, sa, sb);
      if (RES == 2) bn_affine(a, a.rgamma, a.rbeta, a.rmean, a.rinvstd, c, ra, rb);
      float v = (float)a.x[i] * sa + sb;
      if (RES) v += (float)a.r[i] * ra + rb;
      if (a.relu) v = fmaxf(v, 0.f);
      a.y[i] = f2bf(v);
    }
  }
}

// Backward apply: dx = k1*g + k2*x + k3 with g = dy * relu'(mask).
template <bool VEC>
__global__ void __launch_bounds__(256) bn_dx_kernel(const bf16* __restrict__ x, const bf16* __restrict__ mask,
                                                    const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                                    const float* __restrict__ coef, long long M, int C) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  if (VEC) {
    const long long total = M * C / 8;
    const int c0 = (int)(threadIdx.x % (C / 8)) * 8;
    float k1[8], k2[8], k3[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k1[j] = coef[c0 + j];
      k2[j] = coef[C + c0 + j];
      k3[j] = coef[2 * C + c0 + j];
    }
#pragma unroll 2
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += stride) {
      const bf16x8 xv = reinterpret_cast<const bf16x8*>(x)[i];
      const bf16x8 gv = reinterpret_cast<const bf16x8*>(dy)[i];
      bf16x8 mv;
      if (mask) mv = reinterpret_cast<const bf16x8*>(mask)[i];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = (mask && !((float)mv[j] > 0.f)) ? 0.f : (float)gv[j];
        o[j] = f2bf(k1[j] * g + k2[j] * (float)xv[j] + k3[j]);
      }
      reinterpret_cast<bf16x8*>(dx)[i] = o;
    }
  } else {
    const long long total = M * C;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += stride) {
      const int c = (int)(i % C);
      const float g = (mask && !((float)mask[i] > 0.f)) ? 0.f : (float)dy[i];
      dx[i] = f2bf(coef[c] * g + coef[C + c] * (float)x[i] + coef[2 * C + c]);
    }
  }
}

static int ew_grid(long long n) {
  long long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

int bn_stats_grid(int M, int C) { return bn_grid(M, bn_rows_per_pass(C, bn_vec(C))); }

long long bn_stats_ws_floats(int M, int C) {
  const int G = bn_stats_grid(M, C);
  return (long long)(G + cdiv(G, BN_GROUP)) * 2 * C;
}

int bn_stats_counters(int M, int C) { return 1 + cdiv(bn_stats_grid(M, C), BN_GROUP); }

hipError_t bn_stats(const BnStatsArgs& a, int mode, hipStream_t st) {
  if (a.C > 1024 || a.C <= 0 || a.M <= 0) return hipErrorInvalidValue;
  const bool vec = bn_vec(a.C);
  if (!vec && a.C > 256) return hipErrorInvalidValue;
  const int G = bn_grid(a.M, bn_rows_per_pass(a.C, vec));
  if (mode == 0) {
    if (vec)
      hipLaunchKernelGGL((bn_stats_kernel<0, true>), dim3(G), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((bn_stats_kernel<0, false>), dim3(G), dim3(256), 0, st, a);
  } else {
    if (vec)
      hipLaunchKernelGGL((bn_stats_kernel<1, true>), dim3(G), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((bn_stats_kernel<1, false>), dim3(G), dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

bool bn_fused_ok(int C) { return bn_vec(C) && C <= 1024; }

// fused launches: ~8 rows per thread (one round of loads per phase), at most 1008 workgroups of 256
// threads (4 per CU: every workgroup is resident for the in-launch hand-off; 1 + 63 ticket words, the
// generation word is word 64)
static int bn_fused_grid(int M, int C) {
  int g = cdiv(M, bn_rows_per_pass(C, true) * 4);
  return g < 1 ? 1 : (g > 1008 ? 1008 : g);
}

// workgroups of kernel K the device holds at once (occupancy x CUs, queried once): the fused launch's
// grid never exceeds it, so that every workgroup is resident while the others wait for the hand-off
template <typename K>
static int bn_resident_cap(K kernel) {
  static int cap = -1;
  if (cap < 0) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess) per_cu = 1;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 1;
    // three quarters of the device: other streams' kernels (a concurrent all-reduce, a side-stream
    // branch) may hold CUs; the wait is bounded besides (a launch that still could not place every
    // workgroup ends slow, not hung)
    cap = per_cu * cus * 3 / 4;
    if (cap < 1) cap = 1;
  }
  return cap;
}

template <int MODE, int RES>
static hipError_t bn_fused_launch(const BnStatsArgs& a, const BnApplyArgs& p, bf16* dx, unsigned* gen, hipStream_t st) {
  int G = bn_fused_grid(a.M, a.C);
  const int cap = bn_resident_cap(bn_fused_kernel<MODE, RES>);
  if (G > cap) G = cap;
  hipLaunchKernelGGL((bn_fused_kernel<MODE, RES>), dim3(G), dim3(256), 0, st, a, p, dx, gen);
  return hipGetLastError();
}

hipError_t bn_fwd_fused(const BnStatsArgs& a, const BnApplyArgs& p, unsigned* gen, hipStream_t st) {
  if (!bn_fused_ok(a.C) || a.M <= 0 || p.C != a.C || p.M != a.M || p.eval || !gen) return hipErrorInvalidValue;
  const int res = p.r == nullptr ? 0 : (p.rgamma == nullptr ? 1 : 2);
  if (res == 0) return bn_fused_launch<0, 0>(a, p, nullptr, gen, st);
  if (res == 1) return bn_fused_launch<0, 1>(a, p, nullptr, gen, st);
  return bn_fused_launch<0, 2>(a, p, nullptr, gen, st);
}

hipError_t bn_bwd_fused(const BnStatsArgs& a, bf16* dx, unsigned* gen, hipStream_t st) {
  if (!bn_fused_ok(a.C) || a.M <= 0 || !dx || !gen) return hipErrorInvalidValue;
  BnApplyArgs p{};
  return bn_fused_launch<1, 0>(a, p, dx, gen, st);
}

hipError_t bn_apply(const BnApplyArgs& a, hipStream_t st) {
  const bool vec = bn_vec(a.C);
  const long long n = (long long)a.M * a.C / (vec ? 8 : 1);
  const int grid = ew_grid(n);
  const int res = a.r == nullptr ? 0 : (a.rgamma == nullptr ? 1 : 2);
#define DFA_BN_APPLY(R)                                                              \
  if (vec)                                                                           \
    hipLaunchKernelGGL((bn_apply_kernel<R, true>), dim3(grid), dim3(256), 0, st, a); \
  else                                                                               \
    hipLaunchKernelGGL((bn_apply_kernel<R, false>), dim3(grid), dim3(256), 0, st, a);
  if (res == 0) {
    DFA_BN_APPLY(0)
  } else if (res == 1) {
    DFA_BN_APPLY(1)
  } else {
    DFA_BN_APPLY(2)
  }
#undef DFA_BN_APPLY
  return hipGetLastError();
}

hipError_t bn_dx(const bf16* x, const bf16* mask, const bf16* dy, bf16* dx, const float* coef, int M, int C,
                 hipStream_t st) {
  const bool vec = bn_vec(C);
  const long long n = (long long)M * C / (vec ? 8 : 1);
  if (vec)
    hipLaunchKernelGGL(bn_dx_kernel<true>, dim3(ew_grid(n)), dim3(256), 0, st, x, mask, dy, dx, coef, (long long)M, C);
  else
    hipLaunchKernelGGL(bn_dx_kernel<false>, dim3(ew_grid(n)), dim3(256), 0, st, x, mask, dy, dx, coef, (long long)M,
                       C);
  return hipGetLastError();
}

// ---- consumers of epilogue-accumulated sums (kernels.h BnAcc / BnAccFin, csrc/bn_acc.h) ------------------
// The producing conv added fp64 partials of [S, Q] into nrep replicas; every workgroup here finalises the
// per-channel coefficients itself (threads c < C, replicas in fixed order) into LDS, then streams.  The
// replica reads are C * nrep * 16 bytes per workgroup, so the grid is capped to keep them a few MB.
constexpr int kBnAccMaxC = 1024;

// kBnVecs 8-channel vectors per thread per batch; the grid gives every thread about one batch (all of
// its loads in flight at once), within [256, 4096] workgroups
constexpr int kBnVecs = 4;
static int bn_acc_grid(long long nvec, int C, int nrep) {
  (void)C, (void)nrep;
  long long g = (nvec + 256LL * kBnVecs - 1) / (256LL * kBnVecs);
  return (int)std::min(4096LL, std::max(256LL, g));
}

// The nrep replicas of [S, Q] of the CPT channels c + 256 k of this thread, summed in replica order.  Every
// load of a chunk of 8 replicas is issued before the first is used, at a clamped (always valid) address, its
// value selected afterwards: with one branch per replica the compiler waited for each load in turn -- and,
// vmcnt being in order, for the tensor loads issued before them -- a chain of round trips that cost 2-3 us
// per launch on a tiny tensor (scripts/bn_microbench.py).  One chunk (nrep <= 8): one round trip.
template <int CPT, int RC = 8>
__device__ __forceinline__ void bn_fin_sums(const BnAccFin& f, int C, int c, double (&S)[CPT], double (&Q)[CPT]) {
#pragma unroll
  for (int k = 0; k < CPT; ++k) S[k] = 0.0, Q[k] = 0.0;
#pragma unroll
  for (int r0 = 0; r0 < kBnAccMaxRep; r0 += RC) {
    if (r0 >= f.nrep) break;  // (uniform)
    double s[CPT][RC], q[CPT][RC];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int cc = min(c + 256 * k, C - 1);
#pragma unroll
      for (int j = 0; j < RC; ++j) {
        const long long rr = min(r0 + j, f.nrep - 1);
        s[k][j] = f.acc[(2 * rr) * C + cc];
        q[k][j] = f.acc[(2 * rr + 1) * C + cc];
      }
    }
#pragma unroll
    for (int k = 0; k < CPT; ++k)
#pragma unroll
      for (int j = 0; j < RC; ++j) {
        S[k] += r0 + j < f.nrep ? s[k][j] : 0.0;
        Q[k] += r0 + j < f.nrep ? q[k][j] : 0.0;
      }
  }
}

// forward: mean / invstd of channel c from its sums (workgroup 0 also publishes them, updates the running
// statistics and clears f.zero); returns the affine pair (sa, sb) of gamma, beta.  The moments are fp64
// (S, Q and the cancellation in Q / M - m^2); invstd is an fp32 reciprocal square root of the variance.
__device__ __forceinline__ void bn_fin_fwd(const BnAccFin& f, const float* gamma, const float* beta, int C, long long M,
                                           double invM, int c, double S, double Q, float& sa, float& sb) {
  const double m = S * invM;
  double var = Q * invM - m * m;
  if (var < 0.0) var = 0.0;
  const float is = rsqrtf((float)var + f.eps);
  sa = gamma[c] * is;
  sb = beta[c] - (float)m * sa;
  if (blockIdx.x == 0) {
    f.mean[c] = (float)m;
    f.invstd[c] = is;
    if (f.run_mean) {
      const double unb = M > 1 ? var * ((double)M / (double)(M - 1)) : var;
      f.run_mean[c] = (float)((1.0 - f.momentum) * f.run_mean[c] + f.momentum * m);
      f.run_var[c] = (float)((1.0 - f.momentum) * f.run_var[c] + f.momentum * unb);
    }
    if (f.zero)
      for (int r = 0; r < 2 * f.nrep; ++r) f.zero[(long long)r * C + c] = 0.0;
  }
}

// replicas per load batch of the finalisation
#ifndef DFA_BN_FIN_RC
#define DFA_BN_FIN_RC 8
#endif
constexpr int kBnFinRC = DFA_BN_FIN_RC;
// channels per thread of the finalisation (256 threads)
static int bn_cpt(int C) { return C <= 256 ? 1 : (C <= 512 ? 2 : 4); }

// The streaming part of both consumers: a thread's vectors i = i0 + k * stride in batches of kBnVecs, every
// load of a batch issued before its stores (a load behind a store waits for that store too); the first
// batch's loads go out BEFORE the statistics are finalised (they do not depend on them), so the prologue's
// replica reads and the first tensor reads share one round trip.
template <int RES, int CPT>
__global__ void __launch_bounds__(256) bn_apply_acc_kernel(BnApplyArgs a, BnAccFin f, BnAccFin fr) {
  constexpr int RC = kBnFinRC;
  __shared__ float co[4][kBnAccMaxC];  // sa, sb, ra, rb
  const int C = a.C;
  const long long M = a.M;
  const long long total = M * C / 8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const bf16x8* xs = reinterpret_cast<const bf16x8*>(a.x);
  const bf16x8* rs = reinterpret_cast<const bf16x8*>(a.r);
  bf16x8 xv[kBnVecs], rv[kBnVecs];
  auto load = [&](long long base) {
#pragma unroll
    for (int k = 0; k < kBnVecs; ++k) {
      const long long i = min(base + k * stride, total - 1);  // (clamped: not stored)
      xv[k] = xs[i];
      if (RES) rv[k] = rs[i];
    }
  };
  load(i0);
  const double invM = 1.0 / (double)M;
  {
    const int c = threadIdx.x;
    double S[CPT], Q[CPT], RS[CPT], RQ[CPT];
    bn_fin_sums<CPT, RC>(f, C, c, S, Q);
    if (RES == 2) bn_fin_sums<CPT, RC>(fr, C, c, RS, RQ);
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int ck = c + 256 * k;
      if (ck < C) {
        float sa, sb, ra = 1.f, rb = 0.f;
        bn_fin_fwd(f, a.gamma, a.beta, C, M, invM, ck, S[k], Q[k], sa, sb);
        if (RES == 2) bn_fin_fwd(fr, a.rgamma, a.rbeta, C, M, invM, ck, RS[k], RQ[k], ra, rb);
        co[0][ck] = sa;
        co[1][ck] = sb;
        co[2][ck] = ra;
        co[3][ck] = rb;
      }
    }
  }
  __syncthreads();
  const int c0 = (int)(threadIdx.x % (C / 8)) * 8;  // constant: 256 and the grid stride are multiples of C/8
  float sa[8], sb[8], ra[8], rb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sa[j] = co[0][c0 + j];
    sb[j] = co[1][c0 + j];
    ra[j] = RES == 2 ? co[2][c0 + j] : 1.f;
    rb[j] = RES == 2 ? co[3][c0 + j] : 0.f;
  }
  bf16x8* ys = reinterpret_cast<bf16x8*>(a.y);
  for (long long base = i0; base < total; base += kBnVecs * stride) {
    if (base != i0) load(base);
#pragma unroll
    for (int k = 0; k < kBnVecs; ++k) {
      const long long i = base + k * stride;
      if (i >= total) break;
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = (float)xv[k][j] * sa[j] + sb[j];
        if (RES == 1) v += (float)rv[k][j];  // (ra, rb = 1, 0: the same value)
        if (RES == 2) v += (float)rv[k][j] * ra[j] + rb[j];
        if (a.relu) v = fmaxf(v, 0.f);
        o[j] = f2bf(v);
      }
      ys[i] = o;
    }
  }
}

hipError_t bn_apply_acc(const BnApplyArgs& a, const BnAccFin& f, const BnAccFin* fr, hipStream_t st) {
  if (a.C % 8 || a.C > kBnAccMaxC || 256 % (a.C / 8) || a.M <= 0 || !f.acc || f.nrep < 1 ||
      f.nrep > kBnAccMaxRep || (fr && (fr->nrep < 1 || fr->nrep > kBnAccMaxRep)) || a.eval)
    return hipErrorInvalidValue;
  const int res = a.r == nullptr ? 0 : (fr == nullptr ? 1 : 2);
  const int nrep = f.nrep + (fr ? fr->nrep : 0);
  const int grid = bn_acc_grid((long long)a.M * a.C / 8, a.C, nrep);
  const BnAccFin none{};
  const BnAccFin& g = fr ? *fr : none;
#define DFA_BN_APPLY_ACC(R, CPT) \
  hipLaunchKernelGGL((bn_apply_acc_kernel<R, CPT>), dim3(grid), dim3(256), 0, st, a, f, g)
#define DFA_BN_APPLY_ACC_C(R)                      \
  switch (bn_cpt(a.C)) {                           \
    case 1: DFA_BN_APPLY_ACC(R, 1); break;         \
    case 2: DFA_BN_APPLY_ACC(R, 2); break;         \
    default: DFA_BN_APPLY_ACC(R, 4); break;        \
  }
  if (res == 0) {
    DFA_BN_APPLY_ACC_C(0)
  } else if (res == 1) {
    DFA_BN_APPLY_ACC_C(1)
  } else {
    DFA_BN_APPLY_ACC_C(2)
  }
#undef DFA_BN_APPLY_ACC_C
#undef DFA_BN_APPLY_ACC
  return hipGetLastError();
}

// backward: dx = k1 g + k2 x + k3, k from [S = sum g, Q = sum g * xhat]
template <int CPT>
__global__ void __launch_bounds__(256) bn_dx_acc_kernel(const bf16* __restrict__ x, const bf16* __restrict__ g,
                                                        bf16* __restrict__ dx, BnAccFin f, long long M, int C) {
  __shared__ float k[3][kBnAccMaxC];
  const long long total = M * C / 8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const bf16x8* xs = reinterpret_cast<const bf16x8*>(x);
  const bf16x8* gs = reinterpret_cast<const bf16x8*>(g);
  bf16x8 xv[kBnVecs], gv[kBnVecs];
  auto load = [&](long long base) {
#pragma unroll
    for (int kk = 0; kk < kBnVecs; ++kk) {
      const long long i = min(base + kk * stride, total - 1);  // (clamped: not stored)
      xv[kk] = xs[i];
      gv[kk] = gs[i];
    }
  };
  load(i0);
  {
    const int c = threadIdx.x;
    // the per-channel inputs of the coefficients, issued with the replica loads (clamped, one round trip)
    float isd[CPT], gam[CPT], mn[CPT];
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int cc = min(c + 256 * j, C - 1);
      isd[j] = f.invstd[cc];
      gam[j] = f.gamma[cc];
      mn[j] = f.mean[cc];
    }
    double S[CPT], Q[CPT];
    bn_fin_sums<CPT, kBnFinRC>(f, C, c, S, Q);
    const double invM = 1.0 / (double)M;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int cj = c + 256 * j;
      if (cj >= C) continue;
      const double is = isd[j], k1 = (double)gam[j] * is, sm = S[j] * invM, qm = Q[j] * invM;
      const float a1 = (float)k1, a2 = (float)(-k1 * is * qm), a3 = (float)(k1 * ((double)mn[j] * is * qm - sm));
      k[0][cj] = a1;
      k[1][cj] = a2;
      k[2][cj] = a3;
      if (blockIdx.x == 0) {
        f.dbeta[cj] = (float)S[j] * f.gscale;
        f.dgamma[cj] = (float)Q[j] * f.gscale;
        if (f.coef) {
          f.coef[cj] = a1;
          f.coef[C + cj] = a2;
          f.coef[2 * C + cj] = a3;
        }
        if (f.zero)
          for (int r = 0; r < 2 * f.nrep; ++r) f.zero[(long long)r * C + cj] = 0.0;
      }
    }
  }
  __syncthreads();
  const int c0 = (int)(threadIdx.x % (C / 8)) * 8;
  float k1[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k1[j] = k[0][c0 + j];
    k2[j] = k[1][c0 + j];
    k3[j] = k[2][c0 + j];
  }
  bf16x8* ds = reinterpret_cast<bf16x8*>(dx);
  for (long long base = i0; base < total; base += kBnVecs * stride) {
    if (base != i0) load(base);
#pragma unroll
    for (int kk = 0; kk < kBnVecs; ++kk) {
      const long long i = base + kk * stride;
      if (i >= total) break;
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(k1[j] * (float)gv[kk][j] + k2[j] * (float)xv[kk][j] + k3[j]);
      ds[i] = o;
    }
  }
}

hipError_t bn_dx_acc(const bf16* x, const bf16* g, bf16* dx, const BnAccFin& f, int M, int C, hipStream_t st) {
  if (C % 8 || C > kBnAccMaxC || 256 % (C / 8) || M <= 0 || !f.acc || f.nrep < 1 || f.nrep > kBnAccMaxRep ||
      !f.gamma || !f.dgamma)
    return hipErrorInvalidValue;
  const int grid = bn_acc_grid((long long)M * C / 8, C, f.nrep);
  switch (bn_cpt(C)) {
    case 1: hipLaunchKernelGGL(bn_dx_acc_kernel<1>, dim3(grid), dim3(256), 0, st, x, g, dx, f, (long long)M, C); break;
    case 2: hipLaunchKernelGGL(bn_dx_acc_kernel<2>, dim3(grid), dim3(256), 0, st, x, g, dx, f, (long long)M, C); break;
    default: hipLaunchKernelGGL(bn_dx_acc_kernel<4>, dim3(grid), dim3(256), 0, st, x, g, dx, f, (long long)M, C); break;
  }
  return hipGetLastError();
}

// GAP backward (dx[b][p][c] = dy[b][c] / HW) with relu' of the block output and the BatchNorm backward sums
// of dx: a thread keeps one 4-channel group (256 % (C / 4) == 0) over its rows, the workgroup reduces the
// groups through LDS slots (csrc/bn_acc.h)
__global__ void __launch_bounds__(256) gap_bwd_bn_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ mask,
                                                         bf16* __restrict__ dx, int B, int HW, int C, BnAcc e) {
  __shared__ float red[3 * 1024];
  const int cpr = C / 4, rpb = 256 / cpr;
  const int c4 = (int)(threadIdx.x % cpr) * 4;
  const float inv = 1.f / HW;
  BnAccLane bl;
  bacc_zero(bl);
  const BnAccChan bc = bacc_chan(e, c4);
  const long long rows = (long long)B * HW;
  for (long long r = (long long)blockIdx.x * rpb + threadIdx.x / cpr; r < rows; r += (long long)gridDim.x * rpb) {
    const long long o = r * C + c4;
    const long long b = r / HW;
    const bacc_bf16x4 g = *reinterpret_cast<const bacc_bf16x4*>(dy + b * C + c4);
    const bacc_bf16x4 mk = *reinterpret_cast<const bacc_bf16x4*>(mask + o);
    bacc_bf16x4 ov;
    float sv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ov[j] = f2bf((float)mk[j] > 0.f ? (float)g[j] * inv : 0.f);
      sv[j] = (float)ov[j];
    }
    *reinterpret_cast<bacc_bf16x4*>(dx + o) = ov;
    bacc_add4(bl, e, bc, o, sv);
  }
  bacc_stash(red, threadIdx.x / cpr, C, c4, bl);
  __syncthreads();
  bacc_flush(e, red, rpb, C, 0, C, threadIdx.x, 256);
}

hipError_t gap_bwd_bn(const bf16* dy, const bf16* mask, bf16* dx, int B, int HW, int C, const BnAcc& bacc,
                      hipStream_t st) {
  if (C % 4 || C > 1024 || 256 % (C / 4) || !bacc.acc || bacc.mode != 1 || bacc.acc2 || bacc.nrep < 1)
    return hipErrorInvalidValue;
  const long long rows = (long long)B * HW;
  const int rpb = 256 / (C / 4);
  const int grid = (int)std::min<long long>(std::max<long long>(1, (rows + rpb - 1) / rpb), 256);
  hipLaunchKernelGGL(gap_bwd_bn_kernel, dim3(grid), dim3(256), 0, st, dy, mask, dx, B, HW, C, bacc);
  return hipGetLastError();
}

}  // namespace dfa
