// Device helpers of the SGD update shared by the multi-tensor optimizer (csrc/optim.hip) and the
// single-rank LeNet-5 reduce kernel that applies the update itself (csrc/lenet_fused.hip).
#pragma once
#include "common.h"
#include "kernels.h"
#include "lenet_frag.h"

namespace dfa {

// The bf16 compute copies of element i (value w) of a matrix parameter.
__device__ __forceinline__ void emit_copies(const ParamDesc& d, int i, float w, bf16* __restrict__ wbf) {
  if (d.bf_off < 0) return;
  const int K = d.T * d.Ci;
  const int n = i / K;
  const int kk = i - n * K;
  const bf16 wb = f2bf(w);
  if ((d.pad_ >> 28) & 1) {  // tile-mode layouts, element-wise (the LeNet fragment workgroup's path)
    const int t = kk / d.Ci, ci = kk - t * d.Ci;
    wbf[d.bf_off + (long long)n * round_up(K, 32) + kk] = wb;
    wbf[d.bft_off + (long long)ci * round_up(d.T * d.N, 32) + t * d.N + n] = wb;
    return;
  }
  // d.pad_ = KW | Cp << 16 (KW > 0): the primary copy uses the row-segment layout of the fused
  // conv+pool forward, [Npad16][round32(KH * round8(KW*Cp))], column ky*round8(KW*Cp) + kx*Cp + ci
  // d.pad_ = KW | Cp << 16 | pair << 30: pair layout (N <= 8) = 16 rows, rows 8+n hold channel n
  // shifted right by one kernel column (the fused conv+pool forward computes pixels x and x+1)
  const int rKW = d.pad_ & 0xffff;
  // d.pad_ bit 29: the dgrad copy uses the conv+pool dgrad pair layout (csrc/convpool.hip make_dgrad),
  // [16][round32(KH*(KW+1)*N)]: row ci col (a*(KW+1) + KW-1-kx)*N + n and row 8+ci col (a*(KW+1) + KW-kx)*N + n,
  // a = KH-1-ky (the kernel flip of the transposed convolution)
  const int rCp = ((d.pad_ >> 16) & 0xfff) > 0 ? ((d.pad_ >> 16) & 0xfff) : d.Ci;
  const bool rpair = (d.pad_ >> 30) & 1;
  const bool tpair = rKW > 0 && ((d.pad_ >> 29) & 1);
  const int RLp = rKW > 0 ? round_up((rKW + (rpair ? 1 : 0)) * rCp, 8) : K;
  const int Kpad = round_up(rKW > 0 ? (d.T / rKW) * RLp : K, 32);
  const int KpadT = round_up(tpair ? (d.T / rKW) * (rKW + 1) * d.N : d.T * d.N, 32);
  int col = kk;
  if (rKW > 0) {
    const int t = kk / d.Ci, ci = kk - (kk / d.Ci) * d.Ci;
    const int ky = t / rKW, kx = t - (t / rKW) * rKW;
    col = ky * RLp + kx * rCp + ci;
  }
  wbf[d.bf_off + (long long)n * Kpad + col] = wb;
  if (rpair) wbf[d.bf_off + (long long)(n + 8) * Kpad + col + rCp] = wb;
  if (d.bft_off >= 0) {
    const int t = kk / d.Ci;
    const int ci = kk - t * d.Ci;
    if (tpair) {
      const int ky = t / rKW, kx = t - ky * rKW;
      const int c0 = ((d.T / rKW - 1 - ky) * (rKW + 1) + rKW - 1 - kx) * d.N + n;
      wbf[d.bft_off + (long long)ci * KpadT + c0] = wb;
      wbf[d.bft_off + (long long)(ci + 8) * KpadT + c0 + d.N] = wb;
    } else {
      wbf[d.bft_off + (long long)ci * KpadT + t * d.N + n] = wb;
    }
  }
}

// One parameter element: w <- SGD(w, g) with the optimizer's exact (non-contracted) arithmetic,
// momentum written back, bf16 compute copies re-emitted.  hyper = [lr, momentum, wd, grad_scale,
// nesterov].  Returns the new weight.
__device__ __forceinline__ float sgd_apply_one(const ParamDesc& d, int i, float g, float* __restrict__ master,
                                               float* __restrict__ mom_buf, bf16* __restrict__ wbf,
                                               const float* __restrict__ hyper) {
  const float lr = hyper[0], mom = hyper[1], wd = hyper[2], gs = hyper[3];
  const bool nesterov = hyper[4] != 0.f;
  const long long o = d.off + i;
  float v = 0.f;
  const float w = sgd_new_weight(master[o], g, mom != 0.f ? mom_buf[o] : 0.f, lr, mom, wd, gs, nesterov, &v);
  if (mom != 0.f) mom_buf[o] = v;
  master[o] = w;
  emit_copies(d, i, w, wbf);
  return w;
}

}  // namespace dfa
