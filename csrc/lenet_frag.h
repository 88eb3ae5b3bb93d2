// MFMA B fragments of the fused LeNet-5 step's conv weights (csrc/lenet_fused.hip), shared by its
// prep launch and by the optimizer (csrc/optim.hip), which rebuilds them from the weights it just
// updated so that a training step needs no separate prep launch.
//   [NFRAG][64 lanes] x 8 bf16:  conv1 banded (f = ky * 3 + T: column j = output x offset 2 (j & 7)
//   [+ row parity], channel 2T + (j >> 3); k = input column), conv2 forward (step s: column n,
//   k = (tap 4s + g, channel e)), conv2 data gradient pair-banded (step s: column (b = j >> 3,
//   c = j & 7), k = ((ky, u), n) with kx = u - 1 + b).
#pragma once
#include "common.h"

namespace dfa {

constexpr int NFRAG = 37;
constexpr int FR_C1 = 0, FR_C2 = 15, FR_DG = 22;

constexpr int kLeNetFragLanes = NFRAG * 64;
constexpr int kLeNetConvW = 2550;  // conv1 kernel [6][25] then conv2 kernel [16][150]

// Fragment lane fl (fragment fl / 64, lane fl % 64); W(j) = conv weight j of the 2550 above.
template <typename W>
__device__ __forceinline__ bf16x8 lenet_frag_lane(int fl, W&& wt) {
  const int f = fl >> 6, lane = fl & 63, i = lane & 15, g = lane >> 4;
  bf16x8 o;
  if (f < FR_C2) {
    const int ky = f / 3, T = f - 3 * (f / 3), c = 2 * T + (i >> 3), j8 = i & 7;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kx = 8 * g + e - 2 * j8;
      o[e] = f2bf((kx >= 0 && kx < 5) ? wt(c * 25 + ky * 5 + kx) : 0.f);
    }
  } else if (f < FR_DG) {
    const int s = f - FR_C2, tap = 4 * s + g;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf((tap < 25 && e < 6) ? wt(150 + i * 150 + tap * 6 + e) : 0.f);
  } else {
    const int s = f - FR_DG, P = 2 * s + (g >> 1), ky = P / 6, u = P - 6 * (P / 6);
    const int b = i >> 3, c = i & 7, kx = u - 1 + b;
    const bool ok = P < 30 && kx >= 0 && kx < 5 && c < 6;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int n = 8 * (g & 1) + e;
      o[e] = f2bf(ok ? wt(150 + n * 150 + (ky * 5 + kx) * 6 + c) : 0.f);
    }
  }
  return o;
}

// w: the 2550 conv weights (any memory); nt threads of a block build every fragment
__device__ __forceinline__ void lenet_build_frags(const float* w, bf16x8* __restrict__ frag, int tid, int nt) {
  for (int fl = tid; fl < kLeNetFragLanes; fl += nt) frag[fl] = lenet_frag_lane(fl, [&](int j) { return w[j]; });
}

// The SGD update of one parameter with every operation rounded on its own (no contraction), so the
// optimizer's fragment rebuild and the owning workgroup's update produce the same bits.
__device__ __forceinline__ float sgd_new_weight(float w, float gr, float m, float lr, float mom, float wd, float gs,
                                                bool nesterov, float* m_out) {
  float g = __fmul_rn(gr, gs);
  if (wd != 0.f) g = __fadd_rn(g, __fmul_rn(wd, w));
  if (mom != 0.f) {
    const float v = __fadd_rn(__fmul_rn(mom, m), g);
    if (m_out) *m_out = v;
    g = nesterov ? __fadd_rn(g, __fmul_rn(mom, v)) : v;
  }
  return __fsub_rn(w, __fmul_rn(lr, g));
}

}  // namespace dfa
