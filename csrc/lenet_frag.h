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

// Inverse of lenet_frag_lane: store bf16(w) of conv weight j into every fragment element that holds it
// (conv1: 8 banded positions; conv2: 1 forward + 2 pair-banded data-gradient positions).  The update
// workgroup that owns weight j scatters it right after updating it, so the next step's fragments are
// complete when the launch ends (no last-arriver rebuild); elements that hold no weight stay zero from
// the buffer's initial build.
__device__ __forceinline__ void lenet_frag_scatter(void* frag_buf, int j, float w) {
  bf16* fr = reinterpret_cast<bf16*>(frag_buf);
  const bf16 v = f2bf(w);
  auto put = [&](int f, int lane, int e) { fr[((f * 64) + lane) * 8 + e] = v; };
  if (j < 150) {  // conv1 [c][ky][kx]
    const int c = j / 25, r = j - 25 * c, ky = r / 5, kx = r - 5 * ky;
    const int f = ky * 3 + (c >> 1);
#pragma unroll
    for (int j8 = 0; j8 < 8; ++j8) {
      const int t = kx + 2 * j8;
      put(f, (t >> 3) * 16 + (c & 1) * 8 + j8, t & 7);
    }
    return;
  }
  // conv2 [n][tap = ky * 5 + kx][c]
  const int q = j - 150, n = q / 150, r = q - 150 * n, tap = r / 6, c = r - 6 * tap;
  put(FR_C2 + (tap >> 2), (tap & 3) * 16 + n, c);
  const int ky = tap / 5, kx = tap - 5 * ky;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int P = ky * 6 + kx + 1 - b;
    put(FR_DG + (P >> 1), ((P & 1) * 2 + (n >> 3)) * 16 + b * 8 + c, n & 7);
  }
}

// w: the 2550 conv weights (any memory); nt threads of a block build every fragment
__device__ __forceinline__ void lenet_build_frags(const float* w, bf16x8* __restrict__ frag, int tid, int nt) {
  for (int fl = tid; fl < kLeNetFragLanes; fl += nt) frag[fl] = lenet_frag_lane(fl, [&](int j) { return w[j]; });
}

// The SGD update of one parameter with every operation rounded on its own, so the optimizer's fragment
// rebuild and the owning workgroup's update produce the same bits whatever they are inlined into.
// (HIP's __fmul_rn / __fadd_rn are plain operators that -ffp-contract may still fuse into an FMA after
// inlining; the pragma keeps the multiplies and adds created here separate.)
__device__ __forceinline__ float sgd_new_weight(float w, float gr, float m, float lr, float mom, float wd, float gs,
                                                bool nesterov, float* m_out) {
#pragma clang fp contract(off)
  float g = gr * gs;
  if (wd != 0.f) g = g + wd * w;
  if (mom != 0.f) {
    const float v = mom * m + g;
    if (m_out) *m_out = v;
    g = nesterov ? g + mom * v : v;
  }
  return w - lr * g;
}

}  // namespace dfa
