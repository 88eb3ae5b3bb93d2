// Fused dense head (gfx950): the trailing Dense chain of a classifier + softmax-cross-entropy, as
// TWO launches per training step instead of ~3 per layer plus loss kernels.
//
// The reference trains with tf.js per-layer matMul/add/relu ops and a separate loss graph
// (DistributedTfModel.fit, /root/reference/src/common/models.ts:128-142).  For the MNIST
// heads (400->120->84->10 in LeNet-5) every one of those GEMMs is tiny (M = batch, N,K <= 400), so
// per-kernel latency, not FLOPs, is the cost.  Here:
//
//   head_train_kernel   one workgroup per 16 batch rows: X rows are staged in LDS once; each layer's
//                       forward GEMM (MFMA 16x16x32, A from LDS, B = weights straight from L2) writes
//                       its ReLU output back to LDS; softmax-CE runs on the 16 logit rows; the backward
//                       data chain dZ_l = (dZ_{l+1} W_{l+1}) * relu'(H_l) runs in LDS as well and only
//                       dX (for the layer below) plus the transposed per-layer activations H^T and
//                       gradients dZ^T (for the weight gradients) reach HBM.
//   head_wgrad_kernel   one workgroup per 16x16 tile of every dW_l = dZ_l^T H_{l-1} (bias = an extra
//                       column of ones): the full batch reduction inside the workgroup (4 waves split
//                       the batch, LDS combine) -> deterministic, no split-K slabs, no reduce pass.
//                       One extra workgroup sums the per-block loss partials into stats[2].
#include "common.h"
#include "kernels.h"

namespace dfa {

static unsigned long long* g_head_stamps = nullptr;
void head_set_stamps(void* buf) { g_head_stamps = reinterpret_cast<unsigned long long*>(buf); }

// per-block phase clocks (diagnostic; scripts/headstamps.py)
#define HD_STAMP(slot)                                                            \
  do {                                                                            \
    if (a.stamps) {                                                               \
      __builtin_amdgcn_sched_barrier(0);                                          \
      unsigned long long t_;                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                          \
      if (threadIdx.x == 0) a.stamps[blockIdx.x * 32 + (slot)] = t_;              \
    }                                                                             \
  } while (0)

constexpr int HR = 16;  // batch rows per workgroup of the train kernel
constexpr int HW = 16;  // waves per workgroup (both kernels): tiles of a layer spread over 16 waves

__device__ __forceinline__ bf16x8 ld16(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// Z[16][N] = A[16][Kpad] * W^T (+bias, relu) for the column tiles of this wave.
//   A: LDS rows of stride lda (zero padded to Kpad)      W: global [Npad16][Kpad]
//   out: LDS rows of stride ldo (bf16), optional fp32 LDS copy (logits), optional global H^T [N][ldt]
template <int KSMAX>
__device__ __forceinline__ void head_gemm_fwd(const bf16* A, int lda, const bf16* __restrict__ W, int Kpad,
                                              const float* __restrict__ bias, int N, int relu, bf16* out, int ldo,
                                              float* out32, bf16* __restrict__ hT, int ldt, int r0, int rows) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int ks = Kpad / 32;
  const int ntiles = (N + 15) / 16;
  for (int t = wid; t < ntiles; t += HW) {
    const int n = 16 * t + (lane & 15);
    const bf16* wrow = W + (long long)n * Kpad + 8 * (lane >> 4);
    const bf16* arow = A + (lane & 15) * lda + 8 * (lane >> 4);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    // weights: issue every k-step's load before the MFMA chain (L2 latency once per tile)
    bf16x8 b[KSMAX];
#pragma unroll
    for (int s = 0; s < KSMAX; ++s)
      if (s < ks) b[s] = ld16(wrow + 32 * s);
#pragma unroll
    for (int s = 0; s < KSMAX; ++s)
      if (s < ks) acc = mfma16x16x32(ld16(arow + 32 * s), b[s], acc);
    for (int s = KSMAX; s < ks; ++s) acc = mfma16x16x32(ld16(arow + 32 * s), ld16(wrow + 32 * s), acc);
    const float bv = (bias && n < N) ? bias[n] : 0.f;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = acc[r] + bv;
      if (relu) v[r] = fmaxf(v[r], 0.f);
      if (n >= N) v[r] = 0.f;
      const int row = 4 * (lane >> 4) + r;
      out[row * ldo + n] = f2bf(v[r]);
      if (out32) out32[row * 16 + (n & 15)] = v[r];
    }
    if (hT && n < N) {  // H^T[n][r0 + 4*(lane>>4) + r]
      bf16* dst = hT + (long long)n * ldt + r0 + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * (lane >> 4) + r < rows) dst[r] = f2bf(v[r]);
    }
  }
}

// dA[16][K] = dZ[16][Npad32] * W  (W^T rows from the dgrad-layout copy Wt [Kpad16][ldwt]),
// masked by (Aprev > 0) when mask != nullptr.
template <int KSMAX>
__device__ __forceinline__ void head_gemm_bwd(const bf16* dZ, int ldz, const bf16* __restrict__ Wt, int ldwt, int K,
                                              const bf16* mask, int ldm, bf16* out, int ldo, bf16* __restrict__ gout,
                                              int ldg, bf16* __restrict__ gT, int ldt, int r0, int rows,
                                              float scale = 1.f) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int ks = ldwt / 32;
  const int ktiles = (K + 15) / 16;
  for (int t = wid; t < ktiles; t += HW) {
    const int j = 16 * t + (lane & 15);
    const bf16* wrow = Wt + (long long)j * ldwt + 8 * (lane >> 4);
    const bf16* zrow = dZ + (lane & 15) * ldz + 8 * (lane >> 4);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    bf16x8 b[KSMAX];
#pragma unroll
    for (int s = 0; s < KSMAX; ++s)
      if (s < ks) b[s] = ld16(wrow + 32 * s);
#pragma unroll
    for (int s = 0; s < KSMAX; ++s)
      if (s < ks) acc = mfma16x16x32(ld16(zrow + 32 * s), b[s], acc);
    for (int s = KSMAX; s < ks; ++s) acc = mfma16x16x32(ld16(zrow + 32 * s), ld16(wrow + 32 * s), acc);
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * (lane >> 4) + r;
      v[r] = acc[r];
      if (mask && !((float)mask[row * ldm + j] > 0.f)) v[r] = 0.f;
      if (j >= K) v[r] = 0.f;
      if (scale != 1.f) v[r] = (float)f2bf(v[r]) * scale;  // a folded dropout's 1/(1-p)
      if (out) out[row * ldo + j] = f2bf(v[r]);
      if (gout && j < K && row < rows) gout[(long long)(r0 + row) * ldg + j] = f2bf(v[r]);
    }
    if (gT && j < K) {
      bf16* dst = gT + (long long)j * ldt + r0 + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * (lane >> 4) + r < rows) dst[r] = f2bf(v[r]);
    }
  }
}

__global__ void __launch_bounds__(1024) head_train_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * HR;
  const int rows = min(HR, a.B - r0);
  // LDS: X [16][ldx], then per layer l: H_l [16][ld_l] and dZ_l [16][ld_l], logits fp32 [16][16]
  const int ldx = a.L[0].Kpad + 8;  // +8 elements: rows start in different banks
  bf16* xs = reinterpret_cast<bf16*>(smem);
  char* p = smem + round_up(HR * ldx * 2, 16);
  bf16* hs[kHeadMaxLayers];
  bf16* dzs[kHeadMaxLayers];
  int ld[kHeadMaxLayers];
#pragma unroll
  for (int l = 0; l < kHeadMaxLayers; ++l) {
    ld[l] = l < a.nl ? round_up(a.L[l].N, 32) + 8 : 8;
    hs[l] = reinterpret_cast<bf16*>(p);
    dzs[l] = reinterpret_cast<bf16*>(p);
    if (l < a.nl) {
      p += round_up(HR * ld[l] * 2, 16);
      dzs[l] = reinterpret_cast<bf16*>(p);
      p += round_up(HR * ld[l] * 2, 16);
    }
  }
  float* lg = reinterpret_cast<float*>(p);  // [16][16]
  HD_STAMP(0);

  // ---- stage X rows (zero padded to Kpad; rows past B are zero)
  const int D0 = a.L[0].K;
  const int Kp0 = a.L[0].Kpad;
  for (int e = tid; e < HR * (Kp0 / 8); e += 64 * HW) {
    const int r = e / (Kp0 / 8), c8 = 8 * (e - r * (Kp0 / 8));
    bf16x8 v;
    if (r < rows && c8 + 8 <= D0 && (D0 & 7) == 0) {
      v = ld16(a.x + (long long)(r0 + r) * D0 + c8);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (r < rows && c8 + k < D0) ? a.x[(long long)(r0 + r) * D0 + c8 + k] : (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(xs + r * ldx + c8) = v;
  }
  // zero the H / dZ buffers (their padding columns are read as K padding by the next GEMM)
#pragma unroll
  for (int l = 0; l < kHeadMaxLayers; ++l)
    if (l < a.nl)
      for (int e = tid; e < HR * ld[l]; e += 64 * HW) {
        hs[l][e] = (bf16)0.f;
        dzs[l][e] = (bf16)0.f;
      }
  __syncthreads();
  HD_STAMP(1);
  // X^T [D0][ldt] for the weight gradient of layer 0: one feature's 16 rows = 32 contiguous bytes
  if (a.xT)
    for (int c = tid; c < D0; c += 64 * HW) {
      bf16x8 lo, hi;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        lo[r] = xs[r * ldx + c];
        hi[r] = xs[(r + 8) * ldx + c];
      }
      bf16* dst = a.xT + (long long)c * a.ldt + r0;
      if (rows == HR) {
        *reinterpret_cast<bf16x8*>(dst) = lo;
        *reinterpret_cast<bf16x8*>(dst + 8) = hi;
      } else {
        for (int r = 0; r < rows; ++r) dst[r] = r < 8 ? lo[r] : hi[r - 8];
      }
    }

  // ---- forward chain (layer loops unrolled: per-layer arrays stay in registers)
#pragma unroll
  for (int l = 0; l < kHeadMaxLayers; ++l) {
    if (l < a.nl) {
      const HeadLayer& L = a.L[l];
      const bf16* A = l == 0 ? xs : hs[l > 0 ? l - 1 : 0];
      const int lda = l == 0 ? ldx : ld[l > 0 ? l - 1 : 0];
      const bool last = l == a.nl - 1;
      head_gemm_fwd<13>(A, lda, L.w, L.Kpad, L.b, L.N, last ? 0 : 1, hs[l], ld[l], last ? lg : nullptr,
                        last ? nullptr : L.hT, a.ldt, r0, rows);
      __syncthreads();
      HD_STAMP(2 + l);
    }
  }

  // ---- softmax cross-entropy on the 16 logit rows (one lane per row)
  const HeadLayer& LL = a.L[a.nl - 1];
  const int C = LL.N;
  bf16* dz_last = dzs[0];
  int ld_last = ld[0];
#pragma unroll
  for (int l = 1; l < kHeadMaxLayers; ++l)
    if (l == a.nl - 1) {
      dz_last = dzs[l];
      ld_last = ld[l];
    }
  if (tid < HR) {
    const int r = tid;
    float lsum = 0.f, corr = 0.f;
    float pr[16];
    if (r < rows) {
      const long long src = a.idx ? a.idx[r0 + r] : (long long)(r0 + r);
      int y = a.labels[src < 0 ? 0 : (src >= a.nrows ? a.nrows - 1 : src)];
      y = y < 0 ? 0 : (y >= C ? C - 1 : y);
      float m = -INFINITY;
      int am = 0;
      for (int c = 0; c < C; ++c) {
        const float z = lg[r * 16 + c];
        if (a.logits) a.logits[(long long)(r0 + r) * C + c] = z;
        if (z > m) { m = z; am = c; }
      }
      float s = 0.f;
      for (int c = 0; c < C; ++c) {
        pr[c] = __expf(lg[r * 16 + c] - m);
        s += pr[c];
      }
      const float inv = 1.f / s;
      lsum = -(lg[r * 16 + y] - m - __logf(s));
      corr = am == y ? 1.f : 0.f;
      for (int c = 0; c < 16; ++c) {
        const float g = c < C ? (pr[c] * inv - (c == y ? 1.f : 0.f)) * a.grad_scale : 0.f;
        dz_last[r * ld_last + c] = f2bf(g);
        if (c < C && LL.dzT) LL.dzT[(long long)c * a.ldt + r0 + r] = f2bf(g);
      }
    }
    // block partial of [loss_sum, correct] (fixed-order tree over the 16 lanes: deterministic)
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      lsum += __shfl_xor(lsum, o, 16);
      corr += __shfl_xor(corr, o, 16);
    }
    if (tid == 0) {
      a.loss_part[2 * blockIdx.x] = lsum;
      a.loss_part[2 * blockIdx.x + 1] = corr;
    }
  }
  __syncthreads();
  HD_STAMP(6);

  // ---- backward data chain: dZ_{l-1} = (dZ_l W_l) * relu'(H_{l-1}); l = 0 produces dX
#pragma unroll
  for (int l = kHeadMaxLayers - 1; l >= 0; --l) {
    if (l < a.nl) {
      const HeadLayer& L = a.L[l];
      if (l == 0) {
        if (a.dx)
          head_gemm_bwd<4>(dzs[0], ld[0], L.wt, L.ldwt, L.K, a.x_relu ? xs : nullptr, ldx, nullptr, 0, a.dx, L.K,
                           nullptr, 0, r0, rows, a.dx_scale != 0.f ? a.dx_scale : 1.f);
      } else {
        const int lp = l > 0 ? l - 1 : 0;
        head_gemm_bwd<4>(dzs[l], ld[l], L.wt, L.ldwt, L.K, hs[lp], ld[lp], dzs[lp], ld[lp], nullptr, 0, a.L[lp].dzT,
                         a.ldt, r0, rows);
      }
      __syncthreads();
      HD_STAMP(7 + l);
    }
  }
  HD_STAMP(31);
}

// ------------------------------------------------------------------------------------------------
// dW_l[n][k] = sum_b dZ_l^T[n][b] * H_{l-1}^T[k][b]  (k < K),  db_l[n] = sum_b dZ_l^T[n][b]  (k == K)
__global__ void __launch_bounds__(1024) head_wgrad_kernel(HeadArgs a) {
  __shared__ float red[HW][16][17];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int tile = blockIdx.x;
  if (tile == a.wg_tiles) {  // loss partials -> stats: one wave, fixed-order (deterministic) tree
    if (wid == 0) {
      float l = 0.f, c = 0.f;
      for (int i = lane; i < a.nblocks; i += 64) {
        l += a.loss_part[2 * i];
        c += a.loss_part[2 * i + 1];
      }
      l = wave_sum(l);
      c = wave_sum(c);
      if (lane == 0) {
        a.stats[0] = l;
        a.stats[1] = c;
      }
    }
    return;
  }
  int l = 0;
#pragma unroll
  for (int q = 0; q < kHeadMaxLayers - 1; ++q)
    if (l == q && q < a.nl - 1 && tile >= a.L[q].tiles) {
      tile -= a.L[q].tiles;
      l = q + 1;
    }
  HeadLayer L = a.L[0];
  const bf16* hprev = a.xT;
#pragma unroll
  for (int q = 1; q < kHeadMaxLayers; ++q)
    if (l == q) {
      L = a.L[q];
      hprev = a.L[q - 1].hT;
    }
  const int ktiles = (L.K + 1 + 15) / 16;
  const int tn = tile / ktiles, tk = tile - tn * ktiles;
  const int n = 16 * tn + (lane & 15);  // A row (output channel)
  const int k = 16 * tk + (lane & 15);  // B column (input feature / bias)
  const bf16* arow = L.dzT + (long long)min(n, L.N - 1) * a.ldt + 8 * (lane >> 4);
  const bf16* brow = hprev + (long long)min(k, L.K - 1) * a.ldt + 8 * (lane >> 4);
  const bool a_ok = n < L.N, b_ones = k == L.K, b_ok = k < L.K;
  bf16x8 ones, zeros;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ones[e] = (bf16)1.f;
    zeros[e] = (bf16)0.f;
  }
  // batch k-steps (ldt = round32(B), tail columns zero) split over the 16 waves; within a wave 8
  // k-steps (16 16-byte loads) are in flight at once
  const int steps = a.ldt / 32;
  const int per = (steps + HW - 1) / HW;
  const int s0 = wid * per, s1 = min(steps, s0 + per);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < s1; s += 8) {
    bf16x8 av[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int ss = min(s + u, s1 - 1);
      av[u] = ld16(arow + 32 * ss);
      bv[u] = ld16(brow + 32 * ss);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool live = s + u < s1;
      const bf16x8 aa = (a_ok && live) ? av[u] : zeros;
      const bf16x8 bb = b_ok ? bv[u] : (b_ones ? ones : zeros);
      acc = mfma16x16x32(aa, bb, acc);
    }
  }
  // acc[r] = C[row = 4*(lane>>4)+r (n)][col = lane&15 (k)]
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wid][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 256) {
    const int rn = t >> 4, ck = t & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < HW; ++w) v += red[w][rn][ck];
    const int on = 16 * tn + rn, ok = 16 * tk + ck;
    if (on < L.N) {
      if (ok < L.K)
        L.gw[(long long)on * L.K + ok] = v;
      else if (ok == L.K && L.gb)
        L.gb[on] = v;
    }
  }
}

// ------------------------------------------------------------------------------------------------
size_t head_train_lds(const HeadArgs& a) {
  size_t bytes = round_up(HR * (a.L[0].Kpad + 8) * 2, 16);
  for (int l = 0; l < a.nl; ++l) bytes += 2 * round_up(HR * (round_up(a.L[l].N, 32) + 8) * 2, 16);
  return bytes + HR * 16 * 4;
}

static void head_prepare(HeadArgs& a) {
  a.nblocks = cdiv(a.B, HR);
  a.wg_tiles = 0;
  for (int l = 0; l < a.nl; ++l) {
    a.L[l].tiles = cdiv(a.L[l].N, 16) * cdiv(a.L[l].K + 1, 16);
    a.wg_tiles += a.L[l].tiles;
  }
}

// phase bit 1: forward + CE + backward data chain; bit 2: weight gradients + loss reduction
hipError_t head_train(HeadArgs a, int phases, hipStream_t st) {
  a.stamps = g_head_stamps;
  if (a.nl < 1 || a.nl > kHeadMaxLayers || a.L[a.nl - 1].N > 16) return hipErrorInvalidValue;
  head_prepare(a);
  if (phases & 1) {
    const size_t lds = head_train_lds(a);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(head_train_kernel, dim3(a.nblocks), dim3(64 * HW), lds, st, a);
    DFA_HIP_CHECK(hipGetLastError());
  }
  if (phases & 2) hipLaunchKernelGGL(head_wgrad_kernel, dim3(a.wg_tiles + 1), dim3(64 * HW), 0, st, a);
  return hipGetLastError();
}

}  // namespace dfa
