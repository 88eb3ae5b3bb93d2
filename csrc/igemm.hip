// Implicit-GEMM MFMA kernels (gfx950) for every dense / conv2d matmul of the training step.
//
// One kernel family covers what the reference runs through tf.js matMul / conv2d and their
// autodiff (/root/reference/src/common/models.ts:137-142):
//
//   igemm_fwd   C[m][n] = epi( sum_k A[m][k] * Wb[n][k] )
//       MODE_DIRECT  A[m][k] = src[m*lda + k]                     dense fwd / dense dgrad
//       MODE_FWD     A = im2col(src) gathered on the fly (NHWC)   conv fwd
//       MODE_DGRAD   A = transposed-conv gather of dY             conv dgrad (any stride)
//     epilogue: *alpha, +bias[n] (fp32), ReLU, ReLU-mask from the producer activation
//     (relu'(x_prev) fused into dgrad), bf16 or fp32 store.
//
//   igemm_wgrad  G[n][k] = sum_m dY[m][n] * A[m][k]  (+ bias column k==K: sum_m dY[m][n])
//     split over m into fp32 slabs (deterministic), then wgrad_reduce sums the slabs straight
//     into the flat gradient buffer that RCCL all-reduces.
//
// Tiling: 256-thread workgroups (4 waves of 64), v_mfma_f32_16x16x32_bf16, BK = 32,
// double-buffered LDS with register prefetch of the next tile (global loads of tile k+1 are in
// flight while the MFMAs of tile k run), 80-byte padded LDS rows (conflict-free ds_read_b128
// fragment reads), XCD-aware block remap so tiles sharing an A panel share an L2.
#include "common.h"
#include "kernels.h"
#include "bn_acc.h"

namespace dfa {


constexpr int BK = 32;
constexpr int LDS_ROW = BK + 8;  // bf16 elements per LDS row (80 bytes)

// Gather 8 consecutive k of one A row into a bf16x8.
// Row state: rvalid, rbase (element offset of the row's (b) image or direct row), ih0/iw0.
template <int MODE, bool VEC>
struct ALoader {
  // per-row state
  bool rvalid;
  long long rbase;
  int r0, r1;  // FWD: ih0, iw0 ; DGRAD: oh (=ih of dX), ow
  // per-chunk k state (VEC conv): kh, kw, ci of the chunk's first element
  int kh, kw, ci;

  __device__ __forceinline__ void init_row(const IGemmArgs& a, int m) {
    rvalid = m < a.M;
    int mm = rvalid ? m : 0;
    if (MODE == MODE_DIRECT) {
      rbase = (long long)mm * a.lda;
      r0 = r1 = 0;
    } else {
      const int ohw = a.OH * a.OW;
      const int b = mm / ohw;
      const int rem = mm - b * ohw;
      const int oh = rem / a.OW;
      const int ow = rem - oh * a.OW;
      rbase = (long long)b * a.SH * a.SW * a.SC;
      if (MODE == MODE_FWD) {
        r0 = oh * a.stride - a.pad;
        r1 = ow * a.stride_w - a.pad_w;
      } else {
        r0 = oh + a.pad;
        r1 = ow + a.pad_w;
      }
    }
  }
  __device__ __forceinline__ void init_k(const IGemmArgs& a, int k) {
    if (MODE != MODE_DIRECT && VEC) {
      ci = k % a.SC;
      const int t = k / a.SC;
      kh = t / a.KW;
      kw = t - kh * a.KW;
    }
  }
  __device__ __forceinline__ void advance_k(const IGemmArgs& a) {
    if (MODE != MODE_DIRECT && VEC) {
      ci += BK;
      while (ci >= a.SC) {
        ci -= a.SC;
        if (++kw == a.KW) { kw = 0; ++kh; }
      }
    }
  }
  // Source element offset of (row, kh, kw, ci) or -1 when outside the image / not on stride.
  __device__ __forceinline__ long long conv_off(const IGemmArgs& a, int kh_, int kw_, int ci_) const {
    int sh, sw;
    if (MODE == MODE_FWD) {
      sh = r0 + kh_;
      sw = r1 + kw_;
    } else {  // DGRAD: dX(ih,iw) <- dY((ih+pad-kh)/s, (iw+pad-kw)/s)
      int th = r0 - kh_, tw = r1 - kw_;
      if (th < 0 || tw < 0) return -1;
      if ((a.stride | a.stride_w) > 1) {
        if ((th % a.stride) | (tw % a.stride_w)) return -1;
        th /= a.stride;
        tw /= a.stride_w;
      }
      sh = th;
      sw = tw;
    }
    if ((unsigned)sh >= (unsigned)a.SH || (unsigned)sw >= (unsigned)a.SW) return -1;
    return rbase + ((long long)sh * a.SW + sw) * a.SC + ci_;
  }
  // k = first k of the chunk; lut = packed (kh<<24|kw<<16|ci) table for non-VEC conv modes
  __device__ __forceinline__ bf16x8 load(const IGemmArgs& a, int k, const int* lut) const {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)0.0f;
    if (!rvalid) return v;
    if (MODE == MODE_DIRECT) {
      if (VEC) {
        if (k < a.K) v = *reinterpret_cast<const bf16x8*>(a.src + rbase + k);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k + j < a.K) v[j] = a.src[rbase + k + j];
      }
    } else if (VEC) {
      if (kh < a.KH) {
        const long long off = conv_off(a, kh, kw, ci);
        if (off >= 0) v = *reinterpret_cast<const bf16x8*>(a.src + off);
      }
    } else {
      // every element load unconditional (invalid ones read element 0 and are zeroed): a load under a
      // per-element condition compiled to an exec-mask branch and a wait per element
      bf16 x[8];
      bool ok[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool kok = k + j < a.K;
        const int e = lut[kok ? k + j : 0];
        const long long off = conv_off(a, e >> 24, (e >> 16) & 0xff, e & 0xffff);
        ok[j] = kok && off >= 0;
        x[j] = a.src[ok[j] ? off : 0];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = ok[j] ? x[j] : (bf16)0.0f;
    }
    return v;
  }
};

template <int BM, int BN, int WM, int WN, int MODE, bool VEC>
__global__ void __launch_bounds__(256) igemm_fwd_kernel(IGemmArgs a) {
  constexpr int TM = BM / (WM * 16);
  constexpr int TN = BN / (WN * 16);
  constexpr int A_CHUNKS = BM * (BK / 8);           // 16-byte chunks per A tile
  constexpr int B_CHUNKS = BN * (BK / 8);
  constexpr int A_PER_T = (A_CHUNKS + 255) / 256;
  constexpr int B_PER_T = (B_CHUNKS + 255) / 256;
  static_assert(WM * WN == 4, "4 waves");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);                       // [2][BM][LDS_ROW]
  bf16* Bs = As + 2 * BM * LDS_ROW;                               // [2][BN][LDS_ROW]
  int* lut = reinterpret_cast<int*>(Bs + 2 * BN * LDS_ROW);       // [Kpad] (non-VEC conv)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  const int ntn = cdiv(a.N, BN);
  const int ntm = cdiv(a.M, BM);
  const int logical = xcd_remap(blockIdx.x, ntn * ntm);
  const int tile_n = logical % ntn;
  const int tile_m = logical / ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  if (MODE != MODE_DIRECT && !VEC) {
    for (int k = tid; k < a.K; k += 256) {
      const int ci = k % a.SC;
      const int t = k / a.SC;
      const int kh = t / a.KW;
      const int kw = t - kh * a.KW;
      lut[k] = (kh << 24) | (kw << 16) | ci;
    }
    __syncthreads();
  }

  ALoader<MODE, VEC> ald[A_PER_T];
  int a_row[A_PER_T], a_kc[A_PER_T];
#pragma unroll
  for (int i = 0; i < A_PER_T; ++i) {
    const int c = tid + 256 * i;
    a_row[i] = c >> 2;
    a_kc[i] = (c & 3) * 8;
    ald[i].init_row(a, m0 + a_row[i]);
    ald[i].init_k(a, a_kc[i]);
  }

  const int nk = cdiv(a.K, BK);
  bf16x8 ra[A_PER_T], rb[B_PER_T];

  auto gload = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      if (A_CHUNKS % 256 == 0 || tid + 256 * i < A_CHUNKS) ra[i] = ald[i].load(a, k0 + a_kc[i], lut);
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int c = tid + 256 * i;
      if (B_CHUNKS % 256 == 0 || c < B_CHUNKS) {
        const int n = n0 + (c >> 2);
        // weights are zero padded to [Npad16][Kpad32]: rows >= Npad are never touched because
        // BN tiles past Npad are clamped by the N check below.
        if (n < round_up(a.N, 16))
          rb[i] = *reinterpret_cast<const bf16x8*>(a.w + (long long)n * a.Kpad + k0 + (c & 3) * 8);
        else {
#pragma unroll
          for (int j = 0; j < 8; ++j) rb[i][j] = (bf16)0.0f;
        }
      }
    }
  };
  auto sstore = [&](int buf) {
    bf16* as = As + buf * BM * LDS_ROW;
    bf16* bs = Bs + buf * BN * LDS_ROW;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i)
      if (A_CHUNKS % 256 == 0 || tid + 256 * i < A_CHUNKS)
        *reinterpret_cast<bf16x8*>(as + a_row[i] * LDS_ROW + a_kc[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int c = tid + 256 * i;
      if (B_CHUNKS % 256 == 0 || c < B_CHUNKS)
        *reinterpret_cast<bf16x8*>(bs + (c >> 2) * LDS_ROW + (c & 3) * 8) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  sstore(0);
  __syncthreads();

  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
#pragma unroll
      for (int i = 0; i < A_PER_T; ++i) ald[i].advance_k(a);
      gload(kt + 1);
    }
    const bf16* as = As + cur * BM * LDS_ROW;
    const bf16* bs = Bs + cur * BN * LDS_ROW;
    bf16x8 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
      fa[i] = *reinterpret_cast<const bf16x8*>(as + (wm * TM * 16 + i * 16 + frow) * LDS_ROW + fk);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(bs + (wn * TN * 16 + j * 16 + frow) * LDS_ROW + fk);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fa[i], fb[j], acc[i][j]);
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: C/D layout of 16x16 MFMA: col = lane&15, row = 4*(lane>>4) + r
  // (with a.bacc: forward BatchNorm sums of the stored values, csrc/bn_acc.h -- one channel per lane
  // here, so the lanes of a channel are l, l ^ 16, l ^ 32, l ^ 48, then the WM wave rows via LDS)
  const bool bacc = a.bacc.acc != nullptr;
  float* red = reinterpret_cast<float*>(smem);
  if (bacc) __syncthreads();  // LDS is free after the k loop
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    float bs = 0.f, bq = 0.f;
    const int col = n0 + wn * TN * 16 + j * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (col >= a.N) continue;
      const float bv = a.bias ? a.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * TM * 16 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r] * a.alpha + bv;
        const long long o = (long long)row * a.ldc + col;
        if (a.res) {
          const float rv = (float)a.res[o];
          if (!a.resmask || (float)a.resmask[o] > 0.f) v += rv;
        }
        if (a.relu) v = fmaxf(v, 0.f);
        if (a.mask && !((float)a.mask[o] > 0.f)) v = 0.f;
        if (a.out_f32) {
          reinterpret_cast<float*>(a.out)[o] = v;
        } else {
          const bf16 ob = f2bf(v);
          reinterpret_cast<bf16*>(a.out)[o] = ob;
          const float sv = (float)ob;
          bs += sv;
          bq += sv * sv;
        }
      }
    }
    if (bacc) {
      bs += __shfl_xor(bs, 16);
      bq += __shfl_xor(bq, 16);
      bs += __shfl_xor(bs, 32);
      bq += __shfl_xor(bq, 32);
      if (lane < 16) {
        float* p = red + ((long long)wm * BN + wn * TN * 16 + j * 16 + lane) * 3;
        p[0] = bs;
        p[1] = bq;
        p[2] = 0.f;
      }
    }
  }
  if (bacc) {
    __syncthreads();
    bacc_flush(a.bacc, red, WM, BN, n0, a.N, tid, 256);
  }
}

// ------------------------------------------------------------------------------------------
// Weight gradient: G[n][k] = sum_m dY[m][n] * A[m][k]; k == K is the bias column (A = 1).
template <int BN, int BKO, int WN, int WK, int MODE, bool DVEC, bool XVEC>
__global__ void __launch_bounds__(256) igemm_wgrad_kernel(WgradArgs a) {
  constexpr int TN = BN / (WN * 16);
  constexpr int TK = BKO / (WK * 16);
  static_assert(WN * WK == 4, "4 waves");
  constexpr int RS = 32 + 8;                  // LDS row stride (m elements, 80 bytes)
  __shared__ __attribute__((aligned(16))) bf16 Ds[2][BN * RS];   // [n][m]  (dY transposed)
  __shared__ __attribute__((aligned(16))) bf16 Xs[2][BKO * RS];  // [k][m]  (im2col transposed)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid / WK, wk = wid % WK;
  const int Kt = a.K + (a.with_bias ? 1 : 0);
  const int ntn = cdiv(a.N, BN), ntk = cdiv(Kt, BKO);
  const int ntiles = ntn * ntk;
  const int logical = xcd_remap(blockIdx.x, ntiles * a.splits);
  const int split = logical % a.splits;
  const int tile = logical / a.splits;
  const int tn = tile / ntk, tk = tile % ntk;
  const int n0 = tn * BN, k0 = tk * BKO;
  const int mb = split * a.m_per_split;
  const int me = min(a.M, mb + a.m_per_split);

  // thread -> (m, chunk): m fastest so the transposed LDS writes of a wave are contiguous
  const int mm = tid & 31;
  const int chunk = tid >> 5;  // 0..7
  constexpr int DCH = BN / 8, XCH = BKO / 8;
  constexpr int D_PER_T = (DCH + 7) / 8, X_PER_T = (XCH + 7) / 8;

  // per-thread im2col column decomposition, fixed over the whole m loop:
  // packed (kh<<24 | kw<<16 | ci), -1 = past K (zero), -2 = bias column (one)
  int xe[X_PER_T][8];
#pragma unroll
  for (int i = 0; i < X_PER_T; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = k0 + (chunk + 8 * i) * 8 + j;
      int e = -1;
      if (kk < a.K) {
        if (MODE == MODE_DIRECT) {
          e = kk;
        } else {
          const int ci = kk % a.SC;
          const int t = kk / a.SC;
          const int kh = t / a.KW;
          e = (kh << 24) | ((t - kh * a.KW) << 16) | ci;
        }
      } else if (kk == a.K && a.with_bias) {
        e = -2;
      }
      xe[i][j] = e;
    }

  bf16x8 rd[D_PER_T], rx[X_PER_T];
  auto gload = [&](int mstart) {
    const int m = mstart + mm;
    const bool mv = m < me;
#pragma unroll
    for (int i = 0; i < D_PER_T; ++i) {
      const int c = chunk + 8 * i;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)0.f;
      if (c < DCH && mv) {
        const int n = n0 + c * 8;
        const bf16* p = a.dy + (long long)m * a.ldd + n;
        if (DVEC && n + 8 <= a.N) {
          v = *reinterpret_cast<const bf16x8*>(p);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (n + j < a.N) v[j] = p[j];
        }
      }
      rd[i] = v;
    }
    int r0 = 0, r1 = 0;
    long long img = 0;
    if (MODE != MODE_DIRECT && mv) {
      const int ohw = a.OH * a.OW;
      const int b = m / ohw;
      const int rem = m - b * ohw;
      const int oh = rem / a.OW;
      const int ow = rem - oh * a.OW;
      r0 = oh * a.stride - a.pad;
      r1 = ow * a.stride_w - a.pad_w;
      img = (long long)b * a.SH * a.SW * a.SC;
    }
#pragma unroll
    for (int i = 0; i < X_PER_T; ++i) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)0.f;
      if (chunk + 8 * i < XCH && mv) {
        if (MODE == MODE_DIRECT) {
          const bf16* p = a.src + (long long)m * a.lda;
          if (XVEC && xe[i][7] >= 0) {
            v = *reinterpret_cast<const bf16x8*>(p + xe[i][0]);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (xe[i][j] >= 0) v[j] = p[xe[i][j]];
          }
        } else if (XVEC && xe[i][7] >= 0) {
          const int e = xe[i][0];
          const int sh = r0 + (e >> 24), sw = r1 + ((e >> 16) & 0xff);
          if ((unsigned)sh < (unsigned)a.SH && (unsigned)sw < (unsigned)a.SW)
            v = *reinterpret_cast<const bf16x8*>(a.src + img + ((long long)sh * a.SW + sw) * a.SC + (e & 0xffff));
        } else {
          // every element load unconditional (invalid ones read element 0 and are zeroed): a load under
          // a per-element condition compiled to an exec-mask branch and a wait per element
          bf16 xv[8];
          bool ok[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int e = xe[i][j];
            const int sh = r0 + ((e >> 24) & 0xff), sw = r1 + ((e >> 16) & 0xff);
            ok[j] = e >= 0 && (unsigned)sh < (unsigned)a.SH && (unsigned)sw < (unsigned)a.SW;
            xv[j] = a.src[ok[j] ? img + ((long long)sh * a.SW + sw) * a.SC + (e & 0xffff) : 0];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = ok[j] ? xv[j] : (bf16)0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (xe[i][j] == -2) v[j] = (bf16)1.0f;
      }
      rx[i] = v;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < D_PER_T; ++i) {
      const int c = chunk + 8 * i;
      if (c < DCH) {
#pragma unroll
        for (int j = 0; j < 8; ++j) Ds[buf][(c * 8 + j) * RS + mm] = rd[i][j];
      }
    }
#pragma unroll
    for (int i = 0; i < X_PER_T; ++i) {
      const int c = chunk + 8 * i;
      if (c < XCH) {
#pragma unroll
        for (int j = 0; j < 8; ++j) Xs[buf][(c * 8 + j) * RS + mm] = rx[i][j];
      }
    }
  };

  f32x4 acc[TN][TK];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = me > mb ? cdiv(me - mb, 32) : 0;
  if (nsteps > 0) {
    gload(mb);
    sstore(0);
  }
  __syncthreads();
  const int frow = lane & 15, fk = (lane >> 4) * 8;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) gload(mb + (s + 1) * 32);
    bf16x8 fa[TN], fb[TK];
#pragma unroll
    for (int i = 0; i < TN; ++i)
      fa[i] = *reinterpret_cast<const bf16x8*>(&Ds[cur][(wn * TN * 16 + i * 16 + frow) * RS + fk]);
#pragma unroll
    for (int j = 0; j < TK; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(&Xs[cur][(wk * TK * 16 + j * 16 + frow) * RS + fk]);
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TK; ++j) acc[i][j] = mfma16x16x32(fa[i], fb[j], acc[i][j]);
    if (s + 1 < nsteps) sstore(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TN; ++i) {
#pragma unroll
    for (int j = 0; j < TK; ++j) {
      const int k = k0 + wk * TK * 16 + j * 16 + (lane & 15);
      if (k >= Kt) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * TN * 16 + i * 16 + (lane >> 4) * 4 + r;
        if (n >= a.N) continue;
        const float v = acc[i][j][r];
        if (a.splits > 1) {
          a.partial[((long long)split * a.N + n) * Kt + k] = v;
        } else if (k < a.K) {
          a.gw[(long long)n * a.K + k] = v * a.scale;
        } else {
          a.gb[n] = v * a.scale;
        }
      }
    }
  }
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ partial, float* __restrict__ gw,
                                    float* __restrict__ gb, int N, int K, int Kt, int splits,
                                    float scale) {
  const int total = N * Kt;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < splits; ++p) s += partial[(long long)p * total + idx];
    const int n = idx / Kt, k = idx - n * Kt;
    if (k < K)
      gw[(long long)n * K + k] = s * scale;
    else
      gb[n] = s * scale;
  }
}

// ------------------------------------------------------------------------------------------
// host launchers
template <int BM, int BN, int WM, int WN, int MODE, bool VEC>
static hipError_t launch_fwd_cfg(const IGemmArgs& a, hipStream_t st) {
  const int blocks = cdiv(a.M, BM) * cdiv(a.N, BN);
  size_t lds = (size_t)2 * (BM + BN) * LDS_ROW * sizeof(bf16);
  if (MODE != MODE_DIRECT && !VEC) lds += (size_t)a.Kpad * sizeof(int);
  hipLaunchKernelGGL((igemm_fwd_kernel<BM, BN, WM, WN, MODE, VEC>), dim3(blocks), dim3(256), lds, st, a);
  return hipGetLastError();
}

template <int MODE, bool VEC>
static hipError_t launch_fwd_mode(const IGemmArgs& a, hipStream_t st) {
  // Tile choice: N fits one tile where possible; shrink BM when M alone cannot fill 256 CUs.
  const bool small_m = cdiv(a.M, 128) < 512;
  if (a.N <= 16) {
    if (small_m) return launch_fwd_cfg<64, 16, 4, 1, MODE, VEC>(a, st);
    return launch_fwd_cfg<128, 16, 4, 1, MODE, VEC>(a, st);
  }
  if (a.N <= 32) {
    if (small_m) return launch_fwd_cfg<64, 32, 4, 1, MODE, VEC>(a, st);
    return launch_fwd_cfg<128, 32, 4, 1, MODE, VEC>(a, st);
  }
  if (a.N <= 64) {
    if (small_m) return launch_fwd_cfg<64, 64, 2, 2, MODE, VEC>(a, st);
    return launch_fwd_cfg<128, 64, 2, 2, MODE, VEC>(a, st);
  }
  if (small_m) return launch_fwd_cfg<64, 128, 1, 4, MODE, VEC>(a, st);
  return launch_fwd_cfg<128, 128, 2, 2, MODE, VEC>(a, st);
}

static hipError_t igemm_fwd_nodrop(const IGemmArgs& a, int mode, hipStream_t st);

// Can this igemm_fwd call accumulate BatchNorm sums of its output (a.bacc, csrc/bn_acc.h)?  The halo and
// igemm64 kernels (and their split-K combine) in both modes, with the vectorised bf16 epilogue; the
// generic kernel the forward sums only.
bool igemm_bacc_ok(const IGemmArgs& a, int mode) {
  if (mode == MODE_DIRECT || a.out_f32 || a.drop.on || a.pool_code || a.bn.part || a.M <= 0 || a.N <= 0) return false;
  if (a.bacc.nrep < 1 || a.bacc.nrep > kBnAccMaxRep || (a.bacc.mode == 1 && (!a.bacc.x || !a.bacc.mean))) return false;
  if (a.bacc.acc2 && (a.bacc.mode != 1 || !a.bacc.x2 || !a.bacc.mean2)) return false;
  if (!a.irregular && (conv3_halo_supported(a, mode) || igemm64_supported(a, mode))) {
    if ((a.ldc & 3) || (a.N & 3) || ((uintptr_t)a.out & 15) ||
        (((uintptr_t)a.res | (uintptr_t)a.resmask | (uintptr_t)a.mask | (uintptr_t)a.bacc.x | (uintptr_t)a.bacc.x2) & 7))
      return false;
    return a.N <= 1024 && 256 % (a.N / 4) == 0;  // (a split-K combine may apply the epilogue)
  }
  return mode == MODE_FWD && a.bacc.mode == 0 && (a.irregular || !smallc_fwd_supported(a, mode));
}

hipError_t igemm_fwd(const IGemmArgs& a, int mode, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0) return hipSuccess;
  if (a.bacc.acc && !igemm_bacc_ok(a, mode)) return hipErrorInvalidValue;
  if (a.drop.on && (a.out_f32 || a.ldc != a.N)) return hipErrorInvalidValue;
  if (a.irregular && (a.pool_code || a.bn.part)) return hipErrorInvalidValue;
  if (a.pool_code) return igemm64_pool_supported(a) && mode == MODE_FWD ? igemm64(a, mode, st) : hipErrorInvalidValue;
  if (!a.irregular && conv3_halo_supported(a, mode)) return conv3_halo(a, mode, st);
  if (!a.irregular && igemm64_supported(a, mode)) return igemm64(a, mode, st);  // dropout in its epilogues
  if (!a.drop.on) return igemm_fwd_nodrop(a, mode, st);
  IGemmArgs b = a;
  b.drop = DropSpec{};
  DFA_HIP_CHECK(igemm_fwd_nodrop(b, mode, st));
  bf16* o = reinterpret_cast<bf16*>(a.out);
  return dropout(o, o, nullptr, (long long)a.M * a.N, a.drop.p, a.drop.seed, a.drop.step, st);
}

static hipError_t igemm_fwd_nodrop(const IGemmArgs& a, int mode, hipStream_t st) {
  if (!a.irregular && smallc_fwd_supported(a, mode)) return smallc_fwd(a, st);
  const bool aligned = ((uintptr_t)a.src & 15) == 0;
  if (mode == MODE_DIRECT) {
    const bool vec = aligned && a.lda % 8 == 0 && a.K % 8 == 0;
    return vec ? launch_fwd_mode<MODE_DIRECT, true>(a, st) : launch_fwd_mode<MODE_DIRECT, false>(a, st);
  }
  const bool vec = aligned && a.SC % 8 == 0;
  if (mode == MODE_FWD)
    return vec ? launch_fwd_mode<MODE_FWD, true>(a, st) : launch_fwd_mode<MODE_FWD, false>(a, st);
  return vec ? launch_fwd_mode<MODE_DGRAD, true>(a, st) : launch_fwd_mode<MODE_DGRAD, false>(a, st);
}

template <int BN, int BKO, int WN, int WK, int MODE, bool DVEC, bool XVEC>
static hipError_t launch_wgrad_cfg(WgradArgs a, float* workspace, size_t ws_floats, hipStream_t st) {
  const int Kt = a.K + (a.with_bias ? 1 : 0);
  const int tiles = cdiv(a.N, BN) * cdiv(Kt, BKO);
  // enough splits to put ~2 workgroups on each of the 256 CUs, each reducing >= 128 rows
  int splits = cdiv(512, tiles);
  splits = min(splits, cdiv(a.M, 128));
  splits = max(splits, 1);
  while (splits > 1 && (size_t)splits * a.N * Kt > ws_floats) --splits;
  a.m_per_split = round_up(cdiv(a.M, splits), 32);
  splits = cdiv(a.M, a.m_per_split);
  a.splits = splits;
  a.partial = workspace;
  hipLaunchKernelGGL((igemm_wgrad_kernel<BN, BKO, WN, WK, MODE, DVEC, XVEC>), dim3(tiles * splits), dim3(256), 0,
                     st, a);
  DFA_HIP_CHECK(hipGetLastError());
  if (splits > 1) DFA_HIP_CHECK(slab_reduce(workspace, a.gw, a.gb, a.N, a.K, Kt, splits, a.scale, st));
  return hipSuccess;
}

template <int MODE, bool DVEC, bool XVEC>
static hipError_t launch_wgrad_mode(const WgradArgs& a, float* ws, size_t wsf, hipStream_t st) {
  if (a.N <= 16) return launch_wgrad_cfg<16, 64, 1, 4, MODE, DVEC, XVEC>(a, ws, wsf, st);
  if (a.N <= 32) return launch_wgrad_cfg<32, 64, 2, 2, MODE, DVEC, XVEC>(a, ws, wsf, st);
  return launch_wgrad_cfg<64, 64, 2, 2, MODE, DVEC, XVEC>(a, ws, wsf, st);
}

template <int MODE>
static hipError_t launch_wgrad_x(const WgradArgs& a, bool dvec, bool xvec, float* ws, size_t wsf, hipStream_t st) {
  if (dvec) {
    return xvec ? launch_wgrad_mode<MODE, true, true>(a, ws, wsf, st) : launch_wgrad_mode<MODE, true, false>(a, ws, wsf, st);
  }
  return xvec ? launch_wgrad_mode<MODE, false, true>(a, ws, wsf, st) : launch_wgrad_mode<MODE, false, false>(a, ws, wsf, st);
}

hipError_t igemm_wgrad(const WgradArgs& a, int mode, float* workspace, size_t ws_floats, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0) return hipSuccess;
  const bool dvec = ((uintptr_t)a.dy & 15) == 0 && a.ldd % 8 == 0;
  if (mode == MODE_DIRECT) {
    const bool xvec = ((uintptr_t)a.src & 15) == 0 && a.lda % 8 == 0;
    return launch_wgrad_x<MODE_DIRECT>(a, dvec, xvec, workspace, ws_floats, st);
  }
  if (!a.irregular) {
    if (wgrad_halo_supported(a, mode)) return wgrad_halo(a, workspace, ws_floats, st);
    if (wgrad_tr_supported(a, mode)) return wgrad_tr(a, workspace, ws_floats, st);
    if (smallc_wgrad_supported(a, mode)) return smallc_wgrad(a, workspace, ws_floats, st);
  }
  const bool xvec = ((uintptr_t)a.src & 15) == 0 && a.SC % 8 == 0;
  return launch_wgrad_x<MODE_FWD>(a, dvec, xvec, workspace, ws_floats, st);
}

}  // namespace dfa
