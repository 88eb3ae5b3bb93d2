// Convolution weight gradient with hardware-transposed LDS reads (gfx950 ds_read_b64_tr_b16).
//
// G[n][k] = sum_m dY[m][n] * X[m][k] over m = (b, oh, ow) — the conv2d backprop-filter of the
// reference's tf.variableGrads (/root/reference/src/common/models.ts:137-142).
// Both operands are m-major in HBM (dY is NHWC [M][N]; the im2col row of a pixel is
// [KH][KW][C]) while a 16x16x32 MFMA fragment wants 8 consecutive m per lane.  Tiles are staged
// row-major with 16-byte global loads and 16-byte LDS stores, and every fragment is two
// ds_read_b64_tr_b16, which transpose a 4-row x 16-column block per 16-lane group inside the LDS
// read.  (igemm.hip's generic wgrad transposes with eight 2-byte LDS stores per chunk.)
//
//   * workgroup = BN x BK output tile, 4 waves as WN x WK, m-steps of 64 rows, two LDS buffers and a
//     2-step register prefetch (inline-asm loads, hand-counted vmcnt), one barrier per step
//   * m is split over workgroups (split-m); slab_reduce sums the slabs in a fixed order
//   * a conv bias gradient is one more k chunk whose first element reads 1.0 (column K of G)
//   * LDS row stride = 8 x odd dwords (mod 64): the 8 rows one 32-lane half reads with a
//     transposed read sit on 8 disjoint 8-bank groups (conflict-free), and 8 lanes storing the 8
//     consecutive 16-byte chunks of a row cover the 32 store banks once
//   * the MFMA k slots may take the m rows in any order as long as both operands agree: slot
//     8g + 4h + q of a lane in group g is row 16h + 4g + q of the 32-row half step, which is what
//     makes the row blocks of one transposed read contiguous
//   * a thread's k chunk (kh, kw, ci) is fixed for the whole launch; per step only the pixel
//     decomposition (multiply-high division by OW and OH*OW) is recomputed; out-of-image taps and
//     tails read a 16-byte zero constant instead (address select: no load under a branch)
#include "common.h"
#include "kernels.h"
#include "diag.h"

namespace dfa {

namespace {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_vs __attribute__((__vector_size__(8)));

__device__ __forceinline__ bf16x4 tr_read(const bf16* p) {
  auto* lp = (__attribute__((address_space(3))) bf16*)(const_cast<bf16*>(p));
  const bf16x4_vs v =
      __builtin_amdgcn_ds_read_tr16_b64_v4bf16(reinterpret_cast<__attribute__((address_space(3))) bf16x4_vs*>(lp));
  return __builtin_bit_cast(bf16x4, v);
}

constexpr int tr_stride(int cols) { return cols + (((cols / 16) % 2) ? 0 : 16); }

__device__ u32x4_t kZeroTr16 = {0u, 0u, 0u, 0u};  // source of every masked-out 16-byte chunk
// bias gradient = column of ones appended to X at k = K (bf16 1.0 = 0x3F80 in element 0 of the chunk)
__device__ u32x4_t kOneTr16 = {0x3F80u, 0u, 0u, 0u};

// Operand loads from inline asm with hand-counted waits (see igemm64.hip: hipcc's loop-carried
// vmcnt waits otherwise collapse the register prefetch to one step).
__device__ __forceinline__ u32x4_t gload16_tr(const void* p) {
  u32x4_t r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

constexpr int kWgradStages = 2;  // register prefetch depth (m-steps in flight)

// workgroups per CU the LDS allows (2 x 64 rows x (SN + SK) bf16 each): register cap to match
// (capped at MAXOCC: the register budget of MAXOCC workgroups must hold the kernel without spills)
template <int BN, int BK, int BM = 64, int MAXOCC = 4>
constexpr int wgrad_tr_occ() {
  return (160 * 1024) / (2 * BM * (tr_stride(BN) + tr_stride(BK)) * 2) > MAXOCC
             ? MAXOCC
             : (160 * 1024) / (2 * BM * (tr_stride(BN) + tr_stride(BK)) * 2);
}

template <int BN, int BK, int WN, int WK, int BM = 64, int MAXOCC = 4>
__global__ void __launch_bounds__(256, (wgrad_tr_occ<BN, BK, BM, MAXOCC>())) wgrad_tr_kernel(WgradArgs a, FastDiv d_ow, FastDiv d_ohw) {
  constexpr int D = kWgradStages;
  constexpr int SN = tr_stride(BN), SK = tr_stride(BK);
  constexpr int TN = BN / (WN * 16), TK = BK / (WK * 16);
  constexpr int DC = BN / 8, XC = BK / 8;      // 16-byte chunks per tile row
  constexpr int DR = 256 / DC, XR = 256 / XC;  // rows per load pass
  constexpr int DP = BM / DR, XP = BM / XR;    // load passes per step
  static_assert(WN * WK == 4 && 256 % DC == 0 && 256 % XC == 0 && DP >= 1 && XP >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * BM * (SN + SK)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid / WK, wk = wid % WK;
  const int Kt = a.K + (a.with_bias ? 1 : 0);   // output columns (bias gradient = column K)
  const int ntk = cdiv(a.K + (a.with_bias ? 8 : 0), BK);
  const int ntiles = cdiv(a.N, BN) * ntk;
  // tile fastest: the workgroups an XCD runs together share one m range (the same dY / X rows)
  const int logical = xcd_remap(blockIdx.x, ntiles * a.splits);
  const int tile = logical % ntiles, split = logical / ntiles;
  const int n0 = (tile / ntk) * BN, k0 = (tile % ntk) * BK;
  const int mb = split * a.m_per_split;
  const int me = min(a.M, mb + a.m_per_split);

  const int dc = tid % DC, dr = tid / DC;
  const int nn = n0 + dc * 8;
  const bool nval = nn < a.N;
  const int xc = tid % XC, xr = tid / XC;
  const int kk = k0 + xc * 8;
  const bool kval = kk < a.K;
  const bool kbias = a.with_bias && kk == a.K;
  int kh = 0, kw = 0, ci = 0;
  if (kval) {
    ci = kk % a.SC;
    const int t = kk / a.SC;
    kh = t / a.KW;
    kw = t - kh * a.KW;
  }
  const unsigned ohw = (unsigned)(a.OH * a.OW);

  u32x4_t rd[D][DP], rx[D][XP];
  auto gload = [&](int st, int m0) {
#pragma unroll
    for (int i = 0; i < DP; ++i) {
      const int m = m0 + dr + i * DR;
      const bool v = nval && m < me;
      rd[st][i] = gload16_tr(v ? (const void*)(a.dy + (long long)m * a.ldd + nn) : (const void*)&kZeroTr16);
    }
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int m = m0 + xr + i * XR;
      const unsigned mm = (unsigned)min(m, a.M - 1);
      const unsigned b = fdiv(mm, d_ohw);
      const unsigned rem = mm - b * ohw;
      const unsigned oh = fdiv(rem, d_ow);
      const int ow = (int)(rem - oh * (unsigned)a.OW);
      const int ih = (int)oh * a.stride - a.pad + kh;
      const int iw = ow * a.stride - a.pad + kw;
      const bool v = kval && m < me && (unsigned)ih < (unsigned)a.SH && (unsigned)iw < (unsigned)a.SW;
      rx[st][i] = gload16_tr(v ? (const void*)(a.src + (((long long)b * a.SH + ih) * a.SW + iw) * a.SC + ci)
                               : (kbias && m < me) ? (const void*)&kOneTr16 : (const void*)&kZeroTr16);
    }
  };
  auto sstore = [&](int buf, int st) {
    bf16* ds = lds + buf * BM * SN;
    bf16* xs = lds + 2 * BM * SN + buf * BM * SK;
#pragma unroll
    for (int i = 0; i < DP; ++i) *reinterpret_cast<u32x4_t*>(ds + (dr + i * DR) * SN + dc * 8) = rd[st][i];
#pragma unroll
    for (int i = 0; i < XP; ++i) *reinterpret_cast<u32x4_t*>(xs + (xr + i * XR) * SK + xc * 8) = rx[st][i];
  };

  f32x4 acc[TN][TK];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane address: lane 4q+p of group g supplies row (4g + q), columns 4p..4p+3
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int dro = (4 * g + q) * SN + 4 * p + wn * (BN / WN);
  const int xro = (4 * g + q) * SK + 4 * p + wk * (BK / WK);
  const int nsteps = me > mb ? cdiv(me - mb, BM) : 0;
  // prologue: step 0 -> LDS[0]; steps 1..D in flight (register stage of step s = s % D)
  if (nsteps > 0) {
    gload(0, mb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sstore(0, 0);
#pragma unroll
    for (int s = 1; s <= D; ++s)
      if (s < nsteps) gload(s % D, mb + s * BM);
  }
  __syncthreads();
  for (int sb = 0; sb < nsteps; sb += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int s = sb + u;
      if (s < nsteps) {
        const int cur = s & 1;
        const bf16* ds = lds + cur * BM * SN + dro;
        const bf16* xs = lds + 2 * BM * SN + cur * BM * SK + xro;
#pragma unroll
        for (int sub = 0; sub < BM / 32; ++sub) {
          bf16x8 fa[TN], fb[TK];
#pragma unroll
          for (int i = 0; i < TN; ++i) {
            const bf16x4 lo = tr_read(ds + sub * 32 * SN + i * 16);
            const bf16x4 hi = tr_read(ds + (sub * 32 + 16) * SN + i * 16);
            fa[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
#pragma unroll
          for (int j = 0; j < TK; ++j) {
            const bf16x4 lo = tr_read(xs + sub * 32 * SK + j * 16);
            const bf16x4 hi = tr_read(xs + (sub * 32 + 16) * SK + j * 16);
            fb[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
#pragma unroll
          for (int i = 0; i < TN; ++i)
#pragma unroll
            for (int j = 0; j < TK; ++j) acc[i][j] = mfma16x16x32(fa[i], fb[j], acc[i][j]);
        }
        const int nst = (u + 1) % D;  // register stage holding step s + 1
        if (s + 1 < nsteps) {
          if (s + D < nsteps)
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"((DP + XP) * (D - 1)) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          sstore(cur ^ 1, nst);
        }
        __syncthreads();
        if (s + 1 + D < nsteps) gload(nst, mb + (s + 1 + D) * BM);
      }
    }
  }

  // C/D layout of the 16x16 MFMA: column (k) = lane & 15, row (n) = 4 * (lane >> 4) + r
  const int li = lane & 15;
#pragma unroll
  for (int i = 0; i < TN; ++i) {
#pragma unroll
    for (int j = 0; j < TK; ++j) {
      const int k = k0 + wk * (BK / WK) + j * 16 + li;
      if (k >= Kt) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * (BN / WN) + i * 16 + 4 * g + r;
        if (n >= a.N) continue;
        if (a.splits > 1)
          a.partial[((long long)split * a.N + n) * Kt + k] = acc[i][j][r];
        else if (k < a.K)
          a.gw[(long long)n * a.K + k] = acc[i][j][r] * a.scale;
        else
          a.gb[n] = acc[i][j][r] * a.scale;
      }
    }
  }
}

template <int BN, int BK, int WN, int WK, int BM = 64, int MAXOCC = 4>
hipError_t launch_wgrad_tr(WgradArgs a, float* ws, size_t ws_floats, hipStream_t st) {
  const int Kt = a.K + (a.with_bias ? 1 : 0);
  const int tiles = cdiv(a.N, BN) * cdiv(a.K + (a.with_bias ? 8 : 0), BK);
  // about two workgroups per CU (73.7 KB of LDS each at BM = 64), each reducing >= 256 rows
  static const int target = diag_int("wgrad_wg", 512);
  int splits = cdiv(target, tiles);
  splits = min(splits, cdiv(a.M, 256));
  splits = max(splits, 1);
  while (splits > 1 && (size_t)splits * a.N * Kt > ws_floats) --splits;
  a.m_per_split = round_up(cdiv(a.M, splits), BM);
  splits = cdiv(a.M, a.m_per_split);
  a.splits = splits;
  a.partial = ws;
  const FastDiv d_ow = make_fastdiv((unsigned)a.OW), d_ohw = make_fastdiv((unsigned)(a.OH * a.OW));
  hipLaunchKernelGGL((wgrad_tr_kernel<BN, BK, WN, WK, BM, MAXOCC>), dim3(tiles * splits), dim3(256), 0, st, a, d_ow, d_ohw);
  DFA_HIP_CHECK(hipGetLastError());
  if (splits > 1) DFA_HIP_CHECK(slab_reduce(ws, a.gw, a.with_bias ? a.gb : nullptr, a.N, a.K, Kt, splits, a.scale, st));
  return hipSuccess;
}

}  // namespace

bool wgrad_tr_supported(const WgradArgs& a, int mode) {
  return mode == MODE_FWD && (!a.with_bias || a.gb != nullptr) && a.SC % 8 == 0 && a.N % 8 == 0 && a.ldd % 8 == 0 && a.M > 0 &&
         a.OH > 0 && a.OW > 0 && ((uintptr_t)a.dy & 15) == 0 && ((uintptr_t)a.src & 15) == 0;
}

hipError_t wgrad_tr(const WgradArgs& a, float* ws, size_t ws_floats, hipStream_t st) {
  static const int t128 = diag_int("wgrad128", 32);
  // 128 x 128 tiles at 32 rows per step, 3 workgroups per CU (170 VGPRs each: no spills)
  if (a.N >= 128 && t128 == 32) return launch_wgrad_tr<128, 128, 2, 2, 32, 3>(a, ws, ws_floats, st);
  if (a.N >= 128) return launch_wgrad_tr<128, 128, 2, 2>(a, ws, ws_floats, st);
  if (a.N <= 32) return launch_wgrad_tr<32, 128, 1, 4>(a, ws, ws_floats, st);  // Keras CNN conv2: no empty rows
  // 64-channel tiles step 32 rows at a time: 36.9 KB of LDS -> 4 workgroups per CU (ResNet layer 1:
  // 104 -> 82 us).  The 128 x 128 tile at 32 rows would need more than the 128 VGPRs of 4 workgroups per
  // CU and spills, which the inline-asm loads (destinations unprotected until their counted wait)
  // cannot tolerate: it stays at 64 rows.
  return launch_wgrad_tr<64, 128, 2, 2, 32>(a, ws, ws_floats, st);
}

}  // namespace dfa
