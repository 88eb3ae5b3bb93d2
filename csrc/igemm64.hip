// Implicit-GEMM forward / data-gradient MFMA kernel with 64-deep k steps (gfx950), for the
// vectorizable cases of igemm_fwd: dense layers with K % 8 == 0 and NHWC conv / transposed-conv
// gathers with C % 8 == 0 (every ResNet-18 conv but the 3-channel stem).  SURVEY §2.4 O2/O3/O8:
// the reference's tf.js matMul / conv2d forward and the data gradients of its autodiff.
//
//   C[m][n] = epi( sum_k A[m][k] * W[n][k] ),  A = rows of the activation (dense), the im2col row
//   of an output pixel (conv forward) or the transposed-conv gather of dY (data gradient).
//
//   * 4 waves (2 x 2) on a 128x128 / 128x64 / 64x128 tile; v_mfma_f32_16x16x32_bf16; each 64-deep
//     step is two 32-deep halves, so a wave issues 2*TM*TN MFMAs per barrier (32 on 128x128)
//   * register-staged prefetch D steps deep (D register sets) into a double-buffered LDS tile: the
//     16-byte global loads of step k+D are issued right after step k's barrier and stored to LDS after
//     the MFMAs of step k+D-1; one barrier per step
//   * LDS rows of 64 bf16 (128 B) with the 16-byte chunk swizzle c ^ ((row >> 1) & 7): the 16 rows
//     one ds_read_b128 lane group reads sit on 16 distinct 16-byte bank slots
//   * a thread's 16-byte chunk column is fixed (c = tid & 7), so ONE (kh, kw, ci) state per thread
//     advances per step; the per-row pixel state is computed once with multiply-high division
//   * a masked-out load reads a 16-byte zero constant (address select: no load under a branch and no
//     data masking that would force a wait right after the load)
//   * epilogue as igemm.hip: alpha, bias, residual join (res * [resmask > 0]), ReLU, relu'(mask), with
//     the weights as the MFMA A operand so each lane stores 4 adjacent output channels at once
#include "common.h"
#include "kernels.h"
#include "diag.h"
#include "bn_epi.h"
#include "bn_acc.h"

namespace dfa {

namespace {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

#ifndef IGEMM64_STAGES
#define IGEMM64_STAGES 2
#endif
constexpr int kIgemm64Stages = IGEMM64_STAGES;  // register prefetch depth (steps in flight)

__device__ u32x4_t kZero16 = {0u, 0u, 0u, 0u};  // source of every masked-out 16-byte chunk

// Operand loads are issued from inline asm: hipcc's waitcnt pass then does not see them and cannot
// insert its conservative loop-carried `s_waitcnt vmcnt` (it waited for the newest loads before every
// LDS store, collapsing any prefetch depth to one step).  The k loop counts them by hand: the stage
// stored at step k has exactly (D-1) newer stages in flight in the steady state.
__device__ __forceinline__ u32x4_t gload16(const void* p) {
  u32x4_t r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

// FAST path operand loads: raw buffer loads through a wave-uniform descriptor.  The per-k-step part of
// the address is one uniform byte offset (SGPR soffset for the weights, one v_add for the activation
// rows) and a masked-out chunk is an out-of-range voffset (>= num_records): the hardware returns zeros,
// so no select between a data pointer and a zero constant and no 64-bit address math per load.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ i32x4_t make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)(uintptr_t)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xFFFFu));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}

__device__ __forceinline__ u32x4_t bload16(i32x4_t rsrc, unsigned voff, unsigned soff) {
  u32x4_t r;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(r) : "v"(voff), "s"(rsrc), "s"(soff) : "memory");
  return r;
}

// lane exchanges inside groups of 4 lanes (DPP quad_perm: VALU latency, no LDS round trip)
__device__ __forceinline__ int quad_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int quad_xor2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); }
__device__ __forceinline__ float quad_xor1(float v) { return __int_as_float(quad_xor1(__float_as_int(v))); }
__device__ __forceinline__ float quad_xor2(float v) { return __int_as_float(quad_xor2(__float_as_int(v))); }

__device__ __forceinline__ int swz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3); }

// occupancy the LDS footprint allows (2 x (BM + BN) x 128 B per workgroup): 4 workgroups of 40 KB, 3 of
// 48 KB or 2 of 64 KB per CU; the register budget is capped to match (one workgroup = one wave per SIMD)
template <int BM, int BN>
constexpr int igemm64_occ() { return (160 * 1024) / ((BM + BN) * 256) > 4 ? 4 : (160 * 1024) / ((BM + BN) * 256); }

// POOL (conv forward + 2x2 max-pool, the Keras CNN's conv2 -> pool): output rows are taken in
// pool-window-major order, m = (b, window, position), so the four pixels of a window are rows 4q..4q+3
// of a 16-row MFMA block, i.e. four adjacent lanes; the epilogue reduces them with two lane shuffles
// and writes only the pooled map [M/4][N] and a 1-byte argmax code per pooled element (4 = no
// gradient: the ReLU'd max is 0).  d_ow then divides by the pooled width.
//
// FAST (conv gathers with SC % 64 == 0, K == KH*KW*SC, stride-1 data gradient or any forward): every
// 64-deep k step is one filter tap (kh, kw) and one 64-channel block, so the step's address delta is the
// same for every row and lane.  A row keeps a 32-bit byte offset and a bitmask of the taps that land
// inside the image; a step costs ~4 VALU per activation row and none per weight row (the k offset is
// the SGPR soffset), against ~23 VALU per MFMA of the generic gather (igemm64 PMC/ISA, round 2).
//
// PAR (FAST stride-2 data gradient): dX pixels of one parity class (ih % 2, iw % 2) receive only the
// taps with kh = ih + pad (mod 2), kw likewise, so the output rows are grouped by class (class-major
// tiles, rows (b, y, x) -> pixel (b, 2y + py, 2x + px)) and every tile runs only its class's taps:
// 9 -> 1/2/2/4 taps for a 3x3 kernel instead of issuing MFMAs on the 3/4 of the gather that is zero.
template <int BM, int BN, int MODE, int D, bool SPLIT, bool POOL = false, bool FAST = false, bool PAR = false>
__global__ void __launch_bounds__(256, (igemm64_occ<BM, BN>())) igemm64_kernel(IGemmArgs a, FastDiv d_ow, FastDiv d_ohw) {
  static_assert(!POOL || (MODE == MODE_FWD && !SPLIT), "pooled epilogue: plain conv forward only");
  static_assert(!FAST || MODE != MODE_DIRECT, "FAST: conv gathers only");
  static_assert(!PAR || (FAST && MODE == MODE_DGRAD && !SPLIT && !POOL), "PAR: FAST stride-2 data gradient");
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / (WM * 16), TN = BN / (WN * 16);
  constexpr int AP = BM / 32, BP = BN / 32;  // 16-byte chunks per thread and step (8 chunks per 64-deep row)
  static_assert(TM >= 1 && TN >= 1 && AP >= 1 && BP >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * (BM + BN) * 64];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = cdiv(a.N, BN);
  // PAR: class (py, px) of this tile, its row count and size; the tiles of class 0 come first
  int py = 0, px = 0, Mrows = a.M, cHc = 1, cWc = 1;
  int ntm = cdiv(a.M, BM), ptiles = 0;
  if constexpr (PAR) {
    const int nimg = a.M / (a.OH * a.OW);
    int rest = xcd_remap(blockIdx.x, (int)gridDim.x);
    ptiles = (int)gridDim.x;
    for (int cl = 0; cl < 4; ++cl) {
      const int hc = (a.OH - (cl >> 1) + 1) >> 1, wc = (a.OW - (cl & 1) + 1) >> 1;
      const int mc = nimg * hc * wc, tc = cdiv(mc, BM) * ntn;
      if (rest < tc || cl == 3) {
        py = cl >> 1;
        px = cl & 1;
        Mrows = mc;
        cHc = hc;
        cWc = wc;
        ntm = cdiv(mc, BM);
        ptiles = rest;
        break;
      }
      rest -= tc;
    }
  }
  const int nsplit = SPLIT ? a.splits : 1;
  const int logical0 = PAR ? ptiles : xcd_remap(blockIdx.x, ntn * ntm * nsplit);
  const int split = SPLIT ? logical0 / (ntn * ntm) : 0;
  const int logical = SPLIT ? logical0 - split * (ntn * ntm) : logical0;
  const int tile_n = logical % ntn, tile_m = logical / ntn;
  // k steps of this split: [kt_begin, kt_end)
  const int nk_all = cdiv(a.K, 64);
  const int kper = SPLIT ? cdiv(nk_all, nsplit) : nk_all;
  const int kt_begin = split * kper;
  const int kt_end = min(nk_all, kt_begin + kper);
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int c = tid & 7, r0 = tid >> 3;  // chunk column; rows r0 + 32 i

  // per-row source state (fixed over the k loop).  rptr folds the row's pixel offset into a pointer
  // so a k step only adds one 32-bit offset per load (the im2col address math was the VALU hot spot:
  // ~9 VALU per MFMA in the PMC counters)
  long long rbase[AP];
  const bf16* rptr[AP];
  int rh[AP], rw[AP];
  bool rval[AP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int m = m0 + r0 + 32 * i;
    rval[i] = m < Mrows;
    const unsigned mm = (unsigned)min(m, Mrows - 1);
    if (PAR) {  // class-local row (b, y, x); base pixel (y + qh, x + qw), taps at -(jh, jw)
      const int b = (int)mm / (cHc * cWc);
      const int rem = (int)mm - b * cHc * cWc;
      const int y = rem / cWc, x = rem - (rem / cWc) * cWc;
      rbase[i] = (long long)b * a.SH * a.SW * a.SC;
      rh[i] = y + ((py + a.pad) >> 1);
      rw[i] = x + ((px + a.pad) >> 1);
    } else if (MODE == MODE_DIRECT) {
      rbase[i] = (long long)mm * a.lda;
      rh[i] = rw[i] = 0;
    } else {
      const unsigned b = fdiv(mm, d_ohw);
      const unsigned rem = mm - b * (unsigned)(a.OH * a.OW);
      unsigned oh;
      int ow;
      if (POOL) {  // rem = 4 * (ph * OW/2 + pw) + 2 * dy + dx
        const unsigned win = rem >> 2, ph = fdiv(win, d_ow);
        oh = 2 * ph + ((rem >> 1) & 1);
        ow = 2 * (int)(win - ph * (unsigned)(a.OW >> 1)) + (int)(rem & 1);
      } else {
        oh = fdiv(rem, d_ow);
        ow = (int)(rem - oh * (unsigned)a.OW);
      }
      rbase[i] = (long long)b * a.SH * a.SW * a.SC;
      if (MODE == MODE_FWD) {
        rh[i] = (int)oh * a.stride - a.pad;
        rw[i] = ow * a.stride - a.pad;
      } else {
        rh[i] = (int)oh + a.pad;
        rw[i] = ow + a.pad;
      }
    }
    rptr[i] = a.src + rbase[i] + ((long long)rh[i] * a.SW + rw[i]) * a.SC;
  }
  // FAST row state: byte offset of the row's tap-(0,0) pixel + this thread's chunk, and the taps in range
  int roff[FAST ? AP : 1];
  unsigned rtaps[FAST ? AP : 1];
  int woff[FAST ? BP : 1];
  i32x4_t rsA, rsB;
  // uniform k-step state: tap (ukh, ukw) of the tap grid, channel block ucb.  The tap grid is
  // kh = tkh0 + tstep * ukh (tnh taps), kw likewise: the whole filter, or one parity class's taps (PAR)
  int ukh = 0, ukw = 0, ucb = 0;
  int tkh0 = 0, tkw0 = 0, tnh = a.KH, tnw = a.KW;
  constexpr int tstep = PAR ? 2 : 1;
  if constexpr (PAR) {
    tkh0 = (py + a.pad) & 1;
    tkw0 = (px + a.pad) & 1;
    tnh = a.KH > tkh0 ? (a.KH - tkh0 + 1) >> 1 : 0;
    tnw = a.KW > tkw0 ? (a.KW - tkw0 + 1) >> 1 : 0;
  }
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      roff[i] = (int)((rbase[i] + ((long long)rh[i] * a.SW + rw[i]) * a.SC) * 2) + 16 * c;
      unsigned mk = 0;
      if (rval[i]) {
        for (int jh = 0; jh < tnh; ++jh)
          for (int jw = 0; jw < tnw; ++jw) {
            const int sh = MODE == MODE_FWD ? rh[i] + jh : rh[i] - jh;
            const int sw = MODE == MODE_FWD ? rw[i] + jw : rw[i] - jw;
            if ((unsigned)sh < (unsigned)a.SH && (unsigned)sw < (unsigned)a.SW) mk |= 1u << (jh * tnw + jw);
          }
      }
      rtaps[i] = mk;
    }
    const int nimg = a.M / (a.OH * a.OW);
    rsA = make_rsrc(a.src, (unsigned)((long long)nimg * a.SH * a.SW * a.SC * 2));
    const int npad16 = round_up(a.N, 16);
    rsB = make_rsrc(a.w, (unsigned)((long long)npad16 * a.Kpad * 2));
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int n = n0 + r0 + 32 * i;
      woff[i] = n < npad16 ? (int)((long long)n * a.Kpad * 2) + 16 * c : (int)kOOB;
    }
    const int kb = kt_begin * 64;
    const int t = kb / a.SC;
    ucb = (kb - t * a.SC) >> 6;
    ukh = t / a.KW;
    ukw = t - ukh * a.KW;
  }
  const bf16* wptr[BP];
  bool wval[BP];
  const int npad = round_up(a.N, 16);
#pragma unroll
  for (int i = 0; i < BP; ++i) {
    const int n = n0 + r0 + 32 * i;
    wval[i] = n < npad;
    wptr[i] = a.w + (long long)(wval[i] ? n : 0) * a.Kpad;
  }
  // this thread's k chunk: k = kt * 64 + 8c  ->  (kh, kw, ci) for the gathers
  int kk = kt_begin * 64 + 8 * c, kh = 0, kw = 0, ci = kk;
  if (MODE != MODE_DIRECT) {
    ci = kk % a.SC;
    const int t = kk / a.SC;
    kh = t / a.KW;
    kw = t - kh * a.KW;
  }

  // D register stages of prefetched global loads: the loads of step k are issued D iterations before
  // step k is stored to LDS, so ~D * (MFMA time of one step) of memory latency is covered even with a
  // single wave per SIMD (the small-M layers launch one workgroup per CU)
  u32x4_t ra[D][AP], rb[D][BP];
  auto gload = [&](int st) {
    if constexpr (FAST) {
      const int tap = ukh * tnw + ukw;
      const int tpix = ukh * a.SW + ukw;
      const int toff = ((MODE == MODE_FWD ? tpix : -tpix) * a.SC + ucb * 64) * 2;
#pragma unroll
      for (int i = 0; i < AP; ++i) {
        const unsigned vo = ((rtaps[i] >> tap) & 1u) ? (unsigned)(roff[i] + toff) : kOOB;
        ra[st][i] = bload16(rsA, vo, 0u);
      }
      // this step's weight column in bytes (the weights' soffset)
      const unsigned ks = (unsigned)((((tkh0 + tstep * ukh) * a.KW + tkw0 + tstep * ukw) * a.SC + ucb * 64) * 2);
#pragma unroll
      for (int i = 0; i < BP; ++i) rb[st][i] = bload16(rsB, (unsigned)woff[i], ks);
      return;
    }
    const bool kv = kk < a.K;
    // k-step offset of this thread's chunk relative to the row pointer (same for every row)
    const int koff = (MODE == MODE_FWD) ? (kh * a.SW + kw) * a.SC + ci : ci - (kh * a.SW + kw) * a.SC;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      bool v = rval[i] && kv;
      const bf16* p;
      if (MODE == MODE_DIRECT) {
        p = a.src + rbase[i] + kk;
      } else if (MODE == MODE_FWD) {
        const int sh = rh[i] + kh, sw = rw[i] + kw;
        v = v && (unsigned)sh < (unsigned)a.SH && (unsigned)sw < (unsigned)a.SW;
        p = rptr[i] + koff;
      } else if (a.stride == 1) {  // dX(ih, iw) <- dY(ih + pad - kh, iw + pad - kw)
        const int th = rh[i] - kh, tw = rw[i] - kw;
        v = v && (unsigned)th < (unsigned)a.SH && (unsigned)tw < (unsigned)a.SW;
        p = rptr[i] + koff;
      } else {  // dX(ih, iw) <- dY((ih + pad - kh) / s, (iw + pad - kw) / s)
        int th = rh[i] - kh, tw = rw[i] - kw;
        v = v && th >= 0 && tw >= 0 && (th % a.stride) == 0 && (tw % a.stride) == 0;
        th /= a.stride;
        tw /= a.stride;
        v = v && th < a.SH && tw < a.SW;
        p = a.src + rbase[i] + ((long long)th * a.SW + tw) * a.SC + ci;
      }
      // a masked-out chunk reads 16 zero bytes instead (address select, not a data mask: the loaded value
      // is not touched until its LDS store D steps later, so no wait is forced right after the load)
      ra[st][i] = gload16(v ? (const void*)p : (const void*)&kZero16);
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const bool v = wval[i] && kk < a.Kpad;
      rb[st][i] = gload16(v ? (const void*)(wptr[i] + kk) : (const void*)&kZero16);
    }
  };
  auto advance = [&]() {
    kk += 64;
    if constexpr (FAST) {
      if (++ucb * 64 == a.SC) {
        ucb = 0;
        if (++ukw == tnw) {
          ukw = 0;
          ++ukh;
        }
      }
      return;
    }
    if (MODE != MODE_DIRECT) {
      ci += 64;
      while (ci >= a.SC) {
        ci -= a.SC;
        if (++kw == a.KW) {
          kw = 0;
          ++kh;
        }
      }
    }
  };
  auto sstore = [&](int buf, int st) {
    bf16* as = lds + buf * (BM + BN) * 64;
    bf16* bs = as + BM * 64;
#pragma unroll
    for (int i = 0; i < AP; ++i) *reinterpret_cast<u32x4_t*>(as + swz(r0 + 32 * i, c)) = ra[st][i];
#pragma unroll
    for (int i = 0; i < BP; ++i) *reinterpret_cast<u32x4_t*>(bs + swz(r0 + 32 * i, c)) = rb[st][i];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // k steps of this workgroup (a whole K without split-K; the class's taps under PAR)
  const int nk = PAR ? tnh * tnw * (a.SC >> 6) : max(kt_end - kt_begin, 0);
  // prologue: step 0 -> LDS[0]; steps 1..D in flight (register stage of step s = s % D)
  if (nk > 0) gload(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sstore(0, 0);
#pragma unroll
  for (int s = 1; s <= D; ++s) {
    if (s < nk) {
      advance();
      gload(s % D);
    }
  }
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kb = 0; kb < nk; kb += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int kt = kb + u;
      if (kt < nk) {
        const int cur = kt & 1;
        const bf16* as = lds + cur * (BM + BN) * 64;
        const bf16* bs = as + BM * 64;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          bf16x8 fa[TM], fb[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i)
            fa[i] = *reinterpret_cast<const bf16x8*>(as + swz(wm * TM * 16 + i * 16 + fr, h * 4 + fq));
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fb[j] = *reinterpret_cast<const bf16x8*>(bs + swz(wn * TN * 16 + j * 16 + fr, h * 4 + fq));
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(fb[j], fa[i], acc[i][j]);  // D[n][m]
        }
        const int nst = (u + 1) % D;  // register stage holding step kt + 1
        if (kt + 1 < nk) {
          if (kt + D < nk)
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"((AP + BP) * (D - 1)) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          sstore(cur ^ 1, nst);
        }
        __syncthreads();
        if (kt + 1 + D < nk) {  // refill the freed stage with step kt + 1 + D
          advance();
          gload(nst);
        }
      }
    }
  }

  if (SPLIT) {
    // raw fp32 partials [split][M][N]; the reduce kernel applies the epilogue
    float* ws = a.splitk_ws + (long long)split * a.M * a.N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = m0 + wm * TM * 16 + i * 16 + fr;
      if (row >= a.M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col0 = n0 + wn * TN * 16 + j * 16 + fq * 4;
        if (col0 >= a.N) continue;  // N % 4 == 0 on this path
        *reinterpret_cast<f32x4*>(ws + (long long)row * a.N + col0) = acc[i][j];
      }
    }
    return;
  }

  if (POOL) {
    typedef __bf16 bf16x4_p __attribute__((ext_vector_type(4)));
    const unsigned long long dseed = a.drop.on ? drop_seed(a.drop.seed, a.drop.step, a.drop.step_add) : 0ull;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = m0 + wm * TM * 16 + i * 16 + fr;  // the window's rows are lanes fr & ~3 .. + 3
      const long long prow = row >> 2;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col0 = n0 + wn * TN * 16 + j * 16 + fq * 4;
        float mx[4];
        int pc[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // the conv output as the unfused path stored it (bf16), then the first max of the window
          const float v = (float)f2bf(acc[i][j][r] * a.alpha + ((a.bias && col0 + r < a.N) ? a.bias[col0 + r] : 0.f));
          float m = fmaxf(v, quad_xor1(v));
          m = fmaxf(m, quad_xor2(m));
          int p = v == m ? (fr & 3) : 4;
          p = min(p, quad_xor1(p));
          p = min(p, quad_xor2(p));
          mx[r] = m;
          pc[r] = p;
        }
        if ((fr & 3) || row >= a.M || col0 >= a.N) continue;
        bf16x4_p ov;
        unsigned codes = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float o = mx[r];
          int cd = pc[r];
          if (a.relu) {
            if (!(o > 0.f)) cd = 4;
            o = fmaxf(o, 0.f);
          }
          if (a.drop.on) o = drop_keep(dseed, a.drop.thresh, prow * a.N + col0 + r) ? (float)f2bf(o) * a.drop.scale : 0.f;
          ov[r] = f2bf(o);
          codes |= (unsigned)cd << (8 * r);
        }
        *reinterpret_cast<bf16x4_p*>(reinterpret_cast<bf16*>(a.out) + prow * a.ldc + col0) = ov;
        *reinterpret_cast<unsigned*>(a.pool_code + prow * a.N + col0) = codes;
      }
    }
    return;
  }

  // epilogue.  The weights are the MFMA's A operand, so the 16x16 C/D layout puts 4 consecutive output
  // COLUMNS (n = 4 * (lane >> 4) + r) of one output row (m = lane & 15) in a lane: every lane moves
  // one 8-byte bf16x4 (16-byte f32x4) store and 8-byte residual / mask loads instead of four 2-byte ones.
  const bool vec = (a.ldc & 3) == 0 && ((uintptr_t)a.out & 15) == 0 &&
                   (((uintptr_t)a.res | (uintptr_t)a.resmask | (uintptr_t)a.mask) & 7) == 0;
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  if (a.bacc.acc) {
    // BatchNorm sums of the stored values (csrc/bn_acc.h; the host admits only the vectorised epilogue,
    // bf16 output, no dropout): per column group j over the lane's rows, the 16 lanes of the group, then
    // the WM wave rows through LDS slots
    const bool two = a.bacc.acc2 != nullptr;
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();  // LDS is free after the k loop
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = wn * TN * 16 + j * 16 + fq * 4;
      const int col0 = n0 + cl;
      const bool colok = col0 + 3 < a.N;
      // this column group's loads (statistics, residual / masks, BatchNorm inputs) all in flight before
      // its first store: a load behind a store waits for that store too (csrc/bn_acc.h)
      const BnAccChan bc = bacc_chan(a.bacc, colok ? col0 : 0);
      long long oo[TM];
      bf16x4_t prv[TM], prm[TM], pmk[TM];
      BnAccX pxs[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = min(m0 + wm * TM * 16 + i * 16 + fr, Mrows - 1);  // (clamped: skipped below)
        long long orow = row;
        if (PAR) {
          const int b = row / (cHc * cWc);
          const int rem = row - b * cHc * cWc;
          const int y = rem / cWc, x = rem - (rem / cWc) * cWc;
          orow = ((long long)b * a.OH + 2 * y + py) * a.OW + 2 * x + px;
        }
        const long long o = orow * a.ldc + (colok ? col0 : 0);
        oo[i] = o;
#pragma unroll
        for (int r = 0; r < 4; ++r) prv[i][r] = prm[i][r] = pmk[i][r] = (__bf16)1.f;
        if (a.res) {
          prv[i] = *reinterpret_cast<const bf16x4_t*>(a.res + o);
          if (a.resmask) prm[i] = *reinterpret_cast<const bf16x4_t*>(a.resmask + o);
        }
        if (a.mask) pmk[i] = *reinterpret_cast<const bf16x4_t*>(a.mask + o);
        pxs[i] = bacc_loadx(a.bacc, o);
      }
      BnAccLane bl;
      bacc_zero(bl);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = m0 + wm * TM * 16 + i * 16 + fr;
        if (row >= Mrows || !colok) continue;
        const long long o = oo[i];
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * a.alpha + (a.bias ? a.bias[col0 + r] : 0.f);
        if (a.res) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (!a.resmask || (float)prm[i][r] > 0.f) v[r] += (float)prv[i][r];
        }
        if (a.relu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (a.mask) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (!((float)pmk[i][r] > 0.f)) v[r] = 0.f;
        }
        bf16x4_t ov;
        float sv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ov[r] = f2bf(v[r]);
          sv[r] = (float)ov[r];
        }
        *reinterpret_cast<bf16x4_t*>(reinterpret_cast<bf16*>(a.out) + o) = ov;
        bacc_add4x(bl, a.bacc, bc, pxs[i], sv);
      }
      bacc_reduce16(bl, two);
      if (fr == 0) bacc_stash(red, wm, BN, cl, bl);
    }
    __syncthreads();
    bacc_flush(a.bacc, red, WM, BN, n0, a.N, tid, 256);
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = m0 + wm * TM * 16 + i * 16 + fr;
    if (row >= Mrows) continue;
    long long orow = row;
    if (PAR) {  // class-local row -> dX pixel (b, 2y + py, 2x + px)
      const int b = row / (cHc * cWc);
      const int rem = row - b * cHc * cWc;
      const int y = rem / cWc, x = rem - (rem / cWc) * cWc;
      orow = ((long long)b * a.OH + 2 * y + py) * a.OW + 2 * x + px;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col0 = n0 + wn * TN * 16 + j * 16 + fq * 4;
      if (col0 >= a.N) continue;
      const long long o = orow * a.ldc + col0;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * a.alpha + ((a.bias && col0 + r < a.N) ? a.bias[col0 + r] : 0.f);
      if (vec && col0 + 3 < a.N) {
        if (a.res) {
          const bf16x4_t rv = *reinterpret_cast<const bf16x4_t*>(a.res + o);
          bf16x4_t rm;
          if (a.resmask) rm = *reinterpret_cast<const bf16x4_t*>(a.resmask + o);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (!a.resmask || (float)rm[r] > 0.f) v[r] += (float)rv[r];
        }
        if (a.relu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (a.mask) {
          const bf16x4_t mk = *reinterpret_cast<const bf16x4_t*>(a.mask + o);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (!((float)mk[r] > 0.f)) v[r] = 0.f;
        }
        if (a.drop.on) {
          const unsigned long long ds = drop_seed(a.drop.seed, a.drop.step, a.drop.step_add);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = drop_keep(ds, a.drop.thresh, o + r) ? (float)f2bf(v[r]) * a.drop.scale : 0.f;
        }
        if (a.out_f32) {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.out) + o) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
          bf16x4_t ov;
#pragma unroll
          for (int r = 0; r < 4; ++r) ov[r] = f2bf(v[r]);
          *reinterpret_cast<bf16x4_t*>(reinterpret_cast<bf16*>(a.out) + o) = ov;
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (col0 + r >= a.N) continue;
        float x = v[r];
        if (a.res) {
          const float rv = (float)a.res[o + r];
          if (!a.resmask || (float)a.resmask[o + r] > 0.f) x += rv;
        }
        if (a.relu) x = fmaxf(x, 0.f);
        if (a.mask && !((float)a.mask[o + r] > 0.f)) x = 0.f;
        if (a.drop.on)
          x = drop_keep(drop_seed(a.drop.seed, a.drop.step, a.drop.step_add), a.drop.thresh, o + r) ? (float)f2bf(x) * a.drop.scale : 0.f;
        if (a.out_f32)
          reinterpret_cast<float*>(a.out)[o + r] = x;
        else
          reinterpret_cast<bf16*>(a.out)[o + r] = f2bf(x);
      }
    }
  }

  // BatchNorm statistics of this tile's STORED outputs (kernels.h BnEpi), finalised inside the launch:
  // the tile's output is re-read (its own stores, still in this XCD's L2) in 8-byte column chunks,
  // mode 1 with the BN input alongside, reduced over the rows through LDS into one partial row per row
  // tile, then the hierarchical last-arriver finalisation (csrc/bn_epi.h).
  if constexpr (!SPLIT && !POOL && !PAR && BN >= 64) {  // (32-column tiles keep their occupancy)
    if (a.bn.part) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's output stores are complete
      __syncthreads();
      typedef __bf16 bf16x4_b __attribute__((ext_vector_type(4)));
      constexpr int NCH = BN / 4, RPP = 256 / NCH;
      const int ch = tid % NCH, rs = tid / NCH;
      const int col = n0 + 4 * ch;
      float s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f}, mu[4], is[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mu[r] = (a.bn.mode == 1 && col + r < a.N) ? a.bn.mean[col + r] : 0.f;
        is[r] = (a.bn.mode == 1 && col + r < a.N) ? a.bn.invstd[col + r] : 1.f;
      }
      const bf16* ob = reinterpret_cast<const bf16*>(a.out);
      const int rend = min(m0 + BM, a.M);
      if (col + 3 < a.N && (a.ldc & 3) == 0) {
#pragma unroll 4
        for (int row = m0 + rs; row < rend; row += RPP) {
          const long long o = (long long)row * a.ldc + col;
          const bf16x4_b yv = *reinterpret_cast<const bf16x4_b*>(ob + o);
          bf16x4_b xv;
          if (a.bn.mode == 1) xv = *reinterpret_cast<const bf16x4_b*>(a.bn.x + o);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float y = (float)yv[r];
            s4[r] += y;
            q4[r] += a.bn.mode == 1 ? y * (((float)xv[r] - mu[r]) * is[r]) : y * y;
          }
        }
      } else {
        for (int row = m0 + rs; row < rend; row += RPP)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (col + r < a.N) {
              const long long o = (long long)row * a.ldc + col + r;
              const float y = (float)ob[o];
              s4[r] += y;
              q4[r] += a.bn.mode == 1 ? y * (((float)a.bn.x[o] - mu[r]) * is[r]) : y * y;
            }
      }
      float* red = reinterpret_cast<float*>(lds);  // the k loop ended with a barrier: LDS is free
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[(rs * BN + 4 * ch + r) * 2] = s4[r];
        red[(rs * BN + 4 * ch + r) * 2 + 1] = q4[r];
      }
      __syncthreads();
      for (int t = tid; t < 2 * BN; t += 256) {
        const int which = t / BN, c = t - which * BN;
        if (n0 + c >= a.N) continue;
        float v = 0.f;
        for (int w = 0; w < RPP; ++w) v += red[(w * BN + c) * 2 + which];  // fixed row-group order
        st_sc1(a.bn.part + ((long long)tile_m * 2 + which) * a.N + n0 + c, v);
      }
      __shared__ int s_last;
      bn_epi_finalize<256>(a.bn, a.N, a.M, tile_m, tile_n, n0, min(BN, a.N - n0), &s_last);
    }
  }
}

// (a folded dropout rounds the activation to bf16 before scaling, as the standalone pass saw it)
// split-K combine: out = epi(sum_s ws[s]) in a fixed split order (deterministic), 4 columns per thread
// With BatchNorm sums (a.bacc.acc; host: 256 % (N / 4) == 0, so a thread's columns never change over the
// grid-stride loop) every thread accumulates its 4 columns over its rows; the workgroup reduces them
// through LDS slots and adds one partial per column (csrc/bn_acc.h).
__global__ void __launch_bounds__(256) igemm64_splitk_epilogue_kernel(IGemmArgs a) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  const long long total4 = (long long)a.M * (a.N >> 2);
  const bool bacc = a.bacc.acc != nullptr;
  const int cpr = a.N >> 2;  // column groups per row
  BnAccLane bl;
  bacc_zero(bl);
  BnAccChan bc;
  if (bacc) bc = bacc_chan(a.bacc, (int)(threadIdx.x % cpr) * 4);
  // batches of U grid-stride iterations: every load of a batch (split partials, residual / masks,
  // BatchNorm inputs) in flight before its first store (a load behind a store waits for it too)
  constexpr int U = 4;
  const long long gs = (long long)gridDim.x * 256;
  for (long long q0 = (long long)blockIdx.x * 256 + threadIdx.x; q0 < total4; q0 += U * gs) {
    f32x4 sacc[U];
    bf16x4_t prv[U], prm[U], pmk[U];
    BnAccX pxs[U];
    long long oo[U];
    int cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long q = min(q0 + u * gs, total4 - 1);  // (clamped: not stored below)
      const long long row = q / (a.N >> 2);
      const int col0 = (int)(q - row * (a.N >> 2)) * 4;
      cc[u] = col0;
      sacc[u] = *reinterpret_cast<const f32x4*>(a.splitk_ws + row * a.N + col0);
#pragma unroll
      for (int s = 1; s < 4; ++s)  // (the common split counts unrolled so the loads issue together)
        if (s < a.splits) sacc[u] += *reinterpret_cast<const f32x4*>(a.splitk_ws + ((long long)s * a.M + row) * a.N + col0);
      for (int s = 4; s < a.splits; ++s)
        sacc[u] += *reinterpret_cast<const f32x4*>(a.splitk_ws + ((long long)s * a.M + row) * a.N + col0);
      const long long o = row * a.ldc + col0;
      oo[u] = o;
#pragma unroll
      for (int r = 0; r < 4; ++r) prv[u][r] = prm[u][r] = pmk[u][r] = (__bf16)1.f;
      if (a.res) {
        prv[u] = *reinterpret_cast<const bf16x4_t*>(a.res + o);
        if (a.resmask) prm[u] = *reinterpret_cast<const bf16x4_t*>(a.resmask + o);
      }
      if (a.mask) pmk[u] = *reinterpret_cast<const bf16x4_t*>(a.mask + o);
      if (bacc) pxs[u] = bacc_loadx(a.bacc, o);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (q0 + u * gs >= total4) break;
      const int col0 = cc[u];
      const long long o = oo[u];
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = sacc[u][r] * a.alpha + (a.bias ? a.bias[col0 + r] : 0.f);
      if (a.res) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!a.resmask || (float)prm[u][r] > 0.f) v[r] += (float)prv[u][r];
      }
      if (a.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (a.mask) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!((float)pmk[u][r] > 0.f)) v[r] = 0.f;
      }
      if (a.drop.on) {
        const unsigned long long ds = drop_seed(a.drop.seed, a.drop.step, a.drop.step_add);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = drop_keep(ds, a.drop.thresh, o + r) ? (float)f2bf(v[r]) * a.drop.scale : 0.f;
      }
      if (a.out_f32) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.out) + o) = f32x4{v[0], v[1], v[2], v[3]};
      } else {
        bf16x4_t ov;
        float sv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ov[r] = f2bf(v[r]);
          sv[r] = (float)ov[r];
        }
        *reinterpret_cast<bf16x4_t*>(reinterpret_cast<bf16*>(a.out) + o) = ov;
        if (bacc) bacc_add4x(bl, a.bacc, bc, pxs[u], sv);
      }
    }
  }
  if (bacc) {
    __shared__ float red[3 * 1024];  // (256 / cpr) slots x N columns x 3 = 3 * 1024 floats
    const bool two = a.bacc.acc2 != nullptr;
    bacc_stash(red, threadIdx.x / cpr, a.N, (int)(threadIdx.x % cpr) * 4, bl);
    (void)two;
    __syncthreads();
    bacc_flush(a.bacc, red, 256 / cpr, a.N, 0, a.N, threadIdx.x, 256);
  }
}

// the split-K combine's grid: with BatchNorm sums at most 512 workgroups (each adds one partial per column
// and quantity: <= 512 / nrep adds per accumulator address)
static int splitk_epi_grid(const IGemmArgs& a) {
  const long long total4 = (long long)a.M * (a.N / 4);
  return (int)min((total4 + 255) / 256, a.bacc.acc ? 512LL : 4096LL);
}
static bool bacc_combine_ok(const IGemmArgs& a) {
  return a.N % 4 == 0 && a.N <= 1024 && 256 % (a.N / 4) == 0 && !a.out_f32 && !a.drop.on && a.ldc % 4 == 0;
}

// Split-K for under-filled launches: fewer than ~2 workgroups per CU and a long K (ResNet-18 layers 3-4:
// M = B*8*8 or B*4*4 with K up to 4608) leave one wave per SIMD waiting on every step
template <int BM, int BN>
static int splitk_for(const IGemmArgs& a) {
  if (a.pool_code || a.bn.part) return 1;
  const long long tiles = (long long)cdiv(a.M, BM) * cdiv(a.N, BN);
  const int nk = cdiv(a.K, 64);
  if (a.N % 4 || a.ldc % 4 || tiles >= 512 || nk < 32) return 1;
  if (((uintptr_t)a.out & 15) || (((uintptr_t)a.res | (uintptr_t)a.resmask | (uintptr_t)a.mask) & 7)) return 1;
  int s = 1;
  while (s < 4 && tiles * s * 2 <= 1024 && nk / (s * 2) >= 16) s *= 2;
  // severely under-filled (the Keras CNN's 9216 -> 128 dense: 16 tiles): up to 16 splits of >= 4 steps
  if (tiles * s < 256)
    while (s < 16 && tiles * s * 2 <= 512 && nk / (s * 2) >= 4) s *= 2;
  return s;
}

// FAST gather eligibility (see igemm64_kernel): whole 64-channel blocks per tap, <= 32 taps, stride-1
// data gradient, and operands addressable with 32-bit byte offsets below the out-of-range marker
static bool igemm64_fast_ok(const IGemmArgs& a, int mode) {
  if (mode == MODE_DIRECT || a.SC % 64 || a.K != a.KH * a.KW * a.SC || a.KH * a.KW > 32 || a.Kpad < a.K) return false;
  if (mode == MODE_DGRAD && a.stride != 1 && a.stride != 2) return false;
  if (a.OH <= 0 || a.OW <= 0 || a.M % (a.OH * a.OW)) return false;
  static const bool off = diag_int("igemm_fast", 1) == 0;
  if (off) return false;
  const long long sbytes = (long long)(a.M / (a.OH * a.OW)) * a.SH * a.SW * a.SC * 2;
  const long long wbytes = (long long)round_up(a.N, 16) * a.Kpad * 2;
  return sbytes < (1LL << 30) && wbytes < (1LL << 30);
}

template <int BM, int BN, int MODE>
hipError_t launch64(IGemmArgs a, hipStream_t st) {
  const FastDiv d_ow = make_fastdiv((unsigned)max(a.OW, 1)), d_ohw = make_fastdiv((unsigned)max(a.OH * a.OW, 1));
  const int blocks = cdiv(a.M, BM) * cdiv(a.N, BN);
  constexpr int D = kIgemm64Stages;
  if (MODE == MODE_FWD && a.pool_code != nullptr) {
    hipLaunchKernelGGL((igemm64_kernel<BM, BN, MODE_FWD, D, false, true>), dim3(blocks), dim3(256), 0, st, a,
                       make_fastdiv((unsigned)max(a.OW / 2, 1)), d_ohw);
    return hipGetLastError();
  }
  constexpr bool kFastMode = MODE != MODE_DIRECT;
  const bool fast = kFastMode && igemm64_fast_ok(a, MODE);
  if (MODE == MODE_DGRAD && a.stride == 2) {
    if (!fast) {
      hipLaunchKernelGGL((igemm64_kernel<BM, BN, MODE, D, false>), dim3(blocks), dim3(256), 0, st, a, d_ow, d_ohw);
      return hipGetLastError();
    }
    // parity classes: grid = sum of the 4 classes' tiles (no split-K)
    const int nimg = a.M / (a.OH * a.OW);
    int grid = 0;
    for (int cl = 0; cl < 4; ++cl) {
      const int hc = (a.OH - (cl >> 1) + 1) >> 1, wc = (a.OW - (cl & 1) + 1) >> 1;
      grid += cdiv(nimg * hc * wc, BM) * cdiv(a.N, BN);
    }
    constexpr int kParMode = MODE == MODE_DGRAD ? MODE_DGRAD : MODE_FWD;
    hipLaunchKernelGGL((igemm64_kernel<BM, BN, kParMode, D, false, false, true, MODE == MODE_DGRAD>), dim3(grid),
                       dim3(256), 0, st, a, d_ow, d_ohw);
    return hipGetLastError();
  }
  const int s = a.splitk_ws ? splitk_for<BM, BN>(a) : 1;
  if (s > 1) {
    a.splits = s;
    if (fast)
      hipLaunchKernelGGL((igemm64_kernel<BM, BN, MODE, D, true, false, kFastMode>), dim3(blocks * s), dim3(256), 0, st, a, d_ow, d_ohw);
    else
      hipLaunchKernelGGL((igemm64_kernel<BM, BN, MODE, D, true>), dim3(blocks * s), dim3(256), 0, st, a, d_ow, d_ohw);
    DFA_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(igemm64_splitk_epilogue_kernel, dim3(splitk_epi_grid(a)), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  // (prefetch depths 3 and 4 measured equal to 2 on every ResNet-18 shape: scripts/convbench.py)
  if (fast)
    hipLaunchKernelGGL((igemm64_kernel<BM, BN, MODE, D, false, false, kFastMode>), dim3(blocks), dim3(256), 0, st, a, d_ow, d_ohw);
  else
    hipLaunchKernelGGL((igemm64_kernel<BM, BN, MODE, D, false>), dim3(blocks), dim3(256), 0, st, a, d_ow, d_ohw);
  return hipGetLastError();
}

template <int MODE>
hipError_t launch64_mode(const IGemmArgs& a, hipStream_t st) {
  if (a.N <= 32) return launch64<128, 32, MODE>(a, st);  // Keras CNN conv2 (32 channels): no half-empty tiles
  // (a 256 x 64 tile with 4 x 1 waves of 64 x 64 measured 9-16% slower on ResNet layer 1: 8 waves per
  // CU instead of 12)
  if (a.N <= 64) return launch64<128, 64, MODE>(a, st);
  // 128x128 while that still gives >= 2 workgroups per CU, else 64x128
  if ((long long)cdiv(a.M, 128) * cdiv(a.N, 128) >= 512) return launch64<128, 128, MODE>(a, st);
  return launch64<64, 128, MODE>(a, st);
}

}  // namespace

hipError_t igemm64_splitk_combine(const IGemmArgs& a, hipStream_t st) {
  if (a.bacc.acc && !bacc_combine_ok(a)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(igemm64_splitk_epilogue_kernel, dim3(splitk_epi_grid(a)), dim3(256), 0, st, a);
  return hipGetLastError();
}

long long igemm64_splitk_floats(const IGemmArgs& a, int mode) {
  static const bool off = diag_int("igemm_splitk", 1) == 0;
  if (off || !igemm64_supported(a, mode) || a.N <= 64) return 0;
  if ((long long)cdiv(a.M, 128) * cdiv(a.N, 128) >= 512) return 0;  // 128 x 128 tiles: already filled
  const int s = splitk_for<64, 128>(a);
  return s > 1 ? (long long)s * a.M * a.N : 0;
}

// Row tiles (and column ranges) of the launch when it can finalise BatchNorm statistics of its output
// (kernels.h BnEpi): conv forward or data gradient, bf16 output, no pooling, no split-K (those launches
// keep the statistics pass) and no parity-class stride-2 data gradient.  0 = it cannot.
int igemm64_bn_layout(const IGemmArgs& a, int mode, int* ntn) {
  if (mode == MODE_DIRECT || !igemm64_supported(a, mode) || a.pool_code || a.out_f32) return 0;
  if (igemm64_splitk_floats(a, mode) > 0) return 0;
  if (mode == MODE_DGRAD && a.stride == 2 && igemm64_fast_ok(a, mode)) return 0;
  if (a.N <= 32) return 0;  // 128 x 32 tiles are built without the statistics epilogue
  // tile shape as launch64_mode picks it
  const int BN = a.N <= 32 ? 32 : (a.N <= 64 ? 64 : 128);
  const int BM = (a.N <= 64 || (long long)cdiv(a.M, 128) * cdiv(a.N, 128) >= 512) ? 128 : 64;
  if (ntn) *ntn = cdiv(a.N, BN);
  return cdiv(a.M, BM);
}
int igemm64_bn_tiles(const IGemmArgs& a, int mode) { return igemm64_bn_layout(a, mode, nullptr); }

bool igemm64_pool_supported(const IGemmArgs& a) {
  return igemm64_supported(a, MODE_FWD) && a.OH % 2 == 0 && a.OW % 2 == 0 && a.N % 4 == 0 && a.ldc == a.N &&
         !a.out_f32 && !a.mask && !a.res && ((uintptr_t)a.out & 7) == 0 && ((uintptr_t)a.pool_code & 3) == 0;
}

bool igemm64_supported(const IGemmArgs& a, int mode) {
  if (((uintptr_t)a.src & 15) || ((uintptr_t)a.w & 15) || a.Kpad % 8 || a.M <= 0 || a.N <= 0) return false;
  if (mode == MODE_DIRECT) return a.lda % 8 == 0 && a.K % 8 == 0;
  return !a.irregular && a.SC % 8 == 0 && a.OH > 0 && a.OW > 0;
}

hipError_t igemm64(const IGemmArgs& a, int mode, hipStream_t st) {
  if (mode == MODE_DIRECT) return launch64_mode<MODE_DIRECT>(a, st);
  if (mode == MODE_FWD) return launch64_mode<MODE_FWD>(a, st);
  return launch64_mode<MODE_DGRAD>(a, st);
}

}  // namespace dfa
