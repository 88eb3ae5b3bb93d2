// 3x3 / stride-1 / pad-1 convolution weight gradient with halo-tiled LDS staging (gfx950).
//
// G[co][kh][kw][ci] = sum_{b,oh,ow} dY[b][oh][ow][co] * X[b][oh+kh-1][ow+kw-1][ci]: the conv2d
// backprop-filter of the reference's tf.variableGrads (SURVEY §2.4 O8,
// /root/reference/src/common/models.ts:137-142), for every ResNet-18 conv but the stem, the stride-2
// convs and the 1x1 projections.
//
// wgrad_tr.hip treats this as a GEMM over the im2col matrix, so every input pixel is fetched from L2
// nine times (once per tap) and dY once per 128-column tile of G: ~470 MB of L2->LDS traffic for a
// 64-channel 32x32 layer at B = 256, which is what bounded it at ~230-450 TF/s.  Here a workgroup owns
// a 64(co) x 64(ci) x 9-tap block of G and walks 64-pixel tiles of the batch:
//   * a tile is 64 consecutive dY rows = TI images x R rows x W columns (W * R * TI = 64); its input
//     halo, TI x (R+2) x (W+2) pixels x 64 channels with the zero padding materialised, is staged in
//     LDS once and every tap reads it at a shifted row: each input element crosses L2 once per tile
//     (1.1-2.3x for the halo) instead of 9 times
//   * both operands are pixel-major ([pixel][channel] rows, 16-byte global loads, 16-byte LDS stores);
//     the MFMA wants 8 pixels per lane, which two ds_read_b64_tr_b16 per fragment deliver.  Each lane
//     supplies its own row address, so the tap shift is a uniform add to the row of the pixel the k
//     slot names (slot 8g + 4h + q of group g = pixel 16h + 4g + q of the 32-pixel half step)
//   * wave w owns ci columns 16w..16w+15 for all four 16-row co tiles and the nine taps: 36 MFMA
//     accumulators (144 VGPRs); per 32-pixel step it reads the 4 dY fragments once (reused 9x) and one
//     X fragment per tap (reused 4x): 13 fragments per 36 v_mfma_f32_16x16x32_bf16
//   * LDS rows of 64 channels at a stride of 80 bf16 (40 dwords: 8 consecutive rows of a transposed
//     read sit on 8 disjoint 8-bank groups), two buffers of (64 + 160) rows = 70 KB per 4-wave group;
//     the next tile's loads are in registers while the current one computes, one barrier per tile
//   * a workgroup is two such groups (8 waves, 140 KB, one per CU) that walk alternate tiles and sum
//     their blocks through LDS at the end: every CU holds 8 waves but writes one slab, not two — the
//     fp32 slabs (147 KB per workgroup, written and re-read by slab_reduce) are what bounded the
//     4-wave version at 39-45 us on ResNet layers 2-4
//   * the pixel range is split over workgroups (channel block fastest in the XCD-aware order, so the
//     workgroups of one XCD share the same dY / X rows in L2); splits > 1 write fp32 slabs that
//     slab_reduce sums in a fixed order (deterministic)
#include "common.h"
#include "kernels.h"
#include "diag.h"

namespace dfa {

namespace {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_vs __attribute__((__vector_size__(8)));

__device__ __forceinline__ bf16x4 tr_read_h(const bf16* p) {
  auto* lp = (__attribute__((address_space(3))) bf16*)(const_cast<bf16*>(p));
  const bf16x4_vs v =
      __builtin_amdgcn_ds_read_tr16_b64_v4bf16(reinterpret_cast<__attribute__((address_space(3))) bf16x4_vs*>(lp));
  return __builtin_bit_cast(bf16x4, v);
}

__device__ u32x4_t kZeroHalo16 = {0u, 0u, 0u, 0u};  // source of every zero-padding chunk

// operand loads from inline asm, waited for by hand (see igemm64.hip)
__device__ __forceinline__ u32x4_t hload16(const void* p) {
  u32x4_t r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

constexpr int kHP = 64;            // output pixels per tile
constexpr int kHS = 80;            // LDS row stride in bf16 (64 channels + 16)
constexpr int kHXP = 5;            // halo staging passes of 32 rows
constexpr int kHXR = 32 * kHXP;    // halo rows per buffer (>= TI * (R+2) * (W+2))
constexpr int kHBuf = (kHP + kHXR) * kHS;

struct HaloP {
  const bf16* dy;
  const bf16* x;
  float* out;      // slabs [splits][N][K] (splits > 1) or gw [N][K]
  int H, W, C, N, ldd;
  int R, HW2, HR2, hrows, rows_per_tile;
  int ntiles, tps, cblocks, cib_n, splits;
  float scale;
};

// Barrier of one 4-wave group (see conv3_halo.hip group_sync4): the groups walk their tiles independently.
__device__ __forceinline__ void wg_group_sync4(unsigned* ctr, unsigned& gen) {
  gen += 4u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int spin = 0; spin < (1 << 24); ++spin) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= gen) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// G groups of 4 waves share one output block: group gi walks tiles t0 + gi, t0 + gi + G, ... with its own
// LDS buffers, and the groups' partial blocks are summed through LDS before the one slab store (G = 2:
// 8 waves per CU at half the slab bytes of two 4-wave workgroups)
template <int G>
__global__ void __launch_bounds__(256 * G, 2 / G) wgrad_halo_kernel(HaloP p) {
  __shared__ __attribute__((aligned(16))) bf16 lds[G * 2 * kHBuf];
  const int gi = threadIdx.x >> 8;
  const int tid = threadIdx.x & 255, lane = tid & 63, wid = tid >> 6;
  const int logical = xcd_remap(blockIdx.x, p.cblocks * p.splits);
  const int cb = logical % p.cblocks, split = logical / p.cblocks;
  const int n0 = (cb / p.cib_n) * 64, c0 = (cb % p.cib_n) * 64;
  const int tb = split * p.tps;
  const int ntb = max(0, min(p.ntiles, tb + p.tps) - tb);
  const int t0 = tb + gi;                            // this group's tiles: t0, t0 + G, ...
  const int nt = ntb > gi ? (ntb - gi + G - 1) / G : 0;
  const int iters = (ntb + G - 1) / G;               // barrier count, the same for every group
  const int K = 9 * p.C;
  bf16* glds = lds + gi * 2 * kHBuf;

  const FDiv fper(p.HR2 * p.HW2), fhw2(p.HW2), frw(p.R * p.W), fw(p.W);
  // ---- staging map: thread = (row group r, 16-byte chunk ch) of 64-channel rows
  const int ch = tid & 7, r8 = tid >> 3;
  const bf16* dyb = p.dy + n0 + ch * 8;
  const bf16* xb = p.x + c0 + ch * 8;
  int xro[kHXP], xhr[kHXP], xiw[kHXP];  // per pass: row offset from the tile's first row, ih - oh0, iw
#pragma unroll
  for (int i = 0; i < kHXP; ++i) {
    const int j = r8 + 32 * i;
    const int slot = fper.div(j), rem = j - slot * fper.d;  // (float-reciprocal division: 3 VALU)
    const int hr = fhw2.div(rem), hc = rem - hr * p.HW2;
    xro[i] = slot * p.R + hr - 1;
    xhr[i] = j < p.hrows ? hr - 1 : -(1 << 20);  // rows past the halo load nothing
    xiw[i] = hc - 1;
  }
  u32x4_t rd[2], rx[kHXP];
  auto gload = [&](int t) {
    const long long m0 = (long long)t * kHP;
#pragma unroll
    for (int i = 0; i < 2; ++i) rd[i] = hload16(dyb + (m0 + r8 + 32 * i) * p.ldd);
    const int gr0 = t * p.rows_per_tile;  // first output row (b * H + oh) of the tile
    const int oh0 = gr0 % p.H;
#pragma unroll
    for (int i = 0; i < kHXP; ++i) {
      const int ih = oh0 + xhr[i];
      const bool v = (unsigned)ih < (unsigned)p.H && (unsigned)xiw[i] < (unsigned)p.W;
      rx[i] = hload16(v ? (const void*)(xb + ((long long)(gr0 + xro[i]) * p.W + xiw[i]) * p.C)
                        : (const void*)&kZeroHalo16);
    }
  };
  auto sstore = [&](int buf) {
    bf16* ds = glds + buf * kHBuf;
    bf16* xs = ds + kHP * kHS;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4_t*>(ds + (r8 + 32 * i) * kHS + ch * 8) = rd[i];
#pragma unroll
    for (int i = 0; i < kHXP; ++i)
      if (r8 + 32 * i < p.hrows) *reinterpret_cast<u32x4_t*>(xs + (r8 + 32 * i) * kHS + ch * 8) = rx[i];
  };

  // ---- fragment map: lane 4q+pp of group g supplies row 4g+q (+16 for the high half), columns 4pp..
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  int aoff[2][2], boff[2][2];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int s = sub * 32 + 16 * h + 4 * g + q;  // pixel slot of the tile
      const int slot = frw.div(s), q = s - slot * frw.d, rr = fw.div(q), cc = q - rr * p.W;
      aoff[sub][h] = s * kHS + 4 * pp;
      boff[sub][h] = kHP * kHS + ((slot * p.HR2 + rr) * p.HW2 + cc) * kHS + 4 * pp + wid * 16;
    }
  const int tap_row = p.HW2 * kHS;

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  __shared__ unsigned gsync[2];
  if (threadIdx.x < 2) gsync[threadIdx.x] = 0u;
  unsigned ggen = 0u;
  if (nt > 0) {
    gload(t0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sstore(0);
    if (nt > 1) gload(t0 + G);
  }
  __syncthreads();
  (void)iters;
  for (int it = 0; it < nt; ++it) {  // group barriers only: the groups drift apart
    {
      const bf16* base = glds + (it & 1) * kHBuf;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        bf16x8 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bf16x4 lo = tr_read_h(base + aoff[sub][0] + i * 16);
          const bf16x4 hi = tr_read_h(base + aoff[sub][1] + i * 16);
          fa[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int o = kh * tap_row + kw * kHS;
            const bf16x4 lo = tr_read_h(base + boff[sub][0] + o);
            const bf16x4 hi = tr_read_h(base + boff[sub][1] + o);
            const bf16x8 fb = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][kh * 3 + kw] = mfma16x16x32(fa[i], fb, acc[i][kh * 3 + kw]);
          }
      }
      if (it + 1 < nt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sstore((it + 1) & 1);
      }
    }
    if (G > 1) wg_group_sync4(&gsync[gi], ggen);
    else __syncthreads();
    if (it + 2 < nt) gload(t0 + (it + 2) * G);
  }

  if (G > 1) {
    __syncthreads();  // both groups done with their buffers (red overlays them)  // group 1 hands its block to group 0 through LDS, half (co tiles 0-1, then 2-3) at a time
    float* red = reinterpret_cast<float*>(lds);  // [wave][72 registers][64 lanes]
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (gi == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[(wid * 72 + (i * 9 + t) * 4 + r) * 64 + lane] = acc[2 * half + i][t][r];
      }
      __syncthreads();
      if (gi == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[2 * half + i][t][r] += red[(wid * 72 + (i * 9 + t) * 4 + r) * 64 + lane];
      }
      __syncthreads();
    }
    if (gi != 0) return;
  }

  // C/D layout of the 16x16 MFMA: column (ci) = lane & 15, row (co) = 4 * (lane >> 4) + r
  const int ci = c0 + wid * 16 + (lane & 15);
  float* out = p.splits > 1 ? p.out + (long long)split * p.N * K : p.out;
  const float sc = p.splits > 1 ? 1.f : p.scale;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = n0 + i * 16 + 4 * g + r;
        out[(long long)co * K + t * p.C + ci] = acc[i][t][r] * sc;
      }
}

// tile geometry of a W x H image: R rows of TI images per 64-pixel tile; false if it does not tile
bool halo_geom(int H, int W, int& R, int& TI) {
  if (W < 4 || W > 64 || kHP % W != 0) return false;
  const int rpt = kHP / W;
  if (rpt <= H) {
    if (H % rpt != 0) return false;
    R = rpt, TI = 1;
  } else {
    if (rpt % H != 0) return false;
    R = H, TI = rpt / H;
  }
  return TI * (R + 2) * (W + 2) <= kHXR;
}

}  // namespace

bool wgrad_halo_supported(const WgradArgs& a, int mode) {
  static const int on = diag_int("wgrad_halo", 1);
  int R, TI;
  return on && mode == MODE_FWD && !a.with_bias && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 &&
         a.OH == a.SH && a.OW == a.SW && a.SC % 64 == 0 && a.N % 64 == 0 && a.K == 9 * a.SC && a.ldd % 8 == 0 &&
         a.M % kHP == 0 && a.M == a.OH * a.OW * (a.M / (a.OH * a.OW)) && halo_geom(a.SH, a.SW, R, TI) &&
         ((uintptr_t)a.dy & 15) == 0 && ((uintptr_t)a.src & 15) == 0;
}

hipError_t wgrad_halo(const WgradArgs& a, float* ws, size_t ws_floats, hipStream_t st) {
  HaloP p;
  int R = 0, TI = 0;
  halo_geom(a.SH, a.SW, R, TI);
  p.dy = a.dy, p.x = a.src;
  p.H = a.SH, p.W = a.SW, p.C = a.SC, p.N = a.N, p.ldd = a.ldd;
  p.R = R, p.HW2 = a.SW + 2, p.HR2 = R + 2, p.hrows = TI * (R + 2) * (a.SW + 2), p.rows_per_tile = kHP / a.SW;
  p.ntiles = a.M / kHP;
  p.cib_n = a.SC / 64;
  p.cblocks = (a.N / 64) * p.cib_n;
  p.scale = a.scale;
  // one 8-wave workgroup per CU (140 KB of LDS), bounded by the slab workspace
  static const int groups = diag_int("halo_groups", 2) == 1 ? 1 : 2;
  static const int target = diag_int("halo_wg", groups == 2 ? 256 : 512);
  const long long per_split = (long long)a.N * a.K;
  int splits = max(1, cdiv(target, p.cblocks));
  splits = min(splits, p.ntiles);
  while (splits > 1 && (long long)splits * per_split > (long long)ws_floats) --splits;
  p.tps = cdiv(p.ntiles, splits);
  splits = cdiv(p.ntiles, p.tps);
  p.splits = splits;
  p.out = splits > 1 ? ws : a.gw;
  if (groups == 2)
    hipLaunchKernelGGL(wgrad_halo_kernel<2>, dim3(p.cblocks * splits), dim3(512), 0, st, p);
  else
    hipLaunchKernelGGL(wgrad_halo_kernel<1>, dim3(p.cblocks * splits), dim3(256), 0, st, p);
  DFA_HIP_CHECK(hipGetLastError());
  if (splits > 1) DFA_HIP_CHECK(slab_reduce(ws, a.gw, nullptr, a.N, a.K, a.K, splits, a.scale, st));
  return hipSuccess;
}

}  // namespace dfa
