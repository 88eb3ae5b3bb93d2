// 3x3 / stride-1 / pad-1 convolution forward and data gradient with halo-tiled LDS staging (gfx950).
//
//   FWD:   Y[p][co]  = sum_{tap, ci} X[p + off(tap)][ci] * W[co][tap][ci]
//   DGRAD: dX[p][ci] = sum_{tap, co} dY[p + off(tap)][co] * Wt[ci][8 - tap][co]   (flipped taps)
// the reference's tf.js conv2d forward and the data gradient of its autodiff (SURVEY §2.4 O3/O8,
// /root/reference/src/common/models.ts:137-142), for the ResNet-18 CIFAR 3x3 stride-1 convs.
//
// igemm64.hip gathers the im2col rows of every tap from L2: a 128-pixel tile fetches its input 9 times
// per 64-channel block, and the per-CU L2->LDS rate (~70 GB/s) bounds it at 240-600 TF/s.  Here:
//   * a workgroup owns 128 consecutive output pixels (TI images x R rows x W columns) x BN output
//     channels; per 64-channel input block it stages the input halo TI x (R+2) x (W+2) once (zero
//     padding materialised) and runs all nine taps against it as shifted row reads
//   * the weights of one (channel block, tap) step are staged per step (double buffer, XOR-swizzled
//     128-byte rows as in igemm64), loaded into registers one step ahead; they are the MFMA A operand, so each lane ends with 4 consecutive
//     output channels of one pixel (8-byte stores, 8-byte residual / mask loads in the epilogue)
//   * halo rows are 72 bf16 (36 dwords) apart and MFMA column j of pixel tile t is pixel 2j + (t & 1)
//     (+32 for t >= 2): the 16 rows a ds_read_b128 lane group reads, at two consecutive 16-byte chunks,
//     land on 16 distinct 4-bank slots for any tap shift (slot = 9 row + chunk mod 16; the two chunks
//     differ in parity); with W = 16 the image rows of the halo are W + 16 LDS rows apart so that the
//     row crossing inside a lane group keeps that property
//   * the halo is single-buffered: the next block's halo sits in registers from the first tap of the
//     current block and is stored after its ninth (one extra barrier per 9 steps); LDS = halo +
//     2 weight buffers <= 74 KB, so two workgroups share a CU
//   * 4 waves as 2 (pixel halves of 64) x 2 (channel halves of BN/2)
//   * epilogue as igemm64: alpha, residual join (res * [resmask > 0]), ReLU, relu'(mask)
#include <map>
#include <mutex>

#include "common.h"
#include "kernels.h"
#include "diag.h"
#include "bn_acc.h"

namespace dfa {

namespace {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

__device__ u32x4_t kZeroC3 = {0u, 0u, 0u, 0u};  // source of every zero-padding chunk

__device__ __forceinline__ u32x4_t cload16(const void* p) {
  u32x4_t r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

constexpr int kCP = 128;              // output pixels per workgroup
constexpr int kCS = 72;               // halo row stride (bf16)
constexpr int kCXP = 9;               // halo staging passes of 32 rows
constexpr int kCXR = 32 * kCXP;       // staged halo pixels (>= TI * (R+2) * (W+2))
constexpr int kCXL = 320;             // LDS halo rows (>= TI * (R+2) * HWP)

struct C3P {
  const bf16* src;   // NHWC [.][H][W][Cin]
  const bf16* w;     // [Cout_pad][Kpad]: column tapW * Cin + ci
  const bf16* res;
  const bf16* resmask;
  const bf16* mask;
  bf16* out;         // [M][ldc]
  int H, W, Cin, Cout, Kpad, ldc;
  int R, HW2, HR2, hrows, rows_per_tile;
  int HWP;           // LDS pitch of one halo image row, in rows (tiled kernel): W + 2, or W + 16 for W = 16
  int ntiles, nco;
  int tps;           // tiles per workgroup (the persistent 64 -> 64 kernel)
  int ks, cbs;       // split over input channel blocks: ks splits of cbs blocks (ks > 1: raw fp32 partials)
  float* ws;         // [ks][M][Cout] partials, summed + epilogue by igemm64_splitk_combine
  // ks > 1 with tick: no combine launch -- each split writes its partial through to memory and takes a
  // ticket of its output tile; the tile's last arriver sums the partials in split order and runs the
  // kernel's own epilogue (the last arriver resets the ticket)
  unsigned* tick;
  int relu;
  float alpha;
  BnAcc bacc;        // BatchNorm sums of the stored output (ks == 1; csrc/bn_acc.h)
};

__device__ __forceinline__ int wswz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3); }

// epilogue of 4 consecutive output channels of one pixel (as igemm64): alpha, residual join, ReLU, relu';
// `stored` receives the values as stored (bf16-rounded).  The loads (c3_preload) are issued for all of a
// lane's elements before the first store: a load behind a store waits for that store too (csrc/bn_acc.h).
struct C3Pre {
  bf16x4_t rv, rm, mk;
};
// (every tensor the epilogue touches is [M][ldc] bf16 under 4 GB -- conv3_halo_supported -- so one 32-bit
// byte offset per element serves all of them: an SGPR base + VGPR offset per load instead of a 64-bit
// address register pair per pointer and element)
template <typename T>
__device__ __forceinline__ const T& c3_at(const void* base, unsigned boff) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + boff);
}
__device__ __forceinline__ unsigned c3_boff(const C3P& p, long long m, int co) {
  return (unsigned)(m * p.ldc + co) * 2u;
}
__device__ __forceinline__ C3Pre c3_preload(const C3P& p, unsigned boff) {
  C3Pre q;
#pragma unroll
  for (int r = 0; r < 4; ++r) q.rv[r] = q.rm[r] = q.mk[r] = (__bf16)1.f;
  if (p.res) {
    q.rv = c3_at<bf16x4_t>(p.res, boff);
    if (p.resmask) q.rm = c3_at<bf16x4_t>(p.resmask, boff);
  }
  if (p.mask) q.mk = c3_at<bf16x4_t>(p.mask, boff);
  return q;
}
__device__ __forceinline__ BnAccX c3_loadx(const BnAcc& e, unsigned boff) {
  BnAccX r;
  if (e.mode == 1) {
    r.x = c3_at<bacc_bf16x4>(e.x, boff);
    r.x2 = e.acc2 ? c3_at<bacc_bf16x4>(e.x2, boff) : r.x;  // (one BatchNorm: no second read of x)
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) r.x[k] = r.x2[k] = (__bf16)0.f;
  }
  return r;
}
__device__ __forceinline__ void c3_store_pre(const C3P& p, unsigned boff, const f32x4& a, const C3Pre& q,
                                             float (&stored)[4]) {
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = a[r] * p.alpha;
  if (p.res) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (!p.resmask || (float)q.rm[r] > 0.f) v[r] += (float)q.rv[r];
  }
  if (p.relu) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
  }
  if (p.mask) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (!((float)q.mk[r] > 0.f)) v[r] = 0.f;
  }
  bf16x4_t ov;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ov[r] = f2bf(v[r]);
    stored[r] = (float)ov[r];
  }
  *reinterpret_cast<bf16x4_t*>(reinterpret_cast<char*>(p.out) + boff) = ov;
}

// ROW: one step is a kernel row (3 taps, 48 MFMAs per wave at BN = 64) instead of one tap (16): the
// row's weights sit in one LDS buffer (the next row in registers, stored between two barriers), so a
// step pays 2 barriers and one weight wait per 48 MFMAs instead of 1 and 1 per 16.  LDS at BN = 64:
// 46 KB halo + 24 KB = 70 KB, still two workgroups per CU.
template <int BN, bool FLIP, bool ROW>
__global__ void __launch_bounds__(256, 2) conv3_halo_kernel(C3P p) {
  constexpr int TN = BN / 32;          // 16-channel tiles per wave
  constexpr int WP = BN * 8 / 256;     // weight staging passes (32 rows each)
  constexpr int NWB = ROW ? 3 : 2;     // weight buffers (BN x 64 each): the row's 3 taps / a double buffer
  constexpr int RW = ROW ? 3 * WP : WP;
  __shared__ __attribute__((aligned(16))) bf16 lds[kCXL * kCS + NWB * BN * 64];
  bf16* hs = lds;
  bf16* wsb = lds + kCXL * kCS;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int logical = xcd_remap(blockIdx.x, p.ntiles * p.nco * p.ks);
  const int ksp = logical / (p.ntiles * p.nco), lt = logical - ksp * (p.ntiles * p.nco);
  const int tile = lt / p.nco, cob = lt % p.nco;
  const int co0 = cob * BN;
  const int cbb = ksp * p.cbs;                               // this split's first input channel block
  const int ncb = max(0, min(p.Cin / 64 - cbb, p.cbs));      // blocks of this split
  const int S = 9 * ncb;

  const FDiv fper(p.HR2 * p.HW2), fhw2(p.HW2), frw(p.R * p.W), fw(p.W);
  // ---- staging map
  const int ch = tid & 7, r8 = tid >> 3;
  const int gr0 = tile * p.rows_per_tile, oh0 = gr0 % p.H;
  const bf16* hsrc[kCXP];
  bool hval[kCXP];
  int lrow[kCXP];  // LDS row of the staged pixel (image rows HWP apart)
#pragma unroll
  for (int i = 0; i < kCXP; ++i) {
    const int j = r8 + 32 * i;
    const int slot = fper.div(j), rem = j - slot * fper.d;  // (float-reciprocal division: 3 VALU)
    const int hr = fhw2.div(rem), hc = rem - hr * p.HW2;
    const int ih = oh0 + hr - 1, iw = hc - 1;
    hval[i] = j < p.hrows && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    lrow[i] = (slot * p.HR2 + hr) * p.HWP + hc;
    hsrc[i] = p.src + ((long long)(gr0 + slot * p.R + hr - 1) * p.W + iw) * p.Cin + ch * 8;
  }
  const bf16* wsrc = p.w + (long long)(co0 + r8) * p.Kpad + ch * 8;

  u32x4_t rh[kCXP], rw[RW];
  auto load_halo = [&](int cb) {
#pragma unroll
    for (int i = 0; i < kCXP; ++i)
      rh[i] = cload16(hval[i] ? (const void*)(hsrc[i] + (cbb + cb) * 64) : (const void*)&kZeroC3);
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int i = 0; i < kCXP; ++i)
      if (r8 + 32 * i < p.hrows) *reinterpret_cast<u32x4_t*>(hs + lrow[i] * kCS + ch * 8) = rh[i];
  };
  auto load_w = [&](int s) {
    const int cb = s / 9, tap = s - cb * 9;
    const int col = (FLIP ? 8 - tap : tap) * p.Cin + (cbb + cb) * 64;
#pragma unroll
    for (int i = 0; i < WP; ++i) rw[i] = cload16(wsrc + (long long)(32 * i) * p.Kpad + col);
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int i = 0; i < WP; ++i) *reinterpret_cast<u32x4_t*>(wsb + buf * BN * 64 + wswz(r8 + 32 * i, ch)) = rw[i];
  };
  auto load_wrow = [&](int s3) {  // ROW: the 3 taps of kernel row kh of channel block cb
    const int cb = s3 / 3, kh = s3 - cb * 3;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int tap = 3 * kh + kw;
      const int col = (FLIP ? 8 - tap : tap) * p.Cin + (cbb + cb) * 64;
#pragma unroll
      for (int i = 0; i < WP; ++i) rw[kw * WP + i] = cload16(wsrc + (long long)(32 * i) * p.Kpad + col);
    }
  };
  auto store_wrow = [&]() {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int i = 0; i < WP; ++i)
        *reinterpret_cast<u32x4_t*>(wsb + kw * BN * 64 + wswz(r8 + 32 * i, ch)) = rw[(kw * WP + i) % RW];
  };

  // ---- fragment map (16x16x32: lane l holds row / column l & 15, k chunk l >> 4 (+4 for the high half))
  const int fl = lane & 15, fc = lane >> 4;
  int hoff[4];  // halo row (x kCS) of this lane's pixel in each of the wave's 4 pixel tiles
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int s = wm * 64 + 32 * (t >> 1) + 2 * fl + (t & 1);
    const int slot = frw.div(s), q = s - slot * frw.d, rr = fw.div(q), cc = q - rr * p.W;
    hoff[t] = ((slot * p.HR2 + rr) * p.HWP + cc) * kCS + fc * 8;
  }
  int woff[TN][2];
#pragma unroll
  for (int u = 0; u < TN; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h) woff[u][h] = wswz(wn * (BN / 2) + 16 * u + fl, fc + 4 * h);

  f32x4 acc[TN][4];
#pragma unroll
  for (int u = 0; u < TN; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](const bf16* wb, int toff) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 fa[TN], fb[4];
#pragma unroll
      for (int u = 0; u < TN; ++u) fa[u] = *reinterpret_cast<const bf16x8*>(wb + woff[u][h]);
#pragma unroll
      for (int t = 0; t < 4; ++t) fb[t] = *reinterpret_cast<const bf16x8*>(hs + hoff[t] + toff + 32 * h);
#pragma unroll
      for (int u = 0; u < TN; ++u)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[u][t] = mfma16x16x32(fa[u], fb[t], acc[u][t]);
    }
  };

  if constexpr (ROW) {
    const int S3 = 3 * ncb;
    load_halo(0);
    load_wrow(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_halo();
    store_wrow();
    if (S3 > 1) load_wrow(1);
    if (ncb > 1) load_halo(1);
    __syncthreads();
    for (int s3 = 0; s3 < S3; ++s3) {
      const int cb = s3 / 3, kh = s3 - cb * 3;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) mma(wsb + kw * BN * 64, (kh * p.HWP + kw) * kCS);
      if (s3 + 1 < S3) {
        __syncthreads();  // every wave is done with this row's weights (and, after kh = 2, the halo)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        store_wrow();
        if (kh == 2) store_halo();
        __syncthreads();
        if (s3 + 2 < S3) load_wrow(s3 + 2);
        if (kh == 2 && cb + 2 < ncb) load_halo(cb + 2);
      }
    }
  } else {
  // (a two-step register ring for the weights with counted vmcnt waits measured slower on every layer:
  // the loads are not what a step waits for)
  load_halo(0);
  load_w(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  store_halo();
  store_w(0);
  if (S > 1) load_w(1);
  if (ncb > 1) load_halo(1);
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    const int cb = s / 9, tap = s - cb * 9;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = (kh * p.HWP + kw) * kCS;
    mma(wsb + (s & 1) * BN * 64, toff);
    if (s + 1 < S) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      store_w((s + 1) & 1);
      if (tap == 8) {  // next channel block: every wave is done with this halo
        __syncthreads();
        store_halo();
      }
    }
    __syncthreads();
    if (s + 2 < S) load_w(s + 2);
    if (tap == 8 && cb + 2 < ncb) load_halo(cb + 2);
  }
  }

  // C/D layout: row (output channel) 4 * (lane >> 4) + r, column (pixel) lane & 15
  if (p.ks > 1 && p.tick != nullptr) {
    // the split-K partial written through (sc1) to the workspace, then the tile's ticket; only the last of
    // the ks splits goes on, with the ks partials summed in split order (its own from registers)
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        p.ws, (short)0, (int)((long long)p.ks * p.ntiles * kCP * p.Cout * 4), 0x00020000);
    auto woff = [&](int sp, int t, int u) -> int {
      const long long m = (long long)tile * kCP + wm * 64 + 32 * (t >> 1) + 2 * fl + (t & 1);
      const int co = co0 + wn * (BN / 2) + 16 * u + 4 * fc;
      return (int)((((long long)sp * p.ntiles * kCP + m) * p.Cout + co) * 4);
    };
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[u][t]), wr, woff(ksp, t, u), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's partial stores are written through
    __syncthreads();
    __shared__ int s_last;
    if (tid == 0) {
      const unsigned prev = __hip_atomic_fetch_add(p.tick + lt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev == (unsigned)(p.ks - 1);
      if (s_last) __hip_atomic_store(p.tick + lt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the ticket)
    // ks == 2 (the host's condition): the other split's partial added to this one's -- p0 + p1 is the same
    // fp32 value whichever of the two arrives last, so the result does not depend on the arrival order
    const int other = 1 - ksp;
    f32x4 part[4][TN];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
        part[t][u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, woff(other, t, u), 0, 16));
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u) acc[u][t] = ksp == 0 ? acc[u][t] + part[t][u] : part[t][u] + acc[u][t];
  }
  if ((p.ks == 1 || p.tick != nullptr) && p.bacc.acc) {
    // BatchNorm sums of the stored values (csrc/bn_acc.h): per channel group u over the lane's 4 pixels,
    // the 16 lanes of the group, then the two pixel-half waves through LDS slots
    const bool two = p.bacc.acc2 != nullptr;
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();  // every wave is done with the halo / weights: LDS is free
    // the epilogue's loads (residual / mask, the BatchNorm inputs and statistics) in flight before the
    // stores, in batches of UB channel groups (register budget): one round trip per batch
    constexpr int UB = TN < 2 ? TN : 2;
#pragma unroll
    for (int u0 = 0; u0 < TN; u0 += UB) {
      C3Pre pre[UB][4];
      BnAccX px[UB][4];
      BnAccChan bc[UB];
#pragma unroll
      for (int du = 0; du < UB; ++du) {
        const int co = co0 + wn * (BN / 2) + 16 * (u0 + du) + 4 * fc;
        bc[du] = bacc_chan(p.bacc, co);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const unsigned bo = c3_boff(p, (long long)tile * kCP + wm * 64 + 32 * (t >> 1) + 2 * fl + (t & 1), co);
          pre[du][t] = c3_preload(p, bo);
          px[du][t] = c3_loadx(p.bacc, bo);
        }
      }
#pragma unroll
      for (int du = 0; du < UB; ++du) {
        const int u = u0 + du;
        const int cl = wn * (BN / 2) + 16 * u + 4 * fc;
        BnAccLane bl;
        bacc_zero(bl);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const long long m = (long long)tile * kCP + wm * 64 + 32 * (t >> 1) + 2 * fl + (t & 1);
          float sv[4];
          c3_store_pre(p, c3_boff(p, m, co0 + cl), acc[u][t], pre[du][t], sv);
          bacc_add4x(bl, p.bacc, bc[du], px[du][t], sv);
        }
        bacc_reduce16(bl, two);
        if (fl == 0) bacc_stash(red, wm, BN, cl, bl);
      }
    }
    __syncthreads();
    bacc_flush(p.bacc, red, 2, BN, co0, p.Cout, tid, 256);
    return;
  }
  if (p.ks > 1 && p.tick == nullptr) {  // raw partials of this split's channel blocks (combine launch)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const long long m = (long long)tile * kCP + wm * 64 + 32 * (t >> 1) + 2 * fl + (t & 1);
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const int co = co0 + wn * (BN / 2) + 16 * u + 4 * fc;
        *reinterpret_cast<f32x4*>(p.ws + ((long long)ksp * p.ntiles * kCP + m) * p.Cout + co) = acc[u][t];
      }
    }
    return;
  }
  C3Pre pre[4][TN];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < TN; ++u)
      pre[t][u] = c3_preload(p, c3_boff(p, (long long)tile * kCP + wm * 64 + 32 * (t >> 1) + 2 * fl + (t & 1),
                                        co0 + wn * (BN / 2) + 16 * u + 4 * fc));
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const long long m = (long long)tile * kCP + wm * 64 + 32 * (t >> 1) + 2 * fl + (t & 1);
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      float sv[4];
      c3_store_pre(p, c3_boff(p, m, co0 + wn * (BN / 2) + 16 * u + 4 * fc), acc[u][t], pre[t][u], sv);
    }
  }
}

// 64 -> 64 channels (ResNet layer 1, forward and data gradient): the whole 9 x 64 x 64 weight block
// (72 KB) stays in LDS for the workgroup's life, so a tap is MFMAs on LDS reads with no staging and no
// barrier.  A persistent workgroup of two 4-wave groups walks 2 x tpw 128-pixel tiles; each group owns
// one halo buffer and prefetches its next tile's halo into registers while it computes the current one
// (the per-tile setup and the halo latency were most of a 9-step workgroup's life in the tiled kernel).
constexpr int kC64XP = 7;             // halo staging passes per group (224 rows)
constexpr int kC64XR = 32 * kC64XP;

// Barrier of one 4-wave group of a workgroup (the workgroup-wide s_barrier would keep the two groups in
// lockstep, so both would sit in their epilogues -- memory latency, no MFMA -- at the same time).  Lane 0
// of each wave adds one to the group's LDS counter; the wave spins until it holds 4 * (barriers passed).
// Release / acquire at workgroup scope order the group's LDS accesses around it.  A bounded spin: the
// four waves of a resident workgroup always arrive, so the bound is never expected to be reached.
__device__ __forceinline__ void group_sync4(unsigned* ctr, unsigned& gen) {
  gen += 4u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int spin = 0; spin < (1 << 24); ++spin) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= gen) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <bool FLIP>
__global__ void __launch_bounds__(512, 1) conv3_halo_c64_kernel(C3P p) {
  __shared__ __attribute__((aligned(16))) bf16 lds[9 * 64 * 64 + 2 * kC64XR * kCS];
  bf16* wl = lds;  // [tap][co][64 ci], XOR-swizzled 128-byte rows
  const int gi = threadIdx.x >> 8;
  const int tid = threadIdx.x & 255, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  bf16* hs = lds + 9 * 64 * 64 + gi * kC64XR * kCS;
  const int tb = blockIdx.x * p.tps;                          // this workgroup's first tile
  const int nt = max(0, min(p.ntiles, tb + p.tps) - tb);
  const int iters = (nt + 1) / 2;                             // group gi: tiles tb + 2 it + gi

  // ---- weights: 576 rows (tap, co) x 8 chunks, 9 per thread
  {
    u32x4_t rw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int idx = threadIdx.x + 512 * i, row = idx >> 3, ch = idx & 7;
      const int tap = row >> 6, co = row & 63;
      rw[i] = cload16(p.w + (long long)co * p.Kpad + (FLIP ? 8 - tap : tap) * 64 + ch * 8);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int idx = threadIdx.x + 512 * i, row = idx >> 3, ch = idx & 7;
      *reinterpret_cast<u32x4_t*>(wl + (row >> 6) * 4096 + wswz(row & 63, ch)) = rw[i];
    }
  }

  // ---- halo staging map (tile independent part)
  const FDiv fper(p.HR2 * p.HW2), fhw2(p.HW2), frw(p.R * p.W), fw(p.W);
  const int ch = tid & 7, r8 = tid >> 3;
  // (halo row hr - 1 and column hc - 1 packed as two 16-bit halves: the epilogue's preloads need the
  // registers; a row past the halo gets -16384, which no image row offset brings back into range)
  int xro[kC64XP], xhw[kC64XP];
#pragma unroll
  for (int i = 0; i < kC64XP; ++i) {
    const int j = r8 + 32 * i;
    const int slot = fper.div(j), rem = j - slot * fper.d;
    const int hr = fhw2.div(rem), hc = rem - hr * p.HW2;
    xro[i] = slot * p.R + hr - 1;
    xhw[i] = (int)((unsigned)(j < p.hrows ? hr - 1 : -16384) << 16) | ((hc - 1) & 0xffff);
  }
  u32x4_t rh[kC64XP];
  auto load_halo = [&](int t) {
    const int gr0 = t * p.rows_per_tile, oh0 = gr0 % p.H;
#pragma unroll
    for (int i = 0; i < kC64XP; ++i) {
      const int ih = oh0 + (xhw[i] >> 16), iw = (int)(short)(xhw[i] & 0xffff);
      const bool v = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      rh[i] = cload16(v ? (const void*)(p.src + ((long long)(gr0 + xro[i]) * p.W + iw) * 64 + ch * 8)
                        : (const void*)&kZeroC3);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int i = 0; i < kC64XP; ++i)
      if (r8 + 32 * i < p.hrows) *reinterpret_cast<u32x4_t*>(hs + (r8 + 32 * i) * kCS + ch * 8) = rh[i];
  };

  // ---- fragment map (as conv3_halo_kernel<64>)
  const int fl = lane & 15, fc = lane >> 4;
  int hoff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int s = wm * 64 + 32 * (t >> 1) + 2 * fl + (t & 1);
    const int slot = frw.div(s), q = s - slot * frw.d, rr = fw.div(q), cc = q - rr * p.W;
    hoff[t] = ((slot * p.HR2 + rr) * p.HW2 + cc) * kCS + fc * 8;
  }
  int woff[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h) woff[u][h] = wswz(wn * 32 + 16 * u + fl, fc + 4 * h);

  // BatchNorm sums of every stored value of this workgroup's tiles (csrc/bn_acc.h), kept per lane; the
  // per-channel statistics they need (mode 1) sit in LDS, not in 32 registers for the kernel's life
  const bool bacc = p.bacc.acc != nullptr, two = p.bacc.acc2 != nullptr;
  __shared__ float bcs[4][64];  // mean, invstd, mean2, invstd2
  BnAccLane bl[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) bacc_zero(bl[u]);
  if (bacc && threadIdx.x < 16) {
    const BnAccChan c = bacc_chan(p.bacc, 4 * threadIdx.x);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bcs[0][4 * threadIdx.x + r] = c.mu[r];
      bcs[1][4 * threadIdx.x + r] = c.is[r];
      bcs[2][4 * threadIdx.x + r] = c.mu2[r];
      bcs[3][4 * threadIdx.x + r] = c.is2[r];
    }
  }
  auto chan = [&](int col) {
    BnAccChan c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      c.mu[r] = bcs[0][col + r];
      c.is[r] = bcs[1][col + r];
      c.mu2[r] = bcs[2][col + r];
      c.is2[r] = bcs[3][col + r];
    }
    return c;
  };
  __shared__ unsigned gsync[2];  // group barrier counters (group_sync4)
  if (threadIdx.x < 2) gsync[threadIdx.x] = 0u;
  unsigned ggen = 0u;
  if (nt > gi) load_halo(tb + gi);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (nt > gi) store_halo();
  __syncthreads();
  // the two groups run their tiles independently from here (group barriers only): one group's
  // epilogue overlaps the other's MFMAs
  for (int it = 0; it < iters; ++it) {
    const int t = tb + 2 * it + gi;
    const bool cur = 2 * it + gi < nt, nxt = 2 * (it + 1) + gi < nt;
    if (nxt) load_halo(t + 2);
    if (cur) {
      f32x4 acc[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[u][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int toff = (kh * p.HW2 + kw) * kCS;
          const bf16* wt = wl + (kh * 3 + kw) * 4096;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            bf16x8 fa[2], fb[4];
#pragma unroll
            for (int u = 0; u < 2; ++u) fa[u] = *reinterpret_cast<const bf16x8*>(wt + woff[u][h]);
#pragma unroll
            for (int q = 0; q < 4; ++q) fb[q] = *reinterpret_cast<const bf16x8*>(hs + hoff[q] + toff + 32 * h);
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[u][q] = mfma16x16x32(fa[u], fb[q], acc[u][q]);
          }
        }
      group_sync4(&gsync[gi], ggen);  // this group's waves are done with the halo
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (nxt) store_halo();
      // the epilogue's loads (mask / residual, BatchNorm inputs) in flight before the stores, in two
      // batches of pixel tiles (register budget: the whole tile at once spilled); the next halo's
      // registers are free by now
#pragma unroll
      for (int q0 = 0; q0 < 4; q0 += 2) {
        C3Pre pre[2][2];
        BnAccX px[2][2];
#pragma unroll
        for (int dq = 0; dq < 2; ++dq) {
          const long long m = (long long)t * kCP + wm * 64 + 32 * ((q0 + dq) >> 1) + 2 * fl + ((q0 + dq) & 1);
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const unsigned bo = c3_boff(p, m, wn * 32 + 16 * u + 4 * fc);
            pre[dq][u] = c3_preload(p, bo);
            px[dq][u] = c3_loadx(p.bacc, bo);
          }
        }
#pragma unroll
        for (int dq = 0; dq < 2; ++dq) {
          const int q = q0 + dq;
          const long long m = (long long)t * kCP + wm * 64 + 32 * (q >> 1) + 2 * fl + (q & 1);
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            float sv[4];
            c3_store_pre(p, c3_boff(p, m, wn * 32 + 16 * u + 4 * fc), acc[u][q], pre[dq][u], sv);
            if (bacc) bacc_add4x(bl[u], p.bacc, chan(wn * 32 + 16 * u + 4 * fc), px[dq][u], sv);
          }
        }
      }
      group_sync4(&gsync[gi], ggen);  // the next halo is stored
    } else {
      break;  // (this group has no tile left; the other may still be running)
    }
  }
  __syncthreads();  // both groups done
  if (bacc) {  // the halo buffers are free
    float* red = reinterpret_cast<float*>(lds + 9 * 64 * 64);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      bacc_reduce16(bl[u], two);
      if (fl == 0) bacc_stash(red, gi * 2 + wm, 64, wn * 32 + 16 * u + 4 * fc, bl[u]);
    }
    __syncthreads();
    bacc_flush(p.bacc, red, 4, 64, 0, 64, threadIdx.x, 512);
  }
}

// per-tile tickets of the folded split-K combine: zeroed once, each tile's last arriver resets its own, so
// a buffer is zero between launches (graph replays included).  One buffer per (device, stream): two folded
// convs running at once on different streams, or on another device of the process, never share tickets
// (ADVICE r5).  Each device's buffers come from a pool allocated and zeroed outside any stream capture at
// the device's first request (null -- the combine launch -- if that request comes during a capture or
// the pool is used up); a capture stream takes a pool buffer without any allocation.  Folded convs on
// one stream run in stream order, so they share that stream's buffer safely.
constexpr int kC3Tickets = 1024;
constexpr int kC3Pool = 64;  // buffers per device (torch's stream pools are finite, so are the keys)
unsigned* c3_tickets(hipStream_t st) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, unsigned*> tab;
  static std::map<int, std::pair<unsigned*, int>> pool;  // device -> (base, buffers handed out)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = tab.find({dev, st});
  if (it != tab.end()) return it->second;
  auto pit = pool.find(dev);
  if (pit == pool.end()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    unsigned* b = nullptr;
    const size_t bytes = (size_t)kC3Pool * kC3Tickets * sizeof(unsigned);
    if (hipMalloc(&b, bytes) != hipSuccess) return nullptr;
    if (hipMemset(b, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(b);
      return nullptr;
    }
    pit = pool.emplace(dev, std::make_pair(b, 0)).first;
  }
  if (pit->second.second >= kC3Pool) return nullptr;
  unsigned* t = pit->second.first + (size_t)pit->second.second++ * kC3Tickets;
  tab[{dev, st}] = t;
  return t;
}

bool c3_geom(int H, int W, int& R, int& TI) {
  if (W < 4 || W > 64 || kCP % W != 0) return false;
  const int rpt = kCP / W;
  if (rpt <= H) {
    if (H % rpt != 0) return false;
    R = rpt, TI = 1;
  } else {
    if (rpt % H != 0) return false;
    R = H, TI = rpt / H;
  }
  return TI * (R + 2) * (W + 2) <= kCXR && TI * (R + 2) * (W == 16 ? 32 : W + 2) <= kCXL;
}

}  // namespace

bool conv3_halo_supported(const IGemmArgs& a, int mode) {
  static const int on = diag_int("conv_halo", 1);
  int R, TI;
  if (!on || (mode != MODE_FWD && mode != MODE_DGRAD)) return false;
  return a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.SH == a.OH && a.SW == a.OW && a.SC % 64 == 0 &&
         a.N % 64 == 0 && a.K == 9 * a.SC && a.Kpad >= a.K && a.Kpad % 8 == 0 && a.ldc % 4 == 0 && !a.bias &&
         !a.out_f32 && !a.drop.on && !a.pool_code && !a.bn.part &&
         a.M % kCP == 0 && a.M % (a.OH * a.OW) == 0 && c3_geom(a.OH, a.OW, R, TI) &&
         (long long)a.M * a.ldc * 2 < (1LL << 32) &&  // one 32-bit byte offset per epilogue element
         ((uintptr_t)a.src & 15) == 0 && ((uintptr_t)a.w & 15) == 0 && ((uintptr_t)a.out & 7) == 0 &&
         (((uintptr_t)a.res | (uintptr_t)a.resmask | (uintptr_t)a.mask) & 7) == 0;
}

hipError_t conv3_halo(const IGemmArgs& a, int mode, hipStream_t st) {
  C3P p;
  int R = 0, TI = 0;
  c3_geom(a.OH, a.OW, R, TI);
  p.src = a.src, p.w = a.w, p.res = a.res, p.resmask = a.resmask, p.mask = a.mask;
  p.out = reinterpret_cast<bf16*>(a.out);
  p.H = a.OH, p.W = a.OW, p.Cin = a.SC, p.Cout = a.N, p.Kpad = a.Kpad, p.ldc = a.ldc;
  p.R = R, p.HW2 = a.OW + 2, p.HR2 = R + 2, p.hrows = TI * (R + 2) * (a.OW + 2), p.rows_per_tile = kCP / a.OW;
  // W = 16: the 32 pixels of a pixel-interleaved MFMA tile span two image rows; an image-row pitch of
  // W + 16 halo rows keeps their bank slots 16 apart, so the two-chunk ds_read_b128 groups stay
  // conflict-free (24 % conflict cycles on layer 2 with the W + 2 pitch)
  static const int pitch16 = diag_int("conv_halo_pitch16", 1);
  p.HWP = (a.OW == 16 && pitch16) ? 32 : a.OW + 2;
  p.ntiles = a.M / kCP;
  p.relu = a.relu;
  p.alpha = a.alpha;
  p.bacc = a.bacc;
  static const int c64 = diag_int("conv_halo_c64", 1);
  if (c64 && a.SC == 64 && a.N == 64 && p.hrows <= kC64XR && p.ntiles >= 512) {
    // weights resident: one 8-wave workgroup per CU, tiles split evenly (an even count per workgroup)
    p.tps = 2 * cdiv(p.ntiles, 2 * 256);
    p.nco = 1, p.ks = 1, p.cbs = 1, p.ws = nullptr;
    const dim3 grid(cdiv(p.ntiles, p.tps));
    if (mode == MODE_DGRAD) hipLaunchKernelGGL(conv3_halo_c64_kernel<true>, grid, dim3(512), 0, st, p);
    else hipLaunchKernelGGL(conv3_halo_c64_kernel<false>, grid, dim3(512), 0, st, p);
    return hipGetLastError();
  }
  // 128-channel tiles while that still gives >= 2 workgroups per CU
  const bool wide = a.N % 128 == 0 && (long long)p.ntiles * (a.N / 128) >= 512;
  const bool flip = mode == MODE_DGRAD;
  p.nco = a.N / (wide ? 128 : 64);
  // under-filled launches (ResNet layer 4: 256 workgroups of 72 steps) split the input channel blocks
  // over workgroups when the caller provides igemm64's split-K workspace; a fixed-order combine applies
  // the epilogue
  const int ncb = a.SC / 64;
  p.ks = 1, p.cbs = ncb, p.ws = nullptr;
  static const int ksplit = diag_int("conv_halo_splitk", 1);
  if (ksplit && a.splitk_ws && p.ntiles * p.nco < 512) {
    const long long wsf = igemm64_splitk_floats(a, mode);  // what the caller allocated
    static const int ksmax = diag_int("conv_halo_ks", 2);  // 2 measured faster than 4 (layer 4: 38.4 vs 43.1 us)
    int ks = 1;
    while (ks < ksmax && ncb % (2 * ks) == 0 && (long long)p.ntiles * p.nco * ks * 2 <= 1024 &&
           (long long)(2 * ks) * a.M * a.N <= wsf)
      ks *= 2;
    if (ks > 1) p.ks = ks, p.cbs = ncb / ks, p.ws = a.splitk_ws;
  }
  // two splits: the tile's last arriver combines and runs the epilogue in this launch (c3_tickets); the
  // combine launch otherwise
  p.tick = nullptr;
  static const int fold = diag_int("conv_halo_fold", 1);
  if (fold && p.ks == 2 && p.ntiles * p.nco <= kC3Tickets &&
      (long long)p.ks * p.ntiles * kCP * p.Cout * 4 < (1LL << 31))
    p.tick = c3_tickets(st);
  const dim3 grid(p.ntiles * p.nco * p.ks);
  if (wide) {
    if (flip) hipLaunchKernelGGL((conv3_halo_kernel<128, true, false>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((conv3_halo_kernel<128, false, false>), grid, dim3(256), 0, st, p);
  } else {
    static const int row = diag_int("conv_halo_row", 1);  // a kernel row per step (conv3_halo_kernel ROW)
    if (row) {
      if (flip) hipLaunchKernelGGL((conv3_halo_kernel<64, true, true>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((conv3_halo_kernel<64, false, true>), grid, dim3(256), 0, st, p);
    } else {
      if (flip) hipLaunchKernelGGL((conv3_halo_kernel<64, true, false>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((conv3_halo_kernel<64, false, false>), grid, dim3(256), 0, st, p);
    }
  }
  DFA_HIP_CHECK(hipGetLastError());
  if (p.ks > 1 && p.tick == nullptr) {  // the combine applies the epilogue (and the BatchNorm sums)
    IGemmArgs c = a;
    c.splits = p.ks;
    return igemm64_splitk_combine(c, st);
  }
  return hipGetLastError();
}

}  // namespace dfa
