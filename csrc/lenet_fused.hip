// Whole-network LeNet-5 training step in three launches (gfx950 / MI355X).
//
// The reference trains its MNIST CNNs with one tf.js op per layer and per direction
// (DistributedTfModel.fit, /root/reference/src/common/models.ts:137-142).  The
// per-layer design of this repo (convpool.hip + mlphead.hip: 9 launches per step) left LeNet-5 at
// 0.174 ms per 4096-image step, ~60 us of it fixed per-launch cost and the rest VALU-bound im2col.
// LeNet-5 is small enough that a workgroup can keep EVERYTHING of its images on chip, so here:
//
//   lenet_prep_kernel    the conv weights of this step as ready-made MFMA B fragments (banded conv1,
//                        conv2 forward, pair-banded conv2 data gradient): 37 x 1 KB, read by every
//                        workgroup with one 16-byte load per lane and fragment
//   lenet_train_kernel   one workgroup = 8 images (fewer at small batches: lenet_ipw), 8 waves, ~78 KB of
//                        LDS (two workgroups per CU):
//     conv1 5x5 'same' + bias + ReLU + 2x2 max-pool   MFMA with a banded (Toeplitz) weight operand:
//                          A = 32 consecutive input pixels of a row (one aligned ds_read_b128; odd
//                          output columns read a copy of the image shifted by one pixel), so the
//                          4 accumulator rows of a lane are one 2x2 pool window: the pool is in-lane
//     conv2 5x5 + bias + ReLU + pool                  implicit GEMM, output rows in pool-window order
//     dense 400-120-84-10 + softmax-CE + backward     MFMA, weights streamed from L2
//     conv2 weight gradient                           ds_read_b64_tr_b16 transposed reads of both
//                          operands from their natural NHWC images; bias = a column of ones
//     conv2 data gradient                             pair-banded MFMA (two output columns per row)
//     conv1 weight gradient                           A fragments unpooled in registers from the pool
//                          gradient + argmax codes, B = 4 dword reads of the (shifted) input image
//   and writes per-workgroup conv gradient partials plus transposed dense activations/gradients;
//   lenet_reduce_kernel  deterministic reductions: conv partials (one wave per parameter over all
//                        workgroups), dense weight gradients over the batch (MFMA, K = batch), loss.
#include "common.h"
#include "diag.h"
#include "kernels.h"
#include "lenet_frag.h"
#include "ll_exchange.h"
#include "optim_device.h"
#include "ps_device.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace dfa {
namespace {

constexpr int IMG = 8;     // images per workgroup
constexpr int NT = 512;    // threads per workgroup: 8 waves, 2 workgroups per CU = 4 waves per SIMD
constexpr int NW = NT / 64;
constexpr int ccdiv(int a, int b) { return (a + b - 1) / b; }
// LDS carve (bytes), every offset 16-byte aligned
constexpr int XS_ELEMS = IMG * 1024 + 32;           // [8][32][32] padded input (+ tail pad)
constexpr int OFF_XS = 0;
constexpr int OFF_P1 = OFF_XS + XS_ELEMS * 2;       // [8][196][8] bf16 pool1 output, later its gradient
constexpr int OFF_C1 = OFF_P1 + IMG * 196 * 16;     // [8][196] u32 pool1 codes (3 bits per channel)
// conv2 output rows (the GEMM M of phases B / E / F) are numbered per image in blocks of DC2_RS = 104:
// row m = image * 104 + t, t = window * 4 + position < 100 (t = 100 .. 103: padding, a zero gradient)
constexpr int DC2_RS = 104;
constexpr int NM = IMG * DC2_RS;                    // 832 padded conv2 output rows
constexpr int OFF_K = OFF_C1 + IMG * 196 * 4;       // 32 B ones (bf16)
constexpr int OFF_PX = OFF_K + 32;                  // conv2 output row -> P1 pixel [832] u16 (host-built)
constexpr int OFF_FT = OFF_PX + NM * 2;             // conv2 dgrad table [98][2][16] u8 (host-built)
constexpr int OFF_W = OFF_FT + 98 * 2 * 16;         // f32: b1 [6], b2 [16], then 8 int labels
constexpr int OFF_KZ = OFF_W + 128;                 // 32 B zeros (phase G's zero columns)
// the union starts where it always did (OFF_XS1's bank offset from Xs, and so phase A / G's
// conflict-free reads, depend on it)
constexpr int OFF_U = OFF_KZ + 32;
// phases A and G: input shifted left by one pixel; 32 bytes into the union so that its rows sit 24 banks
// from Xs's (the A-operand reads of phase A and the B-operand reads of phase G are then conflict-free:
// scripts/lds_sim.py)
constexpr int OFF_XS1 = OFF_U + 32;
constexpr int LD0 = 424, LD1 = 136, LD2 = 104, LD3 = 40;  // dense row strides (elements)
constexpr int OFF_H0 = OFF_U;
constexpr int OFF_H1 = OFF_H0 + IMG * LD0 * 2;
constexpr int OFF_H2 = OFF_H1 + IMG * LD1 * 2;
constexpr int OFF_Z3 = OFF_H2 + IMG * LD2 * 2;
constexpr int OFF_Z2 = OFF_Z3 + IMG * LD3 * 2;
constexpr int OFF_Z1 = OFF_Z2 + IMG * LD2 * 2;
constexpr int OFF_ZR = OFF_Z1 + IMG * LD1 * 2;      // zero row [LD0] (A rows 8..15 of every dense GEMM)
constexpr int OFF_LG = OFF_ZR + LD0 * 2;            // [8][16] f32 logits
constexpr int OFF_C2 = OFF_LG + IMG * 16 * 4;       // [8][25][16] u8 pool2 codes
constexpr int U_DENSE = OFF_C2 + IMG * 25 * 16 - OFF_U;
constexpr int OFF_DC2 = OFF_U;                      // [832][16] bf16 conv2 output gradient (padded rows)
constexpr int U_DC2 = NM * 16 * 2;
constexpr int OFF_RED = OFF_XS1 + XS_ELEMS * 2;     // [4][16][32] f32 cross-wave conv1 wgrad sums
constexpr int U_G = 32 + XS_ELEMS * 2 + 4 * 16 * 32 * 4;
// conv2 output-gradient row t of an image is stored at row dc2_swz(t) of the image's 104-row block: the
// gathered A-operand reads of phase F then spread over the banks (scripts/lds_sim.py), and phase F's
// table holds the swizzled row itself (no per-step swizzle arithmetic).  The padding rows hold zeros:
// phase F's "no tap" entries read one (dc2_swz(100) = 96).
__device__ __forceinline__ int dc2_swz(int t) { return t ^ ((t >> 3) & 7); }
constexpr int cmax(int a, int b) { return a > b ? a : b; }
// dense biases (f32: dense-1 [120], dense-2 [84], dense-3 [10]), staged in phase 0: read from LDS, a
// bias load never waits behind the weight prefetches issued before it
constexpr int OFF_DB = OFF_U + (cmax(cmax(U_DENSE, U_DC2), U_G) + 15) / 16 * 16;
constexpr int OFF_ST = OFF_DB + 864;                // u64 [16] diagnostic phase clocks (LN_STAMP)
constexpr int LDS_BYTES = OFF_ST + 128;
static_assert(OFF_U == OFF_C1 + IMG * 196 * 4 + 128 + 98 * 2 * 16 + 800 * 2 + 128 && OFF_U % 16 == 0 && OFF_KZ % 16 == 0 && OFF_H1 % 16 == 0 && OFF_ZR % 16 == 0 && OFF_C2 % 16 == 0 && OFF_RED % 16 == 0 && OFF_DB % 16 == 0 && OFF_ST % 16 == 0 &&
                  OFF_PX % 16 == 0 && OFF_W % 16 == 0,
              "LDS carve must stay 16-byte aligned");
static_assert(2 * LDS_BYTES <= 160 * 1024, "two workgroups per CU");

typedef __bf16 bf16x4_vs __attribute__((__vector_size__(8)));

// diagnostic per-phase clocks (scripts/lenetstamps.py): [grid][16] s_memtime after each phase's barrier,
// kept in LDS and written out at the end (a global store mid-kernel makes the compiler's wait-count pass
// wait for every load in flight at the next join, stamps or not)
#define LN_STAMP(slot)                                                            \
  do {                                                                            \
    if (stamps) {                                                                 \
      __builtin_amdgcn_sched_barrier(0);                                          \
      unsigned long long t_;                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                          \
      if (threadIdx.x == 0) STMP[(slot)] = t_;                                    \
    }                                                                             \
  } while (0)

// 16-lane (DPP row) reductions: every lane of the row gets the result (xor 1, xor 2, half-row mirror,
// row mirror: four VALU data moves instead of four LDS permute round trips)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}

__device__ __forceinline__ bf16x4 tr_read(const bf16* p) {
  auto* lp = (__attribute__((address_space(3))) bf16*)(const_cast<bf16*>(p));
  const bf16x4_vs v =
      __builtin_amdgcn_ds_read_tr16_b64_v4bf16(reinterpret_cast<__attribute__((address_space(3))) bf16x4_vs*>(lp));
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    r[e] = a[e];
    r[e + 4] = b[e];
  }
  return r;
}
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void st8(bf16* p, const bf16x8& v) { *reinterpret_cast<bf16x8*>(p) = v; }
__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int e = 0; e < 8; ++e) z[e] = (bf16)0.f;
  return z;
}

// Xs1[e] = Xs[e + 1]: the padded images shifted left by one pixel (dword-aligned funnel shift)
__device__ __forceinline__ void build_shift1(const bf16* Xs, bf16* Xs1) {
  for (int t = threadIdx.x; t < XS_ELEMS / 8 - 1; t += NT) {
    const uint4 lo = *reinterpret_cast<const uint4*>(Xs + 8 * t);
    const unsigned nx = *reinterpret_cast<const unsigned*>(Xs + 8 * t + 8);
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(lo.y, lo.x, 2);
    o.y = __builtin_amdgcn_alignbyte(lo.z, lo.y, 2);
    o.z = __builtin_amdgcn_alignbyte(lo.w, lo.z, 2);
    o.w = __builtin_amdgcn_alignbyte(nx, lo.w, 2);
    *reinterpret_cast<uint4*>(Xs1 + 8 * t) = o;
  }
}

// 2x2 max-pool of one window (elements in (dy, dx) row-major order) + ReLU; code = argmax position
// (first maximum), 4 = inactive (no gradient flows: pooled value <= 0).
__device__ __forceinline__ void pool4(float a00, float a01, float a10, float a11, float& best, unsigned& code) {
  best = a00;
  code = 0;
  if (a01 > best) { best = a01; code = 1; }
  if (a10 > best) { best = a10; code = 2; }
  if (a11 > best) { best = a11; code = 3; }
  if (!(best > 0.f)) { best = 0.f; code = 4; }
}

// Weight fragments of one dense GEMM for the tiles t = w + NW tt this wave owns, loaded ahead of use so
// that the L2 latency of layer l + 1's weights hides behind layer l (W rows of 32 * KS elements).
template <int KS, int NTW>
struct DenseFrags {
  bf16x8 b[NTW][KS];
};
template <int KS, int NTW>
__device__ __forceinline__ void dense_load(DenseFrags<KS, NTW>& f, const bf16* __restrict__ W, int ntiles) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    const int t = w + NW * tt;
    if (t < ntiles) {
      const bf16* wrow = W + (long long)(16 * t + i) * (32 * KS) + 8 * g;
#pragma unroll
      for (int s = 0; s < KS; ++s) f.b[tt][s] = ld8(wrow + 32 * s);
    }
  }
}

// Z[8 rows][N] = A[8][Kpad] W^T (+bias, ReLU); A rows 8..15 of the MFMA tile read the zero row.
template <int KS, int NTW>
__device__ __forceinline__ void dense_fwd(const DenseFrags<KS, NTW>& f, const bf16* A, int lda, const bf16* zr,
                                          const float* __restrict__ bias, int N, bool relu, bf16* out, int ldo,
                                          float* out32, bf16* __restrict__ hT, int ldt, int r0, int rows) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  const int ntiles = (N + 15) / 16;
  const bf16* arow = (i < IMG ? A + i * lda : zr) + 8 * g;
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    const int t = w + NW * tt;
    if (t >= ntiles) break;
    const int n = 16 * t + i;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = mfma16x16x32(ld8(arow + 32 * s), f.b[tt][s], acc);
    if (g >= 2) continue;  // output rows 8..15 are padding
    const float bv = (bias != nullptr && n < N) ? bias[n] : 0.f;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = acc[r] + bv;
      if (relu) v[r] = fmaxf(v[r], 0.f);
      if (n >= N) v[r] = 0.f;
      const int row = 4 * g + r;
      if (out) out[row * ldo + n] = f2bf(v[r]);
      if (out32) out32[row * 16 + (n & 15)] = v[r];
    }
    if (hT != nullptr && n < N) {
      bf16* dst = hT + (long long)n * ldt + r0 + 4 * g;
      if (4 * g + 4 <= rows) {
        bf16x4 pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk[r] = f2bf(v[r]);
        *reinterpret_cast<bf16x4*>(dst) = pk;
      } else {
        for (int r = 0; r < 4; ++r)
          if (4 * g + r < rows) dst[r] = f2bf(v[r]);
      }
    }
  }
}

// dA[8][K] = dZ[8][32*KS] Wt^T, masked by (mask > 0); also dZ^T rows for the weight gradient.
template <int KS, int NTW>
__device__ __forceinline__ void dense_bwd(const DenseFrags<KS, NTW>& f, const bf16* dZ, int ldz, const bf16* zr,
                                          int K, const bf16* mask, int ldm, bf16* out, int ldo,
                                          bf16* __restrict__ gT, int ldt, int r0, int rows) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  const int ktiles = (K + 15) / 16;
  const bf16* zrow = (i < IMG ? dZ + i * ldz : zr) + 8 * g;
#pragma unroll
  for (int tt = 0; tt < NTW; ++tt) {
    const int t = w + NW * tt;
    if (t >= ktiles) break;
    const int j = 16 * t + i;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = mfma16x16x32(ld8(zrow + 32 * s), f.b[tt][s], acc);
    if (g >= 2) continue;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * g + r;
      v[r] = acc[r];
      if (mask != nullptr && !((float)mask[row * ldm + j] > 0.f)) v[r] = 0.f;
      if (j >= K) v[r] = 0.f;
      out[row * ldo + j] = f2bf(v[r]);
    }
    if (gT != nullptr && j < K) {
      bf16* dst = gT + (long long)j * ldt + r0 + 4 * g;
      if (4 * g + 4 <= rows) {
        bf16x4 pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk[r] = f2bf(v[r]);
        *reinterpret_cast<bf16x4*>(dst) = pk;
      } else {
        for (int r = 0; r < 4; ++r)
          if (4 * g + r < rows) dst[r] = f2bf(v[r]);
      }
    }
  }
}

// Image group (IMG images) of train workgroup b of nb: XCD-aware, so that with round-robin dispatch
// (XCD = b mod 8) the groups of XCD x are contiguous -- its workgroups write whole 128-byte lines of the
// transposed activation / gradient rows (no line shared by two XCDs' L2s) and the reduce launch's
// batch chunk x is exactly the columns XCD x wrote.  The tail (nb mod 8 workgroups) keeps b.
__device__ __forceinline__ int lenet_img_group(int b, int nb) {
  const int per = nb / 8;
  if (b >= 8 * per) return b;
  return (b & 7) * per + (b >> 3);
}

// async PS admission of this step's gradient (the extra workgroup of the train launch, see lenet_train):
// lock-free CAS on the shared version, decision published for the reduce launch's owners (epoch-tagged
// with that launch's epoch, which no one advances before it runs), the refresh minimum recorded, then the
// microbatch's completion.
// Owner-applies (p.owner_ring > 0, reduce mode 4): no per-element remote atomic anywhere.  At the start of the
// reduce launch, workgroup 0 (dispatched first; one thread per shard, in parallel) takes the drain lock of every
// shard nobody else is draining and decides how many flagged inbox slots (in sequence order from the shard's
// drained prefix) this launch adds into it; the decisions go out as one {epoch, count, first} word per shard
// (ps_owner_drain_words), which the slot owners read after their jobs.  Deciding here rather than at the
// admission (the train launch's start, ~50 us earlier) keeps the locks for one reduce launch only and lets
// the refresh include every gradient flagged until this launch starts.  The refresh the owners emit contains,
// on every element, each shard's drained prefix (P + n for the shards this launch drains, the prefix read
// before any shard read otherwise) and -- when admitted with sequence number q and every prefix is q -- this
// gradient itself, which the owners add to the values they emit: that count is the refresh minimum
// (ps_device.h).  The own gradient reaches the shards through the inboxes: every owner stores -lr * g of its
// elements into ring slot q % R of the element's shard inbox (plain system-scope stores), the launch's last
// arrival flags the slot at every owner once they have all landed (lenet_ps_arrive).
// (threads 0 .. nshards - 1 of workgroup 0; s_cnt: LDS [kP2PMaxRanks])
__device__ __forceinline__ void lenet_ps_owner_decide(const PSArgs& p, unsigned* s_cnt) {
  const int k = threadIdx.x;
  if (k < p.nshards) {
    const unsigned ep = __hip_atomic_load(p.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const unsigned R = (unsigned)p.owner_ring;
    const unsigned pre = __hip_atomic_load(p.pref + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned P = 0, n = 0, c = pre, free_ = 0;
    if (__hip_atomic_compare_exchange_strong(p.dlock + k, &free_, (unsigned)p.rank + 1u, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
      P = __hip_atomic_load(p.pref + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned* fl = ps_inbox_flags(p, k);
      while (n < R && n < 255u &&
             __hip_atomic_load(const_cast<unsigned*>(fl) + (P + n) % R, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ==
                 P + n + 1u)
        ++n;
      if (n == 0) __hip_atomic_store(p.dlock + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      c = P + n;
    }
    __hip_atomic_store(ps_owner_drain_words(p) + k, ps_owner_word(ep, n, P), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_cnt[k] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned cnt = 0xffffffffu;
    for (int j = 0; j < p.nshards; ++j) cnt = s_cnt[j] < cnt ? s_cnt[j] : cnt;
    // the admission ran in the train launch: its decision and sequence number are here
    const unsigned dec = __hip_atomic_load(p.scratch + kPSDecision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 7u;
    if (dec == kPSAccept && cnt == p.scratch[kPSSeq]) cnt += 1u;  // the owners add this gradient to what they emit
    if (dec == kPSAccept || dec == kPSReject) ps_note_refresh(p, cnt);
  }
}

__device__ __forceinline__ void lenet_ps_admission(const PSArgs& p, bool excl) {
  const long long bid = *p.bid_out;  // (the reduce launch's claim workgroup overwrites it after the decision)
  const unsigned applied0 = ps_read_applied(p);
  const unsigned ep = __hip_atomic_load(p.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const unsigned dec = ps_admit(p, false);  // (consumes the previous launch's record first)
  const bool owner = p.owner_ring > 0;
  // the owners refresh (add to or read the shards) only after this decision, so every one of their
  // refreshes contains at least applied0 fully applied gradients (+ this one when admitted)
  if (!owner && (dec == kPSAccept || dec == kPSReject)) ps_note_refresh(p, applied0 + (dec == kPSAccept ? 1u : 0u));
  // relaxed: the decision's readers are the next (reduce) launch, behind the kernel boundary (a release
  // here wrote back this XCD's L2 under the running train kernel)
  __hip_atomic_store(p.scratch + kPSDecision, (ep << 3) | dec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (excl) {
    // one rank (reduce mode 3): this launch's epoch is current from here on, and the count of applied
    // gradients can include this one already -- its only reader is this rank's next admission, which
    // follows the reduce launch that applies it
    __hip_atomic_store(p.scratch + kPSEpoch, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dec == kPSAccept) ps_publish_applied(p);
  }
  if (dec == kPSAccept && p.done_epoch != nullptr) complete_microbatch(p, bid);
}

// TRIM (a.ipw < IMG, small batches): the per-image loops (conv1, conv2, conv2 weight and data gradient,
// conv1 weight gradient) run over the tiles of this workgroup's live images only; the rest of the LDS images
// stay as phase 0 left them (zero input, zero output gradient), so the skipped tiles would only have added
// zeros.  TRIM = false is the full-batch kernel, every bound a compile-time constant.
template <bool TRIM>
__global__ void __launch_bounds__(NT, 2 * NT / 256) lenet_train_kernel(LeNetArgs a) {
  if ((int)blockIdx.x >= a.nblk) {  // async PS: the admission workgroup
    if (a.ps_admit && threadIdx.x == 0) lenet_ps_admission(a.ps, a.ps_excl != 0);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Xs = reinterpret_cast<bf16*>(smem + OFF_XS);
  bf16* Xs1 = reinterpret_cast<bf16*>(smem + OFF_XS1);
  bf16* P1 = reinterpret_cast<bf16*>(smem + OFF_P1);
  unsigned* C1 = reinterpret_cast<unsigned*>(smem + OFF_C1);
  bf16* KO = reinterpret_cast<bf16*>(smem + OFF_K);       // 16 ones
  unsigned char* FT = reinterpret_cast<unsigned char*>(smem + OFF_FT);
  unsigned short* PX = reinterpret_cast<unsigned short*>(smem + OFF_PX);
  float* WS = reinterpret_cast<float*>(smem + OFF_W);       // b1[6] b2[16]
  bf16* H0 = reinterpret_cast<bf16*>(smem + OFF_H0);
  bf16* H1 = reinterpret_cast<bf16*>(smem + OFF_H1);
  bf16* H2 = reinterpret_cast<bf16*>(smem + OFF_H2);
  bf16* Z3 = reinterpret_cast<bf16*>(smem + OFF_Z3);
  bf16* Z2 = reinterpret_cast<bf16*>(smem + OFF_Z2);
  bf16* Z1 = reinterpret_cast<bf16*>(smem + OFF_Z1);
  bf16* ZR = reinterpret_cast<bf16*>(smem + OFF_ZR);
  float* LG = reinterpret_cast<float*>(smem + OFF_LG);
  unsigned char* C2 = reinterpret_cast<unsigned char*>(smem + OFF_C2);
  bf16* DC2 = reinterpret_cast<bf16*>(smem + OFF_DC2);
  float* RED = reinterpret_cast<float*>(smem + OFF_RED);

  // the wave index in an SGPR: loops and tile selects over it become scalar branches (tid >> 6 was
  // treated as divergent: exec-mask branches, each waiting for all LDS reads in flight)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), i = lane & 15,
            g = lane >> 4;
  const int r0 = lenet_img_group(blockIdx.x, a.nblk) * (TRIM ? a.ipw : IMG);
  const int rows = min(TRIM ? a.ipw : IMG, a.B - r0);
  // per-image loop trip counts (tiles of 16 / 32 rows over rows-of-image blocks of 56, 104, 98, 14)
  const int nA = TRIM ? 2 * ((7 * rows + 1) / 2) : 56;        // conv1: 3.5 M-tiles per image, 2 halves each
  const int nB = TRIM ? (13 * rows + 1) / 2 : NM / 16;        // conv2: 6.5 M-tiles per image
  const int nE = TRIM ? ((13 * rows + 3) / 4 + 1) / 2 * 2 : NM / 32;  // conv2 wgrad: 3.25 steps, paired
  const int nF = TRIM ? (49 * rows + 7) / 8 : 49;             // conv2 dgrad: 6.125 M-tiles per image
  const int nG = TRIM ? 14 * rows : IMG * 14;                 // conv1 wgrad: 14 pool-window rows per image
  const bf16x8* __restrict__ frag = reinterpret_cast<const bf16x8*>(a.frag);
  float* part = a.conv_part + (long long)blockIdx.x * kLeNetConvStride;  // this workgroup's partials
  unsigned long long* const stamps = a.stamps;
  unsigned long long* const STMP = reinterpret_cast<unsigned long long*>(smem + OFF_ST);
  LN_STAMP(0);

  // ---------------------------------------------------------------- phase 0: zero fills, staging
  // Global loads in dependency order (a wait for one load also waits for every load issued before it):
  // first the indices, then the tables / biases, the conv1 fragments and, once its index is back, this
  // thread's input row; everything lands in registers and is stored to LDS after the zero fills.
  const int ximg = tid / 28, xrow = tid - 28 * (tid / 28);  // input row of this thread
  const bool xload = tid < IMG * 28 && ximg < rows;
  const bool lload = tid >= 256 && tid < 256 + IMG && tid - 256 < rows;  // label of image tid - 256
  long long xsrc = 0, lsrc = 0;
  if (xload) xsrc = a.idx ? a.idx[r0 + ximg] : (long long)(r0 + ximg);
  if (lload) lsrc = a.idx ? a.idx[r0 + tid - 256] : (long long)(r0 + tid - 256);
  uint4 tabv = {0u, 0u, 0u, 0u};
  if (tid < 98 * 2) tabv = reinterpret_cast<const uint4*>(a.ftab)[tid];
  else if (tid >= 264 && tid < 264 + NM / 8) tabv = reinterpret_cast<const uint4*>(a.pxtab)[tid - 264];
  static_assert(98 * 2 <= 256 && 264 + NM / 8 <= 448 && 448 + 22 <= NT, "phase 0 staging thread ranges");
  float biasv = 0.f, dbv = 0.f;
  if (tid >= 448 && tid < 448 + 22) biasv = *(tid < 454 ? a.b1 + (tid - 448) : a.b2 + (tid - 454));
  if (tid < 214) dbv = *(tid < 120 ? a.d1b + tid : (tid < 204 ? a.d2b + (tid - 120) : a.d3b + (tid - 204)));
  // conv1 B fragments of this step (lenet_prep_kernel)
  bf16x8 bc[15];
#pragma unroll
  for (int f = 0; f < 15; ++f) bc[f] = frag[(FR_C1 + f) * 64 + lane];
  int lbl = 0;
  if (lload) lbl = a.labels[lsrc < 0 ? 0 : (lsrc >= a.nrows ? a.nrows - 1 : lsrc)];
  unsigned xv[14];
  if (xload) {
    const long long src = xsrc < 0 ? 0 : (xsrc >= a.nrows ? a.nrows - 1 : xsrc);
    if (a.x_u8 != nullptr) {
      const unsigned* p = reinterpret_cast<const unsigned*>(a.x_u8 + src * 784 + xrow * 28);
#pragma unroll
      for (int k = 0; k < 7; ++k) xv[k] = p[k];
    } else {
      const uint2* p = reinterpret_cast<const uint2*>(a.x_bf + src * 784 + xrow * 28);
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const uint2 v = p[k];
        xv[2 * k] = v.x;
        xv[2 * k + 1] = v.y;
      }
    }
  }
  const bf16x8 z8 = zero8();
  // Xs, P1, C1.  P1's channel 6 holds ones: phase E's im2col column (tap 0, channel 6) is then all ones
  // and gives the conv2 bias gradient (conv2's weights of channels 6, 7 are zero, phase F writes channels
  // 0 .. 5 only, phase G reads them only)
  bf16x8 one6 = z8;
  one6[6] = (bf16)1.f;
  for (int e = tid; e < (OFF_K - OFF_XS) / 16; e += NT)
    st8(Xs + 8 * e, (e >= OFF_P1 / 16 && e < OFF_C1 / 16) ? one6 : z8);
  for (int e = tid; e < (OFF_DB - OFF_U) / 16; e += NT) st8(reinterpret_cast<bf16*>(smem + OFF_U) + 8 * e, z8);
  if (tid < 2) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)1.f;
    st8(KO + 8 * tid, o);
  } else if (tid < 4) {
    st8(reinterpret_cast<bf16*>(smem + OFF_KZ) + 8 * (tid - 2), z8);
  }
  if (tid < 98 * 2) reinterpret_cast<uint4*>(FT)[tid] = tabv;
  else if (tid >= 264 && tid < 264 + NM / 8) reinterpret_cast<uint4*>(PX)[tid - 264] = tabv;
  if (tid >= 448 && tid < 448 + 22) WS[tid - 448] = biasv;  // b1 [6], b2 [16]
  float* DB = reinterpret_cast<float*>(smem + OFF_DB);
  if (tid < 214) DB[tid] = dbv;
  // labels of the 8 images (read by the loss phase)
  int* LBL = reinterpret_cast<int*>(WS + 24);
  if (tid >= 256 && tid < 256 + IMG) LBL[tid - 256] = lbl;  // clamped where read (no wait for it here)
  __syncthreads();
  // input rows -> bf16, 2-pixel zero border ('same' padding)
  if (xload) {
    unsigned* dst = reinterpret_cast<unsigned*>(Xs + ximg * 1024 + (xrow + 2) * 32 + 2);
    if (a.x_u8 != nullptr) {
#pragma unroll
      for (int k = 0; k < 7; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float f0 = (float)((xv[k] >> (16 * h)) & 255u) * a.scale;
          const float f1 = (float)((xv[k] >> (16 * h + 8)) & 255u) * a.scale;
          const unsigned lo = __builtin_bit_cast(unsigned short, f2bf(f0));
          const unsigned hi = __builtin_bit_cast(unsigned short, f2bf(f1));
          dst[2 * k + h] = lo | (hi << 16);
        }
    } else {
#pragma unroll
      for (int k = 0; k < 14; ++k) dst[k] = xv[k];
    }
  }
  __syncthreads();
  build_shift1(Xs, Xs1);
  __syncthreads();
  LN_STAMP(1);

  // ---------------------------------------------------------------- phase A: conv1 + ReLU + pool
  // rows m = (image, y, parity): A = row y of the image (parity 1: shifted by one pixel) from column
  // x0; column j of channel-pair tile T = output x = x0 + 2 (j & 7) + parity, channel 2T + (j >> 3).
  // A lane's 4 accumulator rows (y, y+1) x (parity 0, 1) are one 2x2 pool window.
  {
    const float b1c[3] = {WS[(i >> 3)], WS[2 + (i >> 3)], WS[4 + (i >> 3)]};
#pragma unroll 2
    for (int u = w; u < nA; u += NT / 64) {
      const int mt = u >> 1, x0 = (u & 1) * 16;
      const int m = 16 * mt + i;
      const int img = m / 56, rem = m - 56 * (m / 56);
      const bf16* abase = ((rem & 1) ? Xs1 : Xs) + img * 1024 + (rem >> 1) * 32 + x0 + 8 * g;
      f32x4 acc[3];
#pragma unroll
      for (int T = 0; T < 3; ++T) acc[T] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < 5; ++ky) {
        const bf16x8 av = ld8(abase + ky * 32);
#pragma unroll
        for (int T = 0; T < 3; ++T) acc[T] = mfma16x16x32(av, bc[ky * 3 + T], acc[T]);
      }
      const int m0 = 16 * mt + 4 * g;
      const int imgo = m0 / 56, py = (m0 - 56 * (m0 / 56)) >> 2;
      const int px = (x0 >> 1) + (i & 7);
      unsigned cw = 0;
#pragma unroll
      for (int T = 0; T < 3; ++T) {
        float best;
        unsigned code;
        pool4(acc[T][0] + b1c[T], acc[T][1] + b1c[T], acc[T][2] + b1c[T], acc[T][3] + b1c[T], best, code);
        const int c = 2 * T + (i >> 3);
        if (px < 14) P1[((imgo * 14 + py) * 14 + px) * 8 + c] = f2bf(best);
        cw |= code << (3 * c);
      }
      cw |= __shfl_xor(cw, 8, 64);
      if (i < 8 && px < 14) C1[(imgo * 14 + py) * 14 + px] = cw;
    }
  }
  __syncthreads();
  LN_STAMP(2);

  // ---------------------------------------------------------------- phase B: conv2 + ReLU + pool
  // conv2 fragments first, then the dense-1 weights (L2 latency hidden behind conv2): a wait for the
  // fragments then never waits for the dense-1 loads
  bf16x8 bw[7];
#pragma unroll
  for (int s = 0; s < 7; ++s) bw[s] = frag[(FR_C2 + s) * 64 + lane];
  DenseFrags<13, ccdiv(8, NW)> f1;
  dense_load(f1, a.d1w, 8);
  {
    int toff[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int tap = 4 * s + g;
      toff[s] = tap < 25 ? ((tap / 5) * 14 + (tap - 5 * (tap / 5))) * 8 : 0;
    }
    const float b2 = WS[6 + i];
#pragma unroll 2
    for (int mt = w; mt < nB; mt += NT / 64) {  // padded rows: window 25 of an image is padding
      const bf16* abase = P1 + (int)PX[16 * mt + i] * 8;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 7; ++s) acc = mfma16x16x32(ld8(abase + toff[s]), bw[s], acc);
      const int m0 = 16 * mt + 4 * g;
      const int img0 = m0 / DC2_RS, win0 = (m0 - DC2_RS * img0) >> 2;
      float best;
      unsigned code;
      pool4(acc[0] + b2, acc[1] + b2, acc[2] + b2, acc[3] + b2, best, code);
      if (win0 < 25) {
        H0[img0 * LD0 + win0 * 16 + i] = f2bf(best);
        C2[(img0 * 25 + win0) * 16 + i] = (unsigned char)code;
      }
    }
  }
  __syncthreads();
  LN_STAMP(3);

  // ---------------------------------------------------------------- phase C: dense head, CE, backward
  // H0^T for the dense-1 weight gradient (before H0 is overwritten by its gradient)
  for (int k = tid; k < 400; k += NT) {
    bf16* dst = a.h0T + (long long)k * a.ldt + r0;
    if (rows == IMG) {
      bf16x8 v;
#pragma unroll
      for (int r = 0; r < IMG; ++r) v[r] = H0[r * LD0 + k];
      st8(dst, v);
    } else {
      for (int r = 0; r < rows; ++r) dst[r] = H0[r * LD0 + k];
    }
  }
  DenseFrags<4, ccdiv(6, NW)> f2;
  DenseFrags<3, 1> f3;
  dense_load(f2, a.d2w, 6);
  dense_load(f3, a.d3w, 1);
  dense_fwd(f1, H0, LD0, ZR, DB, 120, true, H1, LD1, nullptr, a.h1T, a.ldt, r0, rows);
  __syncthreads();
  DenseFrags<1, ccdiv(6, NW)> g3;
  DenseFrags<3, ccdiv(8, NW)> g2;
  dense_load(g3, a.d3wt, 6);
  dense_load(g2, a.d2wt, 8);
  dense_fwd(f2, H1, LD1, ZR, DB + 120, 84, true, H2, LD2, nullptr, a.h2T, a.ldt, r0, rows);
  __syncthreads();
  dense_fwd(f3, H2, LD2, ZR, DB + 204, 10, false, nullptr, 0, LG, nullptr, a.ldt, r0, rows);
  __syncthreads();
  LN_STAMP(4);
  // softmax-CE of the 8 images, 16 lanes per image (class c = lane & 15; waves 0 and 1): max / first
  // argmax / sum of exponentials by DPP row reductions, one gradient element per lane; the image's loss
  // and hit go to LG columns 14 / 15 of its row (no lane reads a column >= 10)
  if (tid < IMG * 16) {
    const int r = tid >> 4, c = tid & 15;
    const bool live = r < rows;
    const int y = min(max(LBL[r], 0), 9);
    const float z = c < 10 ? LG[r * 16 + c] : -INFINITY;
    if (a.logits && live && c < 10) a.logits[(long long)(r0 + r) * 10 + c] = z;
    const float mx = row16_max(z);
    // first argmax: the lowest class of this image's 16-lane group holding the maximum
    const unsigned long long hit = __ballot(z == mx);
    const int am = __builtin_ctzll((hit >> (16 * (r & 3))) | 0x10000ull);
    const float e = c < 10 ? __expf(z - mx) : 0.f;
    const float ssum = row16_sum(e);
    if (live && c < 10) {
      const float gv = (e * (1.f / ssum) - (c == y ? 1.f : 0.f)) * a.grad_scale;
      Z3[r * LD3 + c] = f2bf(gv);
      a.dz3T[(long long)c * a.ldt + r0 + r] = f2bf(gv);
    }
    if (c == y) LG[r * 16 + 14] = live ? -(z - mx - __logf(ssum)) : 0.f;
    if (c == 15) LG[r * 16 + 15] = (live && am == y) ? 1.f : 0.f;
  }
  __syncthreads();
  if (tid == 0) {
    float ls = 0.f, cs = 0.f;
#pragma unroll
    for (int r = 0; r < IMG; ++r) {
      ls += LG[r * 16 + 14];
      cs += LG[r * 16 + 15];
    }
    a.loss_part[2 * blockIdx.x] = ls;
    a.loss_part[2 * blockIdx.x + 1] = cs;
  }
  // dense-1 data-gradient weights (64 VGPRs per lane): loaded after the loss, whose shuffles would
  // otherwise push the live fragments past the 128-register budget; the loads overlap dense-3 / dense-2
  // backward
  DenseFrags<4, ccdiv(25, NW)> g1;
  dense_load(g1, a.d1wt, 25);
  __syncthreads();
  LN_STAMP(5);
  dense_bwd(g3, Z3, LD3, ZR, 84, H2, LD2, Z2, LD2, a.dz2T, a.ldt, r0, rows);
  __syncthreads();
  dense_bwd(g2, Z2, LD2, ZR, 120, H1, LD1, Z1, LD1, a.dz1T, a.ldt, r0, rows);
  __syncthreads();
  dense_bwd(g1, Z1, LD1, ZR, 400, H0, LD0, H0, LD0, nullptr, 0, r0, rows);  // in place: dP2
  __syncthreads();
  LN_STAMP(6);

  // ---------------------------------------------------------------- phase D: unpool dP2 -> dC2
  {
    bf16x8 dp[2];
    unsigned long long cd[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int it = tid + k * NT;
      if (it < IMG * 50) {
        const int img = it / 50, rem = it - 50 * (it / 50), win = rem >> 1, nh = rem & 1;
        dp[k] = ld8(H0 + img * LD0 + win * 16 + 8 * nh);
        cd[k] = *reinterpret_cast<const unsigned long long*>(C2 + (img * 25 + win) * 16 + 8 * nh);
      }
    }
    __syncthreads();  // dC2 overlays H0 / codes2
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int it = tid + k * NT;
      if (it < IMG * 50) {
        const int img = it / 50, rem = it - 50 * (it / 50), win = rem >> 1, nh = rem & 1;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = ((cd[k] >> (8 * e)) & 255u) == (unsigned)d ? dp[k][e] : (bf16)0.f;
          st8(DC2 + ((img * DC2_RS + dc2_swz(win * 4 + d)) * 16 + 8 * nh), o);
        }
      }
    }
  }
  if (tid < IMG * 8) {  // the 4 zero rows of every image block (after the overlaid H0 / codes were read)
    const int img = tid >> 3, rr = (tid >> 1) & 3, nh = tid & 1;
    st8(DC2 + ((img * DC2_RS + dc2_swz(100 + rr)) * 16 + 8 * nh), zero8());
  }
  __syncthreads();
  LN_STAMP(7);

  // ---------------------------------------------------------------- phase E: conv2 weight gradient
  // dW2[n][(tap, c)] = sum_m dC2[m][n] im2col(P1)[m][(tap, c)]: both operands by transposed reads;
  // wave w owns the 16-column tiles T = w + NW k (taps 2T, 2T + 1); tap 25 is the bias column of ones.
  bf16x8 bd[15];  // conv2 data-gradient fragments for phase F, in flight during this phase
#pragma unroll
  for (int s = 0; s < 15; ++s) bd[s] = frag[(FR_DG + s) * 64 + lane];
  {
    const int q = (lane & 15) >> 2, p = lane & 3;
    constexpr int KT = ccdiv(13, NW);  // column tiles per wave (13 tiles: taps 0..25, tap 25 unused)
    int toff[KT];  // element offset of the lane's tap (taps >= 25: tap 0, its column is dropped)
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      const int tap = 2 * (w + NW * k) + (p >> 1);
      toff[k] = tap < 25 ? ((tap / 5) * 14 + (tap - 5 * (tap / 5))) * 8 + 4 * (p & 1) : 4 * (p & 1);
    }
    const int ntile = (13 - w + NW - 1) / NW;
    f32x4 acc[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) acc[k] = {0.f, 0.f, 0.f, 0.f};
    // the GEMM's M runs over the padded rows (26 steps of 32; the zero rows add nothing).  Step s + 1's
    // dC2 rows and pixel indices are read during step s: the P1 reads of a step depend on its
    // pixel-index reads, a second LDS round trip that was exposed once per step.
    auto ldAv = [&](int s) -> bf16x8 {
      const int mA = 32 * s + 8 * g + q;
      // rows mA and mA + 4 lie in the 8-row block b = 4 s + g, block b - 13 img of image img = b / 13
      const int b = 4 * s + g, sx = (b - 13 * ((b * 79) >> 10)) & 7;
      return cat8(tr_read(DC2 + (mA ^ sx) * 16 + 4 * p), tr_read(DC2 + ((mA + 4) ^ sx) * 16 + 4 * p));
    };
    auto step = [&](const bf16x8& av, unsigned px0, unsigned px1) {
      const bf16* pb0 = P1 + 8 * px0;
      const bf16* pb1 = P1 + 8 * px1;
      // every wave runs KT tiles (a wave with fewer real ones computes a tile it drops): all reads of the
      // step are in flight before its first MFMA
      bf16x4 t0[KT], t1[KT];
#pragma unroll
      for (int k = 0; k < KT; ++k) {
        t0[k] = tr_read(pb0 + toff[k]);
        t1[k] = tr_read(pb1 + toff[k]);
      }
#pragma unroll
      for (int k = 0; k < KT; ++k) acc[k] = mfma16x16x32(av, cat8(t0[k], t1[k]), acc[k]);
    };
    // two register sets, steps 2j (set a) and 2j + 1 (set b): each step's reads were issued one step
    // earlier (no register rotation, which waited for the prefetched data)
    static_assert(NM / 32 % 2 == 0, "phase E pairs its steps");
    const unsigned short* pxl = PX + 8 * g + q;
    bf16x8 ava = ldAv(0);
    unsigned pxa0 = pxl[0], pxa1 = pxl[4];
#pragma unroll 1
    for (int s = 0; s < nE; s += 2) {
      // (scheduling barriers keep the prefetches where they are: the scheduler otherwise hoists every LDS
      // read to the top of the loop body and waits for all of them there)
      const bf16x8 avb = ldAv(s + 1);
      const unsigned pxb0 = pxl[32 * (s + 1)], pxb1 = pxl[32 * (s + 1) + 4];
      __builtin_amdgcn_sched_barrier(0);
      step(ava, pxa0, pxa1);
      __builtin_amdgcn_sched_barrier(0);
      const int sn = s + 2 < nE ? s + 2 : s;  // the last pair re-reads its own rows (unused)
      ava = ldAv(sn);
      pxa0 = pxl[32 * sn];
      pxa1 = pxl[32 * sn + 4];
      __builtin_amdgcn_sched_barrier(0);
      step(avb, pxb0, pxb1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // D[row = output channel 4g + r][col i = (tap 2T + (i >> 3), channel i & 7)]; the bias gradient is
    // column (tap 0, channel 6), P1's ones
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      if (k < ntile) {
        const int T = w + NW * k;
        const int tap = 2 * T + (i >> 3), c = i & 7;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 4 * g + r;
          if (tap < 25 && c < 6) part[(long long)(kLeNetPW2 + n * 150 + tap * 6 + c)] = acc[k][r];
          else if (tap == 0 && c == 6) part[(long long)(kLeNetPB2 + n)] = acc[k][r];
        }
      }
    }
  }
  __syncthreads();  // phase E finished reading P1: it now receives dP1
  LN_STAMP(8);

  // ---------------------------------------------------------------- phase F: conv2 data gradient
  {
    const int bcol = i >> 3, c = i & 7;
#pragma unroll 2
    for (int mt = w; mt < nF; mt += NT / 64) {
      const int m = 16 * mt + i;
      const int img = m / 98, rem = m - 98 * (m / 98);
      const uint4 tv = *reinterpret_cast<const uint4*>(FT + (rem * 2 + (g >> 1)) * 16);
      const unsigned tw[4] = {tv.x, tv.y, tv.z, tv.w};
      // A row of step s: LDS byte offset computed branch-free (a t == 255 tap reads the zero block), read
      // three steps ahead of its MFMA (a select of two addresses compiled to an exec-mask branch, and
      // every read waited for its own data right before the MFMA: the LDS latency of all 15 steps was
      // exposed in series)
      // the table holds the stored row dc2_swz(t) inside the image's block (96, a zero padding row, for
      // "no tap")
      const unsigned dbase = (unsigned)OFF_DC2 + 16u * (unsigned)(g & 1) + 32u * (unsigned)(img * DC2_RS);
      auto ldA = [&](int st) -> bf16x8 {
        const unsigned t = (tw[st >> 2] >> (8 * (st & 3))) & 255u;
        return *reinterpret_cast<const bf16x8*>(smem + dbase + 32u * t);
      };
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      bf16x8 a0 = ldA(0), a1 = ldA(1), a2 = ldA(2);
#pragma unroll
      for (int s = 0; s < 15; ++s) {
        acc = mfma16x16x32(a0, bd[s], acc);
        a0 = a1;
        a1 = a2;
        if (s + 3 < 15) a2 = ldA(s + 3);
      }
      if (c < 6) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // pixel (image, y, 2 X2 + bcol) of row mm = (image * 14 + y) * 7 + X2: index 2 mm + bcol
          const int mm = 16 * mt + 4 * g + r;
          P1[(2 * mm + bcol) * 8 + c] = f2bf(acc[r]);
        }
      }
    }
  }
  __syncthreads();
  build_shift1(Xs, Xs1);  // dC2 is no longer needed: the union takes the shifted input again
  __syncthreads();
  LN_STAMP(9);

  // ---------------------------------------------------------------- phase G: conv1 weight gradient
  // dW1[c][ky][kx] = sum over (image, y, x) of dC1[c][y][x] X[y + ky][x + kx].  The two rows y = 2 py + dy
  // of a pool-window row are stacked in the GEMM's M: row (c, dy) = dy * 6 + c, and X row 2 py + dy + ky
  // is the extended tap ky' = dy + ky (0 .. 5) of row 2 py, so ONE B operand (30 extended taps + a ones
  // column) serves both rows: D[(c, dy)][(ky', kx)], and dW1[c][ky][kx] = D[(c, 0)][(ky, kx)] +
  // D[(c, 1)][(ky + 1, kx)] in the final sum (2 MFMAs per window row instead of 4).  A of lane (row i, g) =
  // dC1[c][2 py + dy][8g .. 8g + 8) unpooled in registers from dP1 + codes (4 windows); no per-image
  // staging, no barrier inside the loop.
  {
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int gdy = i >= 6 && i < 12 ? 1 : 0;  // this lane's A row (c, dy)
    const int ca = i < 6 ? i : (i < 12 ? i - 6 : 5);
    // B of lane (extended tap e = 16T + i, g) = input row 2 py + ky', columns 8g + kx .. + 7 (odd kx: the
    // shifted copy, so the start is a whole dword): four dwords from a dword-aligned address
    // (ds_read2_b32 pairs).  Column 30 (the bias) reads the ones block, column 31 the zero block.
    constexpr int kXs1 = (OFF_XS1 - OFF_XS) / 2;  // Xs1 - Xs in elements
    unsigned boff[2], bconst[2];
    bool breal[2];
#pragma unroll
    for (int T = 0; T < 2; ++T) {
      const int e = 16 * T + i;
      const int ep = e < 30 ? e : 0;
      const int ky = ep / 5, kx = ep - 5 * (ep / 5);
      boff[T] = 2u * (unsigned)(((kx & 1) ? kXs1 : 0) + ky * 32 + 8 * g + 2 * (kx >> 1));  // bytes from Xs
      breal[T] = e < 30;
      bconst[T] = e == 30 ? (unsigned)OFF_K : (unsigned)OFF_KZ;
    }
    // A: the window's dP1 value goes to position code (2 bits: dy * 2 + dx) of the 2x2 window; a lane of
    // row dy takes it when code - 2 dy is 0 or 1 (its dx).  Lanes past the 12 rows or the 14 windows take
    // no value (code forced past 3).
    unsigned cmask[4];
#pragma unroll
    for (int wd = 0; wd < 4; ++wd) cmask[wd] = (4 * g + wd < 14 && i < 12) ? 0u : 8u;
#pragma unroll 2
    for (int rp = w; rp < nG; rp += NT / 64) {
      const int img = rp / 14, py = rp - 14 * (rp / 14);
      const int p0 = (img * 14 + py) * 14 + 4 * g;
      const uint2 cA = *reinterpret_cast<const uint2*>(C1 + p0);
      const uint2 cB = *reinterpret_cast<const uint2*>(C1 + p0 + 2);
      const unsigned cw[4] = {cA.x, cA.y, cB.x, cB.y};
      unsigned aw[4];
#pragma unroll
      for (int wd = 0; wd < 4; ++wd) {
        const unsigned sel = (((cw[wd] >> (3 * ca)) & 7u) | cmask[wd]) - 2u * (unsigned)gdy;
        // in bounds for every lane (windows 14, 15 are the next row's first two or the tail)
        const unsigned pv = *reinterpret_cast<const unsigned short*>(P1 + (p0 + wd) * 8 + ca);
        aw[wd] = sel < 2u ? pv << (sel << 4) : 0u;
      }
      const bf16x8 av = __builtin_bit_cast(bf16x8, uint4{aw[0], aw[1], aw[2], aw[3]});
      const unsigned rowb = (unsigned)OFF_XS + 2u * (unsigned)(img * 1024 + 2 * py * 32);
#pragma unroll
      for (int T = 0; T < 2; ++T) {
        const unsigned* bp = reinterpret_cast<const unsigned*>(smem + (breal[T] ? rowb + boff[T] : bconst[T]));
        const bf16x8 bv = __builtin_bit_cast(bf16x8, uint4{bp[0], bp[1], bp[2], bp[3]});
        acc[T] = mfma16x16x32(av, bv, acc[T]);
      }
    }
    // cross-wave sum: D[row = (c, dy) 4g + r][col = extended tap 16T + i]; waves w and w + 4 share slot
    // w & 3 (the upper half writes, then the lower half adds in place: a [4][16][32] buffer for 8 waves)
    if (w >= 4) {
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) RED[((w & 3) * 16 + 4 * g + r) * 32 + 16 * T + i] = acc[T][r];
    }
    __syncthreads();
    if (w < 4) {
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* q = RED + (w * 16 + 4 * g + r) * 32 + 16 * T + i;
          *q = (NW > 4 ? *q : 0.f) + acc[T][r];
        }
    }
    __syncthreads();
    auto S = [&](int row, int col) {
      return RED[(0 * 16 + row) * 32 + col] + RED[(1 * 16 + row) * 32 + col] + RED[(2 * 16 + row) * 32 + col] +
             RED[(3 * 16 + row) * 32 + col];
    };
    for (int e = tid; e < 6 * 26; e += NT) {
      const int c = e / 26, t = e - 26 * (e / 26);  // t < 25: tap (ky, kx); t == 25: the bias
      if (t < 25) part[(long long)(kLeNetPW1 + c * 25 + t)] = S(c, t) + S(6 + c, t + 5);
      else part[(long long)(kLeNetPB1 + c)] = S(c, 30) + S(6 + c, 30);
    }
  }
  LN_STAMP(10);
  if (stamps && tid < 11) stamps[blockIdx.x * 16 + tid] = STMP[tid];
}

// Conv weights of this step as MFMA B fragments: one block (csrc/lenet_frag.h).  Only launched when
// the optimizer does not rebuild them (the fused step's SGD launch normally does, see optim.hip).
constexpr int PT = 1024;
__global__ void __launch_bounds__(PT) lenet_prep_kernel(const float* __restrict__ w1g, const float* __restrict__ w2g,
                                                        bf16x8* __restrict__ frag) {
  __shared__ float w[kLeNetConvW];
  for (int e = threadIdx.x; e < 150; e += PT) w[e] = w1g[e];
  for (int e = threadIdx.x; e < 2400; e += PT) w[150 + e] = w2g[e];
  __syncthreads();
  lenet_build_frags(w, frag, threadIdx.x, PT);
}

// ------------------------------------------------------------------------------------------------
// Reductions in one launch, deterministic (fixed summation order everywhere).
//
// Slots: dense_tiles 32 x 32 units of the dense weight gradients dW = dZ^T H (bias = input column K) and
// nconv_slots slots of 256 conv parameters (conv slots first by default: slot_dense / slot_conv).  Every slot is split into kChunks = 8 jobs:
// dense job (u, c) sums batch columns [c * chunk_cols, (c + 1) * chunk_cols), conv job (s, c) the
// partial rows of the train workgroups q = c (mod 8).  Job j = slot * 8 + c runs on workgroup j (mod G),
// so with round-robin dispatch and G % 8 == 0 chunk c is always read on XCD c -- the XCD whose train
// workgroups WROTE those columns / rows (the train kernel maps its image groups XCD-aware), and every
// line of H^T / dZ^T / conv partials is fetched into exactly one L2.  (Placement is speed only: any
// dispatch order gives the same bits.)  The jobs spread the ~5 MB of the step's activations over the
// whole chip: per-CU load bandwidth from beyond L2, not the FLOPs, bounds this launch.
//
// Each job writes its partial as a write-through (sc1) slab and takes a ticket; the slot's last arriver
// sums the 8 slabs in chunk order (sc1 loads), becomes the slot's OWNER, and -- multi-rank -- pushes the
// local sums into the peers' LL slots (csrc/ll_exchange.h).  After its jobs a workgroup waits for the
// rank sums of the slots it owns and applies the update (sync SGD, or the async PS decision).
// Then one workgroup: loss partials -> stats; one more (index stream / async PS): stage the next batch.
constexpr int RT = 256;          // reduce workgroup: 4 waves
constexpr int kDU = 32;          // dense unit edge
constexpr int kChunks = 8;       // jobs per slot
constexpr int kConvPer = 256;    // conv parameters per slot
constexpr int kSlotVals = 1024;  // values per slot (dense 32 x 32; conv slots use 256) = kLLSlot
constexpr int kPerThread = kSlotVals / RT;
constexpr int kMaxOwned = 16;    // slots one workgroup may own (host: G >= 8 * slots / kMaxOwned)
constexpr unsigned long long kSuccTimeoutTicks = 100000000ull;  // 1 s of wall_clock64: a granule wait never takes that
static_assert(kSlotVals <= kLLSlot, "LL slot too small");

// The element a thread finalises: descriptor index di into LeNetSgd::d (-1: none) and the element index
// i inside that tensor.
struct Owned {
  int di, i;
};

// Per-workgroup LDS copy of what the slots index at run time (dense layers, gradient outputs, update
// descriptors, SGD hyper-parameters).  Indexing the by-value kernel argument with run-time values would
// make the compiler copy the whole argument block into scratch for every thread; instead the contiguous
// LeNetRedTab image is read straight from the kernel-argument segment, one dword per thread.
struct RedTables : LeNetRedTab {
  float hyper[5];  // lr, momentum, wd, grad_scale, nesterov (read once, not per element)
};

__device__ __forceinline__ void stage_tables(const LeNetRedArgs& a, RedTables* t) {
  constexpr int kWords = (int)(sizeof(LeNetRedTab) / 4);
  static_assert(sizeof(LeNetRedTab) % 4 == 0 && kWords <= RT, "table image");
  typedef const __attribute__((address_space(4))) char kchar;  // the constant (kernel-argument) address space
  typedef const __attribute__((address_space(4))) int kint;
  kint* src = (kint*)((kchar*)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(LeNetRedArgs, tab));
  if ((int)threadIdx.x < kWords) reinterpret_cast<int*>(static_cast<LeNetRedTab*>(t))[threadIdx.x] = src[threadIdx.x];
  if (a.sgd_on && threadIdx.x >= 64 && threadIdx.x < 69) t->hyper[threadIdx.x - 64] = a.sgd.hyper[threadIdx.x - 64];
}

// dense unit u -> layer, output tile row tn (32 outputs), input tile column tk (32 inputs; bias = input K)
__device__ __forceinline__ int dense_unit(const RedTables& t, int u, int& tn, int& tk) {
  int l = 0;
  if (u >= t.L[0].tiles) {
    u -= t.L[0].tiles;
    l = 1;
    if (u >= t.L[1].tiles) {
      u -= t.L[1].tiles;
      l = 2;
    }
  }
  const int nt = (t.L[l].N + kDU - 1) / kDU;
  tk = u / nt;
  tn = u - nt * tk;  // tn fastest
  return l;
}

// Slot order: the conv slots -- the longest jobs -- first, so they are dispatched first and run on CUs
// not yet shared with other jobs (measured: conv jobs 6.0 -> 2.0 us, the step 0.5 us shorter), then the
// dense units.  slot_dense(): the dense unit of a slot, or -1 for a conv slot; slot_conv(): the conv slot.
__device__ __forceinline__ int slot_dense(const LeNetRedArgs& a, int slot) {
  return slot >= a.nconv_slots ? slot - a.nconv_slots : -1;
}
__device__ __forceinline__ int slot_conv(const LeNetRedArgs& a, int slot) { return slot; }

// the element of position pos (< kSlotVals) of `slot`
__device__ __forceinline__ Owned owned_elem(const LeNetRedArgs& a, const RedTables& t, int slot, int pos) {
  const int du = slot_dense(a, slot);
  if (du >= 0) {
    int tn, tk;
    const int l = dense_unit(t, du, tn, tk);
    const int N = t.L[l].N, K = t.L[l].K;
    const int on = kDU * tn + (pos >> 5), ok = kDU * tk + (pos & 31);
    if (on >= N || ok > K) return {-1, 0};
    return ok < K ? Owned{4 + 2 * l, on * K + ok} : Owned{5 + 2 * l, on};
  }
  const int p = slot_conv(a, slot) * kConvPer + pos;
  if (pos >= kConvPer || p >= kLeNetConvParams) return {-1, 0};
  if (p < kLeNetPB1) return {0, p};
  if (p < kLeNetPW2) return {1, p - kLeNetPB1};
  if (p < kLeNetPB2) return {2, p - kLeNetPW2};
  return {3, p - kLeNetPB2};
}

// position of conv weight element (di, i) in the fragment buffer's weight numbering (-1: not a conv weight)
__device__ __forceinline__ int conv_wj(Owned o) { return o.di == 0 ? o.i : o.di == 2 ? 150 + o.i : -1; }

// Dense job (unit u, chunk c): this workgroup's partial of the unit over the chunk's batch columns.  The
// chunk's K-steps are split over the 4 waves; each wave computes all four 16 x 16 sub-tiles of its steps
// (every operand row it loads is used twice); LDS combine.  out[e] = partial of position t + 256 e.
// (nch = 1: the whole batch, the solo path)
__device__ __forceinline__ void dense_job(const LeNetRedArgs& a, const RedTables& t, int u, int c, float* red,
                                          float (&out)[kPerThread], int nch = kChunks) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  int tn, tk;
  const int l = dense_unit(t, u, tn, tk);
  const LeNetDense& L = t.L[l];
  const int cw = nch == 1 ? a.kcols : a.chunk_cols;
  const int col0 = c * cw, col1 = min(a.kcols, col0 + cw);
  const bf16* arow[2];
  const bf16* brow[2];
  bool a_ok[2], b_ok[2], b_one[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n = kDU * tn + 16 * i + (lane & 15), k = kDU * tk + 16 * i + (lane & 15);
    arow[i] = L.dzT + (long long)min(n, L.N - 1) * a.ldt + col0 + 8 * (lane >> 4);
    brow[i] = L.hT + (long long)min(k, L.K - 1) * a.ldt + col0 + 8 * (lane >> 4);
    a_ok[i] = n < L.N;
    b_ok[i] = k < L.K;
    b_one[i] = k == L.K;
  }
  bf16x8 ones, zeros = zero8();
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.f;
  const int steps = col1 > col0 ? (col1 - col0) / 32 : 0;
  const int per = (steps + 3) / 4;
  const int s0 = wid * per, s1 = min(steps, s0 + per);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < s1; s += 4) {
    bf16x8 av[2][4], bv[2][4];
    // unconditional loads (the rows are clamped to valid ones; the MFMA operand selects below drop the
    // padding): a load under a per-group condition compiled to an exec-mask branch per load, each waiting
    // for the one before it
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ss = min(s + q, s1 - 1);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        av[i][q] = ld8(arow[i] + 32 * ss);
        bv[i][q] = ld8(brow[i] + 32 * ss);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool live = s + q < s1;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = mfma16x16x32((a_ok[i] && live) ? av[i][q] : zeros,
                                   b_ok[j] ? bv[j][q] : (b_one[j] ? ones : zeros), acc[i][j]);
    }
  }
  // D[n][k] of sub-tile (i, j): row 16 i + 4 (lane >> 4) + r, column 16 j + (lane & 15); position = row * 32 + col
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wid * kSlotVals + (16 * i + 4 * (lane >> 4) + r) * kDU + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kPerThread; ++e) {
    const int pos = threadIdx.x + RT * e;
    out[e] = ((red[pos] + red[kSlotVals + pos]) + red[2 * kSlotVals + pos]) + red[3 * kSlotVals + pos];
  }
}

// Conv job (slot s, chunk c): parameters 256 s .. 256 s + 255 over the train workgroups' partial rows
// q = c, c + 8, ...: one row (1 KB) per wave-load, the rows split over the 4 waves, LDS combine.
__device__ __forceinline__ void conv_job(const LeNetRedArgs& a, int s, int c, float* red, float (&out)[kPerThread],
                                         int nch = kChunks) {
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int p0 = s * kConvPer + 4 * lane;
  const int pl = min(p0, kLeNetConvStride - 4);  // lanes past the last parameter read the row's padding
  const int nrows = a.nblk > c ? (a.nblk - 1 - c) / nch + 1 : 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i0 = wid; i0 < nrows; i0 += 4 * 16) {
    // every load of the round unconditional (rows clamped, the padding ones dropped below): a per-row
    // condition compiled to an exec-mask branch per load, each waiting for the one before it
    f32x4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = min(i0 + 4 * k, nrows - 1);
      v[k] = *reinterpret_cast<const f32x4*>(a.conv_part + (long long)(c + nch * i) * kLeNetConvStride + pl);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (i0 + 4 * k < nrows) acc += v[k];
  }
  *reinterpret_cast<f32x4*>(red + wid * kSlotVals + 4 * lane) = acc;
  __syncthreads();
  const int pos = threadIdx.x;
  out[0] = ((red[pos] + red[kSlotVals + pos]) + red[2 * kSlotVals + pos]) + red[3 * kSlotVals + pos];
#pragma unroll
  for (int e = 1; e < kPerThread; ++e) out[e] = 0.f;
}

// The new value w of element o becomes the local master and its bf16 compute copies (and, for a conv
// weight, the next step's MFMA fragment).  Dense elements (di >= 4) take the tile-layout copy path only
// (the launcher checks their descriptors): one small inlined body per position instead of the general
// layout switch, which the conv slots (one position per thread) keep.
template <bool DENSE>
__device__ __forceinline__ void red_emit(const LeNetRedArgs& a, const RedTables& t, Owned o, float w) {
  const ParamDesc& d = t.d[o.di];
  a.sgd.master[d.off + o.i] = w;
  if (a.mirror != nullptr) a.mirror[d.off + o.i] = w;  // mode 3: the rank's master shard
  if (DENSE) {
    if (d.bf_off < 0) return;  // a bias
    const int K = d.T * d.Ci;
    const int n = o.i / K, kk = o.i - n * K;
    const bf16 wb = f2bf(w);
    a.sgd.wbf[d.bf_off + (long long)n * round_up(K, 32) + kk] = wb;
    a.sgd.wbf[d.bft_off + (long long)kk * round_up(d.N, 32) + n] = wb;
    return;
  }
  emit_copies(d, o.i, w, a.sgd.wbf);
  const int wj = conv_wj(o);
  if (wj >= 0) lenet_frag_scatter(a.sgd.frag, wj, w);
}

// Finalise element o with gradient v (sync): store the gradient; with the fused update apply SGD to the
// master (w_old / m_old loaded by the caller) and emit the copies; otherwise snapshot what the optimizer
// launch needs.
template <bool DENSE>
__device__ __forceinline__ void red_apply(const LeNetRedArgs& a, const RedTables& t, Owned o, float v, float w_old,
                                          float m_old) {
  if (o.di < 0) return;
  t.g[o.di][o.i] = v;
  if (a.sgd_on) {
    const float* h = t.hyper;
    const float mom = h[1];
    float m_new = 0.f;
    const float nw = sgd_new_weight(w_old, v, mom != 0.f ? m_old : 0.f, h[0], mom, h[2], h[3], h[4] != 0.f, &m_new);
    if (mom != 0.f) a.sgd.mom[t.d[o.di].off + o.i] = m_new;
    red_emit<DENSE>(a, t, o, nw);
  } else if (!DENSE && a.snap != nullptr && conv_wj(o) >= 0) {
    // the conv kernels' weights and momentum as this gradient saw them: the optimizer launch rebuilds
    // the next step's fragments from these (no read of state it is overwriting)
    const int wj = conv_wj(o);
    const long long q = wj < 150 ? wj : wj - 150;
    a.snap[wj] = wj < 150 ? a.w1[q] : a.w2[q];
    a.snap[kLeNetConvW + wj] = a.m1 == nullptr ? 0.f : (wj < 150 ? a.m1[q] : a.m2[q]);
  }
}

// ---- asynchronous SGD against the device parameter server (LeNetRedArgs::ps_on) ------------------------
// The staging workgroup admits or rejects this step's gradient (ps_admit: one lock-free CAS on the
// shared version word, csrc/ps_device.h) as soon as the launch starts -- the decision does not depend on
// the gradient's values -- and publishes the decision on a local word tagged with this launch's epoch.
// The slot owners wait for it only after their jobs (so it is normally already there), then add
// -lr * g to their elements of the sharded master and refresh the local copies from the values the adds
// produced.  No lock is held: the owners of different ranks update the shards in parallel.
// ``pre`` (thread 0): the epoch and decision words as loaded at the workgroup's start, {epoch, decision}, or
// nullptr.  The epoch cannot advance before every owner has passed this wait, and a decision published
// by the train launch's admission workgroup is already there when the reduce launch starts, so the
// common case costs no memory round trip here.
// owner-applies (mode 4), the last arrival of the launch: every owner's shard and inbox stores have landed
// (each drained before arriving), so the drained prefixes go out, then the drain locks are released (a
// rank that takes a lock reads the prefix only after its CAS returned), and an admitted gradient's ring slot
// is flagged at every owner
__device__ __forceinline__ void lenet_ps_owner_publish(const PSArgs& p, bool admitted) {
  const unsigned long long* dw = ps_owner_drain_words(p);
  unsigned held = 0;
  for (int k = 0; k < p.nshards; ++k) {
    const unsigned long long w = __hip_atomic_load(const_cast<unsigned long long*>(dw) + k, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    const unsigned n = (unsigned)(w >> 32) & 0xffu;
    if (n) {
      __hip_atomic_store(p.pref + k, (unsigned)w + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      held |= 1u << k;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int k = 0; k < p.nshards; ++k)
    if ((held >> k) & 1u) __hip_atomic_store(p.dlock + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (admitted) {
    const unsigned q = p.scratch[kPSSeq], R = (unsigned)p.owner_ring;
    for (int k = 0; k < p.nshards; ++k)
      __hip_atomic_store(ps_inbox_flags(p, k) + q % R, q + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// owner-applies: this launch's drain decision (workgroup 0's, made at the launch's start -- normally long done
// when an owner finishes its job): s_P / s_n per shard.  A wait that times out (never expected) drains nothing
// there and sets an error bit.
__device__ __forceinline__ void lenet_ps_owner_load(const PSArgs& p, unsigned ep, unsigned* s_P, unsigned* s_n) {
  if ((int)threadIdx.x < p.nshards) {
    unsigned long long* wp = ps_owner_drain_words(p) + threadIdx.x;
    unsigned long long w = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool ok = ps_owner_word_ep(w) == (ep & 0xffffffu);
    const unsigned long long t0 = ok ? 0ull : wall_clock64();
    while (!ok) {
      __builtin_amdgcn_s_sleep(1);
      w = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = ps_owner_word_ep(w) == (ep & 0xffffffu);
      if (!ok && wall_clock64() - t0 > 2ull * (unsigned long long)p.timeout_ticks) {
        atomicOr(p.stats + 5, 64ull);
        if (p.herr) __hip_atomic_store(p.herr, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    s_P[threadIdx.x] = (unsigned)w;
    s_n[threadIdx.x] = ok ? ((unsigned)(w >> 32) & 0xffu) : 0u;
  }
}

// owner-applies, one element gi of the master: the admitted -lr * g (d) into ring slot q % R of its shard's
// inbox; the shard value, plus -- when this launch drains the shard -- its n flagged slots in sequence order
// (stored back: the lock holder is the shard's only writer); returns the value the local copies take (+ d
// when admitted: the gradient's own update, not yet in the shard)
__device__ __forceinline__ float lenet_ps_owner_elem(const PSArgs& p, float* const* s_shard, float* const* s_inbox,
                                                     const unsigned* s_P, const unsigned* s_n, long long gi, float d,
                                                     bool put, unsigned q) {
  const int k = (int)(gi >> p.shard_shift);
  const long long off = gi & ((1LL << p.shard_shift) - 1);
  const unsigned R = (unsigned)p.owner_ring;
  if (put)
    __hip_atomic_store(reinterpret_cast<unsigned*>(s_inbox[k] + ((long long)(q % R) << p.shard_shift) + off),
                       __float_as_uint(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned* wp = reinterpret_cast<unsigned*>(s_shard[k] + off);
  float v = __uint_as_float(__hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  const unsigned n = s_n[k];
  if (n) {
    const unsigned P = s_P[k];
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      x[j] = (unsigned)j < n ? __uint_as_float(__hip_atomic_load(
                                   reinterpret_cast<unsigned*>(s_inbox[k] + ((long long)((P + j) % R) << p.shard_shift) + off),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
                             : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma clang fp contract(off)
      if ((unsigned)j < n) v += x[j];
    }
    for (unsigned j = 8; j < n; ++j) {  // (rings longer than 8: the bound's rare tail)
#pragma clang fp contract(off)
      v += __uint_as_float(__hip_atomic_load(
          reinterpret_cast<unsigned*>(s_inbox[k] + ((long long)((P + j) % R) << p.shard_shift) + off), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_SYSTEM));
    }
    __hip_atomic_store(wp, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  float out;
  {
#pragma clang fp contract(off)
    out = put ? v + d : v;
  }
  return out;
}

__device__ __forceinline__ unsigned lenet_ps_wait(const LeNetRedArgs& a, unsigned* s_dec,
                                                  const unsigned* pre = nullptr) {
  const PSArgs& p = a.ps;
  if (threadIdx.x == 0) {
    const unsigned ep = (pre ? pre[0] : __hip_atomic_load(p.scratch + kPSEpoch, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)) + 1u;
    const unsigned long long t0 = wall_clock64();
    unsigned dec = kPSFailed;
    bool first = pre != nullptr;
    for (;;) {  // relaxed polls, one acquire once the word matches
      const unsigned w = first ? pre[1] : __hip_atomic_load(p.scratch + kPSDecision, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
      first = false;
      if (ps_epoch_eq(w, ep)) {  // (only the word itself is consumed: no acquire, which invalidated the L2
        dec = w & 7u;              // of the owner's XCD under the other workgroups' jobs)
        break;
      }
      if (wall_clock64() - t0 > 2ull * (unsigned long long)p.timeout_ticks) {
        atomicOr(p.stats + 5, 8ull);
        if (p.herr) __hip_atomic_store(p.herr, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    *s_dec = dec;
  }
  __syncthreads();
  return *s_dec;
}

// Protocol arrivals: one per slot (its owner adds one when done with it) and one from the staging
// workgroup; the last one advances this rank's launch epoch (the decision word's tag).  Workgroups that
// own nothing do not arrive.
__device__ __forceinline__ void lenet_ps_arrive(const LeNetRedArgs& a, unsigned count, unsigned arrivals,
                                                int known_dec = -1, const unsigned* known_ep = nullptr) {
  const PSArgs& p = a.ps;
  __syncthreads();
  if (threadIdx.x == 0 && count > 0) {
    const unsigned prev = __hip_atomic_fetch_add(p.scratch + kPSApplyDone, count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + count == arrivals) {
      // the last arrival: every owner drained its shard adds before arriving, so an admitted gradient is
      // now fully applied (the decision word was published before any owner or the staging arrival)
      const unsigned w = known_dec >= 0 ? (unsigned)known_dec
                                        : __hip_atomic_load(p.scratch + kPSDecision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((w & 7u) == kPSAccept) ps_publish_applied(p);
      if (p.owner_ring > 0) lenet_ps_owner_publish(p, (w & 7u) == kPSAccept);
      __hip_atomic_store(p.scratch + kPSApplyDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // (known_ep: the epoch word as thread 0 of a slot owner loaded it; it cannot have moved since)
      const unsigned ep0 = known_ep ? *known_ep
                                    : __hip_atomic_load(p.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.scratch + kPSEpoch, ep0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// diagnostic phase clocks of the reduce launch (wall clock, 100 MHz, comparable across CUs):
// stamps[block][16]: 0 start, 1 jobs done, 2 decision known, 3 owned slots applied, 4 end, 5 first owned
// slot's rank sums in (LL), 6 first job's partial computed, 7 first ownership combine done; staging
// workgroup (PS): 8 admission start, 9 admission done / decision published, 10 next batch staged
// (kept in LDS and written out when the workgroup ends: a global store mid-kernel makes the compiler's
// wait-count pass wait for every load in flight at the next join, stamps or not)
#define LR_STAMP(slot)                                                              \
  do {                                                                              \
    if (a.stamps) {                                                                 \
      __builtin_amdgcn_sched_barrier(0);                                            \
      const unsigned long long t_ = wall_clock64();                                 \
      __builtin_amdgcn_sched_barrier(0);                                            \
      if (threadIdx.x == 0) lr_st[(slot)] = t_;                                     \
    }                                                                               \
  } while (0)
#define LR_FLUSH()                                                                  \
  do {                                                                              \
    if (a.stamps && threadIdx.x == 0)                                               \
      for (int k_ = 0; k_ < 16; ++k_) a.stamps[blockIdx.x * 16 + k_] = lr_st[k_];   \
  } while (0)

// MODE: 0 single rank, 1 in-kernel LL exchange over the ranks, 2 async parameter server.  One
// instantiation per mode keeps every launch's code small (the instruction cache is shared with the train
// kernel; each workgroup runs its path once, cold).
template <int MODE>
__global__ void __launch_bounds__(RT, 4) lenet_reduce_kernel(LeNetRedArgs a) {
  // MODE 3 (async PS, one rank): the synchronous owners' fused update, gated on the train launch's admission
  // decision and mirrored into the rank's master shard; no arrival protocol (the admission advanced the
  // epoch and published the applied count, ps_device.h)
  // MODE 4 (async PS, owner-applies): mode 2's protocol with the shard updates through the owners' inboxes
  // (lenet_ps_owner_elem: plain stores and loads, no per-element remote atomic)
  constexpr bool LL = MODE == 1, PS = MODE == 2 || MODE == 4, PSX = MODE == 3, OWN = MODE == 4;
  __shared__ float red[4 * kSlotVals];
  __shared__ RedTables tabs;
  __shared__ int owned[kMaxOwned];
  __shared__ unsigned ep[kMaxOwned];
  __shared__ unsigned s_e;
  __shared__ int s_last;
  __shared__ float* s_shard[kP2PMaxRanks];  // PS: the master shards' bases (ps_elem)
  __shared__ float* s_inbox[kP2PMaxRanks];  // OWN: the owners' inbox bases
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  __shared__ unsigned long long lr_st[16];
  if (a.stamps && threadIdx.x < 16) lr_st[threadIdx.x] = 0ull;  // (only thread 0 writes them afterwards)
  LR_STAMP(0);
  const int nslot = a.dense_tiles + a.nconv_slots;
  const int G = a.exch_blocks;
  if ((int)blockIdx.x < G) {
    // async PS: the fully applied count before any shard access of this launch (ps_device.h)
    // (successor mode: the barrier after the tables publishes the shard table too)
    if (OWN && threadIdx.x < kP2PMaxRanks) {
      float* v = nullptr;
#pragma unroll
      for (int k = 0; k < kP2PMaxRanks; ++k)
        if ((int)threadIdx.x == k) v = a.ps.inbox[k];
      s_inbox[threadIdx.x] = v;
    }
    if (PS) ps_stage_shards(a.ps, s_shard, !a.succ);
    if (OWN && blockIdx.x == 0) {
      __shared__ unsigned s_cnt[kP2PMaxRanks];
      lenet_ps_owner_decide(a.ps, s_cnt);  // (its barrier also publishes the shard tables)
    }
    stage_tables(a, &tabs);
    // with the fused sync update, the first owned slot's master / momentum elements are loaded beside
    // its slab loads
    if (MODE == 0 && a.solo) {
      // small batches: workgroup g reduces slot g over the whole batch (one job over every partial row /
      // batch column) and applies the update of its positions itself -- no 8-way split, no granule hand-off
      // (at B = 32 the hand-off between XCDs was ~2.5 us of a ~6 us launch)
      const int slot = blockIdx.x;
      const bool dense = slot_dense(a, slot) >= 0;
      __syncthreads();  // the tables staged above
      Owned o[kPerThread];
      float w0[kPerThread], m0[kPerThread], v[kPerThread];
#pragma unroll
      for (int e = 0; e < kPerThread; ++e) {  // the old master / momentum load beside the job's operands
        o[e] = (dense || e == 0) ? owned_elem(a, tabs, slot, (int)threadIdx.x + RT * e) : Owned{-1, 0};
        w0[e] = m0[e] = 0.f;
        if (a.sgd_on && o[e].di >= 0) {
          const long long off = tabs.d[o[e].di].off + o[e].i;
          w0[e] = a.sgd.master[off];
          m0[e] = a.sgd.mom != nullptr ? a.sgd.mom[off] : 0.f;
        }
      }
      if (dense) dense_job(a, tabs, slot_dense(a, slot), 0, red, v, 1);
      else conv_job(a, slot_conv(a, slot), 0, red, v, 1);
      LR_STAMP(6);
      if (dense) {
#pragma unroll
        for (int e = 0; e < kPerThread; ++e) red_apply<true>(a, tabs, o[e], v[e], w0[e], m0[e]);
      } else {
        red_apply<false>(a, tabs, o[0], v[0], w0[0], m0[0]);
      }
      LR_STAMP(3);
      LR_STAMP(4);
      LR_FLUSH();
      return;
    }
    const bool pre = a.sgd_on && !PS;
    __shared__ float w_pre[kPerThread][RT], m_pre[kPerThread][RT];  // (LDS: not live across the jobs in VGPRs)
    __shared__ float own0[kPerThread][RT];  // the first owned slot's local sums
    __shared__ unsigned s_dec;
    if (a.succ) {
      // successor ownership: this workgroup's job (slot grp, chunk c), published as {epoch, value}
      // granules, then its eighth of slot grp - 1 (positions [c * cnt, (c + 1) * cnt)): one hand-off from
      // the 8 producers, no ticket and no slab reload.  Every wait is on lower-indexed workgroups, which
      // publish before they wait, so in-order dispatch needs no co-residency.
      const int grp = blockIdx.x / kChunks, c = blockIdx.x - kChunks * grp;
      __shared__ unsigned s_ge, s_pe;
      // this launch's epoch: the counter load goes out now and is waited for only after the job (a wait
      // here put a whole memory round trip in front of every job)
      const unsigned ge_prev = threadIdx.x == 0 ? a.gran_ep[blockIdx.x] : 0u;
      // mode 3: the admission's epoch and decision words (written by the train launch), consumed after the job
      unsigned psx_ep = 0u, psx_dec = 0u;
      if (PSX && threadIdx.x == 0) {
        psx_ep = __hip_atomic_load(a.ps.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        psx_dec = __hip_atomic_load(a.ps.scratch + kPSDecision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __shared__ int s_gate;
      __syncthreads();  // the tables staged above are read by every thread of the job
      float part[kPerThread];
      if (grp < nslot) {
        const int du = slot_dense(a, grp);
        if (du >= 0) dense_job(a, tabs, du, c, red, part);
        else conv_job(a, slot_conv(a, grp), c, red, part);
        LR_STAMP(6);
      }
      if (threadIdx.x == 0) {
        s_ge = ge_prev + 1u;
        if (PSX) {
          const bool mine_ep = ps_epoch_eq(psx_dec, psx_ep);
          s_gate = mine_ep && (psx_dec & 7u) == kPSAccept;
          if (!mine_ep && blockIdx.x == 0) atomicOr(a.ps.stats + 5, 8ull);  // (never expected: no update)
        }
      }
      __syncthreads();
      const unsigned ge = s_ge;
      if (grp < nslot) {
        const int npos = slot_dense(a, grp) >= 0 ? kPerThread : 1;
        unsigned long long* g = a.gran + ((long long)grp * kChunks + c) * kSlotVals + threadIdx.x;
#pragma unroll
        for (int e = 0; e < kPerThread; ++e)
          if (e < npos)
            __hip_atomic_store(g + RT * e, ((unsigned long long)ge << 32) | __float_as_uint(part[e]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      }
      LR_STAMP(1);
      // async PS: the epoch and decision words, loaded beside the granule polls below (issued before the
      // job, their wait sat in front of the job's first operand wait)
      unsigned ps_pre[2] = {0u, 0u};
      if (PS && threadIdx.x == 0) {
        ps_pre[0] = __hip_atomic_load(a.ps.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ps_pre[1] = __hip_atomic_load(a.ps.scratch + kPSDecision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int s = grp - 1;
      if (s >= 0) {
        const bool dense = slot_dense(a, s) >= 0;
        const int cnt = dense ? kSlotVals / kChunks : kConvPer / kChunks;
        const int pos = c * cnt + (int)threadIdx.x;
        const bool mine = (int)threadIdx.x < cnt;
        Owned o = mine ? owned_elem(a, tabs, s, pos) : Owned{-1, 0};
        // the old master / momentum values load while the granules are awaited
        float w0 = 0.f, m0 = 0.f, v = 0.f;
        if (a.sgd_on && !PS && o.di >= 0) {
          const long long off = tabs.d[o.di].off + o.i;
          w0 = a.sgd.master[off];
          m0 = a.sgd.mom != nullptr ? a.sgd.mom[off] : 0.f;
        }
        // async PS: the shard is updated in groups of 4 consecutive positions per thread (uncached shard
        // memory at world > 1 takes ~6 k operations per us chip-wide, profiles/r5: a contiguous aligned group
        // of the exclusive writer is ONE 16-byte load and store); the group's addresses and current values
        // load here, beside the granule wait
        float* pg[4] = {nullptr, nullptr, nullptr, nullptr};
        Owned og[4] = {{-1, 0}, {-1, 0}, {-1, 0}, {-1, 0}};
        f32x4 curv = {0.f, 0.f, 0.f, 0.f};
        bool vec = false;
        // (dense slots: 32 threads x 4 positions; conv slots, whose emits are long -- copies and the MFMA
        // fragment -- one position per thread)
        const bool grp4 = PS && dense && (int)threadIdx.x * 4 < cnt;
        const bool one = PS && !dense && mine;
        if (one) {
          og[0] = o;
          pg[0] = o.di >= 0 ? ps_elem(s_shard, a.ps.shard_shift, tabs.d[o.di].off + o.i) : nullptr;
          if (a.ps.excl != 0 && pg[0] != nullptr)
            curv[0] = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(pg[0]), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_SYSTEM));
        }
        if (grp4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            og[j] = owned_elem(a, tabs, s, c * cnt + 4 * (int)threadIdx.x + j);
            pg[j] = og[j].di >= 0 ? ps_elem(s_shard, a.ps.shard_shift, tabs.d[og[j].di].off + og[j].i) : nullptr;
          }
          vec = a.ps.excl != 0 && pg[0] != nullptr && pg[1] == pg[0] + 1 && pg[2] == pg[0] + 2 && pg[3] == pg[0] + 3 &&
                (reinterpret_cast<uintptr_t>(pg[0]) & 15) == 0;
          if (vec) curv = *reinterpret_cast<const f32x4*>(pg[0]);
        }
        if (mine) {
          const unsigned long long* g = a.gran + (long long)s * kChunks * kSlotVals + pos;
          const unsigned long long t0 = wall_clock64();
          for (;;) {  // every chunk's granule in flight per poll; the sum in chunk order (the ticket path's)
            unsigned long long q[kChunks];
#pragma unroll
            for (int cc = 0; cc < kChunks; ++cc)
              q[cc] = __hip_atomic_load(g + cc * kSlotVals, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool ok = true;
#pragma unroll
            for (int cc = 0; cc < kChunks; ++cc) ok = ok && (unsigned)(q[cc] >> 32) == ge;
            if (ok) {
              v = __uint_as_float((unsigned)q[0]);
#pragma unroll
              for (int cc = 1; cc < kChunks; ++cc) v += __uint_as_float((unsigned)q[cc]);
              break;
            }
            if (wall_clock64() - t0 > kSuccTimeoutTicks) {  // never expected: flag it, leave the element
              atomicOr(a.gran_err, 1u);
              if (LL) atomicOr(a.ll.err, 2);
              if (PS) atomicOr(a.ps.stats + 5, 16ull);
              o.di = -1;
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        }
        LR_STAMP(7);
        if (!PS) LR_STAMP(2);
        if (PS) {
          float* vb = red;  // [cnt] local sums (the jobs are done with red)
          if (mine) vb[threadIdx.x] = v;
          const unsigned dec = lenet_ps_wait(a, &s_dec, ps_pre);  // (its barrier also publishes vb)
          LR_STAMP(2);
          const bool upd = dec == kPSAccept || dec == kPSReject;
          const PSArgs& p = a.ps;
          const int q0 = 4 * (int)threadIdx.x;
          float wn[4] = {0.f, 0.f, 0.f, 0.f};  // the shard values after this step (emitted below)
          // an exclusive writer's slot arrival waits for nothing: it goes out now, beside the shard update
          unsigned slot_prev = 0u;
          if (p.excl && !OWN && threadIdx.x == 0)
            slot_prev = __hip_atomic_fetch_add(a.slot_arr + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (OWN) {
            // owner-applies: this launch's drain decision (the admission's), then per element the inbox store
            // of -lr * g (admitted), the shard's drain (when this launch holds its lock) and the emitted value;
            // the drain runs whatever the decision (the lock holder must add every slot it counted)
            __shared__ unsigned s_oP[kP2PMaxRanks], s_on[kP2PMaxRanks], s_oq, s_oep;
            if (threadIdx.x == 0) {
              s_oq = p.scratch[kPSSeq];
              s_oep = ps_pre[0] + 1u;
            }
            __syncthreads();
            lenet_ps_owner_load(p, s_oep, s_oP, s_on);
            __syncthreads();
            const bool put = dec == kPSAccept;
            const unsigned q = s_oq;
            if (grp4) {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (og[j].di >= 0) {
                  float dj;
                  {
#pragma clang fp contract(off)
                    dj = -(tabs.hyper[0] * vb[q0 + j]);
                  }
                  wn[j] = lenet_ps_owner_elem(p, s_shard, s_inbox, s_oP, s_on, tabs.d[og[j].di].off + og[j].i, dj, put, q);
                }
            } else if (one && og[0].di >= 0) {
              float d0;
              {
#pragma clang fp contract(off)
                d0 = -(tabs.hyper[0] * v);
              }
              wn[0] = lenet_ps_owner_elem(p, s_shard, s_inbox, s_oP, s_on, tabs.d[og[0].di].off + og[0].i, d0, put, q);
            }
          } else if (upd && grp4) {
            float d[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
#pragma clang fp contract(off)
              d[j] = -(tabs.hyper[0] * vb[q0 + j]);
            }
            if (vec) {  // exclusive writer: the values loaded above are the shard's current ones
#pragma unroll
              for (int j = 0; j < 4; ++j) wn[j] = dec == kPSAccept ? curv[j] + d[j] : curv[j];
              if (dec == kPSAccept) *reinterpret_cast<f32x4*>(pg[0]) = f32x4{wn[0], wn[1], wn[2], wn[3]};
            } else if (dec == kPSAccept) {
              ps_add<4>(pg, d, wn, p.excl != 0, p);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                wn[j] = pg[j] ? __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(pg[j]), __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_SYSTEM))
                              : 0.f;
            }
          } else if (upd && one && pg[0] != nullptr) {
            float d0;
            {
#pragma clang fp contract(off)
              d0 = -(tabs.hyper[0] * v);
            }
            if (p.excl != 0) {  // exclusive writer: the value loaded above is the shard's current one
              {
#pragma clang fp contract(off)
                wn[0] = dec == kPSAccept ? curv[0] + d0 : curv[0];
              }
              if (dec == kPSAccept)
                __hip_atomic_store(reinterpret_cast<unsigned*>(pg[0]), __float_as_uint(wn[0]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            } else if (dec == kPSAccept) {
              float* const pp[1] = {pg[0]};
              const float dd[1] = {d0};
              float ww[1];
              ps_add<1>(pp, dd, ww, false, p);
              wn[0] = ww[0];
            } else {
              wn[0] = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(pg[0]), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_SYSTEM));
            }
          }
          // this workgroup's shard adds have landed; the slot's last owner of its 8 arrives for the slot (one
          // counter per slot, then nslot + 2 arrivals on the launch's: a flat fan-in of 8 x nslot owners on
          // one word was the launch's tail).  The local emits (rank-private: gradient, local master, compute
          // copies, read by the next launch) follow the arrival instead of delaying it.
          // (an exclusive writer -- one rank -- has no concurrent reader of the shard: its next reader is this
          // rank's next launch, after the kernel boundary; no drain)
          LR_STAMP(11);
          float* wb = red + 128;  // [cnt] the dense groups' new values, one emit per position below
          if (upd && grp4)
#pragma unroll
            for (int j = 0; j < 4; ++j) wb[q0 + j] = wn[j];
          if (!p.excl || OWN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          __shared__ unsigned s_arr;
          if (threadIdx.x == 0) {
            if (!p.excl || OWN)
              slot_prev = __hip_atomic_fetch_add(a.slot_arr + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsigned n = 0;
            if (slot_prev == (unsigned)(kChunks - 1)) {
              __hip_atomic_store(a.slot_arr + s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              n = 1;
            }
            s_arr = n;
          }
          __syncthreads();
          LR_STAMP(12);
          lenet_ps_arrive(a, s_arr, (unsigned)(nslot + 2), (int)dec, ps_pre);  // (an owner knows both)
          LR_STAMP(13);
          if (upd && dense) {
            if (mine && o.di >= 0) {
              tabs.g[o.di][o.i] = v;
              red_emit<true>(a, tabs, o, wb[threadIdx.x]);
            }
          } else if (upd && one && pg[0] != nullptr) {
            tabs.g[og[0].di][og[0].i] = v;
            red_emit<false>(a, tabs, og[0], wn[0]);
          }
          LR_STAMP(5);
        } else {
          bool ok = true;
          unsigned ee = 0;
          if (LL) {  // the rank-order sum of this eighth (its own LL epoch word)
            if (threadIdx.x == 0) s_pe = a.ll.part_epochs[s * kLLParts + c] + 1u;
            __syncthreads();
            ee = s_pe;
            if (mine) {
              ll_push(a.ll, s, pos, ee, v);
              ok = ll_wait_sum(a.ll, s, pos, ee, v, v);
            }
            LR_STAMP(5);
          }
          if (ok && o.di >= 0 && (!PSX || s_gate)) {
            if (dense) red_apply<true>(a, tabs, o, v, w0, m0);
            else red_apply<false>(a, tabs, o, v, w0, m0);
          }
          if (LL) {
            __syncthreads();  // every position consumed before the part's epoch advances
            if (threadIdx.x == 0) a.ll.part_epochs[s * kLLParts + c] = ee;
          }
        }
      }
      LR_STAMP(3);
      // (async PS: the slot owners arrived above; workgroup 0 owns no slot)
      if (threadIdx.x == 0) a.gran_ep[blockIdx.x] = ge;
      LR_STAMP(4);
      LR_FLUSH();
      return;
    }
    int nown = 0, narr = 0;  // slots owned (kept) / slots this workgroup finished last (async PS arrivals)
#pragma unroll 1
    for (int j = blockIdx.x; j < nslot * kChunks; j += G) {
      const int slot = j / kChunks, c = j - kChunks * (j / kChunks);
      __syncthreads();  // red / tabs / s_last of the previous job
      float part[kPerThread];
      const int du = slot_dense(a, slot);
      if (du >= 0) dense_job(a, tabs, du, c, red, part);
      else conv_job(a, slot_conv(a, slot), c, red, part);
      if (j == (int)blockIdx.x) LR_STAMP(6);
      // publish the slab write-through, then the ticket (every storing wave drains first)
      const int npos = slot_dense(a, slot) >= 0 ? kPerThread : 1;
      float* slab = a.slabs + (long long)slot * kChunks * kSlotVals;
#pragma unroll
      for (int e = 0; e < kPerThread; ++e)
        if (e < npos)
          __hip_atomic_store(slab + c * kSlotVals + threadIdx.x + RT * e, part[e], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.tickets + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == (unsigned)(kChunks - 1);
        if (last) __hip_atomic_store(a.tickets + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last;
      }
      __syncthreads();
      if (!s_last) continue;
      ++narr;
      // the slot's owner: local sum of the 8 slabs in chunk order
      if (nown >= kMaxOwned) {  // host guarantees G >= 8 * nslot / kMaxOwned; never spin on a missing owner
        if (threadIdx.x == 0 && LL) atomicOr(a.ll.err, 2);
        continue;
      }
      // write-through (sc1) buffer loads of the slabs, all in flight (an atomic load per value would wait
      // for each one); the first owned slot's old master / momentum values (fused update) are loaded right
      // behind them, so both arrive in one memory round trip (loading and parking those in LDS first had
      // the slab loads wait a whole round trip behind them)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, kChunks * kSlotVals * 4, 0x00020000);
      float x[kChunks][kPerThread];
#pragma unroll
      for (int cc = 0; cc < kChunks; ++cc)
#pragma unroll
        for (int e = 0; e < kPerThread; ++e)
          x[cc][e] = e < npos ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                              rs, (cc * kSlotVals + threadIdx.x + RT * e) * 4, 0, 16))
                              : 0.f;
      if (nown == 0 && pre) {
        // (the position computed here, per job: hoisted out of the job loop, the per-position row / column
        // terms were spilled to scratch)
        int tid_o = threadIdx.x;
        asm volatile("" : "+v"(tid_o));
#pragma unroll
        for (int e = 0; e < kPerThread; ++e) {
          float w = 0.f, m = 0.f;
          if (e < npos) {
            const Owned o = owned_elem(a, tabs, slot, tid_o + RT * e);
            if (o.di >= 0) {
              const long long off = tabs.d[o.di].off + o.i;
              w = a.sgd.master[off];
              m = a.sgd.mom != nullptr ? a.sgd.mom[off] : 0.f;
            }
          }
          w_pre[e][threadIdx.x] = w;
          m_pre[e][threadIdx.x] = m;
        }
      }
      float v[kPerThread];
#pragma unroll
      for (int e = 0; e < kPerThread; ++e) {
        v[e] = x[0][e];
#pragma unroll
        for (int cc = 1; cc < kChunks; ++cc) v[e] += x[cc][e];
      }
      // keep the local sums: the first owned slot's in LDS, later ones (shared-GPU runs) in chunk 0's slab
      // (read back by the same threads after the jobs)
#pragma unroll
      for (int e = 0; e < kPerThread; ++e)
        if (e < npos) {
          if (nown == 0) own0[e][threadIdx.x] = v[e];
          else slab[threadIdx.x + RT * e] = v[e];
        }
      if (LL) {
        const unsigned ee = ll_epoch(a.ll, slot, &s_e);
        if (threadIdx.x == 0) ep[nown] = ee;
#pragma unroll
        for (int e = 0; e < kPerThread; ++e)
          if (e < npos) ll_push(a.ll, slot, threadIdx.x + RT * e, ee, v[e]);
      }
      if (threadIdx.x == 0) owned[nown] = slot;
      ++nown;
      if (nown == 1) LR_STAMP(7);
    }
    __syncthreads();
    LR_STAMP(1);
    const unsigned dec = (PS && nown > 0) ? lenet_ps_wait(a, &s_dec) : 0u;
    __shared__ unsigned s_tP[kP2PMaxRanks], s_tn[kP2PMaxRanks], s_tq, s_tep;
    if (OWN && nown > 0) {  // owner-applies: the admission's drain decision (see the successor path)
      if (threadIdx.x == 0) {
        s_tq = a.ps.scratch[kPSSeq];
        s_tep = __hip_atomic_load(a.ps.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
      }
      __syncthreads();
      lenet_ps_owner_load(a.ps, s_tep, s_tP, s_tn);
      __syncthreads();
    }
    LR_STAMP(2);
#pragma unroll 1
    for (int k = 0; k < nown; ++k) {
      const int slot = owned[k];
      const int npos = slot_dense(a, slot) >= 0 ? kPerThread : 1;
      const float* sum = a.slabs + (long long)slot * kChunks * kSlotVals;
      // gather every position's element, local sum and old weight first (all loads in flight), then
      // the rank sums, then the arithmetic, then the stores: no load waits behind a store
      Owned o[kPerThread];
      float v[kPerThread], w0[kPerThread], m0[kPerThread];
      int tid_o = threadIdx.x;  // (per owned slot, not hoisted: see the job loop)
      asm volatile("" : "+v"(tid_o));
#pragma unroll
      for (int e = 0; e < kPerThread; ++e) {
        const int pos = tid_o + RT * e;
        o[e] = e < npos ? owned_elem(a, tabs, slot, pos) : Owned{-1, 0};
        v[e] = e < npos ? (k == 0 ? own0[e][threadIdx.x] : sum[pos]) : 0.f;
        w0[e] = m0[e] = 0.f;
        if (a.sgd_on && !PS && o[e].di >= 0) {
          if (k == 0 && pre) {
            w0[e] = w_pre[e][threadIdx.x];
            m0[e] = m_pre[e][threadIdx.x];
          } else {
            const long long off = tabs.d[o[e].di].off + o[e].i;
            w0[e] = a.sgd.master[off];
            m0[e] = a.sgd.mom != nullptr ? a.sgd.mom[off] : 0.f;
          }
        }
      }
      if (OWN) {
        const PSArgs& p = a.ps;
        float wn[kPerThread];
#pragma unroll
        for (int e = 0; e < kPerThread; ++e) {
          wn[e] = 0.f;
          if (o[e].di < 0) continue;
          float d;
          {
#pragma clang fp contract(off)
            d = -(tabs.hyper[0] * v[e]);
          }
          wn[e] = lenet_ps_owner_elem(p, s_shard, s_inbox, s_tP, s_tn, tabs.d[o[e].di].off + o[e].i, d,
                                      dec == kPSAccept, s_tq);
        }
        if (dec == kPSAccept || dec == kPSReject) {
#pragma unroll
          for (int e = 0; e < kPerThread; ++e) {
            if (o[e].di < 0) continue;
            tabs.g[o[e].di][o[e].i] = v[e];
            if (npos > 1) red_emit<true>(a, tabs, o[e], wn[e]);
            else if (e == 0) red_emit<false>(a, tabs, o[e], wn[e]);
          }
        }
        if (k == 0) LR_STAMP(5);
        continue;
      }
      if (PS) {
        if (dec == kPSAccept || dec == kPSReject) {
          // the elements' shard addresses; admitted: every add in flight at once (w += -lr * g on the
          // owning shard, the local copies take the value each add produced); rejected: the shards'
          // current values.  The learning rate is the device hyper-parameter (set_lr after capture holds).
          const PSArgs& p = a.ps;
          float* pe[kPerThread];
          float d[kPerThread], wn[kPerThread];
#pragma unroll
          for (int e = 0; e < kPerThread; ++e) {
#pragma clang fp contract(off)
            d[e] = -(tabs.hyper[0] * v[e]);
            pe[e] = o[e].di >= 0 ? ps_elem(s_shard, p.shard_shift, tabs.d[o[e].di].off + o[e].i) : nullptr;
          }
          if (dec == kPSAccept) {
            ps_add<kPerThread>(pe, d, wn, p.excl != 0, p);
          } else {
#pragma unroll
            for (int e = 0; e < kPerThread; ++e)
              wn[e] = pe[e] ? __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(pe[e]), __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_SYSTEM))
                            : 0.f;
          }
#pragma unroll
          for (int e = 0; e < kPerThread; ++e) {
            if (o[e].di < 0) continue;
            tabs.g[o[e].di][o[e].i] = v[e];
            if (npos > 1) red_emit<true>(a, tabs, o[e], wn[e]);
            else if (e == 0) red_emit<false>(a, tabs, o[e], wn[e]);
          }
        }
        if (k == 0) LR_STAMP(5);
        continue;
      }
      bool ok[kPerThread];
#pragma unroll
      for (int e = 0; e < kPerThread; ++e) {
        ok[e] = true;
        // the rank-order sum over the ranks (no all-reduce launch)
        if (LL && e < npos) ok[e] = ll_wait_sum(a.ll, slot, threadIdx.x + RT * e, ep[k], v[e], v[e]);
      }
      if (LL && k == 0) LR_STAMP(5);
      if (npos > 1) {  // a dense unit
#pragma unroll
        for (int e = 0; e < kPerThread; ++e)
          if (ok[e]) red_apply<true>(a, tabs, o[e], v[e], w0[e], m0[e]);
      } else if (ok[0]) {
        red_apply<false>(a, tabs, o[0], v[0], w0[0], m0[0]);
      }
      if (LL) {
        __syncthreads();  // every position of the slot consumed before its epoch advances
        ll_commit(a.ll, slot, ep[k]);
      }
    }
    LR_STAMP(3);
    if (PS) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's shard adds have landed
      lenet_ps_arrive(a, (unsigned)narr, (unsigned)(nslot + 2));
    }
    LR_STAMP(4);
    LR_FLUSH();
    return;
  }
  const int blk = blockIdx.x - G;
  if (blk == 1 && PSX) {
    LR_FLUSH();
    return;
  }
  if (blk == 2 && PSX) {
    // mode 3: the admission (train launch) has read this step's microbatch id already: claim the next one
    // and stage its example indices straight away
    __shared__ long long s_bidx;
    LR_STAMP(8);
    if (a.ps.done_epoch != nullptr) {
      claim_microbatch(a.ps, threadIdx.x, &s_bidx);
    } else if (threadIdx.x == 0) {
      s_bidx = (long long)(__hip_atomic_fetch_add(a.ps.batch_ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) %
                           (unsigned long long)(a.ps.nbatches > 0 ? a.ps.nbatches : 1));
    }
    __syncthreads();
    if (threadIdx.x == 0) *a.ps.bid_out = s_bidx;
    ps_stage_indices(a.ps, s_bidx, threadIdx.x, RT);
    LR_STAMP(10);
    LR_FLUSH();
    return;
  }
  if (blk == 1 && PS) {
    // async: the admission ran in the train launch (lenet_ps_admission); this workgroup's arrival keeps the
    // launch epoch from advancing before the decision of this launch exists
    LR_STAMP(8);
    lenet_ps_arrive(a, 1u, (unsigned)(nslot + 2));
    LR_STAMP(1);
    LR_FLUSH();
    return;
  }
  if (blk == 2 && PS) {
    // beside the admission: claim the next microbatch FCFS on the server (its remote atomics no longer
    // follow the admission's), then -- once the admission has read this step's microbatch id (its decision
    // is out) -- publish the new id and stage its example indices
    __shared__ long long s_bid;
    __shared__ unsigned s_ep;
    LR_STAMP(8);
    if (threadIdx.x == 0)
      s_ep = __hip_atomic_load(a.ps.scratch + kPSEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (a.ps.done_epoch != nullptr) {
      claim_microbatch(a.ps, threadIdx.x, &s_bid);
    } else if (threadIdx.x == 0) {
      s_bid = (long long)(__hip_atomic_fetch_add(a.ps.batch_ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) %
                          (unsigned long long)(a.ps.nbatches > 0 ? a.ps.nbatches : 1));
    }
    __syncthreads();
    LR_STAMP(9);
    if (threadIdx.x == 0) {
      // (the epoch cannot advance before this workgroup arrives: it is one of the launch's arrivals)
      const unsigned long long t0 = wall_clock64();
      while (!ps_epoch_eq(__hip_atomic_load(a.ps.scratch + kPSDecision, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                          s_ep)) {
        if (wall_clock64() - t0 > 2ull * (unsigned long long)a.ps.timeout_ticks) {
          atomicOr(a.ps.stats + 5, 8ull);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      *a.ps.bid_out = s_bid;
    }
    ps_stage_indices(a.ps, s_bid, threadIdx.x, RT);
    LR_STAMP(10);
    lenet_ps_arrive(a, 1u, (unsigned)(nslot + 2));
    LR_FLUSH();
    return;
  }
  if (blk == 1) {  // fused update: stage the next step's batch indices, advance the cursor
    __shared__ long long nxt;
    if (threadIdx.x == 0) nxt = (*a.sgd.cursor + 1) % a.sgd.nsteps;
    __syncthreads();
    copy_i64(a.sgd.dst, a.sgd.src + nxt * a.sgd.B, a.sgd.B, threadIdx.x, RT);
    if (threadIdx.x == 0) *a.sgd.cursor = nxt;
    LR_STAMP(1);
    LR_FLUSH();
    return;
  }
  {  // loss partials -> stats: every load of the block in flight at once, fixed-order sums
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2* lp = reinterpret_cast<const f32x2*>(a.loss_part);
    f32x2 acc = {0.f, 0.f};
    for (int k0 = threadIdx.x; k0 < a.nblk; k0 += RT * 8) {
      f32x2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = k0 + RT * u < a.nblk ? lp[k0 + RT * u] : f32x2{0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    float l = wave_sum(acc.x), c = wave_sum(acc.y);
    __shared__ float s_lc[2][RT / 64];
    if (lane == 0) {
      s_lc[0][wid] = l;
      s_lc[1][wid] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      l = s_lc[0][0];
      c = s_lc[1][0];
#pragma unroll
      for (int w = 1; w < RT / 64; ++w) {
        l += s_lc[0][w];
        c += s_lc[1][w];
      }
      a.stats[0] = l;
      a.stats[1] = c;
      if (a.sgd_on && a.sgd.run_stats != nullptr) {  // device run statistics (trainer callbacks)
        a.sgd.run_stats[0] += l;
        a.sgd.run_stats[1] += c;
        a.sgd.run_stats[2] += 1.f;
      }
    }
  }
  LR_STAMP(1);
  LR_FLUSH();
}

}  // namespace

size_t lenet_train_lds() { return LDS_BYTES; }
// images per train workgroup: the smallest of 1, 2, 4, 8 that keeps the grid within one workgroup per CU
// (256), else 8.  Measured (one MI355X, sync step, 200 steps; profiles/r6/lenet_ipw_sweep.txt): B = 32
// 26.7 us with 1 image per workgroup vs 39.1 with 8; B = 256 28.0 vs 39.9; B = 1024 36.8 (4) vs 43.0 (8) and
// 43.9 (2, 512 workgroups); B = 2048 45.4 (8) vs 48.9 (4).  DISTRIFLOW_DIAG=lenet_ipw=<1|2|4|8> forces one.
int lenet_ipw(int B) {
  static const int forced = diag_int("lenet_ipw", 0);
  if (forced == 1 || forced == 2 || forced == 4 || forced == IMG) return forced;
  int ipw = 1;
  while (ipw < IMG && (B + ipw - 1) / ipw > 256) ipw *= 2;
  return ipw;
}
int lenet_blocks(int B) {
  const int ipw = lenet_ipw(B);
  return (B + ipw - 1) / ipw;
}

static unsigned long long* g_lenet_stamps_host = nullptr;
void lenet_set_stamps(void* buf) { g_lenet_stamps_host = reinterpret_cast<unsigned long long*>(buf); }

size_t lenet_frag_bytes() { return (size_t)NFRAG * 64 * 16; }

// reduce scratch (the trainer's dense_part buffer, zero-initialised): job slabs + arrival tickets
static int lenet_red_slots() {
  const int NK[3][2] = {{120, 400}, {84, 120}, {10, 84}};
  int n = (kLeNetConvParams + kConvPer - 1) / kConvPer;
  for (auto& nk : NK) n += ((nk[0] + kDU - 1) / kDU) * ((nk[1] + 1 + kDU - 1) / kDU);
  return n;
}
// [slabs: slots x 8 x 1024 f32][tickets: round4(slots)][granules: slots x 8 x 1024 u64][per-workgroup
// launch counters: round4(8 x (slots + 1))][granule error word, padded to 4][slot arrivals: round4(slots)]
static int lenet_red_slab_floats() { return lenet_red_slots() * kChunks * kSlotVals; }
static int lenet_red_ep_words() { return (kChunks * (lenet_red_slots() + 1) + 3) / 4 * 4; }
int lenet_dense_part_floats(int B) {
  (void)B;
  return 3 * lenet_red_slab_floats() + 2 * ((lenet_red_slots() + 3) / 4 * 4) + lenet_red_ep_words() + 4;
}
int lenet_red_err_offset() {
  return 3 * lenet_red_slab_floats() + (lenet_red_slots() + 3) / 4 * 4 + lenet_red_ep_words();
}
void lenet_red_bind_scratch(float* base, LeNetRedArgs& r) {
  r.slabs = base;
  base += lenet_red_slab_floats();
  r.tickets = reinterpret_cast<unsigned*>(base);
  base += (lenet_red_slots() + 3) / 4 * 4;
  r.gran = reinterpret_cast<unsigned long long*>(base);  // 16-byte aligned (every term is a multiple of 4)
  base += 2 * lenet_red_slab_floats();
  r.gran_ep = reinterpret_cast<unsigned*>(base);
  base += lenet_red_ep_words();
  r.gran_err = reinterpret_cast<unsigned*>(base);
  base += 4;
  r.slot_arr = reinterpret_cast<unsigned*>(base);
}

hipError_t lenet_train(const LeNetArgs& a_in, LeNetRedArgs r, hipStream_t st) {
  LeNetArgs a = a_in;
  a.stamps = g_lenet_stamps_host;
  // the reduce launch's clocks follow the train kernel's [4096][16] region
  r.stamps = g_lenet_stamps_host ? g_lenet_stamps_host + 4096 * 16 : nullptr;
  if (a.B <= 0 || a.ldt % 32 || a.ldt < a.B || !a.frag || !a.ftab || !a.pxtab) return hipErrorInvalidValue;
  a.ipw = lenet_ipw(a.B);
  const int nblk = (a.B + a.ipw - 1) / a.ipw;
  if (a.prep) {
    hipLaunchKernelGGL(lenet_prep_kernel, dim3(1), dim3(PT), 0, st, a.w1, a.w2,
                       reinterpret_cast<bf16x8*>(const_cast<void*>(a.frag)));
    DFA_HIP_CHECK(hipGetLastError());
  }
  a.nblk = nblk;
  a.ps_admit = r.ps_on;
  // (the admission workgroup runs in this launch: its parameter-server words are checked here)
  if (r.ps_on && (!r.ps.ver || !r.ps.vpulled || !r.ps.bid_out || !r.ps.stats || !r.ps.scratch))
    return hipErrorInvalidValue;
  if (r.ps_on) a.ps = r.ps;
  r.nblk = nblk;
  r.ldt = a.ldt;
  if (r.kcols <= 0 || r.kcols % 32 || r.kcols > a.ldt || r.kcols < a.B) return hipErrorInvalidValue;
  r.nconv_slots = (kLeNetConvParams + kConvPer - 1) / kConvPer;
  // dense units in (layer, tk, tn) order, tn fastest
  int base = 0;
  for (int l = 0; l < 3; ++l) {
    r.L[l].tiles = ((r.L[l].N + kDU - 1) / kDU) * ((r.L[l].K + 1 + kDU - 1) / kDU);
    base += r.L[l].tiles;
  }
  r.dense_tiles = base;
  // the kernel's LDS table image
  for (int l = 0; l < 3; ++l) {
    r.tab.L[l] = r.L[l];
    r.tab.g[4 + 2 * l] = r.L[l].gw;
    r.tab.g[5 + 2 * l] = r.L[l].gb;
  }
  r.tab.g[0] = r.g_w1;
  r.tab.g[1] = r.g_b1;
  r.tab.g[2] = r.g_w2;
  r.tab.g[3] = r.g_b2;
  for (int j = 0; j < 10; ++j) r.tab.d[j] = r.sgd.d[j];
  // chunk c of the batch = the columns of XCD c's train workgroups (lenet_img_group) when B = 4096
  r.chunk_cols = ((r.kcols + kChunks - 1) / kChunks + 31) / 32 * 32;
  if (!r.slabs || !r.tickets) return hipErrorInvalidValue;
  if (r.sgd_on && (!r.sgd.master || !r.sgd.wbf || !r.sgd.hyper || !r.sgd.frag))
    return hipErrorInvalidValue;
  if (r.sgd_on)  // dense weights: tile-layout compute copies (red_emit's fast path), biases: none
    for (int l = 0; l < 3; ++l) {
      const ParamDesc& dw = r.sgd.d[4 + 2 * l];
      const ParamDesc& db = r.sgd.d[5 + 2 * l];
      if (!((dw.pad_ >> 28) & 1) || dw.T != 1 || dw.bf_off < 0 || dw.bft_off < 0 || db.bf_off >= 0)
        return hipErrorInvalidValue;
    }
  const int nslot = r.dense_tiles + r.nconv_slots;
  const int njobs = nslot * kChunks;
  // successor ownership needs one job per workgroup (not the time-shared grid of several ranks on one
  // GPU) and, multi-rank, the per-part LL epoch words
  if (r.succ && (!(r.exch_blocks <= 0 || r.exch_blocks >= njobs) || !r.gran || !r.gran_ep || !r.gran_err ||
                 !r.slot_arr || nslot > lenet_red_slots() || (r.ll_on && !r.ll.part_epochs)))
    r.succ = 0;
  if (r.succ) r.exch_blocks = njobs + kChunks;  // + the owner-only group of the last slot
  else if (r.exch_blocks <= 0 || r.exch_blocks > njobs) r.exch_blocks = njobs;
  // one rank, sync, fused update, small batch: one workgroup per slot (the whole-batch job: <= 64 partial
  // rows and <= 512 batch columns keep it to one load round per wave).  Its sums run in another fp32 order
  // than the 8-way split's (deterministic), so the gradient-only launch -- the multi-rank exchange's
  // self-test compares the exchange against it bit for bit -- keeps the split path.
  // DISTRIFLOW_DIAG=lenet_solo=0|1 forces it off / on.
  {
    static const int solo_diag = diag_int("lenet_solo", -1);
    const bool eligible = !r.ll_on && !r.ps_on && r.sgd_on;
    r.solo = eligible && (solo_diag == 1 || (solo_diag != 0 && nblk <= 64 && r.kcols <= 512)) ? 1 : 0;
    if (r.solo) r.exch_blocks = nslot;
  }
  // a workgroup runs <= ceil(njobs / G) jobs, so it owns at most that many slots
  if ((long long)r.exch_blocks * kMaxOwned < njobs) return hipErrorInvalidValue;
  // 256-thread workgroups at <= 128 VGPRs and ~17 KB LDS: 4 per CU, 1024 on the chip
  if (r.ll_on) {
    // slot s is LL slot s.  Every workgroup that owns a slot waits for the peers' sums of it, so all job
    // workgroups must fit on the chip at once (a waiting owner must never keep a job it depends on, here
    // or on a peer, from being dispatched)
    if (!r.sgd_on || r.ll.world < 2 || r.ll.world > kP2PMaxRanks || r.ll.rank < 0 || r.ll.rank >= r.ll.world ||
        !r.ll.epochs || !r.ll.err || nslot > r.ll.nslots || r.exch_blocks + 2 > 1024)
      return hipErrorInvalidValue;
    for (int k = 0; k < r.ll.world; ++k)
      if (!r.ll.bases[k]) return hipErrorInvalidValue;
  }
  if (r.ps_on) {
    // async PS: the owners wait for workgroup 0's decision (dispatched first)
    if (!r.sgd_on || r.ll_on || r.sgd.src || !r.ps.ver || !r.ps.vpulled || !r.ps.bid_out || !r.ps.stats ||
        !r.ps.scratch || r.exch_blocks + 3 > 1024 || r.sgd.mom || r.ps.nshards < 1 || r.ps.nshards > kP2PMaxRanks ||
        r.ps.shard_shift < 6 || ((r.ps.n - 1) >> r.ps.shard_shift) >= r.ps.nshards)
      return hipErrorInvalidValue;
    for (int k = 0; k < r.ps.nshards; ++k)
      if (!r.ps.shard[k]) return hipErrorInvalidValue;
    // owner-applies (mode 4): a ring slot is rewritten R sequence numbers later; every owner has drained it by
    // then only if an admitted gradient is at most R - 2 behind (ps_apply's rule), and the inbox tables exist
    if (r.ps.owner_ring > 0) {
      if (r.ps.owner_ring > 255 || r.ps.max_stale < 0 || r.ps.owner_ring < r.ps.max_stale + 2 || !r.ps.pref ||
          !r.ps.dlock || r.ps.rank < 0)
        return hipErrorInvalidValue;
      for (int k = 0; k < r.ps.nshards; ++k)
        if (!r.ps.inbox[k]) return hipErrorInvalidValue;
    }
  }
  // async PS with one rank and successor ownership: mode 3 (the synchronous owners' update gated on the
  // admission, mirrored into the one shard; the admission advances the epoch itself).  Decided before the
  // train launch, whose admission workgroup runs the matching protocol.
  const bool psx = r.ps_on && r.ps.excl != 0 && r.succ && r.ps.nshards == 1 && r.ps.owner_ring <= 0;
  a.ps_excl = psx ? 1 : 0;
  r.mirror = psx ? r.ps.shard[0] : nullptr;
  if (a.ipw < IMG)
    hipLaunchKernelGGL(lenet_train_kernel<true>, dim3(nblk + (r.ps_on ? 1 : 0)), dim3(NT), LDS_BYTES, st, a);
  else
    hipLaunchKernelGGL(lenet_train_kernel<false>, dim3(nblk + (r.ps_on ? 1 : 0)), dim3(NT), LDS_BYTES, st, a);
  DFA_HIP_CHECK(hipGetLastError());
  // the index-staging workgroup; async PS: the admission and the claim / staging workgroups
  const int extra = r.ps_on ? 2 : ((r.sgd_on && r.sgd.src) ? 1 : 0);
  const dim3 grid(r.exch_blocks + 1 + extra);
  if (r.ll_on) hipLaunchKernelGGL(lenet_reduce_kernel<1>, grid, dim3(RT), 0, st, r);
  else if (psx) hipLaunchKernelGGL(lenet_reduce_kernel<3>, grid, dim3(RT), 0, st, r);
  else if (r.ps_on && r.ps.owner_ring > 0) hipLaunchKernelGGL(lenet_reduce_kernel<4>, grid, dim3(RT), 0, st, r);
  else if (r.ps_on) hipLaunchKernelGGL(lenet_reduce_kernel<2>, grid, dim3(RT), 0, st, r);
  else hipLaunchKernelGGL(lenet_reduce_kernel<0>, grid, dim3(RT), 0, st, r);
  return hipGetLastError();
}

}  // namespace dfa
