// The reference CNN's dense head (gfx950): flatten 4608 -> dense 128 ReLU -> dropout 0.5 -> dense C
// (softmax cross-entropy), trained by ONE launch for the forward, the loss and both data gradients, plus
// the fused head weight-gradient launch (csrc/mlphead.hip head_wgrad_kernel).
//
// The reference trains this head as tf.js matMul / add / relu / dropout / softmax-CE ops and their
// gradients (/root/reference/experiment/mnist/model.json, DistributedTfModel.fit
// /root/reference/src/common/models.ts:128-142).  Its first GEMM is K = 4608 deep but only N = 128
// wide: at B = 1024 one workgroup per 16 batch rows (the LeNet head kernel) would stream all of W1
// (1.2 MB) through each of 64 CUs.  Here the K dimension is split instead:
//
//   job (row tile rt of 32 batch rows, chunk c of K/8 columns), c = blockIdx % 8 so every XCD keeps
//   its own chunk of W1 / W1^T resident in its L2:
//     1. stage P[rt rows][chunk] in LDS (and write its transpose P^T for the weight gradient)
//     2. Z1 partial = P_chunk W1_chunk^T (MFMA 16x16x32), written as a write-through (sc1) slab
//     3. ticket; the row tile's LAST arriver (the owner) sums the 8 slabs in chunk order, applies bias,
//        ReLU and the folded dropout -> H1, runs dense2 (32 x 128 x C), softmax-CE, dZ2, dH1 = dZ2 W2 *
//        relu'(H1) * 1/(1-p) = dZ1, writes H1^T / dZ1^T / dZ2^T (weight-gradient operands) and the loss
//        partials, and publishes dZ1 (sc1 stores) behind a tagged flag
//     4. all 8 jobs of the row tile: dP_chunk = dZ1 W1_chunk (MFMA), * alpha, relu'(P) -> dp
//   The hand-off is the fence-free sc1 form of csrc/bn_epi.h (stores drained by s_waitcnt vmcnt(0)
//   before the relaxed agent-scope ticket / flag; sc1 loads on the reading side).  The grid is
//   persistent (G <= CU count, a multiple of 8), so the 8 jobs of a row tile always run concurrently
//   and the flag wait cannot starve; the flags compare against a per-launch tag that the last finishing
//   workgroup advances (graph replays need no host-side counter).
// Numerics match the per-layer path (igemm64 forward / split-K epilogue, mlphead dense2 + CE,
// igemm64 data gradient): the same epilogue order and roundings, fp32 sums in a fixed order.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dfa {
namespace {

constexpr int KT = 256;                // threads per workgroup (4 waves)
constexpr int KR = kKHeadRows;         // 32 batch rows per row tile
constexpr int KCH = kKHeadChunks;      // 8 K chunks per row tile
constexpr int N1 = kKHeadN1;           // dense1 width
constexpr int LDH = N1 + 8;            // LDS row stride of H1 / dZ1 tiles (bf16)
constexpr int LDZ2 = 40;               // LDS row stride of the dZ2 tile (32 columns used)
constexpr int SLAB = KR * N1;          // floats per partial slab
constexpr int kStageMax = 12;          // 16-byte P loads per thread when staging (KC <= 768)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 ld16(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

unsigned long long* g_khead_stamps = nullptr;

// per-workgroup phase clocks of its first job (diagnostic; scripts/kheadstamps.py)
#define KH_STAMP(slot)                                                             \
  do {                                                                             \
    if (a.stamps && first) {                                                       \
      __builtin_amdgcn_sched_barrier(0);                                           \
      unsigned long long t_;                                                       \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                           \
      if (threadIdx.x == 0) a.stamps[blockIdx.x * 16 + (slot)] = t_;               \
    }                                                                              \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

struct KHeadLds {
  bf16* ps;   // [32][KC + 8] P tile (then dP in place)
  bf16* hs;   // [32][LDH] H1
  bf16* dz1;  // [32][LDH] dZ1
  bf16* dz2;  // [32][LDZ2] dZ2 (columns >= C zero)
  float* lg;  // [32][16] logits
  int ldp;
};

__device__ __forceinline__ KHeadLds carve(char* smem, int KC) {
  KHeadLds s;
  s.ldp = KC + 8;
  s.ps = reinterpret_cast<bf16*>(smem);
  char* p = smem + round_up(KR * s.ldp * 2, 16);
  s.hs = reinterpret_cast<bf16*>(p);
  p += KR * LDH * 2;
  s.dz1 = reinterpret_cast<bf16*>(p);
  p += KR * LDH * 2;
  s.dz2 = reinterpret_cast<bf16*>(p);
  p += KR * LDZ2 * 2;
  s.lg = reinterpret_cast<float*>(p);
  return s;
}

// The row tile's owner, part 1: Z1 = sum of the 8 slabs in chunk order (this thread's 4 fragments:
// m-tile m, n-tile 2 * wid + t), all write-through loads in flight.
__device__ __forceinline__ void khead_combine(const KHeadArgs& a, int rt, f32x4* z) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float* slab = a.slab + (long long)rt * KCH * SLAB;
  const __amdgpu_buffer_rsrc_t rs = rsrc(slab, KCH * SLAB * 4);
  u32x4 x[KCH][4];
#pragma unroll
  for (int c = 0; c < KCH; ++c)
#pragma unroll
    for (int f = 0; f < 4; ++f)
      x[c][f] = __builtin_amdgcn_raw_buffer_load_b128(rs, (c * SLAB + ((wid * 4 + f) * 64 + lane) * 4) * 4, 0, 16);
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    z[f] = __builtin_bit_cast(f32x4, x[0][f]);
#pragma unroll
    for (int c = 1; c < KCH; ++c) z[f] += __builtin_bit_cast(f32x4, x[c][f]);
  }
}

// Part 2: H1 -> dense2 -> CE -> dZ2 -> dZ1, published.
__device__ __forceinline__ void khead_owner(const KHeadArgs& a, const KHeadLds& s, int rt, const f32x4* z) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, tid = threadIdx.x;
  const int r0 = rt * KR;
  // the small operands: W2 rows, W2^T rows, biases, labels
  bf16x8 w2f[4], w2tf[2];
  if (wid < 2)
#pragma unroll
    for (int k = 0; k < 4; ++k) w2f[k] = ld16(a.w2 + (lane & 15) * N1 + 8 * (lane >> 4) + 32 * k);
#pragma unroll
  for (int t = 0; t < 2; ++t) w2tf[t] = ld16(a.w2t + (16 * (2 * wid + t) + (lane & 15)) * 32 + 8 * (lane >> 4));
  float b1v[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) b1v[t] = a.b1 ? a.b1[16 * (2 * wid + t) + (lane & 15)] : 0.f;
  const float b2v = (a.b2 && (lane & 15) < a.C) ? a.b2[lane & 15] : 0.f;
  int ylab = 0;
  if (tid < KR && r0 + tid < a.B) {
    const long long src = a.idx ? a.idx[r0 + tid] : (long long)(r0 + tid);
    ylab = a.labels[src < 0 ? 0 : (src >= a.nrows ? a.nrows - 1 : src)];
  }
  // ---- 2. H1 = drop(relu(Z1 + b1)) (igemm64 epilogue order), to LDS and H1^T
  const unsigned long long ds = a.drop.on ? drop_seed(a.drop.seed, a.drop.step, a.drop.step_add) : 0ull;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const int m = f >> 1, t = f & 1;
    const int col = 16 * (2 * wid + t) + (lane & 15);
    const int rb = 16 * m + 4 * (lane >> 4);
    const float bv = b1v[t];
    bf16x4 hv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = fmaxf(z[f][r] + bv, 0.f);
      if (a.drop.on)
        v = drop_keep(ds, a.drop.thresh, (long long)(r0 + rb + r) * N1 + col) ? (float)f2bf(v) * a.drop.scale : 0.f;
      if (r0 + rb + r >= a.B) v = 0.f;
      hv[r] = f2bf(v);
      s.hs[(rb + r) * LDH + col] = hv[r];
    }
    *reinterpret_cast<bf16x4*>(a.h1T + (long long)col * a.ldt + r0 + rb) = hv;
  }
  __syncthreads();
  // ---- 3. dense2 forward: logits[32][16] (waves 0, 1: one m-tile each)
  if (wid < 2) {
    const int n = lane & 15;
    const bf16* arow = s.hs + (16 * wid + (lane & 15)) * LDH + 8 * (lane >> 4);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) acc = mfma16x16x32(ld16(arow + 32 * k), w2f[k], acc);
    const float bv = b2v;
#pragma unroll
    for (int r = 0; r < 4; ++r) s.lg[(16 * wid + 4 * (lane >> 4) + r) * 16 + n] = n < a.C ? acc[r] + bv : 0.f;
  }
  __syncthreads();
  // ---- 4. softmax cross-entropy (one lane per row; mlphead's arithmetic), loss partials per 16 rows
  if (tid < KR) {
    const int r = tid, row = r0 + r;
    const int C = a.C;
    float lsum = 0.f, corr = 0.f;
    float g[16];  // (every index static: no private-array indexing)
#pragma unroll
    for (int c = 0; c < 16; ++c) g[c] = 0.f;
    if (row < a.B) {
      const int y = ylab < 0 ? 0 : (ylab >= C ? C - 1 : ylab);
      float z[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) z[c] = s.lg[r * 16 + c];
      float mx = -INFINITY, zy = 0.f;
      int am = 0;
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (c < C) {
          if (a.logits) a.logits[(long long)row * C + c] = z[c];
          if (z[c] > mx) {
            mx = z[c];
            am = c;
          }
          if (c == y) zy = z[c];
        }
      float pr[16];
      float sum = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (c < C) {
          pr[c] = __expf(z[c] - mx);
          sum += pr[c];
        }
      const float inv = 1.f / sum;
      lsum = -(zy - mx - __logf(sum));
      corr = am == y ? 1.f : 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (c < C) g[c] = (pr[c] * inv - (c == y ? 1.f : 0.f)) * a.grad_scale;
    }
#pragma unroll
    for (int c = 0; c < 32; ++c) s.dz2[r * LDZ2 + c] = f2bf(c < 16 ? g[c & 15] : 0.f);
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (c < C) a.dz2T[(long long)c * a.ldt + row] = f2bf(g[c]);
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {  // fixed-order tree over each 16-row half (mlphead's partials)
      lsum += __shfl_xor(lsum, o, 16);
      corr += __shfl_xor(corr, o, 16);
    }
    const int q = (r0 + r) / 16;
    if ((r & 15) == 0 && q < (a.B + 15) / 16) {
      a.loss_part[2 * q] = lsum;
      a.loss_part[2 * q + 1] = corr;
    }
  }
  __syncthreads();
  // ---- 5. dZ1 = (dZ2 W2) * relu'(H1) * dh_scale: n-tiles 2 * wid + t, both m-tiles, K = 32
  {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = 16 * (2 * wid + t) + (lane & 15);
      const bf16x8 b = w2tf[t];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const f32x4 acc = mfma16x16x32(ld16(s.dz2 + (16 * m + (lane & 15)) * LDZ2 + 8 * (lane >> 4)), b,
                                       f32x4{0.f, 0.f, 0.f, 0.f});
        const int rb = 16 * m + 4 * (lane >> 4);
        bf16x4 dv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[r];
          if (!((float)s.hs[(rb + r) * LDH + j] > 0.f)) v = 0.f;
          if (a.dh_scale != 1.f) v = (float)f2bf(v) * a.dh_scale;
          dv[r] = f2bf(v);
          s.dz1[(rb + r) * LDH + j] = dv[r];
        }
        *reinterpret_cast<bf16x4*>(a.dz1T + (long long)j * a.ldt + r0 + rb) = dv;
      }
    }
  }
  __syncthreads();
  // ---- 6. publish dZ1 (write-through) behind the row tile's flag
  {
    const __amdgpu_buffer_rsrc_t ws = rsrc(a.dz1 + (long long)rt * KR * N1, KR * N1 * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + KT * i, row = q >> 4, c8 = (q & 15) * 8;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ld16(s.dz1 + row * LDH + c8)), ws,
                                             (row * N1 + c8) * 2, 0, 16);
    }
  }
}

}  // namespace

void khead_set_stamps(void* buf) { g_khead_stamps = reinterpret_cast<unsigned long long*>(buf); }
// ranks time-sharing one GPU (rehearsals): each rank's persistent grid gets its share of the CUs, so the 8
// jobs of a row tile can be resident together beside the other ranks' kernels (0: the whole chip)
static int g_khead_cap = 0;
constexpr unsigned long long kKHeadWaitTicks = 200000000ull;  // 2 s of wall_clock64 (100 MHz)
void khead_set_grid_cap(int cus) { g_khead_cap = cus > 0 ? cus : 0; }

// KSC: k-steps per chunk at compile time (0: run-time loops).  (Issuing the W1 / W1^T operand loads a
// phase earlier -- behind the P loads, before the flag wait -- measured slower: the ~144 VGPRs they hold
// across the phase spill; docs/RESULTS.md.)
template <int KSC>
__global__ void __launch_bounds__(KT) khead_train_kernel(KHeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the wave index in an SGPR: per-wave tile counts become scalar branches
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), tid = threadIdx.x;
  const int KC = a.K / KCH, KS = KC / 32;
  const KHeadLds s = carve(smem, KC);
  unsigned* tickets = a.sync;
  unsigned* flags = a.sync + a.ntiles;
  unsigned* tagp = a.sync + 2 * a.ntiles;
  __shared__ unsigned s_tag;
  __shared__ int s_last;
  if (tid == 0) s_tag = __hip_atomic_load(tagp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int njobs = a.ntiles * KCH;
#pragma unroll 1
  for (int j = blockIdx.x; j < njobs; j += a.G) {
    const int rt = j / KCH, c = j - KCH * (j / KCH);
    const int r0 = rt * KR, kc0 = c * KC;
    const bool first = j == (int)blockIdx.x;
    __syncthreads();  // LDS of the previous job
    KH_STAMP(0);
    // ---- stage P[r0 .. r0 + 32)[kc0 .. kc0 + KC) (rows past B zero): every load in flight, then LDS
    const int c8n = KC / 8;
    {
      // the staging indices computed here, per job (opaque to loop-invariant motion): hoisted out of the job
      // loop, the 12 row / column pairs were spilled to scratch and reloaded one memory latency apart
      int tid_j = tid;
      asm volatile("" : "+v"(tid_j));
      bf16x8 v[kStageMax];
#pragma unroll
      for (int i = 0; i < kStageMax; ++i) {
        const int e = tid_j + KT * i, r = e / c8n, c8 = 8 * (e - r * c8n);
        if (e < KR * c8n) {
          if (r0 + r < a.B) {
            v[i] = ld16(a.p + (long long)(r0 + r) * a.K + kc0 + c8);
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[i][k] = (bf16)0.f;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < kStageMax; ++i) {
        const int e = tid_j + KT * i, r = e / c8n, c8 = 8 * (e - r * c8n);
        if (e < KR * c8n) *reinterpret_cast<bf16x8*>(s.ps + r * s.ldp + c8) = v[i];
      }
    }
    __syncthreads();
    KH_STAMP(1);
    // ---- P^T (the weight-gradient launch's operand): work item = (column pair, 8-row piece); 4 consecutive
    // lanes write the 4 pieces of one pT row, so a store instruction covers 16 rows x 64 contiguous bytes.
    // Written after the ticket (waiters: while the owner works; the owner: after publishing dZ1), not
    // before the partial -- its stores were drained with the slab's in front of every ticket.
    auto write_pT = [&]() {
      for (int w = tid; w < KC * 2; w += KT) {
        const int cp = w >> 2, q = w & 3;
        unsigned v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = *reinterpret_cast<const unsigned*>(s.ps + (8 * q + r) * s.ldp + 2 * cp);
        bf16x8 lo, hi;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          lo[r] = __builtin_bit_cast(bf16, (unsigned short)(v[r] & 0xffffu));
          hi[r] = __builtin_bit_cast(bf16, (unsigned short)(v[r] >> 16));
        }
        bf16* d0 = a.pT + (long long)(kc0 + 2 * cp) * a.ldt + r0 + 8 * q;
        *reinterpret_cast<bf16x8*>(d0) = lo;
        *reinterpret_cast<bf16x8*>(d0 + a.ldt) = hi;
      }
    };
    KH_STAMP(2);
    // ---- Z1 partial: wave w owns n-tiles 2w, 2w + 1 for both m-tiles.  KSC > 0 (the chunk depth known
    // at compile time): every W1 operand load is issued before the first MFMA (one exposed latency);
    // otherwise ping-pong groups of PF k-steps
    {
      const bf16* wr0 = a.w1 + (long long)(32 * wid + (lane & 15)) * a.ldw1 + kc0 + 8 * (lane >> 4);
      const bf16* wr1 = wr0 + 16LL * a.ldw1;
      const bf16* ar0 = s.ps + (lane & 15) * s.ldp + 8 * (lane >> 4);
      const bf16* ar1 = ar0 + 16 * s.ldp;
      f32x4 acc[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto step = [&](int k, const bf16x8& w0, const bf16x8& w1) {
        const bf16x8 x0 = ld16(ar0 + 32 * k), x1 = ld16(ar1 + 32 * k);
        acc[0] = mfma16x16x32(x0, w0, acc[0]);  // f = 2m + t
        acc[1] = mfma16x16x32(x0, w1, acc[1]);
        acc[2] = mfma16x16x32(x1, w0, acc[2]);
        acc[3] = mfma16x16x32(x1, w1, acc[3]);
      };
      if constexpr (KSC > 0) {
        bf16x8 wb0[KSC], wb1[KSC];
#pragma unroll
        for (int u = 0; u < KSC; ++u) {
          wb0[u] = ld16(wr0 + 32 * u);
          wb1[u] = ld16(wr1 + 32 * u);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep every load ahead of the MFMAs (the scheduler sinks them)
#pragma unroll
        for (int u = 0; u < KSC; ++u) step(u, wb0[u], wb1[u]);
      } else {
        constexpr int PF = 6;
        bf16x8 p0[PF], p1[PF], q0[PF], q1[PF];
        auto load = [&](bf16x8* d0, bf16x8* d1, int k0) {
#pragma unroll
          for (int u = 0; u < PF; ++u)
            if (k0 + u < KS) {
              d0[u] = ld16(wr0 + 32 * (k0 + u));
              d1[u] = ld16(wr1 + 32 * (k0 + u));
            }
        };
        auto run = [&](const bf16x8* d0, const bf16x8* d1, int k0) {
#pragma unroll
          for (int u = 0; u < PF; ++u)
            if (k0 + u < KS) step(k0 + u, d0[u], d1[u]);
        };
        load(p0, p1, 0);
#pragma unroll 1
        for (int s0 = 0; s0 < KS; s0 += 2 * PF) {
          load(q0, q1, s0 + PF);
          run(p0, p1, s0);
          load(p0, p1, s0 + 2 * PF);
          run(q0, q1, s0 + PF);
        }
      }
      const __amdgpu_buffer_rsrc_t ws = rsrc(a.slab + ((long long)rt * KCH + c) * SLAB, SLAB * 4);
#pragma unroll
      for (int f = 0; f < 4; ++f)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[f]), ws, ((wid * 4 + f) * 64 + lane) * 16,
                                               0, 16);
    }
    KH_STAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's slab stores are written through
    __syncthreads();
    if (tid == 0) {
      const unsigned prev = __hip_atomic_fetch_add(tickets + rt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev == (unsigned)(KCH - 1);
      if (s_last) __hip_atomic_store(tickets + rt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    const unsigned tag = s_tag;
    KH_STAMP(4);
    // the dP phase's W1^T operands (KSC > 0: the first two rolling groups) do not depend on dZ1: the waiters
    // issue them before they wait for the owner's flag, the owner right after publishing
    const int ntl = KC / 16, cnt = (ntl - wid + 3) / 4;
    const bf16* wt = a.w1t + (long long)(kc0 + 16 * wid + (lane & 15)) * N1 + 8 * (lane >> 4);
    constexpr int NTW = (2 * KSC + 3) / 4;  // tiles of the busiest wave (KSC > 0)
    constexpr int TG = 3, NG = KSC > 0 ? (NTW + TG - 1) / TG : 1;
    bf16x8 bb[NG][TG][4];
    auto load_g = [&](int g) {
#pragma unroll
      for (int t = 0; t < TG; ++t)
        if (g * TG + t < NTW && g * TG + t < cnt)
#pragma unroll
          for (int k = 0; k < 4; ++k) bb[g][t][k] = ld16(wt + (long long)(64 * (g * TG + t)) * N1 + 32 * k);
    };
    auto load_first = [&]() {
      if constexpr (KSC > 0) {
        if (a.dp) {
          load_g(0);
          if (NG > 1) load_g(1);
        }
      }
    };
    if (s_last) {
      f32x4 z[4];
      khead_combine(a, rt, z);
      khead_owner(a, s, rt, z);
      KH_STAMP(5);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(flags + rt, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      load_first();
      if (!a.dp) write_pT();  // (with dP: after its dZ1 loads are issued, below)
    } else {
      load_first();
      write_pT();
      if (tid == 0) {
        // bounded: the owner runs concurrently by construction (persistent grid <= resident capacity), but a
        // wait that never ends -- e.g. ranks time-sharing a GPU whose other kernels hold the CUs -- must not
        // hang the device: past 2 s the tile is left (its results invalid) and the sticky error word, the
        // workspace's word after the tag and the done counter, is set (ops.khead_error reads it)
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(flags + rt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tag) {
          if (wall_clock64() - t0 > kKHeadWaitTicks) {
            atomicOr(tagp + 2, 1u);  // (tagp + 1 is the done counter of the launch-tag hand-off)
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    KH_STAMP(6);
    if (a.stamps && first && tid == 0) {
      a.stamps[blockIdx.x * 16 + 15] = s_last;
      a.stamps[blockIdx.x * 16 + 14] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // XCC_ID
    }
    if (!a.dp) continue;
    // ---- dP chunk = dZ1 W1_chunk: A = the published dZ1 tile (sc1 loads), B = W1^T rows of the chunk
    {
      const __amdgpu_buffer_rsrc_t rs = rsrc(a.dz1 + (long long)rt * KR * N1, KR * N1 * 2);
      bf16x8 za[2][4];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          za[m][k] = __builtin_bit_cast(
              bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, ((16 * m + (lane & 15)) * N1 + 32 * k + 8 * (lane >> 4)) * 2, 0, 16));
      if (s_last) {  // the owner's P^T, its reads of the P tile done before any wave overwrites it with dP
        write_pT();
        __syncthreads();
      }
      if (a.stamps && first) {  // diagnostic split of the phase: dZ1 arrival, then the W1^T operands
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        KH_STAMP(9);
      }
      // column tiles of the chunk: wave w takes w, w + 4, ...; KSC > 0: the wave's W1^T operands in
      // rolling groups (the first two issued before the flag wait, above); otherwise two tiles per group
      // with ping-pong buffers
      // the tile transposed (W1^T as the A operand, dZ1 as B): a lane holds 4 consecutive columns of one
      // row, so the mask read and the in-place dP write are one 8-byte LDS access each per 16-row half
      // (were 8 + 8 two-byte accesses per tile)
      auto tile = [&](int i, const bf16x8* bb) {
        f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d0 = mfma16x16x32(bb[k], za[0][k], d0);
          d1 = mfma16x16x32(bb[k], za[1][k], d1);
        }
        bf16* p0 = s.ps + (lane & 15) * s.ldp + 16 * (wid + 4 * i) + 4 * (lane >> 4);  // row lane & 15
        bf16* p1 = p0 + 16 * s.ldp;                                                      // and 16 more
        const bf16x4 m0 = *reinterpret_cast<const bf16x4*>(p0), m1 = *reinterpret_cast<const bf16x4*>(p1);
        bf16x4 o0, o1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v0 = d0[r] * a.dp_scale, v1 = d1[r] * a.dp_scale;
          if (a.dp_mask) {
            if (!((float)m0[r] > 0.f)) v0 = 0.f;
            if (!((float)m1[r] > 0.f)) v1 = 0.f;
          }
          o0[r] = f2bf(v0);
          o1[r] = f2bf(v1);
        }
        *reinterpret_cast<bf16x4*>(p0) = o0;
        *reinterpret_cast<bf16x4*>(p1) = o1;
      };
      if constexpr (KSC > 0) {
        // rolling groups of 3 tiles, two groups in flight: ~96 operand VGPRs live instead of 144 (all nine
        // tiles' operands at once spill)
        __builtin_amdgcn_sched_barrier(0);
        if (a.stamps && first) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          KH_STAMP(10);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) {
#pragma unroll
          for (int t = 0; t < TG; ++t)
            if (g * TG + t < NTW && g * TG + t < cnt) tile(g * TG + t, bb[g][t]);
          if (g + 2 < NG) {
            __builtin_amdgcn_sched_barrier(0);
            load_g(g + 2);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      } else {
        bf16x8 pb[4], qb[4];
        auto load = [&](bf16x8* d, int i) {
          if (i < cnt)
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = ld16(wt + (long long)(64 * i) * N1 + 32 * k);
        };
        load(pb, 0);
#pragma unroll 1
        for (int i = 0; i < cnt; i += 2) {
          load(qb, i + 1);
          tile(i, pb);
          load(pb, i + 2);
          if (i + 1 < cnt) tile(i + 1, qb);
        }
      }
    }
    __syncthreads();
    KH_STAMP(7);
    for (int e = tid; e < KR * c8n; e += KT) {
      const int r = e / c8n, c8 = 8 * (e - r * c8n);
      if (r0 + r < a.B)
        *reinterpret_cast<bf16x8*>(a.dp + (long long)(r0 + r) * a.K + kc0 + c8) = ld16(s.ps + r * s.ldp + c8);
    }
  }
  // the last workgroup to finish advances the launch tag (every workgroup read it at its start)
  __syncthreads();
  {
    const bool first = true;
    KH_STAMP(8);
  }
  if (tid == 0) {
    unsigned* done = tagp + 1;
    const unsigned prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned)(a.G - 1)) {
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(tagp, s_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// dW[n][k] = sum_b dZ^T[n][b] X^T[k][b] (k < K), db[n] = the k == K column (X^T row of ones).  One
// workgroup per 64 x 32 output tile over the WHOLE batch (deterministic, no slabs): the 4 waves split
// the batch, each keeps 8 tiles' accumulators and issues its 8 batch steps' operand loads at once, then a
// fixed-order LDS combine.  Tiles sharing a 32-row X^T panel are adjacent on one XCD (xcd_remap).  Capped at
// 256 VGPRs (2 workgroups per CU): the reference CNN's 295 tiles then run in one round, not two (16.7 ->
// 14.6 us, profiles/r6/kernel_table_kc_after.txt).
constexpr int WGN = 64, WGK = 32, WGS = 8;
__global__ void __launch_bounds__(KT, 2) khead_wgrad_kernel(KHeadWgradArgs a) {
  __shared__ f32x4 red[4][8][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, tid = threadIdx.x;
  if ((int)blockIdx.x == a.jobs) {  // loss partials -> stats (fixed-order tree)
    if (wid == 0) {
      float l = 0.f, c = 0.f;
      for (int i = lane; i < a.nloss; i += 64) {
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
  int job = xcd_remap(blockIdx.x, a.jobs);
  const int j0 = a.L[0].nblk * a.L[0].kblk;
  const bool second = job >= j0;
  if (second) job -= j0;
  const KHeadWgradLayer L = second ? a.L[1] : a.L[0];
  const int kb = job / L.nblk, nb = job - kb * L.nblk;  // n blocks of one X^T panel adjacent
  const int n0 = nb * WGN, k0 = kb * WGK;
  const int steps = a.ldt / 32, per = (steps + 3) / 4;
  const int s0 = wid * per, s1 = min(steps, s0 + per);
  const bf16* ar[4];
  const bf16* br[2];
  bool aon[4];
  int bkind[2];  // 0 data, 1 ones, 2 zero
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + 16 * i + (lane & 15);
    aon[i] = n0 + 16 * i < L.N;  // wave-uniform: the tile has a valid row
    ar[i] = L.a + (long long)min(n, L.N - 1) * a.ldt + 8 * (lane >> 4);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = k0 + 16 * j + (lane & 15);
    bkind[j] = k < L.K ? 0 : (k == L.K ? 1 : 2);
    br[j] = L.b + (long long)min(k, L.K - 1) * a.ldt + 8 * (lane >> 4);
  }
  bf16x8 ones, zeros;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ones[e] = (bf16)1.f;
    zeros[e] = (bf16)0.f;
  }
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < s1; s += WGS) {
    bf16x8 av[WGS][4], bv[WGS][2];
#pragma unroll
    for (int u = 0; u < WGS; ++u) {
      const int ss = 32 * min(s + u, s1 - 1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (aon[i]) av[u][i] = ld16(ar[i] + ss);
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[u][j] = ld16(br[j] + ss);
    }
#pragma unroll
    for (int u = 0; u < WGS; ++u) {
      if (s + u >= s1) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 b = bkind[j] == 0 ? bv[u][j] : (bkind[j] == 1 ? ones : zeros);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (aon[i]) acc[i][j] = mfma16x16x32(av[u][i], b, acc[i][j]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) red[wid][2 * i + j][lane] = acc[i][j];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int q = tid + KT * h, f = q >> 6, ln = q & 63;
    const f32x4 v = red[0][f][ln] + red[1][f][ln] + red[2][f][ln] + red[3][f][ln];
    const int i = f >> 1, j = f & 1;
    const int k = k0 + 16 * j + (ln & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 16 * i + 4 * (ln >> 4) + r;
      if (n >= L.N) continue;
      if (k < L.K) L.gw[(long long)n * L.K + k] = v[r];
      else if (k == L.K && L.gb) L.gb[n] = v[r];
    }
  }
}

hipError_t khead_wgrad(KHeadWgradArgs a, hipStream_t st) {
  if (a.ldt <= 0 || a.ldt % 32) return hipErrorInvalidValue;
  a.jobs = 0;
  for (int l = 0; l < 2; ++l) {
    KHeadWgradLayer& L = a.L[l];
    if (L.N <= 0 || L.K <= 0) return hipErrorInvalidValue;
    L.nblk = cdiv(L.N, WGN);
    L.kblk = cdiv(L.K + 1, WGK);
    a.jobs += L.nblk * L.kblk;
  }
  hipLaunchKernelGGL(khead_wgrad_kernel, dim3(a.jobs + 1), dim3(KT), 0, st, a);
  return hipGetLastError();
}

size_t khead_ws_floats(int B, int K) {
  (void)K;
  const size_t nt = (size_t)cdiv(B, KR);
  return nt * KCH * SLAB + nt * KR * N1 / 2 + 2 * nt + 3;  // ... tickets, flags, tag, done counter, error word
}

size_t khead_lds(int K) {
  const int KC = K / KCH;
  return round_up(KR * (KC + 8) * 2, 16) + 2 * KR * LDH * 2 + KR * LDZ2 * 2 + KR * 16 * 4;
}

bool khead_supported(int K, int C) {
  return K > 0 && K % (KCH * 32) == 0 && KR * (K / KCH) / 8 <= KT * kStageMax && C >= 1 && C <= 16 &&
         khead_lds(K) <= 64 * 1024;
}

static int khead_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

hipError_t khead_train(KHeadArgs a, hipStream_t st) {
  if (!khead_supported(a.K, a.C) || a.B <= 0 || a.ldt < round_up(a.B, KR) || a.ldw1 < a.K) return hipErrorInvalidValue;
  a.ntiles = cdiv(a.B, KR);
  if (a.ldt < a.ntiles * KR) return hipErrorInvalidValue;
  // persistent grid: every workgroup resident (one per CU at most), a multiple of 8 so the 8 jobs of a row
  // tile are always in flight together
  const int cap = (g_khead_cap > 0 ? std::min(khead_cus(), g_khead_cap) : khead_cus()) / KCH * KCH;
  a.G = min(a.ntiles * KCH, cap);
  if (a.G < KCH) return hipErrorInvalidValue;
  a.stamps = g_khead_stamps;
  const size_t lds = khead_lds(a.K);
  // the reference CNN's K = 4608 (18 k-steps per chunk) fully unrolled; any other K the generic loops
  if (a.K == 18 * 32 * KCH) hipLaunchKernelGGL(khead_train_kernel<18>, dim3(a.G), dim3(KT), lds, st, a);
  else hipLaunchKernelGGL(khead_train_kernel<0>, dim3(a.G), dim3(KT), lds, st, a);
  return hipGetLastError();
}

}  // namespace dfa
