// One-shot peer-to-peer all-reduce over xGMI for small gradient buckets ("M3/M5 get a
// C++ xGMI all-reduce for small buffers").
//
// The reference averages gradients on the parameter server host after stacking K uploads
// (/root/reference/src/server/federated_server.ts:92-117, /root/reference/src/common/utils.ts:53-75).
// On one MI355X node every rank holds the whole flat gradient and the reduce is latency bound for the
// buffers this framework ships (LeNet-5: 247 KB fp32, Keras CNN: 2.4 MB): a ring needs 2(W-1) dependent
// hops, while the node's xGMI is fully connected (7 links per GPU).  One-shot: every rank publishes its
// slice in an IPC-exported staging buffer, raises a flag in each peer's flag array, and once all W
// flags of that slice are up reads the W copies over all 7 links at once and sums them in rank order
// (so every rank gets bit-identical sums and the replicas never drift).
//
// Protocol (per workgroup b, which always owns elements [b*kChunk, (b+1)*kChunk) of every call):
//   * epoch e = ++epochs[b] (a per-block counter in local memory: identical on all ranks because every
//     rank issues the same sequence of calls, and hipGraph replays keep it advancing on device);
//   * staging half (e & 1) — double buffering makes one flag round per call sufficient: a rank can only
//     start epoch e+2 of block b after every peer raised flag e+1 of block b, which a peer does only after
//     its call with epoch e (and thus its reads of half e&1) completed in stream order;
//   * flags are monotonic (>= e), written with system-scope release stores, polled with system-scope
//     acquire loads, bounded by a wall-clock timeout: a missing peer sets *err and the block exits instead
//     of spinning forever (the host falls back to RCCL when the startup self-test sees an error).
//
// Buffers come from hipExtMallocWithFlags(hipDeviceMallocUncached): flag polls and peer reads never see a
// stale cache line, and writes from a remote GPU land directly in HBM.
#include "common.h"
#include "kernels.h"
#include "ll_exchange.h"

namespace dfa {
namespace {

constexpr int kThreads = kP2PChunk / 8;  // 2 float4 per thread

template <int W>
__global__ __launch_bounds__(kThreads) void p2p_allreduce_kernel(P2PArgs a) {
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  __shared__ unsigned s_e;
  __shared__ int s_bad;
  if (t == 0) {
    s_e = a.epochs[b] + 1u;
    s_bad = 0;
  }
  __syncthreads();
  const unsigned e = s_e;
  const long long base = (long long)b * kP2PChunk;
  const long long stage_off = (long long)(e & 1u) * a.half_floats + base;

  // 1. publish this rank's slice in its own staging half
  f32x4 mine[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long long idx = base + (long long)(i * kThreads + t) * 4;
    if (idx + 3 < a.n) {
      mine[i] = *reinterpret_cast<const f32x4*>(a.data + idx);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) mine[i][j] = (idx + j < a.n) ? a.data[idx + j] : 0.f;
    }
    float* st = reinterpret_cast<float*>(a.bases[a.rank] + a.flag_bytes) + stage_off + (i * kThreads + t) * 4;
    *reinterpret_cast<f32x4*>(st) = mine[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: staging writes visible before the flags
  __syncthreads();

  // 2. raise flag [b][rank] in every peer (lane r writes to rank r), then wait for [b][0..W) locally
  if (t < W) {
    unsigned* f = reinterpret_cast<unsigned*>(a.bases[t]) + (long long)b * kP2PMaxRanks + a.rank;
    __hip_atomic_store(f, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* mf = reinterpret_cast<const unsigned*>(a.bases[a.rank]) + (long long)b * kP2PMaxRanks + t;
    const unsigned long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(mf, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (wall_clock64() - t0 > (unsigned long long)a.timeout_ticks) {
        atomicOr(a.err, 1);
        if (a.herr) __hip_atomic_store(a.herr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_bad = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (s_bad) return;  // epoch not committed: the call is reported failed, never half-applied silently
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");

  // 3. sum the W published copies in rank order (all loads in flight before the adds)
  f32x4 v[W][2];
#pragma unroll
  for (int r = 0; r < W; ++r) {
    const float* src = reinterpret_cast<const float*>(a.bases[r] + a.flag_bytes) + stage_off;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (r == a.rank) {
        v[r][i] = mine[i];
      } else {
        v[r][i] = *reinterpret_cast<const f32x4*>(src + (i * kThreads + t) * 4);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 acc = v[0][i];
#pragma unroll
    for (int r = 1; r < W; ++r) acc += v[r][i];
    acc *= a.scale;
    const long long idx = base + (long long)(i * kThreads + t) * 4;
    if (idx + 3 < a.n) {
      *reinterpret_cast<f32x4*>(a.data + idx) = acc;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (idx + j < a.n) a.data[idx + j] = acc[j];
    }
  }
  if (t == 0) a.epochs[b] = e;
}

// Startup self-test of the in-kernel LL exchange (csrc/ll_exchange.h) that the fused LeNet-5 reduce
// launch folds into its epilogue: one slot per workgroup, one granule per thread, the same push /
// poll / rank-order sum.  Every rank runs the same calls on the same slots, so the per-slot epochs stay
// in step for the kernels that use the slots afterwards.
__global__ void __launch_bounds__(kLLSlot) ll_selftest_kernel(LLComm c, const float* in, float* out) {
  __shared__ unsigned s_e;
  const int slot = blockIdx.x;
  const unsigned e = ll_epoch(c, slot, &s_e);
  const long long i = (long long)slot * kLLSlot + threadIdx.x;
  float o = 0.f;
  ll_allreduce(c, slot, threadIdx.x, e, in[i], o);
  out[i] = o;
  __syncthreads();
  ll_commit(c, slot, e);
}

}  // namespace

hipError_t ll_selftest(const LLComm& c, const float* in, float* out, int nslots, hipStream_t st) {
  if (nslots <= 0 || nslots > c.nslots) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ll_selftest_kernel, dim3(nslots), dim3(kLLSlot), 0, st, c, in, out);
  return hipGetLastError();
}

hipError_t p2p_allreduce(const P2PArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  const long long nb = (a.n + kP2PChunk - 1) / kP2PChunk;
  if (nb > a.max_blocks || a.world < 1 || a.world > kP2PMaxRanks) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nb), block(kThreads);
  switch (a.world) {
    case 1: p2p_allreduce_kernel<1><<<grid, block, 0, st>>>(a); break;
    case 2: p2p_allreduce_kernel<2><<<grid, block, 0, st>>>(a); break;
    case 3: p2p_allreduce_kernel<3><<<grid, block, 0, st>>>(a); break;
    case 4: p2p_allreduce_kernel<4><<<grid, block, 0, st>>>(a); break;
    case 5: p2p_allreduce_kernel<5><<<grid, block, 0, st>>>(a); break;
    case 6: p2p_allreduce_kernel<6><<<grid, block, 0, st>>>(a); break;
    case 7: p2p_allreduce_kernel<7><<<grid, block, 0, st>>>(a); break;
    default: p2p_allreduce_kernel<8><<<grid, block, 0, st>>>(a); break;
  }
  return hipGetLastError();
}

}  // namespace dfa
