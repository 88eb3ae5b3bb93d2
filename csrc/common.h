// Shared device helpers for the distriflow_amd gfx950 (MI355X / CDNA4) kernels.
//
// Conventions used by every kernel in csrc/:
//   * activations are bf16, NHWC, row-major ([rows][channels], channel contiguous)
//   * accumulation is fp32; MFMA tiles are v_mfma_f32_16x16x32_bf16 (wave64)
//   * compute weights are bf16 copies written by the fused SGD kernel, zero padded to
//     [roundup(N,16)][roundup(K,32)] so weight tiles never need bounds checks
//   * every launcher takes an explicit hipStream_t (the caller passes PyTorch's current
//     stream so that the whole training step can be captured into one hipGraph)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfa {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }  // v_cvt_pk_bf16_f32 (RNE, NaN-safe)

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ __forceinline__ int round_up(int a, int b) { return cdiv(a, b) * b; }

// Division of small non-negative ints (a < 2^20, d >= 1) for index tables: 3 VALU instead of the
// ~25-instruction integer division sequence.  (a + 0.5) / d stays >= 0.5/d away from any integer,
// which exceeds the combined v_rcp_f32 + rounding error in that range, so truncation is exact.
struct FDiv {
  int d;
  float inv;
  __device__ __forceinline__ explicit FDiv(int dd) : d(dd), inv(__builtin_amdgcn_rcpf((float)dd)) {}
  __device__ __forceinline__ int div(int a) const { return (int)(((float)a + 0.5f) * inv); }
  __device__ __forceinline__ int mod(int a, int q) const { return a - q * d; }
};

// Unsigned division by a launch constant: q = n / d for 0 <= n < 2^31 as (mulhi(n, mul) + n) >> shr,
// with the magic number computed on the host (pixel decomposition of implicit-GEMM rows).
struct FastDiv {
  unsigned mul, shr;
};

inline FastDiv make_fastdiv(unsigned d) {
  unsigned l = 0;
  while ((1u << l) < d) ++l;
  FastDiv f;
  f.mul = (unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  f.shr = l;
  return f;
}

__device__ __forceinline__ unsigned fdiv(unsigned n, FastDiv f) { return (__umulhi(n, f.mul) + n) >> f.shr; }

// Bijective XCD-aware remap of a 1-D block id: consecutive logical tiles land on the same XCD
// (blocks b and b+8 share an XCD under round-robin dispatch) so neighbouring tiles share L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nx = 8;
  if (nblocks < nx) return bid;
  const int q = nblocks / nx, r = nblocks % nx;
  const int xcd = bid % nx, slot = bid / nx;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + slot;
}

// Counter-based hash RNG (squares-style mixing) used by dropout: the mask is a pure function of
// (seed, index) so the backward pass regenerates it instead of storing it.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint64_t x = idx * 0x9E3779B97F4A7C15ull + seed;
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)x;
}

// Folded dropout (kernels.h DropSpec): the per-launch seed and the keep test of element i
__device__ __forceinline__ unsigned long long drop_seed(unsigned long long seed0, const long long* step, int add = 0) {
  return seed0 ^ (step ? (unsigned long long)(step[0] + add) * 0x9E3779B1ull : 0ull);
}
__device__ __forceinline__ bool drop_keep(unsigned long long seed, unsigned thresh, long long i) {
  return hash_u32(seed, (uint64_t)i) >= thresh;
}

}  // namespace dfa

#define DFA_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) return _e;                                               \
  } while (0)
