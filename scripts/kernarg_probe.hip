// Latency of a dynamically indexed read from a large by-value kernel argument vs the same table in
// device memory, for direct launches and hipGraph replays (scripts/gpu_r3f.sh).  Clock: s_memtime.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Big {
  int tab[1024];
  unsigned long long* out;
  const int* dtab;
  int mode;
};

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__global__ void probe(Big a) {
  __shared__ int sink;
  const unsigned long long t0 = clk();
  int i = (blockIdx.x * 37) & 1023;
  // three dependent reads
  for (int k = 0; k < 3; ++k) i = (a.mode == 0 ? a.tab[i] : a.dtab[i]) & 1023;
  if (threadIdx.x == 0) sink = i;
  __syncthreads();
  const unsigned long long t1 = clk();
  if (threadIdx.x == 0) {
    a.out[2 * blockIdx.x] = t1 - t0;
    a.out[2 * blockIdx.x + 1] = sink;
  }
}

int main() {
  const int G = 256;
  Big a{};
  for (int i = 0; i < 1024; ++i) a.tab[i] = (i * 613 + 5) & 1023;
  int* dtab;
  unsigned long long* out;
  (void)hipMalloc(&dtab, 4096);
  (void)hipMalloc(&out, G * 16);
  (void)hipMemcpy(dtab, a.tab, 4096, hipMemcpyHostToDevice);
  a.out = out;
  a.dtab = dtab;
  hipStream_t st;
  (void)hipStreamCreate(&st);
  std::vector<unsigned long long> h(2 * G);
  for (int graph = 0; graph < 2; ++graph)
    for (int mode = 0; mode < 2; ++mode) {
      a.mode = mode;
      hipGraphExec_t ge = nullptr;
      if (graph) {
        hipGraph_t g;
        (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
        hipLaunchKernelGGL(probe, dim3(G), dim3(64), 0, st, a);
        (void)hipStreamEndCapture(st, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      }
      for (int rep = 0; rep < 5; ++rep) {
        if (graph) (void)hipGraphLaunch(ge, st);
        else hipLaunchKernelGGL(probe, dim3(G), dim3(64), 0, st, a);
      }
      (void)hipStreamSynchronize(st);
      (void)hipMemcpy(h.data(), out, G * 16, hipMemcpyDeviceToHost);
      std::vector<unsigned long long> d;
      for (int b = 0; b < G; ++b) d.push_back(h[2 * b]);
      std::sort(d.begin(), d.end());
      printf("%s %-10s 3 dependent reads: median %llu cycles, max %llu\n", graph ? "graph " : "direct",
             mode == 0 ? "kernarg" : "device", d[G / 2], d[G - 1]);
    }
  return 0;
}
