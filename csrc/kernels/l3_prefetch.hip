// Infinity Cache warm-up for weight-streaming decode GEMMs.
//
// A tensor-parallel decode layer alternates HBM-bound GEMMs with phases that
// leave HBM idle: the decode attention and the residual all-reduces are
// latency chains of a few dozen workgroups (Llama-3-70B TP=8 rank: ~27 us of
// every ~84 us layer). This kernel runs on a side stream during those phases
// and reads the weights the NEXT GEMMs will stream, so they are served from
// the 256 MiB die-level cache (8.6 vs 6.0 TB/s chip-wide, 227 ns vs ~1 us
// latency: MI355X_MICROARCH.md "Infinity Cache", "Indexed rows") instead of
// HBM. It is a pure read: the consumers do not wait for it, so a late or
// missing prefetch costs bandwidth, never correctness.
//
// Regions are read in list order (the consumers' order), 16 B per lane with
// 8 loads in flight per lane; the XOR of everything read is stored only when
// it equals a caller-chosen word, which keeps the loads alive without a
// store per lane.
#include "common.h"

#define L3PF_MAX_REGIONS 8

struct L3PrefetchList {
  const uint4* base[L3PF_MAX_REGIONS];
  long long n16[L3PF_MAX_REGIONS];   // 16-byte vectors per region
  int count;
  unsigned magic;
  unsigned* sink;
};

__global__ __launch_bounds__(256) void l3_prefetch_kernel(L3PrefetchList L) {
  unsigned acc = 0;
  const long long stride = (long long)gridDim.x * 256 * 8;
  for (int r = 0; r < L.count; ++r) {
    const uint4* __restrict__ p = L.base[r];
    const long long n = L.n16[r];
    // consecutive workgroups take consecutive 32 KiB chunks: the region is
    // swept front to back, the order its consumer GEMM reaches it
    for (long long v0 = (long long)blockIdx.x * 256 * 8 + threadIdx.x; v0 < n; v0 += stride) {
      uint4 x[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const long long v = v0 + (long long)i * 256;
        x[i] = v < n ? p[v] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= x[i].x ^ x[i].w;
    }
  }
  if (acc == L.magic) L.sink[0] = acc;
}

// ptrs / bytes: `count` (<= 8) device regions, each a multiple of 16 bytes
extern "C" int loqa_l3_prefetch(const void* const* ptrs, const long long* bytes, int count, int wgs,
                                unsigned* sink, hipStream_t s) {
  if (count < 1 || count > L3PF_MAX_REGIONS || wgs < 1 || wgs > 4096 || !sink)
    return (int)hipErrorInvalidValue;
  L3PrefetchList L{};
  for (int r = 0; r < count; ++r) {
    if (!ptrs[r] || bytes[r] < 0 || bytes[r] % 16) return (int)hipErrorInvalidValue;
    L.base[r] = static_cast<const uint4*>(ptrs[r]);
    L.n16[r] = bytes[r] / 16;
  }
  L.count = count;
  L.magic = 0x7f4a7c15u;
  L.sink = sink;
  hipLaunchKernelGGL(l3_prefetch_kernel, dim3(wgs), dim3(256), 0, s, L);
  return (int)hipGetLastError();
}
