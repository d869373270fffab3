// Shared device helpers for the loqa-hub MI355X (gfx950, CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//   * bf16 tensors are passed as raw uint16 storage (`bf16_t`), converted with
//     bit shifts on load and round-to-nearest-even (v_cvt_pk_bf16_f32) on store.
//   * Memory-bound kernels move data in 16-byte vectors (8 x bf16 per lane):
//     hipcc does not vectorise scalar bf16 loads (guide G13).
//   * Wave size is 64, hard-coded; block sizes are multiples of 64.
//   * Every launcher is `extern "C"`, takes the HIP stream explicitly and returns
//     the hipError_t of the launch so the Python side can fail loudly.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define WAVE 64

__device__ __forceinline__ float bf2f(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&b);
}

// Pack two floats into one dword of two bf16 (lo in the low half).
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack_bf16x2(f[0], f[1]);
  v.y = pack_bf16x2(f[2], f[3]);
  v.z = pack_bf16x2(f[4], f[5]);
  v.w = pack_bf16x2(f[6], f[7]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` needs blockDim.x/64 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

// XCD-aware bijective remap of a linear workgroup id (guide §5 "XCD swizzle must
// be bijective"): consecutive logical tiles land on the same XCD / L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg <= nxcd) return orig;
  const int q = nwg / nxcd, r = nwg % nxcd;
  const int xcd = orig % nxcd;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nxcd;
}
