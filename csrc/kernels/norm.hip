// Fused normalisation kernels (SURVEY §2.4 K4 layernorm, K10 rmsnorm).
//
// One 256-thread workgroup per row; the row stays in registers between the
// statistics pass and the scale pass, so HBM traffic is exactly
//   read x (+ read residual, write residual) + write y.
// Rows are loaded as 16-byte vectors (8 bf16 per lane, guide G13). Supports
// d % 8 == 0 and d <= 256 * 8 * MAXV.
#include "common.h"

#define NORM_THREADS 256
#define MAXV 4

// y = rmsnorm(x [+ residual]) * w.  If residual != nullptr, residual <- x + residual.
__global__ __launch_bounds__(NORM_THREADS) void rmsnorm_kernel(
    const bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int d, float eps) {
  __shared__ float scratch[NORM_THREADS / 64];
  const int row = blockIdx.x;
  const int nvec = d >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * d);
  uint4* rr = residual ? reinterpret_cast<uint4*>(residual + (size_t)row * d) : nullptr;
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    if (c < nvec) {
      unpack8(xr[c], v[i]);
      if (rr) {
        float r[8];
        unpack8(rr[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
        // The residual stream is stored in bf16 (as the model's dtype); the norm
        // is computed from the same rounded values a bf16 reference would see.
        uint4 p = pack8(v[i]);
        rr[c] = p;
        unpack8(p, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / (float)d + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * d);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    if (c < nvec) {
      float wf[8], o[8];
      unpack8(wr[c], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * wf[j];
      yr[c] = pack8(o);
    }
  }
}

// y = layernorm(x [+ residual]) * w + b  (Whisper pre-LN blocks).
__global__ __launch_bounds__(NORM_THREADS) void layernorm_kernel(
    const bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
    bf16_t* __restrict__ y, int d, float eps) {
  __shared__ float scratch[NORM_THREADS / 64];
  const int row = blockIdx.x;
  const int nvec = d >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * d);
  uint4* rr = residual ? reinterpret_cast<uint4*>(residual + (size_t)row * d) : nullptr;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    if (c < nvec) {
      unpack8(xr[c], v[i]);
      if (rr) {
        float r[8];
        unpack8(rr[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
        uint4 p = pack8(v[i]);
        rr[c] = p;
        unpack8(p, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = block_sum(s, scratch) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = v[i][j] - mean;
        q += t * t;
      }
    }
  }
  const float inv = rsqrtf(block_sum(q, scratch) / (float)d + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  const uint4* br = reinterpret_cast<const uint4*>(b);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * d);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    if (c < nvec) {
      float wf[8], bf[8], o[8];
      unpack8(wr[c], wf);
      unpack8(br[c], bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * inv * wf[j] + bf[j];
      yr[c] = pack8(o);
    }
  }
}

extern "C" int loqa_rmsnorm(const void* x, void* residual, const void* w, void* y,
                            int rows, int d, float eps, hipStream_t s) {
  if (d % 8 != 0 || d > NORM_THREADS * 8 * MAXV || rows <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsnorm_kernel, dim3(rows), dim3(NORM_THREADS), 0, s,
                     (const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w, (bf16_t*)y, d, eps);
  return (int)hipGetLastError();
}

extern "C" int loqa_layernorm(const void* x, void* residual, const void* w, const void* b,
                              void* y, int rows, int d, float eps, hipStream_t s) {
  if (d % 8 != 0 || d > NORM_THREADS * 8 * MAXV || rows <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(layernorm_kernel, dim3(rows), dim3(NORM_THREADS), 0, s,
                     (const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w, (const bf16_t*)b,
                     (bf16_t*)y, d, eps);
  return (int)hipGetLastError();
}

// Decoder input embedding: out[r] = bf16(tok_embed[tokens[r]] + pos_embed[positions[r]])
// (Whisper decoder; feeds layernorm as the first residual).
__global__ void embed_pos_kernel(const int* __restrict__ tokens, const int* __restrict__ positions,
                                 const bf16_t* __restrict__ te, const bf16_t* __restrict__ pe,
                                 bf16_t* __restrict__ out, int d) {
  const int row = blockIdx.x;
  const uint4* a = reinterpret_cast<const uint4*>(te + (size_t)tokens[row] * d);
  const uint4* b = reinterpret_cast<const uint4*>(pe + (size_t)positions[row] * d);
  uint4* o = reinterpret_cast<uint4*>(out + (size_t)row * d);
  for (int c = threadIdx.x; c < (d >> 3); c += blockDim.x) {
    float x[8], y[8];
    unpack8(a[c], x);
    unpack8(b[c], y);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += y[j];
    o[c] = pack8(x);
  }
}

extern "C" int loqa_embed_pos(const int* tokens, const int* positions, const void* tok_embed,
                              const void* pos_embed, void* out, int rows, int d, hipStream_t s) {
  if (rows <= 0) return 0;
  if (d % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_pos_kernel, dim3(rows), dim3(128), 0, s, tokens, positions,
                     (const bf16_t*)tok_embed, (const bf16_t*)pos_embed, (bf16_t*)out, d);
  return (int)hipGetLastError();
}
