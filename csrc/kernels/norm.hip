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
// Output row i normalises x row row_idx[i] (or i): the final norm of a decode
// step gathers the logit rows itself instead of a separate index_select.
__global__ __launch_bounds__(NORM_THREADS) void rmsnorm_kernel(
    const bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int d, float eps,
    const int64_t* __restrict__ row_idx) {
  __shared__ float scratch[NORM_THREADS / 64];
  const int row = blockIdx.x;
  const int src = row_idx ? (int)row_idx[row] : row;
  const int nvec = d >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)src * d);
  uint4* rr = residual ? reinterpret_cast<uint4*>(residual + (size_t)row * d) : nullptr;
  // the norm weight does not depend on the statistics: requested with the row,
  // so the scale pass does not wait for a second memory round trip
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  uint4 wpre[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    wpre[i] = c < nvec ? wr[c] : make_uint4(0, 0, 0, 0);
  }
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
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * d);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    if (c < nvec) {
      float wf[8], o[8];
      unpack8(wpre[i], wf);
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
    bf16_t* __restrict__ y, int d, float eps, const int64_t* __restrict__ row_idx) {
  __shared__ float scratch[NORM_THREADS / 64];
  const int row = blockIdx.x;
  const int src = row_idx ? (int)row_idx[row] : row;
  const int nvec = d >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)src * d);
  uint4* rr = residual ? reinterpret_cast<uint4*>(residual + (size_t)row * d) : nullptr;
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  const uint4* br = reinterpret_cast<const uint4*>(b);
  uint4 wpre[MAXV], bpre[MAXV];     // requested with the row (see rmsnorm_kernel)
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    wpre[i] = c < nvec ? wr[c] : make_uint4(0, 0, 0, 0);
    bpre[i] = c < nvec ? br[c] : make_uint4(0, 0, 0, 0);
  }
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
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * d);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    if (c < nvec) {
      float wf[8], bf[8], o[8];
      unpack8(wpre[i], wf);
      unpack8(bpre[i], bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * inv * wf[j] + bf[j];
      yr[c] = pack8(o);
    }
  }
}

// row_idx (int64, may be null) selects the source rows; it is not combined with
// residual (the wrapper rejects that).
extern "C" int loqa_rmsnorm(const void* x, void* residual, const void* w, void* y,
                            int rows, int d, float eps, const int64_t* row_idx, hipStream_t s) {
  if (d % 8 != 0 || d > NORM_THREADS * 8 * MAXV || rows <= 0) return (int)hipErrorInvalidValue;
  if (row_idx && residual) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsnorm_kernel, dim3(rows), dim3(NORM_THREADS), 0, s,
                     (const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w, (bf16_t*)y, d, eps,
                     row_idx);
  return (int)hipGetLastError();
}

extern "C" int loqa_layernorm(const void* x, void* residual, const void* w, const void* b,
                              void* y, int rows, int d, float eps, const int64_t* row_idx,
                              hipStream_t s) {
  if (d % 8 != 0 || d > NORM_THREADS * 8 * MAXV || rows <= 0) return (int)hipErrorInvalidValue;
  if (row_idx && residual) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(layernorm_kernel, dim3(rows), dim3(NORM_THREADS), 0, s,
                     (const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w, (const bf16_t*)b,
                     (bf16_t*)y, d, eps, row_idx);
  return (int)hipGetLastError();
}

// Decoder input embedding: out[r] = bf16(tok_embed[tokens[r]] + pos_embed[positions[r]])
// (Whisper decoder; feeds layernorm as the first residual).
__global__ void embed_pos_kernel(const int* __restrict__ tokens, const int* __restrict__ positions,
                                 const bf16_t* __restrict__ te, const bf16_t* __restrict__ pe,
                                 bf16_t* __restrict__ out, int d) {
  const int row = blockIdx.x;
  const uint4* a = reinterpret_cast<const uint4*>(te + (size_t)max(tokens[row], 0) * d);
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

// Decode-step input of the fused-GEMM path: out[r] = tok_embed[tokens[r]]
// (+ pos_embed[positions[r]], rounded to bf16 once) AND the row statistics the
// first layer's norm prologue reads as one partial tile: rowsq[r] = sum out^2,
// rowsum[r] = sum out (optional). Replaces embedding + a float copy + two
// reductions (four to five launches) with one; the sums are taken over the
// stored bf16 values, as the residual epilogues do.
__global__ __launch_bounds__(NORM_THREADS) void embed_stats_kernel(
    const int* __restrict__ tokens, const int* __restrict__ positions,
    const bf16_t* __restrict__ te, const bf16_t* __restrict__ pe, bf16_t* __restrict__ out,
    float* __restrict__ rowsq, float* __restrict__ rowsum, int d) {
  __shared__ float scratch[NORM_THREADS / 64];
  const int row = blockIdx.x;
  const int nvec = d >> 3;
  const uint4* a = reinterpret_cast<const uint4*>(te + (size_t)max(tokens[row], 0) * d);
  const uint4* b = pe ? reinterpret_cast<const uint4*>(pe + (size_t)positions[row] * d) : nullptr;
  uint4* o = reinterpret_cast<uint4*>(out + (size_t)row * d);
  float ss = 0.f, s1 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NORM_THREADS;
    if (c < nvec) {
      uint4 p = a[c];
      float x[8];
      if (b) {
        float y[8];
        unpack8(p, x);
        unpack8(b[c], y);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] += y[j];
        p = pack8(x);
      }
      o[c] = p;
      unpack8(p, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ss += x[j] * x[j];
        s1 += x[j];
      }
    }
  }
  ss = block_sum(ss, scratch);
  if (threadIdx.x == 0) rowsq[row] = ss;
  if (rowsum) {
    s1 = block_sum(s1, scratch);
    if (threadIdx.x == 0) rowsum[row] = s1;
  }
}

extern "C" int loqa_embed_stats(const int* tokens, const int* positions, const void* tok_embed,
                                const void* pos_embed, void* out, float* rowsq, float* rowsum,
                                int rows, int d, hipStream_t s) {
  if (rows <= 0) return 0;
  if (d % 8 || d > NORM_THREADS * 8 * MAXV || !rowsq) return (int)hipErrorInvalidValue;
  if (pos_embed && !positions) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_stats_kernel, dim3(rows), dim3(NORM_THREADS), 0, s, tokens, positions,
                     (const bf16_t*)tok_embed, (const bf16_t*)pos_embed, (bf16_t*)out, rowsq,
                     rowsum, d);
  return (int)hipGetLastError();
}
