// Consumers of the skinny GEMM's split-K f32 slabs (part[S][Mpad][N]).
// Each kernel sums the S slabs of its input rows in a fixed order (bitwise
// deterministic) in its prologue and fuses the op that follows the GEMM:
//   slab_rmsnorm      : residual += sum; y = rmsnorm(residual) * w     (o / down proj)
//   slab_rope_append  : RoPE(q, k) + paged KV append, q -> bf16        (qkv proj)
//   slab_silu_mul     : silu(gate) * up -> bf16                         (gate|up proj)
//   slab_to_f32       : plain reduction (lm_head logits, S > 1 only)
#include "common.h"

#define NT 256
#define MAXV 4

__device__ __forceinline__ void slab_load8(const float* __restrict__ part, size_t slab_stride,
                                           int S, size_t off, float* v) {
  float4 a = *reinterpret_cast<const float4*>(part + off);
  float4 b = *reinterpret_cast<const float4*>(part + off + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  for (int s = 1; s < S; ++s) {
    a = *reinterpret_cast<const float4*>(part + s * slab_stride + off);
    b = *reinterpret_cast<const float4*>(part + s * slab_stride + off + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
    v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
}

// row i of the output reads slab row src = row_idx ? row_idx[i] : i
__global__ __launch_bounds__(NT) void slab_rmsnorm_kernel(
    const float* __restrict__ part, int S, int Mpad, const int64_t* __restrict__ row_idx,
    bf16_t* __restrict__ residual, int write_residual, const bf16_t* __restrict__ w,
    bf16_t* __restrict__ y, int d, float eps) {
  __shared__ float scratch[NT / 64];
  const int row = blockIdx.x;
  const int src = row_idx ? (int)row_idx[row] : row;
  const size_t slab_stride = (size_t)Mpad * d;
  const int nvec = d >> 3;
  uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)src * d);
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NT;
    if (c < nvec) {
      slab_load8(part, slab_stride, S, (size_t)src * d + c * 8, v[i]);
      float r[8];
      unpack8(rr[c], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] += r[j];
      uint4 p = pack8(v[i]);
      if (write_residual) rr[c] = p;
      unpack8(p, v[i]);
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
    const int c = threadIdx.x + i * NT;
    if (c < nvec) {
      float wf[8], o[8];
      unpack8(wr[c], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * wf[j];
      yr[c] = pack8(o);
    }
  }
}

// qkv slabs: [S][Mpad][(H + 2Hkv) * D]; q_out: [M, H*D] bf16; caches [nb, Hkv, blk, D]
__global__ void slab_rope_append_kernel(const float* __restrict__ part, int S, int Mpad,
                                        const int* __restrict__ positions,
                                        const float2* __restrict__ cs, bf16_t* __restrict__ q_out,
                                        bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
                                        const int* __restrict__ slots, int H, int Hkv, int D,
                                        int blk, const bf16_t* __restrict__ bias) {
  const int t = blockIdx.x;
  const int N = (H + 2 * Hkv) * D;
  const size_t slab_stride = (size_t)Mpad * N;
  const float* row = part + (size_t)t * N;
  const int half = D >> 1;
  const int slot = slots[t];
  const float2* csr = cs ? cs + (size_t)positions[t] * half : nullptr;
  const int pv = half >> 2;
  const int nq = H * pv, nk = Hkv * pv;
  const int dv = D >> 3;
  const int total = nq + nk + Hkv * dv;
  // items: [q rotations | k rotations + append | v appends], spread over gridDim.y blocks
  for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < total; i += gridDim.y * blockDim.x) {
    if (i >= nq + nk) {
      if (slot < 0) continue;
      const int j = i - nq - nk;
      const int h = j / dv, c = (j - h * dv) * 8;
      const int bb = slot / blk, o = slot - bb * blk;
      float v[8];
      slab_load8(part, slab_stride, S, (size_t)t * N + (H + Hkv) * D + h * D + c, v);
      if (bias) {
        float bv[8];
        unpack8(*reinterpret_cast<const uint4*>(bias + (H + Hkv) * D + h * D + c), bv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += bv[j];
      }
      *reinterpret_cast<uint4*>(vc + (((size_t)bb * Hkv + h) * blk + o) * D + c) = pack8(v);
      continue;
    }
    const bool isk = i >= nq;
    const int ii = isk ? i - nq : i;
    const int h = ii / pv, c = (ii - h * pv) * 4;
    const int base = (isk ? H * D : 0) + h * D;
    float a[4], b[4];
    {
      float4 x = *reinterpret_cast<const float4*>(row + base + c);
      float4 y = *reinterpret_cast<const float4*>(row + base + c + half);
      a[0] = x.x; a[1] = x.y; a[2] = x.z; a[3] = x.w; b[0] = y.x; b[1] = y.y; b[2] = y.z; b[3] = y.w;
      for (int s = 1; s < S; ++s) {
        x = *reinterpret_cast<const float4*>(row + s * slab_stride + base + c);
        y = *reinterpret_cast<const float4*>(row + s * slab_stride + base + c + half);
        a[0] += x.x; a[1] += x.y; a[2] += x.z; a[3] += x.w;
        b[0] += y.x; b[1] += y.y; b[2] += y.z; b[3] += y.w;
      }
    }
    if (bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] += bf2f(bias[base + c + j]);
        b[j] += bf2f(bias[base + c + half + j]);
      }
    }
    // round to bf16 first: the projection output is a bf16 tensor in the model
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = bf2f(f2bf(a[j])); b[j] = bf2f(f2bf(b[j])); }
    if (csr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 e = csr[c + j];
        const float ra = a[j] * e.x - b[j] * e.y;
        const float rb = b[j] * e.x + a[j] * e.y;
        a[j] = ra;
        b[j] = rb;
      }
    }
    uint2 lo, hi;
    lo.x = pack_bf16x2(a[0], a[1]); lo.y = pack_bf16x2(a[2], a[3]);
    hi.x = pack_bf16x2(b[0], b[1]); hi.y = pack_bf16x2(b[2], b[3]);
    bf16_t* dst;
    if (!isk) {
      dst = q_out + (size_t)t * H * D + h * D;
    } else {
      if (slot < 0) continue;
      const int bb = slot / blk, o = slot - bb * blk;
      dst = kc + (((size_t)bb * Hkv + h) * blk + o) * D;
    }
    *reinterpret_cast<uint2*>(dst + c) = lo;
    *reinterpret_cast<uint2*>(dst + c + half) = hi;
  }
}

// LayerNorm consumer (Whisper decoder): h = sum_s part + bias (+ residual);
// residual <- h (bf16); y = (h - mean) / sqrt(var + eps) * w + b.
__global__ __launch_bounds__(NT) void slab_layernorm_kernel(
    const float* __restrict__ part, int S, int Mpad, const int64_t* __restrict__ row_idx,
    const bf16_t* __restrict__ pbias, bf16_t* __restrict__ residual, int write_residual,
    const bf16_t* __restrict__ w, const bf16_t* __restrict__ lb, bf16_t* __restrict__ y, int d,
    float eps) {
  __shared__ float scratch[NT / 64];
  const int row = blockIdx.x;
  const int src = row_idx ? (int)row_idx[row] : row;
  const size_t slab_stride = (size_t)Mpad * d;
  const int nvec = d >> 3;
  uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)src * d);
  float v[MAXV][8];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NT;
    if (c < nvec) {
      slab_load8(part, slab_stride, S, (size_t)src * d + c * 8, v[i]);
      float r[8];
      // the projection output (with bias) is a bf16 tensor in the model
      if (pbias) {
        unpack8(reinterpret_cast<const uint4*>(pbias)[c], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j]));
      unpack8(rr[c], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] += r[j];
      uint4 p = pack8(v[i]);
      if (write_residual) rr[c] = p;
      unpack8(p, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[i][j];
    }
  }
  const float mean = block_sum(sum, scratch) / (float)d;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NT;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = v[i][j] - mean;
        ss += t * t;
      }
    }
  }
  __syncthreads();
  const float inv = rsqrtf(block_sum(ss, scratch) / (float)d + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  const uint4* br = reinterpret_cast<const uint4*>(lb);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * d);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * NT;
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

// out[m, n] = act(bf16(sum_s part[s][m][n] + bias[n])), act: 0 identity, 1 GELU(erf)
__global__ void slab_bias_act_kernel(const float* __restrict__ part, int S, int Mpad, int N,
                                     const bf16_t* __restrict__ bias, int act,
                                     bf16_t* __restrict__ out, long long total_vec) {
  const size_t slab_stride = (size_t)Mpad * N;
  const int nv = N >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total_vec;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % nv) * 8;
    float v[8];
    slab_load8(part, slab_stride, S, (size_t)i * 8, v);
    if (bias) {
      float bv[8];
      unpack8(*reinterpret_cast<const uint4*>(bias + c), bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bv[j];
    }
    if (act == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = bf2f(f2bf(v[j]));
        v[j] = 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
      }
    }
    *reinterpret_cast<uint4*>(out + (size_t)i * 8) = pack8(v);
  }
}

// gate|up slabs [S][Mpad][2F] -> out [M, F] bf16 (silu(gate) * up, operands rounded to bf16)
__global__ void slab_silu_mul_kernel(const float* __restrict__ part, int S, int Mpad, int F,
                                     bf16_t* __restrict__ out, long long total_vec) {
  const int fv = F >> 3;
  const size_t slab_stride = (size_t)Mpad * 2 * F;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total_vec;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / fv;
    const int c = (int)(i - row * fv) * 8;
    float g[8], u[8], o[8];
    slab_load8(part, slab_stride, S, (size_t)row * 2 * F + c, g);
    slab_load8(part, slab_stride, S, (size_t)row * 2 * F + F + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gg = bf2f(f2bf(g[j])), uu = bf2f(f2bf(u[j]));
      o[j] = gg / (1.f + __expf(-gg)) * uu;
    }
    *reinterpret_cast<uint4*>(out + row * F + c) = pack8(o);
  }
}

// out[m, n] = sum_s part[s][m][n] for m < M (f32)
__global__ void slab_reduce_kernel(const float* __restrict__ part, int S, int Mpad, int N,
                                   float* __restrict__ out, long long total_vec) {
  const size_t slab_stride = (size_t)Mpad * N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total_vec;
       i += (long long)gridDim.x * blockDim.x) {
    float v[8];
    slab_load8(part, slab_stride, S, (size_t)i * 8, v);
    *reinterpret_cast<float4*>(out + i * 8) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(out + i * 8 + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

extern "C" int loqa_slab_rmsnorm(const float* part, int S, int Mpad, const int64_t* row_idx, int rows,
                                 void* residual, int write_residual, const void* w, void* y, int d,
                                 float eps, hipStream_t st) {
  if (rows <= 0) return 0;
  if (d % 8 || d > NT * 8 * MAXV) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(slab_rmsnorm_kernel, dim3(rows), dim3(NT), 0, st, part, S, Mpad, row_idx,
                     (bf16_t*)residual, write_residual, (const bf16_t*)w, (bf16_t*)y, d, eps);
  return (int)hipGetLastError();
}

extern "C" int loqa_slab_rope_append(const float* part, int S, int Mpad, int M, const int* positions,
                                     const void* cs, void* q_out, void* kc, void* vc,
                                     const int* slots, int H, int Hkv, int D, int blk,
                                     const void* bias, hipStream_t st) {
  if (M <= 0) return 0;
  if (D % 8) return (int)hipErrorInvalidValue;
  const int items = (H + Hkv) * (D / 8) + Hkv * (D / 8);
  hipLaunchKernelGGL(slab_rope_append_kernel, dim3(M, (items + 127) / 128), dim3(128), 0, st, part, S, Mpad, positions,
                     (const float2*)cs, (bf16_t*)q_out, (bf16_t*)kc, (bf16_t*)vc, slots, H, Hkv, D,
                     blk, (const bf16_t*)bias);
  return (int)hipGetLastError();
}

extern "C" int loqa_slab_silu_mul(const float* part, int S, int Mpad, int M, int F, void* out,
                                  hipStream_t st) {
  if (M <= 0) return 0;
  if (F % 8) return (int)hipErrorInvalidValue;
  const long long tv = (long long)M * (F / 8);
  long long blocks = (tv + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(slab_silu_mul_kernel, dim3((unsigned)blocks), dim3(256), 0, st, part, S, Mpad,
                     F, (bf16_t*)out, tv);
  return (int)hipGetLastError();
}

extern "C" int loqa_slab_reduce(const float* part, int S, int Mpad, int M, int N, float* out,
                                hipStream_t st) {
  if (M <= 0) return 0;
  if (N % 8) return (int)hipErrorInvalidValue;
  const long long tv = (long long)M * N / 8;
  long long blocks = (tv + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, part, S, Mpad, N,
                     out, tv);
  return (int)hipGetLastError();
}

extern "C" int loqa_slab_layernorm(const float* part, int S, int Mpad, const int64_t* row_idx,
                                   int rows, const void* pbias, void* residual, int write_residual,
                                   const void* w, const void* b, void* y, int d, float eps,
                                   hipStream_t st) {
  if (rows <= 0) return 0;
  if (d % 8 || d > NT * 8 * MAXV) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(slab_layernorm_kernel, dim3(rows), dim3(NT), 0, st, part, S, Mpad, row_idx,
                     (const bf16_t*)pbias, (bf16_t*)residual, write_residual, (const bf16_t*)w,
                     (const bf16_t*)b, (bf16_t*)y, d, eps);
  return (int)hipGetLastError();
}

extern "C" int loqa_slab_bias_act(const float* part, int S, int Mpad, int M, int N,
                                  const void* bias, int act, void* out, hipStream_t st) {
  if (M <= 0) return 0;
  if (N % 8 || act < 0 || act > 1) return (int)hipErrorInvalidValue;
  const long long tv = (long long)M * N / 8;
  long long blocks = (tv + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(slab_bias_act_kernel, dim3((unsigned)blocks), dim3(256), 0, st, part, S, Mpad,
                     N, (const bf16_t*)bias, act, (bf16_t*)out, tv);
  return (int)hipGetLastError();
}
