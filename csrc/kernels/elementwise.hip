// Memory-bound fused elementwise kernels:
//   K1  pcm16 -> f32 conversion fused with the per-utterance sum of squares used
//       by wake-word arbitration RMS (reference: audio_service.go:1048-1101 and
//       :818-852 do these as two per-sample Go loops).
//   K6  bias + GELU (+ sinusoidal position add) epilogue for Whisper conv/MLP.
//   K11 RoPE on q/k + paged KV-cache append (K16), reading the fused QKV GEMM
//       output in place.
//   K14 SwiGLU gate: silu(gate) * up.
//   K15 grammar-masked argmax over the vocabulary (jump-forward JSON decoding).
// All bf16 traffic is 8-16 bytes per lane (guide G13).
#include "common.h"
#include <float.h>

// ---------------------------------------------------------------- K14 SwiGLU
// in: [T, 2F] = [gate | up], out: [T, F]. 2-D grid (x: 8-wide column vectors,
// y: rows): one 16-byte vector per thread, no per-element 64-bit division (the
// grid-stride form with `i / (F / 8)` ran at 0.8 TB/s on the 318 x 14336
// prefill activations; these kernels are pure streams).
__global__ __launch_bounds__(256) void silu_mul_kernel(const bf16_t* __restrict__ in,
                                                      bf16_t* __restrict__ out, int F) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= (F >> 3)) return;
  const size_t row = blockIdx.y;
  const uint4 gv = reinterpret_cast<const uint4*>(in + row * 2 * F)[c];
  const uint4 uv = reinterpret_cast<const uint4*>(in + row * 2 * F + F)[c];
  float a[8], b[8], o[8];
  unpack8(gv, a);
  unpack8(uv, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = a[j] / (1.f + __expf(-a[j])) * b[j];
  reinterpret_cast<uint4*>(out + row * F)[c] = pack8(o);
}

extern "C" int loqa_silu_mul(const void* in, void* out, long long rows, int F, hipStream_t s) {
  if (F % 8 != 0 || rows <= 0) return (int)hipErrorInvalidValue;
  for (long long r0 = 0; r0 < rows; r0 += 65535) {   // grid.y limit
    const long long n = rows - r0 < 65535 ? rows - r0 : 65535;
    dim3 grid((unsigned)((F / 8 + 255) / 256), (unsigned)n);
    hipLaunchKernelGGL(silu_mul_kernel, grid, dim3(256), 0, s, (const bf16_t*)in + r0 * 2 * F,
                       (bf16_t*)out + r0 * F, F);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------ K6 bias+GELU(+pos)
// x[T, F] <- gelu(x + bias) + pos[(t % pos_period), :]   (bias, pos optional);
// 2-D grid as silu_mul
__global__ __launch_bounds__(256) void gelu_bias_kernel(bf16_t* __restrict__ x,
                                                       const bf16_t* __restrict__ bias,
                                                       const bf16_t* __restrict__ pos, int F,
                                                       int pos_period, long long row0) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= (F >> 3)) return;
  const size_t row = (size_t)row0 + blockIdx.y;
  uint4* p = reinterpret_cast<uint4*>(x + row * F) + c;
  float v[8];
  unpack8(*p, v);
  if (bias) {
    float b[8];
    unpack8(reinterpret_cast<const uint4*>(bias)[c], b);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += b[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.5f * v[j] * (1.f + erff(v[j] * 0.70710678118654752f));
  if (pos) {
    float q[8];
    const size_t prow = row % (size_t)pos_period;
    unpack8(reinterpret_cast<const uint4*>(pos + prow * F)[c], q);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += q[j];
  }
  *p = pack8(v);
}

extern "C" int loqa_gelu_bias(void* x, const void* bias, const void* pos, long long rows, int F,
                              int pos_period, hipStream_t s) {
  if (F % 8 != 0 || rows <= 0 || (pos && pos_period <= 0)) return (int)hipErrorInvalidValue;
  for (long long r0 = 0; r0 < rows; r0 += 65535) {   // grid.y limit
    const long long n = rows - r0 < 65535 ? rows - r0 : 65535;
    dim3 grid((unsigned)((F / 8 + 255) / 256), (unsigned)n);
    hipLaunchKernelGGL(gelu_bias_kernel, grid, dim3(256), 0, s, (bf16_t*)x, (const bf16_t*)bias,
                       (const bf16_t*)pos, F, pos_period, r0);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------ K11/K16 RoPE + KV append
// qkv: [T, stride] with q at [0, Hq*D), k at [Hq*D, (Hq+Hkv)*D), v after it.
// q (and k) are rotated in place (NeoX rotate-half pairing i <-> i + D/2);
// k and v are then written to the paged cache [nblocks, Hkv, blk, D] at
// slot = slots[t] (= block * blk + offset). cs == nullptr disables the rotation
// (Whisper decoder, learned positions). slots[t] < 0 skips the append (padding).
__global__ void rope_kv_append_kernel(bf16_t* __restrict__ qkv, int stride,
                                      const int* __restrict__ positions,
                                      const float2* __restrict__ cs, bf16_t* __restrict__ kc,
                                      bf16_t* __restrict__ vc, const int* __restrict__ slots,
                                      int Hq, int Hkv, int D, int blk) {
  const int t = blockIdx.x;
  bf16_t* row = qkv + (size_t)t * stride;
  const int half = D >> 1;
  const int pv = half >> 2;  // 4-element groups per half-head
  const int slot = slots ? slots[t] : -1;
  const float2* csr = cs ? cs + (size_t)positions[t] * half : nullptr;
  const int nq = Hq * pv, nk = Hkv * pv;
  // q and k rotation (k rotation only materialised into the cache).
  for (int i = threadIdx.x; i < nq + nk; i += blockDim.x) {
    const bool isk = i >= nq;
    const int ii = isk ? i - nq : i;
    const int h = ii / pv, c = (ii - h * pv) * 4;
    bf16_t* base = row + (isk ? Hq * D : 0) + h * D;
    uint2 lo = *reinterpret_cast<const uint2*>(base + c);
    uint2 hi = *reinterpret_cast<const uint2*>(base + c + half);
    if (csr) {
      float a[4] = {__uint_as_float(lo.x << 16), __uint_as_float(lo.x & 0xffff0000u),
                    __uint_as_float(lo.y << 16), __uint_as_float(lo.y & 0xffff0000u)};
      float b[4] = {__uint_as_float(hi.x << 16), __uint_as_float(hi.x & 0xffff0000u),
                    __uint_as_float(hi.y << 16), __uint_as_float(hi.y & 0xffff0000u)};
      float ra[4], rb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float2 e = csr[c + j];
        ra[j] = a[j] * e.x - b[j] * e.y;
        rb[j] = b[j] * e.x + a[j] * e.y;
      }
      lo.x = pack_bf16x2(ra[0], ra[1]);
      lo.y = pack_bf16x2(ra[2], ra[3]);
      hi.x = pack_bf16x2(rb[0], rb[1]);
      hi.y = pack_bf16x2(rb[2], rb[3]);
    }
    if (!isk) {
      *reinterpret_cast<uint2*>(base + c) = lo;
      *reinterpret_cast<uint2*>(base + c + half) = hi;
    } else if (slot >= 0) {
      const int b = slot / blk, o = slot - b * blk;
      bf16_t* dst = kc + (((size_t)b * Hkv + h) * blk + o) * D;
      *reinterpret_cast<uint2*>(dst + c) = lo;
      *reinterpret_cast<uint2*>(dst + c + half) = hi;
    }
  }
  if (slot >= 0) {
    const int b = slot / blk, o = slot - b * blk;
    const int dv = D >> 3;
    for (int i = threadIdx.x; i < Hkv * dv; i += blockDim.x) {
      const int h = i / dv, c = (i - h * dv) * 8;
      const uint4 v = *reinterpret_cast<const uint4*>(row + (Hq + Hkv) * D + h * D + c);
      *reinterpret_cast<uint4*>(vc + (((size_t)b * Hkv + h) * blk + o) * D + c) = v;
    }
  }
}

// Same operation, every load of the row issued before any store: the loop form
// above reads, rotates and writes one 4-element group per trip, and its
// in-place q stores keep the compiler from hoisting the next trip's loads, so
// a thread pays one memory round trip per group (5 at Llama-3-8B's 40 heads).
// Here each thread holds up to RK groups (and its V piece) in registers.
template <int RK>
__global__ __launch_bounds__(128) void rope_kv_append_batched_kernel(
    bf16_t* __restrict__ qkv, int stride, const int* __restrict__ positions,
    const float2* __restrict__ cs, bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
    const int* __restrict__ slots, int Hq, int Hkv, int D, int blk) {
  const int t = blockIdx.x;
  bf16_t* row = qkv + (size_t)t * stride;
  const int half = D >> 1, pv = half >> 2, dv = D >> 3;
  const int nq = Hq * pv, nk = Hkv * pv;
  uint2 lo[RK], hi[RK];
#pragma unroll
  for (int k = 0; k < RK; ++k) {
    const int i = threadIdx.x + k * 128;
    lo[k] = hi[k] = make_uint2(0u, 0u);
    if (i < nq + nk) {
      const bool isk = i >= nq;
      const int ii = isk ? i - nq : i;
      const int h = ii / pv, c = (ii - h * pv) * 4;
      const bf16_t* base = row + (isk ? Hq * D : 0) + h * D;
      lo[k] = *reinterpret_cast<const uint2*>(base + c);
      hi[k] = *reinterpret_cast<const uint2*>(base + c + half);
    }
  }
  const int slot = slots ? slots[t] : -1;
  const bool vok = slot >= 0 && (int)threadIdx.x < Hkv * dv;
  uint4 vv = make_uint4(0u, 0u, 0u, 0u);
  if (vok) {
    const int h = threadIdx.x / dv, c = (threadIdx.x - h * dv) * 8;
    vv = *reinterpret_cast<const uint4*>(row + (Hq + Hkv) * D + h * D + c);
  }
  const float2* csr = cs ? cs + (size_t)positions[t] * half : nullptr;
  float2 e[RK][4];
#pragma unroll
  for (int k = 0; k < RK; ++k) {
    const int i = threadIdx.x + k * 128;
    const int ii = i >= nq ? i - nq : i;
    const int c = (ii - (ii / pv) * pv) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      e[k][j] = (csr && i < nq + nk) ? csr[c + j] : make_float2(1.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < RK; ++k) {
    const int i = threadIdx.x + k * 128;
    if (i >= nq + nk) break;
    const bool isk = i >= nq;
    const int ii = isk ? i - nq : i;
    const int h = ii / pv, c = (ii - h * pv) * 4;
    uint2 l = lo[k], u = hi[k];
    if (csr) {
      float a[4] = {__uint_as_float(l.x << 16), __uint_as_float(l.x & 0xffff0000u),
                    __uint_as_float(l.y << 16), __uint_as_float(l.y & 0xffff0000u)};
      float b[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                    __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
      float ra[4], rb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ra[j] = a[j] * e[k][j].x - b[j] * e[k][j].y;
        rb[j] = b[j] * e[k][j].x + a[j] * e[k][j].y;
      }
      l.x = pack_bf16x2(ra[0], ra[1]);
      l.y = pack_bf16x2(ra[2], ra[3]);
      u.x = pack_bf16x2(rb[0], rb[1]);
      u.y = pack_bf16x2(rb[2], rb[3]);
    }
    if (!isk) {
      bf16_t* base = row + h * D;
      *reinterpret_cast<uint2*>(base + c) = l;
      *reinterpret_cast<uint2*>(base + c + half) = u;
    } else if (slot >= 0) {
      const int b = slot / blk, o = slot - b * blk;
      bf16_t* dst = kc + (((size_t)b * Hkv + h) * blk + o) * D;
      *reinterpret_cast<uint2*>(dst + c) = l;
      *reinterpret_cast<uint2*>(dst + c + half) = u;
    }
  }
  if (vok) {
    const int b = slot / blk, o = slot - b * blk;
    const int h = threadIdx.x / dv, c = (threadIdx.x - h * dv) * 8;
    *reinterpret_cast<uint4*>(vc + (((size_t)b * Hkv + h) * blk + o) * D + c) = vv;
  }
}

extern "C" int loqa_rope_kv_append(void* qkv, int stride, const int* positions, const void* cs,
                                   void* kc, void* vc, const int* slots, int T, int Hq, int Hkv,
                                   int D, int blk, hipStream_t s) {
  if (T <= 0) return 0;
  if (D % 8 != 0 || stride < (Hq + 2 * Hkv) * D || (cs && !positions)) return (int)hipErrorInvalidValue;
  if ((Hq + Hkv) * (D / 8) <= 8 * 128 && Hkv * (D / 8) <= 128) {
    hipLaunchKernelGGL(rope_kv_append_batched_kernel<8>, dim3(T), dim3(128), 0, s, (bf16_t*)qkv,
                       stride, positions, (const float2*)cs, (bf16_t*)kc, (bf16_t*)vc, slots, Hq,
                       Hkv, D, blk);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(rope_kv_append_kernel, dim3(T), dim3(128), 0, s, (bf16_t*)qkv, stride,
                     positions, (const float2*)cs, (bf16_t*)kc, (bf16_t*)vc, slots, Hq, Hkv, D,
                     blk);
  return (int)hipGetLastError();
}

// --------------------------------------------- K1 PCM16 -> f32 + sum of squares
// pcm: concatenated int16 samples of S segments (offsets[S+1] in samples).
// out: f32 samples (x / 32767, as audio_service.go:1078), sumsq[S] accumulates.
#define PCM_CHUNK 8192
__global__ void pcm16_f32_sumsq_kernel(const int16_t* __restrict__ pcm, float* __restrict__ out,
                                       const long long* __restrict__ offsets,
                                       float* __restrict__ sumsq) {
  __shared__ float scratch[4];
  const int seg = blockIdx.y;
  const long long beg = offsets[seg], end = offsets[seg + 1];
  const long long c0 = beg + (long long)blockIdx.x * PCM_CHUNK;
  float acc = 0.f;
  if (c0 < end) {
    const long long c1 = min(end, c0 + PCM_CHUNK);
    for (long long i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
      const float f = (float)pcm[i] * (1.0f / 32767.0f);
      out[i] = f;
      acc += f * f;
    }
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0 && c0 < end) atomicAdd(sumsq + seg, acc);
}

extern "C" int loqa_pcm16_f32_sumsq(const void* pcm, float* out, const long long* offsets,
                                    float* sumsq, int nseg, long long max_seg_len, hipStream_t s) {
  if (nseg <= 0) return 0;
  hipError_t e = hipMemsetAsync(sumsq, 0, sizeof(float) * nseg, s);
  if (e != hipSuccess) return (int)e;
  const long long chunks = max_seg_len <= 0 ? 1 : (max_seg_len + PCM_CHUNK - 1) / PCM_CHUNK;
  hipLaunchKernelGGL(pcm16_f32_sumsq_kernel, dim3((unsigned)chunks, nseg), dim3(256), 0, s,
                     (const int16_t*)pcm, out, offsets, sumsq);
  return (int)hipGetLastError();
}

// Padded variant: segment s lands in row s of out [nseg, ld] (the Whisper
// front end's 30 s window), zero beyond the segment - one launch instead of a
// zero-fill plus a copy per utterance.
__global__ void pcm16_f32_pad_kernel(const int16_t* __restrict__ pcm, float* __restrict__ out,
                                     const long long* __restrict__ offsets, float* __restrict__ sumsq,
                                     long long ld) {
  __shared__ float scratch[4];
  const int seg = blockIdx.y;
  const long long beg = offsets[seg], len = min(offsets[seg + 1] - beg, ld);
  const long long c0 = (long long)blockIdx.x * PCM_CHUNK;
  const long long c1 = min(ld, c0 + PCM_CHUNK);
  float* row = out + (size_t)seg * ld;
  float acc = 0.f;
  for (long long i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
    const float f = i < len ? (float)pcm[beg + i] * (1.0f / 32767.0f) : 0.f;
    row[i] = f;
    acc += f * f;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0 && c0 < len) atomicAdd(sumsq + seg, acc);
}

extern "C" int loqa_pcm16_f32_pad(const void* pcm, float* out, const long long* offsets, float* sumsq,
                                  int nseg, long long ld, hipStream_t s) {
  if (nseg <= 0 || ld <= 0) return nseg < 0 || ld < 0 ? (int)hipErrorInvalidValue : 0;
  hipError_t e = hipMemsetAsync(sumsq, 0, sizeof(float) * nseg, s);
  if (e != hipSuccess) return (int)e;
  const long long chunks = (ld + PCM_CHUNK - 1) / PCM_CHUNK;
  hipLaunchKernelGGL(pcm16_f32_pad_kernel, dim3((unsigned)chunks, nseg), dim3(256), 0, s,
                     (const int16_t*)pcm, out, offsets, sumsq, ld);
  return (int)hipGetLastError();
}

// --------------------------------------------------- K15 grammar-masked argmax
// logits: [B, V] (bf16 if is_bf16 else f32), row stride ld elements.
// mask: [*, W] uint32 bitmask (bit v%32 of word v/32 = token v allowed), or null;
// mask_rows: optional per-row index into the mask table (rows share the
// precomputed grammar-state masks). Each row is split over ARG_CHUNK-token
// workgroups (a 128k vocabulary -> 16 workgroups per row, so B=16 rows fill the
// GPU); each workgroup folds its best (value, index) into one 64-bit atomicMax
// of (order-preserving float key << 32 | ~index) - ties resolve to the lowest
// index like torch.argmax. out_idx[b] = argmax over allowed tokens (or -1).
#define ARG_CHUNK 8192
#define ARG_THREADS 256

__device__ __forceinline__ unsigned long long argpack(float v, int idx) {
  const uint32_t bits = __float_as_uint(v);
  const uint32_t key = (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
  return ((unsigned long long)key << 32) | (0xFFFFFFFFu - (uint32_t)idx);
}

template <bool BF16>
__global__ __launch_bounds__(ARG_THREADS) void masked_argmax_kernel(
    const void* __restrict__ logits, long long ld, int V, const uint32_t* __restrict__ mask,
    const int* __restrict__ mask_rows, int W, unsigned long long* __restrict__ packed) {
  __shared__ unsigned long long sbest[ARG_THREADS / 64];
  const int b = blockIdx.y;
  const int v_begin = blockIdx.x * ARG_CHUNK;
  const int v_end = min(V, v_begin + ARG_CHUNK);
  const uint32_t* m = nullptr;
  if (mask) m = mask + (size_t)(mask_rows ? mask_rows[b] : b) * W;
  unsigned long long best = 0;
  if (BF16) {
    const bf16_t* row = reinterpret_cast<const bf16_t*>(logits) + (size_t)b * ld;
    for (int v0 = v_begin + threadIdx.x * 8; v0 < v_end; v0 += ARG_THREADS * 8) {
      if (v0 + 8 <= v_end && (ld % 8 == 0)) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(row + v0), f);
        const uint32_t bits = m ? (m[v0 >> 5] >> (v0 & 31)) & 0xffu : 0xffu;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((bits >> j) & 1u) best = max(best, argpack(f[j], v0 + j));
      } else {
        for (int v = v0; v < min(v_end, v0 + 8); ++v)
          if (!m || ((m[v >> 5] >> (v & 31)) & 1u)) best = max(best, argpack(bf2f(row[v]), v));
      }
    }
  } else {
    const float* row = reinterpret_cast<const float*>(logits) + (size_t)b * ld;
    for (int v0 = v_begin + threadIdx.x * 4; v0 < v_end; v0 += ARG_THREADS * 4) {
      if (v0 + 4 <= v_end && (ld % 4 == 0)) {
        const float4 f = *reinterpret_cast<const float4*>(row + v0);
        const uint32_t bits = m ? (m[v0 >> 5] >> (v0 & 31)) & 0xfu : 0xfu;
        if (bits & 1u) best = max(best, argpack(f.x, v0));
        if (bits & 2u) best = max(best, argpack(f.y, v0 + 1));
        if (bits & 4u) best = max(best, argpack(f.z, v0 + 2));
        if (bits & 8u) best = max(best, argpack(f.w, v0 + 3));
      } else {
        for (int v = v0; v < min(v_end, v0 + 4); ++v)
          if (!m || ((m[v >> 5] >> (v & 31)) & 1u)) best = max(best, argpack(row[v], v));
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(best, o, 64);
    best = max(best, other);
  }
  if ((threadIdx.x & 63) == 0) sbest[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < ARG_THREADS / 64; ++i) best = max(best, sbest[i]);
    if (best) atomicMax(packed + b, best);
  }
}

__global__ void argmax_unpack_kernel(const unsigned long long* __restrict__ packed, int B,
                                     int* __restrict__ out_idx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) {
    const unsigned long long p = packed[b];
    out_idx[b] = p ? (int)(0xFFFFFFFFu - (uint32_t)(p & 0xFFFFFFFFull)) : -1;
  }
}

// workspace: >= B * 8 bytes (device)
extern "C" int loqa_masked_argmax(const void* logits, int is_bf16, long long ld, int B, int V,
                                  const uint32_t* mask, const int* mask_rows, int W, int* out_idx,
                                  void* workspace, hipStream_t s) {
  if (B <= 0) return 0;
  if ((mask && W * 32 < V) || !workspace) return (int)hipErrorInvalidValue;
  unsigned long long* packed = (unsigned long long*)workspace;
  hipError_t e = hipMemsetAsync(packed, 0, sizeof(unsigned long long) * B, s);
  if (e != hipSuccess) return (int)e;
  dim3 grid((V + ARG_CHUNK - 1) / ARG_CHUNK, B);
  if (is_bf16)
    hipLaunchKernelGGL(masked_argmax_kernel<true>, grid, dim3(ARG_THREADS), 0, s, logits, ld, V, mask,
                       mask_rows, W, packed);
  else
    hipLaunchKernelGGL(masked_argmax_kernel<false>, grid, dim3(ARG_THREADS), 0, s, logits, ld, V,
                       mask, mask_rows, W, packed);
  e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(argmax_unpack_kernel, dim3((B + 63) / 64), dim3(64), 0, s, packed, B, out_idx);
  return (int)hipGetLastError();
}

// ------------------------------------------------- pipelined decode: step I/O
// A decode step graph exchanges its host data without copy-engine operations
// between graphs (each H2D / D2H copy on the decode stream cost a copy-engine
// hand-off of tens of microseconds between two back-to-back step graphs).
// The host stages a step's metadata in pinned memory; the graph's first node
// reads it zero-copy into the graph's device buffers, and its last node writes
// the sampled tokens zero-copy into a pinned result ring. *ctr counts the step
// graphs launched so far (advanced by the last node), so the staging slot
// (ctr % 2) and result slot (ctr % nres) follow the host's launch order.
__global__ __launch_bounds__(256) void step_fetch_kernel(int* __restrict__ d32,
                                                        const int* __restrict__ h32, int n32,
                                                        int stride32, long long* __restrict__ d64,
                                                        const long long* __restrict__ h64, int n64,
                                                        int stride64, const int* __restrict__ ctr,
                                                        int T, int src_off,
                                                        const int* __restrict__ last_tok) {
  const int slot = ctr[0] & 1;
  const int* src = h32 + (size_t)slot * stride32;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n32; i += gridDim.x * 256) {
    int v = src[i];
    if (i < T) {   // tokens: a staged src slot >= 0 takes that sequence's last sampled token
      const int sl = src[src_off + i];
      // a failed step's sentinel (-1 nothing allowed, -2 collective error)
      // must never become an embedding row index: the host fails those
      // sequences when it reads the step, this one only has to stay in bounds
      if (sl >= 0) v = max(last_tok[sl], 0);
    }
    d32[i] = v;
  }
  const long long* src64 = h64 + (size_t)slot * stride64;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n64; i += gridDim.x * 256) d64[i] = src64[i];
}

__global__ __launch_bounds__(256) void step_publish_kernel(const int* __restrict__ out, int n,
                                                          int* __restrict__ res, int stride,
                                                          int nres, int* __restrict__ ctr,
                                                          const int* __restrict__ row_slot,
                                                          int* __restrict__ last_tok) {
  const int c = ctr[0];
  int* dst = res + (size_t)(c % nres) * stride;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int v = out[i];
    dst[i] = v;
    last_tok[row_slot[i]] = v;     // padding rows write the trash slot
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    // wrap at 2 * nres (a common multiple of the 2 staging slots and the nres
    // result slots; the host's step number wraps the same way), so the counter
    // never overflows on a long-running hub
    __hip_atomic_store(ctr, (c + 1) % (2 * nres), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// T: token rows at the head of the staged int32 block; src_off: offset of the
// per-token source-slot array in it (see LLMEngine._decode_graph).
extern "C" int loqa_step_fetch(void* d32, const void* h32, int n32, int stride32, void* d64,
                               const void* h64, int n64, int stride64, const int* ctr, int T,
                               int src_off, const int* last_tok, hipStream_t s) {
  if (n32 < 0 || n32 > stride32 || n64 < 0 || n64 > stride64 || src_off + T > n32)
    return (int)hipErrorInvalidValue;
  int blocks = (n32 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 16 ? 16 : blocks);
  hipLaunchKernelGGL(step_fetch_kernel, dim3(blocks), dim3(256), 0, s, (int*)d32, (const int*)h32, n32,
                     stride32, (long long*)d64, (const long long*)h64, n64, stride64, ctr, T, src_off,
                     last_tok);
  return (int)hipGetLastError();
}

extern "C" int loqa_step_publish(const int* out, int n, void* res, int stride, int nres, int* ctr,
                                 const int* row_slot, int* last_tok, hipStream_t s) {
  if (n < 0 || n > stride || nres < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(step_publish_kernel, dim3(1), dim3(256), 0, s, out, n, (int*)res, stride, nres, ctr,
                     row_slot, last_tok);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Counter-based random init (seeded random-init weights): element
// (r, c) of a [rows, cols] block at (row0, col0) of a conceptual [*, ld] tensor
// gets scale * (u0 + u1 + u2 + u3 - 2) with u_k = fmix32(4 * idx + k + s) / 2^32
// (Irwin-Hall(4): mean 0, variance 1/3 - the caller folds sqrt(3) into scale),
// idx = (row0 + r) * ld + col0 + c. Any shard of a tensor is generated on its
// own, with exactly the values of the unsharded tensor (tensor-parallel ranks
// build their slices without materialising the full model). Integer hashing and
// exact f32 sums: bitwise equal to the CPU path (ops.reference.init_uniform4).
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}

__global__ __launch_bounds__(256) void init_uniform4_kernel(bf16_t* __restrict__ out, long long rows,
                                                            int cols, long long ld, long long row0,
                                                            long long col0, uint32_t s, float scale) {
  const long long n = rows * cols;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long r = i / cols, c = i - r * cols;
    const uint32_t idx = (uint32_t)((row0 + r) * ld + col0 + c);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += (float)(fmix32(idx * 4u + (uint32_t)k + s) >> 8) * (1.0f / 16777216.0f);
    out[i] = f2bf((acc - 2.0f) * scale);
  }
}

extern "C" int loqa_init_uniform4(void* out, long long rows, int cols, long long ld, long long row0,
                                  long long col0, unsigned s, float scale, hipStream_t st) {
  if (rows < 0 || cols < 0 || col0 + cols > ld) return (int)hipErrorInvalidValue;
  const long long n = rows * cols;
  if (n == 0) return 0;
  long long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(init_uniform4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (bf16_t*)out, rows,
                     cols, ld, row0, col0, (uint32_t)s, scale);
  return (int)hipGetLastError();
}
