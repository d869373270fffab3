// VITS text-side kernels:
//   relpos_attention : K19 - text-encoder self-attention with windowed relative
//                      position embeddings (VITS attentions.MultiHeadAttention,
//                      window 4, shared key/value relative tables), masked;
//   expand_sample    : length regulation fused with prior sampling -
//                      z_p[f] = m_p[i(f)] + eps * exp(logs_p[i(f)]) * noise_scale,
//                      i(f) = phoneme covering frame f (binary search in the
//                      cumulative durations), eps from a counter-based hash RNG.
// Activations are channels-last bf16 rows.
#include "common.h"

#define RP_MAXT 512

// one wave per (query, head, batch): lanes split the keys for the logits, then
// the output dims; softmax through wave reductions. T <= RP_MAXT.
__global__ __launch_bounds__(64) void relpos_attention_kernel(
    const bf16_t* __restrict__ qkv, int ldq, const bf16_t* __restrict__ emb_k,
    const bf16_t* __restrict__ emb_v, const int* __restrict__ lens, bf16_t* __restrict__ out,
    int ldo, int T, int H, int D, int window, float scale) {
  __shared__ float p[RP_MAXT];
  __shared__ float qs[256];
  const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z, lane = threadIdx.x;
  const int len = lens ? lens[b] : T;
  const int C = H * D;
  const bf16_t* base = qkv + (size_t)b * T * ldq;
  bf16_t* orow = out + ((size_t)b * T + i) * ldo + h * D;
  if (i >= len) {  // padded query row: zero output (masked downstream)
    for (int d = lane; d < D; d += 64) orow[d] = f2bf(0.f);
    return;
  }
  for (int d = lane; d < D; d += 64) qs[d] = bf2f(base[(size_t)i * ldq + h * D + d]) * scale;
  __syncthreads();
  float mx = -INFINITY;
  for (int j = lane; j < T; j += 64) {
    float s = -1e4f;  // VITS masked_fill value
    if (j < len) {
      const bf16_t* kr = base + (size_t)j * ldq + C + h * D;
      float acc = 0.f;
      for (int d = 0; d < D; ++d) acc += qs[d] * bf2f(kr[d]);
      const int rel = j - i;
      if (rel >= -window && rel <= window) {
        const bf16_t* er = emb_k + (size_t)(rel + window) * D;
        float a2 = 0.f;
        for (int d = 0; d < D; ++d) a2 += qs[d] * bf2f(er[d]);
        acc += a2;
      }
      s = acc;
    }
    p[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < T; j += 64) {
    const float e = __expf(p[j] - mx);
    p[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  __syncthreads();
  for (int d = lane; d < D; d += 64) {
    float acc = 0.f;
    for (int j = 0; j < T; ++j) acc += p[j] * bf2f(base[(size_t)j * ldq + 2 * C + h * D + d]);
    for (int r = -window; r <= window; ++r) {
      const int j = i + r;
      if (j >= 0 && j < T) acc += p[j] * bf2f(emb_v[(size_t)(r + window) * D + d]);
    }
    orow[d] = f2bf(acc * inv);
  }
}

extern "C" int loqa_relpos_attention(const void* qkv, int ldq, const void* emb_k, const void* emb_v,
                                     const int* lens, void* out, int ldo, int B, int T, int H,
                                     int D, int window, float scale, hipStream_t s) {
  if (B <= 0 || T <= 0) return 0;
  if (T > RP_MAXT || D > 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(relpos_attention_kernel, dim3(T, H, B), dim3(64), 0, s, (const bf16_t*)qkv,
                     ldq, (const bf16_t*)emb_k, (const bf16_t*)emb_v, lens, (bf16_t*)out, ldo, T, H,
                     D, window, scale);
  return (int)hipGetLastError();
}

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// standard normal from two hashed uniforms (Box-Muller)
__device__ __forceinline__ float gauss(unsigned seed, unsigned long long idx) {
  const unsigned a = hash32(seed ^ hash32((unsigned)idx ^ 0x9e3779b9U) ^ (unsigned)(idx >> 32));
  const unsigned c = hash32(a ^ 0x85ebca6bU);
  const float u1 = ((a >> 8) + 1) * (1.0f / 16777217.0f);
  const float u2 = (c >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

// stats [B][T][2C] (m_p | logs_p); cum [B][T] inclusive cumulative frame counts;
// z [B][F][C]; frames past flen[b] are zero. The noise of (row, frame, channel)
// does not depend on F, so a frame-padded (graph-bucketed) launch draws the
// same latent as an exact one. seed_dev (optional): the seed read on the
// device, so a captured graph draws fresh noise per replay.
__global__ void expand_sample_kernel(const bf16_t* __restrict__ stats, int ld_stats,
                                     const int* __restrict__ cum, int T,
                                     const int* __restrict__ flen, bf16_t* __restrict__ z, int F,
                                     int C, float noise_scale, unsigned seed,
                                     const unsigned* __restrict__ seed_dev) {
  const int f = blockIdx.x, b = blockIdx.y;
  if (seed_dev) seed = *seed_dev;
  bf16_t* zr = z + ((size_t)b * F + f) * C;
  if (f >= flen[b]) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) zr[c] = f2bf(0.f);
    return;
  }
  const int* cb = cum + (size_t)b * T;
  int lo = 0, hi = T - 1;  // first i with cum[i] > f
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cb[mid] > f) hi = mid; else lo = mid + 1;
  }
  const bf16_t* sr = stats + ((size_t)b * T + lo) * ld_stats;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float m = bf2f(sr[c]), lg = bf2f(sr[C + c]);
    const unsigned long long idx = (((unsigned long long)b << 24) + f) * C + c;
    zr[c] = f2bf(m + gauss(seed, idx) * __expf(lg) * noise_scale);
  }
}

extern "C" int loqa_expand_sample(const void* stats, int ld_stats, const int* cum, int B, int T,
                                  const int* flen, void* z, int F, int C, float noise_scale,
                                  unsigned seed, const unsigned* seed_dev, hipStream_t s) {
  if (B <= 0 || F <= 0) return 0;
  if (F >= (1 << 24)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(expand_sample_kernel, dim3(F, B), dim3(128), 0, s, (const bf16_t*)stats,
                     ld_stats, cum, T, flen, (bf16_t*)z, F, C, noise_scale, seed, seed_dev);
  return (int)hipGetLastError();
}
