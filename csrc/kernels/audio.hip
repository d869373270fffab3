// Whisper audio front-end on the GPU (SURVEY §2.4 K2 log_mel, K3 conv1d stem).
//
// log_mel: the STFT is a GEMM. Each 256-thread workgroup owns 32 frames of one
// utterance: the reflect-padded, Hann-windowed frames are staged in LDS, then
// the four waves run exact-f32 MFMA (v_mfma_f32_32x32x2_f32, guide §3 "FP32-input
// MFMA" - log-mel needs f32 dynamic range, bf16 would not do) against the
// cos/sin DFT basis, square-sum to the power spectrum in LDS, and project onto
// the mel filterbank with a second f32 MFMA. log10 + per-utterance max are fused
// into the epilogue; a tiny second kernel applies whisper's max-8 clamp and
// (x + 4) / 4 scaling and emits bf16.
//
// im2col: k=3, pad=1 conv1d input unfolding so the conv becomes a plain GEMM
// (hipBLASLt) followed by the fused bias+GELU(+pos) epilogue (elementwise.hip).
#include "common.h"
#include <float.h>

#define NFFT 400
#define HOP 160
#define NBINS 201
#define BIN_TILES 7         // 7 x 32 = 224 >= 201 bins
#define BASIS_LD 224
#define FRAMES_PER_WG 32
// LDS row strides are odd (in dwords): the MFMA A operands are read one frame
// (power row) per lane, 32 lanes per ds_read_b32 group with banks (a/4) % 32,
// so an even stride put 2 (400) or 8 (204) rows on each bank - 16- / 4-way
// conflicts (SQ_LDS_BANK_CONFLICT ~9.6 extra cycles per cycle)
#define FRAME_LD 401        // 400 taps + 1
#define POW_LD 203          // 202 used (K padded to even) + 1

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma_f32(float a, float b, const f16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void atomic_max_float(float* addr, float v) {
  if (v >= 0.f)
    atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
  else
    atomicMin(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

// audio: [B, n_samples] f32;  window: [400];  cosb/sinb: [400, 224];
// filt: [n_mels, 201];  out: [B, n_mels, n_frames] f32 (log10 mel);  gmax: [B]
//
// 8 waves: wave w < 7 owns DFT bin tile w (32 bins) for the workgroup's 32
// frames, then waves 0..3 own one 32-mel tile each. Every MFMA chain is split
// into two independent accumulator pairs (even / odd k-steps) and the DFT basis
// for 16 k-steps is loaded before its MFMAs, so a wave is neither one
// dependent MFMA chain nor one global load per k-step (the 4-wave form, two bin
// tiles per wave, measured ~370 us per 30-s utterance).
__global__ __launch_bounds__(512) void logmel_kernel(
    const float* __restrict__ audio, int n_samples, const float* __restrict__ window,
    const float* __restrict__ cosb, const float* __restrict__ sinb,
    const float* __restrict__ filt, int n_mels, float* __restrict__ out, int n_frames,
    float* __restrict__ gmax) {
  __shared__ float frames[FRAMES_PER_WG][FRAME_LD];
  __shared__ float power[FRAMES_PER_WG][POW_LD];
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FRAMES_PER_WG;
  const float* x = audio + (size_t)b * n_samples;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int hi = lane >> 5, lo = lane & 31;

  // 1. reflect-padded (center=True) windowed frames -> LDS
  for (int i = threadIdx.x; i < FRAMES_PER_WG * NFFT; i += blockDim.x) {
    const int f = i / NFFT, n = i - f * NFFT;
    int idx = (f0 + f) * HOP + n - NFFT / 2;
    if (idx < 0) idx = -idx;
    if (idx >= n_samples) idx = 2 * (n_samples - 1) - idx;
    frames[f][n] = (f0 + f < n_frames) ? x[idx] * window[n] : 0.f;
  }
  for (int i = threadIdx.x; i < FRAMES_PER_WG * POW_LD; i += blockDim.x)
    (&power[0][0])[i] = 0.f;
  __syncthreads();

  // 2. power spectrum: wave w handles bin tile w
  if (wave < BIN_TILES) {
    f16v re0, im0, re1, im1;
#pragma unroll
    for (int j = 0; j < 16; ++j) { re0[j] = 0.f; im0[j] = 0.f; re1[j] = 0.f; im1[j] = 0.f; }
    const int bin = wave * 32 + lo;
    const float* cb = cosb + hi * BASIS_LD + bin;
    const float* sb = sinb + hi * BASIS_LD + bin;
    // NFFT = 400 = 12 x 32 + 16: blocks of 16 k-steps (32 taps) then a tail of 8
    int k = 0;
    for (; k + 32 <= NFFT; k += 32) {
      float bc[16], bs[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        bc[u] = cb[(size_t)(k + 2 * u) * BASIS_LD];
        bs[u] = sb[(size_t)(k + 2 * u) * BASIS_LD];
      }
#pragma unroll
      for (int u = 0; u < 16; u += 2) {
        const float a0 = frames[lo][k + 2 * u + hi], a1 = frames[lo][k + 2 * u + 2 + hi];
        re0 = mfma_f32(a0, bc[u], re0);
        im0 = mfma_f32(a0, bs[u], im0);
        re1 = mfma_f32(a1, bc[u + 1], re1);
        im1 = mfma_f32(a1, bs[u + 1], im1);
      }
    }
#pragma unroll
    for (int u = 0; u < (NFFT % 32) / 2; ++u) {
      const float a = frames[lo][k + 2 * u + hi];
      re0 = mfma_f32(a, cb[(size_t)(k + 2 * u) * BASIS_LD], re0);
      im0 = mfma_f32(a, sb[(size_t)(k + 2 * u) * BASIS_LD], im0);
    }
    // C layout: col = lane&31 (bin), row = (j&3) + 8*(j>>2) + 4*hi (frame)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int fr = (j & 3) + 8 * (j >> 2) + 4 * hi;
      const float r = re0[j] + re1[j], im = im0[j] + im1[j];
      if (bin < NBINS) power[fr][bin] = r * r + im * im;
    }
  }
  __syncthreads();

  // 3. mel projection: wave w -> mel tile w (32 mels), K = 202 (power col 201 = 0)
  float wmax = -FLT_MAX;
  if (wave * 32 < n_mels) {
    f16v acc0, acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) { acc0[j] = 0.f; acc1[j] = 0.f; }
    const int mel = wave * 32 + lo;
    const bool mv = mel < n_mels;
    const float* fr_ = filt + (size_t)(mv ? mel : 0) * NBINS;
#pragma unroll 2
    for (int k = 0; k < NBINS + 1; k += 4) {    // 202 = 50 x 4 + 2
      const float f0v = (mv && k + hi < NBINS) ? fr_[k + hi] : 0.f;
      const float f1v = (mv && k + 2 + hi < NBINS && k + 2 < NBINS + 1) ? fr_[k + 2 + hi] : 0.f;
      acc0 = mfma_f32(power[lo][k + hi], f0v, acc0);
      if (k + 2 < NBINS + 1) acc1 = mfma_f32(power[lo][k + 2 + hi], f1v, acc1);
    }
    if (mv) {
      float* orow = out + ((size_t)b * n_mels + mel) * n_frames;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int fr = f0 + (j & 3) + 8 * (j >> 2) + 4 * hi;
        if (fr < n_frames) {
          const float lv = log10f(fmaxf(acc0[j] + acc1[j], 1e-10f));
          orow[fr] = lv;
          wmax = fmaxf(wmax, lv);
        }
      }
    }
  }
  wmax = wave_max(wmax);
  if (lane == 0 && wmax > -FLT_MAX) atomic_max_float(gmax + b, wmax);
}

__global__ void fill_kernel(float* p, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// out_bf16[b, m, t] = (max(x, gmax[b] - 8) + 4) / 4
__global__ void logmel_finalize_kernel(const float* __restrict__ x, const float* __restrict__ gmax,
                                       bf16_t* __restrict__ y, long long per_b, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / per_b);
    const float v = fmaxf(x[i], gmax[b] - 8.f);
    y[i] = f2bf((v + 4.f) * 0.25f);
  }
}

extern "C" int loqa_log_mel(const float* audio, int B, int n_samples, const float* window,
                            const float* cosb, const float* sinb, const float* filt, int n_mels,
                            float* work, float* gmax, void* out_bf16, int n_frames,
                            hipStream_t s) {
  if (B <= 0) return 0;
  if (n_frames <= 0 || n_mels <= 0 || n_mels > 128 || n_samples <= NFFT / 2)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(fill_kernel, dim3((B + 255) / 256), dim3(256), 0, s, gmax, B, -FLT_MAX);
  dim3 grid((n_frames + FRAMES_PER_WG - 1) / FRAMES_PER_WG, B);
  hipLaunchKernelGGL(logmel_kernel, grid, dim3(512), 0, s, audio, n_samples, window, cosb, sinb,
                     filt, n_mels, work, n_frames, gmax);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const long long per_b = (long long)n_mels * n_frames, total = per_b * B;
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(logmel_finalize_kernel, dim3((unsigned)blocks), dim3(256), 0, s, work, gmax,
                     (bf16_t*)out_bf16, per_b, total);
  return (int)hipGetLastError();
}

// --------------------------------------------------------------------- im2col
// x element (b, c, t) at x[b*sb + c*sc + t*st]; cols[(b*Lout + to), c*3 + k] =
// x[b, c, to*stride + k - 1] (zero outside [0, L)).  Row-major [B*Lout, 3C].
__global__ void im2col_k3_kernel(const bf16_t* __restrict__ x, long long sb, long long sc,
                                 long long st, int C, int L, int Lout, int stride,
                                 bf16_t* __restrict__ cols, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / (3LL * C);
    const int col = (int)(i - row * 3LL * C);
    const int b = (int)(row / Lout), to = (int)(row - (long long)b * Lout);
    const int c = col / 3, k = col - c * 3;
    const int t = to * stride + k - 1;
    cols[i] = (t >= 0 && t < L) ? x[b * sb + c * sc + t * st] : (bf16_t)0;
  }
}

extern "C" int loqa_im2col_k3(const void* x, long long sb, long long sc, long long st, int B,
                              int C, int L, int stride, void* cols, hipStream_t s) {
  if (B <= 0) return 0;
  const int Lout = (L + 2 - 3) / stride + 1;
  const long long total = (long long)B * Lout * 3 * C;
  long long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(im2col_k3_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const bf16_t*)x,
                     sb, sc, st, C, L, Lout, stride, (bf16_t*)cols, total);
  return (int)hipGetLastError();
}
