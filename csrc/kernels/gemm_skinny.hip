// Decode-shaped GEMM: out^T[N, M] = W[N, K] * x^T[K, M] for M <= 128 tokens
// (SURVEY §2.4 "GEMM/GEMV for skinny M"; guide §5 table row "GEMV / M <= 16 decode
// weights": operand streamed once, straight to VGPRs, deep prefetch).
//
// Weight-streaming bound: every weight byte is read exactly once per decode
// step, so the kernel is shaped for HBM bandwidth, not MFMA rate:
//   * weights are PRE-SHUFFLED once at load time into MFMA fragment order
//     Wp[N/16][K/32][64 lanes][8]: lane l of v_mfma_f32_16x16x32_bf16 holds row
//     (l&15), k-offset 8*(l>>4). One wave load instruction is then 1 KiB
//     contiguous and a wave walks one contiguous 16-row x K stream - full-burst
//     DRAM access instead of 16 scattered 64-byte row segments;
//   * register ping-pong prefetch: the next UNROLL k-steps (UNROLL*RT KiB per
//     wave) are in flight while the current ones feed the MFMAs;
//   * workgroup = 4 waves splitting its (16*RT rows x K/S) item along K, LDS
//     reduce at the end; split-K S keeps >= 2 workgroups per CU; partial sums
//     go to f32 slabs part[S][Mpad][N] that the NEXT kernel sums in its prologue
//     (slab_ops.hip) - deterministic, no atomics, no extra launch.
#include "common.h"

typedef float float4v_ __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4v_ mfma16(const bf16x8& a, const bf16x8& b, const float4v_& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// streamed-once weights: non-temporal load
__device__ __forceinline__ bf16x8 ldw(const bf16_t* p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<bf16x8*>(&v);
}

__device__ __forceinline__ bf16x8 ldx(const bf16_t* p) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  return *reinterpret_cast<bf16x8*>(&v);
}

template <int RT, int MT, int U>
struct Frag {
  bf16x8 a[U][RT];
  bf16x8 b[U][MT];
};

template <int RT, int MT, int U>
__device__ __forceinline__ void load_frag(Frag<RT, MT, U>& f, const bf16_t* wp, size_t tile_stride,
                                          const bf16_t* xp, long long ldx_, int ks) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < RT; ++i) f.a[u][i] = ldw(wp + (size_t)i * tile_stride + (size_t)(ks + u) * 512);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < MT; ++j) f.b[u][j] = ldx(xp + (size_t)j * 16 * ldx_ + (size_t)(ks + u) * 32);
}

template <int RT, int MT, int U>
__device__ __forceinline__ void mma_frag(const Frag<RT, MT, U>& f, float4v_ (&acc)[RT][MT]) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int i = 0; i < RT; ++i) acc[i][j] = mfma16(f.a[u][i], f.b[u][j], acc[i][j]);
}

template <int RT, int MT, int U>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(const bf16_t* __restrict__ x, long long ldx_,
                                                          const bf16_t* __restrict__ Wp,
                                                          float* __restrict__ part, int N, int K,
                                                          int S, int Mpad) {
  __shared__ float4v_ red[3][RT * MT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile0 = blockIdx.x * RT;          // first 16-row tile
  const int s = blockIdx.y;
  const int KS = K >> 5;                      // k-steps of 32
  const int kw = KS / (S * 4);                // k-steps per wave
  const int ks0 = (s * 4 + wave) * kw;
  const size_t tile_stride = (size_t)KS * 512;  // elements per 16-row tile
  const bf16_t* wp = Wp + (size_t)tile0 * tile_stride + (size_t)lane * 8;
  const bf16_t* xp = x + (size_t)(lane & 15) * ldx_ + 8 * (lane >> 4);

  float4v_ acc[RT][MT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = (float4v_){0.f, 0.f, 0.f, 0.f};

  // ping-pong register prefetch over groups of U k-steps
  const int ng = kw / U;
  Frag<RT, MT, U> f0, f1;
  load_frag(f0, wp, tile_stride, xp, ldx_, ks0);
  int g = 0;
  for (; g + 2 <= ng; g += 2) {
    load_frag(f1, wp, tile_stride, xp, ldx_, ks0 + (g + 1) * U);
    mma_frag(f0, acc);
    if (g + 2 < ng) load_frag(f0, wp, tile_stride, xp, ldx_, ks0 + (g + 2) * U);
    mma_frag(f1, acc);
  }
  if (g < ng) mma_frag(f0, acc);

  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) red[wave - 1][i * MT + j][lane] = acc[i][j];
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        float4v_ v = acc[i][j] + red[0][i * MT + j][lane] + red[1][i * MT + j][lane] +
                     red[2][i * MT + j][lane];
        // C layout (16x16): col = lane&15 (token m), rows n = 4*(lane>>4) + reg
        const int m = j * 16 + (lane & 15);
        const int n = (tile0 + i) * 16 + 4 * (lane >> 4);
        *reinterpret_cast<float4v_*>(part + ((size_t)s * Mpad + m) * N + n) = v;
      }
  }
}

template <int RT, int MT>
static int launch_skinny(const void* x, long long ldx_, const void* Wp, float* part, int N, int K,
                         int S, int Mpad, hipStream_t st) {
  dim3 grid(N / (16 * RT), S);
  const int kw = K / 32 / (S * 4);
  if constexpr (MT <= 2) {
    if (kw % 4 == 0) {
      hipLaunchKernelGGL((skinny_gemm_kernel<RT, MT, 4>), grid, dim3(256), 0, st, (const bf16_t*)x,
                         ldx_, (const bf16_t*)Wp, part, N, K, S, Mpad);
      return (int)hipGetLastError();
    }
  }
  if (kw % 2 == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<RT, MT, 2>), grid, dim3(256), 0, st, (const bf16_t*)x,
                       ldx_, (const bf16_t*)Wp, part, N, K, S, Mpad);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<RT, MT, 1>), grid, dim3(256), 0, st, (const bf16_t*)x,
                       ldx_, (const bf16_t*)Wp, part, N, K, S, Mpad);
  return (int)hipGetLastError();
}

// x: [Mpad, >=K] bf16 (row stride ldx), rows >= M must be finite (zeros);
// Wp: pre-shuffled weight (loqa_shuffle_weight); part: [S, Mpad, N] f32.
extern "C" int loqa_skinny_gemm(const void* x, long long ldx_, const void* Wp, float* part, int Mpad,
                                int N, int K, int S, hipStream_t st) {
  if (S < 1 || K % (S * 4 * 32) != 0 || ldx_ % 8 != 0 || N % 16 != 0) return (int)hipErrorInvalidValue;
  switch (Mpad) {
    case 16:
      if (N % 32) return (int)hipErrorInvalidValue;
      return launch_skinny<2, 1>(x, ldx_, Wp, part, N, K, S, Mpad, st);
    case 32:
      if (N % 32) return (int)hipErrorInvalidValue;
      return launch_skinny<2, 2>(x, ldx_, Wp, part, N, K, S, Mpad, st);
    case 64:
      if (N % 64) return (int)hipErrorInvalidValue;
      return launch_skinny<4, 4>(x, ldx_, Wp, part, N, K, S, Mpad, st);
    case 128:
      if (N % 64) return (int)hipErrorInvalidValue;
      return launch_skinny<4, 8>(x, ldx_, Wp, part, N, K, S, Mpad, st);
    default:
      return (int)hipErrorInvalidValue;
  }
}

// W [N, K] row-major -> Wp[N/16][K/32][64][8] (fragment order of the kernel above)
__global__ void shuffle_weight_kernel(const bf16_t* __restrict__ W, bf16_t* __restrict__ Wp, int N,
                                      int K, long long total_vec) {
  const int KS = K >> 5;
  for (long long v = blockIdx.x * (long long)blockDim.x + threadIdx.x; v < total_vec;
       v += (long long)gridDim.x * blockDim.x) {
    // destination vector v -> (tile, ks, lane)
    const int lane = (int)(v & 63);
    const long long tk = v >> 6;
    const int ks = (int)(tk % KS);
    const long long t = tk / KS;
    const long long row = t * 16 + (lane & 15);
    const int k = ks * 32 + 8 * (lane >> 4);
    *reinterpret_cast<uint4*>(Wp + v * 8) = *reinterpret_cast<const uint4*>(W + row * K + k);
  }
}

extern "C" int loqa_shuffle_weight(const void* W, void* Wp, int N, int K, hipStream_t st) {
  if (N % 16 || K % 32) return (int)hipErrorInvalidValue;
  const long long tv = (long long)N * K / 8;
  long long blocks = (tv + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(shuffle_weight_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const bf16_t*)W, (bf16_t*)Wp, N, K, tv);
  return (int)hipGetLastError();
}
