// Decode-shaped GEMM: out^T[N, M] = W[N, K] * x^T[K, M] for M <= 128 tokens
// (SURVEY §2.4 "GEMM/GEMV for skinny M"; guide §5 table row "GEMV / M <= 16 decode
// weights": operand streamed once, straight to VGPRs, deep unroll).
//
// Weight-streaming bound: every weight byte is read exactly once per step, so
// the kernel is shaped for HBM bandwidth, not MFMA rate:
//   * workgroup = 4 waves over a (16*RT rows of W) x (K/S chunk) item; the 4
//     waves split the chunk along K and reduce through LDS once at the end;
//   * each lane streams 16-byte rows segments of W (the MFMA A fragment of
//     v_mfma_f32_16x16x32_bf16 is 8 contiguous k of one row) with a 4-deep
//     unrolled k loop so each row is fetched in 256-byte bursts;
//   * x (tiny, L2 resident) supplies the B fragment (token on the lane);
//   * split-K (S) is chosen so the grid has >= 2 workgroups per CU; partial
//     results go to f32 slabs part[S][Mpad][N] that the NEXT kernel (rmsnorm /
//     rope+KV-append / SwiGLU, slab_ops.hip) sums in its prologue - a
//     deterministic launch-boundary reduction (guide §5 item 2), no atomics.
#include "common.h"

typedef float float4v_ __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4v_ mfma16(const bf16x8& a, const bf16x8& b, const float4v_& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// streamed-once weights: non-temporal load (guide megakernel row "nt-weights")
__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<bf16x8*>(&v);
}

__device__ __forceinline__ bf16x8 ld16c(const bf16_t* p) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  return *reinterpret_cast<bf16x8*>(&v);
}

template <int RT, int MT, int UNROLL>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                          const bf16_t* __restrict__ W,
                                                          float* __restrict__ part, int N, int K,
                                                          int kchunk, int Mpad) {
  __shared__ float4v_ red[3][RT * MT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * (16 * RT);
  const int s = blockIdx.y;
  const int kw = kchunk >> 2;
  const int kbeg = s * kchunk + wave * kw;
  const int kend = kbeg + kw;
  const int r = lane & 15, kq = 8 * (lane >> 4);
  const bf16_t* ap = W + (size_t)(n0 + r) * K + kq;
  const bf16_t* bp = x + (size_t)r * ldx + kq;

  float4v_ acc[RT][MT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = (float4v_){0.f, 0.f, 0.f, 0.f};

  // UNROLL k-steps of loads are issued back to back before any MFMA consumes
  // them: UNROLL*RT 16-byte weight loads in flight per lane.
  for (int k = kbeg; k < kend; k += 32 * UNROLL) {
    bf16x8 a[UNROLL][RT], b[UNROLL][MT];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int i = 0; i < RT; ++i) a[u][i] = ld16(ap + (size_t)i * 16 * K + k + 32 * u);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int j = 0; j < MT; ++j) b[u][j] = ld16c(bp + (size_t)j * 16 * ldx + k + 32 * u);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int j = 0; j < MT; ++j)
#pragma unroll
        for (int i = 0; i < RT; ++i) acc[i][j] = mfma16(a[u][i], b[u][j], acc[i][j]);
  }
  // cross-wave reduction: waves 1..3 park their accumulators in LDS
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
        const int n = n0 + i * 16 + 4 * (lane >> 4);
        *reinterpret_cast<float4v_*>(part + ((size_t)s * Mpad + m) * N + n) = v;
      }
  }
}

template <int RT, int MT>
static int launch_skinny(const void* x, long long ldx, const void* W, float* part, int N, int K,
                         int S, int Mpad, hipStream_t st) {
  dim3 grid(N / (16 * RT), S);
  const int kw = K / S / 4;
  if (MT <= 2 && kw % 128 == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<RT, MT, 4>), grid, dim3(256), 0, st, (const bf16_t*)x,
                       ldx, (const bf16_t*)W, part, N, K, K / S, Mpad);
  else if (kw % 64 == 0)
    hipLaunchKernelGGL((skinny_gemm_kernel<RT, MT, 2>), grid, dim3(256), 0, st, (const bf16_t*)x,
                       ldx, (const bf16_t*)W, part, N, K, K / S, Mpad);
  else
    hipLaunchKernelGGL((skinny_gemm_kernel<RT, MT, 1>), grid, dim3(256), 0, st, (const bf16_t*)x,
                       ldx, (const bf16_t*)W, part, N, K, K / S, Mpad);
  return (int)hipGetLastError();
}

// x: [Mpad, >=K] bf16 (row stride ldx), rows >= M must be finite (zeros);
// W: [N, K] bf16; part: [S, Mpad, N] f32. Mpad in {16, 32, 64, 128}.
extern "C" int loqa_skinny_gemm(const void* x, long long ldx, const void* W, float* part, int Mpad,
                                int N, int K, int S, hipStream_t st) {
  if (S < 1 || K % (S * 4 * 32) != 0 || ldx % 8 != 0 || K % 8 != 0) return (int)hipErrorInvalidValue;
  switch (Mpad) {
    case 16:
      if (N % 32) return (int)hipErrorInvalidValue;
      return launch_skinny<2, 1>(x, ldx, W, part, N, K, S, Mpad, st);
    case 32:
      if (N % 32) return (int)hipErrorInvalidValue;
      return launch_skinny<2, 2>(x, ldx, W, part, N, K, S, Mpad, st);
    case 64:
      if (N % 64) return (int)hipErrorInvalidValue;
      return launch_skinny<4, 4>(x, ldx, W, part, N, K, S, Mpad, st);
    case 128:
      if (N % 64) return (int)hipErrorInvalidValue;
      return launch_skinny<4, 8>(x, ldx, W, part, N, K, S, Mpad, st);
    default:
      return (int)hipErrorInvalidValue;
  }
}
