// Prefill-shaped GEMM (M ~ 100-512 token rows): Y = X W^T for the Llama
// projections at one parser prompt (PERF.md "prefill GEMMs").
//
// At M ~ 318 hipBLASLt's tiles cover too few CUs for the N = 4096 projections
// (o, down) and its large-N tiles re-read weights; both run at 30-50% of the
// HBM / MFMA roofline. Here the weights are streamed exactly once, in the
// MFMA-fragment order of ops.shuffle_weight (the decode copies: 1 KiB contiguous
// per wave load), and the activation rows stay on chip:
//   workgroup = 4 waves x FT feature tiles of 16 (128 features) x RB row tiles
//               of 16 (160 rows) x one K range (split-K S);
//   per K chunk of 128: the 160 x 128 activation block is staged once in LDS
//   (register double-buffered: the next chunk's rows and weight fragments are
//   in flight while this chunk's MFMAs run), every wave multiplies its
//   weight fragments against all RB row tiles (v_mfma_f32_16x16x32_bf16, A =
//   weights, B = rows, each LDS fragment feeds FT MFMAs).
// Output: bf16 Y [M, N], or f32 split-K slabs [S, M, N] that the consumer
// (slab_rmsnorm / slab_rope_append) sums in a fixed order.
#include "common.h"

#define PG_FT 2            // feature tiles per wave
#define PG_RB 10           // row tiles per workgroup
#define PG_KC 128          // K per LDS chunk (4 k-steps)
#define PG_PAD 8

typedef unsigned u32x4p __attribute__((ext_vector_type(4)));
typedef float f4p __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4p pg_ldw(const bf16_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4p*>(p));
}

__global__ __launch_bounds__(256, 2) void gemm_prefill_kernel(
    const bf16_t* __restrict__ X, int M, int K, const bf16_t* __restrict__ Wp, int N, int S,
    bf16_t* __restrict__ Y, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) bf16_t xs[PG_RB * 16][PG_KC + PG_PAD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int NT = 4 * PG_FT * 16;                 // features per workgroup
  const int nslices = N / NT;
  // XCD-aware order: the row blocks of one feature slice run back to back on
  // the same XCD, so the second reads the weights from L2
  const int mblocks = (M + PG_RB * 16 - 1) / (PG_RB * 16);
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int mb = wg % mblocks;
  const int rest = wg / mblocks;
  const int slice = rest % nslices;
  const int s = rest / nslices;
  if (s >= S) return;
  const int KS = K >> 5;
  const int Ks = K / S;                          // multiple of PG_KC (host-checked)
  const int k0 = s * Ks;
  const int m0 = mb * PG_RB * 16;
  const int nchunks = Ks / PG_KC;
  const int tile0 = slice * (NT / 16) + wave * PG_FT;

  // activation staging: 160 rows x 128 k = 2560 16-byte pieces, 10 per thread
  u32x4p xr[10];
  auto load_x = [&](int kc) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int row = c >> 4, col = (c & 15) * 8;
      const int m = m0 + row;
      xr[i] = m < M ? *reinterpret_cast<const u32x4p*>(X + (size_t)m * K + kc + col) : u32x4p{0, 0, 0, 0};
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int row = c >> 4, col = (c & 15) * 8;
      *reinterpret_cast<u32x4p*>(&xs[row][col]) = xr[i];
    }
  };
  // weight fragments of one chunk: FT tiles x 4 k-steps
  u32x4p wf[PG_FT][4], wn[PG_FT][4];
  auto load_w = [&](int kc, u32x4p (&w)[PG_FT][4]) {
    const int ks0 = kc >> 5;
#pragma unroll
    for (int f = 0; f < PG_FT; ++f)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        w[f][u] = pg_ldw(Wp + ((size_t)(tile0 + f) * KS + ks0 + u) * 512 + lane * 8);
  };
  f4p acc[PG_RB][PG_FT];
#pragma unroll
  for (int r = 0; r < PG_RB; ++r)
#pragma unroll
    for (int f = 0; f < PG_FT; ++f) acc[r][f] = f4p{0.f, 0.f, 0.f, 0.f};

  load_w(k0, wf);
  load_x(k0);
  store_x();
  __syncthreads();
  const int t = lane & 15, kq = 8 * (lane >> 4);
  for (int c = 0; c < nchunks; ++c) {
    const int kc = k0 + c * PG_KC;
    const bool more = c + 1 < nchunks;
    const int kn = more ? kc + PG_KC : kc;      // clamped: unconditional loads
    load_x(kn);
    load_w(kn, wn);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int r = 0; r < PG_RB; ++r) {
        const u32x4p b = *reinterpret_cast<const u32x4p*>(&xs[r * 16 + t][u * 32 + kq]);
#pragma unroll
        for (int f = 0; f < PG_FT; ++f)
          acc[r][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[f][u]),
                                                              __builtin_bit_cast(bf16x8, b), acc[r][f], 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) store_x();
#pragma unroll
    for (int f = 0; f < PG_FT; ++f)
#pragma unroll
      for (int u = 0; u < 4; ++u) wf[f][u] = wn[f][u];
    __syncthreads();
  }
  // epilogue: lane holds features (lane>>4)*4 + j of tile, token lane & 15
#pragma unroll
  for (int r = 0; r < PG_RB; ++r) {
    const int m = m0 + r * 16 + t;
    if (m >= M) continue;
#pragma unroll
    for (int f = 0; f < PG_FT; ++f) {
      const int n = (tile0 + f) * 16 + (lane >> 4) * 4;
      if (part) {
        *reinterpret_cast<f4p*>(part + ((size_t)s * M + m) * N + n) = acc[r][f];
      } else {
        *reinterpret_cast<uint2*>(Y + (size_t)m * N + n) =
            make_uint2(pack_bf16x2(acc[r][f][0], acc[r][f][1]), pack_bf16x2(acc[r][f][2], acc[r][f][3]));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// v2: 2 x 2 waves per workgroup. The v1 layout (4 waves along N, 2 feature
// tiles each) feeds every LDS activation fragment to only 2 MFMAs, so at
// 160 rows its k-loop moves ~125 B/clk/CU of LDS reads plus the staging writes
// and stalls on LDS, not on the MFMA pipe. Here a wave owns RBW row tiles x FT
// feature tiles (FT = 4: each LDS fragment feeds 4 MFMAs, each weight fragment
// RBW), the two row-halves of a workgroup share the weight fragments through
// L1, and the activation block is double-buffered in LDS with ONE barrier per
// 64-deep K chunk (the next chunk's rows and weights are in flight in
// registers while this chunk's MFMAs run). Rows past M are read clamped (their
// outputs are never stored), so every load is unconditional and hipcc keeps
// its counted waits (a predicated load drains the prefetch).
// Epilogues: bf16 Y; f32 split-K slabs; SwiGLU over perm_gate_up pair tiles
// (lanes l < 32 hold gate rows, l ^ 32 their up partners) -> bf16 [M, N / 2].
#define PG2_KC 64
#define PG2_XP (PG2_KC + 8)

template <int WM, int RBW, int FT, int EPI>
__global__ __launch_bounds__(256, (RBW * FT <= 20 ? 2 : 1)) void gemm_prefill2_kernel(
    const bf16_t* __restrict__ X, int M, int K, const bf16_t* __restrict__ Wp, int N, int S,
    bf16_t* __restrict__ Y, float* __restrict__ part) {
  constexpr int WN = 4 / WM;
  constexpr int BM = WM * RBW * 16, BN = WN * FT * 16;
  constexpr int XPT = BM * (PG2_KC / 8) / 256;          // 16-byte activation pieces per thread
  static_assert(XPT * 256 == BM * (PG2_KC / 8), "row block must tile the workgroup");
  __shared__ __attribute__((aligned(16))) bf16_t xs[2][BM][PG2_XP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nslices = N / BN;
  const int mblocks = (M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int mb = wg % mblocks;
  const int rest = wg / mblocks;
  const int slice = rest % nslices;
  const int s = rest / nslices;
  if (s >= S) return;
  const int KS = K >> 5;
  const int Ks = K / S;
  const int k0 = s * Ks;
  const int m0 = mb * BM;
  const int nch = Ks / PG2_KC;
  const int tile0 = slice * (BN / 16) + wn * FT;

  u32x4p xr[XPT];
  auto load_x = [&](int kc) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int row = c >> 3, col = (c & 7) * 8;
      const int m = min(m0 + row, M - 1);
      xr[i] = *reinterpret_cast<const u32x4p*>(X + (size_t)m * K + kc + col);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int row = c >> 3, col = (c & 7) * 8;
      *reinterpret_cast<u32x4p*>(&xs[buf][row][col]) = xr[i];
    }
  };
  u32x4p wf[FT][2], wn2[FT][2];
  auto load_w = [&](int kc, u32x4p (&w)[FT][2]) {
    const int ks0 = kc >> 5;
#pragma unroll
    for (int f = 0; f < FT; ++f)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        w[f][u] = pg_ldw(Wp + ((size_t)(tile0 + f) * KS + ks0 + u) * 512 + lane * 8);
  };
  f4p acc[RBW][FT];
#pragma unroll
  for (int r = 0; r < RBW; ++r)
#pragma unroll
    for (int f = 0; f < FT; ++f) acc[r][f] = f4p{0.f, 0.f, 0.f, 0.f};

  load_w(k0, wf);
  load_x(k0);
  store_x(0);
  __syncthreads();
  const int t = lane & 15, kq = 8 * (lane >> 4);
  const int rw0 = wm * RBW * 16;
  for (int c = 0; c < nch; ++c) {
    const int kc = k0 + c * PG2_KC;
    const bool more = c + 1 < nch;
    const int kn = more ? kc + PG2_KC : kc;       // clamped: unconditional loads
    load_x(kn);
    load_w(kn, wn2);
    const int buf = c & 1;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int r = 0; r < RBW; ++r) {
        const u32x4p b = *reinterpret_cast<const u32x4p*>(&xs[buf][rw0 + r * 16 + t][u * 32 + kq]);
#pragma unroll
        for (int f = 0; f < FT; ++f)
          acc[r][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[f][u]),
                                                              __builtin_bit_cast(bf16x8, b), acc[r][f], 0, 0, 0);
      }
    }
    // the other buffer was last read in the previous chunk, before the
    // barrier that ended it
    store_x(buf ^ 1);
#pragma unroll
    for (int f = 0; f < FT; ++f)
#pragma unroll
      for (int u = 0; u < 2; ++u) wf[f][u] = wn2[f][u];
    __syncthreads();
  }
  // epilogue: lane holds features (lane >> 4) * 4 + j of its tile, row lane & 15
#pragma unroll
  for (int r = 0; r < RBW; ++r) {
    const int m = m0 + rw0 + r * 16 + t;
    if (m >= M) continue;
#pragma unroll
    for (int f = 0; f < FT; ++f) {
      if constexpr (EPI == 2) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float own = bf2f(f2bf(acc[r][f][j]));
          const float oth = __shfl_xor(own, 32, 64);
          o[j] = own / (1.f + __expf(-own)) * oth;
        }
        if (lane < 32)
          *reinterpret_cast<uint2*>(Y + (size_t)m * (N >> 1) + (tile0 + f) * 8 + (lane >> 4) * 4) =
              make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
      } else {
        const int n = (tile0 + f) * 16 + (lane >> 4) * 4;
        if constexpr (EPI == 1) {
          *reinterpret_cast<f4p*>(part + ((size_t)s * M + m) * N + n) = acc[r][f];
        } else {
          *reinterpret_cast<uint2*>(Y + (size_t)m * N + n) =
              make_uint2(pack_bf16x2(acc[r][f][0], acc[r][f][1]), pack_bf16x2(acc[r][f][2], acc[r][f][3]));
        }
      }
    }
  }
}

template <int WM, int RBW, int FT>
static int launch_prefill2(const void* X, int M, int K, const void* Wp, int N, int S, void* Y,
                           float* part, int epi, hipStream_t st) {
  constexpr int BM = WM * RBW * 16, BN = (4 / WM) * FT * 16;
  if (N % BN || K % (S * PG2_KC)) return (int)hipErrorInvalidValue;
  const int grid = ((M + BM - 1) / BM) * (N / BN) * S;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, (const bf16_t*)X, M, K, (const bf16_t*)Wp,
                       N, S, (bf16_t*)Y, part);
  };
  if (epi == 1) args(gemm_prefill2_kernel<WM, RBW, FT, 1>);
  else if (epi == 2) args(gemm_prefill2_kernel<WM, RBW, FT, 2>);
  else args(gemm_prefill2_kernel<WM, RBW, FT, 0>);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// v3: 2 x 2 waves with BOTH operands staged through LDS. v2's 2 x 2 layouts
// load every weight fragment twice (once per row-half wave) straight into
// VGPRs, and its 1 x 4 layout feeds each LDS activation fragment to only 2
// MFMAs; here the workgroup stages its (BN / 16) x 2 weight fragments of a
// 64-deep K chunk once (fragment order: 1 KiB contiguous per fragment, read
// back with lane-linear ds_read_b128 - no bank conflicts) next to the padded
// activation block, so a wave's activation fragment feeds FT MFMAs and its
// weight fragment RBW MFMAs with no duplicate global loads. Same one-barrier
// double-buffered pipeline and epilogues as v2.
template <int RBW, int FT, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_prefill3_kernel(
    const bf16_t* __restrict__ X, int M, int K, const bf16_t* __restrict__ Wp, int N, int S,
    bf16_t* __restrict__ Y, float* __restrict__ part) {
  constexpr int BM = 2 * RBW * 16, BN = 2 * FT * 16, NT = BN / 16;
  constexpr int XPT = BM * (PG2_KC / 8) / 256;           // 16-byte activation pieces per thread
  constexpr int WPT = NT * 2 * 64 / 256;                 // 16-byte weight pieces per thread
  static_assert(XPT * 256 == BM * (PG2_KC / 8) && WPT * 256 == NT * 2 * 64, "tiling");
  // ONE shared array (a second __shared__ object can make hipcc drain loads
  // before every LDS read): [2][BM][XP] activations, then [2][NT][2][512] weights
  __shared__ __attribute__((aligned(16))) bf16_t sm[2 * BM * PG2_XP + 2 * NT * 2 * 512];
  bf16_t* const xs0 = sm;
  bf16_t* const ws0 = sm + 2 * BM * PG2_XP;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nslices = N / BN;
  const int mblocks = (M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int mb = wg % mblocks;
  const int rest = wg / mblocks;
  const int slice = rest % nslices;
  const int s = rest / nslices;
  if (s >= S) return;
  const int KS = K >> 5;
  const int Ks = K / S;
  const int k0 = s * Ks;
  const int m0 = mb * BM;
  const int nch = Ks / PG2_KC;
  const int tile_base = slice * NT;

  u32x4p xr[XPT], wr[WPT];
  auto load = [&](int kc) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int row = c >> 3, col = (c & 7) * 8;
      const int m = min(m0 + row, M - 1);
      xr[i] = *reinterpret_cast<const u32x4p*>(X + (size_t)m * K + kc + col);
    }
    const int ks0 = kc >> 5;
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int c = threadIdx.x + 256 * i;          // (tile, kstep, lane) piece
      const int t = c >> 7, u = (c >> 6) & 1, l = c & 63;
      wr[i] = pg_ldw(Wp + ((size_t)(tile_base + t) * KS + ks0 + u) * 512 + l * 8);
    }
  };
  auto store = [&](int buf) {
    bf16_t* xs = xs0 + buf * BM * PG2_XP;
    bf16_t* ws = ws0 + buf * NT * 2 * 512;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int row = c >> 3, col = (c & 7) * 8;
      *reinterpret_cast<u32x4p*>(xs + row * PG2_XP + col) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int c = threadIdx.x + 256 * i;
      *reinterpret_cast<u32x4p*>(ws + c * 8) = wr[i];
    }
  };
  f4p acc[RBW][FT];
#pragma unroll
  for (int r = 0; r < RBW; ++r)
#pragma unroll
    for (int f = 0; f < FT; ++f) acc[r][f] = f4p{0.f, 0.f, 0.f, 0.f};

  load(k0);
  store(0);
  __syncthreads();
  const int t = lane & 15, kq = 8 * (lane >> 4);
  const int rw0 = wm * RBW * 16;
  for (int c = 0; c < nch; ++c) {
    const int kc = k0 + c * PG2_KC;
    const int kn = c + 1 < nch ? kc + PG2_KC : kc;   // clamped: unconditional loads
    load(kn);
    const int buf = c & 1;
    const bf16_t* xs = xs0 + buf * BM * PG2_XP;
    const bf16_t* ws = ws0 + buf * NT * 2 * 512;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      u32x4p wf[FT];
#pragma unroll
      for (int f = 0; f < FT; ++f)
        wf[f] = *reinterpret_cast<const u32x4p*>(ws + ((wn * FT + f) * 2 + u) * 512 + lane * 8);
#pragma unroll
      for (int r = 0; r < RBW; ++r) {
        const u32x4p b = *reinterpret_cast<const u32x4p*>(xs + (rw0 + r * 16 + t) * PG2_XP + u * 32 + kq);
#pragma unroll
        for (int f = 0; f < FT; ++f)
          acc[r][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[f]),
                                                              __builtin_bit_cast(bf16x8, b), acc[r][f], 0, 0, 0);
      }
    }
    store(buf ^ 1);      // the other buffer's last readers passed the previous barrier
    __syncthreads();
  }
  const int tile0 = tile_base + wn * FT;
#pragma unroll
  for (int r = 0; r < RBW; ++r) {
    const int m = m0 + rw0 + r * 16 + t;
    if (m >= M) continue;
#pragma unroll
    for (int f = 0; f < FT; ++f) {
      if constexpr (EPI == 2) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float own = bf2f(f2bf(acc[r][f][j]));
          const float oth = __shfl_xor(own, 32, 64);
          o[j] = own / (1.f + __expf(-own)) * oth;
        }
        if (lane < 32)
          *reinterpret_cast<uint2*>(Y + (size_t)m * (N >> 1) + (tile0 + f) * 8 + (lane >> 4) * 4) =
              make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
      } else {
        const int n = (tile0 + f) * 16 + (lane >> 4) * 4;
        if constexpr (EPI == 1) {
          *reinterpret_cast<f4p*>(part + ((size_t)s * M + m) * N + n) = acc[r][f];
        } else {
          *reinterpret_cast<uint2*>(Y + (size_t)m * N + n) =
              make_uint2(pack_bf16x2(acc[r][f][0], acc[r][f][1]), pack_bf16x2(acc[r][f][2], acc[r][f][3]));
        }
      }
    }
  }
}

template <int RBW, int FT>
static int launch_prefill3(const void* X, int M, int K, const void* Wp, int N, int S, void* Y,
                           float* part, int epi, hipStream_t st) {
  constexpr int BM = 2 * RBW * 16, BN = 2 * FT * 16;
  if (N % BN || K % (S * PG2_KC)) return (int)hipErrorInvalidValue;
  const int grid = ((M + BM - 1) / BM) * (N / BN) * S;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, (const bf16_t*)X, M, K, (const bf16_t*)Wp,
                       N, S, (bf16_t*)Y, part);
  };
  if (epi == 1) args(gemm_prefill3_kernel<RBW, FT, 1>);
  else if (epi == 2) args(gemm_prefill3_kernel<RBW, FT, 2>);
  else args(gemm_prefill3_kernel<RBW, FT, 0>);
  return (int)hipGetLastError();
}

// v2 entry: layout = 0 (2 x 2 waves of 5 row tiles x 4 feature tiles: 160 x 128
// workgroup tile), 1 (2 x 2 of 10 x 4: 320 x 128), 2 (2 x 2 of 5 x 2: 160 x 64),
// 3 (1 x 4 waves of 10 x 2: 160 x 128, v1's layout), 4 (1 x 4 of 10 x 4: 160 x 256);
// v3 (both operands through LDS, 2 x 2 waves): 5 (5 x 4: 160 x 128), 6 (5 x 8:
// 160 x 256), 7 (10 x 4: 320 x 128).
// epi 0: Y bf16 [M, N] (S = 1); 1: f32 slabs part [S, M, N]; 2: SwiGLU of
// perm_gate_up pair tiles, Y bf16 [M, N / 2] (S = 1).
extern "C" int loqa_gemm_prefill2(const void* X, int M, int K, const void* Wp, int N, int S, void* Y,
                                  float* part, int epi, int layout, hipStream_t st) {
  if (M <= 0 || S < 1 || epi < 0 || epi > 2 || (epi != 1 && S != 1) || (epi == 1 && !part) ||
      (epi != 1 && !Y))
    return (int)hipErrorInvalidValue;
  switch (layout) {
    case 0: return launch_prefill2<2, 5, 4>(X, M, K, Wp, N, S, Y, part, epi, st);
    case 1: return launch_prefill2<2, 10, 4>(X, M, K, Wp, N, S, Y, part, epi, st);
    case 2: return launch_prefill2<2, 5, 2>(X, M, K, Wp, N, S, Y, part, epi, st);
    case 3: return launch_prefill2<1, 10, 2>(X, M, K, Wp, N, S, Y, part, epi, st);
    case 4: return launch_prefill2<1, 10, 4>(X, M, K, Wp, N, S, Y, part, epi, st);
    case 5: return launch_prefill3<5, 4>(X, M, K, Wp, N, S, Y, part, epi, st);
    case 6: return launch_prefill3<5, 8>(X, M, K, Wp, N, S, Y, part, epi, st);
    case 7: return launch_prefill3<10, 4>(X, M, K, Wp, N, S, Y, part, epi, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// X [M, K] bf16 row-major; Wp = shuffle_weight(W [N, K]); S split-K ranges.
// part != nullptr: f32 slabs [S, M, N]; else Y [M, N] bf16 (S must be 1).
extern "C" int loqa_gemm_prefill(const void* X, int M, int K, const void* Wp, int N, int S, void* Y,
                                 float* part, hipStream_t st) {
  const int NT = 4 * PG_FT * 16;
  if (M <= 0 || N % NT || S < 1 || K % (S * PG_KC) || (!part && S != 1) || (!part && !Y))
    return (int)hipErrorInvalidValue;
  const int mblocks = (M + PG_RB * 16 - 1) / (PG_RB * 16);
  const int grid = mblocks * (N / NT) * S;
  hipLaunchKernelGGL(gemm_prefill_kernel, dim3(grid), dim3(256), 0, st, (const bf16_t*)X, M, K,
                     (const bf16_t*)Wp, N, S, (bf16_t*)Y, part);
  return (int)hipGetLastError();
}
