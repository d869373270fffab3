// Prefill-shaped GEMM (M ~ 64 - a few thousand token rows): Y = X W^T for the
// Llama prompt projections and the Whisper encoder (SURVEY §2.4 N2 / N4;
// PERF.md "Round 3").
//
// At M ~ 318 hipBLASLt's tiles cover too few CUs for the N = 4096 projections
// (o, down) and its large-N tiles re-read weights. Here the weights are
// streamed exactly once, in the MFMA-fragment order of ops.shuffle_weight (the
// decode copies: 1 KiB contiguous per wave load), and the activation rows stay
// on chip (v_mfma_f32_16x16x32_bf16, A = weights, B = rows). Output: bf16 Y,
// f32 split-K slabs [S, M, N] that the consumer (slab_rmsnorm /
// slab_layernorm / slab_rope_append) sums in a fixed order, or SwiGLU.
// (The round-2 version of this kernel - 4 waves along N, 128-deep chunks, two
// barriers per chunk - is superseded by layout 3 below: faster on every shape.)
#include "common.h"

typedef unsigned u32x4p __attribute__((ext_vector_type(4)));
typedef float f4p __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4p pg_ldw(const bf16_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4p*>(p));
}

// ---------------------------------------------------------------------------
// Workgroup = 4 waves as WM (rows) x 4 / WM (features); a wave owns RBW row
// tiles x FT feature tiles of 16. Per 64-deep K chunk the workgroup's
// activation block is staged once in LDS (padded rows, double-buffered, ONE
// barrier per chunk: the next chunk's rows and this wave's weight fragments
// are in flight in registers while this chunk's MFMAs run); each wave streams
// its own weight fragments straight into VGPRs. Rows past M are read clamped
// (their outputs are never stored), so every load is unconditional and hipcc
// keeps its counted waits (a predicated load drains the prefetch).
// Measured (profiles/r3_prefill_gemm2_layouts.txt): the 1 x 4 layout (3) is the
// fastest on every prefill / encoder shape - in the 2 x 2 layouts each weight
// fragment is fetched by two waves, which costs more than the better LDS
// fragment reuse saves.
// Epilogues: bf16 Y; f32 split-K slabs; SwiGLU over perm_gate_up pair tiles
// (lanes l < 32 hold gate rows, l ^ 32 their up partners) -> bf16 [M, N / 2].
#define PG2_KC 64

// XP: LDS row length in elements. 64 + 16 (160-B rows = 40 dwords): the
// fragment reads (ds_read_b128, lane l: row l & 15, 16-B piece l >> 4, banks
// (a/4) % 64 over the 16-lane groups of MI355X_MICROARCH.md §LDS) and the
// 8-lane-contiguous chunk stores are both conflict-free. The earlier 144-B
// rows (64 + 8) read 2-way (SQ_LDS_BANK_CONFLICT 0.65 extra cycles per cycle);
// measured 0-2% faster (down S8 49.3 -> 48.7 us, S4 63.7 -> 62.4 us at M = 318).
#define PG2_XP (PG2_KC + 16)
template <int WM, int RBW, int FT, int EPI, int XP>
__global__ __launch_bounds__(256, (RBW * FT <= 20 ? 2 : 1)) void gemm_prefill2_kernel(
    const bf16_t* __restrict__ X, int M, int K, const bf16_t* __restrict__ Wp, int N, int S,
    bf16_t* __restrict__ Y, float* __restrict__ part) {
  constexpr int WN = 4 / WM;
  constexpr int BM = WM * RBW * 16, BN = WN * FT * 16;
  constexpr int XPT = BM * (PG2_KC / 8) / 256;          // 16-byte activation pieces per thread
  static_assert(XPT * 256 == BM * (PG2_KC / 8), "row block must tile the workgroup");
  __shared__ __attribute__((aligned(16))) bf16_t xs[2][BM][XP];
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

template <int WM, int RBW, int FT, int XP = PG2_XP>
static int launch_prefill2(const void* X, int M, int K, const void* Wp, int N, int S, void* Y,
                           float* part, int epi, hipStream_t st) {
  constexpr int BM = WM * RBW * 16, BN = (4 / WM) * FT * 16;
  if (N % BN || K % (S * PG2_KC)) return (int)hipErrorInvalidValue;
  const int grid = ((M + BM - 1) / BM) * (N / BN) * S;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, (const bf16_t*)X, M, K, (const bf16_t*)Wp,
                       N, S, (bf16_t*)Y, part);
  };
  if (epi == 1) args(gemm_prefill2_kernel<WM, RBW, FT, 1, XP>);
  else if (epi == 2) args(gemm_prefill2_kernel<WM, RBW, FT, 2, XP>);
  else args(gemm_prefill2_kernel<WM, RBW, FT, 0, XP>);
  return (int)hipGetLastError();
}

// v2 entry: layout = 0 (2 x 2 waves of 5 row tiles x 4 feature tiles: 160 x 128
// workgroup tile), 1 (2 x 2 of 10 x 4: 320 x 128), 2 (2 x 2 of 5 x 2: 160 x 64),
// 3 (1 x 4 waves of 10 x 2: 160 x 128, v1's layout), 4 (1 x 4 of 10 x 4: 160 x 256).
// (A v3 staging the weights through LDS as well - no duplicate fragment loads
// in the 2 x 2 layouts - measured slower than layout 3 on every shape and was
// dropped: profiles/r3_prefill_gemm3_layouts.txt.)
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
    default: return (int)hipErrorInvalidValue;
  }
}
