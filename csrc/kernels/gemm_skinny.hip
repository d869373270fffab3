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
#include "attn_decode.h"
#include "car_common.h"
#include <stdlib.h>

// launch priority of the calling host thread (attn_decode.hip)
extern thread_local int g_loqa_launch_prio;

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

// Source of the activation fragments: plain loads, or (XS = 1) sc1 buffer
// loads - x was stored write-through by a prologue item of the SAME launch
// (guide §6 Guideline 16: every handed-off byte read with sc1, no acquire)
struct XSrc {
  const bf16_t* x0;                 // x base (offsets are taken from it)
  __amdgpu_buffer_rsrc_t r;
};

template <int XS>
__device__ __forceinline__ bf16x8 ldx_s(const bf16_t* p, const XSrc& xs) {
  if constexpr (XS) {
    const u32x4 v = __builtin_bit_cast(
        u32x4, __builtin_amdgcn_raw_buffer_load_b128(xs.r, (unsigned)((p - xs.x0) * 2), 0, 16));
    return __builtin_bit_cast(bf16x8, v);
  } else {
    return ldx(p);
  }
}

// workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not
// for its outstanding global loads (__syncthreads' release fence would drain
// the weight prefetch)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int RT, int MT, int U>
struct Frag {
  bf16x8 a[U][RT];
  bf16x8 b[U][MT];
};

template <int RT, int MT, int U>
__device__ __forceinline__ void load_frag_w(Frag<RT, MT, U>& f, const bf16_t* wp, size_t tile_stride, int ks) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < RT; ++i) f.a[u][i] = ldw(wp + (size_t)i * tile_stride + (size_t)(ks + u) * 512);
}

template <int RT, int MT, int U, int XS = 0>
__device__ __forceinline__ void load_frag_x(Frag<RT, MT, U>& f, const bf16_t* xp, long long ldx_, int ks,
                                            const XSrc& xs) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < MT; ++j) f.b[u][j] = ldx_s<XS>(xp + (size_t)j * 16 * ldx_ + (size_t)(ks + u) * 32, xs);
}

template <int RT, int MT, int U, int XS = 0>
__device__ __forceinline__ void load_frag(Frag<RT, MT, U>& f, const bf16_t* wp, size_t tile_stride,
                                          const bf16_t* xp, long long ldx_, int ks,
                                          const XSrc& xs = XSrc{}) {
  load_frag_w(f, wp, tile_stride, ks);
  load_frag_x<RT, MT, U, XS>(f, xp, ldx_, ks, xs);
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

// Ping-pong stream over ng groups of U k-steps; f0 already holds group
// ``rot`` (groups are visited in the rotated order rot, rot+1, ... mod ng).
// The steady-state loop issues the next group UNCONDITIONALLY before consuming
// the current one: a conditional refill inside the loop body makes the
// consumer block a join point of the refill / no-refill paths, and hipcc's
// waitcnt pass then takes the stricter count of the two (vmcnt(0)) - every
// iteration drained the prefetch and only ONE group was ever in flight.
template <int RT, int MT, int U, int XS = 0>
__device__ __forceinline__ void stream_k(Frag<RT, MT, U>& f0, Frag<RT, MT, U>& f1,
                                         float4v_ (&acc)[RT][MT], const bf16_t* wp,
                                         size_t tile_stride, const bf16_t* xp, long long ldx_,
                                         int ks0, int ng, int rot, const XSrc& xs = XSrc{}) {
  auto ks = [&](int g) { int q = g + rot; q -= q >= ng ? ng : 0; return ks0 + q * U; };
  // sched_barrier(0) pins each phase: without it the machine scheduler sinks
  // the refill loads between the MFMAs to save registers, collapsing the
  // prefetch distance to 3-5 loads
  int g = 0;
  for (; g + 2 < ng; g += 2) {
    load_frag<RT, MT, U, XS>(f1, wp, tile_stride, xp, ldx_, ks(g + 1), xs);
    __builtin_amdgcn_sched_barrier(0);
    mma_frag(f0, acc);
    __builtin_amdgcn_sched_barrier(0);
    load_frag<RT, MT, U, XS>(f0, wp, tile_stride, xp, ldx_, ks(g + 2), xs);
    __builtin_amdgcn_sched_barrier(0);
    mma_frag(f1, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (g + 1 < ng) {
    load_frag<RT, MT, U, XS>(f1, wp, tile_stride, xp, ldx_, ks(g + 1), xs);
    __builtin_amdgcn_sched_barrier(0);
    mma_frag(f0, acc);
    mma_frag(f1, acc);
  } else {
    mma_frag(f0, acc);
  }
}

template <int RT, int MT, int U>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(const bf16_t* __restrict__ x, long long ldx_,
                                                          const bf16_t* __restrict__ Wp,
                                                          float* __restrict__ part, int N, int K,
                                                          int S, int Mpad) {
  __shared__ float4v_ red[3][RT * MT][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s = blockIdx.y;
  const int KS = K >> 5;                      // k-steps of 32
  const int kw = KS / (S * 4);                // k-steps per wave
  const int ks0 = (s * 4 + wave) * kw;
  const size_t tile_stride = (size_t)KS * 512;  // elements per 16-row tile
  const bf16_t* xp = x + (size_t)(lane & 15) * ldx_ + 8 * (lane >> 4);
  const int ngroups = N / (16 * RT);
  // grid-stride over tile groups: a capped grid (one workgroup per CU) leaves
  // CU slots free for the concurrent decoder stream (see tune_fused_splits)
  for (int tg = blockIdx.x; tg < ngroups; tg += gridDim.x) {
    const int tile0 = tg * RT;                  // first 16-row tile
    const bf16_t* wp = Wp + (size_t)tile0 * tile_stride + (size_t)lane * 8;
    float4v_ acc[RT][MT];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc[i][j] = (float4v_){0.f, 0.f, 0.f, 0.f};

    // ping-pong register prefetch over groups of U k-steps
    Frag<RT, MT, U> f0, f1;
    load_frag(f0, wp, tile_stride, xp, ldx_, ks0);
    stream_k(f0, f1, acc, wp, tile_stride, xp, ldx_, ks0, kw / U, 0);

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
    __syncthreads();                            // red is reused by the next group
  }
}

template <int RT, int MT>
static int launch_skinny(const void* x, long long ldx_, const void* Wp, float* part, int N, int K,
                         int S, int Mpad, int max_wgs, hipStream_t st) {
  int gx = N / (16 * RT);
  if (max_wgs > 0 && gx * S > max_wgs) gx = max_wgs / S > 0 ? max_wgs / S : 1;
  dim3 grid(gx, S);
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
// max_wgs > 0 caps the grid (workgroups loop over tile groups).
extern "C" int loqa_skinny_gemm(const void* x, long long ldx_, const void* Wp, float* part, int Mpad,
                                int N, int K, int S, int max_wgs, hipStream_t st) {
  if (S < 1 || K % (S * 4 * 32) != 0 || ldx_ % 8 != 0 || N % 16 != 0) return (int)hipErrorInvalidValue;
  switch (Mpad) {
    case 16:
      if (N % 32) return (int)hipErrorInvalidValue;
      return launch_skinny<2, 1>(x, ldx_, Wp, part, N, K, S, Mpad, max_wgs, st);
    case 32:
      if (N % 32) return (int)hipErrorInvalidValue;
      return launch_skinny<2, 2>(x, ldx_, Wp, part, N, K, S, Mpad, max_wgs, st);
    case 64:
      if (N % 64) return (int)hipErrorInvalidValue;
      return launch_skinny<4, 4>(x, ldx_, Wp, part, N, K, S, Mpad, max_wgs, st);
    case 128:
      if (N % 64) return (int)hipErrorInvalidValue;
      return launch_skinny<4, 8>(x, ldx_, Wp, part, N, K, S, Mpad, max_wgs, st);
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

// ============================================================================
// x through LDS (XL): the mid-M form (Mpad 64 / 128: decode steps that carry a
// chunked-prefill slice or long jump-forward runs). At M >= 64 the register
// form above reads Mpad/16 KiB of activation fragments per 1 KiB weight
// fragment, from L2, once per WAVE: at Mpad 64 the activation stream was 4x
// the weight stream and the step took 2.2x the Mpad-16 time. In the XL form
// the 4 waves of a workgroup own 4 row tiles over the SAME k range; each
// U-k-step chunk of x is loaded once per workgroup (256 threads, 16-byte
// pieces, prefetched into registers one chunk ahead) and written to LDS, and
// every wave reads its MFMA B fragments from there (16 B per lane). Weights keep
// the register ping-pong stream (one group of U k-steps in flight).
// LDS image: one 64-B row per (k-step, x row), its four 16-B pieces XOR-swizzled
// by (row >> 1) & 3. ds_read_b128 banks are (a/4) % 64 over four 16-lane groups
// ({0-3,12-15,20-27}, ...) and ds_write_b128 banks (a/4) % 32 over 8-lane groups
// (MI355X_MICROARCH.md, LDS): with the swizzle both the fragment reads (lane l:
// row l & 15, piece l >> 4) and the chunk stores (4 lanes per row) are
// conflict-free. (The earlier 80-B padded rows were conflict-free only under
// 32-bank rules: SQ_LDS_BANK_CONFLICT measured ~1 extra cycle per cycle.)
constexpr int XROW = 32;   // LDS row: 32 k values (64 B), pieces swizzled
__device__ __forceinline__ int xs_piece(int row, int q) { return (q ^ ((row >> 1) & 3)) * 8; }

template <int RT, int U>
struct WFrag {
  bf16x8 a[U][RT];
};

template <int RT, int U>
__device__ __forceinline__ void load_w(WFrag<RT, U>& f, const bf16_t* wp, size_t tile_stride, int ks) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < RT; ++i) f.a[u][i] = ldw(wp + (size_t)i * tile_stride + (size_t)(ks + u) * 512);
}

// one chunk of x: U k-steps x MP rows = MP * U * 4 pieces of 16 B
template <int MP, int U>
struct XRegs {
  static constexpr int NP = (MP * U * 4) / 256;
  uint4 v[NP];
};

// Piece -> thread map: the 4 16-B pieces of a row's k-step fastest, then
// rows, then the chunk's U k-steps. (A whole-line map - a row's U k-steps
// across 4U consecutive lanes - measured 1-2% slower end to end.)
template <int MP, int U>
__device__ __forceinline__ void xc_piece(int idx, int& row, int& u, int& q) {
  q = idx & 3;
  const int rest = idx >> 2;
  row = rest % MP;
  u = rest / MP;
}

template <int MP, int U>
__device__ __forceinline__ void load_xc(XRegs<MP, U>& r, const bf16_t* x, long long ldx_, int ks) {
#pragma unroll
  for (int p = 0; p < XRegs<MP, U>::NP; ++p) {
    int row, u, q;
    xc_piece<MP, U>(p * 256 + (int)threadIdx.x, row, u, q);
    r.v[p] = *reinterpret_cast<const uint4*>(x + (size_t)row * ldx_ + (size_t)(ks + u) * 32 + q * 8);
  }
}

template <int MP, int U>
__device__ __forceinline__ void store_xc(const XRegs<MP, U>& r, bf16_t* xs) {
#pragma unroll
  for (int p = 0; p < XRegs<MP, U>::NP; ++p) {
    int row, u, q;
    xc_piece<MP, U>(p * 256 + (int)threadIdx.x, row, u, q);
    *reinterpret_cast<uint4*>(xs + (size_t)(u * MP + row) * XROW + xs_piece(row, q)) = r.v[p];
  }
}

template <int RT, int MT, int U>
__device__ __forceinline__ void mma_xl(const WFrag<RT, U>& f, float4v_ (&acc)[RT][MT], const bf16_t* xs,
                                       int lane) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    bf16x8 b[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(xs + (size_t)(u * MT * 16 + j * 16 + (lane & 15)) * XROW +
                                              xs_piece(lane & 15, lane >> 4));
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int i = 0; i < RT; ++i) acc[i][j] = mfma16(f.a[u][i], b[j], acc[i][j]);
  }
}

// The XL stream. On entry chunk 0 of x (xr) and weight group 0 (f0) are in
// flight, x issued first, so storing xr waits for x only. Each chunk: issue the
// next chunk's x, then the next weight group (both unconditional, clamped to
// the last chunk: no join point drains the prefetch, see stream_k), consume the
// current chunk from LDS, then (barrier) overwrite LDS with the next chunk.
template <int RT, int MT, int U>
__device__ __forceinline__ void stream_k_xl(WFrag<RT, U>& f0, WFrag<RT, U>& f1, XRegs<MT * 16, U>& xr,
                                            float4v_ (&acc)[RT][MT], const bf16_t* wp,
                                            size_t tile_stride, const bf16_t* x, long long ldx_,
                                            bf16_t* xs, int ks0, int ng, int lane) {
  auto ks = [&](int g) { return ks0 + (g < ng ? g : ng - 1) * U; };
  store_xc<MT * 16, U>(xr, xs);
  lds_barrier();
  int g = 0;
  for (; g + 2 < ng; g += 2) {
    load_xc<MT * 16, U>(xr, x, ldx_, ks(g + 1));
    load_w(f1, wp, tile_stride, ks(g + 1));
    __builtin_amdgcn_sched_barrier(0);
    mma_xl(f0, acc, xs, lane);
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
    store_xc<MT * 16, U>(xr, xs);
    lds_barrier();
    load_xc<MT * 16, U>(xr, x, ldx_, ks(g + 2));
    load_w(f0, wp, tile_stride, ks(g + 2));
    __builtin_amdgcn_sched_barrier(0);
    mma_xl(f1, acc, xs, lane);
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
    store_xc<MT * 16, U>(xr, xs);
    lds_barrier();
  }
  if (g + 1 < ng) {
    load_xc<MT * 16, U>(xr, x, ldx_, ks(g + 1));
    load_w(f1, wp, tile_stride, ks(g + 1));
    __builtin_amdgcn_sched_barrier(0);
    mma_xl(f0, acc, xs, lane);
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
    store_xc<MT * 16, U>(xr, xs);
    lds_barrier();
    mma_xl(f1, acc, xs, lane);
  } else {
    mma_xl(f0, acc, xs, lane);
  }
}

// ============================================================================
// Fused decode GEMMs: the skinny GEMM above with its follow-on op moved into
// the epilogue and the preceding RMSNorm moved into the operand load, so a
// Llama decode layer is 5 launches instead of 10:
//   qkv     : prologue rmsnorm(attn_norm) | epilogue RoPE + paged KV append + q
// (RMSNorm: the norm weight is folded into the weight rows at load time and the
//  per-row 1/rms scale, a property of the row, is applied to the accumulator,
//  so the operand stream stays the plain prefetch pipeline)
//   o       : epilogue residual add + per-tile row sum of squares
//   gate|up : prologue rmsnorm(mlp_norm)  | epilogue silu(gate) * up -> bf16
//   down    : epilogue residual add + per-tile row sum of squares
// Split-K (S > 1) partials are reduced inside the launch by the last arriving
// workgroup of each 32-row tile (guide §5 "in-launch split-K reduction":
// write-through sc1 slab stores -> vmcnt(0) -> barrier -> relaxed agent ticket;
// the reducer takes an agent acquire and sums the S slabs in fixed order, so
// results are bitwise identical to the launch-boundary reduce). The RMSNorm
// scale of a row is rebuilt in every consumer workgroup from the producer's
// per-tile partial sums of squares in a fixed order (deterministic, no atomics).
// Weight rows are permuted at load time so one 32-row tile holds (gate, up)
// feature pairs, or the (c, c + D/2) RoPE pairs of one head.
typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
enum { EPI_SILU = 1, EPI_RESID = 2, EPI_ROPE = 3, EPI_ACT = 4 };
enum { NORM_NONE = 0, NORM_RMS = 1, NORM_LN = 2 };

// Host-side parameter block (mirrored by a ctypes.Structure in ops/_lib.py).
struct FusedParams {
  const void* x; long long ldx; const void* Wp; float* part; int* counters;
  int Mpad, N, K, S, mode, norm;
  const float* rowsq_in; const float* rowsum_in; int rowstat_tiles; float eps;
  const float* colsum; const float* bias;
  void* out; long long ldo; int act;
  void* residual; float* rowsq_out; float* rowsum_out;
  const int* positions; const void* cs; void* q_out; void* kc; void* vc; const int* slots;
  int H, Hkv, D, blk;
  int rt;                 // output tile rows / 16 (1, 2; 4 at Mpad 64)
  int wr;                 // waves along the rows (1, or 4 with S == 1; any S with xl)
  int xl;                 // x through LDS (wr == 4; Mpad 32 / 64 / 128)
  // prologue items (see PRO below): 0 none, 1 the residual all-reduce of the
  // previous row-parallel GEMM (x = the residual it updates), 2 the decode
  // attention whose output is x
  int pro; int* pro_ctr; int pro_wgs;
  void* car; int car_which, car_nblk;                // pro 1: all-reduce handle, input buffer, blocks
  const void* att_q; long long att_q_stride; const void* att_kc; const void* att_vc;   // pro 2
  const int* att_cu_q; const int* att_ctx; const int* att_bt; int att_max_blocks, att_blk;
  int att_B, att_Hq, att_Hkv, att_split_keys, att_num_splits, att_total_q;
  float att_scale; float* att_part_o; float* att_part_ml; int* att_counters;
};

struct FusedArgs {
  const bf16_t* x; long long ldx; const bf16_t* Wp; float* part; int N, K, S, Mpad;
  int* counters;
  const float* rowsq_in; const float* rowsum_in; int rowstat_tiles; float eps;  // norm row stats
  const float* colsum; const float* bias;   // LayerNorm mean correction, output bias (per row of W)
  bf16_t* out; long long ldo; int act;                                        // EPI_SILU / EPI_ACT
  bf16_t* residual; float* rowsq_out; float* rowsum_out;                      // EPI_RESID
  const int* positions; const float2* cs; bf16_t* q_out; bf16_t* kc; bf16_t* vc;
  const int* slots; int H, Hkv, D, blk;                                       // EPI_ROPE
  int prio;                                     // s_setprio 3 for the launch (attn_decode.h)
  // PRO: [0, pro_items) tickets run items, the next pro_gx * S take tiles
  int pro_items, pro_gx, pro_tiles; int* pro_ctr;
  int pro_sleep0, pro_sleep;                    // gate poll back-off: 64 x, then 8 x s_sleep units
  long long x_bytes, rs_bytes;                  // sc1 loads of x / the row statistics
  CarPeers car_peers; long long car_in_off, car_res_off, car_st_off;   // PRO_CAR
  int car_rank, car_world, car_nblk;
  AttnDecArgs att; int att_ns;                  // PRO_ATT
};

enum { PRO_NONE = 0, PRO_CAR = 1, PRO_ATT = 2 };
#define PRO_SPIN_LIMIT (1 << 24)

// the tiles' wait for every prologue item of the launch (bounded spin; a
// failed collective still counts its item, and the step's argmax turns the
// sticky error word into error tokens)
template <int ACQ>
__device__ __forceinline__ void pro_gate(const FusedArgs& a) {
  if (threadIdx.x == 0) {
    // back off first: a few hundred waiting workgroups polling one counter
    // line at agent scope would queue the items' own atomics behind them
    unsigned spins = 0;
    if (__hip_atomic_load(&a.pro_ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.pro_items) {
      for (int i = 0; i < a.pro_sleep0; ++i) __builtin_amdgcn_s_sleep(64);
      while (__hip_atomic_load(&a.pro_ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.pro_items) {
        if (++spins > PRO_SPIN_LIMIT) break;
        for (int i = 0; i < a.pro_sleep; ++i) __builtin_amdgcn_s_sleep(8);
      }
    }
  }
  lds_barrier();       // not __syncthreads: that would drain the weight prefetch
  // ACQ: an agent-scope acquire (invalidates this CU's L1 and the XCD's L2)
  // instead of sc1 loads: x and the statistics are then read with plain,
  // L2-cached loads (the items stored them write-through)
  if constexpr (ACQ) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// WR: waves along the rows. WR = 1: the 4 waves split the tile's K range
// (LDS reduce); WR = 4: every wave owns its own (16 * RT)-row tile over the
// whole K range of the split - the 4 waves then read the SAME activation
// fragments at about the same time, so x is fetched from L2 once per
// workgroup (L1 hits for the other 3) instead of once per wave, and no
// cross-wave reduction is needed (measured on cold weights, M = 16: the
// gate|up stream went from 48 us to 39 us). WR > 1 requires S == 1.
template <int RT, int MT, int WR>
struct FusedSmem {
  static constexpr int WK = 4 / WR;
  static constexpr int NRED = WK > 1 ? WR * (WK - 1) * RT * MT * 64 : 1;
  static constexpr int NSM = NRED * 4 > 1024 ? NRED * 4 : 1024;   // floats: reduce / prologue / ticket
};

// One (16 * RT * WR)-row output tile of the fused GEMM (a workgroup's whole
// GEMM work; `return` = this workgroup's GEMM part is done)
template <int RT, int MT, int U, int WR, int MODE, int NORM, int XL, int PRO = 0, int ACQ = 0>
__device__ __forceinline__ void skinny_fused_tile(const FusedArgs& a, float* smem, bf16_t* xs, const int bx,
                                                  const int by) {
  constexpr int WK = 4 / WR;                     // waves along K
  static_assert(!XL || WR == 4, "XL needs the 4 waves along rows");
  // XL + RoPE at MT 8: the RoPE cos/sin operands (RT * MT * 8 VGPRs) are
  // loaded after the k loop instead of being held through it
  constexpr bool EARLY_EPI = !(XL && MODE == EPI_ROPE && MT > 4);
  float4v_* red = reinterpret_cast<float4v_*>(smem);
  float* sred = smem;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave % WR, wk = wave / WR;
  const int tile = bx * WR + wr;                 // (16 * RT)-row output tile
  const int s = by;                              // K split
  const int KS = a.K >> 5;
  const int kw = KS / (a.S * WK);
  const int ks0 = (s * WK + wk) * kw;
  const size_t tile_stride = (size_t)KS * 512;
  const bf16_t* wp = a.Wp + (size_t)(tile * RT) * tile_stride + (size_t)lane * 8;
  const bf16_t* xp = a.x + (size_t)(lane & 15) * a.ldx + 8 * (lane >> 4);

  // the first weight group is requested before the norm prologue: the row
  // statistics only scale the accumulator, so the stream need not wait for
  // them (the prologue's two L2 round trips then hide under the first fill)
  Frag<RT, MT, XL ? 1 : U> f0, f1;
  WFrag<RT, XL ? U : 1> w0, w1;
  XRegs<XL ? MT * 16 : 64, XL ? U : 1> xr;
  const int ng = kw / U;
  // (a k-start rotation per workgroup measured 5-10 % SLOWER on every shape:
  // the in-step x reuse across neighbouring workgroups in L2 matters more)
  const int rot = 0;
  constexpr int XS = PRO != PRO_NONE && !ACQ;
  XSrc xsrc{a.x, __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.x), 0,
                                                    (int)(XS ? a.x_bytes : 0), 0x00020000)};
  if constexpr (XL) {
    load_xc<MT * 16, U>(xr, a.x, a.ldx, ks0);      // x first: storing it waits for x only
    load_w(w0, wp, tile_stride, ks0);
  } else if constexpr (PRO != PRO_NONE) {
    // the first weight group streams while the prologue items (the residual
    // all-reduce, or the attention producing x) finish; x and the row
    // statistics only after them, with sc1 loads
    load_frag_w(f0, wp, tile_stride, ks0 + rot * U);
    pro_gate<ACQ>(a);
    load_frag_x<RT, MT, (XL ? 1 : U), XS>(f0, xp, a.ldx, ks0 + rot * U, xsrc);
  } else {
    load_frag(f0, wp, tile_stride, xp, a.ldx, ks0 + rot * U);
  }

  // Epilogue operands (residual tile, bias, LayerNorm column sums, RoPE
  // positions / cos-sin / cache slots) are requested now, by the epilogue
  // wave only: their latency hides under the weight stream instead of adding
  // one or two dependent round trips after the last MFMA.
  const int nq = 4 * (lane >> 4);
  uint2 rres[RT][MT];
  float4 bvec[RT], cvec[RT];
  int eslot[MT];
  float2 ecs[RT][MT][4];
  // RoPE epilogue operands: 16-row pair tiles, rows 0-7 = features c..c+7 of
  // the first half, rows 8-15 = their RoPE partners c+D/2..; lanes (l>>4) & 1
  // pick c's 4-row half
  auto load_rope_ops = [&]() {
    const int tph = a.D / 16, nq_t = a.H * tph, nk_t = a.Hkv * tph;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = j * 16 + (lane & 15);
      eslot[j] = a.slots[m];
      if (a.cs) {
        const int pos = a.positions[m];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
          const int pt = tile * RT + i;
          if (pt < nq_t + nk_t) {
            const int tt = pt >= nq_t ? pt - nq_t : pt;
            const int c = (tt % tph) * 8 + 4 * ((lane >> 4) & 1);
            const float2* e = a.cs + (size_t)pos * (a.D >> 1) + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) ecs[i][j][r] = e[r];
          }
        }
      }
    }
  };
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    bvec[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    cvec[i] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < MT; ++j) rres[i][j] = make_uint2(0u, 0u);
  }
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    eslot[j] = -1;
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) ecs[i][j][r] = make_float2(1.f, 0.f);
  }
  if (wk == 0) {
    if (a.bias) {
#pragma unroll
      for (int i = 0; i < RT; ++i)
        bvec[i] = *reinterpret_cast<const float4*>(a.bias + tile * (16 * RT) + i * 16 + nq);
    }
    if constexpr (NORM == NORM_LN) {
#pragma unroll
      for (int i = 0; i < RT; ++i)
        cvec[i] = *reinterpret_cast<const float4*>(a.colsum + tile * (16 * RT) + i * 16 + nq);
    }
    if constexpr (MODE == EPI_RESID) {
#pragma unroll
      for (int j = 0; j < MT; ++j)
#pragma unroll
        for (int i = 0; i < RT; ++i)
          rres[i][j] = *reinterpret_cast<const uint2*>(
              a.residual + (size_t)(j * 16 + (lane & 15)) * a.N + tile * (16 * RT) + i * 16 + nq);
    } else if constexpr (MODE == EPI_ROPE && EARLY_EPI) {
      load_rope_ops();
    }
  }

  float sc[MT], mu[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) sc[j] = 1.f, mu[j] = 0.f;
  if constexpr (NORM != NORM_NONE) {
    // row statistics from the producer's per-tile partial sums (fixed order):
    // RMSNorm scale rsqrt(E[x^2] + eps); LayerNorm also the mean
    const int Mp = a.Mpad, G = 256 / Mp;
    const int m = threadIdx.x % Mp, g = threadIdx.x / Mp;
    // loads issued 16 at a time before any add (a dependent loop would
    // serialise one memory latency per tile)
    float aq = 0.f, as = 0.f;
    for (int base = 0; base < a.rowstat_tiles; base += 16 * G) {
      float vq[16], vs[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int t = base + g + i * G;
        const bool ok = t < a.rowstat_tiles;
        if constexpr (XS)
          vq[i] = ok ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                           __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.rowsq_in), 0,
                                                             (int)a.rs_bytes, 0x00020000),
                           (unsigned)(((size_t)t * Mp + m) * 4), 0, 16))
                     : 0.f;
        else
          vq[i] = ok ? a.rowsq_in[(size_t)t * Mp + m] : 0.f;
        if constexpr (NORM == NORM_LN) vs[i] = ok ? a.rowsum_in[(size_t)t * Mp + m] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        aq += vq[i];
        if constexpr (NORM == NORM_LN) as += vs[i];
      }
    }
    sred[g * Mp + m] = aq;
    if constexpr (NORM == NORM_LN) sred[512 + g * Mp + m] = as;
    lds_barrier();
    if (threadIdx.x < Mp) {
      float tq = 0.f, ts = 0.f;
      for (int q = 0; q < G; ++q) {
        tq += sred[q * Mp + threadIdx.x];
        if constexpr (NORM == NORM_LN) ts += sred[512 + q * Mp + threadIdx.x];
      }
      const float mean = ts / (float)a.K;
      const float var = fmaxf(tq / (float)a.K - mean * mean, 0.f);
      sred[768 + threadIdx.x] = rsqrtf(var + a.eps);   // [768, 896): up to Mpad 128 rows
      sred[896 + threadIdx.x] = mean;
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      sc[j] = sred[768 + j * 16 + (lane & 15)];
      mu[j] = sred[896 + j * 16 + (lane & 15)];
    }
    lds_barrier();
  }

  float4v_ acc[RT][MT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = (float4v_){0.f, 0.f, 0.f, 0.f};
  if constexpr (XL) {
    stream_k_xl(w0, w1, xr, acc, wp, tile_stride, a.x, a.ldx, xs, ks0, ng, lane);
    if constexpr (MODE == EPI_ROPE && !EARLY_EPI) load_rope_ops();
  } else {
    stream_k<RT, MT, (XL ? 1 : U), XS>(f0, f1, acc, wp, tile_stride, xp, a.ldx, ks0, ng, rot, xsrc);
  }

  if constexpr (WK > 1) {
    // red[wr][wk - 1][i * MT + j][lane]
    auto ridx = [&](int q, int ij) { return ((wr * (WK - 1) + q) * RT * MT + ij) * 64 + lane; };
    if (wk > 0) {
#pragma unroll
      for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) red[ridx(wk - 1, i * MT + j)] = acc[i][j];
    }
    __syncthreads();
    if (wk == 0) {
#pragma unroll
      for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j)
#pragma unroll
          for (int q = 0; q < WK - 1; ++q) acc[i][j] += red[ridx(q, i * MT + j)];
    }
  }
  if ((WR == 1 || XL) && a.S > 1) {
    // publish this split's partial (tile-contiguous slab, sc1 write-through),
    // take a ticket; the last arriver reduces with sc1 loads (no acquire fence:
    // every handed-off byte is stored and loaded sc1, guide §6 Guideline 16).
    // WR == 1: wave 0 holds the workgroup's tile; XL (WR == 4): every wave
    // publishes and tickets its own tile.
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        a.part, 0, (int)((size_t)(a.N / (16 * RT * WR)) * WR * a.S * RT * MT * 64 * 16), 0x00020000);
    const int slab0 = tile * a.S * RT * MT;
    if (WR > 1 || wave == 0) {
#pragma unroll
      for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4_, acc[i][j]), rsrc,
              (((slab0 + s * RT * MT) + i * MT + j) * 64 + lane) * 16, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (WR > 1) {
      int t = 0;
      if (lane == 0) {
        t = __hip_atomic_fetch_add(&a.counters[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == a.S - 1)
          __hip_atomic_store(&a.counters[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      t = __shfl(t, 0, 64);
      if (t != a.S - 1) return;
    } else {
      __syncthreads();
      if (threadIdx.x == 0) {
        const int t = __hip_atomic_fetch_add(&a.counters[tile], 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        if (t == a.S - 1)
          __hip_atomic_store(&a.counters[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sred[0] = (float)t;
      }
      __syncthreads();
      if ((int)sred[0] != a.S - 1 || wave != 0) return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // fixed summation order (split 0..S-1) whichever block arrives last
    float4v_ tot[RT][MT];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) tot[i][j] = float4v_{0.f, 0.f, 0.f, 0.f};
    // QB slabs per batch, every load issued before the adds (a rolled loop
    // pays one L2 round trip per split); out-of-range slots add exact zeros
    constexpr int QB = (8 / (RT * MT)) > 2 ? 8 / (RT * MT) : 2;
    for (int q0 = 0; q0 < a.S; q0 += QB) {
      float4v_ v[QB][RT][MT];
#pragma unroll
      for (int qq = 0; qq < QB; ++qq)
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
          for (int j = 0; j < MT; ++j)
            v[qq][i][j] = q0 + qq < a.S
                              ? __builtin_bit_cast(float4v_, __builtin_amdgcn_raw_buffer_load_b128(
                                                                 rsrc, (((slab0 + (q0 + qq) * RT * MT) + i * MT + j) * 64 + lane) * 16, 0, 16))
                              : float4v_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int qq = 0; qq < QB; ++qq)
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
          for (int j = 0; j < MT; ++j) tot[i][j] += v[qq][i][j];
    }
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc[i][j] = tot[i][j];
  } else if (wk != 0) {
    return;
  }

  // ---- epilogue (the wk == 0 wave of each row tile): acc[i][j] = C[n0 + 4*(lane>>4) + r][m] for i = tile half
  // Norms: the norm weight g is folded into W at load time, so the row scale
  // factors out of the k-sum: RMSNorm  y = s * (W g) x;  LayerNorm
  // y = s * ((W g) x - mean * colsum) with colsum[n] = sum_k (W g)[n][k]; the
  // LayerNorm shift (W b) is folded into the bias.
  if constexpr (NORM == NORM_RMS) {
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc[i][j] *= sc[j];
  } else if constexpr (NORM == NORM_LN) {
#pragma unroll
    for (int i = 0; i < RT; ++i) {
      const float4 cv = cvec[i];
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        acc[i][j][0] = sc[j] * (acc[i][j][0] - mu[j] * cv.x);
        acc[i][j][1] = sc[j] * (acc[i][j][1] - mu[j] * cv.y);
        acc[i][j][2] = sc[j] * (acc[i][j][2] - mu[j] * cv.z);
        acc[i][j][3] = sc[j] * (acc[i][j][3] - mu[j] * cv.w);
      }
    }
  }
  if (a.bias) {
#pragma unroll
    for (int i = 0; i < RT; ++i) {
      const float4 bv = bvec[i];
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        acc[i][j][0] += bv.x; acc[i][j][1] += bv.y; acc[i][j][2] += bv.z; acc[i][j][3] += bv.w;
      }
    }
  }
  if constexpr (MODE == EPI_SILU) {
    // 16-row pair tiles (perm_gate_up): rows 0-7 gate, rows 8-15 the matching
    // up rows -> lane l (l < 32) holds gate, lane l ^ 32 its up partner
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int m = j * 16 + (lane & 15);
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float own = bf2f(f2bf(acc[i][j][r]));
          const float oth = __shfl_xor(own, 32, 64);
          o[r] = own / (1.f + __expf(-own)) * oth;
        }
        if (lane < 32) {
          uint2 w2;
          w2.x = pack_bf16x2(o[0], o[1]);
          w2.y = pack_bf16x2(o[2], o[3]);
          *reinterpret_cast<uint2*>(a.out + (size_t)m * a.ldo + (tile * RT + i) * 8 + nq) = w2;
        }
      }
  } else if constexpr (MODE == EPI_RESID) {
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = j * 16 + (lane & 15);
      float sq = 0.f, sm = 0.f;
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        bf16_t* rp = a.residual + (size_t)m * a.N + tile * (16 * RT) + i * 16 + nq;
        const uint2 rv = rres[i][j];
        const float r0 = bf2f(rv.x & 0xffff), r1 = bf2f(rv.x >> 16);
        const float r2 = bf2f(rv.y & 0xffff), r3 = bf2f(rv.y >> 16);
        const float h0 = bf2f(f2bf(acc[i][j][0] + r0)), h1 = bf2f(f2bf(acc[i][j][1] + r1));
        const float h2 = bf2f(f2bf(acc[i][j][2] + r2)), h3 = bf2f(f2bf(acc[i][j][3] + r3));
        uint2 w2;
        w2.x = pack_bf16x2(h0, h1);
        w2.y = pack_bf16x2(h2, h3);
        *reinterpret_cast<uint2*>(rp) = w2;
        sq += h0 * h0 + h1 * h1 + h2 * h2 + h3 * h3;
        sm += h0 + h1 + h2 + h3;
      }
      sq += __shfl_xor(sq, 16, 64);
      sq += __shfl_xor(sq, 32, 64);
      sm += __shfl_xor(sm, 16, 64);
      sm += __shfl_xor(sm, 32, 64);
      if (lane < 16) {
        a.rowsq_out[(size_t)tile * a.Mpad + m] = sq;
        if (a.rowsum_out) a.rowsum_out[(size_t)tile * a.Mpad + m] = sm;
      }
    }
  } else if constexpr (MODE == EPI_ROPE) {
    // perm_rope_qkv: q / k as 16-row pair tiles (rows 0-7 = first-half features
    // c.., rows 8-15 = partners c+D/2..: lane l and l ^ 32 hold a RoPE pair);
    // v rows in natural order
    const int D = a.D, half = D >> 1, tph = D / 16;
    const int nq_t = a.H * tph, nk_t = a.Hkv * tph;
    const bool lower = lane < 32;
#pragma unroll
    for (int i = 0; i < RT; ++i) {
      const int pt = tile * RT + i;
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int m = j * 16 + (lane & 15);
        const int slot = eslot[j];
        if (pt < nq_t + nk_t) {
          const bool isk = pt >= nq_t;
          const int tt = isk ? pt - nq_t : pt;
          const int head = tt / tph;
          const int c = (tt - head * tph) * 8 + 4 * ((lane >> 4) & 1) + (lower ? 0 : half);
          float ov[4];
          if (a.cs) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float own = bf2f(f2bf(acc[i][j][r]));
              const float oth = __shfl_xor(own, 32, 64);
              const float2 cs = ecs[i][j][r];
              // lower: x0 cos - x1 sin; upper (own = x1, oth = x0): x1 cos + x0 sin
              ov[r] = own * cs.x + (lower ? -oth : oth) * cs.y;
            }
          } else {  // no rotary embedding (Whisper): plain q / k rows
#pragma unroll
            for (int r = 0; r < 4; ++r) ov[r] = acc[i][j][r];
          }
          uint2 w2;
          w2.x = pack_bf16x2(ov[0], ov[1]);
          w2.y = pack_bf16x2(ov[2], ov[3]);
          if (!isk) {
            *reinterpret_cast<uint2*>(a.q_out + (size_t)m * a.H * D + head * D + c) = w2;
          } else {
            if (slot < 0) continue;
            const int bb = slot / a.blk, o = slot - bb * a.blk;
            *reinterpret_cast<uint2*>(a.kc + (((size_t)bb * a.Hkv + head) * a.blk + o) * D + c) = w2;
          }
        } else {
          if (slot < 0) continue;
          const int bb = slot / a.blk, o = slot - bb * a.blk;
          const int row = (pt - nq_t - nk_t) * 16 + nq;
          const int head = row / D, c = row - head * D;
          uint2 w2;
          w2.x = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
          w2.y = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
          *reinterpret_cast<uint2*>(a.vc + (((size_t)bb * a.Hkv + head) * a.blk + o) * D + c) = w2;
        }
      }
    }
  } else if constexpr (MODE == EPI_ACT) {
    if (a.act == 2) {
      // f32 output (tensor-parallel partial sums: the all-reduce adds them in
      // f32 before the one bf16 rounding of the residual, as the single-GPU
      // residual epilogue does)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int m = j * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < RT; ++i)
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.out) + (size_t)m * a.ldo +
                                     tile * (16 * RT) + i * 16 + nq) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = bf2f(f2bf(acc[i][j][r]));
          o[r] = a.act == 1 ? 0.5f * x * (1.f + erff(x * 0.70710678118654752f)) : x;
        }
        uint2 w2;
        w2.x = pack_bf16x2(o[0], o[1]);
        w2.y = pack_bf16x2(o[2], o[3]);
        *reinterpret_cast<uint2*>(a.out + (size_t)m * a.ldo + tile * (16 * RT) + i * 16 + nq) = w2;
      }
    }
  }
}

// PRO (prologue items): a launch whose input x is produced by a short
// latency-bound step - the tensor-parallel residual all-reduce of the
// previous row-parallel GEMM (PRO_CAR, x = the residual it updates, its
// statistics tiles = this GEMM's norm prologue) or the decode attention
// (PRO_ATT, x = its output) - runs that step INSIDE this launch: workgroups
// draw tickets from a counter; the first pro_items tickets run the items
// (all-reduce blocks / attention items, their results stored write-through),
// later tickets take GEMM tiles, whose weight stream starts at once and which
// wait for every item (pro_gate) before reading x with sc1 loads. The kernel
// boundary and the GEMM's first-load latency disappear behind the step; a
// tile never waits for work that is not already running (items are taken
// first), so any grid size is deadlock-free on its own GPU. The last
// workgroup out resets the counters (graph replays).
template <int RT, int MT, int U, int WR, int MODE, int NORM, int XL = 0, int PRO = PRO_NONE, int ACQ = 0>
__global__ __launch_bounds__(256) void skinny_fused_kernel(FusedArgs a) {
  constexpr int NSM = FusedSmem<RT, MT, WR>::NSM;
  constexpr int ASM = PRO == PRO_ATT ? (int)(sizeof(DecSmem<128>) / 4) : 0;
  constexpr int SMF = (NSM > ASM ? NSM : ASM) + 4;
  __shared__ __attribute__((aligned(16))) float smem[SMF];
  __shared__ __attribute__((aligned(16))) bf16_t xs[XL ? U * MT * 16 * XROW : 8];
  if (a.prio) __builtin_amdgcn_s_setprio(3);     // kernel argument: wave-uniform
  if constexpr (PRO == PRO_NONE) {
    skinny_fused_tile<RT, MT, U, WR, MODE, NORM, XL>(a, smem, xs, blockIdx.x, blockIdx.y);
  } else {
    int* sflag = reinterpret_cast<int*>(smem) + (SMF - 1);
    for (;;) {
      __syncthreads();                            // smem / sflag of the previous item
      if (threadIdx.x == 0)
        sflag[0] = __hip_atomic_fetch_add(&a.pro_ctr[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int t = __builtin_amdgcn_readfirstlane(sflag[0]);
      if (t < a.pro_items) {
        if constexpr (PRO == PRO_CAR) {
          car_resid_block<1, 1>(a.car_peers, a.car_in_off, a.car_res_off, a.car_st_off,
                                const_cast<bf16_t*>(a.x), const_cast<float*>(a.rowsq_in), a.Mpad, a.K,
                                a.car_rank, a.car_world, t, a.car_nblk);
        } else {
          const int split = t % a.att_ns, rest = t / a.att_ns;
          attn_decode_body<128, 0, 1, 0, DEC_WAVES, 1>(a.att, split, rest % a.att.Hkv, rest / a.att.Hkv,
                                                       *reinterpret_cast<DecSmem<128>*>(smem));
        }
        // the item's write-through stores are complete -> count it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
          __hip_atomic_fetch_add(&a.pro_ctr[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      const int g = t - a.pro_items;
      if (g < a.pro_tiles) {
        skinny_fused_tile<RT, MT, U, WR, MODE, NORM, 0, PRO, ACQ>(a, smem, xs, g % a.pro_gx, g / a.pro_gx);
        continue;
      }
      // exit ticket: the last workgroup out leaves the counters zeroed
      if (threadIdx.x == 0 && g - a.pro_tiles == (int)gridDim.x - 1) {
        __hip_atomic_store(&a.pro_ctr[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.pro_ctr[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      break;
    }
  }
}

// Deep prefetch (LOQA_FUSED_DEEP bit mask, Mpad 16): bit 0 - a wave's whole k
// range in ONE prefetch group when it is 10 k-steps (Whisper d = 1280, S = 1:
// every weight load of the wave in flight at once instead of two 2-step
// groups at a time); bit 1 - 8-step groups when it is a multiple of 8 (Llama
// K = 4096; measured slower in the pipeline: 3.51 -> 3.68 ms per LLM step); bit 2 -
// the same 8-step groups for the o / qkv shapes only. The decode
// GEMMs are latency-bound beside the concurrent decoder: fewer dependent
// prefetch rounds per kernel, not bandwidth, is what a shorter kernel needs.
static int g_fused_deep = -1;

template <int RT, int MT, int WR, int MODE, int NORM>
static int launch_fused(const FusedArgs& a, hipStream_t st) {
  constexpr int WK = 4 / WR;
  dim3 grid(a.N / (16 * RT * WR), a.S);
  const int kw = a.K / 32 / (a.S * WK);
  if (g_fused_deep < 0) {
    const char* e = getenv("LOQA_FUSED_DEEP");
    g_fused_deep = e ? atoi(e) : 0;
  }
  if constexpr (MT == 1) {
    if ((g_fused_deep & 1) && kw == 10) {
      hipLaunchKernelGGL((skinny_fused_kernel<RT, 1, 10, WR, MODE, NORM>), grid, dim3(256), 0, st, a);
      return (int)hipGetLastError();
    }
    if ((g_fused_deep & 2) && kw % 8 == 0) {
      hipLaunchKernelGGL((skinny_fused_kernel<RT, 1, 8, WR, MODE, NORM>), grid, dim3(256), 0, st, a);
      return (int)hipGetLastError();
    }
    // bit 2 (value 4): only the short Llama GEMMs (o, qkv: N <= 6144, K = 4096),
    // whose <= 256 workgroups hold one 4-wave group per CU - bytes in flight
    // per CU, not occupancy, bound them
    if ((g_fused_deep & 4) && kw % 8 == 0 && a.N <= 6144 && a.K <= 4096) {
      hipLaunchKernelGGL((skinny_fused_kernel<RT, 1, 8, WR, MODE, NORM>), grid, dim3(256), 0, st, a);
      return (int)hipGetLastError();
    }
    // bit 3 (value 8): any grid of at most one workgroup per CU (a tensor-
    // parallel rank's shard GEMMs: 80-256 workgroups, nothing beside them) -
    // twice the bytes in flight per CU
    if ((g_fused_deep & 8) && kw % 8 == 0 && (long long)grid.x * grid.y <= 256) {
      hipLaunchKernelGGL((skinny_fused_kernel<RT, 1, 8, WR, MODE, NORM>), grid, dim3(256), 0, st, a);
      return (int)hipGetLastError();
    }
  }
  if (MT <= 2 && kw % 4 == 0)   // Mpad 64: at most 2 k-steps per prefetch group (VGPRs)
    hipLaunchKernelGGL((skinny_fused_kernel<RT, MT, (MT <= 2 ? 4 : 2), WR, MODE, NORM>), grid, dim3(256), 0, st, a);
  else if (kw % 2 == 0)
    hipLaunchKernelGGL((skinny_fused_kernel<RT, MT, 2, WR, MODE, NORM>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((skinny_fused_kernel<RT, MT, 1, WR, MODE, NORM>), grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

template <int RT, int MODE, int NORM>
static int dispatch_mt(const FusedArgs& a, int wr, hipStream_t st) {
  switch (a.Mpad) {
    case 16:
      if (wr == 4) return launch_fused<RT, 1, 4, MODE, NORM>(a, st);
      return launch_fused<RT, 1, 1, MODE, NORM>(a, st);
    case 32:
      if (wr == 4) return launch_fused<RT, 2, 4, MODE, NORM>(a, st);
      return launch_fused<RT, 2, 1, MODE, NORM>(a, st);
    default:
      if (wr == 4) return launch_fused<RT, 4, 4, MODE, NORM>(a, st);
      return launch_fused<RT, 4, 1, MODE, NORM>(a, st);
  }
}

// XL dispatch: Mpad 32 (MT 2) / 64 (MT 4) / 128 (MT 8), 4 waves along rows, any split-K.
// Prefetch group = one LDS chunk: 4 k-steps, 2 when the VGPR budget is tight.
template <int RT, int MT, int MODE, int NORM>
static int launch_xl(const FusedArgs& a, hipStream_t st) {
  dim3 grid(a.N / (16 * RT * 4), a.S);
  const int kw = a.K / 32 / a.S;
  constexpr int UA = (RT * MT >= 16) ? 2 : 4;
  if (kw % UA == 0)
    hipLaunchKernelGGL((skinny_fused_kernel<RT, MT, UA, 4, MODE, NORM, 1>), grid, dim3(256), 0, st, a);
  else if (kw % 2 == 0)
    hipLaunchKernelGGL((skinny_fused_kernel<RT, MT, 2, 4, MODE, NORM, 1>), grid, dim3(256), 0, st, a);
  else if constexpr (MT * 16 * 4 >= 256)   // a 1-k-step x chunk must cover the 256 threads' pieces
    hipLaunchKernelGGL((skinny_fused_kernel<RT, MT, 1, 4, MODE, NORM, 1>), grid, dim3(256), 0, st, a);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

template <int MODE, int NORM>
static int dispatch_xl(const FusedArgs& a, int rt, hipStream_t st) {
  if (a.Mpad == 32) return rt == 2 ? launch_xl<2, 2, MODE, NORM>(a, st) : launch_xl<1, 2, MODE, NORM>(a, st);
  if (a.Mpad == 64) return rt == 2 ? launch_xl<2, 4, MODE, NORM>(a, st) : launch_xl<1, 4, MODE, NORM>(a, st);
  return rt == 2 ? launch_xl<2, 8, MODE, NORM>(a, st) : launch_xl<1, 8, MODE, NORM>(a, st);
}

// rt: rows per output tile / 16 (1 or 2, every mode: the paired epilogues pair
// rows inside each 16-row tile through a lane shuffle, so 16-row tiles give
// twice the workgroups without a K split, i.e. without a reduction tail).
// wr: waves along the rows (1 or 4; 4 only with S == 1).
template <int MODE, int NORM>
static int dispatch_fused(const FusedArgs& a, int rt, int wr, hipStream_t st) {
  // 64-row tiles at Mpad 64 (chunked prefill through the compact weights):
  // the activation tile is then re-read from L2 by half as many workgroups
  if (rt == 4) {
    if (wr == 4) return launch_fused<4, 4, 4, MODE, NORM>(a, st);
    return launch_fused<4, 4, 1, MODE, NORM>(a, st);
  }
  if (rt == 1) return dispatch_mt<1, MODE, NORM>(a, wr, st);
  return dispatch_mt<2, MODE, NORM>(a, wr, st);
}

template <int MODE>
static int dispatch_norm(const FusedArgs& a, int norm, int rt, int wr, int xl, hipStream_t st) {
  if (xl) {
    switch (norm) {
      case NORM_NONE: return dispatch_xl<MODE, NORM_NONE>(a, rt, st);
      case NORM_RMS: return dispatch_xl<MODE, NORM_RMS>(a, rt, st);
      case NORM_LN: return dispatch_xl<MODE, NORM_LN>(a, rt, st);
      default: return (int)hipErrorInvalidValue;
    }
  }
  switch (norm) {
    case NORM_NONE: return dispatch_fused<MODE, NORM_NONE>(a, rt, wr, st);
    case NORM_RMS: return dispatch_fused<MODE, NORM_RMS>(a, rt, wr, st);
    case NORM_LN: return dispatch_fused<MODE, NORM_LN>(a, rt, wr, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// prologue-item launches (PRO_CAR / PRO_ATT): WR 1, no XL, Mpad 16 / 32,
// 4-step prefetch groups; a 1-D grid of at most ``wgs`` workgroups that draw
// items and tiles from the ticket counter
static int g_pro_acq = -1;   // LOQA_PRO_ACQ: 1 = acquire + plain loads, 0 = sc1 loads

template <int RT, int MT, int MODE, int NORM, int PRO>
static int launch_pro(const FusedArgs& a, int wgs, hipStream_t st) {
  if (g_pro_acq < 0) {
    const char* e = getenv("LOQA_PRO_ACQ");
    g_pro_acq = e ? atoi(e) : 0;
  }
  if (g_pro_acq)
    hipLaunchKernelGGL((skinny_fused_kernel<RT, MT, 4, 1, MODE, NORM, 0, PRO, 1>), dim3(wgs), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((skinny_fused_kernel<RT, MT, 4, 1, MODE, NORM, 0, PRO, 0>), dim3(wgs), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

template <int MODE, int NORM, int PRO>
static int dispatch_pro(const FusedArgs& a, int rt, int wgs, hipStream_t st) {
  if (a.Mpad == 16) return rt == 1 ? launch_pro<1, 1, MODE, NORM, PRO>(a, wgs, st)
                                   : launch_pro<2, 1, MODE, NORM, PRO>(a, wgs, st);
  return rt == 1 ? launch_pro<1, 2, MODE, NORM, PRO>(a, wgs, st) : launch_pro<2, 2, MODE, NORM, PRO>(a, wgs, st);
}

static int fused_prologue(const FusedParams* p, FusedArgs& a, hipStream_t st) {
  const int Mpad = p->Mpad, N = p->N, K = p->K, S = p->S;
  if (p->xl || p->wr != 1 || (Mpad != 16 && Mpad != 32) || (p->rt != 1 && p->rt != 2) ||
      (K / 32 / (S * 4)) % 4 || !p->pro_ctr)
    return (int)hipErrorInvalidValue;
  static int ncu = 0;
  if (ncu <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return (int)hipErrorInvalidValue;
  }
  a.pro_ctr = p->pro_ctr;
  static int sl0 = -1, sl = -1;
  if (sl0 < 0) {
    const char* e0 = getenv("LOQA_PRO_SLEEP0");
    const char* e1 = getenv("LOQA_PRO_SLEEP");
    sl0 = e0 ? atoi(e0) : 2;      // ~3.4 us before the first re-poll
    sl = e1 ? atoi(e1) : 4;       // ~0.9 us between polls
  }
  a.pro_sleep0 = sl0;
  a.pro_sleep = sl < 1 ? 1 : sl;
  a.pro_gx = N / (16 * p->rt);
  a.pro_tiles = a.pro_gx * S;
  a.x_bytes = (long long)Mpad * p->ldx * 2;
  a.rs_bytes = (long long)(p->rowstat_tiles > 0 ? p->rowstat_tiles : 1) * Mpad * 4;
  if (p->pro == PRO_CAR) {
    // x = the residual [Mpad, d = K] the all-reduce updates; its statistics
    // tiles (world x nblk) are this GEMM's norm input
    if ((p->mode != EPI_SILU && p->mode != EPI_ROPE) || p->norm != NORM_RMS || !p->car || p->car_nblk < 1 ||
        p->car_nblk > CAR_MAX_BLOCKS || p->ldx != K)
      return (int)hipErrorInvalidValue;
    size_t in_bytes = 0;
    const int rc = car_prologue_args(p->car, p->car_which, &a.car_peers, &a.car_in_off, &a.car_res_off,
                                     &a.car_st_off, &a.car_rank, &a.car_world, &in_bytes);
    if (rc) return rc;
    const int cw = K / a.car_world / p->car_nblk, vpr = cw / 4;
    if (K % (a.car_world * p->car_nblk) || cw % 8 || vpr > 64 || (vpr & (vpr - 1)) ||
        (size_t)Mpad * K * 4 > in_bytes || p->rowstat_tiles != a.car_world * p->car_nblk)
      return (int)hipErrorInvalidValue;
    a.car_nblk = p->car_nblk;
    a.pro_items = p->car_nblk;
  } else if (p->pro == PRO_ATT) {
    // x = the attention output [Mpad, Hq * 128] (row stride ldx)
    if ((p->mode != EPI_ACT && p->mode != EPI_RESID) || p->norm != NORM_NONE || !p->att_q || !p->att_kc ||
        !p->att_vc || !p->att_cu_q || !p->att_ctx || !p->att_bt || !p->att_part_o || !p->att_part_ml ||
        !p->att_counters || p->att_Hkv < 1 || p->att_Hq % p->att_Hkv || p->att_Hq * 128 != K ||
        p->att_blk < 16 || (p->att_blk & (p->att_blk - 1)) || p->att_split_keys % DEC_TILE ||
        p->att_num_splits < 1 || p->att_B < 1 || p->att_total_q > Mpad)
      return (int)hipErrorInvalidValue;
    a.att = AttnDecArgs{(const bf16_t*)p->att_q, p->att_q_stride, (const bf16_t*)p->att_kc,
                        (const bf16_t*)p->att_vc, 0, nullptr, p->att_cu_q, p->att_ctx, p->att_bt,
                        p->att_max_blocks, p->att_blk, p->att_Hq, p->att_Hkv,
                        p->att_scale * 1.4426950408889634f, 1, p->att_split_keys, p->att_num_splits,
                        p->att_part_o, p->att_part_ml, p->att_total_q, p->att_counters,
                        const_cast<bf16_t*>(a.x), p->ldx, 0, 0, 0, a.x_bytes};
    a.att_ns = p->att_num_splits;
    a.pro_items = p->att_num_splits * p->att_Hkv * p->att_B;
  } else {
    return (int)hipErrorInvalidValue;
  }
  const int cap = p->pro_wgs > 0 ? p->pro_wgs : ncu;
  const int total = a.pro_items + a.pro_tiles;
  const int wgs = total < cap ? total : cap;
  if (p->pro == PRO_CAR) {
    if (p->mode == EPI_SILU) return dispatch_pro<EPI_SILU, NORM_RMS, PRO_CAR>(a, p->rt, wgs, st);
    return dispatch_pro<EPI_ROPE, NORM_RMS, PRO_CAR>(a, p->rt, wgs, st);
  }
  if (p->mode == EPI_ACT) return dispatch_pro<EPI_ACT, NORM_NONE, PRO_ATT>(a, p->rt, wgs, st);
  return dispatch_pro<EPI_RESID, NORM_NONE, PRO_ATT>(a, p->rt, wgs, st);
}

// mode: 1 silu (out [Mpad, ldo >= N/2]), 2 residual (+bias) + row sum-of-squares
// (+ row sums), 3 (RoPE if cs) + paged KV append + q, 4 act(bias + x W^T) -> out
// (act 0 identity, 1 GELU-erf). norm: 1 RMSNorm / 2 LayerNorm of x (the bf16
// residual) with the norm weight folded into Wp; the row statistics come from
// rowstat_tiles partial sums. part: S * Mpad * N f32 scratch (S > 1,
// tile-contiguous slabs); counters: >= N/(16*rt) zeroed ints. Row statistics of
// the residual epilogue are written per (16*rt)-row tile.
extern "C" int loqa_skinny_fused(const FusedParams* p, hipStream_t st) {
  const int Mpad = p->Mpad, N = p->N, K = p->K, S = p->S;
  if (S < 1 || K % (S * 128) || p->ldx % 8 || N % 32 ||
      (Mpad != 16 && Mpad != 32 && Mpad != 64 && !(Mpad == 128 && p->xl)))
    return (int)hipErrorInvalidValue;
  if (p->xl && (p->wr != 4 || Mpad < 32 || (p->rt != 1 && p->rt != 2) || N % (64 * p->rt)))
    return (int)hipErrorInvalidValue;
  if (S > 1 && (!p->part || !p->counters)) return (int)hipErrorInvalidValue;
  if (p->norm && (!p->rowsq_in || p->rowstat_tiles < 1)) return (int)hipErrorInvalidValue;
  if (p->norm == NORM_LN && (!p->rowsum_in || !p->colsum)) return (int)hipErrorInvalidValue;
  if (p->mode == EPI_ROPE && (p->D % 16 || N != (p->H + 2 * p->Hkv) * p->D))
    return (int)hipErrorInvalidValue;
  if ((p->mode == EPI_SILU || p->mode == EPI_ACT) && (!p->out || p->ldo % 4))
    return (int)hipErrorInvalidValue;
  if (p->rt != 1 && p->rt != 2 && !(p->rt == 4 && Mpad == 64)) return (int)hipErrorInvalidValue;
  if (p->mode == EPI_RESID && (!p->residual || !p->rowsq_out)) return (int)hipErrorInvalidValue;
  if (p->wr != 1 && (p->wr != 4 || (S != 1 && !p->xl) || N % (64 * p->rt)))
    return (int)hipErrorInvalidValue;
  FusedArgs a{(const bf16_t*)p->x, p->ldx, (const bf16_t*)p->Wp, p->part, N, K, S, Mpad,
              p->counters, p->rowsq_in, p->rowsum_in, p->rowstat_tiles, p->eps, p->colsum,
              p->bias, (bf16_t*)p->out, p->ldo, p->act, (bf16_t*)p->residual, p->rowsq_out,
              p->rowsum_out, p->positions, (const float2*)p->cs, (bf16_t*)p->q_out,
              (bf16_t*)p->kc, (bf16_t*)p->vc, p->slots, p->H, p->Hkv, p->D, p->blk};
  a.prio = g_loqa_launch_prio;
  if (p->pro) return fused_prologue(p, a, st);
  switch (p->mode) {
    case EPI_SILU: return dispatch_norm<EPI_SILU>(a, p->norm, p->rt, p->wr, p->xl, st);
    case EPI_RESID: return dispatch_norm<EPI_RESID>(a, p->norm, p->rt, p->wr, p->xl, st);
    case EPI_ROPE: return dispatch_norm<EPI_ROPE>(a, p->norm, p->rt, p->wr, p->xl, st);
    case EPI_ACT: return dispatch_norm<EPI_ACT>(a, p->norm, p->rt, p->wr, p->xl, st);
    default: return (int)hipErrorInvalidValue;
  }
}
