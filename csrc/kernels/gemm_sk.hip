// Split-K LDS-tiled MFMA GEMM with an in-launch reduction and fused epilogues:
// Y[M, N] = X[M, K] W[N, K]^T for the projections of a prompt pass (Llama
// prefill: M = a few hundred to a few thousand rows) and the Whisper encoder.
//
// Why split-K inside the launch: at M ~ 300 a projection has few output tiles
// (qkv 6144 x 4096: 240 tiles of 128 x 64; o / down 4096 wide: 160), far fewer
// than the 256 CUs x 2-3 resident workgroups, and a whole tile's K loop is one
// workgroup's serial latency. Splitting each tile's K range over S workgroups
// fills the machine; the S partial accumulators are summed by the LAST
// workgroup of the tile to finish (agent-scope release / ticket / acquire,
// guide §5 "In-launch split-K reduction"), which then runs the epilogue - no
// f32 slabs for a later kernel to re-read and no extra launch. The sum is in
// fixed chunk order over the published partials (the reducer's own included),
// so the result is bitwise identical whoever arrives last.
//
// Main loop: as gemm_tile.hip - BK = 64 stages of (BN + BM) rows x 128 B filled
// by global_load_lds with the LDS bank swizzle on the source address, NBUF - 1
// stages in flight across raw s_barriers (counted vmcnt), XCD-aware workgroup
// order with a tile's K chunks adjacent on one XCD.
//
// Epilogues (applied once per output element, by the tile's reducer):
//   SK_BF16   y = bf16(acc (+ bias)), optionally GELU (Whisper encoder fc1)
//   SK_SWIGLU y[:, f] = silu(gate_f) * up_f (a wave tile holds TN/2 gate and the
//             matching TN/2 up features, row-permuted at staging)
//   SK_RESID  y = bf16(y + (acc + bias)): the row-parallel projections (o,
//             down, encoder o / fc2) add straight into the residual stream, one
//             rounding.
#include "common.h"

#define SK_BK 64

enum { SK_BF16 = 0, SK_SWIGLU = 1, SK_RESID = 2 };

struct GemmSkParams {
  const void* x; long long ldx;   // [M, K] bf16 rows
  const void* w;                  // [N, K] bf16 row-major (SwiGLU: gate rows [0, N/2), up [N/2, N))
  int M, N, K, S;                 // S: K chunks per output tile
  int epi, act;                   // act (SK_BF16): 0 none, 1 GELU (erf) after the bias
  const float* bias;              // [N] f32 or null (SK_BF16, SK_RESID)
  void* y; long long ldy;         // bf16 output (SK_RESID: the residual, updated in place)
  float* ws;                      // S > 1: [tiles][S][BM * BN] f32 partials
  int* counters;                  // S > 1: [tiles] ints, zero on entry (left zero)
  int layout;
};

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt at their maxima (gfx9 encoding:
// vmcnt[3:0] in bits 3:0, vmcnt[5:4] in bits 15:14)
template <int N>
__device__ __forceinline__ void sk_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int WN, int WM, int FN, int FM, int NBUF, int EPI>
__global__ __launch_bounds__(64 * WN * WM) void gemm_sk_kernel(GemmSkParams p) {
  constexpr int NW = WN * WM;
  constexpr int TN = 16 * FN, TM = 16 * FM;      // wave tile: TN features x TM rows
  constexpr int BN = TN * WN, BM = TM * WM;
  constexpr int ROWS = BN + BM;
  constexpr int STAGE = ROWS * 128;             // bytes per stage
  constexpr int IPW = ROWS / 8 / NW;            // glds instructions per wave per stage
  static_assert(IPW * 8 * NW == ROWS, "stage rows must split evenly over the waves");
  static_assert(EPI != SK_SWIGLU || FN % 2 == 0, "SwiGLU pairs gate / up fragments");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NBUF * STAGE];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int M = p.M, N = p.N, S = p.S;
  const int mblocks = (M + BM - 1) / BM;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int s = id % S, tile = id / S;
  const int mb = tile % mblocks, nb = tile / mblocks;
  const int KT = p.K / SK_BK;
  const int kt0 = (int)(((long long)s * KT) / S), kt1 = (int)(((long long)(s + 1) * KT) / S);
  const int nt = kt1 - kt0;
  const int m0 = mb * BM, n0 = nb * BN;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ W = reinterpret_cast<const bf16_t*>(p.w);

  // per-lane source of each of this wave's stage instructions (k offset added per stage)
  const bf16_t* src[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int r = 8 * (wave * IPW + i) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    if (r < BN) {
      int row;
      if constexpr (EPI == SK_SWIGLU) {
        const int blk = r / TN, rr = r - blk * TN;
        const int f = (n0 >> 1) + blk * (TN / 2) + (rr % (TN / 2));
        row = rr < TN / 2 ? f : (N >> 1) + f;
      } else {
        row = n0 + r;
      }
      src[i] = W + (size_t)row * p.K + c * 8;
    } else {
      const int m = min(m0 + r - BN, M - 1);
      src[i] = X + (size_t)m * p.ldx + c * 8;
    }
  }

  auto stage = [&](int buf, int kt) {
    const int kc = kt * SK_BK;
#pragma unroll
    for (int i = 0; i < IPW; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src[i] + kc),
          (__attribute__((address_space(3))) void*)(lds + buf * STAGE + (wave * IPW + i) * 1024), 16, 0, 0);
  };

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto frag = [&](int buf, int row, int c) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(lds + buf * STAGE + row * 128 + 16 * (c ^ ((row >> 1) & 7)));
  };
  auto compute = [&](int buf) {
    // Half 0's fragments (activations first), then its MFMAs row by row with
    // half 1's fragment reads issued between them (sched barriers pin the
    // order), then half 1's MFMAs: only half 0's reads are exposed, and at most
    // FN + FM + 2 LDS reads are ever outstanding (the 4-bit lgkmcnt: with more
    // pending, the waitcnt pass can only wait for all of them).
    static_assert(FN + FM + 2 <= 15, "outstanding LDS reads exceed lgkmcnt");
    bf16x8 af[2][FN], bfr[2][FM];
    {
      constexpr int sub = 0;
#pragma unroll
      for (int j = 0; j < FM; ++j) bfr[0][j] = frag(buf, BN + wm * TM + 16 * j + fr, 4 * sub + fq);
#pragma unroll
      for (int i = 0; i < FN; ++i) af[0][i] = frag(buf, wn * TN + 16 * i + fr, 4 * sub + fq);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FN; ++i) {
#pragma unroll
      for (int j = 0; j < FM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[0][j], acc[i][j], 0, 0, 0);
      {
        constexpr int sub = 1;
        af[1][i] = frag(buf, wn * TN + 16 * i + fr, 4 * sub + fq);
        if (i < FM) {
          const int j = i;
          bfr[1][j] = frag(buf, BN + wm * TM + 16 * j + fr, 4 * sub + fq);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = FN; j < FM; ++j) {
      constexpr int sub = 1;
      bfr[1][j] = frag(buf, BN + wm * TM + 16 * j + fr, 4 * sub + fq);
    }
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[1][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  int issued = 0;
#pragma unroll
  for (int q = 0; q < NBUF - 1; ++q)
    if (q < nt) {
      stage(q, kt0 + q);
      ++issued;
    }
  for (int t = 0; t < nt; ++t) {
    // stage t has landed once at most (issued - t - 1) newer stages are pending
    // (up to NBUF - 2 in steady state; fewer in the last iterations)
    const int newer = issued - t - 1;
    if (NBUF >= 4 && newer >= 2) sk_wait_vm<IPW * 2>();
    else if (NBUF >= 3 && newer >= 1) sk_wait_vm<IPW>();
    else sk_wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    // the buffer refilled here was last read in iteration t - 1, which every
    // wave finished before the barrier above
    if (issued < nt) {
      stage(issued % NBUF, kt0 + issued);
      ++issued;
    }
    compute(t % NBUF);
  }

  // ---- split-K: publish this chunk's partial, the tile's last arriver sums them
  if (S > 1) {
    constexpr int PER_WAVE = FN * FM * 256;      // floats per wave partial (16 B per lane per fragment)
    float* mine = p.ws + (((size_t)tile * S + s) * NW + wave) * PER_WAVE;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
        *reinterpret_cast<float4v*>(mine + ((i * FM + j) * 64 + lane) * 4) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds);     // the one LDS array (guide §5 item 4a)
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int t = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == S - 1;
      if (last) __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // fixed chunk order 0..S-1, every partial (this workgroup's own included)
    // read back from the workspace: the sum does not depend on who arrived
    // last, and needs no second accumulator array (the 256 x 256 tile has no
    // registers for one). Loads go in groups of up to 16 fragments.
    constexpr int GI = FM >= 16 ? 1 : (16 / FM < FN ? 16 / FM : FN);
    static_assert(FN % GI == 0, "fragment groups");
    for (int c = 0; c < S; ++c) {
      const float* theirs = p.ws + (((size_t)tile * S + c) * NW + wave) * PER_WAVE;
#pragma unroll
      for (int i0 = 0; i0 < FN; i0 += GI) {
        float4v v[GI][FM];
#pragma unroll
        for (int i = 0; i < GI; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j)
            v[i][j] = *reinterpret_cast<const float4v*>(theirs + (((i0 + i) * FM + j) * 64 + lane) * 4);
#pragma unroll
        for (int i = 0; i < GI; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc[i0 + i][j] = c == 0 ? v[i][j] : acc[i0 + i][j] + v[i][j];
      }
    }
  }

  // ---- epilogue: acc[i][j] = C[n = n0 + TN wn + 16 i + 4 fq + r][m = m0 + TM wm + 16 j + fr]
  bf16_t* Y = reinterpret_cast<bf16_t*>(p.y);
  if constexpr (EPI == SK_SWIGLU) {
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + 16 * j + fr;
      if (m >= M) continue;
#pragma unroll
      for (int i = 0; i < FN / 2; ++i) {
        const int f = (n0 >> 1) + wn * (TN / 2) + 16 * i + 4 * fq;
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float g = bf2f(f2bf(acc[i][j][r])), u = bf2f(f2bf(acc[i + FN / 2][j][r]));
          o[r] = g / (1.f + __expf(-g)) * u;
        }
        *reinterpret_cast<uint2*>(Y + (size_t)m * p.ldy + f) =
            make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
      }
    }
  } else if constexpr (EPI == SK_RESID) {
    float4 bv[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = n0 + wn * TN + 16 * i + 4 * fq;
      bv[i] = p.bias ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + 16 * j + fr;
      if (m >= M) continue;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * TN + 16 * i + 4 * fq;
        uint2* yp = reinterpret_cast<uint2*>(Y + (size_t)m * p.ldy + n);
        const uint2 rv = *yp;
        const float o0 = bf2f(rv.x & 0xffff) + (acc[i][j][0] + bv[i].x);
        const float o1 = bf2f(rv.x >> 16) + (acc[i][j][1] + bv[i].y);
        const float o2 = bf2f(rv.y & 0xffff) + (acc[i][j][2] + bv[i].z);
        const float o3 = bf2f(rv.y >> 16) + (acc[i][j][3] + bv[i].w);
        *yp = make_uint2(pack_bf16x2(o0, o1), pack_bf16x2(o2, o3));
      }
    }
  } else {
    float4 bv[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = n0 + wn * TN + 16 * i + 4 * fq;
      bv[i] = p.bias ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + 16 * j + fr;
      if (m >= M) continue;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * TN + 16 * i + 4 * fq;
        float o[4] = {acc[i][j][0] + bv[i].x, acc[i][j][1] + bv[i].y, acc[i][j][2] + bv[i].z,
                      acc[i][j][3] + bv[i].w};
        if (p.act == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = bf2f(f2bf(o[r]));
            o[r] = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
          }
        }
        *reinterpret_cast<uint2*>(Y + (size_t)m * p.ldy + n) =
            make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
      }
    }
  }
}

template <int WN, int WM, int FN, int FM, int NBUF>
static int sk_launch(const GemmSkParams& p, hipStream_t st) {
  constexpr int BN = 16 * FN * WN, BM = 16 * FM * WM;
  if (p.N % BN || p.K % SK_BK || p.S > p.K / SK_BK) return (int)hipErrorInvalidValue;
  const long long tiles = (long long)((p.M + BM - 1) / BM) * (p.N / BN);
  const long long grid = tiles * p.S;
  if (grid > 0x7fffffff) return (int)hipErrorInvalidValue;
  dim3 block(64 * WN * WM);
  switch (p.epi) {
    case SK_SWIGLU:
      if constexpr (FN % 2 == 0) {
        hipLaunchKernelGGL((gemm_sk_kernel<WN, WM, FN, FM, NBUF, SK_SWIGLU>), dim3(grid), block, 0, st, p);
        break;
      } else {
        return (int)hipErrorInvalidValue;
      }
    case SK_RESID:
      hipLaunchKernelGGL((gemm_sk_kernel<WN, WM, FN, FM, NBUF, SK_RESID>), dim3(grid), block, 0, st, p);
      break;
    default:
      hipLaunchKernelGGL((gemm_sk_kernel<WN, WM, FN, FM, NBUF, SK_BF16>), dim3(grid), block, 0, st, p);
  }
  return (int)hipGetLastError();
}

// layout -> (features BN x rows BM, waves, stages):
//   0: 128 x 128, 2 x 2 waves of 64 x 64, 2 stages (64 KB LDS)
//   1: 128 x  64, 2 x 2 waves of 64 x 32, 2 stages (48 KB)
//   2: 256 x  64, 4 x 1 waves of 64 x 64, 2 stages (80 KB)
//   3: 256 x 128, 4 x 2 waves of 64 x 64, 2 stages (96 KB)
//   4: 128 x  64, 3 stages (72 KB)
//   5: 128 x 128, 3 stages (96 KB)
//   6: 256 x 256, 2 x 4 waves of 128 x 64, 2 stages (128 KB)
//   7:  64 x  64, 2 x 2 waves of 32 x 32, 2 stages (32 KB)
//   8: 256 x  64, 3 stages (120 KB)
//   9: 256 x 128, 3 stages (144 KB): two 48 KB stages in flight per CU
//  10: 128 x 128, 4 stages (128 KB)
//  11: 128 x  64, 4 stages (96 KB)
// (short-K shapes - the Whisper encoder's K = 1280, 20 stages - are bound by
// the bytes one CU keeps in flight: a deeper ring is the lever there)
extern "C" int loqa_gemm_sk(const GemmSkParams* p, hipStream_t st) {
  if (!p || p->M <= 0 || p->S < 1 || p->epi < 0 || p->epi > 2 || !p->x || !p->w || !p->y)
    return (int)hipErrorInvalidValue;
  if (p->S > 1 && (!p->ws || !p->counters)) return (int)hipErrorInvalidValue;
  if (p->ldx % 8 || p->ldy % 4) return (int)hipErrorInvalidValue;
  if ((p->epi == SK_SWIGLU && p->bias) || (p->epi != SK_BF16 && p->act)) return (int)hipErrorInvalidValue;
  switch (p->layout) {
    case 0: return sk_launch<2, 2, 4, 4, 2>(*p, st);
    case 1: return sk_launch<2, 2, 4, 2, 2>(*p, st);
    case 2: return sk_launch<4, 1, 4, 4, 2>(*p, st);
    case 3: return sk_launch<4, 2, 4, 4, 2>(*p, st);
    case 4: return sk_launch<2, 2, 4, 2, 3>(*p, st);
    case 5: return sk_launch<2, 2, 4, 4, 3>(*p, st);
    case 6: return sk_launch<2, 4, 8, 4, 2>(*p, st);
    case 7: return sk_launch<2, 2, 2, 2, 2>(*p, st);
    case 8: return sk_launch<4, 1, 4, 4, 3>(*p, st);
    case 9: return sk_launch<4, 2, 4, 4, 3>(*p, st);
    case 10: return sk_launch<2, 2, 4, 4, 4>(*p, st);
    case 11: return sk_launch<2, 2, 4, 2, 4>(*p, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// tile geometry of a layout (features, rows) for the host-side planner
extern "C" int loqa_gemm_sk_dims(int layout, int* bn, int* bm) {
  static const int dims[12][2] = {{128, 128}, {128, 64}, {256, 64}, {256, 128}, {128, 64},
                                  {128, 128}, {256, 256}, {64, 64}, {256, 64}, {256, 128},
                                  {128, 128}, {128, 64}};
  if (layout < 0 || layout > 11) return (int)hipErrorInvalidValue;
  *bn = dims[layout][0];
  *bm = dims[layout][1];
  return 0;
}
