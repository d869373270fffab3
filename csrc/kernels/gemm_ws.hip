// Row-resident weight-streaming MFMA GEMM for prompt passes:
// Y[M, N] = X[M, K] W[N, K]^T with M up to a few hundred rows (one prefill pass
// of the intent decoder: ~300 - 1200 prompt tokens).
//
// At M ~ 300 a projection is bounded by streaming its weights (gate|up: 235 MB,
// ~45 us at HBM speed) about as much as by its MFMA work, and a square output
// tile either pads M badly (128-row tiles: 384 rows for 300) or re-reads every
// weight tile once per row block. Here a workgroup owns BN = 128 output
// features x ALL the pass's rows (BM = M rounded up to 64, at most 384), so
// every weight byte is read from HBM exactly once and the only re-read operand
// is the small activation block (L2-resident). 8 waves = 2 (features) x 4
// (rows); a wave computes 64 features x BM / 4 rows with 16x16x32 bf16 MFMAs.
//
// The two operands have different latencies, so they are staged at different
// depths (guide §5 "Pipelining across barriers"): weight K-stages (16 KB, from
// HBM) NBW deep, activation K-stages (BM x 128 B, from L2) NBX deep, all by
// global_load_lds with the bank swizzle on the source address, issued
// activation-first so ONE counted vmcnt per step (the newest weight stage may
// stay in flight) retires both; raw s_barrier, never __syncthreads in the loop.
// Both 32-deep halves of a step's fragments are requested before its first MFMA.
//
// Epilogues as gemm_sk.hip: bf16 (+ f32 bias, GELU), SwiGLU (a wave's 64
// features = 32 gate + the matching 32 up rows, permuted at staging), residual
// add in place (+ bias), one rounding.
//
// Split-K (S > 1): the K range is cut into S chunks, each its own workgroup,
// summed inside the launch by the tile's last arriving chunk (gemm_sk.hip's
// protocol: partial stores -> vmcnt(0) -> agent release -> relaxed ticket; the
// last arriver takes an agent acquire and adds the S partials in fixed chunk
// order). A workgroup's operand ingestion is (BM + 128) x K/S: at ~300 rows
// the activation block dominates it, so fewer K per workgroup is what lets
// more workgroups than 128-feature tiles share the pass (down: 32 tiles x 8
// chunks). Chunk-major workgroup order: the workgroups of one K chunk (one
// activation slice, L2-resident) run together.
#include "common.h"

#define WS_BK 64

enum { WS_BF16 = 0, WS_SWIGLU = 1, WS_RESID = 2 };

struct GemmWsParams {
  const void* x; long long ldx;   // [M, K] bf16 rows
  const void* w;                  // [N, K] bf16 row-major (SwiGLU: gate rows [0, N/2), up [N/2, N))
  int M, N, K;
  int epi, act;                   // act (WS_BF16): 1 GELU (erf) after the bias
  const float* bias;              // [N] f32 or null (bf16 / resid)
  void* y; long long ldy;         // bf16 output (WS_RESID: the residual, updated in place)
  int bm;                         // rows per workgroup (multiple of 64, <= 64 * FM of the launch)
  int S;                          // K chunks (>= 1)
  float* ws;                      // S > 1: [tiles][S][bm * 128] f32 partials
  int* counters;                  // S > 1: [tiles] ints, zero on entry (left zero)
};

template <int N>
__device__ __forceinline__ void ws_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int FM, int NBW, int NBX, int EPI>
__global__ __launch_bounds__(512) void gemm_ws_kernel(GemmWsParams p) {
  constexpr int WN = 2, WM = 4, NW = 8, FN = 4;
  constexpr int TN = 16 * FN, TM = 16 * FM;      // wave tile: 64 features x TM rows
  constexpr int BN = TN * WN, BM = TM * WM;      // 128 x 64 FM
  constexpr int WSTAGE = BN * 128, XSTAGE = BM * 128;
  constexpr int IW = BN / 8 / NW;                // glds per wave per weight stage (2)
  constexpr int IX = BM / 8 / NW;                // glds per wave per activation stage (FM)
  static_assert(IW * 8 * NW == BN && IX * 8 * NW == BM, "stage rows split evenly over the waves");
  static_assert(NBW >= 2 && NBX >= 2 && NBX <= NBW, "stage depths");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NBW * WSTAGE + NBX * XSTAGE];
  unsigned char* const wl = lds;
  unsigned char* const xl = lds + NBW * WSTAGE;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int M = p.M, N = p.N;
  const int mblocks = (M + p.bm - 1) / p.bm;
  const int tiles = mblocks * (N / BN), S = p.S;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int s = id / tiles, tile = id - s * tiles;
  const int mb = tile % mblocks, nb = tile / mblocks;   // a weight tile's row blocks adjacent
  const int m0 = mb * p.bm, n0 = nb * BN;
  const int KT = p.K / WS_BK;
  const int kt0 = (int)(((long long)s * KT) / S), kt1 = (int)(((long long)(s + 1) * KT) / S);
  const int nt = kt1 - kt0;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ W = reinterpret_cast<const bf16_t*>(p.w);

  const bf16_t* wsrc[IW];
#pragma unroll
  for (int i = 0; i < IW; ++i) {
    const int r = 8 * (wave * IW + i) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    int row;
    if constexpr (EPI == WS_SWIGLU) {
      const int blk = r / TN, rr = r - blk * TN;
      const int f = (n0 >> 1) + blk * (TN / 2) + (rr % (TN / 2));
      row = rr < TN / 2 ? f : (N >> 1) + f;
    } else {
      row = n0 + r;
    }
    wsrc[i] = W + (size_t)row * p.K + (size_t)kt0 * WS_BK + c * 8;
  }
  const bf16_t* xsrc[IX];
#pragma unroll
  for (int i = 0; i < IX; ++i) {
    const int r = 8 * (wave * IX + i) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int m = min(m0 + min(r, p.bm - 1), M - 1);
    xsrc[i] = X + (size_t)m * p.ldx + (size_t)kt0 * WS_BK + c * 8;
  }
  auto stage_w = [&](int kt) {
    unsigned char* dst = wl + (kt % NBW) * WSTAGE;
#pragma unroll
    for (int i = 0; i < IW; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + kt * WS_BK),
                                       (__attribute__((address_space(3))) void*)(dst + (wave * IW + i) * 1024),
                                       16, 0, 0);
  };
  auto stage_x = [&](int kt) {
    unsigned char* dst = xl + (kt % NBX) * XSTAGE;
#pragma unroll
    for (int i = 0; i < IX; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xsrc[i] + kt * WS_BK),
                                       (__attribute__((address_space(3))) void*)(dst + (wave * IX + i) * 1024),
                                       16, 0, 0);
  };

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto frag = [&](const unsigned char* base, int row, int c) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(base + row * 128 + 16 * (c ^ ((row >> 1) & 7)));
  };
  auto compute = [&](int kt) {
    const unsigned char* wb = wl + (kt % NBW) * WSTAGE;
    const unsigned char* xb = xl + (kt % NBX) * XSTAGE;
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
      for (int j = 0; j < FM; ++j) bfr[0][j] = frag(xb, wm * TM + 16 * j + fr, 4 * sub + fq);
#pragma unroll
      for (int i = 0; i < FN; ++i) af[0][i] = frag(wb, wn * TN + 16 * i + fr, 4 * sub + fq);
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
        af[1][i] = frag(wb, wn * TN + 16 * i + fr, 4 * sub + fq);
        if (i < FM) {
          const int j = i;
          bfr[1][j] = frag(xb, wm * TM + 16 * j + fr, 4 * sub + fq);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = FN; j < FM; ++j) {
      constexpr int sub = 1;
      bfr[1][j] = frag(xb, wm * TM + 16 * j + fr, 4 * sub + fq);
    }
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[1][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // Issue order, one virtual step v at a time: X(v + NBX - 1), then
  // W(v + NBW - 1). vmcnt retires in issue order, so at the top of step t the
  // wait is for the later-issued of X(t) / W(t); what was issued after it may
  // stay in flight: with NBX = 2 < NBW = 3 that is W(t + 1) (weights get two
  // steps of cover, activations one), with NBX = NBW = 3 it is X(t + 1) and
  // W(t + 1) (two steps for both). Near the end those stages do not exist.
  static_assert(NBW == 3 && (NBX == 2 || NBX == 3), "the counted waits below assume these depths");
  for (int v = -(NBW - 1); v < 0; ++v) {
    if (v + NBX - 1 >= 0 && v + NBX - 1 < nt) stage_x(v + NBX - 1);
    if (v + NBW - 1 < nt) stage_w(v + NBW - 1);
  }
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) {
      if constexpr (NBX == 2) ws_wait_vm<IW>();
      else ws_wait_vm<IW + IX>();
    } else {
      ws_wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    // the buffers refilled here were last read in step t - 1, which every
    // wave finished before the barrier above
    if (t + NBX - 1 < nt) stage_x(t + NBX - 1);
    if (t + NBW - 1 < nt) stage_w(t + NBW - 1);
    compute(t);
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
    int* flag = reinterpret_cast<int*>(lds);     // every wave is past its last LDS read
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
    // fixed chunk order 0..S-1, this workgroup's own partial read back too:
    // the sum does not depend on which chunk arrived last
    constexpr int GI = 16 / FM >= FN ? FN : (16 / FM >= 2 ? 2 : 1);
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
  const int mend = min(M, m0 + p.bm);
  if constexpr (EPI == WS_SWIGLU) {
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + 16 * j + fr;
      if (m >= mend) continue;
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
      if (m >= mend) continue;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * TN + 16 * i + 4 * fq;
        uint2* yp = reinterpret_cast<uint2*>(Y + (size_t)m * p.ldy + n);
        float o[4] = {acc[i][j][0] + bv[i].x, acc[i][j][1] + bv[i].y, acc[i][j][2] + bv[i].z,
                      acc[i][j][3] + bv[i].w};
        if constexpr (EPI == WS_RESID) {
          const uint2 rv = *yp;
          o[0] += bf2f(rv.x & 0xffff);
          o[1] += bf2f(rv.x >> 16);
          o[2] += bf2f(rv.y & 0xffff);
          o[3] += bf2f(rv.y >> 16);
        } else if (p.act == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = bf2f(f2bf(o[r]));
            o[r] = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
          }
        }
        *yp = make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
      }
    }
  }
}

template <int FM, int NBW, int NBX>
static int ws_launch(const GemmWsParams& p, hipStream_t st) {
  const int grid = ((p.M + p.bm - 1) / p.bm) * (p.N / 128) * p.S;
  switch (p.epi) {
    case WS_SWIGLU:
      hipLaunchKernelGGL((gemm_ws_kernel<FM, NBW, NBX, WS_SWIGLU>), dim3(grid), dim3(512), 0, st, p);
      break;
    case WS_RESID:
      hipLaunchKernelGGL((gemm_ws_kernel<FM, NBW, NBX, WS_RESID>), dim3(grid), dim3(512), 0, st, p);
      break;
    default:
      hipLaunchKernelGGL((gemm_ws_kernel<FM, NBW, NBX, WS_BF16>), dim3(grid), dim3(512), 0, st, p);
  }
  return (int)hipGetLastError();
}

// depth: 0 = (weight stages 3, activation stages 2), 1 = (3, 3); the LDS of
// (3 * 16 KB + NBX * bm * 128 B) must fit 160 KB (depth 1: bm <= 256).
extern "C" int loqa_gemm_ws(const GemmWsParams* p, int depth, hipStream_t st) {
  if (!p || p->M <= 0 || p->epi < 0 || p->epi > 2 || !p->x || !p->w || !p->y) return (int)hipErrorInvalidValue;
  if (p->N % 128 || p->K % WS_BK || p->K < WS_BK || p->ldx % 8 || p->ldy % 4 || p->bm < 64 || p->bm % 64 ||
      p->bm > 384 || depth < 0 || depth > 1 || p->S < 1 || p->S > p->K / WS_BK)
    return (int)hipErrorInvalidValue;
  if (p->S > 1 && (!p->ws || !p->counters)) return (int)hipErrorInvalidValue;
  if ((p->epi == WS_SWIGLU && (p->bias || p->act)) || (p->epi == WS_RESID && p->act))
    return (int)hipErrorInvalidValue;
  const int fm = p->bm / 64;
  if (depth == 1) {
    switch (fm) {
      case 1: return ws_launch<1, 3, 3>(*p, st);
      case 2: return ws_launch<2, 3, 3>(*p, st);
      case 3: return ws_launch<3, 3, 3>(*p, st);
      case 4: return ws_launch<4, 3, 3>(*p, st);
      default: return (int)hipErrorInvalidValue;
    }
  }
  switch (fm) {
    case 1: return ws_launch<1, 3, 2>(*p, st);
    case 2: return ws_launch<2, 3, 2>(*p, st);
    case 3: return ws_launch<3, 3, 2>(*p, st);
    case 4: return ws_launch<4, 3, 2>(*p, st);
    case 5: return ws_launch<5, 3, 2>(*p, st);
    case 6: return ws_launch<6, 3, 2>(*p, st);
    default: return (int)hipErrorInvalidValue;
  }
}
