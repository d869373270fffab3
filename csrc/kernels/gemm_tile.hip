// LDS-tiled MFMA GEMM for large-M projections: Y[M, N] = X[M, K] W[N, K]^T.
//
// Where it runs: the Whisper encoder projections (M =
// 1500 per utterance), the conv stem (k = 3 conv1d as an implicit im2col over
// the time-major input rows), the cross-attention K/V of all decoder layers in
// one launch, and the Llama prompt qkv / gate|up (SwiGLU epilogue). Both
// operands are K-contiguous row-major tensors (nn.Linear weights as loaded, no
// shuffled copy).
//
// Structure (guide §5 "Canonical CDNA GEMM", T1/T2/T4):
//   * workgroup = WN x WM waves, each wave a (16 FN) x (16 FM) output block (FN x FM
//     v_mfma_f32_16x16x32_bf16 tiles, W fragments as the A operand so a lane
//     holds 4 consecutive output features of one row: 8-byte bf16 stores);
//   * BK = 64: one stage = (BN + BM) rows x 128 B, filled by global_load_lds
//     (16 B per lane, 1 KiB per wave instruction). The LDS image is lane-linear,
//     so the bank swizzle is applied on the SOURCE address: row r's 16-byte
//     chunk c lives in slot c ^ ((r >> 1) & 7). A ds_read_b128 of 16 rows at one
//     chunk then touches 16 distinct (half-row, slot) pairs: conflict-free;
//   * NBUF stages, NBUF - 1 in flight: the wait before a stage's barrier is a
//     COUNTED vmcnt (the newer stages' DMAs stay in flight across the raw
//     s_barrier; __syncthreads would drain them);
//   * XCD-aware workgroup order (xcd_remap), m fastest: consecutive workgroups
//     of an XCD share the weight tile in its L2;
//   * split-K S writes f32 slabs [S, M, N] that a slab consumer sums.
#include "common.h"

#define GT_BK 64

enum { GT_BF16 = 0, GT_SLABS = 1, GT_SWIGLU = 2 };

struct GemmTileParams {
  const void* x; long long ldx;   // [M, K] rows (conv: input rows [B * conv_tin, cin], row stride ldx)
  const void* w;                  // [N, K] row-major; SwiGLU: gate rows [0, N/2), up rows [N/2, N)
  int M, N, K, S;
  int epi, act;                   // act: 0 none, 1 GELU (erf)
  const float* bias;              // [N] f32 or null (bf16 / slabs with S == 1)
  const void* pos; int pos_rows;  // bf16 [pos_rows, N] added after act, row m % pos_rows; or null
  void* y; long long ldy;         // bf16 out (SwiGLU: [M, N/2])
  float* part;                    // f32 slabs [S, M, N]
  int conv_cin, conv_tin, conv_tout, conv_stride;  // conv_cin > 0: implicit im2col, k = tap * cin + c
  const void* zeros;              // >= conv_cin zero bf16 (conv taps outside the input)
  int layout;
};

__device__ __forceinline__ void gt_wait_vm(int n) {
  // s_waitcnt vmcnt(n) only (expcnt / lgkmcnt at their maxima), n in 0..63
  // (compile-time at every call site after unrolling)
  switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt(0x0F70); break;
    case 6: __builtin_amdgcn_s_waitcnt(0x0F76); break;
    case 8: __builtin_amdgcn_s_waitcnt(0x0F78); break;
    case 12: __builtin_amdgcn_s_waitcnt(0x0F7C); break;
    case 16: __builtin_amdgcn_s_waitcnt(0x4F70); break;
    default: __builtin_amdgcn_s_waitcnt(0x0F70); break;
  }
}

template <int WN, int WM, int FN, int FM, int NBUF, int EPI, bool CONV>
__global__ __launch_bounds__(64 * WN * WM) void gemm_tile_kernel(GemmTileParams p) {
  constexpr int NW = WN * WM;
  constexpr int TN = 16 * FN, TM = 16 * FM;      // wave tile: TN features x TM rows
  constexpr int BN = TN * WN, BM = TM * WM;
  constexpr int ROWS = BN + BM;
  constexpr int STAGE = ROWS * 128;             // bytes per stage
  constexpr int IPW = ROWS / 8 / NW;            // glds instructions per wave per stage
  static_assert(IPW * 8 * NW == ROWS, "stage rows must split evenly over the waves");
  static_assert(IPW * (NBUF - 2) <= 16, "gt_wait_vm covers 0, 6, 8, 12, 16");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NBUF * STAGE];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int M = p.M, N = p.N;
  const int mblocks = (M + BM - 1) / BM, nblocks = N / BN;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int mb = id % mblocks, rest = id / mblocks;
  const int nb = rest % nblocks, s = rest / nblocks;
  if (s >= p.S) return;
  const int Ks = p.K / p.S, kbeg = s * Ks, nt = Ks / GT_BK;
  const int m0 = mb * BM, n0 = nb * BN;
  const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(p.x);
  const bf16_t* __restrict__ W = reinterpret_cast<const bf16_t*>(p.w);

  // per-lane source of each of this wave's stage instructions (k offset added per stage)
  const bf16_t* src[IPW];
  int cb[IPW], ct[IPW];          // conv: input row of (b, t, tap 0) and t * stride - 1
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int r = 8 * (wave * IPW + i) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    if (r < BN) {
      int row;
      if constexpr (EPI == GT_SWIGLU) {
        // TN-row blocks = one wave's TN / 2 gate + the matching TN / 2 up features
        const int blk = r / TN, rr = r - blk * TN;
        const int f = (n0 >> 1) + blk * (TN / 2) + (rr % (TN / 2));
        row = rr < TN / 2 ? f : (N >> 1) + f;
      } else {
        row = n0 + r;
      }
      src[i] = W + (size_t)row * p.K + c * 8;
      cb[i] = -1;
      ct[i] = 0;
    } else {
      const int m = min(m0 + r - BN, M - 1);
      if constexpr (CONV) {
        const int b = m / p.conv_tout, t = m - b * p.conv_tout;
        cb[i] = b * p.conv_tin;
        ct[i] = t * p.conv_stride - 1;
        src[i] = X + c * 8;
      } else {
        src[i] = X + (size_t)m * p.ldx + c * 8;
        cb[i] = 0;
        ct[i] = 0;
      }
    }
  }

  auto stage = [&](int buf, int kt) {
    const int kc = kbeg + kt * GT_BK;
    int tap = 0, c0 = kc;
    if constexpr (CONV) {
      tap = kc / p.conv_cin;
      c0 = kc - tap * p.conv_cin;
    }
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const bf16_t* g;
      if (CONV && cb[i] >= 0) {
        // conv input rows keep only their 16-byte chunk offset (c * 8) in src;
        // a tap outside [0, T_in) reads the same chunk of the zero row
        const int tt = ct[i] + tap;
        const int c8 = (int)(src[i] - X);
        g = (tt >= 0 && tt < p.conv_tin) ? X + (size_t)(cb[i] + tt) * p.ldx + c0 + c8
                                         : reinterpret_cast<const bf16_t*>(p.zeros) + c8;
      } else {
        g = src[i] + kc;
      }
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)g,
          (__attribute__((address_space(3))) void*)(lds + buf * STAGE + (wave * IPW + i) * 1024), 16, 0, 0);
    }
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
  // both 32-deep halves of the stage are requested before the first MFMA, so
  // the second half's LDS reads are in flight under the first half's MFMAs
  auto compute = [&](int buf) {
    bf16x8 af[2][FN], bfr[2][FM];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
      for (int i = 0; i < FN; ++i) af[sub][i] = frag(buf, wn * TN + 16 * i + fr, 4 * sub + fq);
#pragma unroll
      for (int j = 0; j < FM; ++j) bfr[sub][j] = frag(buf, BN + wm * TM + 16 * j + fr, 4 * sub + fq);
    }
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[sub][i], bfr[sub][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  // prologue: NBUF - 1 stages in flight
  int issued = 0;
#pragma unroll
  for (int q = 0; q < NBUF - 1; ++q)
    if (q < nt) {
      stage(q, q);
      ++issued;
    }
  for (int t = 0; t < nt; ++t) {
    // stage t has landed once at most (issued - t - 1) newer stages are pending
    const int newer = issued - t - 1;
    if (NBUF >= 3 && newer >= 1) gt_wait_vm(IPW * (NBUF - 2));
    else gt_wait_vm(0);
    __builtin_amdgcn_s_barrier();
    // the buffer refilled here was last read in iteration t - 1, which every
    // wave finished before the barrier above
    if (issued < nt) {
      stage(issued % NBUF, issued);
      ++issued;
    }
    compute(t % NBUF);
  }

  // ---- epilogue: acc[i][j] = C[n = n0 + TN wn + 16 i + 4 fq + r][m = m0 + TM wm + 16 j + fr]
  if constexpr (EPI == GT_SWIGLU) {
    bf16_t* Y = reinterpret_cast<bf16_t*>(p.y);
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
  } else if constexpr (EPI == GT_SLABS) {
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + 16 * j + fr;
      if (m >= M) continue;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = n0 + wn * TN + 16 * i + 4 * fq;
        *reinterpret_cast<float4v*>(p.part + ((size_t)s * M + m) * N + n) = acc[i][j];
      }
    }
  } else {
    bf16_t* Y = reinterpret_cast<bf16_t*>(p.y);
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
      const bf16_t* pr = p.pos ? reinterpret_cast<const bf16_t*>(p.pos) + (size_t)(m % p.pos_rows) * N : nullptr;
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
        if (pr) {
          const uint2 pv = *reinterpret_cast<const uint2*>(pr + n);
          o[0] = bf2f(f2bf(o[0])) + bf2f(pv.x & 0xffff);
          o[1] = bf2f(f2bf(o[1])) + bf2f(pv.x >> 16);
          o[2] = bf2f(f2bf(o[2])) + bf2f(pv.y & 0xffff);
          o[3] = bf2f(f2bf(o[3])) + bf2f(pv.y >> 16);
        }
        *reinterpret_cast<uint2*>(Y + (size_t)m * p.ldy + n) =
            make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
      }
    }
  }
}

template <int WN, int WM, int FN, int FM, int NBUF>
static int gt_launch(const GemmTileParams& p, hipStream_t st) {
  constexpr int BN = 16 * FN * WN, BM = 16 * FM * WM;
  if (p.N % BN || p.K % (p.S * GT_BK)) return (int)hipErrorInvalidValue;
  const int grid = ((p.M + BM - 1) / BM) * (p.N / BN) * p.S;
  dim3 block(64 * WN * WM);
  if (p.conv_cin > 0) {
    // the implicit-im2col loader's per-lane row state spills beside the
    // larger wave tiles: conv runs on the 64 x 64 wave tiles only
    if constexpr (FN * FM > 16) return (int)hipErrorInvalidValue;
    else {
      if (p.epi != GT_BF16) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_tile_kernel<WN, WM, FN, FM, NBUF, GT_BF16, true>), dim3(grid), block, 0, st, p);
    }
  } else if (p.epi == GT_SLABS) {
    hipLaunchKernelGGL((gemm_tile_kernel<WN, WM, FN, FM, NBUF, GT_SLABS, false>), dim3(grid), block, 0, st, p);
  } else if (p.epi == GT_SWIGLU) {
    hipLaunchKernelGGL((gemm_tile_kernel<WN, WM, FN, FM, NBUF, GT_SWIGLU, false>), dim3(grid), block, 0, st, p);
  } else {
    hipLaunchKernelGGL((gemm_tile_kernel<WN, WM, FN, FM, NBUF, GT_BF16, false>), dim3(grid), block, 0, st, p);
  }
  return (int)hipGetLastError();
}

// layout (features x rows): 0 128x128 (2x2 waves) 2 stages, 1 128x128 3 stages, 2 256x128 8 waves
// 2 stages, 3 128x256 8 waves 2 stages, 4 256x128 3 stages, 5 128x256 3 stages, 6-9 larger
// wave tiles (below).
extern "C" int loqa_gemm_tile(const GemmTileParams* p, hipStream_t st) {
  if (!p || p->M <= 0 || p->S < 1 || p->epi < 0 || p->epi > 2 || !p->x || !p->w) return (int)hipErrorInvalidValue;
  if (p->epi == GT_SLABS ? !p->part : !p->y) return (int)hipErrorInvalidValue;
  if (p->epi != GT_SLABS && p->S != 1) return (int)hipErrorInvalidValue;
  if (p->ldx % 8 || (p->epi != GT_SLABS && p->ldy % 4)) return (int)hipErrorInvalidValue;
  if (p->epi == GT_SWIGLU && (p->bias || p->pos || p->act)) return (int)hipErrorInvalidValue;
  if (p->pos && p->pos_rows < 1) return (int)hipErrorInvalidValue;
  if (p->conv_cin > 0 && (p->conv_cin % GT_BK || p->K != 3 * p->conv_cin || !p->zeros ||
                          p->conv_tout < 1 || p->conv_stride < 1 || p->M % p->conv_tout))
    return (int)hipErrorInvalidValue;
  switch (p->layout) {
    case 0: return gt_launch<2, 2, 4, 4, 2>(*p, st);
    case 1: return gt_launch<2, 2, 4, 4, 3>(*p, st);
    case 2: return gt_launch<4, 2, 4, 4, 2>(*p, st);
    case 3: return gt_launch<2, 4, 4, 4, 2>(*p, st);
    case 4: return gt_launch<4, 2, 4, 4, 3>(*p, st);
    case 5: return gt_launch<2, 4, 4, 4, 3>(*p, st);
    case 6: return gt_launch<2, 4, 8, 4, 2>(*p, st);   // 256 x 256, wave tile 128 x 64
    case 7: return gt_launch<4, 2, 4, 8, 2>(*p, st);   // 256 x 256, wave tile 64 x 128
    case 8: return gt_launch<2, 2, 8, 4, 2>(*p, st);   // 256 x 128, 4 waves of 128 x 64
    case 9: return gt_launch<2, 2, 4, 8, 2>(*p, st);   // 128 x 256, 4 waves of 64 x 128
    default: return (int)hipErrorInvalidValue;
  }
}
