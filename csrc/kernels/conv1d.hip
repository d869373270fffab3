// Implicit-GEMM 1-D convolution on MFMA for the VITS / HiFi-GAN stack
// (K20 wavenet_gated_conv, K21 conv_transpose1d_upsample via
// polyphase, K22 mrf_resblock convs, K23 tanh_out_pcm16).
//
// Activations are channels-last bf16 [B][T][C] (a row per time step, so a
// 16-channel k-slice of one time step is one 16-byte load). The convolution is
// the GEMM  Y[t][co] = sum_{tap, ci} X[t*stride + tap*dil - pad][ci] * W[co][tap][ci]
// with M = time, N = output channels, K = taps x input channels:
//   * a wave owns a 32(t) x 32(co) tile, v_mfma_f32_32x32x16_bf16, A = input
//     rows (shifted per tap: the sliding window is an address offset, no
//     im2col buffer), B = W^T read straight from the [co][tap][ci] weights;
//   * a workgroup = 4 waves stacked along time (128 x 32), so a weight slice
//     is fetched once per workgroup from L2 and the shifted input rows of
//     neighbouring taps hit L1;
//   * the input pre-activation (leaky ReLU of HiFi-GAN / MRF) is applied to the
//     A fragment in registers, the epilogue fuses bias, ReLU / tanh / the
//     WaveNet gate tanh(a)*sigmoid(b) (channel pairs interleaved in 16-blocks,
//     partner value exchanged across lanes l, l^16), residual add, scale,
//     accumulate (MRF average), length mask and the bf16 or PCM16 store.
//   * transposed convolutions run as `stride` polyphase launches whose output
//     index is to*ostride + ophase.
#include "common.h"

struct ConvArgs {
  const bf16_t* x; long long xb; int ldx;       // input [B][Tin][ldx]
  const bf16_t* w;                               // [Cout_pad][K][Cin]
  const bf16_t* bias;                            // [Cout_pad] or null
  void* y; long long yb; int ldy;                // output [B][Tout_total][ldy]
  const bf16_t* res; long long rb; int ldr;      // added before alpha (same time index as y)
  const bf16_t* acc; long long ab; int lda;      // added after alpha (may alias y)
  const int* lens;                               // valid output length per batch (or null)
  int Tin, Cin, Tq, Cout, K, dil, pad, stride;  // Tq = number of output steps computed
  int ostride, ophase, Tout;                     // y index = to*ostride + ophase, < Tout
  int pre_act; float pre_slope;                  // 0 none, 1 leaky-relu(slope)
  int post_act;                                  // 0 none, 1 relu, 2 tanh, 3 gated
  float alpha;
  int out_pcm16;                                 // y is int16 PCM: clamp(v,-1,1)*32767
  int cout_real;                                 // channels actually stored (gated: of the output)
};

#define CONV_U 8   // K slices per load group

__device__ __forceinline__ float16v mfma32(const bf16x8& a, const bf16x8& b, const float16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Epilogue: C[t][co], lane column co = co0 + (lane & 31), rows t over registers.
__device__ __forceinline__ void conv_epilogue(const ConvArgs& p, const float16v& acc, int b, int t0,
                                              int co0, int lane) {
  const int r = lane & 31, kh = lane >> 5;
  // Two phases: every row's residual / accumulator element is requested first
  // (clamped addresses, one wait), then the values are finished and stored -
  // a load-use pair per row serialised 16 memory round trips per wave.
  const int co = co0 + r;
  const float bias = p.bias ? bf2f(p.bias[co]) : 0.f;
  const int vlen = p.lens ? p.lens[b] : p.Tout;
  int oc = co;
  bool lane_ok = true;
  if (p.post_act == 3) {            // sigmoid half hands its value to the partner lane
    lane_ok = !(r & 16);
    oc = (co0 >> 1) + (r & 15);
  }
  lane_ok = lane_ok && oc < p.cout_real;
  const int occ = lane_ok ? oc : 0;
  float rv[16], cv[16];
  int oix[16];
  unsigned okm = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int trow = t0 + (j & 3) + 8 * (j >> 2) + 4 * kh;
    const int oi = trow * p.ostride + p.ophase;
    const bool ok = lane_ok && trow < p.Tq && oi >= 0 && oi < p.Tout;
    okm |= (unsigned)ok << j;
    oix[j] = ok ? oi : 0;
    rv[j] = 0.f;
    cv[j] = 0.f;
  }
  // one wave-uniform branch per operand around all 16 loads: no join point
  // between a load and the next (a join makes the compiler drain vmcnt)
  if (p.res) {
    const bf16_t* rbase = p.res + (size_t)b * p.rb + occ;
#pragma unroll
    for (int j = 0; j < 16; ++j) rv[j] = bf2f(rbase[(size_t)oix[j] * p.ldr]);
  }
  if (p.acc) {
    const bf16_t* abase = p.acc + (size_t)b * p.ab + occ;
#pragma unroll
    for (int j = 0; j < 16; ++j) cv[j] = bf2f(abase[(size_t)oix[j] * p.lda]);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int trow = t0 + (j & 3) + 8 * (j >> 2) + 4 * kh;
    float v = acc[j] + bias;
    float partner = 0.f;
    if (p.post_act == 3) partner = __shfl_xor(v, 16, 64);
    if (!((okm >> j) & 1)) continue;
    const int oi = trow * p.ostride + p.ophase;
    if (p.post_act == 1) {
      v = fmaxf(v, 0.f);
    } else if (p.post_act == 2) {
      v = tanhf(v);
    } else if (p.post_act == 3) {
      // bf16-rounded operands, as the unfused model computes them
      const float a = bf2f(f2bf(v)), g = bf2f(f2bf(partner));
      v = tanhf(a) * (1.f / (1.f + __expf(-g)));
    }
    v += rv[j];
    v *= p.alpha;
    v += cv[j];
    if (oi >= vlen) v = 0.f;
    if (p.out_pcm16) {
      const float c = fminf(fmaxf(v, -1.f), 1.f);
      reinterpret_cast<short*>(p.y)[(size_t)b * p.yb + (size_t)oi * p.ldy + oc] =
          (short)__float2int_rn(c * 32767.f);
    } else {
      reinterpret_cast<bf16_t*>(p.y)[(size_t)b * p.yb + (size_t)oi * p.ldy + oc] = f2bf(v);
    }
  }
}

__global__ __launch_bounds__(256) void conv1d_mfma_kernel(ConvArgs p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.z;
  const int t0 = (blockIdx.x * 4 + wave) * 32;   // first output step of this wave
  const int co0 = blockIdx.y * 32;
  const int r = lane & 31, kh = lane >> 5;
  const bf16_t* xb = p.x + (size_t)b * p.xb;
  float16v acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  if (t0 < p.Tq) {
    // K slices s = tap * nC + c (16 input channels each), taken CONV_U at a
    // time: every slice's x and w fragments of a group are requested before
    // the group's first MFMA, so CONV_U x 2 16-byte loads per lane are in
    // flight instead of one dependent pair per MFMA (the loop was load-latency
    // bound: 2.4% MFMA busy, profiles/r4_pmc_vits.txt). Same slice order as a
    // plain tap-major loop, so the sums are unchanged. Loads past the end are
    // clamped to the last slice and their MFMAs skipped (wave-uniform).
    const int to = t0 + r;
    const bool tv = to < p.Tq;
    const int tbase = to * p.stride - p.pad;
    const int nC = p.Cin >> 4, KC = p.K * nC;
    const bf16_t* wrow = p.w + (size_t)(co0 + r) * p.K * p.Cin + 8 * kh;
    const bf16_t* xcol = xb + 8 * kh;
    for (int s0 = 0; s0 < KC; s0 += CONV_U) {
      uint4 av[CONV_U], bv[CONV_U];
#pragma unroll
      for (int u = 0; u < CONV_U; ++u) {
        const int sl = min(s0 + u, KC - 1);
        const int tap = sl / nC, c = sl - tap * nC;
        const int ti = tbase + tap * p.dil;
        const bool ok = tv && ti >= 0 && ti < p.Tin;
        const uint4 xv = *reinterpret_cast<const uint4*>(xcol + (size_t)(ok ? ti : 0) * p.ldx + 16 * c);
        av[u] = ok ? xv : make_uint4(0, 0, 0, 0);
        bv[u] = *reinterpret_cast<const uint4*>(wrow + (size_t)tap * p.Cin + 16 * c);
      }
#pragma unroll
      for (int u = 0; u < CONV_U; ++u) {
        if (s0 + u >= KC) break;          // wave-uniform
        uint4 a = av[u];
        if (p.pre_act == 1) {
          float f[8];
          unpack8(a, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = f[j] > 0.f ? f[j] : f[j] * p.pre_slope;
          a = pack8(f);
        }
        acc = mfma32(*reinterpret_cast<const bf16x8*>(&a), *reinterpret_cast<const bf16x8*>(&bv[u]), acc);
      }
    }
  }
  conv_epilogue(p, acc, b, t0, co0, lane);
}

// LDS-staged form for stride-1 convolutions (every VITS conv: the polyphase
// transposed convolutions run stride 1 with an output stride): the workgroup's
// 128 output steps need input rows [t0 - pad, t0 + 128 + (K - 1) * dil - pad)
// of each CC-channel chunk, staged ONCE in LDS (pre-activation applied while
// staging) and read by all 4 waves at every tap's shifted offset; the
// 32 x K x CC weight slice is staged once too. The register form above re-reads
// each input row K times per wave and the weights once per wave from L1 / L2
// (~1 GB of operand traffic for one 76 800-row HiFi-GAN conv: 2.3% MFMA busy,
// profiles/r4_pmc_vits.txt). Rows are padded by 16 B so a wave's 32 lanes,
// reading 16 B each at a fixed row stride, do not all hit the same banks.
// Same K-slice order (tap-major, then channel) as the register form.
template <int CC>
__global__ __launch_bounds__(256) void conv1d_lds_kernel(ConvArgs p) {
  constexpr int XS = CC + 8;                     // padded row (bf16 elements)
  constexpr int NC16 = CC / 16;
  extern __shared__ __attribute__((aligned(16))) bf16_t conv_smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.z;
  const int tw0 = blockIdx.x * 128;              // first output step of the workgroup
  const int t0 = tw0 + wave * 32;                // this wave's
  const int co0 = blockIdx.y * 32;
  const int r = lane & 31, kh = lane >> 5;
  const int R = 128 + (p.K - 1) * p.dil;         // staged input rows per chunk
  bf16_t* xs = conv_smem;                        // [R][XS]
  bf16_t* ws = conv_smem + (size_t)R * XS;       // [32 * K][XS]
  const bf16_t* xb = p.x + (size_t)b * p.xb;
  const int row0 = tw0 - p.pad;                  // input row of staged row 0
  float16v acc;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  // A chunk's operands go global -> registers -> LDS: every 16-byte piece of
  // the chunk is requested before any is stored (a load-store pair per loop
  // trip serialised one memory round trip per trip, 4-8 per chunk), and the
  // NEXT chunk's pieces are requested right after this chunk's are stored, so
  // their latency hides under this chunk's MFMAs (staged rows R <= 256 and
  // K <= 16, checked on the host).
  constexpr int PPR = NC16 * 2;                  // 16-byte pieces per staged row
  constexpr int XMAX = PPR;                      // 256 rows x PPR pieces / 256 threads
  constexpr int WMAX = 16 * PPR / 8;             // 32 x 16 taps x PPR pieces / 256 threads
  const int nx = R * PPR, nw = 32 * p.K * PPR;
  uint4 xv[XMAX], wv[WMAX];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int j = 0; j < XMAX; ++j) {
      const int i = threadIdx.x + j * 256;
      const int row = i / PPR, piece = i - row * PPR;
      const int ti = row0 + row;
      xv[j] = (i < nx && ti >= 0 && ti < p.Tin)
                  ? *reinterpret_cast<const uint4*>(xb + (size_t)ti * p.ldx + c0 + 8 * piece)
                  : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < WMAX; ++j) {
      const int i = threadIdx.x + j * 256;
      const int rowk = i / PPR, piece = i - rowk * PPR;
      const int co = rowk / p.K, tap = rowk - co * p.K;
      wv[j] = i < nw ? *reinterpret_cast<const uint4*>(
                           p.w + ((size_t)(co0 + co) * p.K + tap) * p.Cin + c0 + 8 * piece)
                     : make_uint4(0, 0, 0, 0);
    }
  };
  load_chunk(0);
  for (int c0 = 0; c0 < p.Cin; c0 += CC) {
    __syncthreads();                             // previous chunk's reads are done
    // input rows: R x CC bf16, pre-activation applied while storing
#pragma unroll
    for (int j = 0; j < XMAX; ++j) {
      const int i = threadIdx.x + j * 256;
      if (i < nx) {
        const int row = i / PPR, piece = i - row * PPR;
        uint4 v = xv[j];
        if (p.pre_act == 1) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = f[q] > 0.f ? f[q] : f[q] * p.pre_slope;
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(xs + (size_t)row * XS + 8 * piece) = v;
      }
    }
    // weights: 32 output channels x K taps x CC
#pragma unroll
    for (int j = 0; j < WMAX; ++j) {
      const int i = threadIdx.x + j * 256;
      if (i < nw) {
        const int rowk = i / PPR, piece = i - rowk * PPR;
        *reinterpret_cast<uint4*>(ws + (size_t)rowk * XS + 8 * piece) = wv[j];
      }
    }
    if (c0 + CC < p.Cin) load_chunk(c0 + CC);    // lands during this chunk's MFMAs
    __syncthreads();
    if (t0 < p.Tq) {
      const bf16_t* xl = xs + (size_t)(wave * 32 + r) * XS + 8 * kh;
      const bf16_t* wl = ws + (size_t)r * p.K * XS + 8 * kh;
      for (int tap = 0; tap < p.K; ++tap) {
        const bf16_t* xt = xl + (size_t)tap * p.dil * XS;
        const bf16_t* wt = wl + (size_t)tap * XS;
#pragma unroll
        for (int c = 0; c < NC16; ++c) {
          const uint4 av = *reinterpret_cast<const uint4*>(xt + 16 * c);
          const uint4 bv = *reinterpret_cast<const uint4*>(wt + 16 * c);
          acc = mfma32(*reinterpret_cast<const bf16x8*>(&av), *reinterpret_cast<const bf16x8*>(&bv), acc);
        }
      }
    }
  }
  if (t0 < p.Tq) conv_epilogue(p, acc, b, t0, co0, lane);
}

extern "C" int loqa_conv1d(const void* x, long long xb, int ldx, const void* w, const void* bias,
                           void* y, long long yb, int ldy, const void* res, long long rb, int ldr,
                           const void* acc, long long ab, int lda, const int* lens, int B, int Tin,
                           int Cin, int Tq, int Cout, int K, int dil, int pad, int stride,
                           int ostride, int ophase, int Tout, int pre_act, float pre_slope,
                           int post_act, float alpha, int out_pcm16, int cout_real,
                           hipStream_t s) {
  if (B <= 0 || Tq <= 0) return 0;
  if (Cin % 16 || Cout % 32 || ldx % 8 || K < 1 || stride < 1 || ostride < 1 ||
      (post_act == 3 && out_pcm16))
    return (int)hipErrorInvalidValue;
  ConvArgs p{(const bf16_t*)x, xb, ldx, (const bf16_t*)w, (const bf16_t*)bias, y, yb, ldy,
             (const bf16_t*)res, rb, ldr, (const bf16_t*)acc, ab, lda, lens, Tin, Cin, Tq, Cout,
             K, dil, pad, stride, ostride, ophase, Tout, pre_act, pre_slope, post_act, alpha,
             out_pcm16, cout_real};
  dim3 grid((Tq + 127) / 128, Cout / 32, B);
  if (stride == 1 && Cin % 32 == 0 && 128 + (K - 1) * dil <= 256 && K <= 16) {
    // LDS form: 64-channel chunks when the staged rows + weight slice fit in
    // 64 KiB (two workgroups per CU), else 32-channel chunks
    const int R = 128 + (K - 1) * dil;
    auto lds_of = [&](int cc) { return (size_t)(R + 32 * K) * (cc + 8) * sizeof(bf16_t); };
    if (Cin % 64 == 0 && lds_of(64) <= 64 * 1024) {
      hipLaunchKernelGGL(conv1d_lds_kernel<64>, grid, dim3(256), lds_of(64), s, p);
      return (int)hipGetLastError();
    }
    if (lds_of(32) <= 64 * 1024) {
      hipLaunchKernelGGL(conv1d_lds_kernel<32>, grid, dim3(256), lds_of(32), s, p);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL(conv1d_mfma_kernel, grid, dim3(256), 0, s, p);
  return (int)hipGetLastError();
}
