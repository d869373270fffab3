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

__device__ __forceinline__ float16v mfma32(const bf16x8& a, const bf16x8& b, const float16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
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
    const int to = t0 + r;
    const bf16_t* wrow = p.w + (size_t)(co0 + r) * p.K * p.Cin + 8 * kh;
    for (int tap = 0; tap < p.K; ++tap) {
      const int ti = to * p.stride + tap * p.dil - p.pad;
      const bool ok = to < p.Tq && ti >= 0 && ti < p.Tin;
      const bf16_t* xr = xb + (size_t)(ok ? ti : 0) * p.ldx + 8 * kh;
      const bf16_t* wr = wrow + (size_t)tap * p.Cin;
      for (int c = 0; c < p.Cin; c += 16) {
        uint4 av = ok ? *reinterpret_cast<const uint4*>(xr + c) : make_uint4(0, 0, 0, 0);
        const uint4 bv = *reinterpret_cast<const uint4*>(wr + c);
        if (p.pre_act == 1) {
          float f[8];
          unpack8(av, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = f[j] > 0.f ? f[j] : f[j] * p.pre_slope;
          av = pack8(f);
        }
        acc = mfma32(*reinterpret_cast<const bf16x8*>(&av), *reinterpret_cast<const bf16x8*>(&bv), acc);
      }
    }
  }
  // epilogue: C[t][co], lane column co = co0 + (lane & 31), rows t over registers
  const int co = co0 + r;
  const float bias = p.bias ? bf2f(p.bias[co]) : 0.f;
  const int vlen = p.lens ? p.lens[b] : p.Tout;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int trow = t0 + (j & 3) + 8 * (j >> 2) + 4 * kh;
    float v = acc[j] + bias;
    float partner = 0.f;
    if (p.post_act == 3) partner = __shfl_xor(v, 16, 64);
    if (trow >= p.Tq) continue;
    const int oi = trow * p.ostride + p.ophase;
    if (oi < 0 || oi >= p.Tout) continue;
    int oc = co;
    if (p.post_act == 1) {
      v = fmaxf(v, 0.f);
    } else if (p.post_act == 2) {
      v = tanhf(v);
    } else if (p.post_act == 3) {
      if (r & 16) continue;  // sigmoid half: its value was handed to the partner lane
      // bf16-rounded operands, as the unfused model computes them
      const float a = bf2f(f2bf(v)), g = bf2f(f2bf(partner));
      v = tanhf(a) * (1.f / (1.f + __expf(-g)));
      oc = (co0 >> 1) + (r & 15);
    }
    if (oc >= p.cout_real) continue;
    if (p.res) v += bf2f(p.res[(size_t)b * p.rb + (size_t)oi * p.ldr + oc]);
    v *= p.alpha;
    if (p.acc) v += bf2f(p.acc[(size_t)b * p.ab + (size_t)oi * p.lda + oc]);
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
  hipLaunchKernelGGL(conv1d_mfma_kernel, grid, dim3(256), 0, s, p);
  return (int)hipGetLastError();
}
