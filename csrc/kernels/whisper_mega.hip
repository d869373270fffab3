// Whisper decoder step as ONE persistent launch (docs/PERF.md
// open item "Whisper decoder: 256 dependent launches per step").
//
// The fused path runs 8 dependent kernels per layer (qkv, self-attention, o,
// xq, cross-attention, xo, fc1, fc2): 256 launches per step, each one
// latency-bound (~3 MB of weights for a few token rows). Here the whole layer
// stack is a static work list executed by G persistent workgroups:
//
//   work item  = (layer, phase, index); phases per layer:
//     0 qkv   : LayerNorm ln1 (recomputed per item from the residual rows) ->
//               16 output features -> bias -> q rows / paged K,V append
//     1 self  : (sequence, head) causal attention over the paged cache
//     2 o     : 16 features of attn @ Wo^T + bias, added into the residual
//     3 xq    : LayerNorm lnx -> 16 features of the cross-attention query
//     4 cross : (sequence, head, 256-key split) over the encoder K|V rows, the
//               last arriving split merges the partials (fixed order)
//     5 xo    : residual += cross @ Wxo^T + bias
//     6 fc1   : LayerNorm ln2 -> 16 features -> bias -> GELU(erf)
//     7 fc2   : residual += m @ Wfc2^T + bias
//   item i runs on workgroup i % G, in increasing i. An item of phase p waits
//   until every item of phase p - 1 has signalled (one agent-scope counter per
//   (layer, phase)). BEFORE waiting it issues its dependency-free loads: its
//   weight fragments (GEMM items) or its encoder K/V rows (cross items), so the
//   HBM round trip overlaps the previous phase's tail.
//
// Deadlock freedom without co-residency: a workgroup only ever waits for items
// with a smaller index, which belong to workgroups that are resident or will
// be (nothing waits on this kernel), and every spin is bounded (error flag).
// Data handed between workgroups (residual, q, attention outputs, GELU
// activations, new K/V rows, split partials) is stored and loaded with sc1
// (device-coherent) buffer operations, as in the in-launch split-K reductions
// of gemm_skinny.hip; counters are relaxed agent atomics after vmcnt(0).
//
// GEMMs: v_mfma_f32_16x16x32_bf16 with the pre-shuffled weights of
// ops.shuffle_weight as the A operand (16 features x 32 k per fragment) and the
// token rows as the B operand; the 4 waves split K and reduce through LDS.
#include "common.h"

#define MP 16            // token rows per step (Mpad)
#define HD 64            // head dim
#define NPH 8            // phases per layer
#define SC1 16           // buffer-op cache policy bit: device-coherent
#define PF 10            // weight k-steps per wave in flight
#define XSK 256          // cross-attention keys per split (4 waves x 64)

typedef unsigned u32x4m __attribute__((ext_vector_type(4)));
typedef unsigned u32x2m __attribute__((ext_vector_type(2)));
typedef float f4m __attribute__((ext_vector_type(4)));

struct MegaLayer {
  const bf16_t* w[6];    // shuffled weights: qkv, o, xq, xo, fc1, fc2
  const bf16_t* b[6];    // biases (same order)
  const bf16_t* ln[6];   // ln1 w, b; lnx w, b; ln2 w, b
  bf16_t* kc;            // paged self-attention cache [nb, H, blk, HD]
  bf16_t* vc;
  const bf16_t* xkv;     // encoder rows [rows, 2d]: K | V
};

struct MegaParams {
  const MegaLayer* layers; int L;
  bf16_t* x;             // [MP, d] residual (in / out)
  bf16_t* qb;            // [MP, d] self-attention queries
  bf16_t* ab;            // [MP, d] attention output (self, then cross)
  bf16_t* xqb;           // [MP, d] cross-attention queries
  bf16_t* mb;            // [MP, ffn] GELU activations
  float* part;           // [B, H, nsplit, MP, 66] cross-attention split partials
  int* sync;             // err (sticky) | [L * NPH] done counters | [B * H] tickets (zeroed per step)
  const int* slots;      // [MP] cache slot per token row (-1: padding)
  const int* cu_q;       // [B + 1]
  const int* ctx_lens;   // [B]
  const int* block_tables;
  int max_blocks, blk;
  const int* enc_starts; // [B] first encoder row
  const int* enc_lens;   // [B]
  int B, d, H, ffn, nsplit;
  int kv_bytes;          // bytes of one layer's K (= V) cache
  float eps, scale_log2;
  long long* dbg;        // optional [items, 5] s_memrealtime stamps (profiling)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4m ld_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, SC1);
}
__device__ __forceinline__ u32x4m ldw(const bf16_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4m*>(p));
}
__device__ __forceinline__ float lo_bf(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

struct MegaSmem {
  union {
    bf16_t act[MP][1280 + 8];                 // LayerNorm'ed rows (K = d <= 1280)
    struct {
      bf16_t vs[4][64][HD + 8];               // per-wave V chunk
      float ps[4][MP][64];                    // per-wave probabilities
      float qs[MP][HD];                       // scaled queries
      float os[4][MP][HD];                    // per-wave O for the merge
      float ms[4][MP], ls[4][MP];
    } at;
  };
  float red[4][64][4];                        // GEMM cross-wave reduction
  long long ts[5];                            // profiling stamps (thread 0)
};

__device__ __forceinline__ void phase_counts(const MegaParams& p, int* n) {
  n[0] = 3 * p.d / 16; n[1] = p.B * p.H; n[2] = p.d / 16; n[3] = p.d / 16;
  n[4] = p.B * p.H * p.nsplit; n[5] = p.d / 16; n[6] = p.ffn / 16; n[7] = p.d / 16;
}

// thread 0 spins (bounded) until *c >= target; the barrier releases the rest
__device__ void wait_for(int* c, int target, int* err) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 21)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// every thread's sc1 stores are complete before the counter moves
__device__ void signal_done(int* c) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ GEMM item
// 16 output features [tile * 16, +16) for the MP token rows.
// LN: input = LayerNorm(x rows) staged in LDS (K = d); else input rows are read
// sc1 straight into the B fragments.
__device__ f4m gemm_item(const MegaParams& p, MegaSmem& sm, const bf16_t* Wp, int K, int tile,
                         bool ln, const bf16_t* in, int in_ld, const bf16_t* lnw,
                         const bf16_t* lnb, int* wait_c, int wait_n, int* err) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int KS = K >> 5, KSW = KS >> 2, ks0 = wave * KSW;
  const bf16_t* wbase = Wp + ((size_t)tile * KS + ks0) * 512 + lane * 8;
  u32x4m wf[PF];
#pragma unroll
  for (int u = 0; u < PF; ++u) wf[u] = ldw(wbase + (size_t)min(u, KSW - 1) * 512);
  if (wait_c) wait_for(wait_c, wait_n, err);
  if (threadIdx.x == 0) sm.ts[1] = __builtin_amdgcn_s_memrealtime();
  const auto rin = rsrc(in, (unsigned)(MP * in_ld * 2));
  if (ln) {
    // thread t: row t >> 4, 16 threads per row, d / 16 contiguous elements each
    const int row = threadIdx.x >> 4, seg = threadIdx.x & 15;
    const int per = K >> 4, nv = per >> 3;
    u32x4m xv[10];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      xv[i] = i < nv ? ld_sc1(rin, (unsigned)((row * in_ld + seg * per + i * 8) * 2)) : u32x4m{0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j) s += lo_bf(xv[i][j]) + hi_bf(xv[i][j]);
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)K;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 10; ++i)
      if (i < nv)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float a = lo_bf(xv[i][j]) - mean, b = hi_bf(xv[i][j]) - mean;
          ss += a * a + b * b;
        }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) ss += __shfl_xor(ss, o, 64);
    const float rstd = rsqrtf(ss / (float)K + p.eps);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (i < nv) {
      const int k0 = seg * per + i * 8;
      const uint4 wv = *reinterpret_cast<const uint4*>(lnw + k0);
      const uint4 bv = *reinterpret_cast<const uint4*>(lnb + k0);
      const unsigned wu[4] = {wv.x, wv.y, wv.z, wv.w}, bu[4] = {bv.x, bv.y, bv.z, bv.w};
      unsigned o4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = (lo_bf(xv[i][j]) - mean) * rstd * lo_bf(wu[j]) + lo_bf(bu[j]);
        const float b = (hi_bf(xv[i][j]) - mean) * rstd * hi_bf(wu[j]) + hi_bf(bu[j]);
        o4[j] = pack_bf16x2(a, b);
      }
      *reinterpret_cast<uint4*>(&sm.act[row][k0]) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) sm.ts[2] = __builtin_amdgcn_s_memrealtime();
  f4m acc = {0.f, 0.f, 0.f, 0.f};
  const int t = lane & 15, kq = 8 * (lane >> 4);
  for (int c = 0; c < KSW; c += PF) {
    if (c > 0) {
#pragma unroll
      for (int u = 0; u < PF; ++u) wf[u] = ldw(wbase + (size_t)min(c + u, KSW - 1) * 512);
    }
    u32x4m xf[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int k = (ks0 + min(c + u, KSW - 1)) * 32 + kq;
      if (ln) {
        const uint4 v = *reinterpret_cast<const uint4*>(&sm.act[t][k]);
        xf[u] = u32x4m{v.x, v.y, v.z, v.w};
      } else {
        xf[u] = ld_sc1(rin, (unsigned)((t * in_ld + k) * 2));
      }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (c + u < KSW)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[u]),
                                                      __builtin_bit_cast(bf16x8, xf[u]), acc, 0, 0, 0);
  }
  // 4 waves (K quarters) -> wave 0
#pragma unroll
  for (int r = 0; r < 4; ++r) sm.red[wave][lane][r] = acc[r];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int w = 1; w < 4; ++w)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += sm.red[w][lane][r];
  }
  return acc;   // wave 0: features tile*16 + (lane>>4)*4 + r, token lane & 15
}

// ------------------------------------------------------------ attention item
// one wave's 64-key chunk: lane = key; K row in kr, V row staged to LDS
__device__ __forceinline__ void attn_chunk(MegaSmem& sm, int wave, int lane, const u32x4m (&kr)[8],
                                           const u32x4m (&vr)[8], bool key_ok, int key, int qlen,
                                           bool causal, int qpos0, float (&m)[MP], float (&l)[MP],
                                           float (&o)[MP]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    *reinterpret_cast<uint4*>(&sm.at.vs[wave][lane][8 * i]) = make_uint4(vr[i][0], vr[i][1], vr[i][2], vr[i][3]);
#pragma unroll
  for (int i = 0; i < MP; ++i) {
    if (i < qlen) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        s += sm.at.qs[i][8 * c + 2 * j] * lo_bf(kr[c][j]) + sm.at.qs[i][8 * c + 2 * j + 1] * hi_bf(kr[c][j]);
    const bool ok = key_ok && (!causal || key <= qpos0 + i);
    s = ok ? s : -INFINITY;
    const float mx = wave_max(s);
    const float mn = fmaxf(m[i], mx);
    const float alpha = exp2f(m[i] - mn);
    const float pe = ok ? exp2f(s - mn) : 0.f;
    l[i] = l[i] * alpha + wave_sum(pe);
    m[i] = mn;
    sm.at.ps[wave][i][lane] = pe;
    o[i] *= alpha;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int i = 0; i < MP; ++i) {
    if (i < qlen) {
      float a = 0.f;
#pragma unroll 8
      for (int k = 0; k < 64; ++k) a += sm.at.ps[wave][i][k] * bf2f(sm.at.vs[wave][k][lane]);
      o[i] += a;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ void attn_item(const MegaParams& p, MegaSmem& sm, const MegaLayer& Lw, bool cross,
                          int b, int h, int sp, int* wait_c, int wait_n, int* err) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int d = p.d, q0 = p.cu_q[b], qlen = min(p.cu_q[b + 1] - q0, MP);
  u32x4m kr[8], vr[8];
  int kbeg = 0, kend = 0, key = 0;
  if (cross) {
    // encoder K / V rows do not depend on this step: request them before waiting
    kbeg = sp * XSK;
    kend = min(p.enc_lens[b], kbeg + XSK);
    key = kbeg + wave * 64 + lane;
    const bool ok = key < kend;
    const bf16_t* kp = Lw.xkv + (size_t)(p.enc_starts[b] + (ok ? key : kbeg)) * (2 * d) + h * HD;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      kr[i] = ok ? *reinterpret_cast<const u32x4m*>(kp + 8 * i) : u32x4m{0, 0, 0, 0};
      vr[i] = ok ? *reinterpret_cast<const u32x4m*>(kp + d + 8 * i) : u32x4m{0, 0, 0, 0};
    }
  }
  wait_for(wait_c, wait_n, err);
  if (threadIdx.x == 0) sm.ts[1] = __builtin_amdgcn_s_memrealtime();
  const int nsplit = cross ? max(1, min(p.nsplit, (p.enc_lens[b] + XSK - 1) / XSK)) : 1;
  if (qlen <= 0 || sp >= nsplit) return;
  // scaled queries -> LDS
  {
    const bf16_t* qsrc = cross ? p.xqb : p.qb;
    const auto rq = rsrc(qsrc, (unsigned)(MP * d * 2));
    for (int e = threadIdx.x; e < qlen * (HD / 8); e += 256) {
      const int i = e / (HD / 8), c = e % (HD / 8);
      const u32x4m v = ld_sc1(rq, (unsigned)(((q0 + i) * d + h * HD + 8 * c) * 2));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sm.at.qs[i][8 * c + 2 * j] = lo_bf(v[j]) * p.scale_log2;
        sm.at.qs[i][8 * c + 2 * j + 1] = hi_bf(v[j]) * p.scale_log2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) sm.ts[2] = __builtin_amdgcn_s_memrealtime();
  float m[MP], l[MP], o[MP];
#pragma unroll
  for (int i = 0; i < MP; ++i) { m[i] = -1e30f; l[i] = 0.f; o[i] = 0.f; }
  if (cross) {
    attn_chunk(sm, wave, lane, kr, vr, key < kend, key, qlen, false, 0, m, l, o);
  } else {
    const int ctx = p.ctx_lens[b];
    const auto rk = rsrc(Lw.kc, (unsigned)p.kv_bytes), rv = rsrc(Lw.vc, (unsigned)p.kv_bytes);
    const int* bt = p.block_tables + (size_t)b * p.max_blocks;
    for (int c0 = wave * 64; c0 < ctx; c0 += 256) {
      const int kk = c0 + lane;
      const bool ok = kk < ctx;
      const int kc = ok ? kk : c0;
      const int bid = bt[kc / p.blk];
      const unsigned off = (unsigned)((((size_t)bid * p.H + h) * p.blk + (kc % p.blk)) * HD * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        kr[i] = ld_sc1(rk, off + 16 * i);
        vr[i] = ld_sc1(rv, off + 16 * i);
      }
      attn_chunk(sm, wave, lane, kr, vr, ok, kk, qlen, true, ctx - qlen, m, l, o);
    }
  }
  // merge the 4 waves (fixed order)
#pragma unroll
  for (int i = 0; i < MP; ++i) {
    if (i < qlen) {
      sm.at.os[wave][i][lane] = o[i];
      if (lane == 0) { sm.at.ms[wave][i] = m[i]; sm.at.ls[wave][i] = l[i]; }
    }
  }
  __syncthreads();
  if (wave != 0) return;
  const auto rp = rsrc(p.part, (unsigned)(p.B * p.H * p.nsplit * MP * 66 * 4));
  const auto ro = rsrc(p.ab, (unsigned)(MP * d * 2));
  for (int i = 0; i < qlen; ++i) {
    float M = -1e30f;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, sm.at.ms[w][i]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float sc = exp2f(sm.at.ms[w][i] - M);
      L += sm.at.ls[w][i] * sc;
      O += sm.at.os[w][i][lane] * sc;
    }
    if (nsplit == 1) {
      const float y = L > 0.f ? O / L : 0.f;
      __builtin_amdgcn_raw_buffer_store_b16(f2bf(y), ro, (unsigned)(((q0 + i) * d + h * HD + lane) * 2), 0, SC1);
    } else {
      const unsigned base = (unsigned)(((((b * p.H + h) * p.nsplit + sp) * MP + i) * 66) * 4);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(O), rp, base + (2 + lane) * 4, 0, SC1);
      if (lane == 0) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(M), rp, base, 0, SC1);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(L), rp, base + 4, 0, SC1);
      }
    }
  }
  if (nsplit == 1) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int* tk = p.sync + 1 + p.L * NPH + b * p.H + h;
  int t = 0;
  if (lane == 0) {
    t = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == nsplit - 1) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  t = __shfl(t, 0, 64);
  if (t != nsplit - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int i = 0; i < qlen; ++i) {
    float M = -1e30f;
    for (int s2 = 0; s2 < nsplit; ++s2) {
      const unsigned base = (unsigned)(((((b * p.H + h) * p.nsplit + s2) * MP + i) * 66) * 4);
      M = fmaxf(M, __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, base, 0, SC1)));
    }
    float L = 0.f, O = 0.f;
    for (int s2 = 0; s2 < nsplit; ++s2) {
      const unsigned base = (unsigned)(((((b * p.H + h) * p.nsplit + s2) * MP + i) * 66) * 4);
      const float ms = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, base, 0, SC1));
      const float ls = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, base + 4, 0, SC1));
      const float os = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, base + (2 + lane) * 4, 0, SC1));
      const float sc = exp2f(ms - M);
      L += ls * sc;
      O += os * sc;
    }
    const float y = L > 0.f ? O / L : 0.f;
    __builtin_amdgcn_raw_buffer_store_b16(f2bf(y), ro, (unsigned)(((q0 + i) * d + h * HD + lane) * 2), 0, SC1);
  }
}

// ------------------------------------------------------------------- kernel
__global__ __launch_bounds__(256, 1) void whisper_mega_kernel(MegaParams p) {
  __shared__ __attribute__((aligned(16))) MegaSmem sm;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int n[NPH];
  phase_counts(p, n);
  int C = 0;
#pragma unroll
  for (int i = 0; i < NPH; ++i) C += n[i];
  const int total = C * p.L;
  int* err = p.sync;
  int* done = p.sync + 1;
  const int d = p.d;
  for (int it = blockIdx.x; it < total; it += gridDim.x) {
    const int l = it / C;
    int r = it - l * C, ph = 0, wait_n = n[NPH - 1];
#pragma unroll
    for (int i = 0; i < NPH - 1; ++i)   // unrolled: n[] stays in registers
      if (ph == i && r >= n[i]) { r -= n[i]; ph = i + 1; wait_n = n[i]; }
    if (threadIdx.x == 0) sm.ts[0] = sm.ts[1] = sm.ts[2] = __builtin_amdgcn_s_memrealtime();
    const MegaLayer& Lw = p.layers[l];
    int* wait_c = ph > 0 ? done + l * NPH + ph - 1 : (l > 0 ? done + (l - 1) * NPH + NPH - 1 : nullptr);
    if (ph == 1 || ph == 4) {
      const int bh = ph == 1 ? r : r / p.nsplit;
      attn_item(p, sm, Lw, ph == 4, bh / p.H, bh % p.H, ph == 4 ? r % p.nsplit : 0, wait_c, wait_n, err);
    } else {
      const int wi = ph == 0 ? 0 : ph == 2 ? 1 : ph == 3 ? 2 : ph == 5 ? 3 : ph == 6 ? 4 : 5;
      const bool ln = ph == 0 || ph == 3 || ph == 6;
      const int K = ph == 7 ? p.ffn : d;
      const bf16_t* in = ln ? p.x : ph == 7 ? p.mb : p.ab;
      const int in_ld = ph == 7 ? p.ffn : d;
      const bf16_t* lnw = ln ? Lw.ln[ph == 0 ? 0 : ph == 3 ? 2 : 4] : nullptr;
      const bf16_t* lnb = ln ? Lw.ln[ph == 0 ? 1 : ph == 3 ? 3 : 5] : nullptr;
      const f4m acc = gemm_item(p, sm, Lw.w[wi], K, r, ln, in, in_ld, lnw, lnb, wait_c, wait_n, err);
      if (wave == 0) {
        const int f0 = r * 16 + (lane >> 4) * 4, t = lane & 15;
        const bf16_t* bias = Lw.b[wi];
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[j] + bf2f(bias[f0 + j]);
        const u32x2m pk = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
        if (ph == 0) {
          if (f0 < d) {
            __builtin_amdgcn_raw_buffer_store_b64(pk, rsrc(p.qb, MP * d * 2), (unsigned)((t * d + f0) * 2), 0, SC1);
          } else {
            const int s = p.slots[t];
            if (s >= 0) {
              const int fk = f0 - (f0 < 2 * d ? d : 2 * d);
              const int hh = fk / HD, dd = fk % HD;
              const unsigned off = (unsigned)((((size_t)(s / p.blk) * p.H + hh) * p.blk + (s % p.blk)) * HD + dd) * 2;
              __builtin_amdgcn_raw_buffer_store_b64(pk, rsrc(f0 < 2 * d ? Lw.kc : Lw.vc, (unsigned)p.kv_bytes),
                                                    off, 0, SC1);
            }
          }
        } else if (ph == 3) {
          __builtin_amdgcn_raw_buffer_store_b64(pk, rsrc(p.xqb, MP * d * 2), (unsigned)((t * d + f0) * 2), 0, SC1);
        } else if (ph == 6) {
          float g[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) g[j] = 0.5f * v[j] * (1.f + erff(v[j] * 0.70710678118654752f));
          const u32x2m gk = {pack_bf16x2(g[0], g[1]), pack_bf16x2(g[2], g[3])};
          __builtin_amdgcn_raw_buffer_store_b64(gk, rsrc(p.mb, MP * p.ffn * 2), (unsigned)((t * p.ffn + f0) * 2), 0, SC1);
        } else {   // residual phases 2, 5, 7
          const auto rx = rsrc(p.x, MP * d * 2);
          const unsigned off = (unsigned)((t * d + f0) * 2);
          const u32x2m xo = __builtin_amdgcn_raw_buffer_load_b64(rx, off, 0, SC1);
          const u32x2m nk = {pack_bf16x2(v[0] + lo_bf(xo[0]), v[1] + hi_bf(xo[0])),
                             pack_bf16x2(v[2] + lo_bf(xo[1]), v[3] + hi_bf(xo[1]))};
          __builtin_amdgcn_raw_buffer_store_b64(nk, rx, off, 0, SC1);
        }
      }
    }
    if (threadIdx.x == 0) sm.ts[3] = __builtin_amdgcn_s_memrealtime();
    signal_done(done + l * NPH + ph);
    if (p.dbg && threadIdx.x == 0) {
      sm.ts[4] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
      for (int k = 0; k < 5; ++k) p.dbg[(size_t)it * 5 + k] = sm.ts[k];
    }
  }
}

extern "C" int loqa_whisper_mega(const MegaParams* hp, int grid, hipStream_t s) {
  const MegaParams& p = *hp;
  if (p.L <= 0 || p.B <= 0 || p.H * HD != p.d || p.d % 128 || p.d > 1280 || p.ffn % 128 ||
      p.ffn > 4 * 1280 || p.nsplit < 1 || p.blk <= 0 || grid <= 0 || !p.sync || !p.layers)
    return (int)hipErrorInvalidValue;
  // counters and tickets restart every step; the error word stays set
  const size_t sync_bytes = (size_t)(p.L * NPH + p.B * p.H) * sizeof(int);
  hipError_t e = hipMemsetAsync(p.sync + 1, 0, sync_bytes, s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(whisper_mega_kernel, dim3(grid), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}
