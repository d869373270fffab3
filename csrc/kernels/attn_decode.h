// Decode / jump-forward attention over the paged KV cache: the shared body of
// attn_decode.hip's kernel and of the fused qkv + attention launch
// (gemm_skinny.hip, ATTN mode). Design notes: attn_decode.hip.
#pragma once
#include "common.h"

#define DEC_TILE 32
#define DEC_WAVES 4

typedef short v4s_ __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float16v mfma32d(const bf16x8& a, const bf16x8& b, const float16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// The V tiles are dead once the key loop ends, so the merge buffer aliases them:
// 51 KB (D = 128) instead of 92 KB lets three workgroups share a CU, so a
// 512-workgroup grid is resident in one round instead of two.
// NW waves per workgroup (4; 8 for the single-pass form, see attn_decode.hip)
template <int D, int NW = DEC_WAVES>
struct DecSmem {
  union {
    bf16_t v[NW][DEC_TILE][D + 32];               // per-wave V tile (padded rows)
    float o[NW - 1][D / 32][16][64];               // O^T partials of waves 1..NW-1
  };
  float ml[NW][2][64];                             // (m, l) per wave per lane
};

// K/V source: paged caches [nb, Hkv, blk, D] via block_tables, or (block_tables
// == nullptr) contiguous rows kc/vc[(kv_start[b] + key) * kv_stride + kvh * D]
// (Whisper cross-attention over the encoder output, read in place).
// Kernel arguments (one struct: the same body runs as its own launch and as
// the attention phase of the fused qkv GEMM, gemm_skinny.hip).
struct AttnDecArgs {
  const bf16_t* q; long long q_stride; const bf16_t* kc; const bf16_t* vc; long long kv_stride;
  const int* kv_start; const int* cu_q; const int* ctx_lens; const int* block_tables;
  int max_blocks, blk, Hq, Hkv; float scale_log2; int causal, split_keys, num_splits;
  float* part_o; float* part_ml; int total_q; int* counters; bf16_t* out; long long o_stride;
  // SC1 bodies (the fused GEMM's attention workers): byte sizes of q and of
  // one K (= V) cache, for the write-through-coherent buffer loads
  long long q_bytes, kv_bytes;
  int prio;      // wave issue priority of the launch (loqa_set_launch_prio), 0 = default
  long long o_bytes;   // bytes of out (OSC1 write-through stores)
};

// Launch priority of the calling host thread: kernels launched (or captured)
// by a thread that set it run their waves at s_setprio 3, so a latency-bound
// decoder sharing the CUs with a bandwidth-bound one wins the per-SIMD issue
// arbitration (MI355X_MICROARCH.md: priority, then age). Thread-local: the
// STT and LLM schedulers launch from their own threads.
extern thread_local int g_loqa_launch_prio;

// 16-byte load; SC1: a buffer load with the sc1 policy (reads what another
// workgroup stored write-through in this launch, without an L2-invalidating
// acquire fence - guide §6 Guideline 16)
template <int SC1>
__device__ __forceinline__ uint4 ld16(const bf16_t* base, size_t elem, long long nbytes) {
  if constexpr (SC1) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(base), 0, (int)nbytes, 0x00020000);
    const u32x4_ v = __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(elem * 2), 0, 16);
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const uint4*>(base + elem);
  }
}

// One workgroup's work item (split, kv head, sequence) - the body of the
// standalone kernel, whose grid is (splits, kv heads, sequences); 256
// threads, 4 waves.
// output store: plain, or write-through (OSC1: the attention runs as a
// prologue item of the GEMM that consumes its output in the same launch)
template <int OSC1>
__device__ __forceinline__ void st_attn_out(bf16_t* base, long long nbytes, size_t elem, uint2 v) {
  if constexpr (OSC1) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)nbytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2_{v.x, v.y}, r, (unsigned)(elem * 2), 0, 16);
  } else {
    *reinterpret_cast<uint2*>(base + elem) = v;
  }
}

template <int D, int PF, int LOOP = 0, int SC1 = 0, int NW = DEC_WAVES, int OSC1 = 0>
__device__ __forceinline__ void attn_decode_body(const AttnDecArgs& A, const int split, const int kvh,
                                                 const int b, DecSmem<D, NW>& sm) {
  const bf16_t* __restrict__ q = A.q;
  const long long q_stride = A.q_stride;
  const bf16_t* __restrict__ kc = A.kc;
  const bf16_t* __restrict__ vc = A.vc;
  const long long kv_stride = A.kv_stride;
  const int* __restrict__ kv_start = A.kv_start;
  const int* __restrict__ cu_q = A.cu_q;
  const int* __restrict__ ctx_lens = A.ctx_lens;
  const int* __restrict__ block_tables = A.block_tables;
  const int max_blocks = A.max_blocks, blk = A.blk, Hq = A.Hq, Hkv = A.Hkv;
  const float scale_log2 = A.scale_log2;
  const int causal = A.causal, split_keys = A.split_keys, num_splits = A.num_splits;
  float* __restrict__ part_o = A.part_o;
  float* __restrict__ part_ml = A.part_ml;
  const int total_q = A.total_q;
  int* __restrict__ counters = A.counters;
  bf16_t* __restrict__ out = A.out;
  const long long o_stride = A.o_stride;
  // LOOP: the thread index through an opaque move: when this body runs in a loop
  // (the fused qkv GEMM's attention workers) the compiler would otherwise
  // hoist every lane-dependent address term out of the loop and hold them all
  // in VGPRs across it (+90 VGPRs, spills at D = 128)
  int tid = threadIdx.x;
  if constexpr (LOOP) asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
  constexpr int NS = D / 16, NDT = D / 32, CH = D / 8;
  constexpr int VPL = DEC_TILE * CH / 64;  // 16-byte V chunks per lane per tile
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar tile math
  const int h = lane >> 5, r = lane & 31;
  const int G = Hq / Hkv;
  const bool paged = block_tables != nullptr;
  const int* bt = paged ? block_tables + (size_t)b * max_blocks : nullptr;
  // the first tile's block-table entries do not depend on the context length:
  // request them (clamped in-row) together with the sequence metadata below,
  // so the first K/V loads wait for one scalar round trip instead of two
  int nbt0 = 0, nbt1 = 0;
  {
    const int bi = min((split * split_keys + wave * DEC_TILE) / blk, max_blocks - 1);
    if (paged) {
      nbt0 = bt[bi];
      nbt1 = bt[min(bi + 1, max_blocks - 1)];
    }
  }
  const int q0 = cu_q[b], qlen = cu_q[b + 1] - q0;
  const int klen = ctx_lens[b];
  const int qi = r / G;
  const int head = kvh * G + (r - qi * G);
  const bool row_valid = qi < qlen && r < (32 / G) * G;
  const int qpos = klen - qlen + qi;
  const int kbeg = split * split_keys;
  const int kend = min(klen, kbeg + split_keys);
  // splits past the context contribute nothing: leave before any load (the
  // combine only reads the first ceil(klen / split_keys) splits). The grid is
  // sized for the longest context a captured graph can see, so most of these
  // workgroups would otherwise occupy a CU for a full pass.
  if (split > 0 && kbeg >= klen) return;
  const size_t kv0 = paged ? 0 : (size_t)kv_start[b];

  bf16x8 qf[NS];
  {
    const bf16_t* qr = q + (size_t)(q0 + (row_valid ? qi : 0)) * q_stride + (size_t)head * D;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint4 v = row_valid ? ld16<SC1>(q, (size_t)(qr - q) + 16 * s + 8 * h, A.q_bytes)
                          : make_uint4(0, 0, 0, 0);
      qf[s] = *reinterpret_cast<bf16x8*>(&v);
    }
  }
  float16v acc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  float m_run = -1e30f, l_run = 0.f;

  // the tile's (at most two) cache blocks: wave-uniform scalar lookups
  // nbt0 / nbt1 hold the block-table entries of tile kt on entry; the next
  // tile's (kt + 4 * 32) are requested before this tile's K / V so the lookup
  // is off the loop's dependent chain
  auto load_tile = [&](int kt, uint4 (&kraw)[NS], uint4 (&vraw)[VPL]) {
    int base0 = 0, base1 = 0, bi0 = 0;
    if (paged) {
      bi0 = kt / blk;
      base0 = nbt0;
      base1 = (blk < DEC_TILE && bi0 + 1 < max_blocks) ? nbt1 : base0;
      const int bn = min((kt + NW * DEC_TILE) / blk, max_blocks - 1);
      nbt0 = bt[bn];
      nbt1 = bt[min(bn + 1, max_blocks - 1)];
    }
    auto row_off = [&](int key) -> size_t {
      if (paged) {
        const int local = key - bi0 * blk;
        const int bid = local >= blk ? base1 : base0;
        return (((size_t)bid * Hkv + kvh) * blk + (local & (blk - 1))) * D;
      }
      return (kv0 + key) * (size_t)kv_stride + (size_t)kvh * D;
    };
    const int key = kt + r;
    const bool ok = key < kend;
    const size_t off = row_off(ok ? key : kt);
#pragma unroll
    for (int s = 0; s < NS; ++s)
      kraw[s] = ok ? (SC1 && paged ? ld16<SC1>(kc, off + 16 * s + 8 * h, A.kv_bytes)
                                   : ld16<0>(kc, off + 16 * s + 8 * h, 0))
                   : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      const int kr = c / CH, cc = (c - kr * CH) * 8;
      const int k2 = kt + kr;
      vraw[i] = k2 < kend ? (SC1 && paged ? ld16<SC1>(vc, row_off(k2) + cc, A.kv_bytes)
                                          : ld16<0>(vc, row_off(k2) + cc, 0))
                          : make_uint4(0, 0, 0, 0);
    }
  };

  auto process_tile = [&](int kt, uint4 (&kraw)[NS], uint4 (&vraw)[VPL]) {
    // S^T = K Q^T
    float16v st;
#pragma unroll
    for (int j = 0; j < 16; ++j) st[j] = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) st = mfma32d(*reinterpret_cast<bf16x8*>(&kraw[s]), qf[s], st);
    // V tile -> this wave's LDS region (wave-private: no workgroup barrier)
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      const int kr = c / CH, cc = (c - kr * CH) * 8;
      *reinterpret_cast<uint4*>(&sm.v[wave][kr][cc]) = vraw[i];
    }
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int key = kt + (j & 3) + 8 * (j >> 2) + 4 * h;
      float sv = st[j] * scale_log2;
      if (key >= kend || (causal && key > qpos)) sv = -INFINITY;
      st[j] = sv;
      mx = fmaxf(mx, sv);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    float ls = 0.f;
    bf16x8 pf[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = exp2f(st[8 * s2 + j] - m_new);
        ls += e;
        pf[s2][j] = (__bf16)e;
      }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < NDT; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[i][j] *= alpha;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int g = lane >> 4, li = lane & 15;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int c0 = 32 * dt + 16 * (g & 1) + 4 * (li & 3);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int kb = 16 * s2 + 4 * h + (li >> 2);
        const v4s_ lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s_*)(&sm.v[wave][kb][c0]));
        const v4s_ hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s_*)(&sm.v[wave][kb + 8][c0]));
        short8 a8;
        a8[0] = lo[0]; a8[1] = lo[1]; a8[2] = lo[2]; a8[3] = lo[3];
        a8[4] = hi[0]; a8[5] = hi[1]; a8[6] = hi[2]; a8[7] = hi[3];
        acc[dt] = mfma32d(*reinterpret_cast<bf16x8*>(&a8), pf[s2], acc[dt]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };

  constexpr int STEP = NW * DEC_TILE;
  int kt = kbeg + wave * DEC_TILE;
  if constexpr (PF) {
    // ping-pong: the next tile's K / V are requested before this tile is
    // consumed (a key split longer than 4 tiles otherwise pays one memory
    // round trip per tile). The prefetch is unconditional (clamped to the
    // current tile past the end) so no join point drains it (see stream_k).
    // Measured on the Whisper cross-attention (1500 keys, 3-12 splits): no
    // gain at 512-key splits and a loss at shorter ones (183 vs 120 VGPRs
    // halves occupancy), so both head dims launch PF = 0. (The ISA shows why
    // it cannot gain as written: the per-lane predicated loads and the
    // run-time paged / contiguous branch put every consumer behind a join,
    // so the waitcnt pass drains the prefetch - only vmcnt(0) waits. A
    // version with clamped unconditional loads, a compile-time PAGED flag and
    // a peeled ping-pong got partial waits but measured 10-60% slower: the
    // allocator then recycles the in-flight buffers' registers as MFMA
    // destinations, which forces early waits.)
    uint4 ka[NS], va[VPL], kb[NS], vb[VPL];
    if (kt < kend) load_tile(kt, ka, va);
    while (kt < kend) {
      load_tile(kt + STEP < kend ? kt + STEP : kt, kb, vb);
      process_tile(kt, ka, va);
      kt += STEP;
      if (kt >= kend) break;
      load_tile(kt + STEP < kend ? kt + STEP : kt, ka, va);
      process_tile(kt, kb, vb);
      kt += STEP;
    }
  } else {
    for (; kt < kend; kt += STEP) {
      uint4 kraw[NS], vraw[VPL];
      load_tile(kt, kraw, vraw);
      process_tile(kt, kraw, vraw);
    }
  }

  // ---- merge the 4 waves' online-softmax states through LDS (o aliases v: every
  // wave must be done reading its V tile before any wave writes its O^T)
  __syncthreads();
  sm.ml[wave][0][lane] = m_run;
  sm.ml[wave][1][lane] = l_run;
  if (wave > 0) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int j = 0; j < 16; ++j) sm.o[wave - 1][dt][j][lane] = acc[dt][j];
  }
  __syncthreads();
  const int nsplit = min(num_splits, max(1, (klen + split_keys - 1) / split_keys));
  if (wave == 0) {
    float mstar = m_run;
#pragma unroll
    for (int w = 1; w < NW; ++w) mstar = fmaxf(mstar, sm.ml[w][0][lane]);
    const float s0 = exp2f(m_run - mstar);
    float l = l_run * s0;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[dt][j] *= s0;
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float sw = exp2f(sm.ml[w][0][lane] - mstar);
      l += sm.ml[w][1][lane] * sw;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[dt][j] += sw * sm.o[w - 1][dt][j][lane];
    }
    const size_t tok = (size_t)(q0 + qi);
    if (nsplit == 1) {
      if (!row_valid) return;
      const size_t orow = tok * (size_t)o_stride + (size_t)head * D;
      const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          float f[4] = {acc[dt][4 * g4] * inv, acc[dt][4 * g4 + 1] * inv, acc[dt][4 * g4 + 2] * inv,
                        acc[dt][4 * g4 + 3] * inv};
          st_attn_out<OSC1>(out, A.o_bytes, orow + 32 * dt + 8 * g4 + 4 * h,
                            make_uint2(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3])));
        }
      return;
    }
    // publish this split's partial write-through, then take a ticket
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(
        part_o, 0, (int)((size_t)num_splits * total_q * Hq * D * 4), 0x00020000);
    const auto rm = __builtin_amdgcn_make_buffer_rsrc(
        part_ml, 0, (int)((size_t)num_splits * total_q * Hq * 2 * 4), 0x00020000);
    const int row = (int)tok * Hq + head;
    if (row_valid) {
      const int ob = (split * total_q * Hq + row) * D * 4;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4v v = {acc[dt][4 * g4], acc[dt][4 * g4 + 1], acc[dt][4 * g4 + 2], acc[dt][4 * g4 + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_, v), ro,
                                                 ob + (32 * dt + 8 * g4 + 4 * h) * 4, 0, 16);
        }
      if (h == 0) {
        const float2 ml = make_float2(mstar, l);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_, ml), rm,
                                              (split * total_q * Hq + row) * 8, 0, 16);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int* cnt = counters + (size_t)b * Hkv + kvh;
    if (lane == 0) {
      const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == nsplit - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sm.ml[0][0][0] = __int_as_float(t);
    }
  }
  if (nsplit == 1) return;
  __syncthreads();
  if (__float_as_int(sm.ml[0][0][0]) != nsplit - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // Last split: the WHOLE workgroup merges every split's partial (split
  // order fixed, sc1 loads only). Thread t owns row t / 8 of the 32-row tile
  // and D / 8 of its columns; each batch's loads are all issued before any is
  // consumed (a rolled loop pays one L2 round trip per split).
  {
    constexpr int CW = D / 8, NV = CW / 4;     // columns / float4 per thread
    constexpr int MLB = 16, OB = 16 / NV;      // (m, l) pairs / partials per batch
    const int rr = tid >> 3, c0 = (tid & 7) * CW;
    const int qr = rr / G;
    if (!(qr < qlen && rr < (32 / G) * G)) return;
    const int hr = kvh * G + (rr - qr * G);
    const size_t tokr = (size_t)(q0 + qr);
    const int row = (int)tokr * Hq + hr;
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(
        part_o, 0, (int)((size_t)num_splits * total_q * Hq * D * 4), 0x00020000);
    const auto rm = __builtin_amdgcn_make_buffer_rsrc(
        part_ml, 0, (int)((size_t)num_splits * total_q * Hq * 2 * 4), 0x00020000);
    // the first batch of partials is requested together with the (m, l)
    // pairs: one L2 round trip before the first accumulate, not two
    auto load_o = [&](int sp0, float4v (&v)[OB][NV]) {
#pragma unroll
      for (int i = 0; i < OB; ++i) {
        const int sp = sp0 + i < nsplit ? sp0 + i : 0;
#pragma unroll
        for (int k = 0; k < NV; ++k)
          v[i][k] = __builtin_bit_cast(float4v, __builtin_amdgcn_raw_buffer_load_b128(
                                                    ro, ((sp * total_q * Hq + row) * D + c0 + 4 * k) * 4, 0, 16));
      }
    };
    float4v v[OB][NV];
    load_o(0, v);
    float msx = -1e30f;
    float2 mlr[MLB];
    for (int sp0 = 0; sp0 < nsplit; sp0 += MLB) {
#pragma unroll
      for (int i = 0; i < MLB; ++i)
        mlr[i] = sp0 + i < nsplit
                     ? __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(
                                                      rm, ((sp0 + i) * total_q * Hq + row) * 8, 0, 16))
                     : make_float2(-1e30f, 0.f);
#pragma unroll
      for (int i = 0; i < MLB; ++i) msx = fmaxf(msx, mlr[i].x);
    }
    const bool ml_cached = nsplit <= MLB;
    float o[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) o[c] = 0.f;
    float L = 0.f;
    for (int sp0 = 0; sp0 < nsplit; sp0 += OB) {
      if (sp0 > 0) load_o(sp0, v);
#pragma unroll
      for (int i = 0; i < OB; ++i) {
        const int sp = sp0 + i;
        if (sp >= nsplit) break;
        float2 ml = make_float2(-1e30f, 0.f);
        if (ml_cached) {
#pragma unroll
          for (int q2 = 0; q2 < MLB; ++q2)
            if (q2 == sp) ml = mlr[q2];
        } else {
          ml = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(
                                              rm, (sp * total_q * Hq + row) * 8, 0, 16));
        }
        const float w = exp2f(ml.x - msx);
        L += w * ml.y;
#pragma unroll
        for (int k = 0; k < NV; ++k)
#pragma unroll
          for (int e = 0; e < 4; ++e) o[4 * k + e] += w * v[i][k][e];
      }
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    const size_t orow = tokr * (size_t)o_stride + (size_t)hr * D + c0;
#pragma unroll
    for (int k = 0; k < NV; ++k)
      st_attn_out<OSC1>(out, A.o_bytes, orow + 4 * k,
                        make_uint2(pack_bf16x2(o[4 * k] * inv, o[4 * k + 1] * inv),
                                   pack_bf16x2(o[4 * k + 2] * inv, o[4 * k + 3] * inv)));
  }
}

