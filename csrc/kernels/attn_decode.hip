// Decode / jump-forward attention over the paged KV cache.
//
// Decode attention is a pure KV-streaming problem: a few query rows per kv
// head (GQA group x jump-forward tokens <= 32 -> ONE 32-row MFMA tile), so K
// and V must be read exactly once per step and the reads must be in flight
// together. A workgroup = 4 waves = (sequence, kv head, 128-key split); each
// wave owns one 32-key tile, so the whole split's K/V is requested at once
// (no serial tile-after-tile latency chain):
//
//   S^T = K Q^T    : K rows go straight from HBM into the MFMA A fragments
//                    (16 B per lane per k-slice, no LDS); Q^T is register-resident.
//   O^T += V^T P^T : V goes through the wave's private LDS tile and is read with
//                    ds_read_b64_tr_b16 (guide T10); P^T is the exp2'ed S^T
//                    accumulator repacked to bf16 in registers.
//   merge          : the 4 waves' (m, l, O^T) are merged through LDS by wave 0.
//   split combine  : a sequence that fits one split is normalised and written
//                    directly; otherwise wave 0 publishes its split partial
//                    (sc1 write-through stores), takes a ticket on the
//                    (sequence, kv head) counter, and the last arriving split
//                    merges all partials (sc1 loads, fixed split order) and
//                    writes the bf16 output - no second launch (guide §5
//                    "In-launch split-K reduction", §6 Guideline 16).
// Paged block-table entries are wave-uniform per 32-key tile (tiles are
// 32-aligned, blk is a power of two >= 16), so they are scalar loads and the
// K/V addresses need no per-lane dependent lookup.
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
template <int D>
struct DecSmem {
  union {
    bf16_t v[DEC_WAVES][DEC_TILE][D + 32];        // per-wave V tile (padded rows)
    float o[DEC_WAVES - 1][D / 32][16][64];        // O^T partials of waves 1..3
  };
  float ml[DEC_WAVES][2][64];                      // (m, l) per wave per lane
};

// K/V source: paged caches [nb, Hkv, blk, D] via block_tables, or (block_tables
// == nullptr) contiguous rows kc/vc[(kv_start[b] + key) * kv_stride + kvh * D]
// (Whisper cross-attention over the encoder output, read in place).
template <int D, int PF>
__global__ __launch_bounds__(256, 2) void attn_decode_kernel(
    const bf16_t* __restrict__ q, long long q_stride, const bf16_t* __restrict__ kc,
    const bf16_t* __restrict__ vc, long long kv_stride, const int* __restrict__ kv_start,
    const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
    const int* __restrict__ block_tables, int max_blocks, int blk, int Hq, int Hkv,
    float scale_log2, int causal, int split_keys, int num_splits, float* __restrict__ part_o,
    float* __restrict__ part_ml, int total_q, int* __restrict__ counters, bf16_t* __restrict__ out,
    long long o_stride) {
  constexpr int NS = D / 16, NDT = D / 32, CH = D / 8;
  constexpr int VPL = DEC_TILE * CH / 64;  // 16-byte V chunks per lane per tile
  __shared__ __attribute__((aligned(16))) DecSmem<D> sm;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar tile math
  const int h = lane >> 5, r = lane & 31;
  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
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
      uint4 v = row_valid ? *reinterpret_cast<const uint4*>(qr + 16 * s + 8 * h) : make_uint4(0, 0, 0, 0);
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
      const int bn = min((kt + DEC_WAVES * DEC_TILE) / blk, max_blocks - 1);
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
      kraw[s] = ok ? *reinterpret_cast<const uint4*>(kc + off + 16 * s + 8 * h) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      const int kr = c / CH, cc = (c - kr * CH) * 8;
      const int k2 = kt + kr;
      vraw[i] = k2 < kend ? *reinterpret_cast<const uint4*>(vc + row_off(k2) + cc)
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

  constexpr int STEP = DEC_WAVES * DEC_TILE;
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
    for (int w = 1; w < DEC_WAVES; ++w) mstar = fmaxf(mstar, sm.ml[w][0][lane]);
    const float s0 = exp2f(m_run - mstar);
    float l = l_run * s0;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[dt][j] *= s0;
#pragma unroll
    for (int w = 1; w < DEC_WAVES; ++w) {
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
      bf16_t* orow = out + tok * (size_t)o_stride + (size_t)head * D;
      const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          float f[4] = {acc[dt][4 * g4] * inv, acc[dt][4 * g4 + 1] * inv, acc[dt][4 * g4 + 2] * inv,
                        acc[dt][4 * g4 + 3] * inv};
          *reinterpret_cast<uint2*>(orow + 32 * dt + 8 * g4 + 4 * h) = make_uint2(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]));
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
    const int rr = threadIdx.x >> 3, c0 = (threadIdx.x & 7) * CW;
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
    bf16_t* orow = out + tokr * (size_t)o_stride + (size_t)hr * D + c0;
#pragma unroll
    for (int k = 0; k < NV; ++k)
      *reinterpret_cast<uint2*>(orow + 4 * k) =
          make_uint2(pack_bf16x2(o[4 * k] * inv, o[4 * k + 1] * inv),
                     pack_bf16x2(o[4 * k + 2] * inv, o[4 * k + 3] * inv));
  }
}

// q: [Tq, >=Hq*D] bf16; K/V paged caches [nb, Hkv, blk, D] (block_tables) or
// contiguous rows (kv_stride, kv_start); out [Tq, Hq*D] bf16.
// Requires G * max_q <= 32 and split_keys % 32 == 0; counters: >= B * Hkv zeroed ints
// (left zeroed); paged blk a power of two >= 16.
extern "C" int loqa_attn_decode(const void* q, long long q_stride, const void* kc, const void* vc,
                                long long kv_stride, const int* kv_start, void* o,
                                long long o_stride, const int* cu_q, const int* ctx_lens,
                                const int* block_tables, int max_blocks, int blk, int B, int max_q,
                                int Hq, int Hkv, int D, float scale, int causal, int split_keys,
                                int num_splits, float* part_o, float* part_ml, int total_q,
                                int* counters, hipStream_t s) {
  if (B <= 0 || total_q <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv || (Hq / Hkv) * max_q > 32 || split_keys % DEC_TILE || num_splits < 1 ||
      (D != 64 && D != 128) || !part_o || !part_ml || !counters)
    return (int)hipErrorInvalidValue;
  if (block_tables && (blk < 16 || (blk & (blk - 1)))) return (int)hipErrorInvalidValue;
  if (!block_tables && (!kv_start || kv_stride % 8)) return (int)hipErrorInvalidValue;
  dim3 grid(num_splits, Hkv, B);
  const float sl2 = scale * 1.4426950408889634f;
  if (D == 128)
    hipLaunchKernelGGL((attn_decode_kernel<128, 0>), grid, dim3(256), 0, s, (const bf16_t*)q, q_stride,
                       (const bf16_t*)kc, (const bf16_t*)vc, kv_stride, kv_start, cu_q, ctx_lens,
                       block_tables, max_blocks, blk, Hq, Hkv, sl2, causal, split_keys, num_splits,
                       part_o, part_ml, total_q, counters, (bf16_t*)o, o_stride);
  else
    hipLaunchKernelGGL((attn_decode_kernel<64, 0>), grid, dim3(256), 0, s, (const bf16_t*)q, q_stride,
                       (const bf16_t*)kc, (const bf16_t*)vc, kv_stride, kv_start, cu_q, ctx_lens,
                       block_tables, max_blocks, blk, Hq, Hkv, sl2, causal, split_keys, num_splits,
                       part_o, part_ml, total_q, counters, (bf16_t*)o, o_stride);
  return (int)hipGetLastError();
}
