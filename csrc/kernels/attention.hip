// Flash attention forward for CDNA4.
//
// One kernel family covers every attention in the hub:
//   * PREFILL mode  - 128 query rows of ONE head per workgroup (Whisper encoder,
//                     Llama prompt prefill, VITS text encoder). Causal or not.
//                     Served by attn_prefill2_kernel below (8 waves, key range
//                     split between two wave groups); LOQA_ATTN_V1=1 selects
//                     the original 4-wave attn_fwd_kernel.
//   * GROUPED mode  - all query heads of ONE kv head x a few query tokens per
//                     workgroup (decode / jump-forward extend, GQA), with
//                     split-K over the context and a separate combine kernel.
// K/V come either from a contiguous [T, H_kv, D] tensor (cu_k offsets) or from
// the paged KV cache [n_blocks, H_kv, BLK, D] through a block table.
//
// MFMA formulation (v_mfma_f32_32x32x16_bf16, 4 waves, 32 query rows per wave):
//   S^T = K * Q^T  : A = K rows (ds_read_b128 from a padded LDS tile),
//                    B = Q^T fragment kept in VGPRs for the whole KV loop.
//                    The query lands on the MFMA lane, so the softmax row
//                    max/sum is in-register + one lane^32 exchange.
//   O^T += V^T * P^T : the S^T accumulator, exp2'ed and packed to bf16, IS the B
//                    operand (guide §3 "accumulator tile as next operand"); the
//                    V^T fragment comes from ds_read_b64_tr_b16 transposed reads
//                    of the row-major V tile (guide T10). O^T also has the
//                    query on the lane, so the online-softmax rescale is a
//                    per-lane scalar multiply.
// LDS rows are padded (K: +16 B, V: +64 B) so that both the b128 row reads and
// the tr_b16 reads are bank-conflict free (guide §2, G4).
#include "common.h"
#include <cstdlib>

#define ATT_THREADS 256
#define ATT_WAVES 4
#define KV_TILE 64

typedef short v4s __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct AttnParams {
  const bf16_t* q;
  long long q_stride;  // elements between consecutive query tokens (head stride = D)
  const bf16_t* k;
  const bf16_t* v;
  long long kv_stride;  // contiguous mode: elements between tokens
  bf16_t* o;
  long long o_stride;
  const int* cu_q;          // [B+1]
  const int* cu_k;          // [B+1] contiguous mode (or [B] starts when ctx_lens given)
  const int* ctx_lens;      // [B]   paged mode
  const int* block_tables;  // [B, max_blocks]
  int max_blocks;
  int blk;
  int Hq, Hkv;
  float scale_log2;
  int causal;
  int split_keys;  // GROUPED: keys per split (multiple of KV_TILE)
  int num_splits;
  float* part_o;   // [num_splits, Tq, Hq, D]
  float* part_ml;  // [num_splits, Tq, Hq, 2]
  int total_q;
};

template <int D>
struct AttnSmem {
  bf16_t k[KV_TILE][D + 8];
  bf16_t v[KV_TILE][D + 32];
};

__device__ __forceinline__ float16v mfma32(const bf16x8& a, const bf16x8& b, const float16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int D, bool PAGED, bool GROUPED, int QR>
__global__ __launch_bounds__(ATT_THREADS, QR == 2 ? 2 : 1) void attn_fwd_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) AttnSmem<D> sm;
  constexpr int NS = D / 16;  // k-slices of the QK^T product
  constexpr int NDT = D / 32; // 32-wide d tiles of O^T
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  // XCD-aware order (prefill / encoder grids of hundreds to thousands of
  // workgroups): the dispatcher deals consecutive ids round-robin over the 8
  // XCDs, each with its own L2. Remap so each XCD gets a CONTIGUOUS run of
  // logical (q-tile, head, sequence) ids: the q-tiles of one head, which all
  // read that head's K/V, then share one L2 instead of filling eight.
  // Bijective for any grid size (guide T1).
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (!GROUPED) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int n = gx * gy * gridDim.z;
    const int lin = bx + gx * (by + gy * bz);
    const int xcd = lin & 7, qn = n >> 3, rn = n & 7;
    const int logical = (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (lin >> 3);
    bx = logical % gx;
    by = (logical / gx) % gy;
    bz = logical / (gx * gy);
  }
  const int b = bz;
  const int q0 = p.cu_q[b];
  const int qlen = p.cu_q[b + 1] - q0;
  int k0 = 0, klen;
  if (PAGED) {
    klen = p.ctx_lens[b];
  } else {
    // contiguous K/V: start cu_k[b]; length ctx_lens[b] if given, else cu_k[b+1]-cu_k[b]
    k0 = p.cu_k[b];
    klen = p.ctx_lens ? p.ctx_lens[b] : p.cu_k[b + 1] - k0;
  }
  const int G = p.Hq / p.Hkv;

  // ---- row mapping: this lane's query rows (token index within seq, head).
  // Prefill at D = 64 gives each wave QR = 2 groups of 32 query rows: every K /
  // V fragment read from LDS then feeds two MFMAs (the D = 64 kernel is bound
  // by LDS read volume per wave, not by MFMA issue).
  constexpr int RPW = 32 * QR;                // query rows per wave
  int qi[QR], head, kvh;
  int row_lo, row_hi;  // token range covered by the workgroup (for causal bound)
  bool row_valid[QR];
  if (GROUPED) {
    const int r = wave * 32 + (lane & 31);
    kvh = by;
    qi[0] = r / G;
    head = kvh * G + (r - qi[0] * G);
    row_lo = 0;
    row_hi = min(qlen, (ATT_WAVES * 32) / G) - 1;
    row_valid[0] = qi[0] < qlen && (ATT_WAVES * 32) / G > 0 && r < (ATT_WAVES * 32 / G) * G;
  } else {
    head = by;
    kvh = head / G;
    row_lo = bx * (ATT_WAVES * RPW);
    row_hi = min(qlen - 1, row_lo + ATT_WAVES * RPW - 1);
#pragma unroll
    for (int qh = 0; qh < QR; ++qh) {
      qi[qh] = row_lo + wave * RPW + qh * 32 + (lane & 31);
      row_valid[qh] = qi[qh] < qlen;
    }
  }
  if (!GROUPED && row_lo >= qlen) return;

  // ---- key range of this workgroup
  int kbeg = 0, kend = klen;
  int split = 0;
  if (GROUPED) {
    split = bx;
    kbeg = split * p.split_keys;
    kend = min(klen, kbeg + p.split_keys);
  }
  if (p.causal) kend = min(kend, klen - qlen + row_hi + 1);

  // ---- Q^T fragments (B operand): lane (query, h) holds Q[q][16s + 8h .. +7]
  bf16x8 qf[QR][NS];
#pragma unroll
  for (int qh = 0; qh < QR; ++qh) {
    const bf16_t* qrow = p.q + (size_t)(q0 + (row_valid[qh] ? qi[qh] : 0)) * p.q_stride + (size_t)head * D;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint4 v = row_valid[qh] ? *reinterpret_cast<const uint4*>(qrow + 16 * s + 8 * h) : make_uint4(0, 0, 0, 0);
      qf[qh][s] = *reinterpret_cast<bf16x8*>(&v);
    }
  }

  float16v acc[QR][NDT];
  float m_run[QR], l_run[QR];
#pragma unroll
  for (int qh = 0; qh < QR; ++qh) {
#pragma unroll
    for (int i = 0; i < NDT; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[qh][i][j] = 0.f;
    m_run[qh] = -1e30f;
    l_run[qh] = 0.f;
  }

  const int* btab = PAGED ? p.block_tables + (size_t)b * p.max_blocks : nullptr;
  constexpr int CH = D / 8;  // 16-byte chunks per row

  for (int kt = kbeg; kt < kend; kt += KV_TILE) {
    // ---- stage K and V tile (64 keys) into LDS
    __syncthreads();
#pragma unroll
    for (int c = threadIdx.x; c < KV_TILE * CH; c += ATT_THREADS) {
      const int kr = c / CH, cc = (c - kr * CH) * 8;
      const int key = kt + kr;
      uint4 kv4 = make_uint4(0, 0, 0, 0), vv4 = make_uint4(0, 0, 0, 0);
      if (key < kend) {
        size_t off;
        if (PAGED) {
          const int bi = key / p.blk, bo = key - bi * p.blk;
          off = (((size_t)btab[bi] * p.Hkv + kvh) * p.blk + bo) * D + cc;
        } else {
          off = (size_t)(k0 + key) * p.kv_stride + (size_t)kvh * D + cc;
        }
        kv4 = *reinterpret_cast<const uint4*>(p.k + off);
        vv4 = *reinterpret_cast<const uint4*>(p.v + off);
      }
      *reinterpret_cast<uint4*>(&sm.k[kr][cc]) = kv4;
      *reinterpret_cast<uint4*>(&sm.v[kr][cc]) = vv4;
    }
    __syncthreads();

    // ---- S^T = K Q^T for the two 32-key halves (each K fragment feeds QR MFMAs)
    float16v st[QR][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int qh = 0; qh < QR; ++qh)
#pragma unroll
        for (int j = 0; j < 16; ++j) st[qh][t][j] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&sm.k[32 * t + (lane & 31)][16 * s + 8 * h]);
#pragma unroll
        for (int qh = 0; qh < QR; ++qh) st[qh][t] = mfma32(a, qf[qh][s], st[qh][t]);
      }
    }
    // ---- mask + online softmax (row = this lane's query)
    bf16x8 pf[QR][2][2];
#pragma unroll
    for (int qh = 0; qh < QR; ++qh) {
      const int qpos = klen - qlen + qi[qh];  // absolute position for causal masking
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int key = kt + 32 * t + (j & 3) + 8 * (j >> 2) + 4 * h;
          float sv = st[qh][t][j] * p.scale_log2;
          if (key >= kend || (p.causal && key > qpos)) sv = -INFINITY;
          st[qh][t][j] = sv;
          mx = fmaxf(mx, sv);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run[qh], mx);
      const float alpha = exp2f(m_run[qh] - m_new);
      float ls = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float e = exp2f(st[qh][t][8 * s2 + j] - m_new);
            ls += e;
            pf[qh][t][s2][j] = (__bf16)e;
          }
      ls += __shfl_xor(ls, 32, 64);
      l_run[qh] = l_run[qh] * alpha + ls;
      m_run[qh] = m_new;
#pragma unroll
      for (int i = 0; i < NDT; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[qh][i][j] *= alpha;
    }

    // ---- O^T += V^T P^T (each V^T fragment feeds QR MFMAs)
    const int g = lane >> 4, li = lane & 15;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int c0 = 32 * dt + 16 * (g & 1) + 4 * (li & 3);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int kb = 32 * t + 16 * s2 + 4 * h + (li >> 2);
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(&sm.v[kb][c0]));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(&sm.v[kb + 8][c0]));
          short8 a8;
          a8[0] = lo[0]; a8[1] = lo[1]; a8[2] = lo[2]; a8[3] = lo[3];
          a8[4] = hi[0]; a8[5] = hi[1]; a8[6] = hi[2]; a8[7] = hi[3];
#pragma unroll
          for (int qh = 0; qh < QR; ++qh)
            acc[qh][dt] = mfma32(*reinterpret_cast<bf16x8*>(&a8), pf[qh][t][s2], acc[qh][dt]);
        }
    }
  }

#pragma unroll
  for (int qh = 0; qh < QR; ++qh) {
    if (!row_valid[qh]) continue;
    const size_t tok = (size_t)(q0 + qi[qh]);
    if (GROUPED && p.num_splits > 1) {
      // unnormalised partial result + (m, l) for the combine kernel
      float* po = p.part_o + (((size_t)split * p.total_q + tok) * p.Hq + head) * D;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * dt + 8 * g4 + 4 * h;
          *reinterpret_cast<float4*>(po + d0) = make_float4(acc[qh][dt][4 * g4], acc[qh][dt][4 * g4 + 1],
                                                            acc[qh][dt][4 * g4 + 2], acc[qh][dt][4 * g4 + 3]);
        }
      if (h == 0) {
        float* pm = p.part_ml + (((size_t)split * p.total_q + tok) * p.Hq + head) * 2;
        pm[0] = m_run[qh];
        pm[1] = l_run[qh];
      }
      continue;
    }
    const float inv = l_run[qh] > 0.f ? 1.f / l_run[qh] : 0.f;
    bf16_t* orow = p.o + tok * p.o_stride + (size_t)head * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * h;
        uint2 w;
        w.x = pack_bf16x2(acc[qh][dt][4 * g4] * inv, acc[qh][dt][4 * g4 + 1] * inv);
        w.y = pack_bf16x2(acc[qh][dt][4 * g4 + 2] * inv, acc[qh][dt][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d0) = w;
      }
  }
}

// ---------------------------------------------------------------------------
// PREFILL / ENCODER attention, split-KV inside the workgroup.
//
// The 4-wave prefill kernel above gives one workgroup 128-256 query rows of one
// head, so a Whisper encoder pass at batch 1 (1500 frames x 20 heads) is 120
// workgroups on a 256-CU chip with ONE wave per SIMD: the softmax VALU, the
// K/V staging and the MFMAs of that wave serialize (measured 107 us per layer,
// ~110 TFLOP/s). Here a workgroup is 8 waves over 128 query rows: waves 0-3
// take the first half of the key tiles, waves 4-7 the second half (same query
// rows, same lane layout), so every CU holds two waves per SIMD whose MFMA and
// VALU phases overlap, and the grid doubles. Each half streams its K/V tiles
// through registers into its own double-buffered LDS ring (guide T14: issue the
// global loads of tile i+1 before computing tile i, write them to LDS after) -
// one barrier per tile, no drain. The halves merge their (m, l, O) through LDS
// at the end. Softmax work per score: max on raw scores, one fma + exp2 (scale
// folded), masking only on the tail / causal-diagonal tiles (wave-uniform test).
template <int D>
struct AttnSmem2 {
  bf16_t k[2][2][KV_TILE][D + 8];   // [half][stage]
  bf16_t v[2][2][KV_TILE][D + 32];
};

template <int D, bool PAGED>
__global__ __launch_bounds__(512, 1) void attn_prefill2_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) AttnSmem2<D> sm;
  constexpr int NS = D / 16, NDT = D / 32, CH = D / 8;
  constexpr int NC = KV_TILE * CH / 256;      // 16-byte chunks per thread per operand
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int half = wave >> 2, w4 = wave & 3;
  const int th = threadIdx.x & 255;
  const int h = lane >> 5;
  int bx, by, bz;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const int n = gx * gy * gridDim.z;
    const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int logical = xcd_remap(lin, n);
    bx = logical % gx;
    by = (logical / gx) % gy;
    bz = logical / (gx * gy);
  }
  const int b = bz;
  const int q0 = p.cu_q[b];
  const int qlen = p.cu_q[b + 1] - q0;
  int k0 = 0, klen;
  if (PAGED) {
    klen = p.ctx_lens[b];
  } else {
    k0 = p.cu_k[b];
    klen = p.ctx_lens ? p.ctx_lens[b] : p.cu_k[b + 1] - k0;
  }
  const int head = by, kvh = head / (p.Hq / p.Hkv);
  const int row_lo = bx * 128;
  if (row_lo >= qlen) return;                               // whole workgroup: uniform
  const int row_hi = min(qlen - 1, row_lo + 127);
  const int qi = row_lo + w4 * 32 + (lane & 31);
  const bool row_valid = qi < qlen;
  const int qpos_lo = klen - qlen + row_lo + w4 * 32;       // wave's first / last query position
  const int qpos_hi = qpos_lo + 31;
  int kend = klen;
  if (p.causal) kend = min(kend, klen - qlen + row_hi + 1);
  const int ntiles = kend > 0 ? (kend + KV_TILE - 1) / KV_TILE : 0;
  const int n0 = (ntiles + 1) >> 1;
  const int my_t0 = half ? n0 : 0;
  const int my_n = half ? ntiles - n0 : n0;

  bf16x8 qf[NS];
  {
    const bf16_t* qrow = p.q + (size_t)(q0 + (row_valid ? qi : 0)) * p.q_stride + (size_t)head * D;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint4 v = row_valid ? *reinterpret_cast<const uint4*>(qrow + 16 * s + 8 * h) : make_uint4(0, 0, 0, 0);
      qf[s] = *reinterpret_cast<bf16x8*>(&v);
    }
  }
  float16v acc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  float m_run = -1e30f, l_run = 0.f;
  const float sl2 = p.scale_log2;

  const int* btab = PAGED ? p.block_tables + (size_t)b * p.max_blocks : nullptr;
  // Loads are unconditional (rows past kend re-read the last key - finite
  // values whose scores are masked to -inf, so P = 0 exactly; a half past its
  // last tile re-reads a valid tile): a load under a branch makes hipcc fall
  // back to vmcnt(0) at the first MFMA, serialising the prefetch.
#define ATT2_ROW_OFF(KT, i, key_, cc_)                                                \
    const int c = th + (i) * 256;                                                     \
    const int kr = c / CH, cc_ = (c - kr * CH) * 8;                                   \
    const int key_ = min((KT) + kr, kend - 1);                                        \
    size_t off;                                                                       \
    if (PAGED) {                                                                      \
      const int bi = key_ / p.blk, bo = key_ - bi * p.blk;                            \
      off = (((size_t)btab[bi] * p.Hkv + kvh) * p.blk + bo) * D + cc_;                \
    } else {                                                                          \
      off = (size_t)(k0 + key_) * p.kv_stride + (size_t)kvh * D + cc_;                \
    }
#define ATT2_LOAD1(SRC, KT, R)                                                        \
  _Pragma("clang loop unroll(full)") for (int i = 0; i < NC; ++i) {                   \
    ATT2_ROW_OFF(KT, i, key, cc)                                                      \
    R[i] = *reinterpret_cast<const u32x4*>(SRC + off);                                \
  }
#define ATT2_STORE1(DST, R)                                                           \
  _Pragma("clang loop unroll(full)") for (int i = 0; i < NC; ++i) {                   \
    const int c = th + i * 256;                                                       \
    const int kr = c / CH, cc = (c - kr * CH) * 8;                                    \
    *reinterpret_cast<u32x4*>(&DST[kr][cc]) = R[i];                                   \
  }
  // S^T = K Q^T for the tile in K stage KST (two 32-key halves; the query is
  // this lane's column)
#define ATT2_QK(KST, ST)                                                              \
  {                                                                                   \
    const bf16_t(*ks_)[D + 8] = sm.k[half][KST];                                      \
    _Pragma("unroll") for (int t = 0; t < 2; ++t) {                                   \
      _Pragma("unroll") for (int j = 0; j < 16; ++j) ST[t][j] = 0.f;                  \
      _Pragma("unroll") for (int s = 0; s < NS; ++s) {                                \
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&ks_[32 * t + (lane & 31)][16 * s + 8 * h]); \
        ST[t] = mfma32(a, qf[s], ST[t]);                                              \
      }                                                                               \
    }                                                                                 \
  }

  // online softmax of the scores ST of the tile at key KT, then O^T += V^T P^T
  // with V from V stage VST
  auto softmax_pv = [&](float16v (&st)[2], int vst, int kt) __attribute__((always_inline)) {
    // masking only where a key can be invalid for this wave (wave-uniform test)
    if (kt + KV_TILE > kend || (p.causal && kt + KV_TILE - 1 > qpos_lo)) {
      const int lim = (p.causal ? min(kend, klen - qlen + qi + 1) : kend) - kt - 4 * h;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (32 * t + (j & 3) + 8 * (j >> 2) >= lim) st[t][j] = -INFINITY;
    }
    float mx = st[0][0];
#pragma unroll
    for (int j = 1; j < 16; ++j) mx = fmaxf(mx, st[0][j]);
#pragma unroll
    for (int j = 0; j < 16; ++j) mx = fmaxf(mx, st[1][j]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx * sl2);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    bf16x8 pf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          pf[t][s2][j] = (__bf16)__builtin_amdgcn_exp2f(fmaf(st[t][8 * s2 + j], sl2, -m_new));
    // row sums on the matrix core (ones . P^T: every output row is the sum
    // over the tile's 64 keys of the bf16 P that also feeds O), which has
    // slack here, instead of 32 VALU adds + a cross-lane exchange
    {
      bf16x8 ones;
#pragma unroll
      for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
      float16v ls = {};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) ls = mfma32(ones, pf[t][s2], ls);
      l_run = l_run * alpha + ls[0];
    }
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < NDT; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[i][j] *= alpha;
    const bf16_t(*vt_s)[D + 32] = sm.v[half][vst];
    const int g = lane >> 4, li = lane & 15;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int c0 = 32 * dt + 16 * (g & 1) + 4 * (li & 3);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int kb = 32 * t + 16 * s2 + 4 * h + (li >> 2);
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(&vt_s[kb][c0]));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(&vt_s[kb + 8][c0]));
          short8 a8;
          a8[0] = lo[0]; a8[1] = lo[1]; a8[2] = lo[2]; a8[3] = lo[3];
          a8[4] = hi[0]; a8[5] = hi[1]; a8[6] = hi[2]; a8[7] = hi[3];
          acc[dt] = mfma32(*reinterpret_cast<bf16x8*>(&a8), pf[t][s2], acc[dt]);
        }
    }
  };
#define ATT2_BARRIER()                                                                \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                  \
  __builtin_amdgcn_s_barrier();                                                       \
  asm volatile("" ::: "memory");

  // two K/V stages; tile i+1 is loaded to registers while tile i is computed
  if (ntiles > 0) {
    const int kt0 = min(my_t0, ntiles - 1) * KV_TILE;
    u32x4 kreg[NC], vreg[NC];   // native vectors: HIP's uint4 struct copies stay in scratch
    ATT2_LOAD1(p.k, kt0, kreg)
    ATT2_LOAD1(p.v, kt0, vreg)
    ATT2_STORE1(sm.k[half][0], kreg)
    ATT2_STORE1(sm.v[half][0], vreg)
  }
  for (int it = 0; it < n0; ++it) {
    const int stage = it & 1;
    const int kt = (my_t0 + it) * KV_TILE;
    const int ktn = min(my_t0 + it + 1, ntiles - 1) * KV_TILE;   // next tile (clamped)
    u32x4 kreg[NC], vreg[NC];
    ATT2_LOAD1(p.k, ktn, kreg)                       // lands during this tile's math
    ATT2_LOAD1(p.v, ktn, vreg)
    ATT2_BARRIER()                                   // stage `stage` written by every wave
    if (it < my_n && !(p.causal && kt > qpos_hi)) {
      float16v st[2];
      ATT2_QK(stage, st)
      softmax_pv(st, stage, kt);
    }
    // that stage was last read before this tile's barrier; past a half's last
    // tile the write is never read
    ATT2_STORE1(sm.k[half][stage ^ 1], kreg)
    ATT2_STORE1(sm.v[half][stage ^ 1], vreg)
  }
#undef ATT2_ROW_OFF
#undef ATT2_LOAD1
#undef ATT2_STORE1
#undef ATT2_QK
#undef ATT2_BARRIER

  // ---- merge the two halves: waves 4-7 hand (m, l, O) to waves 0-3 through LDS
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();                        // every wave done with the K/V rings
  asm volatile("" ::: "memory");
  float* xo = reinterpret_cast<float*>(&sm);           // [4 waves][NDT * 16][64 lanes]
  float* xml = xo + 4 * NDT * 16 * 64;                 // [4 waves][2][64 lanes]
  if (half) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int j = 0; j < 16; ++j) xo[(w4 * NDT * 16 + dt * 16 + j) * 64 + lane] = acc[dt][j];
    xml[(w4 * 2) * 64 + lane] = m_run;
    xml[(w4 * 2 + 1) * 64 + lane] = l_run;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (half || !row_valid) return;
  const float m1 = xml[(w4 * 2) * 64 + lane], l1 = xml[(w4 * 2 + 1) * 64 + lane];
  const float m = fmaxf(m_run, m1);
  const float a0 = exp2f(m_run - m), a1 = exp2f(m1 - m);
  const float l = l_run * a0 + l1 * a1;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  const float s0 = a0 * inv, s1 = a1 * inv;
  bf16_t* orow = p.o + (size_t)(q0 + qi) * p.o_stride + (size_t)head * D;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d0 = 32 * dt + 8 * g4 + 4 * h;
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        o[r] = acc[dt][4 * g4 + r] * s0 + xo[(w4 * NDT * 16 + dt * 16 + 4 * g4 + r) * 64 + lane] * s1;
      *reinterpret_cast<uint2*>(orow + d0) = make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
    }
}

// Combine split-K partials: one workgroup of D threads per (token, head).
__global__ void attn_combine_kernel(const float* __restrict__ part_o,
                                    const float* __restrict__ part_ml, bf16_t* __restrict__ o,
                                    long long o_stride, int total_q, int Hq, int D,
                                    int num_splits) {
  const int tok = blockIdx.x, head = blockIdx.y, d = threadIdx.x;
  float mstar = -1e30f;
  for (int s = 0; s < num_splits; ++s)
    mstar = fmaxf(mstar, part_ml[(((size_t)s * total_q + tok) * Hq + head) * 2]);
  float l = 0.f, acc = 0.f;
  for (int s = 0; s < num_splits; ++s) {
    const size_t idx = ((size_t)s * total_q + tok) * Hq + head;
    const float w = exp2f(part_ml[idx * 2] - mstar);
    l += w * part_ml[idx * 2 + 1];
    acc += w * part_o[idx * D + d];
  }
  o[(size_t)tok * o_stride + (size_t)head * D + d] = f2bf(l > 0.f ? acc / l : 0.f);
}

template <int D, bool PAGED, bool GROUPED>
static int launch_attn(const AttnParams& p, int B, int max_q, hipStream_t s) {
  dim3 grid;
  // QR = 2 (64 query rows per wave) where it pays: D = 64 prefill / encoder
  constexpr int QR = (!GROUPED && D == 64) ? 2 : 1;
  static const bool v1 = getenv("LOQA_ATTN_V1") != nullptr;
  if (!GROUPED && !v1) {
    grid = dim3((max_q + 127) / 128, p.Hq, B);
    hipLaunchKernelGGL((attn_prefill2_kernel<D, PAGED>), grid, dim3(512), 0, s, p);
    return (int)hipGetLastError();
  }
  if (GROUPED)
    grid = dim3(p.num_splits, p.Hkv, B);
  else
    grid = dim3((max_q + ATT_WAVES * 32 * QR - 1) / (ATT_WAVES * 32 * QR), p.Hq, B);
  hipLaunchKernelGGL((attn_fwd_kernel<D, PAGED, GROUPED, QR>), grid, dim3(ATT_THREADS), 0, s, p);
  return (int)hipGetLastError();
}

// mode: 0 = prefill (rows = q tokens of one head), 1 = grouped decode/extend.
extern "C" int loqa_attention(const void* q, long long q_stride, const void* k, const void* v,
                              long long kv_stride, void* o, long long o_stride, const int* cu_q,
                              const int* cu_k, const int* ctx_lens, const int* block_tables,
                              int max_blocks, int blk, int B, int max_q, int Hq, int Hkv, int D,
                              float scale, int causal, int mode, int split_keys, int num_splits,
                              float* part_o, float* part_ml, int total_q, hipStream_t s) {
  if (B <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv != 0 || (D != 64 && D != 128)) return (int)hipErrorInvalidValue;
  const bool paged = block_tables != nullptr;
  if (paged && (!ctx_lens || blk <= 0)) return (int)hipErrorInvalidValue;
  if (!paged && !cu_k) return (int)hipErrorInvalidValue;
  if (mode == 1) {
    if ((ATT_WAVES * 32) / (Hq / Hkv) < max_q) return (int)hipErrorInvalidValue;
    if (num_splits < 1 || split_keys % KV_TILE != 0) return (int)hipErrorInvalidValue;
    if (num_splits > 1 && (!part_o || !part_ml)) return (int)hipErrorInvalidValue;
  }
  AttnParams p;
  p.q = (const bf16_t*)q; p.q_stride = q_stride;
  p.k = (const bf16_t*)k; p.v = (const bf16_t*)v; p.kv_stride = kv_stride;
  p.o = (bf16_t*)o; p.o_stride = o_stride;
  p.cu_q = cu_q; p.cu_k = cu_k; p.ctx_lens = ctx_lens; p.block_tables = block_tables;
  p.max_blocks = max_blocks; p.blk = blk; p.Hq = Hq; p.Hkv = Hkv;
  p.scale_log2 = scale * 1.4426950408889634f; p.causal = causal;
  p.split_keys = split_keys; p.num_splits = num_splits; p.part_o = part_o; p.part_ml = part_ml;
  p.total_q = total_q;
  int rc;
#define DISPATCH(DD)                                                                    \
  if (mode == 0) rc = paged ? launch_attn<DD, true, false>(p, B, max_q, s)              \
                            : launch_attn<DD, false, false>(p, B, max_q, s);            \
  else rc = paged ? launch_attn<DD, true, true>(p, B, max_q, s)                         \
                  : launch_attn<DD, false, true>(p, B, max_q, s);
  if (D == 64) { DISPATCH(64) } else { DISPATCH(128) }
#undef DISPATCH
  if (rc != 0) return rc;
  if (mode == 1 && num_splits > 1) {
    hipLaunchKernelGGL(attn_combine_kernel, dim3(total_q, Hq), dim3(D), 0, s, part_o, part_ml,
                       (bf16_t*)o, o_stride, total_q, Hq, D, num_splits);
    rc = (int)hipGetLastError();
  }
  return rc;
}
