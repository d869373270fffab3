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
#include "attn_decode.h"

thread_local int g_loqa_launch_prio = 0;

extern "C" void loqa_set_launch_prio(int prio) { g_loqa_launch_prio = prio; }

template <int D, int PF, int NW = DEC_WAVES, int OCC = 2>
__global__ __launch_bounds__(NW * 64, OCC) void attn_decode_kernel(AttnDecArgs a) {
  if (a.prio) __builtin_amdgcn_s_setprio(3);     // kernel argument: wave-uniform
  __shared__ __attribute__((aligned(16))) DecSmem<D, NW> sm;
  attn_decode_body<D, PF, 0, 0, NW>(a, blockIdx.x, blockIdx.y, blockIdx.z, sm);
}

// Single-pass form (waves = 8): a workgroup of 8 waves covers 256 keys per
// pass and, for the short contexts of an intent parse (<= 512 keys), the
// whole context in ONE split - no partial publish, ticket or last-arriver
// merge (the split combine's three dependent memory round trips), the 8
// waves' states merged through LDS only. With PF the second tile of a wave
// is requested before the first is consumed. For a tensor-parallel rank
// (one kv head per rank: 8 sequences -> 8 workgroups) the combine was the
// larger part of the kernel.

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
                                int* counters, int waves, int pf, hipStream_t s) {
  if (B <= 0 || total_q <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv || (Hq / Hkv) * max_q > 32 || split_keys % DEC_TILE || num_splits < 1 ||
      (D != 64 && D != 128) || !part_o || !part_ml || !counters)
    return (int)hipErrorInvalidValue;
  if (block_tables && (blk < 16 || (blk & (blk - 1)))) return (int)hipErrorInvalidValue;
  if (!block_tables && (!kv_start || kv_stride % 8)) return (int)hipErrorInvalidValue;
  dim3 grid(num_splits, Hkv, B);
  const float sl2 = scale * 1.4426950408889634f;
  const AttnDecArgs a{(const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, kv_stride,
                      kv_start, cu_q, ctx_lens, block_tables, max_blocks, blk, Hq, Hkv, sl2, causal,
                      split_keys, num_splits, part_o, part_ml, total_q, counters, (bf16_t*)o,
                      o_stride, 0, 0, g_loqa_launch_prio, 0};
  if (waves != 4 && waves != 8) return (int)hipErrorInvalidValue;
  if (waves == 8) {   // 512 threads: 2 waves per SIMD, 256 registers each (no PF at D = 128)
    if (D == 128)
      hipLaunchKernelGGL((attn_decode_kernel<128, 0, 8, 1>), grid, dim3(512), 0, s, a);
    else if (pf)
      hipLaunchKernelGGL((attn_decode_kernel<64, 1, 8, 1>), grid, dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((attn_decode_kernel<64, 0, 8, 1>), grid, dim3(512), 0, s, a);
    return (int)hipGetLastError();
  }
  if (pf) {           // 4 waves, one per SIMD: the whole register file for the prefetch
    if (D == 128)
      hipLaunchKernelGGL((attn_decode_kernel<128, 1, 4, 1>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((attn_decode_kernel<64, 1, 4, 1>), grid, dim3(256), 0, s, a);
    return (int)hipGetLastError();
  }
  if (D == 128)
    hipLaunchKernelGGL((attn_decode_kernel<128, 0>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((attn_decode_kernel<64, 0>), grid, dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
