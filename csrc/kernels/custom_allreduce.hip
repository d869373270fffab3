// One-shot all-reduce over IPC-mapped peer buffers.
//
// Tensor-parallel decode all-reduces are latency-bound (B x 8192 bf16 = 16-256 KB
// per call, 2 per layer): a ring pays 2(world-1) link hops and drives 1-2 of
// the 7 xGMI links. Here every rank stages its tensor in its own IPC-exported
// buffer, signals the peers, and every rank then reads all world slices
// directly over the point-to-point links in parallel and sums them in f32 -
// one hop, all links busy.
//
// Memory: one hipDeviceMallocUncached region per rank (signals + 2 data
// slots), exported with hipIpcGetMemHandle and opened by every peer; uncached
// so neither L2 holds a stale copy of a peer's flag or slot.
// Protocol per call (epoch e = per-rank device counter, bumped by the last
// block of the call, so graph replays stay consistent):
//   block b copies slice b of the input into slot e%2 of its own region ->
//   system release -> writes start[b][rank] = e in every peer's region ->
//   waits for start[b][q] == e from all q (bounded spin, error flag on
//   timeout) -> sums slice b over all peers' slots -> writes the output ->
//   end barrier (same flags, second set) so no peer overwrites a slot that is
//   still being read.
#include "common.h"
#include <stdlib.h>

#include "car_common.h"
// 16-byte vector sum over the peers' slots at vector index v (fixed peer order)
template <bool F32>
__device__ __forceinline__ uint4 car_sum16(const CarPeers& peers, size_t slot_off, int world,
                                           long long v) {
  if constexpr (F32) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < world; ++q) {
      const float4 x = reinterpret_cast<const float4*>(peers.base[q] + slot_off)[v];
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    }
    return *reinterpret_cast<uint4*>(&acc);
  } else {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < world; ++q) {
      float f[8];
      unpack8(reinterpret_cast<const uint4*>(peers.base[q] + slot_off)[v], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    return pack8(acc);
  }
}

// element type: bf16 (8 per 16-byte vector) or f32 (4 per vector, the decode
// GEMM's split-K slab is all-reduced before its consumer reduces it)
template <bool F32>
__global__ __launch_bounds__(256) void car_oneshot_kernel(CarPeers peers, const void* __restrict__ in,
                                                          void* __restrict__ out, long long nbytes,
                                                          int rank, int world, long long slot_bytes) {
  CarSignals* me = reinterpret_cast<CarSignals*>(peers.base[rank]);
  const unsigned e = ld_sys(&me->epoch) + 1;  // every block reads it before anyone bumps it
  const int blk = blockIdx.x;
  const long long nv = nbytes >> 4;             // 16-byte vectors
  const long long per = (nv + CAR_BLOCKS - 1) / CAR_BLOCKS;
  const long long v0 = blk * per, v1 = v0 + per < nv ? v0 + per : nv;
  const size_t slot_off = sizeof(CarSignals) + (size_t)(e & 1) * slot_bytes;
  uint4* mine = reinterpret_cast<uint4*>(peers.base[rank] + slot_off);
  const uint4* src = reinterpret_cast<const uint4*>(in);
  for (long long v = v0 + threadIdx.x; v < v1; v += blockDim.x) mine[v] = src[v];
  if (car_barrier(peers, rank, world, 0, blk, e)) {
    uint4* dst = reinterpret_cast<uint4*>(out);
    // fixed peer order: bitwise identical on every rank
    for (long long v = v0 + threadIdx.x; v < v1; v += blockDim.x)
      dst[v] = car_sum16<F32>(peers, slot_off, world, v);
    car_barrier(peers, rank, world, 1, blk, e);
  }
  // the last block to finish publishes the epoch for the next call
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned d = __hip_atomic_fetch_add(&me->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == CAR_BLOCKS - 1) {
      st_sys(&me->done, 0u);
      st_sys(&me->epoch, e);
    }
  }
}

// Two-shot (bandwidth-bound sizes, e.g. prefill activations): rank r owns
// slice r of the tensor. Block b (of every rank) stages chunk b of every slice
// -> start barrier -> sums chunk b of ITS slice over all peers (each link
// carries 1/world of the tensor) and writes it back into its own slot and the
// output -> mid barrier -> gathers chunk b of every other slice from its owner
// -> end barrier. Per rank ~2N bytes cross the links instead of world * N.
template <bool F32>
__global__ __launch_bounds__(256) void car_twoshot_kernel(CarPeers peers, const void* __restrict__ in,
                                                          void* __restrict__ out, long long nbytes,
                                                          int rank, int world, long long slot_bytes) {
  CarSignals* me = reinterpret_cast<CarSignals*>(peers.base[rank]);
  const unsigned e = ld_sys(&me->epoch) + 1;
  const int blk = blockIdx.x;
  const long long sv = (nbytes >> 4) / world;                 // vectors per slice
  const long long per = (sv + CAR_BLOCKS - 1) / CAR_BLOCKS;
  const long long c0 = blk * per, c1 = c0 + per < sv ? c0 + per : sv;
  const size_t slot_off = sizeof(CarSignals) + (size_t)(e & 1) * slot_bytes;
  uint4* mine = reinterpret_cast<uint4*>(peers.base[rank] + slot_off);
  const uint4* src = reinterpret_cast<const uint4*>(in);
  uint4* dst = reinterpret_cast<uint4*>(out);
  for (int q = 0; q < world; ++q)
    for (long long v = c0 + threadIdx.x; v < c1; v += blockDim.x) mine[q * sv + v] = src[q * sv + v];
  if (car_barrier(peers, rank, world, 0, blk, e)) {
    for (long long v = c0 + threadIdx.x; v < c1; v += blockDim.x) {
      const long long i = rank * sv + v;
      const uint4 r = car_sum16<F32>(peers, slot_off, world, i);
      mine[i] = r;
      dst[i] = r;
    }
    if (car_barrier(peers, rank, world, 2, blk, e)) {
      for (int q = 0; q < world; ++q) {
        if (q == rank) continue;
        const uint4* theirs = reinterpret_cast<const uint4*>(peers.base[q] + slot_off);
        for (long long v = c0 + threadIdx.x; v < c1; v += blockDim.x) dst[q * sv + v] = theirs[q * sv + v];
      }
      car_barrier(peers, rank, world, 1, blk, e);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned d = __hip_atomic_fetch_add(&me->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == CAR_BLOCKS - 1) {
      st_sys(&me->done, 0u);
      st_sys(&me->epoch, e);
    }
  }
}

// ---------------------------------------------------------------------------
// Tensor-parallel decode step collectives (models/llama.py forward_decode_fused
// at tp > 1). The row-parallel o / down GEMMs write their f32 partial sums
// straight into this rank's IPC input buffer (ops.skinny_fused "act" epilogue
// with f32 output, out = CustomAllReduce.inbuf); one kernel then sums every
// rank's partial into the replicated residual and emits the row statistics
// the next fused GEMM's norm prologue reads - the all-reduce IS the residual
// epilogue.
//
// No end barrier: the o and down projections alternate between two sets of
// input / result / statistics buffers (and the argmax exchange has its own),
// so a buffer is rewritten only after some LATER call's start barrier, which
// no peer passes before it finished reading the earlier contents (every call
// is a kernel boundary on each rank's stream).
//
// Peer data is read with system-coherent buffer loads (sc0 | sc1: straight
// from the owner's memory, never a stale L2 line); the buffers live in the
// uncached region, so the GEMM's stores are in memory when its kernel ends.
template <int LEAN>
__global__ __launch_bounds__(256) void car_resid_kernel(CarPeers peers, long long in_off, long long res_off,
                                                        long long st_off, bf16_t* __restrict__ residual,
                                                        float* __restrict__ rowsq_out, int Mpad, int d,
                                                        int rank, int world) {
  car_resid_block<LEAN, 0>(peers, in_off, res_off, st_off, residual, rowsq_out, Mpad, d, rank, world,
                           blockIdx.x, gridDim.x);
}

// Vocab-parallel masked argmax combine: every rank publishes one
// 64-bit record per row - [63:49] epoch, [48:17] order-preserving bits of the
// row's best local logit, [16:0] 2^17-1 - global token id (larger = smaller id,
// so ties go to the lowest id) - and every rank takes the max over ranks. The
// record carries its own epoch, so no separate flag or fence is needed.
__device__ __forceinline__ unsigned long long car_ld64_sys(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void car_argmax_kernel(CarPeers peers, long long key_off,
                                                         const float* __restrict__ logits, long long ld,
                                                         const int* __restrict__ idx, int B, int lo,
                                                         int* __restrict__ out, int rank, int world) {
  CarSignals* me = reinterpret_cast<CarSignals*>(peers.base[rank]);
  const unsigned e = ld_sys(&me->epoch) + 1;
  const unsigned long long tag = (unsigned long long)(e & 0x7fffu) << 49;
  // every row is rewritten each call (rows >= B as "nothing"), so a stale
  // record is always from an earlier call with a different 15-bit epoch
  for (int b = threadIdx.x; b < CAR_KEY_ROWS; b += blockDim.x) {
    const int i = b < B ? idx[b] : -1;
    unsigned long long key = 0;   // nothing allowed on this shard
    if (i >= 0) {
      const unsigned u = __float_as_uint(logits[(size_t)b * ld + i]);
      const unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
      key = ((unsigned long long)ord << 17) | (unsigned long long)(0x1ffffu - (unsigned)(i + lo));
    }
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(peers.base[rank] + key_off) + b;
    __hip_atomic_store(dst, tag | key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  bool ok = true;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    unsigned long long best = 0;
    for (int q = 0; q < world; ++q) {
      const unsigned long long* src =
          reinterpret_cast<const unsigned long long*>(peers.base[q] + key_off) + b;
      unsigned long long v;
      unsigned spins = ld_sys(&me->error) ? CAR_SPIN_LIMIT : 0u;
      while (((v = car_ld64_sys(src)) >> 49) != (e & 0x7fffu)) {
        if (++spins > CAR_SPIN_LIMIT) {
          st_sys(&me->error, 1u);
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!ok) break;
      const unsigned long long k = v & ((1ull << 49) - 1);
      best = k > best ? k : best;
    }
    out[b] = !ok ? CAR_ERR_TOKEN : best == 0 ? -1 : (int)(0x1ffffu - (unsigned)(best & 0x1ffffu));
  }
  // the sticky error word rides on every step's sampled tokens: any collective
  // of this step (or an earlier one) that timed out turns every row into
  // CAR_ERR_TOKEN, so the host sees it in the result it reads anyway - no
  // separate read of the word per step
  __syncthreads();
  if (ld_sys(&me->error))
    for (int b = threadIdx.x; b < B; b += blockDim.x) out[b] = CAR_ERR_TOKEN;
  car_epoch_done(me, e, 1);
}

// Single-process emulation of a TP=world residual all-reduce (TP=1 runs the
// W shard partials itself): block (q, b) does exactly what block b of rank q
// does in phase 1 of car_resid_kernel, over plain loads of the W partials
// [world][Mpad][d] f32, and writes the combined residual slice and the
// statistics tile q * nblk + b. Phase 2 (the all-gather) has nothing to do in
// one process.
__global__ __launch_bounds__(256) void tp_emul_resid_kernel(const float* __restrict__ partials,
                                                            bf16_t* __restrict__ residual,
                                                            float* __restrict__ rowsq_out, int Mpad, int d,
                                                            int world, int nblk) {
  const int q = blockIdx.x / nblk, blk = blockIdx.x % nblk;
  const int owned = d / world, cw = owned / nblk;
  const int c0 = q * owned + blk * cw;
  const int vpr = cw >> 2;
  const int rpp = 256 / vpr, r0 = threadIdx.x / vpr, cv = threadIdx.x % vpr;
  const size_t plane = (size_t)Mpad * d;
  for (int m0 = 0; m0 < Mpad; m0 += rpp) {
    const int m = m0 + r0;
    const bool act = r0 < rpp && m < Mpad;
    float sq = 0.f;
    if (act) {
      const size_t el = (size_t)m * d + c0 + cv * 4;
      const uint2 rv = *reinterpret_cast<const uint2*>(residual + el);
      car_u32x4 v[CAR_MAX_WORLD];
#pragma unroll
      for (int r = 0; r < CAR_MAX_WORLD; ++r)
        if (r < world) v[r] = *reinterpret_cast<const car_u32x4*>(partials + r * plane + el);
      uint2 o;
      sq = car_resid_math(rv, v, world, o);
      *reinterpret_cast<uint2*>(residual + el) = o;
    }
    sq = car_row_butterfly(sq, vpr);
    if (cv == 0 && act) rowsq_out[((size_t)q * nblk + blk) * Mpad + m] = sq;
  }
}

extern "C" int loqa_tp_emul_resid(const float* partials, void* residual, float* rowsq_out, int Mpad, int d,
                                  int world, int nblk, hipStream_t s) {
  if (world < 1 || world > CAR_MAX_WORLD || nblk < 1 || nblk > CAR_MAX_BLOCKS || d % (world * nblk) ||
      Mpad < 1)
    return (int)hipErrorInvalidValue;
  const int cw = d / world / nblk, vpr = cw / 4;
  if (cw % 8 || vpr > 64 || (vpr & (vpr - 1))) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(tp_emul_resid_kernel, dim3(world * nblk), dim3(256), 0, s, partials, (bf16_t*)residual,
                     rowsq_out, Mpad, d, world, nblk);
  return (int)hipGetLastError();
}

struct CarHandle {
  int rank, world;
  size_t bytes, slot_bytes, in_bytes;
  char* local;
  CarPeers peers;
  bool opened[CAR_MAX_WORLD];
};

// region: [signals][slot 0][slot 1][f32 input 0][f32 input 1][bf16 result 0]
// [bf16 result 1][stats 0][stats 1][argmax keys]; in_bytes = one f32 input
#define CAR_ST_BYTES (CAR_MAX_BLOCKS * 128 * 4)
static size_t car_in_off(const CarHandle* h, int which) {
  return sizeof(CarSignals) + 2 * h->slot_bytes + (size_t)which * h->in_bytes;
}
static size_t car_res_off(const CarHandle* h, int which) {
  return car_in_off(h, 2) + (size_t)which * (h->in_bytes / 2);
}
static size_t car_st_off(const CarHandle* h, int which) {
  return car_res_off(h, 2) + (size_t)which * CAR_ST_BYTES;
}
static size_t car_key_off(const CarHandle* h) { return car_st_off(h, 2); }

extern "C" void* loqa_car_create(int rank, int world, long long slot_bytes, long long in_bytes) {
  if (world < 1 || world > CAR_MAX_WORLD || rank < 0 || rank >= world || slot_bytes % 16 ||
      in_bytes % 512 || in_bytes < 0)
    return nullptr;
  CarHandle* h = new CarHandle();
  h->rank = rank;
  h->world = world;
  h->slot_bytes = (size_t)slot_bytes;
  h->in_bytes = (size_t)in_bytes;
  h->bytes = car_key_off(h) + CAR_KEY_ROWS * 8;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&h->local), h->bytes, hipDeviceMallocUncached) !=
      hipSuccess) {
    delete h;
    return nullptr;
  }
  hipMemset(h->local, 0, sizeof(CarSignals));
  hipMemset(h->local + car_key_off(h), 0, CAR_KEY_ROWS * 8);
  hipDeviceSynchronize();
  for (int q = 0; q < CAR_MAX_WORLD; ++q) {
    h->peers.base[q] = nullptr;
    h->opened[q] = false;
  }
  h->peers.base[rank] = h->local;
  return h;
}

extern "C" int loqa_car_handle(void* hp, void* out /* sizeof(hipIpcMemHandle_t) bytes */) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  return (int)hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(out), h->local);
}

extern "C" int loqa_car_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// handles: world consecutive hipIpcMemHandle_t (own slot ignored)
extern "C" int loqa_car_open(void* hp, const void* handles) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  const hipIpcMemHandle_t* hs = static_cast<const hipIpcMemHandle_t*>(handles);
  for (int q = 0; q < h->world; ++q) {
    if (q == h->rank) continue;
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, hs[q], hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    h->peers.base[q] = static_cast<char*>(p);
    h->opened[q] = true;
  }
  return 0;
}

// n elements of bf16 (is_f32 = 0) or f32 (is_f32 = 1); n * size % 16 == 0.
// One-shot below CAR_TWOSHOT_MIN_BYTES (latency-bound decode), two-shot above.
extern "C" int loqa_car_allreduce(void* hp, const void* in, void* out, long long n, int is_f32,
                                  hipStream_t s) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  if (n <= 0) return 0;
  const long long nbytes = n * (is_f32 ? 4 : 2);
  if (nbytes % 16 || (size_t)nbytes > h->slot_bytes) return (int)hipErrorInvalidValue;
  for (int q = 0; q < h->world; ++q)
    if (!h->peers.base[q]) return (int)hipErrorInvalidValue;
  const bool two = h->world > 1 && nbytes >= CAR_TWOSHOT_MIN_BYTES && nbytes % (16LL * h->world) == 0;
  auto k = two ? (is_f32 ? car_twoshot_kernel<true> : car_twoshot_kernel<false>)
               : (is_f32 ? car_oneshot_kernel<true> : car_oneshot_kernel<false>);
  hipLaunchKernelGGL(k, dim3(CAR_BLOCKS), dim3(256), 0, s, h->peers, in, out, nbytes, h->rank,
                     h->world, (long long)h->slot_bytes);
  return (int)hipGetLastError();
}

// this rank's TP f32 input buffer `which` (0 / 1): the row-parallel GEMM's output
extern "C" void* loqa_car_inbuf(void* hp, int which) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  if (which < 0 || which > 1 || h->in_bytes == 0) return nullptr;
  return h->local + car_in_off(h, which);
}

// residual [Mpad, d] += sum over ranks of f32 input buffer `which` ([Mpad, d]);
// row sums of squares -> rowsq_out [world * nblk, Mpad]. d / world / nblk
// columns per block: a multiple of 8, at most 256 (<= 64 f32x4 lanes per row).
extern "C" int loqa_car_resid(void* hp, int which, void* residual, float* rowsq_out, int Mpad, int d,
                              int nblk, hipStream_t s) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  if (which < 0 || which > 1 || nblk < 1 || nblk > CAR_MAX_BLOCKS || d % (h->world * nblk) ||
      Mpad < 1 || Mpad > 128)
    return (int)hipErrorInvalidValue;
  const int cw = d / h->world / nblk, vpr = cw / 4;
  if (cw % 8 || vpr > 64 || (vpr & (vpr - 1)) || (size_t)Mpad * d * 4 > h->in_bytes)
    return (int)hipErrorInvalidValue;
  for (int q = 0; q < h->world; ++q)
    if (!h->peers.base[q]) return (int)hipErrorInvalidValue;
  static int lean = -1;
  if (lean < 0) {
    // default on: 7.46 -> 6.69 ms per config-5 rank step, multi-process TP
    // tests bitwise (profiles/r5_config5_lean_allreduce.txt)
    const char* ev = getenv("LOQA_CAR_LEAN");
    lean = ev ? atoi(ev) : 1;
  }
  hipLaunchKernelGGL(lean ? car_resid_kernel<1> : car_resid_kernel<0>, dim3(nblk), dim3(256), 0, s, h->peers,
                     (long long)car_in_off(h, which), (long long)car_res_off(h, which),
                     (long long)car_st_off(h, which), (bf16_t*)residual, rowsq_out, Mpad, d, h->rank,
                     h->world);
  return (int)hipGetLastError();
}

int car_prologue_args(void* hp, int which, CarPeers* peers, long long* in_off, long long* res_off,
                      long long* st_off, int* rank, int* world, size_t* in_bytes) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  if (!h || which < 0 || which > 1 || h->in_bytes == 0) return (int)hipErrorInvalidValue;
  for (int q = 0; q < h->world; ++q)
    if (!h->peers.base[q]) return (int)hipErrorInvalidValue;
  *peers = h->peers;
  *in_off = (long long)car_in_off(h, which);
  *res_off = (long long)car_res_off(h, which);
  *st_off = (long long)car_st_off(h, which);
  *rank = h->rank;
  *world = h->world;
  *in_bytes = h->in_bytes;
  return 0;
}

// out[b] = global argmax over ranks of (logits[b, idx[b]], idx[b] + lo); -1 if
// no rank allowed any token, CAR_ERR_TOKEN if a collective timed out.
// idx: this rank's masked argmax (-1 = none).
// shard: this rank's vocab width; every global id (lo .. lo + shard - 1) must
// fit the record's 17-bit id field.
extern "C" int loqa_car_argmax(void* hp, const float* logits, long long ld, const int* idx, int B,
                               int lo, int shard, int* out, hipStream_t s) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  if (B < 1 || B > CAR_KEY_ROWS || lo < 0 || lo + shard - 1 > CAR_MAX_TOKEN_ID || shard < 1)
    return (int)hipErrorInvalidValue;
  for (int q = 0; q < h->world; ++q)
    if (!h->peers.base[q]) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(car_argmax_kernel, dim3(1), dim3(256), 0, s, h->peers, (long long)car_key_off(h),
                     logits, ld, idx, B, lo, out, h->rank, h->world);
  return (int)hipGetLastError();
}

// 1 when a barrier timed out (a peer never arrived), 0 if not, a negative
// hipError_t when the word cannot be read (the device is in a failed state)
extern "C" int loqa_car_error(void* hp) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  unsigned v = 0;
  const hipError_t e = hipMemcpy(&v, &reinterpret_cast<CarSignals*>(h->local)->error,
                                 sizeof(unsigned), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return -(int)e;
  return v ? 1 : 0;
}

// copy `bytes` of device memory into input buffer `which` (start-up self-test)
extern "C" int loqa_car_fill_inbuf(void* hp, int which, const void* src, long long bytes,
                                   hipStream_t s) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  if (which < 0 || which > 1 || bytes < 0 || (size_t)bytes > h->in_bytes) return (int)hipErrorInvalidValue;
  return (int)hipMemcpyAsync(h->local + car_in_off(h, which), src, (size_t)bytes,
                             hipMemcpyDeviceToDevice, s);
}

// clear this rank's sticky error word (start-up self-test only)
extern "C" int loqa_car_clear_error(void* hp) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  return (int)hipMemset(&reinterpret_cast<CarSignals*>(h->local)->error, 0, sizeof(unsigned));
}

extern "C" void loqa_car_destroy(void* hp) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  if (!h) return;
  for (int q = 0; q < h->world; ++q)
    if (h->opened[q]) hipIpcCloseMemHandle(h->peers.base[q]);
  hipFree(h->local);
  delete h;
}
