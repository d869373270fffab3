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

#define CAR_MAX_WORLD 8
#define CAR_BLOCKS 32
#define CAR_SPIN_LIMIT (1 << 26)

#define CAR_TWOSHOT_MIN_BYTES (512 << 10)

struct CarSignals {
  unsigned start[CAR_BLOCKS][CAR_MAX_WORLD];
  unsigned end[CAR_BLOCKS][CAR_MAX_WORLD];
  unsigned mid[CAR_BLOCKS][CAR_MAX_WORLD];     // two-shot: reduce-scatter -> all-gather
  unsigned epoch;
  unsigned done;
  unsigned error;
  unsigned pad[61];
};

struct CarPeers {
  char* base[CAR_MAX_WORLD];  // every rank's region (own rank included)
};

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ bool car_barrier(CarPeers peers, int rank, int world, int which, int blk, unsigned e) {
  // every thread 0 of a block publishes; the block waits as a whole
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope release
    for (int q = 0; q < world; ++q) {
      CarSignals* s = reinterpret_cast<CarSignals*>(peers.base[q]);
      st_sys(which == 0 ? &s->start[blk][rank] : which == 1 ? &s->end[blk][rank] : &s->mid[blk][rank], e);
    }
  }
  bool ok = true;
  if (threadIdx.x < world) {
    CarSignals* me = reinterpret_cast<CarSignals*>(peers.base[rank]);
    const unsigned* f = which == 0 ? &me->start[blk][threadIdx.x]
                        : which == 1 ? &me->end[blk][threadIdx.x] : &me->mid[blk][threadIdx.x];
    unsigned spins = 0;
    while (ld_sys(f) != e) {
      if (++spins > CAR_SPIN_LIMIT) {
        st_sys(&me->error, 1u);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  return __syncthreads_and(ok);
}

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

struct CarHandle {
  int rank, world;
  size_t bytes, slot_bytes;
  char* local;
  CarPeers peers;
  bool opened[CAR_MAX_WORLD];
};

extern "C" void* loqa_car_create(int rank, int world, long long slot_bytes) {
  if (world < 1 || world > CAR_MAX_WORLD || rank < 0 || rank >= world || slot_bytes % 16)
    return nullptr;
  CarHandle* h = new CarHandle();
  h->rank = rank;
  h->world = world;
  h->slot_bytes = (size_t)slot_bytes;
  h->bytes = sizeof(CarSignals) + 2 * (size_t)slot_bytes;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&h->local), h->bytes, hipDeviceMallocUncached) !=
      hipSuccess) {
    delete h;
    return nullptr;
  }
  hipMemset(h->local, 0, sizeof(CarSignals));
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

// nonzero when a barrier timed out (a peer never arrived)
extern "C" int loqa_car_error(void* hp) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  unsigned v = 0;
  hipMemcpy(&v, &reinterpret_cast<CarSignals*>(h->local)->error, sizeof(unsigned),
            hipMemcpyDeviceToHost);
  return (int)v;
}

extern "C" void loqa_car_destroy(void* hp) {
  CarHandle* h = static_cast<CarHandle*>(hp);
  if (!h) return;
  for (int q = 0; q < h->world; ++q)
    if (h->opened[q]) hipIpcCloseMemHandle(h->peers.base[q]);
  hipFree(h->local);
  delete h;
}
