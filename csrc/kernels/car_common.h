// Device side of the tensor-parallel residual all-reduce (custom_allreduce.hip):
// the IPC region layout, flag helpers and the per-block body, shared with the
// fused decode GEMM whose prologue runs the all-reduce (gemm_skinny.hip).
#pragma once
#include "common.h"

#define CAR_MAX_WORLD 8
#define CAR_BLOCKS 32          // blocks of the one-/two-shot kernels
#define CAR_MAX_BLOCKS 64      // flag rows (the residual kernel may use up to 64 blocks)
// bounded waits (~several seconds); once any wait of this rank timed out the
// sticky error word makes every later wait give up at once, so a diverged TP
// group fails fast instead of spinning out every remaining collective
#define CAR_SPIN_LIMIT (1 << 22)

#define CAR_TWOSHOT_MIN_BYTES (512 << 10)

struct CarSignals {
  unsigned start[CAR_MAX_BLOCKS][CAR_MAX_WORLD];
  unsigned end[CAR_MAX_BLOCKS][CAR_MAX_WORLD];
  unsigned mid[CAR_MAX_BLOCKS][CAR_MAX_WORLD];     // two-shot: reduce-scatter -> all-gather
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


__device__ __forceinline__ bool car_barrier(CarPeers peers, int rank, int world, int which, int blk, unsigned e) {
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
    unsigned spins = ld_sys(&me->error) ? CAR_SPIN_LIMIT : 0u;
    // epochs only grow, and a peer is at most one call ahead (it cannot pass
    // the next barrier before this rank arrives there): wait for >= e
    while ((int)(ld_sys(f) - e) < 0) {
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

#define CAR_KEY_ROWS 256      // rows of the argmax exchange
#define CAR_ERR_TOKEN (-2)    // argmax output of a step whose collectives failed
#define CAR_MAX_TOKEN_ID 0x1ffff  // 17-bit token ids in the argmax records
#define CAR_SYS 17            // buffer-op cache policy: sc0 | sc1 (system coherent)

typedef unsigned car_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_car __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t car_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// start barrier of block `blk` only (the data was written by earlier kernels)
__device__ __forceinline__ bool car_arrive_wait(const CarPeers& peers, int rank, int world, int blk,
                                                unsigned e) {
  if (threadIdx.x == 0) {
    for (int q = 0; q < world; ++q)
      st_sys(&reinterpret_cast<CarSignals*>(peers.base[q])->start[blk][rank], e);
  }
  bool ok = true;
  if (threadIdx.x < world) {
    CarSignals* me = reinterpret_cast<CarSignals*>(peers.base[rank]);
    const unsigned* f = &me->start[blk][threadIdx.x];
    unsigned spins = ld_sys(&me->error) ? CAR_SPIN_LIMIT : 0u;
    while ((int)(ld_sys(f) - e) < 0) {
      if (++spins > CAR_SPIN_LIMIT) {
        st_sys(&me->error, 1u);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return __syncthreads_and(ok);
}

__device__ __forceinline__ void car_epoch_done(CarSignals* me, unsigned e, int nblk) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned d = __hip_atomic_fetch_add(&me->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned)nblk - 1) {
      st_sys(&me->done, 0u);
      st_sys(&me->epoch, e);
    }
  }
}

// Residual all-reduce of the TP decode step, reduce-scatter + all-gather:
//   phase 1: rank r owns the column slice [r * d/W, (r+1) * d/W). Its block b
//            sums, for sub-slice b of that, residual + every rank's f32 partial
//            (system-coherent loads, fixed rank order), rounds to bf16 ONCE,
//            writes the result into its local residual and its IPC result
//            buffer, and the sub-slice's row sums of squares into its IPC stats;
//   phase 2: after a second barrier, it copies sub-slice b of every other
//            rank's owned slice (bf16 results) and stats tiles.
// Bytes read per rank: Mpad * d * 4 (f32 slices) + (W-1)/W * Mpad * d * 2,
// vs W * Mpad * d * 2 for a one-shot bf16 sum - and f32 partials keep the
// numerics of the single-GPU residual epilogue (one rounding).
// rowsq_out gets W * nblk tiles: tile q * nblk + b = rank q's sub-slice b.
// One row chunk of a residual all-reduce block: residual slice + the world
// f32 partials in rank order (one bf16 rounding) and the sub-slice's row sum of
// squares (fixed fma order, then a butterfly over the row's lanes). Shared by
// the IPC kernel and its single-process emulation (tp_emul_resid_kernel), so
// the emulation is bitwise the same arithmetic.
__device__ __forceinline__ float car_resid_math(uint2 rv, const car_u32x4* v, int world, uint2& o) {
  float acc[4] = {bf2f(rv.x & 0xffff), bf2f(rv.x >> 16), bf2f(rv.y & 0xffff), bf2f(rv.y >> 16)};
#pragma unroll
  for (int q = 0; q < CAR_MAX_WORLD; ++q) {
    if (q >= world) break;
    acc[0] += __uint_as_float(v[q].x); acc[1] += __uint_as_float(v[q].y);
    acc[2] += __uint_as_float(v[q].z); acc[3] += __uint_as_float(v[q].w);
  }
  o.x = pack_bf16x2(acc[0], acc[1]);
  o.y = pack_bf16x2(acc[2], acc[3]);
  const float h0 = bf2f(o.x & 0xffff), h1 = bf2f(o.x >> 16), h2 = bf2f(o.y & 0xffff), h3 = bf2f(o.y >> 16);
  return __builtin_fmaf(h3, h3, __builtin_fmaf(h2, h2, __builtin_fmaf(h1, h1, h0 * h0)));
}

__device__ __forceinline__ float car_row_butterfly(float sq, int vpr) {
  for (int o = 1; o < vpr; o <<= 1) sq += __shfl_xor(sq, o, 64);
  return sq;
}

// LEAN: the phase-2 publish without the system-scope release fences (an L2
// write-back each): everything a peer reads here lives in the uncached IPC
// region and is stored with system-coherent (sc0 | sc1) buffer stores, so
// draining this rank's stores (vmcnt(0)) before the flag store already orders
// data before flag; peers read with sc0 | sc1 loads, so no acquire is needed.
template <int LEAN>
__device__ __forceinline__ bool car_publish_wait(const CarPeers& peers, int rank, int world, int blk,
                                                 unsigned e) {
  if constexpr (!LEAN) {
    return car_barrier(peers, rank, world, 2, blk, e);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int q = 0; q < world; ++q)
        st_sys(&reinterpret_cast<CarSignals*>(peers.base[q])->mid[blk][rank], e);
    }
    bool ok = true;
    if (threadIdx.x < world) {
      CarSignals* me = reinterpret_cast<CarSignals*>(peers.base[rank]);
      const unsigned* f = &me->mid[blk][threadIdx.x];
      unsigned spins = ld_sys(&me->error) ? CAR_SPIN_LIMIT : 0u;
      while ((int)(ld_sys(f) - e) < 0) {
        if (++spins > CAR_SPIN_LIMIT) {
          st_sys(&me->error, 1u);
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    return __syncthreads_and(ok);
  }
}

// local result stores of car_resid_block: plain, or write-through (sc1)
template <int SC1>
__device__ __forceinline__ void car_st_b64(bf16_t* base, unsigned bytes, size_t off, uint2 v) {
  if constexpr (SC1)
    __builtin_amdgcn_raw_buffer_store_b64(u32x2_car{v.x, v.y}, car_rsrc(base, bytes), (unsigned)off, 0, 16);
  else
    *reinterpret_cast<uint2*>(reinterpret_cast<char*>(base) + off) = v;
}
template <int SC1>
__device__ __forceinline__ void car_st_b128(bf16_t* base, unsigned bytes, size_t off, car_u32x4 v) {
  if constexpr (SC1)
    __builtin_amdgcn_raw_buffer_store_b128(v, car_rsrc(base, bytes), (unsigned)off, 0, 16);
  else
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(base) + off) = uint4{v.x, v.y, v.z, v.w};
}
template <int SC1>
__device__ __forceinline__ void car_st_b32(float* base, unsigned bytes, size_t off, float v) {
  if constexpr (SC1)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), car_rsrc(base, bytes), (unsigned)off, 0, 16);
  else
    *reinterpret_cast<float*>(reinterpret_cast<char*>(base) + off) = v;
}

// Block ``blk`` of ``nblk`` of the residual all-reduce: the body of
// car_resid_kernel, and of the residual all-reduce prologue items of the next
// fused GEMM (gemm_skinny.hip, PRO_CAR). SC1: the local results (residual
// slice, statistics tiles) are stored write-through, for consumers in the
// SAME launch that read them with sc1 loads (guide §6 Guideline 16).
template <int LEAN, int SC1>
__device__ __forceinline__ void car_resid_block(const CarPeers& peers, long long in_off, long long res_off,
                                                long long st_off, bf16_t* __restrict__ residual,
                                                float* __restrict__ rowsq_out, int Mpad, int d,
                                                int rank, int world, int blk, int nblk) {
  CarSignals* me = reinterpret_cast<CarSignals*>(peers.base[rank]);
  const unsigned e = ld_sys(&me->epoch) + 1;
  const int owned = d / world, cw = owned / nblk;     // columns per rank / per block
  const int c0 = rank * owned + blk * cw;
  const unsigned in_bytes = (unsigned)((size_t)Mpad * d * 4), res_bytes = (unsigned)((size_t)Mpad * d * 2);
  const unsigned st_bytes = (unsigned)((size_t)nblk * Mpad * 4);
  const unsigned out_st_bytes = (unsigned)((size_t)world * nblk * Mpad * 4);
  bool ok = car_arrive_wait(peers, rank, world, blk, e);
  if (ok) {
    const int vpr = cw >> 2;                           // f32x4 vectors per row
    const int rpp = 256 / vpr, r0 = threadIdx.x / vpr, cv = threadIdx.x % vpr;
    bf16_t* rmine = reinterpret_cast<bf16_t*>(peers.base[rank] + res_off);
    float* smine = reinterpret_cast<float*>(peers.base[rank] + st_off);
    for (int m0 = 0; m0 < Mpad; m0 += rpp) {
      const int m = m0 + r0;
      const bool act = r0 < rpp && m < Mpad;
      float sq = 0.f;
      if (act) {
        const size_t el = (size_t)m * d + c0 + cv * 4;
        const uint2 rv = *reinterpret_cast<const uint2*>(residual + el);
        car_u32x4 v[CAR_MAX_WORLD];
#pragma unroll
        for (int q = 0; q < CAR_MAX_WORLD; ++q)
          if (q < world)
            v[q] = __builtin_amdgcn_raw_buffer_load_b128(car_rsrc(peers.base[q] + in_off, in_bytes),
                                                         (unsigned)(el * 4), 0, CAR_SYS);
        uint2 o;
        sq = car_resid_math(rv, v, world, o);
        car_st_b64<SC1>(residual, res_bytes, el * 2, o);
        if constexpr (LEAN)
          __builtin_amdgcn_raw_buffer_store_b64(u32x2_car{o.x, o.y}, car_rsrc(rmine, res_bytes),
                                                (unsigned)(el * 2), 0, CAR_SYS);
        else
          *reinterpret_cast<uint2*>(rmine + el) = o;
      }
      sq = car_row_butterfly(sq, vpr);
      if (cv == 0 && act) {
        if constexpr (LEAN)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sq), car_rsrc(smine, st_bytes),
                                                (unsigned)(((size_t)blk * Mpad + m) * 4), 0, CAR_SYS);
        else
          smine[(size_t)blk * Mpad + m] = sq;
        car_st_b32<SC1>(rowsq_out, out_st_bytes, (((size_t)rank * nblk + blk) * Mpad + m) * 4, sq);
      }
    }
    // phase 2: publish (release at system scope, as car_barrier; LEAN: see
    // car_publish_wait), then gather every other rank's rounded sub-slice b
    // and its statistics
    ok = car_publish_wait<LEAN>(peers, rank, world, blk, e);
    if (ok) {
      const int vb = cw >> 3;                          // bf16x8 vectors per row of a sub-slice
      for (int q = 0; q < world; ++q) {
        if (q == rank) continue;
        const int cq = q * owned + blk * cw;
        const auto rr = car_rsrc(peers.base[q] + res_off, res_bytes);
        for (int t = threadIdx.x; t < Mpad * vb; t += 256) {
          const int m = t / vb, c = t - m * vb;
          const size_t el = (size_t)m * d + cq + c * 8;
          const car_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rr, (unsigned)(el * 2), 0, CAR_SYS);
          car_st_b128<SC1>(residual, res_bytes, el * 2, v);
        }
        const auto rs = car_rsrc(peers.base[q] + st_off, st_bytes);
        for (int m = threadIdx.x; m < Mpad; m += 256)
          car_st_b32<SC1>(rowsq_out, out_st_bytes, (((size_t)q * nblk + blk) * Mpad + m) * 4,
                          __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                              rs, (unsigned)(((size_t)blk * Mpad + m) * 4), 0, CAR_SYS)));
      }
    }
  }
  car_epoch_done(me, e, nblk);
}


// host: the peer table and region offsets of handle ``hp`` for input buffer
// ``which`` (custom_allreduce.hip), for a GEMM launch that runs the residual
// all-reduce as its prologue (gemm_skinny.hip PRO_CAR); 0 on success
int car_prologue_args(void* hp, int which, CarPeers* peers, long long* in_off, long long* res_off,
                      long long* st_off, int* rank, int* world, size_t* in_bytes);
