// Native host runtime for the MI355X voice hub.
//
//  * PcmStager   - pinned (hipHostMalloc) host slots that relay PCM frames are
//                  appended into as they arrive on the gRPC stream, then moved
//                  to HBM with hipMemcpyAsync on the consuming stream (or, opt-in,
//                  a dedicated H2D stream); a HIP
//                  event per transfer gates slot reuse (SURVEY §2.4 "Host<->device
//                  data path"). Replaces the reference's per-sample Go
//                  conversion loop + WAV/HTTP round trip (audio_service.go:1048,
//                  stt_client.go:365).
//  * BlockPool   - paged KV-cache block allocator with per-sequence block tables,
//                  reference counts and a prefix cache so prompts that share the
//                  parser template prefix share KV blocks.
//                  The cache is looked up by a chained hash but every hit is
//                  verified against the block's stored token prefix, so a hash
//                  collision can never hand out another prompt's KV.
// Exposed through a flat C ABI (loaded with ctypes after torch, so the process
// has exactly one HIP runtime).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

// ------------------------------------------------------------------ PcmStager
struct Slot {
  int16_t* host = nullptr;  // pinned
  int64_t len = 0;          // samples written
  bool busy = false;        // owned by a producer or in flight
  hipEvent_t done = nullptr;
  bool in_flight = false;
  // stream-in mode: device mirror of the slot, filled while the relay speaks
  int16_t* dev = nullptr;
  int64_t flushed = 0;      // samples already copied to dev (issued on the H2D stream)
  hipEvent_t flush_ev = nullptr;
};

struct PcmStager {
  std::vector<Slot> slots;
  int64_t cap = 0;  // samples per slot
  std::mutex mu;
  hipStream_t h2d = nullptr;
  bool own_h2d = false;     // created here (destroyed here) vs set by the caller
  bool stream_in = false;   // per-chunk copies into the device mirrors
};

// ------------------------------------------------------------------ BlockPool
struct Seq {
  std::vector<int32_t> blocks;
  int64_t len = 0;  // tokens stored
};

struct BlockPool {
  int32_t num_blocks = 0, block_size = 0;
  std::vector<int32_t> refcnt;
  std::deque<int32_t> free_list;
  std::unordered_map<int64_t, Seq> seqs;
  // prefix cache: chained hash of full blocks -> candidate block ids (each
  // holds one reference); a cached block keeps the WHOLE token prefix it ends
  // (tokens 0 .. its last token), compared on every hit
  std::unordered_multimap<uint64_t, int32_t> prefix;
  struct Cached {
    uint64_t hash;
    std::vector<int32_t> toks;
  };
  std::unordered_map<int32_t, Cached> cached;
  uint64_t hash_mask = ~0ULL;  // tests narrow it to force collisions
  std::mutex mu;

  // cached block whose stored prefix equals toks[0:n], or -1
  int32_t lookup(uint64_t h, const int32_t* toks, int n) const {
    auto range = prefix.equal_range(h);
    for (auto it = range.first; it != range.second; ++it) {
      const Cached& c = cached.at(it->second);
      if ((int)c.toks.size() == n && std::memcmp(c.toks.data(), toks, sizeof(int32_t) * n) == 0)
        return it->second;
    }
    return -1;
  }
  void uncache(int32_t b) {
    auto c = cached.find(b);
    if (c == cached.end()) return;
    auto range = prefix.equal_range(c->second.hash);
    for (auto it = range.first; it != range.second; ++it) {
      if (it->second == b) {
        prefix.erase(it);
        break;
      }
    }
    cached.erase(c);
  }

  int32_t take() {
    if (free_list.empty()) {
      // evict an unreferenced cached prefix block
      for (auto it = cached.begin(); it != cached.end(); ++it) {
        const int32_t b = it->first;
        if (refcnt[b] == 1) {
          uncache(b);
          refcnt[b] = 0;
          return take_fresh(b);
        }
      }
      return -1;
    }
    const int32_t b = free_list.front();
    free_list.pop_front();
    return take_fresh(b);
  }
  int32_t take_fresh(int32_t b) {
    refcnt[b] = 1;
    return b;
  }
  void release(int32_t b) {
    if (--refcnt[b] == 0) free_list.push_back(b);
  }
};

uint64_t mix_hash(uint64_t h, const int32_t* toks, int n) {
  // FNV-1a over the token ids, chained from the previous block's hash
  uint64_t x = h ^ 0xcbf29ce484222325ULL;
  for (int i = 0; i < n; ++i) {
    x ^= (uint64_t)(uint32_t)toks[i];
    x *= 0x100000001b3ULL;
  }
  return x;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- stager API
// own_stream = 0: each upload is issued on the consuming stream itself. A
// stream created here, after the serving streams, would take the next of the
// process's hardware queues (HIP maps streams to queues in creation order) and
// can land on a decoder's queue (both decoders ~2x slower when they share one;
// docs/PERF.md, "the 1.8x cliff"). The PCM copy is ~1 MB, so serialising it
// on the encoder stream costs nothing measurable.
void* loqa_stager_create(int nslots, long long samples_per_slot, int own_stream) {
  auto* s = new PcmStager();
  s->cap = samples_per_slot;
  s->slots.resize(nslots);
  if (own_stream && hipStreamCreateWithFlags(&s->h2d, hipStreamNonBlocking) != hipSuccess) {
    delete s;
    return nullptr;
  }
  s->own_h2d = own_stream != 0;
  for (auto& sl : s->slots) {
    if (hipHostMalloc((void**)&sl.host, sizeof(int16_t) * samples_per_slot, hipHostMallocDefault) !=
            hipSuccess ||
        hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess) {
      return nullptr;
    }
  }
  return s;
}

void loqa_stager_destroy(void* h) {
  auto* s = static_cast<PcmStager*>(h);
  if (!s) return;
  for (auto& sl : s->slots) {
    if (sl.done && sl.in_flight) hipEventSynchronize(sl.done);
  }
  if (s->h2d) hipStreamSynchronize(s->h2d);
  for (auto& sl : s->slots) {
    if (sl.host) hipHostFree(sl.host);
    if (sl.done) hipEventDestroy(sl.done);
    if (sl.dev) hipFree(sl.dev);
    if (sl.flush_ev) hipEventDestroy(sl.flush_ev);
  }
  if (s->h2d && s->own_h2d) hipStreamDestroy(s->h2d);
  delete s;
}

// Stream-in mode (SURVEY §2.4 "Host<->device data path"): every slot gets a
// device mirror, and loqa_stager_flush copies the samples appended since the
// last flush with hipMemcpyAsync on `stream` - a placed side stream owned by
// the caller (utils/streams.py "h2d"), so the transfer runs while the relay is
// still speaking and end of speech only copies the tail. Returns 0 or a HIP
// error (a failed mirror allocation leaves the mode off).
int loqa_stager_set_stream(void* h, hipStream_t stream, int stream_in) {
  auto* s = static_cast<PcmStager*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  if (s->h2d && s->own_h2d) return (int)hipErrorInvalidValue;
  s->h2d = stream;
  if (stream_in && !s->stream_in) {
    for (auto& sl : s->slots) {
      if (!sl.dev) {
        hipError_t e = hipMalloc((void**)&sl.dev, sizeof(int16_t) * (size_t)s->cap);
        if (e != hipSuccess) return (int)e;
        e = hipEventCreateWithFlags(&sl.flush_ev, hipEventDisableTiming);
        if (e != hipSuccess) return (int)e;
      }
    }
    s->stream_in = true;
  }
  return 0;
}

// Copy the samples appended since the last flush into the slot's device
// mirror on the H2D stream when at least min_samples are pending. Returns the
// samples issued (0: below the threshold or not in stream-in mode), or a
// negative HIP error.
long long loqa_stager_flush(void* h, int slot, long long min_samples) {
  auto* s = static_cast<PcmStager*>(h);
  Slot& sl = s->slots[slot];
  if (!s->stream_in || !sl.dev) return 0;
  const long long n = sl.len - sl.flushed;
  if (n <= 0 || n < min_samples) return 0;
  hipError_t e = hipMemcpyAsync(sl.dev + sl.flushed, sl.host + sl.flushed, (size_t)n * 2,
                                hipMemcpyHostToDevice, s->h2d);
  if (e == hipSuccess) e = hipEventRecord(sl.flush_ev, s->h2d);
  if (e != hipSuccess) return -(long long)e;
  sl.flushed = sl.len;
  return n;
}

long long loqa_stager_flushed(void* h, int slot) {
  return static_cast<PcmStager*>(h)->slots[slot].flushed;
}

// Acquire a free slot (reclaiming slots whose transfer completed). -1 if none.
int loqa_stager_acquire(void* h) {
  auto* s = static_cast<PcmStager*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  for (size_t i = 0; i < s->slots.size(); ++i) {
    Slot& sl = s->slots[i];
    if (sl.busy && sl.in_flight && hipEventQuery(sl.done) == hipSuccess) {
      sl.busy = false;
      sl.in_flight = false;
    }
    if (!sl.busy) {
      sl.busy = true;
      sl.len = 0;
      sl.flushed = 0;
      return (int)i;
    }
  }
  return -1;
}

// Append little-endian PCM16 bytes; an odd trailing byte is dropped (as the
// reference does). Returns samples appended, or -1 on overflow.
long long loqa_stager_append(void* h, int slot, const uint8_t* bytes, long long nbytes) {
  auto* s = static_cast<PcmStager*>(h);
  Slot& sl = s->slots[slot];
  const long long n = nbytes / 2;
  if (sl.len + n > s->cap) return -1;
  std::memcpy(sl.host + sl.len, bytes, (size_t)n * 2);
  sl.len += n;
  return n;
}

long long loqa_stager_len(void* h, int slot) { return static_cast<PcmStager*>(h)->slots[slot].len; }

const void* loqa_stager_host_ptr(void* h, int slot) {
  return static_cast<PcmStager*>(h)->slots[slot].host;
}

// Async H2D of the slot's samples into dst (device): on the stager's own H2D
// stream (then `wait_stream`, the compute stream, waits for the copy) or, with
// no own stream, on `wait_stream` itself. The slot is recycled once the copy's
// event has completed.
// Stream-in mode: only the samples not yet flushed cross PCIe now (on the H2D
// stream), `wait_stream` waits for the slot's last flush event, and the
// mirror is copied device-to-device into dst on `wait_stream`.
int loqa_stager_upload(void* h, int slot, void* dst, long long max_samples, hipStream_t wait_stream) {
  auto* s = static_cast<PcmStager*>(h);
  Slot& sl = s->slots[slot];
  const long long n = sl.len < max_samples ? sl.len : max_samples;
  hipError_t e = hipSuccess;
  if (s->stream_in && sl.dev && sl.flushed > 0) {   // (never flushed: the direct copy below)
    if (n > sl.flushed) {
      e = hipMemcpyAsync(sl.dev + sl.flushed, sl.host + sl.flushed, (size_t)(n - sl.flushed) * 2,
                         hipMemcpyHostToDevice, s->h2d);
      if (e == hipSuccess) e = hipEventRecord(sl.flush_ev, s->h2d);
      if (e != hipSuccess) return (int)e;
      sl.flushed = n;
    }
    if (sl.flushed > 0) e = hipStreamWaitEvent(wait_stream, sl.flush_ev, 0);
    if (e == hipSuccess && n > 0)
      e = hipMemcpyAsync(dst, sl.dev, (size_t)n * 2, hipMemcpyDeviceToDevice, wait_stream);
    if (e == hipSuccess) e = hipEventRecord(sl.done, wait_stream);
    if (e != hipSuccess) return (int)e;
    std::lock_guard<std::mutex> g(s->mu);
    sl.in_flight = true;
    return 0;
  }
  hipStream_t cs = s->h2d ? s->h2d : wait_stream;
  if (n > 0) e = hipMemcpyAsync(dst, sl.host, (size_t)n * 2, hipMemcpyHostToDevice, cs);
  if (e != hipSuccess) return (int)e;
  e = hipEventRecord(sl.done, cs);
  if (e != hipSuccess) return (int)e;
  if (wait_stream && s->h2d) e = hipStreamWaitEvent(wait_stream, sl.done, 0);
  std::lock_guard<std::mutex> g(s->mu);
  sl.in_flight = true;
  return (int)e;
}

// Plain async H2D copy (a slot chain's host-buffered tail).
int loqa_memcpy_h2d_async(void* dst, const void* src, long long nbytes, hipStream_t stream) {
  return (int)hipMemcpyAsync(dst, src, (size_t)nbytes, hipMemcpyHostToDevice, stream);
}

void loqa_stager_release(void* h, int slot) {
  auto* s = static_cast<PcmStager*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  Slot& sl = s->slots[slot];
  if (!sl.in_flight) sl.busy = false;  // otherwise reclaimed on event completion
}

// ------------------------------------------------------------- block pool API
void* loqa_pool_create(int num_blocks, int block_size) {
  auto* p = new BlockPool();
  p->num_blocks = num_blocks;
  p->block_size = block_size;
  p->refcnt.assign(num_blocks, 0);
  for (int i = 0; i < num_blocks; ++i) p->free_list.push_back(i);
  return p;
}

void loqa_pool_destroy(void* h) { delete static_cast<BlockPool*>(h); }

// Test hook: keep only the masked bits of the prefix hash (mask 0 makes every
// block collide, so lookups must be decided by the stored tokens alone).
void loqa_pool_debug_hash_mask(void* h, unsigned long long mask) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  p->hash_mask = mask;
}

int loqa_pool_free_blocks(void* h) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  int n = (int)p->free_list.size();
  for (auto& kv : p->cached)
    if (p->refcnt[kv.first] == 1) ++n;
  return n;
}

// Register a sequence and try to reuse cached full prefix blocks for `toks`.
// Returns the number of tokens whose KV is already present (multiple of block
// size, always < ntok so at least one token is computed), or -1 on error.
long long loqa_pool_add_seq(void* h, long long seq_id, const int32_t* toks, int ntok) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  if (p->seqs.count(seq_id)) return -1;
  Seq sq;
  uint64_t hsh = 0;
  const int bs = p->block_size;
  for (int i = 0; i + bs < ntok; i += bs) {  // keep >= 1 token to compute
    hsh = mix_hash(hsh, toks + i, bs) & p->hash_mask;
    const int32_t b = p->lookup(hsh, toks, i + bs);
    if (b < 0) break;
    p->refcnt[b]++;
    sq.blocks.push_back(b);
    sq.len += bs;
  }
  p->seqs.emplace(seq_id, std::move(sq));
  return p->seqs[seq_id].len;
}

// Reserve KV slots for n more tokens; writes slot ids (block*bs + off) to out.
int loqa_pool_append(void* h, long long seq_id, int n, int32_t* out_slots) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  auto it = p->seqs.find(seq_id);
  if (it == p->seqs.end()) return -1;
  Seq& sq = it->second;
  const int bs = p->block_size;
  for (int i = 0; i < n; ++i) {
    const long long pos = sq.len + i;
    const int bi = (int)(pos / bs);
    if (bi >= (int)sq.blocks.size()) {
      const int32_t b = p->take();
      if (b < 0) return -2;  // out of KV memory
      sq.blocks.push_back(b);
    }
    out_slots[i] = sq.blocks[bi] * bs + (int)(pos % bs);
  }
  sq.len += n;
  return 0;
}

// Publish the sequence's full blocks of `toks` (its first ntok tokens) to the
// prefix cache so later prompts with the same prefix can reuse them.
int loqa_pool_cache_prefix(void* h, long long seq_id, const int32_t* toks, int ntok) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  auto it = p->seqs.find(seq_id);
  if (it == p->seqs.end()) return -1;
  const int bs = p->block_size;
  uint64_t hsh = 0;
  for (int i = 0, bi = 0; i + bs <= ntok && bi < (int)it->second.blocks.size(); i += bs, ++bi) {
    hsh = mix_hash(hsh, toks + i, bs) & p->hash_mask;
    const int32_t b = it->second.blocks[bi];
    if (p->cached.count(b) || p->lookup(hsh, toks, i + bs) >= 0) continue;
    p->prefix.emplace(hsh, b);
    p->cached.emplace(b, BlockPool::Cached{hsh, std::vector<int32_t>(toks, toks + i + bs)});
    p->refcnt[b]++;  // the cache's own reference
  }
  return 0;
}

// One decode / prefill step's KV metadata in a single call (the per-sequence
// seq_len / append / block_table round trips from Python cost ~50 us per
// sequence per step on the scheduler's critical path). For the B sequences,
// append n[i] tokens each and fill, for a padded step of T_pad tokens and
// B_pad sequences: positions / slots (concatenated per sequence; padding rows
// position 0, slot -1), cu_q [B_pad + 1] (padding sequences empty), ctx_lens
// [B_pad], block_tables [B_pad][max_blocks] (zero padded) and, if lidx, the
// index of each sequence's last token (lidx_len entries, rest 0).
// Returns 0; -1 unknown sequence, -2 out of KV blocks, -3 shape overflow.
int loqa_pool_step_meta(void* h, int B, const long long* seq_ids, const int* n, int B_pad, int T_pad,
                        int max_blocks, int32_t* positions, int32_t* slots, int32_t* cu, int32_t* ctx,
                        int32_t* bt, long long* lidx, int lidx_len) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  if (B > B_pad || (lidx && B > lidx_len)) return -3;
  int T = 0;
  for (int i = 0; i < B; ++i) T += n[i];
  if (T > T_pad) return -3;
  for (int i = 0; i < T_pad; ++i) {
    positions[i] = 0;
    slots[i] = -1;
  }
  std::memset(bt, 0, sizeof(int32_t) * (size_t)B_pad * max_blocks);
  const int bs = p->block_size;
  int off = 0;
  cu[0] = 0;
  for (int i = 0; i < B; ++i) {
    auto it = p->seqs.find(seq_ids[i]);
    if (it == p->seqs.end()) return -1;
    Seq& sq = it->second;
    for (int j = 0; j < n[i]; ++j) {
      const long long pos = sq.len + j;
      const int bi = (int)(pos / bs);
      if (bi >= (int)sq.blocks.size()) {
        const int32_t b = p->take();
        if (b < 0) return -2;
        sq.blocks.push_back(b);
      }
      positions[off + j] = (int32_t)pos;
      slots[off + j] = sq.blocks[bi] * bs + (int)(pos % bs);
    }
    sq.len += n[i];
    off += n[i];
    cu[i + 1] = off;
    ctx[i] = (int32_t)sq.len;
    const int nb = (int)sq.blocks.size();
    if (nb > max_blocks) return -3;
    std::memcpy(bt + (size_t)i * max_blocks, sq.blocks.data(), sizeof(int32_t) * nb);
    if (lidx) lidx[i] = off - 1;
  }
  for (int i = B; i < B_pad; ++i) {
    cu[i + 1] = off;
    ctx[i] = 0;
  }
  if (lidx)
    for (int i = B; i < lidx_len; ++i) lidx[i] = 0;
  return 0;
}

int loqa_pool_block_table(void* h, long long seq_id, int32_t* out, int max_blocks) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  auto it = p->seqs.find(seq_id);
  if (it == p->seqs.end()) return -1;
  const int n = (int)it->second.blocks.size();
  if (n > max_blocks) return -2;
  for (int i = 0; i < n; ++i) out[i] = it->second.blocks[i];
  return n;
}

long long loqa_pool_seq_len(void* h, long long seq_id) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  auto it = p->seqs.find(seq_id);
  return it == p->seqs.end() ? -1 : it->second.len;
}

// Roll a sequence back to its first new_len tokens (a discarded speculative
// step of the pipelined decode): blocks past the new length go back to the
// pool. Returns 0, -1 unknown sequence, -2 new_len beyond the sequence.
int loqa_pool_truncate(void* h, long long seq_id, long long new_len) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  auto it = p->seqs.find(seq_id);
  if (it == p->seqs.end()) return -1;
  Seq& sq = it->second;
  if (new_len < 0 || new_len > sq.len) return -2;
  const size_t keep = (size_t)((new_len + p->block_size - 1) / p->block_size);
  while (sq.blocks.size() > keep) {
    p->release(sq.blocks.back());
    sq.blocks.pop_back();
  }
  sq.len = new_len;
  return 0;
}

int loqa_pool_free_seq(void* h, long long seq_id) {
  auto* p = static_cast<BlockPool*>(h);
  std::lock_guard<std::mutex> g(p->mu);
  auto it = p->seqs.find(seq_id);
  if (it == p->seqs.end()) return -1;
  for (int32_t b : it->second.blocks) p->release(b);
  p->seqs.erase(it);
  return 0;
}

}  // extern "C"
