// Lock-step control ring for tensor-parallel serving.
//
// A TP group runs one LLM engine per rank; every rank must launch the same
// decode steps, in the same order, with the same batch - the only input that
// is not already identical on every rank (the sampled tokens are: the argmax
// combine is bitwise deterministic) is WHICH requests arrived before each
// scheduler iteration. Rank 0 (the leader, which owns the hub front end)
// publishes one record per iteration - the new requests, or nothing - and the
// followers replay it.
//
// Transport: one POSIX shared-memory region per TP group on the node
// (/dev/shm), a ring of fixed-size slots, a monotonic `published` counter
// written by the leader and one `consumed` counter per follower. A record
// larger than a slot is split into continuation chunks. Publishing is a
// memcpy and a release store (~1 us); a follower that is waiting spins
// briefly, then sleeps in growing steps, so an idle hub costs no CPU.
//
// Liveness: every rank stamps its own heartbeat word (steady-clock us, from a
// thread of its own); the leader reads the followers' ages to detect a lost
// follower even while the hub is idle (no collective would notice it then).
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>

namespace {

constexpr uint64_t kMagic = 0x4c4f51415443544cull;  // "LOQATCTL"
constexpr int kMaxWorld = 64;
constexpr uint32_t kFlagMore = 1u;   // chunk continues in the next slot
constexpr uint32_t kFlagStop = 2u;   // the leader has shut down

struct Header {
  uint64_t magic;
  uint32_t world, nslots;
  uint64_t slot_bytes;
  alignas(64) std::atomic<uint64_t> published;
  alignas(64) std::atomic<uint64_t> consumed[kMaxWorld];
  alignas(64) std::atomic<int64_t> beat[kMaxWorld];   // steady-clock us; 0 = never
};

int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct SlotHead {
  uint64_t seq;
  uint32_t len;
  uint32_t flags;
};

struct Ctl {
  int rank = 0;
  Header* hdr = nullptr;
  char* slots = nullptr;
  size_t map_bytes = 0;
  std::string name;
  bool owner = false;
};

size_t region_bytes(uint32_t nslots, uint64_t slot_bytes) {
  return sizeof(Header) + (size_t)nslots * (sizeof(SlotHead) + slot_bytes);
}

char* slot_ptr(Ctl* c, uint64_t seq) {
  const size_t stride = sizeof(SlotHead) + c->hdr->slot_bytes;
  return c->slots + (size_t)(seq % c->hdr->nslots) * stride;
}

// spin ~50 us, then sleep 20 us .. 1 ms; false once `deadline` passes
template <class Pred>
bool wait_for(Pred ready, int64_t timeout_us) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  int64_t sleep_us = 20;
  for (int i = 0;; ++i) {
    if (ready()) return true;
    const int64_t el = std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t0).count();
    if (timeout_us >= 0 && el > timeout_us) return false;
    if (el < 50) continue;
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    if (sleep_us < 1000) sleep_us += sleep_us / 2;
  }
}

}  // namespace

extern "C" {

// rank 0 creates (replacing a stale region of the same name), followers open
// the existing region (call after the leader's create, e.g. behind a barrier).
void* loqa_tpctl_open(const char* name, int rank, int world, int nslots, long long slot_bytes) {
  if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world || nslots < 2 || slot_bytes < 64)
    return nullptr;
  Ctl* c = new Ctl();
  c->rank = rank;
  c->name = name;
  c->map_bytes = region_bytes((uint32_t)nslots, (uint64_t)slot_bytes);
  int fd;
  if (rank == 0) {
    shm_unlink(name);
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)c->map_bytes) != 0) {
      if (fd >= 0) close(fd);
      delete c;
      return nullptr;
    }
    c->owner = true;
  } else {
    fd = shm_open(name, O_RDWR, 0600);
    if (fd < 0) {
      delete c;
      return nullptr;
    }
  }
  void* p = mmap(nullptr, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (c->owner) shm_unlink(name);
    delete c;
    return nullptr;
  }
  c->hdr = static_cast<Header*>(p);
  c->slots = static_cast<char*>(p) + sizeof(Header);
  if (rank == 0) {
    std::memset(p, 0, sizeof(Header));
    c->hdr->world = (uint32_t)world;
    c->hdr->nslots = (uint32_t)nslots;
    c->hdr->slot_bytes = (uint64_t)slot_bytes;
    std::atomic_thread_fence(std::memory_order_release);
    reinterpret_cast<std::atomic<uint64_t>*>(&c->hdr->magic)->store(kMagic, std::memory_order_release);
  } else if (c->hdr->magic != kMagic || c->hdr->world != (uint32_t)world ||
             c->hdr->nslots != (uint32_t)nslots || c->hdr->slot_bytes != (uint64_t)slot_bytes) {
    munmap(p, c->map_bytes);
    delete c;
    return nullptr;
  }
  return c;
}

// the name can go once every rank has mapped the region (the mapping stays)
void loqa_tpctl_unlink(void* h) {
  Ctl* c = static_cast<Ctl*>(h);
  if (c && c->owner) shm_unlink(c->name.c_str());
}

// leader: one record (n bytes; stop != 0 marks shutdown). 0, or -1 when a
// follower stopped consuming for `timeout_us` (ring full).
int loqa_tpctl_publish(void* h, const void* data, long long n, int stop, long long timeout_us) {
  Ctl* c = static_cast<Ctl*>(h);
  if (!c || c->rank != 0 || n < 0) return -2;
  Header* hd = c->hdr;
  const char* src = static_cast<const char*>(data);
  long long off = 0;
  do {
    const uint64_t seq = hd->published.load(std::memory_order_relaxed);
    const bool ok = wait_for([&] {
      for (uint32_t r = 1; r < hd->world; ++r)
        if (seq - hd->consumed[r].load(std::memory_order_acquire) >= hd->nslots) return false;
      return true;
    }, timeout_us);
    if (!ok) return -1;
    const long long len = (n - off) < (long long)hd->slot_bytes ? (n - off) : (long long)hd->slot_bytes;
    char* s = slot_ptr(c, seq);
    SlotHead sh{seq, (uint32_t)len, (uint32_t)((off + len < n ? kFlagMore : 0u) | (stop ? kFlagStop : 0u))};
    std::memcpy(s, &sh, sizeof(sh));
    if (len) std::memcpy(s + sizeof(SlotHead), src + off, (size_t)len);
    hd->published.store(seq + 1, std::memory_order_release);
    off += len;
  } while (off < n);
  return 0;
}

// follower: the next record into buf (cap bytes). Returns its length, or -1 on
// timeout (nothing consumed), -3 when cap is too small (the record is skipped),
// and sets *stop when the leader marked it as its last.
long long loqa_tpctl_recv(void* h, void* buf, long long cap, int* stop, long long timeout_us) {
  Ctl* c = static_cast<Ctl*>(h);
  if (!c || c->rank == 0) return -2;
  Header* hd = c->hdr;
  std::atomic<uint64_t>& mine = hd->consumed[c->rank];
  char* dst = static_cast<char*>(buf);
  long long total = 0;
  bool overflow = false;
  *stop = 0;
  for (bool first = true;; first = false) {
    const uint64_t seq = mine.load(std::memory_order_relaxed);
    // the first chunk may take `timeout_us`; continuations follow at once
    if (!wait_for([&] { return hd->published.load(std::memory_order_acquire) > seq; },
                  first ? timeout_us : 10000000))
      return first ? -1 : -4;
    const char* s = slot_ptr(c, seq);
    SlotHead sh;
    std::memcpy(&sh, s, sizeof(sh));
    if (sh.seq != seq) return -5;      // overwritten: the ring protocol broke
    if (total + sh.len <= cap)
      std::memcpy(dst + total, s + sizeof(SlotHead), sh.len);
    else
      overflow = true;
    total += sh.len;
    mine.store(seq + 1, std::memory_order_release);
    if (sh.flags & kFlagStop) *stop = 1;
    if (!(sh.flags & kFlagMore)) break;
  }
  return overflow ? -3 : total;
}

// this rank's heartbeat
void loqa_tpctl_beat(void* h) {
  Ctl* c = static_cast<Ctl*>(h);
  if (c) c->hdr->beat[c->rank].store(now_us(), std::memory_order_release);
}

// microseconds since rank r last beat; -1 if it never did
long long loqa_tpctl_beat_age(void* h, int r) {
  Ctl* c = static_cast<Ctl*>(h);
  if (!c || r < 0 || r >= (int)c->hdr->world) return -2;
  const int64_t b = c->hdr->beat[r].load(std::memory_order_acquire);
  return b == 0 ? -1 : (long long)(now_us() - b);
}

void loqa_tpctl_close(void* h) {
  Ctl* c = static_cast<Ctl*>(h);
  if (!c) return;
  if (c->hdr) munmap(c->hdr, c->map_bytes);
  if (c->owner) shm_unlink(c->name.c_str());
  delete c;
}

}  // extern "C"
