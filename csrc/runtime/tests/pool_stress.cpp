// Host-side stress test of the paged-KV BlockPool (runtime.cpp), built with
// -fsanitize=address,undefined or -fsanitize=thread (sanitizers on
// host code). Several threads run random sequence lifecycles (add with prefix
// reuse, append, publish prefix, free) against one pool; invariants checked at
// the end: every block is either free, cached, or owned, and freeing every
// sequence returns the pool to (free + cached) == num_blocks.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <random>
#include <thread>
#include <unistd.h>
#include <cstring>
#include <vector>

extern "C" {
void* loqa_pool_create(int num_blocks, int block_size);
void loqa_pool_destroy(void* h);
int loqa_pool_free_blocks(void* h);
long long loqa_pool_add_seq(void* h, long long seq_id, const int32_t* toks, int ntok);
int loqa_pool_append(void* h, long long seq_id, int n, int32_t* out_slots);
int loqa_pool_cache_prefix(void* h, long long seq_id, const int32_t* toks, int ntok);
int loqa_pool_block_table(void* h, long long seq_id, int32_t* out, int max_blocks);
long long loqa_pool_seq_len(void* h, long long seq_id);
int loqa_pool_free_seq(void* h, long long seq_id);
void* loqa_tpctl_open(const char* name, int rank, int world, int nslots, long long slot_bytes);
void loqa_tpctl_unlink(void* h);
int loqa_tpctl_publish(void* h, const void* data, long long n, int stop, long long timeout_us);
long long loqa_tpctl_recv(void* h, void* buf, long long cap, int* stop, long long timeout_us);
void loqa_tpctl_close(void* h);
}

int main() {
  const int NB = 512, BS = 16, THREADS = 4, ITERS = 400;
  void* pool = loqa_pool_create(NB, BS);
  std::atomic<long long> next_id{1};
  std::atomic<int> errors{0};
  auto worker = [&](int tid) {
    std::mt19937 rng(1234 + tid);
    std::vector<int32_t> prefix(96);
    for (auto& t : prefix) t = (int32_t)(rng() % 1000);
    for (int it = 0; it < ITERS; ++it) {
      const long long id = next_id++;
      std::vector<int32_t> toks(prefix.begin(), prefix.begin() + 16 * (1 + rng() % 5));
      for (int i = 0; i < (int)(rng() % 40); ++i) toks.push_back((int32_t)(rng() % 1000));
      const long long hit = loqa_pool_add_seq(pool, id, toks.data(), (int)toks.size());
      if (hit < 0 || hit % BS || hit >= (long long)toks.size()) { ++errors; continue; }
      std::vector<int32_t> slots(toks.size());
      const int n = (int)(toks.size() - hit);
      if (loqa_pool_append(pool, id, n, slots.data()) != 0) {  // pool exhausted: legal
        loqa_pool_free_seq(pool, id);
        continue;
      }
      if (loqa_pool_seq_len(pool, id) != (long long)toks.size()) ++errors;
      for (int i = 0; i < n; ++i)
        if (slots[i] < 0 || slots[i] >= NB * BS) ++errors;
      int32_t table[64];
      const int nb = loqa_pool_block_table(pool, id, table, 64);
      if (nb != (int)((toks.size() + BS - 1) / BS)) ++errors;
      if (rng() % 2) loqa_pool_cache_prefix(pool, id, toks.data(), (int)toks.size());
      if (loqa_pool_free_seq(pool, id) != 0) ++errors;
    }
  };
  std::vector<std::thread> ts;
  for (int t = 0; t < THREADS; ++t) ts.emplace_back(worker, t);
  for (auto& t : ts) t.join();
  const int free_blocks = loqa_pool_free_blocks(pool);
  if (free_blocks != NB) {
    std::printf("leak: %d of %d blocks reclaimable\n", free_blocks, NB);
    ++errors;
  }
  loqa_pool_destroy(pool);
  std::printf("pool_stress: %d errors\n", errors.load());

  // TP lock-step control ring: one leader thread publishes records of varying
  // size (some larger than a slot: continuation chunks) through a ring of 4
  // slots, three follower threads must see every record, in order, intact.
  {
    const int W = 4, RECS = 3000, SLOT = 256;
    char name[64];
    std::snprintf(name, sizeof name, "/loqa_tpctl_stress_%d", (int)getpid());
    void* lead = loqa_tpctl_open(name, 0, W, 4, SLOT);
    if (!lead) { std::printf("tpctl: open failed\n"); return 1; }
    std::vector<void*> fol(W, nullptr);
    for (int r = 1; r < W; ++r) fol[r] = loqa_tpctl_open(name, r, W, 4, SLOT);
    loqa_tpctl_unlink(lead);
    std::atomic<int> ring_errors{0};
    auto payload = [](int i, std::vector<unsigned char>& v) {
      v.resize((size_t)((i * 37) % 900));
      for (size_t k = 0; k < v.size(); ++k) v[k] = (unsigned char)(i * 31 + k);
    };
    std::vector<std::thread> fs;
    for (int r = 1; r < W; ++r)
      fs.emplace_back([&, r] {
        std::vector<unsigned char> buf(4096), want;
        for (int i = 0;; ++i) {
          int stop = 0;
          const long long n = loqa_tpctl_recv(fol[r], buf.data(), (long long)buf.size(), &stop,
                                              10000000);
          if (n < 0) { ++ring_errors; return; }
          if (stop) { if (i != RECS) ++ring_errors; return; }
          payload(i, want);
          if ((size_t)n != want.size() || (n && std::memcmp(buf.data(), want.data(), want.size())))
            ++ring_errors;
        }
      });
    std::vector<unsigned char> v;
    for (int i = 0; i < RECS; ++i) {
      payload(i, v);
      if (loqa_tpctl_publish(lead, v.data(), (long long)v.size(), 0, 10000000) != 0) ++ring_errors;
    }
    loqa_tpctl_publish(lead, nullptr, 0, 1, 10000000);
    for (auto& t : fs) t.join();
    for (int r = 1; r < W; ++r) loqa_tpctl_close(fol[r]);
    loqa_tpctl_close(lead);
    std::printf("tpctl_stress: %d errors\n", ring_errors.load());
    errors += ring_errors.load();
  }
  return errors.load() == 0 ? 0 : 1;
}
