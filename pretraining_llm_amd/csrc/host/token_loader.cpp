// Native token-window loader (host C++, C ABI, no Python/torch dependency).
//
// Replaces the reference's per-sample Python loop over a numpy memmap
// (data_loader/data_loader.py:32-50: torch.randint offsets, list-comprehension
// slices, astype(int64), torch.stack) with:
//   * one mmap of the flat uint16 token file (reference on-disk format,
//     scripts/data_preprocess.py:47-62);
//   * CONTIGUOUS per-rank shards [r*N/W, (r+1)*N/W) instead of the reference's
//     strided data[rank::world] interleave (which destroys text contiguity,
//     SURVEY.md D6);
//   * a seeded counter-based RNG (splitmix64 of (seed, rank, batch, row)), so a
//     batch is a pure function of its index: resume = start at batch k, and any
//     rank/batch can be regenerated bit-exactly;
//   * a producer thread that fills a ring of ready int64 (x, y) batches ahead
//     of the trainer, widened from uint16 in the gather loop.
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

namespace {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Loader {
  const uint16_t* base = nullptr;
  size_t map_bytes = 0;
  int fd = -1;
  int64_t lo = 0, n = 0;  // shard [lo, lo+n)
  int B = 0, T = 0;
  uint64_t seed = 0;
  int64_t rank = 0;
  int nslots = 2;
  std::vector<std::vector<int64_t>> xs, ys;
  std::vector<int64_t> slot_batch;
  int64_t next_produce = 0, next_consume = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<bool> stop{false};
  std::thread worker;

  int64_t offset(int64_t batch, int row) const {
    const uint64_t h = splitmix64(seed ^ splitmix64((uint64_t)rank * 0x100000001B3ull ^ splitmix64((uint64_t)batch * 65537ull + (uint64_t)row)));
    return lo + (int64_t)(h % (uint64_t)(n - T));
  }
  void fill(int64_t batch, int64_t* x, int64_t* y) const {
    for (int r = 0; r < B; ++r) {
      const int64_t o = offset(batch, r);
      const uint16_t* src = base + o;
      int64_t* xr = x + (int64_t)r * T;
      int64_t* yr = y + (int64_t)r * T;
      for (int t = 0; t < T; ++t) {
        xr[t] = src[t];
        yr[t] = src[t + 1];
      }
    }
  }
  void run() {
    for (;;) {
      int slot;
      int64_t batch;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop.load() || next_produce - next_consume < nslots; });
        if (stop.load()) return;
        batch = next_produce;
        slot = (int)(batch % nslots);
      }
      fill(batch, xs[slot].data(), ys[slot].data());
      {
        std::lock_guard<std::mutex> lk(mu);
        slot_batch[slot] = batch;
        next_produce = batch + 1;
      }
      cv.notify_all();
    }
  }
};

}  // namespace

extern "C" {

// returns nullptr on failure (missing file, shard shorter than T+1)
void* pllm_loader_create(const char* path, int64_t rank, int64_t world, int B, int T, uint64_t seed,
                         int64_t start_batch, int prefetch) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return nullptr;
  }
  const size_t bytes = (size_t)st.st_size;
  const int64_t ntok = (int64_t)(bytes / 2);
  void* p = mmap(nullptr, bytes, PROT_READ, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    close(fd);
    return nullptr;
  }
  madvise(p, bytes, MADV_RANDOM);
  auto* L = new Loader();
  L->base = (const uint16_t*)p;
  L->map_bytes = bytes;
  L->fd = fd;
  const int64_t per = ntok / (world > 0 ? world : 1);
  L->lo = per * rank;
  L->n = (rank == world - 1) ? ntok - L->lo : per;
  L->B = B;
  L->T = T;
  L->seed = seed;
  L->rank = rank;
  if (L->n < (int64_t)T + 2) {
    munmap(p, bytes);
    close(fd);
    delete L;
    return nullptr;
  }
  L->nslots = prefetch > 0 ? prefetch : 1;
  L->xs.assign(L->nslots, std::vector<int64_t>((size_t)B * T));
  L->ys.assign(L->nslots, std::vector<int64_t>((size_t)B * T));
  L->slot_batch.assign(L->nslots, -1);
  L->next_produce = L->next_consume = start_batch;
  L->worker = std::thread([L] { L->run(); });
  return L;
}

// copy the next batch into caller buffers (e.g. pinned host memory); returns its batch index
int64_t pllm_loader_next(void* h, int64_t* x, int64_t* y) {
  auto* L = (Loader*)h;
  int64_t batch;
  int slot;
  {
    std::unique_lock<std::mutex> lk(L->mu);
    batch = L->next_consume;
    slot = (int)(batch % L->nslots);
    L->cv.wait(lk, [&] { return L->next_produce > batch; });
  }
  const size_t bytes = (size_t)L->B * L->T * sizeof(int64_t);
  memcpy(x, L->xs[slot].data(), bytes);
  memcpy(y, L->ys[slot].data(), bytes);
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->next_consume = batch + 1;
  }
  L->cv.notify_all();
  return batch;
}

// synchronous, stateless: the batch with index `batch` (for tests / regeneration)
void pllm_loader_batch_at(void* h, int64_t batch, int64_t* x, int64_t* y) { ((Loader*)h)->fill(batch, x, y); }

int64_t pllm_loader_shard_tokens(void* h) { return ((Loader*)h)->n; }

void pllm_loader_destroy(void* h) {
  auto* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop.store(true);
  }
  L->cv.notify_all();
  if (L->worker.joinable()) L->worker.join();
  munmap((void*)L->base, L->map_bytes);
  close(L->fd);
  delete L;
}

}  // extern "C"
