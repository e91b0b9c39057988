// Stand-alone self-test of the native token loader for sanitizer builds (SURVEY.md §5.2 race
// detection): compiled together with ../token_loader.cpp (this directory is not part of the _host.so build) under -fsanitize=thread (the producer
// thread / consumer hand-off) or -fsanitize=address,undefined (mmap bounds, the copy loops) by
// tests/test_host_sanitizers.py.  Exercises: every consumed batch equals the stateless
// regeneration of its index (ring hand-off intact), several prefetch depths and ranks, resume at
// a start batch, and destruction while the producer is blocked on a full ring.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <vector>

extern "C" {
void* pllm_loader_create(const char* path, int64_t rank, int64_t world, int B, int T, uint64_t seed,
                         int64_t start_batch, int prefetch);
int64_t pllm_loader_next(void* h, int64_t* x, int64_t* y);
void pllm_loader_batch_at(void* h, int64_t batch, int64_t* x, int64_t* y);
int64_t pllm_loader_shard_tokens(void* h);
void pllm_loader_destroy(void* h);
}

static int fail(const char* what) {
  fprintf(stderr, "loader_selftest FAILED: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/pllm_loader_selftest.bin";
  const int64_t ntok = 200003;
  {
    std::vector<uint16_t> tok(ntok);
    for (int64_t i = 0; i < ntok; ++i) tok[i] = (uint16_t)((i * 2654435761u) % 50257u);
    FILE* f = fopen(path, "wb");
    if (!f || fwrite(tok.data(), 2, ntok, f) != (size_t)ntok) return fail("write token file");
    fclose(f);
  }
  if (pllm_loader_create("/nonexistent/pllm.bin", 0, 1, 2, 8, 1, 0, 2) != nullptr) return fail("missing file accepted");
  const int B = 4, T = 64;
  std::vector<int64_t> x(B * T), y(B * T), rx(B * T), ry(B * T);
  for (int world : {1, 3}) {
    for (int64_t rank = 0; rank < world; ++rank) {
      for (int prefetch : {1, 2, 4}) {
        void* h = pllm_loader_create(path, rank, world, B, T, 1234 + prefetch, 5, prefetch);
        if (!h) return fail("create");
        const int64_t n = pllm_loader_shard_tokens(h);
        for (int64_t want = 5; want < 45; ++want) {
          if (pllm_loader_next(h, x.data(), y.data()) != want) return fail("batch order");
          pllm_loader_batch_at(h, want, rx.data(), ry.data());
          if (memcmp(x.data(), rx.data(), x.size() * 8) || memcmp(y.data(), ry.data(), y.size() * 8))
            return fail("consumed batch differs from its regeneration");
          for (int i = 0; i < B * T; ++i)
            if (i % T != T - 1 && x[i + 1] != y[i]) return fail("targets are not the inputs shifted by one");
        }
        if (n <= T) return fail("shard size");
        pllm_loader_destroy(h);
      }
    }
  }
  // destroy while the producer waits on a full ring, and right after creation
  for (int i = 0; i < 20; ++i) {
    void* h = pllm_loader_create(path, 0, 1, B, T, i, 0, 2);
    if (!h) return fail("create (destroy test)");
    if (i & 1) {
      pllm_loader_next(h, x.data(), y.data());
      usleep(2000);
    }
    pllm_loader_destroy(h);
  }
  unlink(path);
  printf("loader_selftest ok\n");
  return 0;
}
