// Multi-threaded stress test of the host runtime core (csrc/runtime_core.h), built without GPU code
// under ThreadSanitizer and under AddressSanitizer+UBSan by tests/test_native_sanitizers.py.
//
// Workers race on one BatchDispenser exactly like the async parameter server's receive loop and
// callbacks do: claim a batch, "compute" it, and either complete it or drop it (a rejected, too
// stale gradient), while a reader thread polls every accessor.  Invariants checked at the end:
// each (epoch, batch) was completed exactly once, dropped batches were re-dispatched, and the
// dispenser reports done.  A StalenessGate is hammered concurrently; its counters must add up.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "runtime_core.h"

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

int main() {
  const int64_t N = 6000, BS = 32;  // 187 full batches + ragged last (smallLastBatch)
  const int EPOCHS = 3, THREADS = 8;
  dfa::BatchDispenser d(N, BS, EPOCHS, /*small_last=*/true, /*shuffle=*/true, 7);
  const int64_t NB = d.num_batches();
  CHECK(NB == (N + BS - 1) / BS);
  std::vector<std::atomic<int>> completed(EPOCHS * NB);
  for (auto& c : completed) c.store(0);
  std::atomic<int64_t> drops{0}, claims{0};
  std::atomic<bool> stop{false};

  std::thread reader([&] {
    int64_t sink = 0;
    while (!stop.load()) {
      sink += d.epoch() + d.remaining() + d.dispatched() + d.redispatch_rounds() + (d.done() ? 1 : 0);
      auto st = d.state();
      sink += (int64_t)st.incomplete.size();
      sink += (int64_t)d.example_indices(0).size();
    }
    CHECK(sink >= 0);
  });

  std::vector<std::thread> workers;
  for (int t = 0; t < THREADS; ++t) {
    workers.emplace_back([&, t] {
      uint64_t x = 0x9e3779b97f4a7c15ull * (t + 1);
      for (;;) {
        auto [done, b, ep, start, size] = d.next();
        if (done) break;
        claims.fetch_add(1);
        CHECK(b >= 0 && b < NB && ep >= 0 && ep < EPOCHS);
        CHECK(start == b * BS && size >= 1 && size <= BS && start + size <= N);
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        if (x % 5 == 0) {  // gradient rejected: batch stays incomplete
          drops.fetch_add(1);
          continue;
        }
        if (d.complete(b, ep)) completed[ep * NB + b].fetch_add(1);
      }
    });
  }
  for (auto& w : workers) w.join();
  stop.store(true);
  reader.join();

  for (int e = 0; e < EPOCHS; ++e)
    for (int64_t b = 0; b < NB; ++b) CHECK(completed[e * NB + b].load() == 1);
  CHECK(d.done());
  CHECK(drops.load() > 0 && d.redispatch_rounds() > 0);
  CHECK(claims.load() >= EPOCHS * NB + drops.load());

  dfa::BatchDispenser empty(10, 32, 2, false, false, 0);  // no batch at all: done, never hangs
  CHECK(empty.num_batches() == 0 && empty.done() && std::get<0>(empty.next()));

  dfa::StalenessGate gate(3);
  std::vector<std::thread> gs;
  for (int t = 0; t < THREADS; ++t)
    gs.emplace_back([&, t] {
      for (int i = 0; i < 20000; ++i) gate.admit(i - (i + t) % 7, i);
    });
  std::thread gr([&] {
    for (int i = 0; i < 2000; ++i) CHECK(gate.accepted() + gate.rejected() >= 0 && gate.histogram().size() <= 4);
  });
  for (auto& g : gs) g.join();
  gr.join();
  CHECK(gate.accepted() + gate.rejected() == (int64_t)THREADS * 20000);
  int64_t hsum = 0;
  for (int64_t h : gate.histogram()) hsum += h;
  CHECK(hsum == gate.accepted());
  std::printf("runtime_stress ok: %lld claims, %lld drops, %lld redispatch rounds\n", (long long)claims.load(),
              (long long)drops.load(), (long long)d.redispatch_rounds());
  return 0;
}
