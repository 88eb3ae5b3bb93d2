// Host-side runtime core of distriflow_amd (C++17, no GPU code, no Python): header-only so the
// same classes are compiled into _C.so (csrc/native_runtime.cpp adds the pybind11 layer) and into
// the sanitizer stress test (tests/native/runtime_stress.cpp, built with -fsanitize=thread and
// -fsanitize=address,undefined by tests/test_native_sanitizers.py).
//
//  * BatchDispenser — the first-come-first-serve microbatch queue of DistributedDataset
//    (/root/reference/src/server/dataset.ts:21-67): per-epoch set of incomplete batch ids, a live
//    cursor that skips batches already completed, and re-dispatch of un-acknowledged batches once
//    the cursor runs off the end (at-least-once processing).  Adds what the
//    reference only declares: smallLastBatch (ragged last batch, dataset.ts:27 is unused there),
//    optional per-epoch shuffling, and a serialisable state for checkpoint/resume.
//  * StalenessGate — the parameter server's version bookkeeping for asynchronous SGD with bounded
//    staleness (README.md:27 "maximumStaleness", not implemented by the reference): accepts an
//    update computed on version v at server version V iff V - v <= max_staleness, tracks
//    accept/reject counters and the staleness histogram.
// Every public member takes the object's mutex (the server's receive loop and user callbacks may
// run on different threads); each call is O(1) amortised.
#pragma once

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <tuple>
#include <vector>

namespace dfa {

struct DispenserState {
  int epoch = 0;
  int64_t cursor = 0;
  std::vector<int64_t> incomplete;
  std::vector<int64_t> perm;
  int64_t dispatched = 0;
};

class BatchDispenser {
 public:
  BatchDispenser(int64_t num_examples, int64_t batch_size, int epochs, bool small_last_batch, bool shuffle,
                 uint64_t seed)
      : n_(num_examples), bs_(batch_size), epochs_(epochs), small_last_(small_last_batch), shuffle_(shuffle),
        rng_(seed) {
    if (batch_size <= 0) throw std::invalid_argument("batch_size must be > 0");
    if (num_examples < 0) throw std::invalid_argument("num_examples must be >= 0");
    nb_ = small_last_ ? (n_ + bs_ - 1) / bs_ : n_ / bs_;
    start_epoch();
  }

  // -> (done, batch_id, epoch, start, size)
  std::tuple<bool, int64_t, int, int64_t, int64_t> next() {
    std::lock_guard<std::mutex> g(mu_);
    if (nb_ == 0 || epoch_ >= epochs_) return {true, -1, epoch_, 0, 0};
    if (remaining_ == 0) {
      ++epoch_;
      if (epoch_ >= epochs_) return {true, -1, epoch_, 0, 0};
      start_epoch();
    }
    int64_t id = advance();
    if (id < 0) {  // cursor exhausted but batches still incomplete: re-dispatch from the front
      cursor_ = 0;
      ++redispatch_rounds_;
      ++redispatched_epoch_;
      id = advance();
    }
    ++dispatched_;
    const int64_t start = id * bs_;
    const int64_t size = std::min(bs_, n_ - start);
    return {false, id, epoch_, start, size};
  }

  // Mark a batch of the CURRENT epoch complete; returns false for unknown / already-complete ids
  // (a late duplicate of a re-dispatched batch, or an id from a previous epoch).
  bool complete(int64_t batch, int epoch) {
    std::lock_guard<std::mutex> g(mu_);
    if (epoch != epoch_ || batch < 0 || batch >= nb_) return false;
    if (!incomplete_[batch]) return false;
    incomplete_[batch] = 0;
    --remaining_;
    return true;
  }

  int64_t num_batches() const { return nb_; }  // immutable after construction
  int epoch() const {
    std::lock_guard<std::mutex> g(mu_);
    return epoch_;
  }
  int64_t remaining() const {
    std::lock_guard<std::mutex> g(mu_);
    return remaining_;
  }
  int64_t dispatched() const {
    std::lock_guard<std::mutex> g(mu_);
    return dispatched_;
  }
  int64_t redispatch_rounds() const {
    std::lock_guard<std::mutex> g(mu_);
    return redispatch_rounds_;
  }
  // A dataset that yields no batch (fewer examples than one batch, smallLastBatch off) is done
  // from the start, so a server waiting on it terminates instead of running into its timeout.
  bool done() const {
    std::lock_guard<std::mutex> g(mu_);
    return nb_ == 0 || epoch_ >= epochs_ || (remaining_ == 0 && epoch_ + 1 >= epochs_);
  }

  // Permutation-aware example indices of a batch in the current epoch order.
  std::vector<int64_t> example_indices(int64_t batch) const {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int64_t> out;
    if (batch < 0 || batch >= nb_) return out;
    const int64_t start = batch * bs_, end = std::min(n_, start + bs_);
    out.reserve(end - start);
    for (int64_t i = start; i < end; ++i) out.push_back(shuffle_ ? perm_[i] : i);
    return out;
  }

  DispenserState state() const {
    std::lock_guard<std::mutex> g(mu_);
    DispenserState s;
    s.epoch = epoch_;
    s.cursor = cursor_;
    for (int64_t i = 0; i < nb_; ++i)
      if (incomplete_[i]) s.incomplete.push_back(i);
    s.perm = perm_;
    s.dispatched = dispatched_;
    return s;
  }

  void load_state(const DispenserState& s) {
    std::lock_guard<std::mutex> g(mu_);
    epoch_ = s.epoch;
    cursor_ = s.cursor;
    perm_ = s.perm;
    dispatched_ = s.dispatched;
    std::fill(incomplete_.begin(), incomplete_.end(), 0);
    remaining_ = 0;
    for (int64_t b : s.incomplete) {
      if (b >= 0 && b < nb_ && !incomplete_[b]) {
        incomplete_[b] = 1;
        ++remaining_;
      }
    }
  }

 private:
  void start_epoch() {
    incomplete_.assign(nb_, 1);
    remaining_ = nb_;
    cursor_ = 0;
    redispatched_epoch_ = 0;
    if (shuffle_) {
      perm_.resize(n_);
      std::iota(perm_.begin(), perm_.end(), 0);
      std::shuffle(perm_.begin(), perm_.end(), rng_);
    }
  }
  int64_t advance() {
    while (cursor_ < nb_ && !incomplete_[cursor_]) ++cursor_;
    if (cursor_ >= nb_) return -1;
    return cursor_++;
  }

  int64_t n_, bs_;
  int epochs_;
  bool small_last_, shuffle_;
  std::mt19937_64 rng_;
  int64_t nb_ = 0;
  int epoch_ = 0;
  int64_t cursor_ = 0, remaining_ = 0, dispatched_ = 0, redispatch_rounds_ = 0, redispatched_epoch_ = 0;
  std::vector<uint8_t> incomplete_;
  std::vector<int64_t> perm_;
  mutable std::mutex mu_;
};

class StalenessGate {
 public:
  explicit StalenessGate(int64_t max_staleness) : max_(max_staleness) {}

  // Decide for an update computed on `grad_version` arriving at server version `server_version`.
  bool admit(int64_t grad_version, int64_t server_version) {
    std::lock_guard<std::mutex> g(mu_);
    const int64_t s = server_version - grad_version;
    if (s < 0 || (max_ >= 0 && s > max_)) {
      ++rejected_;
      return false;
    }
    ++accepted_;
    if ((size_t)s >= hist_.size()) hist_.resize(s + 1, 0);
    ++hist_[s];
    return true;
  }
  int64_t accepted() const {
    std::lock_guard<std::mutex> g(mu_);
    return accepted_;
  }
  int64_t rejected() const {
    std::lock_guard<std::mutex> g(mu_);
    return rejected_;
  }
  int64_t max_staleness() const { return max_; }  // immutable
  std::vector<int64_t> histogram() const {
    std::lock_guard<std::mutex> g(mu_);
    return hist_;
  }

 private:
  const int64_t max_;
  int64_t accepted_ = 0, rejected_ = 0;
  std::vector<int64_t> hist_;
  mutable std::mutex mu_;
};

}  // namespace dfa
