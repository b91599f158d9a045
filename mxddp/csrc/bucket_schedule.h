// Host-side bucket state machine of the gradient reducer (reducer.cpp), kept free of HIP so it
// can be unit-tested in a plain host build with AddressSanitizer / UBSan
// (csrc/host_tests/selftest.cpp, tests/test_host_sanitizers.py).
//
// Buckets count down as their parameters are marked ready; they are released strictly in
// bucket order (every rank must issue its collectives in the same order).  Marking a parameter
// twice in one backward pass, or releasing a bucket whose count is not zero, is a race in the
// caller and throws.
#pragma once
#include <algorithm>
#include <cstddef>
#include <stdexcept>
#include <string>
#include <vector>

namespace mx {

class BucketSchedule {
 public:
  struct Bucket {
    size_t offset, numel;
    int total, pending;
    bool ready;
  };

  BucketSchedule() = default;
  BucketSchedule(const std::vector<std::pair<size_t, size_t>>& buckets, const std::vector<int>& param_bucket)
      : param_bucket_(param_bucket) {
    for (const auto& b : buckets) buckets_.push_back(Bucket{b.first, b.second, 0, 0, false});
    for (int pb : param_bucket_) {
      check(pb >= 0 && pb < (int)buckets_.size(), "param assigned to unknown bucket");
      buckets_[pb].total++;
    }
    marked_.assign(param_bucket_.size(), 0);
    prepare();
  }

  void prepare() {
    for (auto& b : buckets_) {
      b.pending = b.total;
      b.ready = false;
    }
    std::fill(marked_.begin(), marked_.end(), 0);
    next_ = 0;
  }

  // returns true when the parameter's bucket became ready
  bool mark(int p) {
    check(p >= 0 && p < (int)param_bucket_.size(), "mark_ready: bad parameter index");
    check(!marked_[p], "parameter marked ready twice in one backward pass (reentrant backward or "
                       "shared parameter); reducer state would race");
    marked_[p] = 1;
    Bucket& b = buckets_[param_bucket_[p]];
    check(b.pending > 0, "bucket count underflow");
    if (--b.pending == 0) {
      b.ready = true;
      return true;
    }
    return false;
  }

  void mark_bucket(int bi) {
    check(bi >= 0 && bi < (int)buckets_.size(), "mark_bucket_ready: bad bucket");
    buckets_[bi].pending = 0;
    buckets_[bi].ready = true;
  }

  // next bucket that may be launched now (in order), or -1
  int pop_ready() {
    if (next_ >= (int)buckets_.size() || !buckets_[next_].ready) return -1;
    check(buckets_[next_].pending == 0, "bucket launched before all its gradients were ready");
    return next_++;
  }

  // end of backward: buckets with unused parameters are released as they are
  void release_all() {
    for (auto& b : buckets_)
      if (!b.ready) {
        b.pending = 0;
        b.ready = true;
      }
  }

  const Bucket& bucket(int i) const { return buckets_[i]; }
  int size() const { return (int)buckets_.size(); }
  int launched() const { return next_; }

 private:
  static void check(bool ok, const char* msg) {
    if (!ok) throw std::runtime_error(std::string("mxddp check failed: ") + msg);
  }
  std::vector<Bucket> buckets_;
  std::vector<int> param_bucket_;
  std::vector<char> marked_;
  int next_ = 0;
};

}  // namespace mx
