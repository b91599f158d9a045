// Host-only self-test of the C++ runtime pieces that do not need a GPU, built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host side only
// (tests/test_host_sanitizers.py: hipcc -Xarch_host -fsanitize=address ...; GPU sanitizers are
// not available on this pool).  SURVEY §5.2 (race detection / sanitizers).
//
//  * BucketSchedule (reducer state machine): in-order release, completeness, double-mark and
//    out-of-range detection, randomized mark orders (fuzz);
//  * FastDiv (the multiply-high division every kernel uses for index math): the host mirror of
//    FastDiv::div against exact division over all divisors the kernels use;
//  * ConvShape::make output-size arithmetic.
#include <cstdint>
#include <cstdio>
#include <random>
#include <stdexcept>
#include <vector>

#include "bucket_schedule.h"
#include "common.h"
#include "ops.h"

using mx::BucketSchedule;

static int failures = 0;
#define EXPECT(cond, msg)                                      \
  do {                                                         \
    if (!(cond)) {                                             \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
      ++failures;                                              \
    }                                                          \
  } while (0)

template <class F>
static bool throws(F f) {
  try {
    f();
  } catch (const std::runtime_error&) {
    return true;
  }
  return false;
}

static void test_schedule_basic() {
  // 5 params -> 3 buckets; bucket 0 = last params (first produced by backward)
  BucketSchedule s({{100, 20}, {40, 60}, {0, 40}}, {2, 2, 1, 0, 0});
  EXPECT(s.size() == 3, "size");
  EXPECT(s.pop_ready() == -1, "nothing ready before marks");
  EXPECT(!s.mark(4), "bucket 0 half");
  EXPECT(s.mark(3), "bucket 0 complete");
  EXPECT(s.pop_ready() == 0 && s.pop_ready() == -1, "bucket 0 released alone");
  EXPECT(!s.mark(0), "bucket 2 half");
  EXPECT(s.pop_ready() == -1, "bucket 2 not ready, bucket 1 blocks");
  EXPECT(s.mark(1), "bucket 2 complete");
  EXPECT(s.pop_ready() == -1, "in-order: bucket 1 still pending");
  EXPECT(s.mark(2), "bucket 1 complete");
  EXPECT(s.pop_ready() == 1 && s.pop_ready() == 2 && s.pop_ready() == -1, "1 then 2");
  EXPECT(throws([&] { s.mark(2); }), "double mark must throw");
  EXPECT(throws([&] { s.mark(7); }), "bad index must throw");
  EXPECT(throws([&] { s.mark(-1); }), "negative index must throw");
  s.prepare();
  EXPECT(s.launched() == 0 && s.pop_ready() == -1, "prepare resets");
  s.mark(3);
  s.release_all();  // unused params in buckets 0(partial) 1 2
  int n = 0;
  while (s.pop_ready() >= 0) ++n;
  EXPECT(n == 3, "release_all releases every bucket");
  EXPECT(throws([] { BucketSchedule bad({{0, 1}}, {0, 1}); }), "unknown bucket must throw");
}

static void test_schedule_fuzz() {
  std::mt19937 rng(1234);
  for (int it = 0; it < 2000; ++it) {
    const int nb = 1 + rng() % 8, np = nb + rng() % 40;
    std::vector<int> pb(np);
    for (int p = 0; p < np; ++p) pb[p] = p < nb ? p : (int)(rng() % nb);
    std::vector<std::pair<size_t, size_t>> spans;
    for (int b = 0; b < nb; ++b) spans.emplace_back(b * 64, 64);
    BucketSchedule s(spans, pb);
    std::vector<int> order(np);
    for (int p = 0; p < np; ++p) order[p] = p;
    std::shuffle(order.begin(), order.end(), rng);
    std::vector<int> left(nb, 0);
    for (int p : pb) left[p]++;
    int expect_next = 0;
    for (int p : order) {
      s.mark(p);
      left[pb[p]]--;
      for (int b = s.pop_ready(); b >= 0; b = s.pop_ready()) {
        EXPECT(b == expect_next, "fuzz: release order");
        EXPECT(left[b] == 0, "fuzz: released an incomplete bucket");
        ++expect_next;
      }
    }
    EXPECT(expect_next == nb, "fuzz: every bucket released once all params are marked");
  }
}

static uint32_t host_div(const mx::FastDiv& f, uint32_t n) {  // mirror of FastDiv::div
  const uint32_t hi = (uint32_t)(((uint64_t)n * f.m) >> 32);
  return (hi + n) >> f.s;
}

static void test_fastdiv() {
  std::mt19937 rng(7);
  const uint32_t special[] = {0u, 1u, 2u, 3u, 1023u, 1024u, 65535u, 65536u, 0x7ffffffeu, 0x7fffffffu};
  for (uint32_t d = 1; d <= 5000; ++d) {
    const mx::FastDiv f(d);
    for (uint32_t n : special) EXPECT(host_div(f, n) == n / d, "fastdiv special value");
    for (int i = 0; i < 64; ++i) {
      const uint32_t n = rng() & 0x7fffffffu;
      if (host_div(f, n) != n / d) {
        std::fprintf(stderr, "fastdiv d=%u n=%u got %u\n", d, n, host_div(f, n));
        ++failures;
        return;
      }
    }
  }
  for (uint32_t d : {50176u, 100352u, 3136u * 32u, 1u << 20, 12345678u}) {  // pixel counts
    const mx::FastDiv f(d);
    for (int i = 0; i < 4096; ++i) {
      const uint32_t n = rng() & 0x7fffffffu;
      EXPECT(host_div(f, n) == n / d, "fastdiv large divisor");
    }
  }
}

static void test_convshape() {
  const auto a = mx::ConvShape::make(32, 3, 224, 224, 64, 7, 7, 2, 2, 3, 3);
  EXPECT(a.P == 112 && a.Q == 112, "resnet stem 224 -> 112");
  const auto b = mx::ConvShape::make(64, 101, 32, 32, 106, 3, 3, 2, 2, 1, 1);
  EXPECT(b.P == 16 && b.Q == 16, "pyramidnet stride-2 entry 32 -> 16");
  const auto c = mx::ConvShape::make(64, 1, 28, 28, 32, 3, 3, 1, 1, 0, 0);
  EXPECT(c.P == 26 && c.Q == 26, "mnist conv1 valid 28 -> 26");
}

int main() {
  test_schedule_basic();
  test_schedule_fuzz();
  test_fastdiv();
  test_convshape();
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("ALL OK\n");
  return 0;
}
