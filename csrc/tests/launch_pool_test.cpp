// Native ThreadSanitizer / ASan driver of the group-launch thread pool (runtime/launch_pool.h):
// runs of growing and shrinking width (new workers join between runs and must wait for the next
// generation, never run a finished run's task), every task writing its own plain (non-atomic)
// slot that the caller reads right after run() returns, concurrent callers serialised by the
// pool, and idle gaps long enough for the workers to leave their spin and sleep.
//   clang++ -std=c++17 -O1 -g -fsanitize=thread -I csrc csrc/tests/launch_pool_test.cpp -lpthread
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "runtime/launch_pool.h"

int main() {
  pddl::LaunchPool pool;
  std::vector<long> slot(16, 0);
  long expect_sum = 0;
  const int widths[] = {2, 3, 8, 5, 16, 1, 12};
  for (int round = 0; round < 300; ++round) {
    const int n = widths[round % 7];
    std::vector<int> hits(n, 0);
    pool.run(n, [&](size_t i) {
      slot[i] += (long)(round + 1);   // plain writes, ordered by run()'s return
      hits[i] += 1;
    });
    for (int i = 0; i < n; ++i)
      if (hits[i] != 1) {
        std::fprintf(stderr, "round %d: task %d ran %d times\n", round, i, hits[i]);
        return 1;
      }
    expect_sum += (long)(round + 1) * n;
    if (round % 50 == 49) std::this_thread::sleep_for(std::chrono::milliseconds(2));   // workers sleep
  }
  // two callers at once: runs never interleave, every task still runs exactly once
  std::vector<long> a(8, 0), b(8, 0);
  std::thread other([&] {
    for (int r = 0; r < 200; ++r) pool.run(8, [&](size_t i) { a[i] += 1; });
  });
  for (int r = 0; r < 200; ++r) pool.run(8, [&](size_t i) { b[i] += 1; });
  other.join();
  long sum = 0;
  for (long v : slot) sum += v;
  for (int i = 0; i < 8; ++i)
    if (a[i] != 200 || b[i] != 200) {
      std::fprintf(stderr, "concurrent callers: slot %d ran %ld / %ld times\n", i, a[i], b[i]);
      return 1;
    }
  if (sum != expect_sum) {
    std::fprintf(stderr, "sum %ld != %ld\n", sum, expect_sum);
    return 1;
  }
  std::printf("launch_pool_test: ok\n");
  return 0;
}
