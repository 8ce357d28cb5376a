// Standalone reproducer for the round-5 hipGraphLaunch segfault (profiles/r5_graph_crash.txt):
// HIP graphs with parallel branches (the engine's two-stream backward forks a side stream into
// every captured step) launched on the LEGACY DEFAULT STREAM after other graph executables of
// the process were created, run and destroyed.  No torch, no pddl code: plain HIP runtime calls
// in the order torch.cuda.CUDAGraph makes them (stream capture in thread-local mode on a created
// stream, fork / join through events, instantiate, destroy the hipGraph_t, hipGraphLaunch).
//
//   hipcc --offload-arch=gfx950 -O2 csrc/tests/graph_replay_repro.cpp -o /tmp/graph_repro
//   /tmp/graph_repro [rounds=200]
//
// Every replay's kernels add to device counters; the program checks the counts after each
// scenario and prints one line per scenario.  A fault inside hipGraphLaunch kills the process
// (SIGSEGV, exit 139) at a printed scenario, which then names the runtime as the owner: the
// program has no other state.  Scenarios (each launches on stream 0 = legacy default and on a
// created stream, so both paths run in the same process):
//   A  one 2-branch exec, replayed `rounds` times
//   B  8 execs of 2..5 branches; execs 0..3 destroyed; 4..7 replayed
//   C  churn: per round create an exec of (round % 4 + 2) branches, replay it on a created
//      stream, destroy the previous one, replay the new one on stream 0
//   D  as C with the capture's side streams destroyed and re-created every round (torch creates
//      side streams from its pool; an exec keeps a stream pointer only if the runtime copies it)
//   E  the Mirrored replica driver's churn (2-3 replicas x 6 chain-shaped execs, event forks to
//      comm streams, everything destroyed per round), then a fresh two-stream exec
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                             \
    }                                                                                           \
  } while (0)

__global__ void bump(unsigned long long* c, int slot) {
  if (threadIdx.x == 0) atomicAdd(c + slot, 1ull);
}

// Capture a graph whose work forks into `branches` parallel streams (one kernel each, plus one
// on the origin before the fork and one after the join), the engine's fork / join pattern.
static hipGraphExec_t make_exec(hipStream_t origin, std::vector<hipStream_t>& side, int branches,
                                unsigned long long* ctr, int slot0) {
  hipGraph_t g = nullptr;
  std::vector<hipEvent_t> ev(2 * branches + 1);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipStreamBeginCapture(origin, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, origin, ctr, slot0);
  CK(hipEventRecord(ev[0], origin));
  for (int b = 0; b < branches; ++b) {
    CK(hipStreamWaitEvent(side[b], ev[0], 0));
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, side[b], ctr, slot0 + 1 + b);
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, side[b], ctr, slot0 + 1 + b);
    CK(hipEventRecord(ev[1 + b], side[b]));
    CK(hipStreamWaitEvent(origin, ev[1 + b], 0));
  }
  hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, origin, ctr, slot0);
  CK(hipStreamEndCapture(origin, &g));
  hipGraphExec_t ex = nullptr;
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  CK(hipGraphDestroy(g));   // (torch keeps only the executable unless keep_graph)
  for (auto& e : ev) CK(hipEventDestroy(e));
  return ex;
}

// The engine's two-stream backward shape: ONE side stream forked `pairs` times (per layer: the
// origin's data-gradient kernel, an event, the side stream's weight-gradient kernel after it),
// the origin waiting on the side stream every 3 pairs (gradient-ring back-pressure) and joining
// it at the end; two = false: every kernel on the origin (the single-stream schedule).
// Kernels per replay: 2 * pairs + 2.
static hipGraphExec_t make_chain_exec(hipStream_t origin, hipStream_t side, int pairs, bool two,
                                      unsigned long long* ctr, int slot) {
  hipGraph_t g = nullptr;
  std::vector<hipEvent_t> ev(2 * pairs + 2);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipStreamBeginCapture(origin, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, origin, ctr, slot);
  for (int p = 0; p < pairs; ++p) {
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, origin, ctr, slot);
    if (!two) {
      hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, origin, ctr, slot + 1);
      continue;
    }
    CK(hipEventRecord(ev[2 * p], origin));
    CK(hipStreamWaitEvent(side, ev[2 * p], 0));
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, side, ctr, slot + 1);
    CK(hipEventRecord(ev[2 * p + 1], side));
    if (p % 3 == 2) CK(hipStreamWaitEvent(origin, ev[2 * p + 1], 0));
  }
  if (two) {
    CK(hipEventRecord(ev[2 * pairs], side));
    CK(hipStreamWaitEvent(origin, ev[2 * pairs], 0));
  }
  hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, origin, ctr, slot);
  CK(hipStreamEndCapture(origin, &g));
  hipGraphExec_t ex = nullptr;
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  CK(hipGraphDestroy(g));
  for (auto& e : ev) CK(hipEventDestroy(e));
  return ex;
}

static unsigned long long expect_total(int branches, int replays) { return (unsigned long long)replays * (2 + 2 * branches); }

static bool check(const char* tag, unsigned long long* ctr, unsigned long long want) {
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(64);
  CK(hipMemcpy(h.data(), ctr, 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  unsigned long long got = 0;
  for (auto v : h) got += v;
  std::printf("%s: kernel executions %llu, expected %llu -> %s\n", tag, got, want, got == want ? "ok" : "MISMATCH");
  std::fflush(stdout);
  CK(hipMemset(ctr, 0, 64 * sizeof(unsigned long long)));
  CK(hipDeviceSynchronize());
  return got == want;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 200;
  unsigned long long* ctr = nullptr;
  CK(hipMalloc(&ctr, 64 * sizeof(unsigned long long)));
  CK(hipMemset(ctr, 0, 64 * sizeof(unsigned long long)));
  hipStream_t cap, launch;
  CK(hipStreamCreate(&cap));
  CK(hipStreamCreate(&launch));
  std::vector<hipStream_t> side(8);
  for (auto& s : side) CK(hipStreamCreate(&s));
  bool ok = true;

  {  // A
    std::printf("A: one 2-branch exec, %d replays on stream 0\n", rounds);
    std::fflush(stdout);
    hipGraphExec_t ex = make_exec(cap, side, 2, ctr, 0);
    for (int r = 0; r < rounds; ++r) CK(hipGraphLaunch(ex, 0));
    ok &= check("A", ctr, expect_total(2, rounds));
    CK(hipGraphExecDestroy(ex));
  }
  {  // B
    std::printf("B: 8 execs (2..5 branches), 0..3 destroyed, 4..7 replayed %d times on stream 0\n", rounds);
    std::fflush(stdout);
    std::vector<hipGraphExec_t> ex(8);
    for (int i = 0; i < 8; ++i) ex[i] = make_exec(cap, side, 2 + i % 4, ctr, 8 * (i % 8));
    for (int i = 0; i < 8; ++i) CK(hipGraphLaunch(ex[i], launch));   // run every one once
    CK(hipStreamSynchronize(launch));
    unsigned long long want = 0;
    for (int i = 0; i < 8; ++i) want += expect_total(2 + i % 4, 1);
    for (int i = 0; i < 4; ++i) CK(hipGraphExecDestroy(ex[i]));
    for (int r = 0; r < rounds; ++r)
      for (int i = 4; i < 8; ++i) CK(hipGraphLaunch(ex[i], 0));
    for (int i = 4; i < 8; ++i) want += expect_total(2 + i % 4, rounds);
    ok &= check("B", ctr, want);
    for (int i = 4; i < 8; ++i) CK(hipGraphExecDestroy(ex[i]));
  }
  {  // C
    std::printf("C: exec churn, %d rounds (create, run on a created stream, destroy the previous, run on stream 0)\n",
                rounds);
    std::fflush(stdout);
    hipGraphExec_t prev = nullptr;
    unsigned long long want = 0;
    for (int r = 0; r < rounds; ++r) {
      const int nb = 2 + r % 4;
      hipGraphExec_t ex = make_exec(cap, side, nb, ctr, 8 * (r % 8));
      CK(hipGraphLaunch(ex, launch));
      if (prev) CK(hipGraphExecDestroy(prev));
      CK(hipGraphLaunch(ex, 0));
      want += expect_total(nb, 2);
      prev = ex;
    }
    CK(hipGraphExecDestroy(prev));
    ok &= check("C", ctr, want);
  }
  {  // D
    std::printf("D: as C, side streams destroyed and re-created every round, %d rounds\n", rounds);
    std::fflush(stdout);
    hipGraphExec_t prev = nullptr;
    unsigned long long want = 0;
    for (int r = 0; r < rounds; ++r) {
      const int nb = 2 + r % 4;
      hipGraphExec_t ex = make_exec(cap, side, nb, ctr, 8 * (r % 8));
      CK(hipGraphLaunch(ex, launch));
      CK(hipStreamSynchronize(launch));
      for (auto& s : side) {
        CK(hipStreamDestroy(s));
        CK(hipStreamCreate(&s));
      }
      if (prev) CK(hipGraphExecDestroy(prev));
      CK(hipGraphLaunch(ex, 0));
      want += expect_total(nb, 2);
      prev = ex;
    }
    CK(hipGraphExecDestroy(prev));
    ok &= check("D", ctr, want);
  }
  {  // E
    // The Mirrored replica driver's pattern (tests/test_gpu_runtime.py
    // test_graphed_replicas_match_eager_replicas, then a whole-step capture: the in-process
    // sequence that faults, profiles/r6_graph_repro.txt): per round R = 2 or 3 replicas, each
    // 5 segment execs + 1 "optimizer" exec (chain shape, one-stream in 2 of 3 rounds), replayed
    // 4 steps on per-replica created launch streams with every segment forked by an event to a
    // per-replica comm stream and the optimizer after the comm stream; then all destroyed.
    // Finally a fresh two-stream chain exec is captured and replayed on a created stream.
    std::printf("E: replica-driver churn, %d rounds, then a fresh two-stream exec\n", rounds / 10);
    std::fflush(stdout);
    unsigned long long want = 0;
    for (int r = 0; r < rounds / 10; ++r) {
      const int R = 2 + r % 2;
      const bool two = r % 3 == 2;
      std::vector<hipStream_t> ls(R), cs(R), rs(R);
      std::vector<std::vector<hipGraphExec_t>> ex(R);
      std::vector<std::vector<hipEvent_t>> ev(R, std::vector<hipEvent_t>(6));
      for (int i = 0; i < R; ++i) {
        CK(hipStreamCreate(&ls[i]));
        CK(hipStreamCreate(&cs[i]));
        CK(hipStreamCreate(&rs[i]));
        for (auto& e : ev[i]) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (int k = 0; k < 6; ++k) ex[i].push_back(make_chain_exec(cap, rs[i], k < 5 ? 12 : 1, two && k < 5, ctr, 2 * k));
      }
      for (int step = 0; step < 4; ++step) {
        for (int k = 0; k < 5; ++k)
          for (int i = 0; i < R; ++i) {
            CK(hipGraphLaunch(ex[i][k], ls[i]));
            CK(hipEventRecord(ev[i][k], ls[i]));
            CK(hipStreamWaitEvent(cs[i], ev[i][k], 0));
          }
        for (int i = 0; i < R; ++i) {
          CK(hipEventRecord(ev[i][5], cs[i]));
          CK(hipStreamWaitEvent(ls[i], ev[i][5], 0));
          CK(hipGraphLaunch(ex[i][5], ls[i]));
        }
      }
      want += (unsigned long long)R * 4 * (5 * (2 * 12 + 2) + (2 * 1 + 2));
      CK(hipDeviceSynchronize());
      for (int i = 0; i < R; ++i) {
        for (auto e : ex[i]) CK(hipGraphExecDestroy(e));
        for (auto e : ev[i]) CK(hipEventDestroy(e));
        CK(hipStreamDestroy(ls[i]));
        CK(hipStreamDestroy(cs[i]));
        CK(hipStreamDestroy(rs[i]));
      }
    }
    hipStream_t s2, l2;
    CK(hipStreamCreate(&s2));
    CK(hipStreamCreate(&l2));
    hipGraphExec_t fresh = make_chain_exec(cap, s2, 40, true, ctr, 20);
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(fresh, l2));
    want += 3ull * (2 * 40 + 2);
    CK(hipGraphExecDestroy(fresh));
    ok &= check("E", ctr, want);
    CK(hipStreamDestroy(s2));
    CK(hipStreamDestroy(l2));
  }
  for (auto& s : side) CK(hipStreamDestroy(s));
  CK(hipStreamDestroy(cap));
  CK(hipStreamDestroy(launch));
  CK(hipFree(ctr));
  std::printf("graph_replay_repro: %s\n", ok ? "all scenarios completed, counts match" : "COUNT MISMATCH");
  return ok ? 0 : 1;
}
