// Native crash reports for GPU runs: on SIGSEGV / SIGBUS / SIGABRT the faulting thread writes
// its native call stack (glibc backtrace, symbolised from the dynamic symbol tables: HIP
// runtime, RCCL, torch, this extension) to stderr or a file, then hands the signal to the handler that
// was installed before (Python's faulthandler prints the Python stacks and re-raises).
//
// rocgdb / core dumps are not available on the GPU pool, so this is how a crash inside a
// runtime call (e.g. hipGraphLaunch) names the frames it happened in.
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

#include <string>

#include <pybind11/pybind11.h>

namespace {

constexpr int kSigs[] = {SIGSEGV, SIGBUS, SIGABRT, SIGFPE, SIGILL};
constexpr int kNSig = sizeof(kSigs) / sizeof(kSigs[0]);
struct sigaction g_prev[kNSig];
bool g_installed = false;
int g_fd = 2;   // (a file: pytest's fd capture swallows what a dying process writes to fd 2)

void write_str(const char* s) {
  ssize_t r = write(g_fd, s, strlen(s));
  (void)r;
}

void on_fatal(int sig, siginfo_t* info, void* uctx) {
  int idx = 0;
  while (idx < kNSig && kSigs[idx] != sig) ++idx;
  write_str("\n[pddl crash trace] fatal signal ");
  write_str(strsignal(sig));
  char buf[64];
  // (async-signal-safe hex formatting of the faulting address)
  const unsigned long a = reinterpret_cast<unsigned long>(info ? info->si_addr : nullptr);
  int n = 0;
  buf[n++] = ' ';
  buf[n++] = '@';
  buf[n++] = '0';
  buf[n++] = 'x';
  for (int s = 60; s >= 0; s -= 4) buf[n++] = "0123456789abcdef"[(a >> s) & 15];
  buf[n++] = '\n';
  buf[n] = 0;
  write_str(buf);
  void* frames[96];
  const int nf = backtrace(frames, 96);
  backtrace_symbols_fd(frames, nf, g_fd);
  write_str("[pddl crash trace] end of native stack\n");
  // chain: restore the previous disposition and re-deliver
  if (idx < kNSig) {
    sigaction(sig, &g_prev[idx], nullptr);
    if (g_prev[idx].sa_flags & SA_SIGINFO) {
      if (g_prev[idx].sa_sigaction) {
        g_prev[idx].sa_sigaction(sig, info, uctx);
        return;
      }
    } else if (g_prev[idx].sa_handler != SIG_DFL && g_prev[idx].sa_handler != SIG_IGN) {
      g_prev[idx].sa_handler(sig);
      return;
    }
  }
  raise(sig);
}

bool install(const std::string& path) {
  if (!path.empty()) {
    const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (fd >= 0) g_fd = fd;
  }
  if (g_installed) return true;
  {
    void* warm[2];
    backtrace(warm, 2);   // (loads libgcc's unwinder now, not inside the signal handler)
  }
  static char alt_stack[1 << 16];
  stack_t ss{};
  ss.ss_sp = alt_stack;
  ss.ss_size = sizeof(alt_stack);
  sigaltstack(&ss, nullptr);
  for (int i = 0; i < kNSig; ++i) {
    struct sigaction sa {};
    sa.sa_sigaction = on_fatal;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(kSigs[i], &sa, &g_prev[i]);
  }
  g_installed = true;
  return true;
}

}  // namespace

void register_crash_trace(pybind11::module& m) {
  m.def("install_crash_trace", &install, pybind11::arg("path") = std::string(),
        "On a fatal signal write the native call stack to `path` (appended; default stderr), then chain "
        "to the previous handler (install after faulthandler.enable() so the Python stacks follow).");
}
