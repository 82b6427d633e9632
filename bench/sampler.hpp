// sampler.hpp — a profiler-free sampling of where the host spends its time (measurement only).
//
// With PN_SAMPLE=<prefix> in the environment, pn_sampler::start(tag) arms a timer (every PN_SAMPLE_US
// microseconds of wall clock, default 50, delivered to the calling thread) and the SIGPROF handler records the
// interrupted instruction pointer; stop() writes one line per sample to <prefix>.<tag>: the module it fell in ("exe"
// for the executable) and the address relative to that module's load base, which scripts/sample_report.py
// symbolizes (inlined frames included) and folds.  No perf counters are needed: the container and the GPU boxes
// expose none to an ordinary user.
#pragma once

#include <link.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace pn_sampler {

struct State {
  uint64_t* buf = nullptr;
  volatile uint64_t n = 0;
  uint64_t cap = 0;
  uintptr_t base = 0;
  const char* path = nullptr;
  char path_buf[512] = {};
  timer_t timer{};
};
inline State g;

inline void on_prof(int, siginfo_t*, void* uc) {
  const auto* u = static_cast<const ucontext_t*>(uc);
  const uint64_t i = g.n;
  if (i < g.cap) {
    g.buf[i] = (uint64_t)u->uc_mcontext.gregs[REG_RIP];
    g.n = i + 1;
  }
}

inline int find_base(dl_phdr_info* info, size_t, void* out) {
  if (info->dlpi_name == nullptr || info->dlpi_name[0] == 0) { // the executable itself
    *static_cast<uintptr_t*>(out) = info->dlpi_addr;
    return 1;
  }
  return 0;
}

// arm the sampler when PN_SAMPLE names a file prefix (samples go to <prefix>.<tag>; returns false otherwise)
inline bool start(const char* tag) {
  const char* pre = std::getenv("PN_SAMPLE");
  if (!pre || !pre[0]) return false;
  std::snprintf(g.path_buf, sizeof g.path_buf, "%s.%s", pre, tag);
  g.path = g.path_buf;
  g.n = 0;
  const char* us = std::getenv("PN_SAMPLE_US");
  const long period = us ? std::atol(us) : 50;
  g.cap = 1u << 22;
  if (!g.buf) g.buf = static_cast<uint64_t*>(std::malloc(g.cap * sizeof(uint64_t)));
  dl_iterate_phdr(find_base, &g.base);
  struct sigaction sa = {};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGPROF, &sa, nullptr);
  // a high-resolution timer on the monotonic clock, delivered to this thread (ITIMER_PROF ticks at the kernel's HZ)
  sigevent ev = {};
  ev.sigev_notify = SIGEV_THREAD_ID;
  ev.sigev_signo = SIGPROF;
  ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
  if (timer_create(CLOCK_MONOTONIC, &ev, &g.timer) != 0) return false;
  itimerspec t = {};
  t.it_interval.tv_nsec = period * 1000;
  t.it_value.tv_nsec = period * 1000;
  timer_settime(g.timer, 0, &t, nullptr);
  return true;
}

struct Module {
  uintptr_t lo, hi, base;
  const char* name;
};
inline int collect_modules(dl_phdr_info* info, size_t, void* out) {
  auto* v = static_cast<std::vector<Module>*>(out);
  for (int i = 0; i < info->dlpi_phnum; i++) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[i];
    if (ph.p_type != PT_LOAD) continue;
    const uintptr_t lo = info->dlpi_addr + ph.p_vaddr;
    v->push_back({lo, lo + ph.p_memsz, info->dlpi_addr, info->dlpi_name});
  }
  return 0;
}

// one line per sample: the module (the executable: "exe") and the address relative to its load base
inline void stop() {
  if (!g.path) return;
  timer_delete(g.timer);
  signal(SIGPROF, SIG_IGN);
  std::vector<Module> mods;
  dl_iterate_phdr(collect_modules, &mods);
  if (FILE* f = std::fopen(g.path, "w")) {
    for (uint64_t i = 0; i < g.n; i++) {
      const uintptr_t a = g.buf[i];
      const Module* m = nullptr;
      for (const Module& x : mods)
        if (a >= x.lo && a < x.hi) m = &x;
      if (m) std::fprintf(f, "%s\t%lx\n", (m->name && m->name[0]) ? m->name : "exe", (unsigned long)(a - m->base));
      else std::fprintf(f, "?\t%lx\n", (unsigned long)a);
    }
    std::fclose(f);
  }
  g.path = nullptr;
}

} // namespace pn_sampler
