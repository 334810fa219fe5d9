/* sampler.c — leaf-PC sampling profiler for the host planner (a development
 * tool; nothing in the product loads it). Loaded with ctypes by
 * tools/plan_profile.py: sg_sampler_start(hz, stacks) arms ITIMER_PROF, whose
 * SIGPROF lands on whichever thread is burning CPU; the handler stores that
 * thread's instruction pointer and, with stacks, up to DEPTH return addresses
 * from glibc's backtrace() (not async-signal-safe in general, but once the
 * unwinder is loaded it is good enough for a development profiler).
 * sg_sampler_stop() disarms and returns the sample count;
 * sg_sampler_pcs() exposes the buffer for symbolisation (dladdr + addr2line).
 *
 *   gcc -O2 -shared -fPIC -o tools/_sampler.so tools/sampler.c
 */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdint.h>
#include <string.h>
#include <sys/time.h>
#include <ucontext.h>

#define CAP (1 << 20)
#define DEPTH 12
static uintptr_t pcs[CAP];
static uintptr_t stacks[CAP][DEPTH];  /* return addresses, innermost first (stack mode) */
static volatile long n_samples;
static int with_stacks;

static void on_prof(int sig, siginfo_t* si, void* uc_) {
  (void)sig;
  (void)si;
  ucontext_t* uc = (ucontext_t*)uc_;
  long k = __atomic_fetch_add(&n_samples, 1, __ATOMIC_RELAXED);
  if (k < CAP) {
    pcs[k] = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
    if (with_stacks) {
      void* fr[DEPTH + 2];
      int n = backtrace(fr, DEPTH + 2); /* frame 0: this handler, 1: the signal trampoline */
      for (int i = 0; i < DEPTH; ++i) stacks[k][i] = i + 2 < n ? (uintptr_t)fr[i + 2] : 0;
    }
  }
}

int sg_sampler_start(int hz, int stack_mode) {
  void* warm[4];
  backtrace(warm, 4); /* loads the unwinder before the first signal */
  with_stacks = stack_mode;
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, 0)) return -1;
  n_samples = 0;
  struct itimerval it;
  it.it_interval.tv_sec = 0;
  it.it_interval.tv_usec = 1000000 / (hz > 0 ? hz : 1000);
  it.it_value = it.it_interval;
  return setitimer(ITIMER_PROF, &it, 0);
}

long sg_sampler_stop(void) {
  struct itimerval it;
  memset(&it, 0, sizeof it);
  setitimer(ITIMER_PROF, &it, 0);
  return n_samples < CAP ? n_samples : CAP;
}

const uintptr_t* sg_sampler_pcs(void) { return pcs; }
const uintptr_t* sg_sampler_stacks(void) { return &stacks[0][0]; }
int sg_sampler_depth(void) { return DEPTH; }
