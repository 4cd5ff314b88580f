/* Debug aid (not product code): on SIGSEGV/SIGABRT print the native backtrace of the faulting
 * thread to stderr, then hand the signal to the previous handler.  Loaded with ctypes by
 * tools/segv_run.py before the program runs, so a crash in an exit handler names its library.
 * Build: gcc -O1 -g -fPIC -shared tools/segv_trace.c -o tools/libsegv_trace.so */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_old_segv, g_old_abrt;

static void on_fault(int sig, siginfo_t* si, void* ctx) {
  static const char hdr[] = "\n[segv_trace] fatal signal, native backtrace:\n";
  write(2, hdr, sizeof hdr - 1);
  void* frames[64];
  int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  struct sigaction* old = sig == SIGSEGV ? &g_old_segv : &g_old_abrt;
  sigaction(sig, old, NULL);
  if (old->sa_flags & SA_SIGINFO) {
    if (old->sa_sigaction) old->sa_sigaction(sig, si, ctx);
  } else if (old->sa_handler != SIG_DFL && old->sa_handler != SIG_IGN) {
    old->sa_handler(sig);
  }
  raise(sig);
}

__attribute__((constructor)) static void install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_old_segv);
  sigaction(SIGABRT, &sa, &g_old_abrt);
}
