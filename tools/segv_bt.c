/* Diagnostic: on SIGSEGV / SIGBUS print the faulting address and the native
 * backtrace (raw addresses + the library each lives in, with its load base,
 * so frames in libamdhip64 can be symbolised offline), then hand the signal
 * to the handler that was installed before (Python's faulthandler).
 * Loaded by tests/conftest.py when TT_SEGV_BT=1.  Host code only. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_prev_segv, g_prev_bus;

static int g_fd = 2;

static void put(const char* s) { (void)!write(g_fd, s, strlen(s)); }

static void handler(int sig, siginfo_t* info, void* uctx) {
  (void)uctx;
  char line[512];
  snprintf(line, sizeof line, "\n[segv_bt] signal %d at address %p\n", sig, info ? info->si_addr : 0);
  put(line);
  void* frames[64];
  int n = backtrace(frames, 64);
  for (int i = 0; i < n; ++i) {
    Dl_info di;
    memset(&di, 0, sizeof di);
    if (dladdr(frames[i], &di) && di.dli_fname) {
      snprintf(line, sizeof line, "[segv_bt] #%02d %p %s+0x%lx (%s)\n", i, frames[i], di.dli_fname,
               (unsigned long)((char*)frames[i] - (char*)di.dli_fbase), di.dli_sname ? di.dli_sname : "?");
    } else {
      snprintf(line, sizeof line, "[segv_bt] #%02d %p ?\n", i, frames[i]);
    }
    put(line);
  }
  /* restore the previous handler; returning re-executes the faulting
   * instruction, which now reaches it */
  sigaction(SIGSEGV, &g_prev_segv, NULL);
  sigaction(SIGBUS, &g_prev_bus, NULL);
}

/* path: a file the backtrace is appended to (pytest captures fd 2) */
int tt_segv_bt_install(const char* path) {
  if (g_fd == 2 && path && *path) {
    int fd = open(path, O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) g_fd = fd;
  }
  struct sigaction cur;
  if (sigaction(SIGSEGV, NULL, &cur) == 0 && (cur.sa_flags & SA_SIGINFO) && cur.sa_sigaction == handler)
    return 0; /* already first in line */
  void* warm[2];
  backtrace(warm, 2); /* loads libgcc_s outside the handler */
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGSEGV, &sa, &g_prev_segv)) return -1;
  if (sigaction(SIGBUS, &sa, &g_prev_bus)) return -1;
  return 0;
}
