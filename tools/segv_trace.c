/* Debug aid (host only): a SIGSEGV / SIGABRT handler that prints the native backtrace of the
 * faulting thread to stderr, for crashes after the Python interpreter has finalized (where
 * faulthandler is already off).  Loaded by tests/conftest.py when DBSCAN_SEGV_TRACE=1.
 *   gcc -O1 -g -shared -fPIC tools/segv_trace.c -o tools/segv_trace.so */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig) {
    void* frames[64];
    const char msg[] = "\n[segv_trace] fatal signal, native backtrace:\n";
    if (write(2, msg, sizeof(msg) - 1) < 0) return;
    int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

void segv_trace_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_fault;
    sigaction(SIGSEGV, &sa, 0);
    sigaction(SIGBUS, &sa, 0);
}

__attribute__((constructor)) static void install_at_load(void) { segv_trace_install(); }
