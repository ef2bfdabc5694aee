/* abrt_bt.c — host-side diagnostic: on SIGABRT print the C backtrace (backtrace_symbols_fd) to
 * stderr, then die with the default action.  Loaded with ctypes.CDLL before the code under test. */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_abrt(int sig)
{
    void *buf[64];
    const char msg[] = "\n[abrt_bt] SIGABRT backtrace:\n";
    write(2, msg, sizeof msg - 1);
    int n = backtrace(buf, 64);
    backtrace_symbols_fd(buf, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) static void install(void)
{
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = on_abrt;
    sigaction(SIGABRT, &sa, 0);
}
