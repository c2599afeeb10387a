// Opt-in crash diagnostics for the host library. With MPG_ABORT_TRACE=1 in
// the environment, a SIGABRT / SIGSEGV / SIGBUS handler writes the native
// stack (glibc backtrace) to stderr, then re-raises with the default action.
// Off by default: nothing is installed unless the variable is set. Used by
// tools/exit_probe.py to locate process-exit faults.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>

namespace {

void on_fatal(int sig) {
    static const char head[] = "\n[mpg] fatal signal, native stack:\n";
    (void)!write(2, head, sizeof head - 1);
    void* frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) void install_abort_trace() {
    const char* env = std::getenv("MPG_ABORT_TRACE");
    if (!env || *env != '1') return;
    void* warm[2];
    (void)backtrace(warm, 2);  // loads libgcc_s now, not inside the handler
    struct sigaction sa;
    std::memset(&sa, 0, sizeof sa);
    sa.sa_handler = on_fatal;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_RESETHAND;
    sigaction(SIGABRT, &sa, nullptr);
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
}

}  // namespace
