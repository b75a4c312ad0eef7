// sampler.hh -- tools only: a program-counter sampler forced into a
// measurement program's build (-include), for programs that make no HIP
// calls (the null glue: a signal interrupts HIP's ioctls).  With SAMPLES=file
// in the environment it samples the main thread's PC every 20 us of wall
// time from start to exit and writes one line per sample: the offset from
// the executable's start, or the shared object's name
// (tools/chain_prof/resolve.py turns that into lines and functions).
#include <dlfcn.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

extern "C" char __executable_start;
namespace clk_sampler {
static uintptr_t pc[1 << 23];
static volatile size_t npc = 0;
static void on_prof(int, siginfo_t *, void *uc)
{
    if (npc < (1u << 23))
        pc[npc++] = (uintptr_t)((ucontext_t *)uc)->uc_mcontext.gregs[REG_RIP];
}
__attribute__((constructor)) static void arm()
{
    if (!getenv("SAMPLES"))
        return;
    struct sigaction sa = {};
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, nullptr);
    sigevent ev = {};
    ev.sigev_notify = SIGEV_THREAD_ID;
    ev.sigev_signo = SIGPROF;
    ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
    timer_t tm;
    if (timer_create(CLOCK_MONOTONIC, &ev, &tm) == 0) {
        itimerspec its = {{0, 20000}, {0, 20000}};
        timer_settime(tm, 0, &its, nullptr);
    }
}
__attribute__((destructor)) static void dump()
{
    const char *path = getenv("SAMPLES");
    if (!path)
        return;
    signal(SIGPROF, SIG_IGN);
    if (getenv("SAMPLES_DEBUG"))
        fprintf(stderr, "sampler: %zu samples\n", (size_t)npc);
    FILE *f = fopen(path, "w");
    if (!f)
        return;
    for (size_t k = 0; k < npc; k++) {
        Dl_info di;
        if (dladdr((void *)pc[k], &di) && di.dli_fbase == (void *)&__executable_start)
            fprintf(f, "0x%lx\n", (unsigned long)(pc[k] - (uintptr_t)&__executable_start));
        else
            fprintf(f, "@%s\n", dladdr((void *)pc[k], &di) && di.dli_fname ? di.dli_fname : "?");
    }
    fclose(f);
}
}   // namespace clk_sampler
