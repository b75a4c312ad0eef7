/* preload_sampler.c -- tools only, for this container (never on the GPU box,
 * whose harness owns LD_PRELOAD): a program-counter sampler for a program we
 * do not rebuild (Click's userlevel driver over the null glue).
 *   gcc -O2 -shared -fPIC preload_sampler.c -o /tmp/sampler.so -ldl -lrt
 *   SAMPLES=/tmp/s.txt LD_PRELOAD=/tmp/sampler.so click ...
 * One line per sample of the main thread (every 50 us of wall time): the
 * object file and the PC's offset in it; tools/core_profile/fold.py turns
 * them into functions. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#define CAP (1u << 23)
static uintptr_t pc[CAP];
static volatile size_t npc;

static void on_prof(int sig, siginfo_t *si, void *uc)
{
    (void)sig, (void)si;
    if (npc < CAP)
        pc[npc++] = (uintptr_t)((ucontext_t *)uc)->uc_mcontext.gregs[REG_RIP];
}

__attribute__((constructor)) static void arm(void)
{
    if (!getenv("SAMPLES"))
        return;
    struct sigaction sa = {0};
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, NULL);
    struct sigevent ev = {0};
    ev.sigev_notify = SIGEV_THREAD_ID;
    ev.sigev_signo = SIGPROF;
    ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
    timer_t tm;
    /* wall-clock ticks (a thread CPU-time timer ticks at the scheduler's
       granularity): a sample while the thread waits shows where it waits */
    /* SAMPLES_DELAY_MS (default 0): the first sample that long after start --
       a program initialising HIP is left alone until then (a signal in the
       middle of its first ioctls made the runtime report no device) */
    const char *dl = getenv("SAMPLES_DELAY_MS");
    const long delay_ms = dl ? atol(dl) : 0;
    if (timer_create(CLOCK_MONOTONIC, &ev, &tm) == 0) {
        struct itimerspec its = {{0, 50000}, {delay_ms / 1000, delay_ms % 1000 * 1000000 + (delay_ms ? 0 : 50000)}};
        timer_settime(tm, 0, &its, NULL);
    }
}

__attribute__((destructor)) static void dump(void)
{
    const char *path = getenv("SAMPLES");
    if (!path)
        return;
    signal(SIGPROF, SIG_IGN);
    FILE *f = fopen(path, "a");              /* (a program may link it twice) */
    if (!f)
        return;
    for (size_t k = 0; k < npc; k++) {
        Dl_info di;
        if (dladdr((void *)pc[k], &di) && di.dli_fname)
            fprintf(f, "%s 0x%lx\n", di.dli_fname, (unsigned long)(pc[k] - (uintptr_t)di.dli_fbase));
        else
            fprintf(f, "? 0x%lx\n", (unsigned long)pc[k]);
    }
    fclose(f);
}
