// tools/sampler.c -- a tiny SIGPROF sampling profiler for the host control
// plane (no perf/valgrind in this image).  Build and use:
//
//   gcc -O2 -shared -fPIC -o tools/libsampler.so tools/sampler.c -ldl -lpthread
//   python tools/host_profile.py /tmp/prof [bench.py args]
//   python tools/sampler_report.py /tmp/prof.<pid>
//
// Every 1 ms the stack of every running thread is recorded; at exit
// (to SAMPLER_OUT.<pid>) each frame is written as "<object>:<offset>" for addr2line.
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <ucontext.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <dirent.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#define MAX_SAMPLES 400000
#define MAX_DEPTH 24

static void* g_frames[MAX_SAMPLES][MAX_DEPTH];
static int g_depth[MAX_SAMPLES];
static volatile int g_count;

// Frame-pointer walk from the interrupted context (build the code under
// study with -fno-omit-frame-pointer); async-signal-safe, unlike backtrace().
static void on_prof(int sig, siginfo_t* si, void* ctx)
{
    (void)sig;
    (void)si;
    const int i = __sync_fetch_and_add(&g_count, 1);
    if (i >= MAX_SAMPLES)
        return;
    const ucontext_t* uc = (const ucontext_t*)ctx;
    uintptr_t pc = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
    uintptr_t fp = (uintptr_t)uc->uc_mcontext.gregs[REG_RBP];
    const uintptr_t sp = (uintptr_t)uc->uc_mcontext.gregs[REG_RSP];
    int d = 0;
    g_frames[i][d++] = (void*)(pc + 1);
    while (d < MAX_DEPTH && fp >= sp && fp < sp + (8u << 20) && (fp & 7) == 0) {
        const uintptr_t* f = (const uintptr_t*)fp;
        const uintptr_t ret = f[1], next = f[0];
        if (ret < 4096)
            break;
        g_frames[i][d++] = (void*)ret;
        if (next <= fp)
            break;
        fp = next;
    }
    g_depth[i] = d;
}

static void dump(void)
{
    const char* path = getenv("SAMPLER_OUT");
    if (!path)
        return;
    const int n = g_count < MAX_SAMPLES ? g_count : MAX_SAMPLES;
    if (n == 0)
        return;
    char name[4096];
    snprintf(name, sizeof(name), "%s.%d", path, (int)getpid());
    FILE* f = fopen(name, "w");
    if (!f)
        return;
    for (int i = 0; i < n; ++i) {
        fprintf(f, "S");
        for (int k = 0; k < g_depth[i]; ++k) {
            Dl_info info;
            if (dladdr(g_frames[i][k], &info) && info.dli_fname)
                fprintf(f, " %s:%lx", info.dli_fname,
                        (unsigned long)((char*)g_frames[i][k] - (char*)info.dli_fbase) - 1);
            else
                fprintf(f, " ?:%lx", (unsigned long)g_frames[i][k]);
        }
        fprintf(f, "\n");
    }
    fclose(f);
}

// A process-wide ITIMER_PROF signal reaches one thread per tick, so with
// many busy threads most of them go unseen.  Instead a helper thread wakes
// every millisecond and signals each thread that is running (state R).
static volatile int g_stop;

static void* ticker(void* arg)
{
    (void)arg;
    const pid_t pid = getpid();
    const pid_t self = (pid_t)syscall(SYS_gettid);
    char path[256], buf[512];
    while (!g_stop) {
        struct timespec ts = {0, 1000000};
        nanosleep(&ts, NULL);
        DIR* d = opendir("/proc/self/task");
        if (!d)
            continue;
        struct dirent* e;
        while ((e = readdir(d)) != NULL) {
            const pid_t tid = (pid_t)atoi(e->d_name);
            if (tid <= 0 || tid == self)
                continue;
            snprintf(path, sizeof(path), "/proc/self/task/%d/stat", (int)tid);
            const int fd = open(path, O_RDONLY);
            if (fd < 0)
                continue;
            const ssize_t n = read(fd, buf, sizeof(buf) - 1);
            close(fd);
            if (n <= 0)
                continue;
            buf[n] = 0;
            const char* rp = strrchr(buf, ')');
            if (rp && rp[1] == ' ' && rp[2] == 'R')
                syscall(SYS_tgkill, pid, tid, SIGPROF);
        }
        closedir(d);
    }
    return NULL;
}

static void stop(void)
{
    g_stop = 1;
    dump();
}

__attribute__((constructor)) static void start(void)
{
    if (!getenv("SAMPLER_OUT"))
        return;
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_RESTART | SA_SIGINFO;
    sigaction(SIGPROF, &sa, NULL);
    pthread_t t;
    pthread_create(&t, NULL, ticker, NULL);
    pthread_detach(t);
    atexit(stop);
}
