// tools/malloc_sites.c -- PROFILING AID ONLY: counts heap allocations by call
// site (LD_PRELOAD).  Every malloc/calloc/realloc is counted; every 16th one
// records a 6-frame backtrace.  At exit the sites with the most samples are
// printed as "<count> obj+off <- obj+off ..." (symbolize with addr2line).
//   gcc -O2 -shared -fPIC -o tools/libmalloc_sites.so tools/malloc_sites.c -ldl
//   LD_PRELOAD=tools/libmalloc_sites.so MALLOC_SITES_OUT=/tmp/ms.txt python bench.py ...
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

extern void* __libc_malloc(size_t);
extern void* __libc_calloc(size_t, size_t);
extern void* __libc_realloc(void*, size_t);
extern void __libc_free(void*);

#define DEPTH 6
#define SLOTS 65536
typedef struct
{
    void* pc[DEPTH];
    unsigned long n;
} Site;
static Site g_sites[SLOTS];
static unsigned long g_calls, g_frees, g_sampled;
static __thread int t_in;

static void record(void)
{
    unsigned long c = __atomic_add_fetch(&g_calls, 1, __ATOMIC_RELAXED);
    if ((c & 15) || t_in)
        return;
    t_in = 1;
    void* bt[DEPTH + 2];
    int n = backtrace(bt, DEPTH + 2);
    uint64_t h = 1469598103934665603ull;
    void* pc[DEPTH] = {0};
    for (int i = 2; i < n && i - 2 < DEPTH; ++i) {
        pc[i - 2] = bt[i];
        h = (h ^ (uint64_t)(uintptr_t)bt[i]) * 1099511628211ull;
    }
    for (unsigned k = 0; k < 64; ++k) {
        Site* s = &g_sites[(h + k) & (SLOTS - 1)];
        if (s->n == 0) {
            // (racy claim: a rare lost or merged sample is fine for a profile)
            memcpy(s->pc, pc, sizeof(pc));
            __atomic_add_fetch(&s->n, 1, __ATOMIC_RELAXED);
            break;
        }
        if (memcmp(s->pc, pc, sizeof(pc)) == 0) {
            __atomic_add_fetch(&s->n, 1, __ATOMIC_RELAXED);
            break;
        }
    }
    __atomic_add_fetch(&g_sampled, 1, __ATOMIC_RELAXED);
    t_in = 0;
}

void* malloc(size_t n)
{
    record();
    return __libc_malloc(n);
}
void* calloc(size_t a, size_t b)
{
    record();
    return __libc_calloc(a, b);
}
void* realloc(void* p, size_t n)
{
    record();
    return __libc_realloc(p, n);
}
void free(void* p)
{
    if (p)
        __atomic_add_fetch(&g_frees, 1, __ATOMIC_RELAXED);
    __libc_free(p);
}

static int cmp(const void* a, const void* b)
{
    const Site* x = a;
    const Site* y = b;
    return x->n < y->n ? 1 : x->n > y->n ? -1 : 0;
}

__attribute__((destructor)) static void dump(void)
{
    const char* path = getenv("MALLOC_SITES_OUT");
    char buf[512];
    if (path)
        snprintf(buf, sizeof(buf), "%s.%d", path, (int)getpid());
    FILE* f = path ? fopen(buf, "w") : stderr;
    if (!f)
        return;
    t_in = 1;
    static Site s[SLOTS];
    memcpy(s, g_sites, sizeof(s));
    qsort(s, SLOTS, sizeof(Site), cmp);
    fprintf(f, "calls %lu frees %lu sampled %lu (1 in 16)\n", g_calls, g_frees, g_sampled);
    for (int i = 0; i < 60 && s[i].n; ++i) {
        fprintf(f, "%lu", s[i].n);
        for (int d = 0; d < DEPTH && s[i].pc[d]; ++d) {
            Dl_info di;
            if (dladdr(s[i].pc[d], &di) && di.dli_fname)
                fprintf(f, " %s+%lx", di.dli_fname, (unsigned long)((char*)s[i].pc[d] - (char*)di.dli_fbase));
            else
                fprintf(f, " ?%p", s[i].pc[d]);
        }
        fprintf(f, "\n");
    }
    if (f != stderr)
        fclose(f);
}
