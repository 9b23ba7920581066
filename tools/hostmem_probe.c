// Host first-touch probe (no GPU): how fast can fresh anonymous memory be made writable on this host?
// The mesh copy of the C5 extraction (988 MB device -> host numpy) is bound by the destination's page
// faults (profiles/r05_d2h_probe.jsonl).  Measures, for a 1 GiB buffer, the rate of writing every byte
// once with T threads for: plain malloc (4 KiB faults unless THP "always"), a 2 MiB-aligned mapping with
// madvise(MADV_HUGEPAGE), MAP_POPULATE (kernel pre-faults at mmap time, then the write), and a second
// write to memory already present (the ceiling).  Prints one JSON line.
//   gcc -O2 -pthread -o tools/_ab/hostmem_probe tools/hostmem_probe.c
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

typedef struct { char* p; size_t n; } Job;
static void* fill(void* a) {
    Job* j = (Job*)a;
    memset(j->p, 1, j->n);
    return NULL;
}

static double touch(char* p, size_t n, int T) {
    pthread_t th[64];
    Job jobs[64];
    size_t per = (n / T + 4095) & ~(size_t)4095;
    double t0 = now();
    for (int i = 0; i < T; i++) {
        size_t lo = (size_t)i * per, hi = lo + per < n ? lo + per : n;
        jobs[i].p = p + lo;
        jobs[i].n = hi > lo ? hi - lo : 0;
        pthread_create(&th[i], NULL, fill, &jobs[i]);
    }
    for (int i = 0; i < T; i++) pthread_join(th[i], NULL);
    return n / (now() - t0) / 1e9;
}

static void read_file(const char* path, char* out, size_t cap) {
    FILE* f = fopen(path, "r");
    out[0] = 0;
    if (!f) { snprintf(out, cap, "unreadable"); return; }
    if (!fgets(out, (int)cap, f)) out[0] = 0;
    fclose(f);
    size_t l = strlen(out);
    while (l && (out[l - 1] == '\n')) out[--l] = 0;
}

int main(void) {
    const size_t n = (size_t)1 << 30;
    char thp[256], defrag[256];
    read_file("/sys/kernel/mm/transparent_hugepage/enabled", thp, sizeof thp);
    read_file("/sys/kernel/mm/transparent_hugepage/defrag", defrag, sizeof defrag);
    printf("{\"bytes\": %zu, \"thp_enabled\": \"%s\", \"thp_defrag\": \"%s\", \"runs\": [", n, thp, defrag);
    const int Ts[] = {1, 4, 8, 16};
    int first = 1;
    for (int k = 0; k < 4; k++) {
        int T = Ts[k];
        char* a = (char*)malloc(n);
        double g_malloc = touch(a, n, T);
        double g_again = touch(a, n, T);
        free(a);
        char* m = (char*)mmap(NULL, n + (2u << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        char* h = (char*)(((uintptr_t)m + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1));
        int adv = madvise(h, n, MADV_HUGEPAGE);
        double g_huge = touch(h, n, T);
        munmap(m, n + (2u << 20));
        double t0 = now();
        char* q = (char*)mmap(NULL, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        double t_pop = now() - t0;
        double g_pop_write = touch(q, n, T);
        munmap(q, n);
        printf("%s{\"threads\": %d, \"malloc_first_gbs\": %.2f, \"present_gbs\": %.2f, \"hugepage_madvise_rc\": %d, "
               "\"hugepage_first_gbs\": %.2f, \"populate_ms\": %.1f, \"populate_then_write_gbs\": %.2f, "
               "\"populate_total_gbs\": %.2f}",
               first ? "" : ", ", T, g_malloc, g_again, adv, g_huge, 1e3 * t_pop, g_pop_write,
               n / (t_pop + n / (g_pop_write * 1e9)) / 1e9);
        first = 0;
    }
    printf("]}\n");
    return 0;
}
