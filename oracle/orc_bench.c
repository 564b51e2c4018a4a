/*
 * TEST INFRASTRUCTURE ONLY -- timing harness for bench.py's cpu_baseline leg.
 *
 * Runs the oracle's Clay single-node repair (orc_clay_perform_coding, the
 * stage-by-stage restatement of ClayCodeErasureDecodingStep.doDecodeSingle,
 * ClayCodeErasureDecodingStep.java:118-221, over InputOutputByteTableCodingLoop,
 * InputOutputByteTableCodingLoop.java:12-89) on `threads` host threads, each on its
 * own ClayCodeErasureDecodingStep object and its own stripes -- the way the
 * reference runs one decoding step per helper/coordinator thread.  This is the
 * SURVEY.md section 8(d) "one worker per host core, independent stripes" baseline.
 * Nothing here is used by the product (libecx.so).
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ecx_oracle.h"

typedef struct {
    int k, m, erased, buf, slots, per_thread;
    uint8_t *const *stripes; /* [threads * per_thread][slots], NULL = absent */
    double seconds;
    int tid;
    long long repairs;
    double elapsed;
    int status;
} worker_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *worker(void *arg) {
    worker_t *w = (worker_t *)arg;
    orc_clay *c = NULL;
    int e[1] = {w->erased};
    w->status = orc_clay_create(w->k, w->m, e, 1, &c);
    if (w->status != 0) return NULL;
    int alpha = orc_clay_alpha(c);
    uint8_t *out_mem = (uint8_t *)calloc((size_t)alpha, (size_t)w->buf);
    uint8_t **outs = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)alpha);
    for (int z = 0; z < alpha; z++) outs[z] = out_mem + (size_t)z * (size_t)w->buf;
    uint8_t *const *mine = w->stripes + (size_t)w->tid * (size_t)w->per_thread * (size_t)w->slots;
    /* one untimed warm-up repair */
    w->status = orc_clay_perform_coding(c, mine, outs, w->buf);
    long long n = 0;
    double t0 = now_s(), el = 0.0;
    while (w->status == 0) {
        w->status = orc_clay_perform_coding(c, mine + (size_t)(n % w->per_thread) * (size_t)w->slots, outs, w->buf);
        n++;
        el = now_s() - t0;
        if (el >= w->seconds) break;
    }
    w->repairs = n;
    w->elapsed = el;
    free(outs);
    free(out_mem);
    orc_clay_free(c);
    return NULL;
}

int orc_bench_clay_repair(int data_units, int parity_units, int erased, int buf_size, uint8_t *const *stripes,
                          int per_thread, int threads, double seconds, long long *repairs, double *elapsed) {
    if (threads < 1 || per_thread < 1 || buf_size < 1) return ORC_E_ILLEGAL_ARGUMENT;
    orc_clay *probe = NULL;
    int e[1] = {erased};
    int st = orc_clay_create(data_units, parity_units, e, 1, &probe); /* also initialises the GF tables */
    if (st != 0) return st;
    int slots = (data_units + parity_units) * orc_clay_alpha(probe);
    orc_clay_free(probe);

    worker_t *w = (worker_t *)calloc((size_t)threads, sizeof(worker_t));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int i = 0; i < threads; i++) {
        w[i] = (worker_t){data_units, parity_units, erased, buf_size, slots, per_thread, stripes, seconds, i, 0, 0.0, 0};
        pthread_create(&th[i], NULL, worker, &w[i]);
    }
    long long total = 0;
    double max_el = 0.0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        if (w[i].status != 0) st = w[i].status;
        total += w[i].repairs;
        if (w[i].elapsed > max_el) max_el = w[i].elapsed;
    }
    free(th);
    free(w);
    *repairs = total;
    *elapsed = max_el;
    return st;
}
