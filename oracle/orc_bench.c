/*
 * TEST INFRASTRUCTURE ONLY -- timing harness for bench.py's cpu_baseline leg.
 *
 * Runs one oracle operation per BASELINE workload on `threads` host threads, each with
 * its own codec object and its own stripes -- the way the reference runs one decoding
 * step per helper/coordinator thread (the SURVEY.md section 8(d) "one worker per host
 * core, independent stripes" baseline):
 *   ORC_BENCH_CLAY       Clay repair: orc_clay_perform_coding, the stage-by-stage
 *                        restatement of ClayCodeErasureDecodingStep.performCoding
 *                        (ClayCodeErasureDecodingStep.java:53-221) over
 *                        InputOutputByteTableCodingLoop (InputOutputByteTableCodingLoop.java:12-89)
 *   ORC_BENCH_RS_DECODE  ReedSolomon.decodeMissing in place (ReedSolomon.java:189-286);
 *                        RS(3,1) is the LRC local-group repair (LRCErasureCodeExample.kt:100-131)
 *   ORC_BENCH_RS_ENCODE  ReedSolomon.encodeParity (ReedSolomon.java:94-108), the operation
 *                        ReedSolomonBenchmark.java times
 *   ORC_BENCH_RS_CHECK   ReedSolomon.isParityCorrect with a temp buffer (ReedSolomon.java:159-178),
 *                        the "Check" half of ReedSolomonBenchmark.java:73-87,126-149; a stripe
 *                        whose parity is wrong fails the run, as the benchmark throws
 * Nothing here is used by the product (libecx.so).
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ecx_oracle.h"

typedef struct {
    int op, k, m, n_erased, buf, slots, per_thread;
    const int *erased;
    uint8_t *const *units; /* [threads * per_thread][slots], NULL = absent */
    double seconds;
    int tid;
    long long reps;
    double elapsed;
    int status;
} worker_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* One operation on one unit, with the worker's own codec object. */
typedef struct {
    orc_clay *clay;
    orc_rs *rs;
    uint8_t *present; /* RS decode: shard flags */
    uint8_t **outs;   /* Clay: |E| * alpha repaired sub-chunks */
    uint8_t *out_mem;
    uint8_t *temp;    /* RS check: the benchmark's tempBuffer (one shard) */
} op_state;

static int op_init(worker_t *w, op_state *s) {
    memset(s, 0, sizeof(*s));
    if (w->op == ORC_BENCH_CLAY) {
        int st = orc_clay_create(w->k, w->m, w->erased, w->n_erased, &s->clay);
        if (st) return st;
        const int nout = w->n_erased * orc_clay_alpha(s->clay);
        s->out_mem = (uint8_t *)calloc((size_t)nout, (size_t)w->buf);
        s->outs = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)nout);
        if (!s->out_mem || !s->outs) return ORC_E_NOMEM;
        for (int z = 0; z < nout; z++) s->outs[z] = s->out_mem + (size_t)z * (size_t)w->buf;
        return 0;
    }
    int st = orc_rs_create(w->k, w->m, &s->rs);
    if (st) return st;
    s->present = (uint8_t *)malloc((size_t)(w->k + w->m));
    if (!s->present) return ORC_E_NOMEM;
    memset(s->present, 1, (size_t)(w->k + w->m));
    for (int i = 0; i < w->n_erased; i++) s->present[w->erased[i]] = 0;
    if (w->op == ORC_BENCH_RS_CHECK && !(s->temp = (uint8_t *)malloc((size_t)w->buf))) return ORC_E_NOMEM;
    return 0;
}

static int op_run(worker_t *w, op_state *s, uint8_t *const *unit) {
    switch (w->op) {
    case ORC_BENCH_CLAY: return orc_clay_perform_coding(s->clay, unit, s->outs, w->buf);
    case ORC_BENCH_RS_DECODE: return orc_rs_decode_missing(s->rs, unit, s->present, w->k + w->m, w->buf, 0, w->buf);
    case ORC_BENCH_RS_ENCODE: return orc_rs_encode_parity(s->rs, unit, w->k + w->m, w->buf, 0, w->buf);
    case ORC_BENCH_RS_CHECK: {
        const int ok = orc_rs_is_parity_correct(s->rs, unit, w->k + w->m, w->buf, 0, w->buf, s->temp, w->buf);
        return ok == 1 ? 0 : (ok < 0 ? ok : ORC_E_ILLEGAL_ARGUMENT); /* "parity not correct" */
    }
    default: return ORC_E_ILLEGAL_ARGUMENT;
    }
}

static void op_free(op_state *s) {
    free(s->outs);
    free(s->out_mem);
    free(s->present);
    free(s->temp);
    if (s->clay) orc_clay_free(s->clay);
    if (s->rs) orc_rs_free(s->rs);
}

static void *worker(void *arg) {
    worker_t *w = (worker_t *)arg;
    op_state s;
    w->status = op_init(w, &s);
    uint8_t *const *mine = w->units + (size_t)w->tid * (size_t)w->per_thread * (size_t)w->slots;
    if (w->status == 0) w->status = op_run(w, &s, mine); /* one untimed warm-up operation */
    long long n = 0;
    double t0 = now_s(), el = 0.0;
    while (w->status == 0) {
        w->status = op_run(w, &s, mine + (size_t)(n % w->per_thread) * (size_t)w->slots);
        n++;
        el = now_s() - t0;
        if (el >= w->seconds) break;
    }
    w->reps = n;
    w->elapsed = el;
    op_free(&s);
    return NULL;
}

int orc_bench_run(int op, int data, int parity, const int *erased, int n_erased, int buf_size,
                  uint8_t *const *units, int slots, int per_thread, int threads, double seconds, long long *reps,
                  double *elapsed) {
    if (threads < 1 || per_thread < 1 || buf_size < 1 || slots < 1 || n_erased < 0) return ORC_E_ILLEGAL_ARGUMENT;
    if (op != ORC_BENCH_CLAY && op != ORC_BENCH_RS_DECODE && op != ORC_BENCH_RS_ENCODE && op != ORC_BENCH_RS_CHECK)
        return ORC_E_ILLEGAL_ARGUMENT;
    (void)orc_mul_table(); /* the GF tables, built before the threads start */
    worker_t *w = (worker_t *)calloc((size_t)threads, sizeof(worker_t));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    if (!w || !th) {
        free(w);
        free(th);
        return ORC_E_NOMEM;
    }
    for (int i = 0; i < threads; i++) {
        w[i] = (worker_t){op, data, parity, n_erased, buf_size, slots, per_thread, erased, units, seconds, i, 0, 0.0, 0};
        pthread_create(&th[i], NULL, worker, &w[i]);
    }
    int st = 0;
    long long total = 0;
    double max_el = 0.0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        if (w[i].status != 0) st = w[i].status;
        total += w[i].reps;
        if (w[i].elapsed > max_el) max_el = w[i].elapsed;
    }
    free(th);
    free(w);
    *reps = total;
    *elapsed = max_el;
    return st;
}

int orc_bench_clay_repair(int data_units, int parity_units, int erased, int buf_size, uint8_t *const *stripes,
                          int per_thread, int threads, double seconds, long long *repairs, double *elapsed) {
    orc_clay *probe = NULL;
    int e[1] = {erased};
    int st = orc_clay_create(data_units, parity_units, e, 1, &probe);
    if (st != 0) return st;
    const int slots = (data_units + parity_units) * orc_clay_alpha(probe);
    orc_clay_free(probe);
    return orc_bench_run(ORC_BENCH_CLAY, data_units, parity_units, e, 1, buf_size, stripes, slots, per_thread, threads,
                         seconds, repairs, elapsed);
}
