/*
 * ecx_oracle.c -- TEST INFRASTRUCTURE ONLY (see ecx_oracle.h).
 *
 * Byte-at-a-time C restatement of the reference JVM CPU path.  Loop orders,
 * row-selection rules and buffer semantics (aliasing, in-place writes into
 * non-present shards, fresh zero arrays for nulls) follow the Java code so
 * that the outputs are the reference's outputs for ANY input bytes, not only
 * for valid codewords.  Never linked into the product.
 */
#include "ecx_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ======================================================================
 * java.util.Random -- JDK public specification (48-bit LCG 0x5DEECE66D).
 * Used by ClayCode.getInputs (ClayCode.java:50,62) and ReedSolomonTest
 * (ReedSolomonTest.java:92,181).
 * ==================================================================== */
#define JR_MULT 0x5DEECE66DULL
#define JR_MASK ((1ULL << 48) - 1)

void orc_jrandom_init(orc_jrandom *r, int64_t seed) { r->seed = ((uint64_t)seed ^ JR_MULT) & JR_MASK; }

static int32_t jr_next(orc_jrandom *r, int bits) {
    r->seed = (r->seed * JR_MULT + 0xBULL) & JR_MASK;
    return (int32_t)(r->seed >> (48 - bits));
}

int32_t orc_jrandom_next_int(orc_jrandom *r) { return jr_next(r, 32); }

int32_t orc_jrandom_next_int_bound(orc_jrandom *r, int32_t bound) {
    if (bound <= 0) return ORC_E_ILLEGAL_ARGUMENT;
    if ((bound & -bound) == bound) return (int32_t)(((int64_t)bound * (int64_t)jr_next(r, 31)) >> 31);
    int32_t bits, val;
    do {
        bits = jr_next(r, 31);
        val = bits % bound;
    } while (bits - val + (bound - 1) < 0);
    return val;
}

void orc_jrandom_next_bytes(orc_jrandom *r, uint8_t *out, int len) {
    for (int i = 0; i < len;) {
        int32_t rnd = orc_jrandom_next_int(r);
        for (int n = (len - i < 4) ? len - i : 4; n-- > 0; rnd >>= 8) out[i++] = (uint8_t)rnd;
    }
}

/* ======================================================================
 * Galois.java
 * ==================================================================== */
#define FIELD_SIZE 256
#define GENERATING_POLYNOMIAL 29 /* Galois.java:43 */

static int16_t g_log[256];
static uint8_t g_exp[510];
static uint8_t g_mul[256 * 256];
static int g_ready = 0;

/* Galois.generateLogTable, Galois.java:259-276 */
int orc_gen_log_table(int polynomial, int16_t out[256]) {
    for (int i = 0; i < FIELD_SIZE; i++) out[i] = -1;
    int b = 1;
    for (int log = 0; log < FIELD_SIZE - 1; log++) {
        if (out[b] != -1) return ORC_E_ILLEGAL_ARGUMENT; /* "duplicate logarithm" */
        out[b] = (int16_t)log;
        b = b << 1;
        if (FIELD_SIZE <= b) b = (b - FIELD_SIZE) ^ polynomial;
    }
    return ORC_OK;
}

/* Galois.generateExpTable, Galois.java:281-289 */
void orc_gen_exp_table(const int16_t log_table[256], uint8_t out[510]) {
    memset(out, 0, 510);
    for (int i = 1; i < FIELD_SIZE; i++) {
        int log = log_table[i];
        out[log] = (uint8_t)i;
        out[log + FIELD_SIZE - 1] = (uint8_t)i;
    }
}

/* Galois.multiply, Galois.java:199-209 (log/exp path) */
static uint8_t gf_mul_logexp(uint8_t a, uint8_t b) {
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

static void gf_init(void) {
    if (g_ready) return;
    orc_gen_log_table(GENERATING_POLYNOMIAL, g_log);
    orc_gen_exp_table(g_log, g_exp);
    /* Galois.generateMultiplicationTable, Galois.java:298-306 */
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++) g_mul[a * 256 + b] = gf_mul_logexp((uint8_t)a, (uint8_t)b);
    g_ready = 1;
}

const int16_t *orc_log_table(void) { gf_init(); return g_log; }
const uint8_t *orc_exp_table(void) { gf_init(); return g_exp; }
const uint8_t *orc_mul_table(void) { gf_init(); return g_mul; }

uint8_t orc_gf_multiply(uint8_t a, uint8_t b) { gf_init(); return gf_mul_logexp(a, b); }

/* Galois.divide, Galois.java:214-228 */
int orc_gf_divide(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0) return 0;
    if (b == 0) return ORC_E_ILLEGAL_ARGUMENT;
    int r = g_log[a] - g_log[b];
    if (r < 0) r += 255;
    return g_exp[r];
}

/* Galois.exp, Galois.java:239-254 */
uint8_t orc_gf_exp(uint8_t a, int n) {
    gf_init();
    if (n == 0) return 1;
    if (a == 0) return 0;
    int r = g_log[a] * n;
    while (255 <= r) r -= 255;
    return g_exp[r];
}

/* Galois.allPossiblePolynomials, Galois.java:314-326 */
int orc_all_possible_polynomials(int *out) {
    int16_t tmp[256];
    int n = 0;
    for (int i = 0; i < FIELD_SIZE; i++)
        if (orc_gen_log_table(i, tmp) == ORC_OK) out[n++] = i;
    return n;
}

/* ======================================================================
 * Matrix.java
 * ==================================================================== */

/* Matrix.times, Matrix.java:193-210 */
int orc_matrix_times(const uint8_t *a, int ar, int ac, const uint8_t *b, int br, int bc, uint8_t *out) {
    gf_init();
    if (ac != br) return ORC_E_ILLEGAL_ARGUMENT;
    for (int r = 0; r < ar; r++)
        for (int c = 0; c < bc; c++) {
            uint8_t v = 0;
            for (int i = 0; i < ac; i++) v ^= gf_mul_logexp(a[r * ac + i], b[i * bc + c]);
            out[r * bc + c] = v;
        }
    return ORC_OK;
}

/* Matrix.invert + gaussianElimination, Matrix.java:273-346, on the
 * augmented [M | I] work matrix (rows are swapped as whole rows). */
int orc_matrix_invert(const uint8_t *m, int n, uint8_t *out) {
    gf_init();
    int cols = 2 * n;
    uint8_t *w = (uint8_t *)calloc((size_t)n * cols, 1);
    uint8_t *tmp = (uint8_t *)malloc((size_t)cols);
    if (!w || !tmp) { free(w); free(tmp); return ORC_E_NOMEM; }
    for (int r = 0; r < n; r++) {
        memcpy(w + r * cols, m + r * n, (size_t)n);
        w[r * cols + n + r] = 1;
    }
    for (int r = 0; r < n; r++) {
        if (w[r * cols + r] == 0) {
            for (int below = r + 1; below < n; below++) {
                if (w[below * cols + r] != 0) {
                    memcpy(tmp, w + r * cols, (size_t)cols);
                    memcpy(w + r * cols, w + below * cols, (size_t)cols);
                    memcpy(w + below * cols, tmp, (size_t)cols);
                    break;
                }
            }
        }
        if (w[r * cols + r] == 0) { free(w); free(tmp); return ORC_E_SINGULAR; }
        if (w[r * cols + r] != 1) {
            uint8_t scale = (uint8_t)orc_gf_divide(1, w[r * cols + r]);
            for (int c = 0; c < cols; c++) w[r * cols + c] = gf_mul_logexp(w[r * cols + c], scale);
        }
        for (int below = r + 1; below < n; below++) {
            uint8_t scale = w[below * cols + r];
            if (scale != 0)
                for (int c = 0; c < cols; c++) w[below * cols + c] ^= gf_mul_logexp(scale, w[r * cols + c]);
        }
    }
    for (int d = 0; d < n; d++)
        for (int above = 0; above < d; above++) {
            uint8_t scale = w[above * cols + d];
            if (scale != 0)
                for (int c = 0; c < cols; c++) w[above * cols + c] ^= gf_mul_logexp(scale, w[d * cols + c]);
        }
    for (int r = 0; r < n; r++) memcpy(out + r * n, w + r * cols + n, (size_t)n);
    free(w);
    free(tmp);
    return ORC_OK;
}

/* ======================================================================
 * Coding loops
 * ==================================================================== */

/* InputOutputByteTableCodingLoop.codeSomeShards, InputOutputByteTableCodingLoop.java:12-44:
 * input-major, first input assigns, later inputs XOR-accumulate, 256-B table rows. */
void orc_code_some_shards(const uint8_t *const *matrix_rows, uint8_t *const *inputs, int input_count,
                          uint8_t *const *outputs, int output_count, int offset, int byte_count) {
    gf_init();
    if (input_count <= 0) return;
    {
        const uint8_t *in = inputs[0];
        for (int o = 0; o < output_count; o++) {
            uint8_t *out = outputs[o];
            const uint8_t *row = g_mul + 256 * matrix_rows[o][0];
            for (int b = offset; b < offset + byte_count; b++) out[b] = row[in[b]];
        }
    }
    for (int i = 1; i < input_count; i++) {
        const uint8_t *in = inputs[i];
        for (int o = 0; o < output_count; o++) {
            uint8_t *out = outputs[o];
            const uint8_t *row = g_mul + 256 * matrix_rows[o][i];
            for (int b = offset; b < offset + byte_count; b++) out[b] ^= row[in[b]];
        }
    }
}

/* CodingLoopBase.checkSomeShards (CodingLoopBase.java:18-41) when temp_buffer is NULL,
 * else the OutputInputByte variant of InputOutputByteTableCodingLoop.java:47-89. */
int orc_check_some_shards(const uint8_t *const *matrix_rows, uint8_t *const *inputs, int input_count,
                          uint8_t *const *to_check, int check_count, int offset, int byte_count,
                          uint8_t *temp) {
    gf_init();
    if (temp == NULL) {
        for (int b = offset; b < offset + byte_count; b++)
            for (int o = 0; o < check_count; o++) {
                uint8_t v = 0;
                for (int i = 0; i < input_count; i++) v ^= g_mul[256 * matrix_rows[o][i] + inputs[i][b]];
                if (to_check[o][b] != v) return 0;
            }
        return 1;
    }
    for (int o = 0; o < check_count; o++) {
        const uint8_t *row0 = g_mul + 256 * matrix_rows[o][0];
        for (int b = offset; b < offset + byte_count; b++) temp[b] = row0[inputs[0][b]];
        for (int i = 1; i < input_count; i++) {
            const uint8_t *row = g_mul + 256 * matrix_rows[o][i];
            for (int b = offset; b < offset + byte_count; b++) temp[b] ^= row[inputs[i][b]];
        }
        for (int b = offset; b < offset + byte_count; b++)
            if (temp[b] != to_check[o][b]) return 0;
    }
    return 1;
}

/* InputOutputByteTableCodingLoopSingle.codeSomeShards, InputOutputByteTableCodingLoopSingle.java:4-20 */
void orc_code_single(const uint8_t *const *matrix_rows, const uint8_t *input, int index, uint8_t *output,
                     int output_index, int offset, int byte_count, int is_first_time) {
    gf_init();
    const uint8_t *row = g_mul + 256 * matrix_rows[output_index][index];
    for (int b = offset; b < offset + byte_count; b++) {
        if (is_first_time) output[b] = row[input[b]];
        else output[b] ^= row[input[b]];
    }
}

/* ======================================================================
 * ReedSolomon.java
 * ==================================================================== */
struct orc_rs {
    int k, m, n;
    uint8_t *matrix;      /* n x k */
    uint8_t **parity_rows; /* m pointers into matrix */
};

int orc_rs_create(int data_shards, int parity_shards, orc_rs **out) {
    gf_init();
    *out = NULL;
    /* ReedSolomon.java:48-50 */
    if (256 < data_shards + parity_shards) return ORC_E_TOO_MANY_SHARDS;
    if (data_shards <= 0 || parity_shards < 0) return ORC_E_ILLEGAL_ARGUMENT;
    int k = data_shards, n = data_shards + parity_shards;
    orc_rs *rs = (orc_rs *)calloc(1, sizeof(orc_rs));
    rs->k = k; rs->m = parity_shards; rs->n = n;
    /* buildMatrix (ReedSolomon.java:373-385) + vandermonde (:396-404) */
    uint8_t *vm = (uint8_t *)malloc((size_t)n * k);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) vm[r * k + c] = orc_gf_exp((uint8_t)r, c);
    uint8_t *inv = (uint8_t *)malloc((size_t)k * k);
    int st = orc_matrix_invert(vm, k, inv); /* top square = first k rows */
    if (st) { free(vm); free(inv); free(rs); return st; }
    rs->matrix = (uint8_t *)malloc((size_t)n * k);
    orc_matrix_times(vm, n, k, inv, k, k, rs->matrix);
    free(vm);
    free(inv);
    rs->parity_rows = (uint8_t **)malloc(sizeof(uint8_t *) * (parity_shards ? parity_shards : 1));
    for (int i = 0; i < parity_shards; i++) rs->parity_rows[i] = rs->matrix + (size_t)(k + i) * k;
    *out = rs;
    return ORC_OK;
}

void orc_rs_free(orc_rs *rs) {
    if (!rs) return;
    free(rs->matrix);
    free(rs->parity_rows);
    free(rs);
}

int orc_rs_data_count(const orc_rs *rs) { return rs->k; }
int orc_rs_parity_count(const orc_rs *rs) { return rs->m; }
void orc_rs_matrix(const orc_rs *rs, uint8_t *out) { memcpy(out, rs->matrix, (size_t)rs->n * rs->k); }

/* checkBuffersAndSizes, ReedSolomon.java:338-363 (all shards share one length) */
static int rs_check(const orc_rs *rs, int shard_count, int shard_len, int offset, int byte_count) {
    if (shard_count != rs->n) return ORC_E_ILLEGAL_ARGUMENT;
    if (offset < 0 || byte_count < 0) return ORC_E_ILLEGAL_ARGUMENT;
    if (shard_len < offset + byte_count) return ORC_E_ILLEGAL_ARGUMENT;
    return ORC_OK;
}

/* encodeParity, ReedSolomon.java:94-108 */
int orc_rs_encode_parity(orc_rs *rs, uint8_t *const *shards, int shard_count, int shard_len, int offset,
                         int byte_count) {
    int st = rs_check(rs, shard_count, shard_len, offset, byte_count);
    if (st) return st;
    orc_code_some_shards((const uint8_t *const *)rs->parity_rows, shards, rs->k, shards + rs->k, rs->m, offset,
                         byte_count);
    return ORC_OK;
}

/* encodeParitySingle, ReedSolomon.java:110-118 (isFirstTime=false: always XOR) */
int orc_rs_encode_parity_single(orc_rs *rs, const uint8_t *shard, uint8_t *output, int input_index,
                                int output_index, int offset, int byte_count) {
    if (output_index < 0 || output_index >= rs->m || input_index < 0 || input_index >= rs->k) return ORC_E_INDEX;
    orc_code_single((const uint8_t *const *)rs->parity_rows, shard, input_index, output, output_index, offset,
                    byte_count, 0);
    return ORC_OK;
}

/* isParityCorrect (both overloads), ReedSolomon.java:129-178 */
int orc_rs_is_parity_correct(orc_rs *rs, uint8_t *const *shards, int shard_count, int shard_len, int first_byte,
                             int byte_count, uint8_t *temp, int temp_len) {
    int st = rs_check(rs, shard_count, shard_len, first_byte, byte_count);
    if (st) return st;
    if (temp && temp_len < first_byte + byte_count) return ORC_E_ILLEGAL_ARGUMENT;
    return orc_check_some_shards((const uint8_t *const *)rs->parity_rows, shards, rs->k, shards + rs->k, rs->m,
                                 first_byte, byte_count, temp);
}

/* decodeMissing, ReedSolomon.java:189-286 */
int orc_rs_decode_missing(orc_rs *rs, uint8_t *const *shards, const uint8_t *present, int shard_count,
                          int shard_len, int offset, int byte_count) {
    int st = rs_check(rs, shard_count, shard_len, offset, byte_count);
    if (st) return st;
    const int k = rs->k, n = rs->n;
    int number_present = 0;
    for (int i = 0; i < n; i++) number_present += present[i] ? 1 : 0;
    if (number_present == n) return ORC_OK;
    if (number_present < k) return ORC_E_NOT_ENOUGH_SHARDS;

    uint8_t *sub = (uint8_t *)malloc((size_t)k * k);
    uint8_t *inv = (uint8_t *)malloc((size_t)k * k);
    uint8_t **sub_shards = (uint8_t **)malloc(sizeof(uint8_t *) * k);
    int row = 0;
    for (int mr = 0; mr < n && row < k; mr++) { /* first k present rows, ascending (:226-236) */
        if (present[mr]) {
            memcpy(sub + row * k, rs->matrix + (size_t)mr * k, (size_t)k);
            sub_shards[row] = shards[mr];
            row++;
        }
    }
    st = orc_matrix_invert(sub, k, inv);
    if (st) { free(sub); free(inv); free(sub_shards); return st; }

    int cap = rs->m > 0 ? rs->m : 1;
    uint8_t **outs = (uint8_t **)malloc(sizeof(uint8_t *) * cap);
    const uint8_t **rows = (const uint8_t **)malloc(sizeof(uint8_t *) * cap);
    int oc = 0;
    for (int i = 0; i < k; i++) /* missing data shards from the k sub shards (:254-265) */
        if (!present[i]) {
            if (oc >= cap) { st = ORC_E_INDEX; goto done; }
            outs[oc] = shards[i];
            rows[oc] = inv + (size_t)i * k;
            oc++;
        }
    orc_code_some_shards(rows, sub_shards, k, outs, oc, offset, byte_count);
    oc = 0;
    for (int i = k; i < n; i++) /* missing parity from ALL data shards (:273-285) */
        if (!present[i]) {
            outs[oc] = shards[i];
            rows[oc] = rs->parity_rows[i - k];
            oc++;
        }
    orc_code_some_shards(rows, shards, k, outs, oc, offset, byte_count);
done:
    free(outs);
    free(rows);
    free(sub);
    free(inv);
    free(sub_shards);
    return st;
}

/* decodeMissingSingle, ReedSolomon.java:288-333.  The reference replaces
 * outputs[j] with fresh arrays when (isFirst && shardIndex < k); here the
 * caller's arrays are written (assign when isFirst, XOR otherwise), which is
 * the same result for the caller that reads outputs[] afterwards.  A missing
 * matrix row (output j beyond the missing data shards) is the reference's NPE. */
int orc_rs_decode_missing_single(orc_rs *rs, const uint8_t *shard, int shard_index, int index,
                                 const uint8_t *present, uint8_t *const *outputs, int output_count, int offset,
                                 int byte_count, int is_first) {
    (void)shard_index;
    const int k = rs->k, n = rs->n;
    uint8_t *sub = (uint8_t *)malloc((size_t)k * k);
    uint8_t *inv = (uint8_t *)malloc((size_t)k * k);
    int row = 0;
    for (int mr = 0; mr < n && row < k; mr++)
        if (present[mr]) { memcpy(sub + row * k, rs->matrix + (size_t)mr * k, (size_t)k); row++; }
    int st = row < k ? ORC_E_SINGULAR : orc_matrix_invert(sub, k, inv);
    if (st) { free(sub); free(inv); return st; }
    int cap = rs->m;
    const uint8_t **rows = (const uint8_t **)calloc((size_t)(cap > 0 ? cap : 1), sizeof(uint8_t *));
    int oc = 0;
    for (int i = 0; i < k; i++)
        if (!present[i]) {
            if (oc >= cap) { st = ORC_E_INDEX; goto done; }
            rows[oc++] = inv + (size_t)i * k;
        }
    if (output_count > cap) { st = ORC_E_INDEX; goto done; }
    for (int j = 0; j < output_count; j++) {
        if (rows[j] == NULL) { st = ORC_E_NULL; goto done; }
        if (index < 0 || index >= k) { st = ORC_E_INDEX; goto done; }
        orc_code_single(rows, shard, index, outputs[j], j, offset, byte_count, is_first);
    }
done:
    free(rows);
    free(sub);
    free(inv);
    return st;
}

/* ======================================================================
 * Clay: ClayCodeErasureDecodingStep.java (+ ClayCodeUtil :676-944)
 *
 * Buffers are byte pointers (NULL = Java null).  Every array the Java code
 * allocates comes from a per-call arena; aliasing (temp[i] = inputs[z][i])
 * is pointer aliasing, and decodeMissing writes into the arrays of
 * non-present shards in place, exactly as the JVM does.
 * ==================================================================== */
struct orc_clay {
    int k, m, n, q, t, alpha;
    int *erased;
    int n_erased;
    int is_test; /* -DisTest=true: decodeDecoupledPlane's isTest branch on single repairs (:571-581) */
    orc_rs *pair; /* ReedSolomon.create(2,2) -- ClayCode.java:33 */
    orc_rs *rs;   /* ReedSolomon.create(k,m) -- ClayCode.java:34 */
};

typedef struct {
    uint8_t **blocks;
    int n, cap;
    int size;
} arena_t;

static uint8_t *arena_zero(arena_t *a) {
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 64;
        a->blocks = (uint8_t **)realloc(a->blocks, sizeof(uint8_t *) * a->cap);
    }
    uint8_t *p = (uint8_t *)calloc((size_t)(a->size > 0 ? a->size : 1), 1);
    a->blocks[a->n++] = p;
    return p;
}

static void arena_free(arena_t *a) {
    for (int i = 0; i < a->n; i++) free(a->blocks[i]);
    free(a->blocks);
}

static uint8_t *arena_clone(arena_t *a, const uint8_t *src) { /* cloneBufferData :723-740 */
    uint8_t *p = arena_zero(a);
    memcpy(p, src, (size_t)a->size);
    return p;
}

static int ipow(int b, int e) {
    int r = 1;
    while (e-- > 0) r *= b;
    return r;
}

/* ClayCodeUtil ctor :690-695 (t is INTEGER division, alpha = q^t) */
int orc_clay_create_ex(int data_units, int parity_units, const int *erased, int n_erased, int is_test,
                       orc_clay **out) {
    int st = orc_clay_create(data_units, parity_units, erased, n_erased, out);
    if (st == ORC_OK) (*out)->is_test = is_test != 0;
    return st;
}

int orc_clay_create(int data_units, int parity_units, const int *erased, int n_erased, orc_clay **out) {
    *out = NULL;
    if (parity_units <= 0 || data_units <= 0) return ORC_E_ILLEGAL_ARGUMENT;
    orc_clay *c = (orc_clay *)calloc(1, sizeof(orc_clay));
    c->k = data_units; c->m = parity_units; c->n = data_units + parity_units;
    c->q = parity_units;
    c->t = (parity_units + data_units) / parity_units;
    c->alpha = ipow(c->q, c->t);
    c->n_erased = n_erased;
    c->erased = (int *)malloc(sizeof(int) * (n_erased > 0 ? n_erased : 1));
    for (int i = 0; i < n_erased; i++) c->erased[i] = erased[i];
    int st = orc_rs_create(2, 2, &c->pair);
    if (!st) st = orc_rs_create(data_units, parity_units, &c->rs);
    if (st) { orc_clay_free(c); return st; }
    *out = c;
    return ORC_OK;
}

void orc_clay_free(orc_clay *c) {
    if (!c) return;
    orc_rs_free(c->pair);
    orc_rs_free(c->rs);
    free(c->erased);
    free(c);
}

int orc_clay_q(const orc_clay *c) { return c->q; }
int orc_clay_t(const orc_clay *c) { return c->t; }
int orc_clay_alpha(const orc_clay *c) { return c->alpha; }

static void z_vector(const orc_clay *c, int z, int *v) { /* getZVector :774-783, v[0] most significant */
    for (int i = c->t - 1; i >= 0; --i) { v[i] = z % c->q; z /= c->q; }
}
static int z_index(const orc_clay *c, const int *v) { /* getZ :757-766 */
    int z = 0, p = 1;
    for (int i = c->t - 1; i >= 0; --i) { z += v[i] * p; p *= c->q; }
    return z;
}
static int node_index(const orc_clay *c, int x, int y) { return x + c->q * y; } /* :847-849 */
static int node_x(const orc_clay *c, int i) { return i % c->q; }              /* :855-860 */
static int node_y(const orc_clay *c, int i) { return i / c->q; }
static int couple_plane(const orc_clay *c, int x, int y, int z) { /* getCouplePlaneIndex :911-915 */
    int v[64];
    z_vector(c, z, v);
    v[y] = x;
    return z_index(c, v);
}

/* getHelperPlanesIndexes :924-941 */
int orc_clay_helper_planes(const orc_clay *c, int k, int *out) {
    int x = node_x(c, k), y = node_y(c, k), j = 0, v[64];
    if (y >= c->t) return ORC_E_INDEX;
    for (int i = 0; i < c->alpha; i++) {
        z_vector(c, i, v);
        if (v[y] == x) out[j++] = i;
    }
    return j;
}

static int is_erased(const orc_clay *c, int idx) {
    for (int i = 0; i < c->n_erased; i++)
        if (c->erased[i] == idx) return 1;
    return 0;
}

/* getErasureType :884-903 */
static int erasure_type(const orc_clay *c, int idx, int z) {
    int v[64];
    z_vector(c, z, v);
    int x = node_x(c, idx), y = node_y(c, idx);
    if (v[y] == x) return 0;
    if (is_erased(c, node_index(c, v[y], y))) return 2;
    return 1;
}

/* getIntersectionScore :804-817 */
static int intersection_score(const orc_clay *c, int z) {
    int v[64], s = 0;
    z_vector(c, z, v);
    for (int i = 0; i < c->n_erased; i++) {
        int e = c->erased[i];
        if (v[node_y(c, e)] == node_x(c, e)) s++;
    }
    return s;
}

/* getPairWiseCouple :630-666 -- RS(2,2).decodeMissing over (A, A', B, B');
 * out[0], out[1] = the arrays at the null positions, in ascending order. */
static int pairwise(orc_clay *c, arena_t *ar, uint8_t *in[4], uint8_t **out0, uint8_t **out1) {
    int lost[2] = {0, 0}, nl = 0;
    uint8_t *arr[4];
    uint8_t present[4];
    for (int i = 0; i < 4; i++) {
        if (in[i] == NULL) {
            if (nl >= 2) return ORC_E_INDEX;
            lost[nl++] = i;
        }
    }
    for (int i = 0; i < 4; i++) arr[i] = in[i] ? in[i] : arena_zero(ar); /* getByteArray :599-609 */
    for (int i = 0; i < 4; i++) present[i] = 1;                          /* getShardPresent :611-620 */
    present[lost[0]] = 0;
    present[lost[1]] = 0;
    int st = orc_rs_decode_missing(c->pair, arr, present, 4, ar->size, 0, ar->size);
    if (st) return st;
    *out0 = arr[lost[0]];
    if (out1) *out1 = arr[lost[1]];
    return ORC_OK;
}

/* decodeDecoupledPlane :542-597 (the default, non-isTest branch: decodeMissing) */
static int decode_decoupled_plane(orc_clay *c, arena_t *ar, uint8_t **plane, const int *erased, int ne) {
    int n = c->n, nulls = 0;
    uint8_t *arr[256];
    uint8_t present[256];
    for (int i = 0; i < n; i++)
        if (plane[i] == NULL) nulls++;
    if (nulls > ne) return ORC_E_INDEX; /* tmpOutputs[r++] overflow (:556-562) */
    for (int i = 0; i < n; i++) arr[i] = plane[i] ? plane[i] : arena_zero(ar);
    for (int i = 0; i < n; i++) present[i] = 1;
    for (int i = 0; i < ne; i++)
        if (erased[i] < n) present[erased[i]] = 0;
    int st = orc_rs_decode_missing(c->rs, arr, present, n, ar->size, 0, ar->size);
    if (st) return st;
    for (int i = 0; i < ne; i++) plane[erased[i]] = arr[erased[i]];
    for (int i = 0; i < n; i++)
        if (plane[i] == NULL) return ORC_E_NULL; /* decoupledPlane[i].position(...) on a null */
    return ORC_OK;
}

/* decodeDecoupledPlane :542-597 with -DisTest=true on a single repair (isSingle), the branch
 * of :571-581: after the same tmpOutputs / getShardPresent / getByteArray preamble (:548-567),
 * for i = 0 .. n-|E|-1: rsRawDecoder.decodeMissingSingle(decoupledPlaneAsBytes[i + |E|],
 * i + |E|, i, shardPresent, outputs, 0, bufSize, i == 0) into the fresh byte[|E|][bufSize]
 * `outputs` (:569), then decoupledPlaneAsBytes[erasedIndexes[i]] = outputs[i] (:579-581).
 * It takes shard i + |E| as the i-th present one (bug B2); a missing parity shard has no
 * matrix row, the reference's NullPointerException (B3, orc_rs_decode_missing_single). */
static int decode_decoupled_plane_is_test(orc_clay *c, arena_t *ar, uint8_t **plane, const int *erased, int ne) {
    int n = c->n, nulls = 0;
    uint8_t *arr[256], *outs[64];
    uint8_t present[256];
    for (int i = 0; i < n; i++)
        if (plane[i] == NULL) nulls++;
    if (nulls > ne) return ORC_E_INDEX; /* tmpOutputs[r++] overflow (:556-562) */
    if (ne > 64) return ORC_E_INDEX;
    for (int i = 0; i < n; i++) arr[i] = plane[i] ? plane[i] : arena_zero(ar); /* getByteArray :599-609 */
    for (int i = 0; i < n; i++) present[i] = 1;
    for (int i = 0; i < ne; i++)
        if (erased[i] < n) present[erased[i]] = 0;
    for (int j = 0; j < ne; j++) outs[j] = arena_zero(ar); /* new byte[erasedIndexes.length][bufSize] */
    for (int i = 0; i < n - ne; i++) {
        int st = orc_rs_decode_missing_single(c->rs, arr[i + ne], i + ne, i, present, outs, ne, 0, ar->size, i == 0);
        if (st) return st;
    }
    for (int j = 0; j < ne; j++) plane[erased[j]] = outs[j];
    return ORC_OK;
}

/* getDecoupledHelperPlane :435-492.  helper[hp*n + node] */
static int decoupled_helper_plane(orc_clay *c, arena_t *ar, uint8_t *const *helper, const int *hidx, int nh,
                                  int hp, int erased, uint8_t **temp) {
    int z = hidx[hp], v[64];
    z_vector(c, z, v);
    int ey = node_y(c, erased);
    for (int i = 0; i < c->q * c->t; i++) {
        int x = node_x(c, i), y = node_y(c, i);
        if (y == ey) continue;
        if (v[y] == x) {
            temp[i] = helper[hp * c->n + i];
        } else {
            int cz = couple_plane(c, x, y, z), chp = 0;
            for (int j = 0; j < nh; j++)
                if (hidx[j] == cz) { chp = j; break; }
            int cc = node_index(c, v[y], y);
            uint8_t *in[4] = {helper[hp * c->n + i], helper[chp * c->n + cc], NULL, NULL};
            if (in[0] == NULL || in[1] == NULL) return ORC_E_INDEX; /* 3 nulls -> lostCouples overflow */
            uint8_t *o0;
            int st = pairwise(c, ar, in, &o0, NULL);
            if (st) return st;
            temp[i] = arena_clone(ar, o0);
        }
    }
    return ORC_OK;
}

/* The per-helper-plane body shared by both doDecodeSingle overloads
 * (:171-203 and :255-281): decouple, RS-decode the erased column, emit U(z,e)
 * and re-couple C(z',e) through each column mate. */
static int decode_single_plane(orc_clay *c, arena_t *ar, uint8_t *const *helper, const int *hidx, int nh, int i,
                               int erased, uint8_t *const *outputs /* [alpha][1] */) {
    int n = c->n, y = node_y(c, erased), z = hidx[i];
    int column[64];
    for (int x = 0; x < c->q; x++) column[x] = node_index(c, x, y);
    uint8_t *plane[256];
    for (int j = 0; j < n; j++) plane[j] = NULL;
    int st = decoupled_helper_plane(c, ar, helper, hidx, nh, i, erased, plane);
    if (st) return st;
    st = c->is_test ? decode_decoupled_plane_is_test(c, ar, plane, column, c->q)
                    : decode_decoupled_plane(c, ar, plane, column, c->q);
    if (st) return st;
    for (int x = 0; x < c->q; x++) {
        int node = node_index(c, x, y);
        if (node == erased) {
            memcpy(outputs[z], plane[node], (size_t)ar->size);
        } else {
            int cz = couple_plane(c, x, y, z);
            uint8_t *in[4] = {NULL, helper[i * n + node], NULL, plane[node]};
            if (in[1] == NULL) return ORC_E_INDEX;
            uint8_t *o0;
            st = pairwise(c, ar, in, &o0, NULL);
            if (st) return st;
            memcpy(outputs[cz], o0, (size_t)ar->size);
        }
    }
    return ORC_OK;
}

/* doDecodeSingle overload 1 (:118-221).  in[z*n + node]. */
static int do_decode_single(orc_clay *c, arena_t *ar, uint8_t *const *in, uint8_t *const *outputs, int erased) {
    int hidx[4096];
    int nh = orc_clay_helper_planes(c, erased, hidx);
    if (nh < 0) return nh;
    uint8_t **helper = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)nh * c->n);
    for (int h = 0; h < nh; h++) /* getHelperPlanes :291-300 */
        for (int j = 0; j < c->n; j++) helper[h * c->n + j] = in[hidx[h] * c->n + j];
    int st = ORC_OK;
    for (int i = 0; i < nh && !st; i++) st = decode_single_plane(c, ar, helper, hidx, nh, i, erased, outputs);
    free(helper);
    return st;
}

/* doDecodeMulti (:311-421).  `in` is the caller's n*alpha array; the Java code
 * writes decoded planes back into its local newIn[][] -- a private copy here. */
static int do_decode_multi(orc_clay *c, arena_t *ar, uint8_t *const *in_flat, uint8_t *const *outputs) {
    int n = c->n, a = c->alpha, ne = c->n_erased;
    uint8_t **in = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)n * a);
    for (int i = 0; i < n * a; i++) in[i] = in_flat[i];
    int max_is = 0;
    for (int z = 0; z < a; z++) {
        int s = intersection_score(c, z);
        if (s > max_is) max_is = s;
    }
    int *zs = (int *)malloc(sizeof(int) * a);
    uint8_t **temp = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)a * n);
    int st = ORC_OK;
    for (int is = 0; is <= max_is && !st; ++is) {
        int nz = 0;
        for (int z = 0; z < a; z++) /* getAllIntersectionScores :824-839, ascending z */
            if (intersection_score(c, z) == is) zs[nz++] = z;
        if (nz == 0) continue;
        for (int j = 0; j < nz && !st; j++) {
            int z = zs[j], v[64];
            uint8_t **tp = temp + (size_t)j * n;
            z_vector(c, z, v);
            for (int i = 0; i < n; i++) { /* getDecoupledPlane :500-534 */
                int x = node_x(c, i), y = node_y(c, i);
                if (in[z * n + i] != NULL) {
                    if (v[y] == x) {
                        tp[i] = in[z * n + i];
                    } else {
                        int cz = couple_plane(c, x, y, z), cc = node_index(c, v[y], y);
                        uint8_t *p4[4] = {in[z * n + i], in[cz * n + cc], NULL, NULL};
                        if (p4[1] == NULL) { st = ORC_E_INDEX; break; }
                        uint8_t *o0;
                        st = pairwise(c, ar, p4, &o0, NULL);
                        if (st) break;
                        tp[i] = arena_clone(ar, o0);
                    }
                } else {
                    tp[i] = NULL;
                }
            }
            if (!st) st = decode_decoupled_plane(c, ar, tp, c->erased, ne);
        }
        for (int j = 0; j < nz && !st; j++) {
            int z = zs[j];
            uint8_t **tp = temp + (size_t)j * n;
            for (int kk = 0; kk < ne && !st; kk++) {
                int e = c->erased[kk];
                int type = erasure_type(c, e, z);
                if (type == 0) {
                    in[z * n + e] = tp[e];
                    memcpy(outputs[z * ne + kk], tp[e], (size_t)ar->size);
                } else {
                    int v[64];
                    z_vector(c, z, v);
                    int ex = node_x(c, e), ey = node_y(c, e);
                    int cz = couple_plane(c, ex, ey, z);
                    int cidx = node_index(c, v[ey], ey);
                    uint8_t *o0;
                    if (type == 1) {
                        uint8_t *p4[4] = {NULL, in[cz * n + cidx], tp[e], NULL};
                        if (p4[1] == NULL) { st = ORC_E_INDEX; break; }
                        st = pairwise(c, ar, p4, &o0, NULL);
                    } else {
                        int tci = -1; /* realZIndexes.indexOf(couplePlaneIndex) */
                        for (int jj = 0; jj < nz; jj++)
                            if (zs[jj] == cz) { tci = jj; break; }
                        if (tci < 0) { st = ORC_E_INDEX; break; }
                        uint8_t *p4[4] = {NULL, NULL, tp[e], temp[(size_t)tci * n + cidx]};
                        st = pairwise(c, ar, p4, &o0, NULL);
                    }
                    if (st) break;
                    in[z * n + e] = arena_clone(ar, o0);
                    memcpy(outputs[z * ne + kk], o0, (size_t)ar->size);
                }
            }
        }
    }
    free(zs);
    free(temp);
    free(in);
    return st;
}

/* performCoding(ByteBuffer[],ByteBuffer[]) :64-107 */
int orc_clay_perform_coding(orc_clay *c, uint8_t *const *inputs, uint8_t *const *outputs, int buf_size) {
    if (c->n_erased == 0) return ORC_OK;
    int any = 0;
    for (int i = 0; i < c->n * c->alpha; i++)
        if (inputs[i]) { any = 1; break; }
    if (!any) return ORC_E_ILLEGAL_ARGUMENT; /* findFirstValidInput :712-721 */
    arena_t ar = {0};
    ar.size = buf_size;
    int st;
    if (c->n_erased == 1) {
        /* doDecodeSingle writes outputs[z][0] */
        st = do_decode_single(c, &ar, inputs, outputs, c->erased[0]);
    } else {
        st = do_decode_multi(c, &ar, inputs, outputs);
    }
    arena_free(&ar);
    return st;
}

/* doDecodeSingle overload 2 (:225-282), as driven by ClayCodeHelper.kt:34-53 */
int orc_clay_decode_single_helper(orc_clay *c, uint8_t *const *helper_coupled, int helper_i,
                                  uint8_t *const *outputs, int erased_index, int buf_size) {
    int hidx[4096];
    int nh = orc_clay_helper_planes(c, erased_index, hidx);
    if (nh < 0) return nh;
    if (helper_i < 0 || helper_i >= nh) return ORC_E_INDEX;
    arena_t ar = {0};
    ar.size = buf_size;
    int st = decode_single_plane(c, &ar, helper_coupled, hidx, nh, helper_i, erased_index, outputs);
    arena_free(&ar);
    return st;
}

/* ClayCode.getInputs, ClayCode.java:47-77: one Random(123456); data sub-chunk
 * k (flat, plane-major) iff k % n < numDataUnits, filled by nextBytes in k order. */
int orc_clay_get_inputs(int data_units, int parity_units, int block_size, uint8_t *flat, uint8_t *present) {
    int n = data_units + parity_units;
    int t = n / parity_units;
    int alpha = ipow(parity_units, t);
    orc_jrandom r;
    orc_jrandom_init(&r, 123456);
    int counter = 0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < alpha; j++) {
            int k = i * alpha + j;
            if (counter < data_units) {
                orc_jrandom_next_bytes(&r, flat + (size_t)k * block_size, block_size);
                present[k] = 1;
            } else {
                memset(flat + (size_t)k * block_size, 0, (size_t)block_size);
                present[k] = 0;
            }
            counter = (counter + 1) % n;
        }
    return ORC_OK;
}
