/*
 * ecx_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, byte-at-a-time restatement of the reference's JVM CPU path
 * (krishnarb3/repair-pipelining: rs/, clay/, lrc/).  It exists to CHECK the
 * HIP engine (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg)
 * and is never linked into, loaded by, or called from the product library
 * (repair-pipelining_amd/).  Every function names the reference file:line
 * it restates; the file legend is SURVEY.md section 0.1.
 *
 * Parity pinning: the GF(2^8) tables, Matrix and ReedSolomon layers are
 * pinned against the reference's own JUnit known-answer vectors
 * (GaloisTest.java, MatrixTest.java, ReedSolomonTest.java), see
 * tests/golden/ and tests/test_oracle_golden.py.  The Clay and LRC layers
 * have no reference test vectors; they are pinned by
 * faithful restatement over the KAT-pinned RS core plus self-consistency
 * (repair reproduces the erased node) and the survey's cross-check digests.
 *
 * Error convention: functions return 0 (or a boolean 0/1) on success and a
 * negative ORC_E_* code where the Java code throws.
 */
#ifndef ECX_ORACLE_H
#define ECX_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORC_OK = 0,
    ORC_E_ILLEGAL_ARGUMENT = -1,   /* IllegalArgumentException */
    ORC_E_NOT_ENOUGH_SHARDS = -2,  /* "Not enough shards present" */
    ORC_E_SINGULAR = -3,           /* "Matrix is singular" */
    ORC_E_TOO_MANY_SHARDS = -4,    /* "too many shards - max is 256" */
    ORC_E_INDEX = -5,              /* ArrayIndexOutOfBoundsException */
    ORC_E_NULL = -6,               /* NullPointerException */
    ORC_E_NOMEM = -7
};

/* ---- java.util.Random (public JDK specification) ---- */
typedef struct { uint64_t seed; } orc_jrandom;
void orc_jrandom_init(orc_jrandom *r, int64_t seed);
int32_t orc_jrandom_next_int(orc_jrandom *r);
int32_t orc_jrandom_next_int_bound(orc_jrandom *r, int32_t bound);
void orc_jrandom_next_bytes(orc_jrandom *r, uint8_t *out, int len);

/* ---- Galois.java ---- */
int orc_gen_log_table(int polynomial, int16_t out[256]);
void orc_gen_exp_table(const int16_t log_table[256], uint8_t out[510]);
const int16_t *orc_log_table(void);
const uint8_t *orc_exp_table(void);
const uint8_t *orc_mul_table(void); /* 256*256, [a][b] */
uint8_t orc_gf_multiply(uint8_t a, uint8_t b);
int orc_gf_divide(uint8_t a, uint8_t b); /* <0 on divide by zero */
uint8_t orc_gf_exp(uint8_t a, int n);
int orc_all_possible_polynomials(int *out /* >= 256 */);

/* ---- Matrix.java (row-major bytes) ---- */
int orc_matrix_times(const uint8_t *a, int ar, int ac, const uint8_t *b, int br, int bc, uint8_t *out);
int orc_matrix_invert(const uint8_t *m, int n, uint8_t *out);

/* ---- InputOutputByteTableCodingLoop.java / CodingLoopBase.java ---- */
void orc_code_some_shards(const uint8_t *const *matrix_rows, uint8_t *const *inputs, int input_count,
                          uint8_t *const *outputs, int output_count, int offset, int byte_count);
int orc_check_some_shards(const uint8_t *const *matrix_rows, uint8_t *const *inputs, int input_count,
                          uint8_t *const *to_check, int check_count, int offset, int byte_count,
                          uint8_t *temp_buffer);
void orc_code_single(const uint8_t *const *matrix_rows, const uint8_t *input, int index,
                     uint8_t *output, int output_index, int offset, int byte_count, int is_first_time);

/* ---- ReedSolomon.java ---- */
typedef struct orc_rs orc_rs;
int orc_rs_create(int data_shards, int parity_shards, orc_rs **out);
void orc_rs_free(orc_rs *rs);
int orc_rs_data_count(const orc_rs *rs);
int orc_rs_parity_count(const orc_rs *rs);
void orc_rs_matrix(const orc_rs *rs, uint8_t *out /* total x data */);
int orc_rs_encode_parity(orc_rs *rs, uint8_t *const *shards, int shard_count, int shard_len,
                         int offset, int byte_count);
int orc_rs_encode_parity_single(orc_rs *rs, const uint8_t *shard, uint8_t *output, int input_index,
                                int output_index, int offset, int byte_count);
int orc_rs_is_parity_correct(orc_rs *rs, uint8_t *const *shards, int shard_count, int shard_len,
                             int first_byte, int byte_count, uint8_t *temp_buffer, int temp_len);
int orc_rs_decode_missing(orc_rs *rs, uint8_t *const *shards, const uint8_t *shard_present,
                          int shard_count, int shard_len, int offset, int byte_count);
int orc_rs_decode_missing_single(orc_rs *rs, const uint8_t *shard, int shard_index, int index,
                                 const uint8_t *shard_present, uint8_t *const *outputs, int output_count,
                                 int offset, int byte_count, int is_first);

/* ---- ClayCodeErasureDecodingStep.java / ClayCode.java / ClayCodeHelper.kt ---- */
typedef struct orc_clay orc_clay;
int orc_clay_create(int data_units, int parity_units, const int *erased, int n_erased, orc_clay **out);
/* is_test != 0: the reference run with -DisTest=true (decodeDecoupledPlane :571-581 on single repairs) */
int orc_clay_create_ex(int data_units, int parity_units, const int *erased, int n_erased, int is_test,
                       orc_clay **out);
void orc_clay_free(orc_clay *c);
int orc_clay_q(const orc_clay *c);
int orc_clay_t(const orc_clay *c);
int orc_clay_alpha(const orc_clay *c);
int orc_clay_helper_planes(const orc_clay *c, int erased_index, int *out);
/* performCoding: inputs n*alpha plane-major (NULL = absent), outputs n_erased*alpha. */
int orc_clay_perform_coding(orc_clay *c, uint8_t *const *inputs, uint8_t *const *outputs, int buf_size);
/* doDecodeSingle overload 2: helper_coupled is [num_helper_planes][n] row-major. */
int orc_clay_decode_single_helper(orc_clay *c, uint8_t *const *helper_coupled, int helper_i,
                                  uint8_t *const *outputs /* alpha x 1 */, int erased_index, int buf_size);
/* ClayCode.getInputs: flat n*alpha*B buffer, present[] flags (data sub-chunks only). */
int orc_clay_get_inputs(int data_units, int parity_units, int block_size, uint8_t *flat, uint8_t *present);

/* orc_bench.c -- timing harness (bench.py cpu_baseline): `threads` workers, each with its
 * own Clay step object, repair `erased` on their own `per_thread` stripes for `seconds`.
 * stripes: [threads*per_thread][n*alpha] sub-chunk pointers (NULL = absent). */
enum { ORC_BENCH_CLAY = 0, ORC_BENCH_RS_DECODE = 1, ORC_BENCH_RS_ENCODE = 2, ORC_BENCH_RS_CHECK = 3 };
/* Generic form: `op` on units of `slots` pointers ([threads*per_thread][slots]): Clay
 * (data, parity, erased) repair of n*alpha sub-chunk pointers, or RS(data, parity)
 * decodeMissing (erased = the missing shards) / encodeParity over n shard pointers of
 * buf_size bytes, in place. */
int orc_bench_run(int op, int data, int parity, const int *erased, int n_erased, int buf_size,
                  uint8_t *const *units, int slots, int per_thread, int threads, double seconds, long long *reps,
                  double *elapsed);
int orc_bench_clay_repair(int data_units, int parity_units, int erased, int buf_size, uint8_t *const *stripes,
                          int per_thread, int threads, double seconds, long long *repairs, double *elapsed);

#ifdef __cplusplus
}
#endif
#endif
