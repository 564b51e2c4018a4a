/*
 * ecx.h -- C ABI of the MI355X GF(256) erasure engine (libecx.so).
 *
 * This is the drop-in boundary for the reference's coding path
 * (krishnarb3/repair-pipelining, rs/ + clay/ + lrc/).  Every entry point
 * names the reference interface it replaces (file:line; file legend in
 * SURVEY.md section 0.1).  A JVM binding (JNI) maps byte[] / ByteBuffer onto
 * these plain pointers; see INTEGRATION.md.
 *
 * Conventions
 *   - Every function returns int: 0 (ECX_OK) or a non-negative result on
 *     success, a negative ECX_E_* code where the Java code throws.
 *     ecx_last_error() gives the thread-local message.
 *   - "Host" (per-call) entry points take caller-owned host buffers (the Java
 *     byte[][] of the reference).  Above the per-call crossover (ecx_tune.h
 *     "host_exec_kib", default 1 MiB per shard / sub-chunk, measured with 1 and
 *     16 caller threads) the bytes are staged to HBM, one fused kernel applies
 *     the composed GF(256) map and the results are copied back; at or below it
 *     the calling thread applies the same map (AVX-512 GFNI / AVX2, host_exec.cpp),
 *     which is faster than a PCIe round trip there.  That is a latency path of a
 *     device-backed library, not a fallback: without a usable HIP device every
 *     such call returns ECX_E_DEVICE, whatever its size.
 *   - "Batch" entry points take DEVICE pointers (HBM-resident stripes) and a
 *     hipStream_t passed as void*; they only enqueue work.  For the many-stream
 *     RS / LRC-encode maps on batches of >= 256 MiB of input, the first calls of a
 *     new layout time the candidate launch shapes with events on that stream (read
 *     later without blocking) and keep the fastest; every shape writes the same bytes
 *     (ecx_tune.h "layout_select").
 *   - Byte order / layout: a shard or sub-chunk is `byte_count` contiguous
 *     bytes.  Clay stripes are plane-major as in the reference
 *     (ClayCodeErasureDecodingStep.java:84-97): input slot z*n + node,
 *     output slot z*|E| + j.
 *   - Thread safety: all entry points may be called concurrently; codec
 *     objects are immutable after creation except for their internal,
 *     lock-protected map cache.
 */
#ifndef ECX_H
#define ECX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- status */
enum ecx_status {
    ECX_OK = 0,
    ECX_E_ILLEGAL_ARGUMENT = -1,  /* IllegalArgumentException (sizes, offsets, counts)  */
    ECX_E_NOT_ENOUGH_SHARDS = -2, /* "Not enough shards present"  ReedSolomon.java:211-213 */
    ECX_E_SINGULAR = -3,          /* "Matrix is singular"          Matrix.java:311-313      */
    ECX_E_TOO_MANY_SHARDS = -4,   /* "too many shards - max is 256" ReedSolomon.java:48-50  */
    ECX_E_INDEX = -5,             /* ArrayIndexOutOfBoundsException (e.g. Clay (k+m)%m!=0) */
    ECX_E_NULL = -6,              /* NullPointerException (decodeMissingSingle, bug B3)    */
    ECX_E_NOMEM = -7,             /* host or device allocation failed                      */
    ECX_E_DEVICE = -10            /* no HIP device / HIP runtime error                     */
};

const char *ecx_status_string(int status);
const char *ecx_last_error(void);
int ecx_version(void);

/* ---------------------------------------------------------------- device */
int ecx_device_count(int *count);
int ecx_set_device(int device);     /* per calling thread */
int ecx_synchronize(void *stream);  /* hipStreamSynchronize(stream) */

/* ---------------------------------------------------------------- Galois.java (host planner) */
int ecx_gf_multiply(int a, int b);               /* Galois.multiply  Galois.java:199-209 */
int ecx_gf_divide(int a, int b);                 /* Galois.divide    Galois.java:214-228 */
int ecx_gf_exp(int a, int n);                    /* Galois.exp       Galois.java:239-254 */
int ecx_gf_tables(int16_t *log_table /*256*/, uint8_t *exp_table /*510*/,
                  uint8_t *mul_table /*65536*/); /* Galois.java:59,103,178 */

/* ---------------------------------------------------------------- Matrix.java (host planner) */
int ecx_matrix_times(const uint8_t *a, int a_rows, int a_cols, const uint8_t *b, int b_rows, int b_cols,
                     uint8_t *out);                              /* Matrix.times   Matrix.java:193-210 */
int ecx_matrix_invert(const uint8_t *m, int n, uint8_t *out);   /* Matrix.invert  Matrix.java:273-346 */

/* ---------------------------------------------------------------- CodingLoop.java (host, GPU-executed) */
/* CodingLoop.codeSomeShards (CodingLoop.java:79-85; default implementation
 * InputOutputByteTableCodingLoop.java:12-44): outputs[o][offset..+byte_count) =
 * sum_i matrix_rows[o*input_count + i] * inputs[i][...].  Outputs are overwritten. */
int ecx_code_some_shards(const uint8_t *matrix_rows, const uint8_t *const *inputs, int input_count,
                         uint8_t *const *outputs, int output_count, int offset, int byte_count);
/* CodingLoop.checkSomeShards (CodingLoop.java:110-117): 1 if to_check equals the
 * coded outputs, 0 otherwise.  temp_buffer is accepted for signature parity and unused. */
int ecx_check_some_shards(const uint8_t *matrix_rows, const uint8_t *const *inputs, int input_count,
                          const uint8_t *const *to_check, int check_count, int offset, int byte_count,
                          uint8_t *temp_buffer);
/* InputOutputByteTableCodingLoopSingle.codeSomeShards (…Single.java:4-20):
 * output (=, or ^= when !is_first_time) matrix_rows[output_index*row_length + index] * input. */
int ecx_code_single(const uint8_t *matrix_rows, int row_length, const uint8_t *input, int index,
                    uint8_t *output, int output_index, int offset, int byte_count, int is_first_time);

/* ---------------------------------------------------------------- ReedSolomon.java */
typedef struct ecx_rs ecx_rs;
/* Codec objects: equal codecs (same k, m -- for Clay also virtual nodes and erased list)
 * are one shared, reference-counted object, so per-file / per-repair creates reuse the
 * compiled device plans.  Every create must be paired with one destroy; the last destroy
 * parks the codec in a bounded cache of 64 idle codecs, and one evicted from it frees its
 * device state.  Do not destroy a codec while batch work enqueued with it is in flight. */
int ecx_rs_create(int data_shards, int parity_shards, ecx_rs **out); /* ReedSolomon.create :34-61 */
void ecx_rs_destroy(ecx_rs *rs);
int ecx_rs_matrix(const ecx_rs *rs, uint8_t *out /* total x data */); /* buildMatrix :373-385 */
/* getDataShardCount / getParityShardCount (ReedSolomon.java:63-75); bindings size their
 * argument checks with it (the JNI shim's checkBuffersAndSizes, :338-363). */
int ecx_rs_shape(const ecx_rs *rs, int *data_shards, int *parity_shards);
int ecx_rs_encode_parity(ecx_rs *rs, uint8_t *const *shards, int shard_count, int shard_length, int offset,
                         int byte_count);                            /* encodeParity :94-108 */
int ecx_rs_encode_parity_single(ecx_rs *rs, const uint8_t *shard, uint8_t *output, int input_index,
                                int output_index, int offset, int byte_count); /* :110-118 */
int ecx_rs_is_parity_correct(ecx_rs *rs, uint8_t *const *shards, int shard_count, int shard_length,
                             int first_byte, int byte_count, uint8_t *temp_buffer,
                             int temp_length);                       /* isParityCorrect :129-178 */
int ecx_rs_decode_missing(ecx_rs *rs, uint8_t *const *shards, const uint8_t *shard_present, int shard_count,
                          int shard_length, int offset, int byte_count); /* decodeMissing :189-286 */
/* decodeMissingSingle :288-333.  outputs[j] are caller arrays written in place
 * (assigned when is_first, XOR-accumulated otherwise). */
int ecx_rs_decode_missing_single(ecx_rs *rs, const uint8_t *shard, int shard_index, int index,
                                 const uint8_t *shard_present, uint8_t *const *outputs, int output_count,
                                 int offset, int byte_count, int is_first);

/* ---------------------------------------------------------------- compiled GF maps (device batch) */
/* An ecx_map is one composed GF(256) linear map (a code + erasure pattern),
 * compiled into the kernel's table format and resident on the device.
 * Batch layout: input slot j of stripe s is at in + s*in_stripe_stride + in_slot[j]*in_slot_stride;
 * output row o goes to out + s*out_stripe_stride + out_slot[o]*out_slot_stride. */
typedef struct ecx_map ecx_map;
int ecx_map_create(const uint8_t *matrix /* n_out x n_in */, int n_out, int n_in, const int *in_slot,
                   const int *out_slot, ecx_map **out);
void ecx_map_destroy(ecx_map *map);
int ecx_map_info(const ecx_map *map, int *n_out, int *n_in, int *nnz);
int ecx_map_matrix(const ecx_map *map, uint8_t *matrix /* n_out x n_in */, int *in_slot, int *out_slot);
/* Largest input and output slot index the map reads / writes (-1 = none).  A batch over
 * nstripes stripes of byte_count bytes touches (nstripes-1)*stripe_stride +
 * max_slot*slot_stride + byte_count bytes of each buffer: the extent a binding checks
 * against the caller's buffer (a Java ByteBuffer's capacity) before any device work. */
int ecx_map_slot_extent(const ecx_map *map, int *max_in_slot, int *max_out_slot);
int ecx_map_apply_batch(const ecx_map *map, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                        uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                        int64_t byte_count, void *stream);

/* ReedSolomon.encodeParity (ReedSolomon.java:94-108) over nstripes device-resident
 * stripes, in place: stripe s's shard i is base + s*stripe_stride + i*shard_stride; the
 * parity shards k..n-1 are overwritten for bytes [offset, offset + byte_count). */
int ecx_rs_encode_parity_batch(ecx_rs *rs, uint8_t *base, int64_t stripe_stride, int64_t shard_stride,
                               int64_t nstripes, int64_t offset, int64_t byte_count, void *stream);
/* ReedSolomon.isParityCorrect (ReedSolomon.java:129-178; the "Check" half of
 * ReedSolomonBenchmark.java:73-87,126-149) over nstripes device-resident stripes (same layout
 * as ecx_rs_encode_parity_batch), read-only: verdict[s] (a device byte array of nstripes) is
 * set to 1 when every parity shard of stripe s equals the parity of its data over bytes
 * [offset, offset + byte_count), else 0.  Nothing is written to the shards. */
int ecx_rs_is_parity_correct_batch(ecx_rs *rs, const uint8_t *base, int64_t stripe_stride, int64_t shard_stride,
                                   int64_t nstripes, int64_t offset, int64_t byte_count, uint8_t *verdict,
                                   void *stream);
/* ReedSolomon.decodeMissing (ReedSolomon.java:189-286) over nstripes device-resident
 * stripes, in place (same layout): every shard with shard_present[i] == 0 is rebuilt,
 * data from the first k present shards (ascending index), parity from all data -- the
 * reference's map exactly.  Fewer than k present: ECX_E_NOT_ENOUGH_SHARDS. */
int ecx_rs_decode_missing_batch(ecx_rs *rs, const uint8_t *shard_present, uint8_t *base, int64_t stripe_stride,
                                int64_t shard_stride, int64_t nstripes, int64_t offset, int64_t byte_count,
                                void *stream);

/* The engine's layout contract for RS batches in HBM (the reference
 * keeps every shard in its own byte[], ReedSolomonBenchmark.java:198, so the device layout
 * is the caller's choice).  BLOCKED layout of nstripes stripes of n = k + m shards of
 * byte_count bytes, in block_bytes blocks (full = byte_count / block_bytes, tail = the rest):
 *   body  [nstripes][full][n][block_bytes] at base -- a stripe block-major, the way Clay
 *         stores its sub-chunks plane-major (ClayCodeErasureDecodingStep.java:84-97);
 *   tails [nstripes][n][tail] at base + nstripes * full * n * block_bytes.
 * It occupies exactly nstripes * n * byte_count bytes.  Measured against the natural
 * back-to-back shards (scripts/rs_layout_contract.py): RS(17,3) encodeParity on 200,000-B
 * shards 0.695 -> 0.760 of HBM (32 KiB blocks), RS(12,4) 2-erasure decode on 4 MiB shards
 * 0.754 -> 0.816 (64 KiB blocks).
 * ecx_rs_blocked_layout fills layout[3] = {block_bytes, full, tail} for RS(k, m) and a shard
 * size: the largest power of two with n blocks within 1 MiB (4 KiB..1 MiB), or one block of
 * byte_count bytes below that. */
int ecx_rs_blocked_layout(int data_shards, int parity_shards, int64_t byte_count, int64_t *layout);
/* The recommended shard pitch of the plain [stripe][shard][pitch] layout when the caller cannot
 * block: the smallest odd multiple of 4 KiB >= byte_count (RS(12,4) 4 MiB: 0.754 -> 0.789;
 * RS(17,3) 200,000 B: 0.695 -> 0.718). */
int ecx_rs_recommended_pitch(int data_shards, int parity_shards, int64_t byte_count, int64_t *pitch);
/* ecx_rs_encode_parity_batch over the blocked layout (block_bytes > 0; 0 = the recommended
 * block), in place: two launches, the full blocks and the tails, on `stream`. */
int ecx_rs_encode_parity_blocked_batch(ecx_rs *rs, uint8_t *base, int64_t nstripes, int64_t byte_count,
                                       int64_t block_bytes, void *stream);
/* ecx_rs_decode_missing_batch over the blocked layout, in place (the same map). */
int ecx_rs_decode_missing_blocked_batch(ecx_rs *rs, const uint8_t *shard_present, uint8_t *base, int64_t nstripes,
                                        int64_t byte_count, int64_t block_bytes, void *stream);

/* The same two blocked batches (encodeParity / decodeMissing, ReedSolomon.java:94-108, :189-286)
 * from HOST memory, in place (base: nstripes * n * byte_count bytes of
 * pageable or pinned host memory in the blocked layout): the full blocks, then the tails, each a
 * pipelined host batch (H2D -> map -> D2H of the written shards only, as ecx_map_apply_batch_host).
 * Synchronous; a caller that keeps its stripes blocked on the host feeds the device the layout
 * the kernels run fastest on without an unpacking pass. */
int ecx_rs_encode_parity_blocked_batch_host(ecx_rs *rs, uint8_t *base, int64_t nstripes, int64_t byte_count,
                                            int64_t block_bytes);
int ecx_rs_decode_missing_blocked_batch_host(ecx_rs *rs, const uint8_t *shard_present, uint8_t *base,
                                             int64_t nstripes, int64_t byte_count, int64_t block_bytes);
/* The same over several GPUs of this process: each of the two passes is split over the device
 * entries as ecx_map_apply_batch_host_devices splits a batch -- the full blocks as nstripes * full
 * small stripes, the tails by stripes (by byte ranges when there are fewer than entries). */
int ecx_rs_encode_parity_blocked_batch_host_devices(ecx_rs *rs, uint8_t *base, int64_t nstripes, int64_t byte_count,
                                                    int64_t block_bytes, const int *devices, int ndev);
int ecx_rs_decode_missing_blocked_batch_host_devices(ecx_rs *rs, const uint8_t *shard_present, uint8_t *base,
                                                     int64_t nstripes, int64_t byte_count, int64_t block_bytes,
                                                     const int *devices, int ndev);

/* As ecx_map_apply_batch, but XOR-accumulates: out ^= M * in. */
int ecx_map_accumulate_batch(const ecx_map *map, const uint8_t *in, int64_t in_stripe_stride,
                             int64_t in_slot_stride, uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride,
                             int64_t nstripes, int64_t byte_count, void *stream);

/* Maps of the codec entry points (owned by the codec; do not destroy). */
int ecx_rs_encode_map(ecx_rs *rs, const ecx_map **out);              /* encodeParity, slots = shard index */
int ecx_rs_decode_map(ecx_rs *rs, const uint8_t *shard_present, const ecx_map **out); /* decodeMissing */

/* ---------------------------------------------------------------- batched partial sums (repair pipelining) */
/* Batched ReedSolomon.decodeMissingSingle (ReedSolomon.java:288-333) as used along the
 * pipelined chain (ClayCodeNode.kt:182-186, :225-228): one helper's contribution to EVERY
 * missing shard, over nstripes stripes: acc[s][o] (=, or ^= unless is_first)
 * D[o][shard_index] * in[s], with o over the missing shards in ascending index order.
 * Unlike the reference (bug B3) the rows include missing PARITY shards (the composed
 * decodeMissing map), so a parity-node repair can be pipelined too.  A present shard that
 * is not among the first k present contributes zero (the reference's first-k rule). */
int ecx_rs_decode_partial_batch(ecx_rs *rs, const uint8_t *shard_present, int shard_index, const uint8_t *in,
                                int64_t in_stripe_stride, uint8_t *acc, int64_t acc_stripe_stride,
                                int64_t acc_row_stride, int64_t nstripes, int64_t byte_count, int is_first,
                                void *stream);
/* Batched ReedSolomon.encodeParitySingle (ReedSolomon.java:110-118; LRC chains,
 * NodeHelper.kt:89): acc[s][p] (=, or ^= unless is_first) parityRows[p][input_index] * in[s]
 * for every parity row p. */
int ecx_rs_encode_partial_batch(ecx_rs *rs, int input_index, const uint8_t *in, int64_t in_stripe_stride,
                                uint8_t *acc, int64_t acc_stripe_stride, int64_t acc_row_stride, int64_t nstripes,
                                int64_t byte_count, int is_first, void *stream);

/* ---------------------------------------------------------------- ClayCodeErasureDecodingStep.java */
typedef struct ecx_clay ecx_clay;
/* new ClayCodeErasureDecodingStep(erasedIndexes, RS(2,2), RS(k,m)) -- ClayCode.java:28-41, :43-51 */
int ecx_clay_create(int data_units, int parity_units, const int *erased, int n_erased, ecx_clay **out);
/* Shortened Clay: Clay(data+virtual, parity) whose data nodes
 * [data, data+virtual) are virtual all-zero nodes, e.g. Clay(10,4) = Clay(12,4)
 * with 2 virtual nodes (the reference's integer t = (k+m)/m cannot build
 * Clay(10,4), ClayCodeErasureDecodingStep.java:692).  Every slot index, erased
 * index and geometry query then refers to the data+parity REAL nodes; the
 * results equal the reference Clay(12,4) run with the virtual nodes zero-filled. */
int ecx_clay_create_shortened(int data_units, int parity_units, int virtual_units, const int *erased, int n_erased,
                              ecx_clay **out);
/* ecx_clay_create_shortened with flags.  ECX_CLAY_IS_TEST: the single-node repair's plane
 * decode takes decodeDecoupledPlane's -DisTest=true branch (ClayCodeErasureDecodingStep.java:
 * 571-581): decodeMissingSingle per helper, assuming the erased row is nodes 0..q-1 (bug B2).
 * For the other rows it computes the reference's (different) map, and where that row holds a
 * parity node the reference throws NullPointerException (B3): ECX_E_NULL from performCoding.
 * Multi-erasure decodes (and encode) are unaffected, as in the reference. */
enum { ECX_CLAY_IS_TEST = 1 };
int ecx_clay_create_ex(int data_units, int parity_units, int virtual_units, const int *erased, int n_erased, int flags,
                       ecx_clay **out);
void ecx_clay_destroy(ecx_clay *clay); /* drops one reference (see ecx_rs_create) */
int ecx_clay_geometry(const ecx_clay *clay, int *q, int *t, int *alpha); /* ClayCodeUtil :690-695 */
int ecx_clay_helper_planes(const ecx_clay *clay, int erased_index, int *out /* alpha */); /* :924-941 */
/* The step's real node count n (= data + parity; virtual nodes excluded), its number of
 * erased nodes and alpha: performCoding takes n*alpha inputs and n_erased*alpha outputs
 * (the "Invalid inputs/outputs length" checks, ClayCodeErasureDecodingStep.java:76-82). */
int ecx_clay_shape(const ecx_clay *clay, int *nodes, int *n_erased, int *alpha);
/* performCoding(ECChunk[],ECChunk[]) -- ClayCodeErasureDecodingStep.java:53-107.
 * inputs: n*alpha host pointers, NULL = absent; outputs: n_erased*alpha host pointers. */
int ecx_clay_perform_coding(ecx_clay *clay, const uint8_t *const *inputs, uint8_t *const *outputs, int buf_size);
/* doDecodeSingle overload 2 (:225-282), as driven per helper plane by
 * ClayCodeHelper.getHelperPlanesAndDecode (ClayCodeHelper.kt:19-56).
 * helper_coupled: [num_helper_planes][n] host pointers; outputs: alpha host pointers. */
int ecx_clay_decode_single_helper(ecx_clay *clay, const uint8_t *const *helper_coupled, int helper_i,
                                  uint8_t *const *outputs, int erased_index, int buf_size);
/* The composed performCoding map for the standard null pattern (erased nodes
 * absent, every other sub-chunk present): input slot z*n+node, output slot z*|E|+j. */
int ecx_clay_map(ecx_clay *clay, const ecx_map **out);
/* Batched device-resident performCoding over nstripes stripes: stripe s holds
 * n*alpha sub-chunks of buf_size bytes at in + s*in_stripe_stride + slot*in_sub_stride
 * and receives |E|*alpha sub-chunks at out + s*out_stripe_stride + slot*out_sub_stride. */
int ecx_clay_perform_coding_batch(ecx_clay *clay, const uint8_t *in, int64_t in_stripe_stride,
                                  int64_t in_sub_stride, uint8_t *out, int64_t out_stripe_stride,
                                  int64_t out_sub_stride, int64_t nstripes, int64_t buf_size, void *stream);

/* ---------------------------------------------------------------- LRC (device batch, in place) */
/* LRCErasureCode.kt:5-9 / LRCErasureUtil.kt:3-6: K=12 data blocks in local groups of
 * R=3, one RS(3,1) parity each (parity row [1,1,1], i.e. XOR), N=16 blocks in the
 * LRCErasureCodeExample.kt:48 order (group g = blocks 4g..4g+3, parity 4g+3).
 * Block b of stripe s is at stripes + s*stripe_stride + b*block_stride. */
/* The composed map: block_present == NULL -> encode, else decode (owned by the library). */
int ecx_lrc_map(const uint8_t *block_present /* 16 flags or NULL */, const ecx_map **out);
/* encode / encodeUsingSingle (LRCErasureCodeExample.kt:30-98): writes the 4 group parities. */
int ecx_lrc_encode_batch(uint8_t *stripes, int64_t stripe_stride, int64_t block_stride, int64_t nstripes,
                         int64_t block_size, void *stream);
/* decode (LRCErasureCodeExample.kt:100-131): rebuilds every non-present block from
 * its group (decodeMissing per group).  Two blocks missing in one group ->
 * ECX_E_NOT_ENOUGH_SHARDS, as RS(3,1).decodeMissing throws. */
int ecx_lrc_decode_batch(uint8_t *stripes, int64_t stripe_stride, int64_t block_stride,
                         const uint8_t *block_present /* 16 flags */, int64_t nstripes, int64_t block_size,
                         void *stream);

/* ---------------------------------------------------------------- host-memory batches */
/* The reference's repair starts and ends in host memory: helper sub-chunks arrive on
 * sockets into ByteBuffers (ClayCoordinator.kt:372-395) and leave the same way
 * (ClayCodeNode.kt:330-347).  A JNI shim hands over their addresses via
 * GetDirectBufferAddress (ECChunk.toBuffers, ECChunk.java:81-95).
 * These calls take the batch layouts above with HOST pointers.  Chunks of stripes are
 * pipelined H2D -> kernel -> D2H on internal streams, and only the map's used input
 * slots cross PCIe.  The calls are synchronous.  Pinned memory (ecx_host_alloc /
 * ecx_host_register) runs at the PCIe rate.  Outputs may point into the input stripes
 * (in-place decodeMissing) when no output slot is also an input slot. */
int ecx_map_apply_batch_host(const ecx_map *map, const uint8_t *in, int64_t in_stripe_stride,
                             int64_t in_slot_stride, uint8_t *out, int64_t out_stripe_stride,
                             int64_t out_slot_stride, int64_t nstripes, int64_t byte_count);
int ecx_clay_perform_coding_batch_host(ecx_clay *clay, const uint8_t *in, int64_t in_stripe_stride,
                                       int64_t in_sub_stride, uint8_t *out, int64_t out_stripe_stride,
                                       int64_t out_sub_stride, int64_t nstripes, int64_t buf_size);
/* The same over several GPUs of this process (one host thread, stream set and
 * buffer ring per GPU).  Device j of `devices` (ndev entries, HIP ordinals; repeats allowed)
 * takes the contiguous stripe range [j*S/ndev, (j+1)*S/ndev) (the remainder spread over the
 * first ranges, as shard_stripes), on a worker thread of its own; the call returns when every
 * worker has finished.  With fewer stripes than entries (one or two huge stripes) the entries
 * split the bytes of every slot instead, in 4 KiB units, so each still moves a share over its
 * own link.  An out-of-range device id or ndev <= 0 is refused
 * (ECX_E_ILLEGAL_ARGUMENT) before anything is copied; on a failure every device is drained and
 * the first failing device's status is returned.  The calling thread's current device is
 * unchanged. */
int ecx_map_apply_batch_host_devices(const ecx_map *map, const uint8_t *in, int64_t in_stripe_stride,
                                     int64_t in_slot_stride, uint8_t *out, int64_t out_stripe_stride,
                                     int64_t out_slot_stride, int64_t nstripes, int64_t byte_count,
                                     const int *devices, int ndev);
int ecx_clay_perform_coding_batch_host_devices(ecx_clay *clay, const uint8_t *in, int64_t in_stripe_stride,
                                               int64_t in_sub_stride, uint8_t *out, int64_t out_stripe_stride,
                                               int64_t out_sub_stride, int64_t nstripes, int64_t buf_size,
                                               const int *devices, int ndev);
/* ReedSolomon.isParityCorrect (ReedSolomon.java:129-178) over nstripes HOST-memory stripes
 * (the layout of ecx_rs_is_parity_correct_batch, host pointers): each chunk of stripes goes
 * H2D and through the read-only check kernel, and only the verdict bytes come back --
 * verdict[s] (a host byte array of nstripes) = 1 when stripe s's parity is correct over bytes
 * [offset, offset + byte_count), else 0.  Synchronous; the _devices form splits the stripes
 * over a device list as ecx_map_apply_batch_host_devices does; with fewer stripes than entries
 * each entry checks a byte range of every shard, and a stripe passes when every range does. */
int ecx_rs_is_parity_correct_batch_host(ecx_rs *rs, const uint8_t *base, int64_t stripe_stride,
                                        int64_t shard_stride, int64_t nstripes, int64_t offset,
                                        int64_t byte_count, uint8_t *verdict);
int ecx_rs_is_parity_correct_batch_host_devices(ecx_rs *rs, const uint8_t *base, int64_t stripe_stride,
                                                int64_t shard_stride, int64_t nstripes, int64_t offset,
                                                int64_t byte_count, uint8_t *verdict, const int *devices,
                                                int ndev);
/* Page-locked host memory for the calls above (e.g. backing direct ByteBuffers). */
int ecx_host_alloc(int64_t nbytes, void **out);
int ecx_host_free(void *ptr);
int ecx_host_register(void *ptr, int64_t nbytes);
int ecx_host_unregister(void *ptr);

/* ---------------------------------------------------------------- synthetic data / verification (device) */
/* Deterministic counter-based fill: byte i of the region = f(seed, i). */
int ecx_fill_random(uint8_t *dst, int64_t nbytes, uint64_t seed, void *stream);
/* Count bytes that differ between two strided sets of nrows rows of row_bytes each;
 * result accumulated into *d_count (device uint64). */
int ecx_count_mismatch(const uint8_t *a, int64_t a_stride, const uint8_t *b, int64_t b_stride, int64_t nrows,
                       int64_t row_bytes, uint64_t *d_count, void *stream);

#ifdef __cplusplus
}
#endif
#endif
