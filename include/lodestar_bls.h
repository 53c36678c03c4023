/*
 * lodestar_bls.h — C ABI of the MI355X BLS12-381 signature-set verifier.
 *
 * This is the drop-in boundary for Lodestar's IBlsVerifier hot path
 * (SURVEY.md §8(b)).  Plain pointers and sizes only; no torch / HIP types.
 * Every entry point returns an lb_status code (0 = OK) and never throws.
 *
 * Reference interfaces each entry point replaces (paths under the reference repo):
 *   lb_verify_jobs / lb_batch_*   packages/beacon-node/src/chain/bls/multithread/worker.ts:32-108
 *                                 (verifyManySignatureSets: BlsWorkReq[] -> per-job results),
 *                                 packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39
 *                                 (verifySignatureSetsMaybeBatch) and the blst calls it makes
 *                                 (Signature.fromBytes(sig, affine, true), verifyMultipleSignatures,
 *                                 Signature.verify).
 *   lb_aggregate_pubkeys          packages/beacon-node/src/chain/bls/utils.ts:5-16
 *                                 (getAggregatedPubkey) + PublicKey.toBytes(uncompressed),
 *                                 packages/beacon-node/src/chain/bls/multithread/index.ts:126,160.
 *   lb_batch_partial /
 *   lb_fp12_product_is_one        the multi-GPU split of blst Pairing.commit()+finalverify()
 *                                 (SURVEY.md §8(e)): per-GPU Fp12 partial products, one
 *                                 final exponentiation over their product.
 *
 * Data formats (all ZCash BLS12-381 encodings, big-endian):
 *   pubkey      96 B uncompressed affine G1 (x || y), as the reference's main thread
 *               serialises it (PointFormat.uncompressed); infinity = 0x40 || 0^95.
 *   signing root 32 B (ISignatureSet.signingRoot).
 *   signature   96 B compressed G2 (ISignatureSet.signature).
 *   Fp12 partial 576 B: 12 Fp coefficients, tower order c0.c0.c0, c0.c0.c1, c0.c1.c0, ...
 *
 * Job results (int32 per job): 1 = valid, 0 = invalid, -code = the job rejects with
 * error `code` (lb_error_name(code) gives the blst error string the reference throws).
 */
#ifndef LODESTAR_BLS_H
#define LODESTAR_BLS_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status / error codes: blst BLST_ERROR values plus Lodestar's own errors */
#define LB_OK 0
#define LB_BAD_ENCODING 1
#define LB_POINT_NOT_ON_CURVE 2
#define LB_POINT_NOT_IN_GROUP 3
#define LB_AGGR_TYPE_MISMATCH 4
#define LB_VERIFY_FAIL 5
#define LB_PK_IS_INFINITY 6
#define LB_BAD_SCALAR 7
#define LB_INVALID_SIZE 10           /* "BLST_INVALID_SIZE" (multithread.test.ts:97) */
#define LB_EMPTY_AGGREGATE_ARRAY 11  /* bls.PublicKey.aggregate([]) */
#define LB_EMPTY_SIGNATURE_SET 12    /* "Empty signature set" (maybeBatch.ts:29-31) */
#define LB_ERR_ARGUMENT 100          /* bad C-ABI arguments (NULL, inconsistent offsets) */
#define LB_ERR_DEVICE 101            /* HIP runtime failure */
#define LB_ERR_NO_DEVICE 102         /* no usable gfx950 device */

typedef struct lb_engine lb_engine;
typedef struct lb_batch lb_batch;

/* Human-readable blst-style name for a status code ("BLST_INVALID_SIZE", ...). */
const char* lb_error_name(int32_t code);

/* ABI version (bumped on incompatible changes). */
int32_t lb_abi_version(void);

/*
 * One engine = one batch in flight on one GPU (own HIP streams and device workspaces); a process
 * may drive several engines per GPU concurrently (the reference runs one job package per worker
 * thread at a time, multithread/index.ts:290-381).  device < 0 = current.  Returns
 * LB_ERR_DEVICE once the per-device engine cap is reached (10, or LB_MAX_ENGINES_PER_DEVICE;
 * each engine's scratch for the largest private segment is reserved at creation, so an exhausted
 * pool fails here instead of aborting a queue later).
 */
int32_t lb_engine_create(int32_t device, lb_engine** out);
/*
 * The same with flags.  LB_ENGINE_LATENCY: the engine is the device's latency engine (the
 * reference's verifyOnMainThread path, multithread/index.ts:138-151): its streams run on a
 * reserved set of CUs (LB_LATENCY_CUS, default 8) and it always takes the small-batch latency
 * forms; engines created AFTER it on the device run on the remaining CUs, so a 1-set call does not
 * queue behind the pool's batches.  Create the latency engine first (engines created before it keep
 * every CU; a warning is printed).  The partition lasts while a latency engine exists: engines
 * created after the last one is destroyed get the whole device again.  CU-masked streams are
 * blocking streams (they synchronise with the legacy null stream).
 */
#define LB_ENGINE_LATENCY 1u
int32_t lb_engine_create_ex(int32_t device, uint32_t flags, lb_engine** out);
void lb_engine_destroy(lb_engine* e);
/* CUs the engine's streams may use: the device's count, the reserved CUs for a latency engine, or
 * the rest while a partition exists.  0 for NULL. */
int32_t lb_engine_cu_count(const lb_engine* e);

/*
 * Upload one batch of jobs into device memory (copies; the caller keeps its buffers).
 *   n_jobs        number of jobs (one job = one BlsWorkReq / one verifySignatureSets chunk)
 *   job_offsets   n_jobs+1 prefix sums over sets (job j = sets [job_offsets[j], job_offsets[j+1]))
 *   set_pk_offsets n_sets+1 prefix sums over pubkeys (set i aggregates pubkeys
 *                 [set_pk_offsets[i], set_pk_offsets[i+1]); a `single` set has exactly one)
 *   pubkeys       set_pk_offsets[n_sets] x 96 B
 *   signing_roots n_sets x 32 B
 *   signatures    n_sets x 96 B
 *   sig_sizes     optional n_sets original signature byte lengths (NULL = all 96); a set whose
 *                 length is not 96 makes its job reject with LB_INVALID_SIZE
 */
int32_t lb_batch_create(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                        const uint32_t* set_pk_offsets, const uint8_t* pubkeys,
                        const uint8_t* signing_roots, const uint8_t* signatures,
                        const uint32_t* sig_sizes, lb_batch** out);
void lb_batch_destroy(lb_batch* b);
uint32_t lb_batch_num_sets(const lb_batch* b);
uint32_t lb_batch_num_jobs(const lb_batch* b);

/*
 * Verify a resident batch: out_job[n_jobs] receives 1 / 0 / -code per job.
 * scalars: n_sets non-zero 64-bit blinding words, or NULL to draw them from the OS
 * CSPRNG (getrandom), as blst's verifyMultipleSignatures draws 8 random bytes per set.
 * A word w = hi:lo stands for the blinding value r = lo + hi * lambda mod q, lambda = -x^2
 * (the GLV eigenvalue; oracle/bls_oracle.py blinding_scalar).  Like blst's 64-bit integer,
 * a uniform word is a uniform draw from 2^64 - 1 distinct values, and it halves the blinding
 * scalar multiplications (lb_curve.h jac_mul_glv).
 * All valid jobs are checked with ONE final exponentiation; a failing batch is bisected
 * over a product tree of jobs down to the invalid ones.
 */
int32_t lb_batch_verify(lb_engine* e, lb_batch* b, const uint64_t* scalars, int32_t* out_job);

/*
 * Multi-GPU split.  lb_batch_partial runs the batch up to its root partial product
 *   f = prod_i ML(r_i PK_i, H(m_i)) * ML(-G1, sum_i r_i sig_i)        (576 B, see above)
 * and per-job error codes (out_job: -code for rejecting jobs, 1 otherwise).
 * lb_fp12_product_is_one multiplies n such partials and runs one final exponentiation;
 * *ok = 1 iff the product is 1 in GT (every valid job of every partial verifies).
 * On a 0 verdict, lb_batch_search_after_partial localises each shard's invalid jobs from the
 * state its lb_batch_partial left in the engine (the shard's own final exponentiation, then the
 * invalid-set search, with the same blinding): no second pipeline run.  It returns
 * LB_ERR_ARGUMENT if any other call ran on the engine in between (then call lb_batch_verify).
 * Replaces the reference's per-job re-verification of a failing chunk
 * (packages/beacon-node/src/chain/bls/multithread/worker.ts:76-98) for a sharded segment.
 */
int32_t lb_batch_partial(lb_engine* e, lb_batch* b, const uint64_t* scalars, uint8_t* out576,
                         int32_t* out_job);
int32_t lb_fp12_product_is_one(lb_engine* e, const uint8_t* partials576, uint32_t n, int32_t* ok);
int32_t lb_batch_search_after_partial(lb_engine* e, lb_batch* b, int32_t* out_job);

/*
 * Upload + verify in one call (the worker's verifyManySignatureSets, worker.ts:32-108): inputs go
 * into an engine-owned device workspace that is grown once and reused (no per-call device
 * allocation).  Inputs in pinned host memory (lb_host_alloc) are DMA'd directly; pageable inputs
 * are staged by the HIP runtime.
 */
int32_t lb_verify_jobs(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                       const uint32_t* set_pk_offsets, const uint8_t* pubkeys,
                       const uint8_t* signing_roots, const uint8_t* signatures,
                       const uint32_t* sig_sizes, const uint64_t* scalars, int32_t* out_job);
/* lb_verify_jobs over the resident pubkey table (pk_indices as in lb_batch_create_indexed) */
int32_t lb_verify_jobs_indexed(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                               const uint32_t* set_pk_offsets, const uint32_t* pk_indices,
                               const uint8_t* signing_roots, const uint8_t* signatures,
                               const uint32_t* sig_sizes, const uint64_t* scalars, int32_t* out_job);

/* Pinned (page-locked) host memory for request staging; NULL on failure. */
void* lb_host_alloc(size_t bytes);
void lb_host_free(void* p);

/*
 * G1 pubkey aggregation (getAggregatedPubkey + toBytes(uncompressed)):
 * out96[n_sets x 96] = ZCash uncompressed sum of each set's pubkeys; out_status[n_sets]
 * = LB_OK or the error (bad encoding / not on curve / LB_EMPTY_AGGREGATE_ARRAY).
 */
int32_t lb_aggregate_pubkeys(lb_engine* e, uint32_t n_sets, const uint32_t* set_pk_offsets,
                             const uint8_t* pubkeys, uint8_t* out96, int32_t* out_status);

/*
 * G2 signature aggregation, bls.Signature.aggregate(sigs).toBytes() as the op pools use it for
 * block production (beacon-node/src/chain/opPools/aggregatedAttestationPool.ts:321,
 * attestationPool.ts:184, syncContributionAndProofPool.ts:185).
 * Group g sums signatures [group_offsets[g], group_offsets[g+1]) of sigs96 (96 B compressed
 * each; sig_sizes as in lb_batch_create, NULL = all 96); validate != 0 adds the G2 subgroup
 * check of Signature.fromBytes(.., true).  out96[g] = compressed sum (infinity = 0xc0 || 0^95),
 * out_status[g] = LB_OK, the first bad signature's decode error, or LB_EMPTY_AGGREGATE_ARRAY.
 */
int32_t lb_aggregate_signatures(lb_engine* e, uint32_t n_groups, const uint32_t* group_offsets,
                                const uint8_t* sigs96, const uint32_t* sig_sizes, int32_t validate,
                                uint8_t* out96, int32_t* out_status);

/*
 * Batch G1 decompression (48 B compressed -> 96 B uncompressed), the pubkey cache's one-time
 * deserialisation (state-transition/src/cache/pubkeyCache.ts:56-77).  validate != 0 adds
 * PublicKey.keyValidate: infinity -> LB_PK_IS_INFINITY, not in G1 -> LB_POINT_NOT_IN_GROUP.
 */
int32_t lb_g1_decompress(lb_engine* e, uint32_t n, const uint8_t* in48, uint8_t* out96, int32_t* out_status,
                         int32_t validate);

/*
 * SSZ merkleization (the hashing of signing-root production: getBlockSignatureSets ->
 * computeSigningRoot, state-transition/src/signatureSets/index.ts:64-111, src/util/signingRoot.ts:7-13;
 * SURVEY.md §8(f) row 2).  Tree t hashes chunks [chunk_offsets[t], chunk_offsets[t+1]) of
 * chunks32 (32 B each) padded with zero chunks to 2^depths[t] leaves; mix_lengths[t] != UINT64_MAX
 * mixes in that length (SSZ lists / bitlists).  out_roots32[t] = the 32-byte root.
 */
int32_t lb_merkleize(lb_engine* e, uint32_t n_trees, const uint32_t* chunk_offsets, const uint8_t* chunks32,
                     const uint32_t* depths, const uint64_t* mix_lengths, uint8_t* out_roots32);

/*
 * KZG (EIP-4844 blobs; the c-kzg calls behind packages/beacon-node/src/util/kzg.ts:15-65, SURVEY.md
 * §8(f) row 4).  The host side (lodestar_amd/kzg.py) does the scalar-field work; these do the group
 * work on the GPU.
 *
 * lb_kzg_load_setup (ckzg.loadTrustedSetup, kzg.ts:54-67): the monomial-form setup as Lodestar's
 * trusted_setup.bin holds it -- n_g1 compressed [tau^i] G1 (48 B each) and at least two compressed
 * [tau^i] G2 (96 B each; [tau^0] G2 and [tau^1] G2 are kept).  Every point is decoded and checked
 * (curve, subgroup); out_status[i] per G1 point, and LB_POINT_NOT_IN_GROUP is returned for a bad
 * G2 point.  Replaces any previously loaded setup of this engine.
 */
int32_t lb_kzg_load_setup(lb_engine* e, const uint8_t* g1_48, uint32_t n_g1, const uint8_t* g2_96, uint32_t n_g2,
                          int32_t* out_status);

/*
 * G1 linear combination out48 = compress(sum_i s_i P_i) (the spec's g1_lincomb): P_i = setup point i
 * (points48 == NULL; n <= the loaded setup size), or n compressed points (points48).  scalars32:
 * n little-endian 32-byte scalars below r.  Returns the decode error of the first bad point.
 */
int32_t lb_g1_lincomb(lb_engine* e, uint32_t n, const uint8_t* points48, const uint8_t* scalars32, uint8_t* out48);

/*
 * verify_kzg_proof_impl: *ok = 1 iff e(C - [y] G1, -G2) e(proof, [tau] G2 - [z] G2) == 1, else 0;
 * *ok = -code if C or proof fails to decode.  z32, y32: little-endian scalars below r.
 */
int32_t lb_kzg_verify_proof(lb_engine* e, const uint8_t* commitment48, const uint8_t* z32, const uint8_t* y32,
                            const uint8_t* proof48, int32_t* ok);

/*
 * Synthetic-data helpers for tests and the benchmark (not on the verification path):
 * SecretKey.toPublicKey and SecretKey.sign as used by the reference's own tests
 * (test/e2e/chain/bls/multithread.test.ts:28-31).  Secret keys are 32-byte big-endian < r.
 */
int32_t lb_sk_to_pk(lb_engine* e, uint32_t n, const uint8_t* sks32, uint8_t* out48, uint8_t* out96);
int32_t lb_sign(lb_engine* e, uint32_t n, const uint8_t* sks32, const uint8_t* msgs32, uint8_t* out96);

/*
 * GPU-resident pubkey table (the epoch cache's index2pubkey,
 * state-transition/src/cache/pubkeyCache.ts:56-77, epochContext.ts:704).  Keys are decoded once
 * (48-byte compressed or 96-byte uncompressed, key_size says which) into affine Montgomery form in
 * HBM; out_status[n] gets LB_OK or the decode error (validate != 0 adds the infinity + subgroup
 * checks of PublicKey.keyValidate).  Appending extends the table (new validators); the table
 * belongs to the engine.
 */
int32_t lb_pubkey_table_append(lb_engine* e, uint32_t n, const uint8_t* keys, uint32_t key_size, int32_t validate,
                               int32_t* out_status, uint32_t* out_first_index);
uint32_t lb_pubkey_table_size(const lb_engine* e);

/*
 * Like lb_batch_create, but set i aggregates table entries pk_indices[set_pk_offsets[i] ..
 * set_pk_offsets[i+1]) instead of carrying pubkey bytes (4 bytes per key on the bus instead of 96).
 * An index beyond the table makes that set's job reject with LB_ERR_ARGUMENT.  pk_indices may be
 * NULL only when no set carries a key (set_pk_offsets[n_sets] == 0), else LB_ERR_ARGUMENT.
 */
int32_t lb_batch_create_indexed(lb_engine* e, uint32_t n_jobs, const uint32_t* job_offsets,
                                const uint32_t* set_pk_offsets, const uint32_t* pk_indices,
                                const uint8_t* signing_roots, const uint8_t* signatures,
                                const uint32_t* sig_sizes, lb_batch** out);

/*
 * Per-stage device timings of the last lb_batch_verify / lb_batch_partial on this engine,
 * measured with HIP events on the engine's stream.  names[i] / ms[i] for i < *n (max cap).
 */
int32_t lb_engine_set_profiling(lb_engine* e, int32_t enable);
int32_t lb_engine_last_profile(lb_engine* e, const char** names, float* ms, int32_t cap, int32_t* n);

#ifdef __cplusplus
}
#endif
#endif /* LODESTAR_BLS_H */
