/*
 * lb_napi.c — thin N-API (C) addon over the C ABI in include/lodestar_bls.h.
 *
 * This is the binding a Lodestar maintainer adds next to packages/beacon-node/src/chain/bls
 * (INTEGRATION.md).  It replaces two boundaries of the reference: the JS -> native one inside
 * @chainsafe/blst (node-gyp addon under maybeBatch.ts:18-37) and the worker_threads one
 * (structured clone of BlsWorkReq[], multithread/index.ts:330):
 *   - inputs are COPIED out of the JS typed arrays before the call returns, so JS may reuse
 *     its buffers at once (the reference structured-clones them);
 *   - GPU work runs on the engine's own native thread (one per engine, started with its first
 *     request), never on the event loop, and settles a Promise on the JS thread through a
 *     thread-safe function.  Round 6: not the libuv pool (napi_async_work), whose 4 default
 *     threads a pool of >= 4 engines occupied for whole batches, so a verifyOnMainThread call
 *     (and Lodestar's own fs / crypto work) waited for a free thread;
 *   - errors come back as codes and become Error objects whose message is the blst error
 *     string ("BLST_INVALID_SIZE", ...), as @chainsafe/blst throws them.
 *
 *   - request buffers are pinned host memory (lb_host_alloc) from a small free-list pool, so the
 *     engine's uploads are direct DMA and no page-locking happens per call;
 *   - argument lengths are checked against the offsets before anything is queued (TypeError).
 *
 * Exports:
 *   createEngine(device: number, flags?: number) -> External   (flags: 1 = LB_ENGINE_LATENCY)
 *       (the first call raises GPU_MAX_HW_QUEUES to 16 when it is unset or lower -- HIP's and the
 *       GPU boxes' default is 4 -- so the three HIP streams of each engine get their own hardware
 *       queue)
 *   hwQueues() -> number    (the GPU_MAX_HW_QUEUES the HIP runtime was initialised with)
 *   destroyEngine(engine)   (deferred until the engine's in-flight requests have settled)
 *   verifyJobs(engine, jobOffsets: Uint32Array, setPkOffsets: Uint32Array,
 *              pubkeys: Uint8Array (96 B per key) | pkIndices: Uint32Array (resident table),
 *              signingRoots: Uint8Array, signatures: Uint8Array, sigSizes: Uint32Array | null)
 *     -> Promise<Int32Array>   (per job: 1 valid, 0 invalid, -code rejects)
 *   verifyJobsSync(...same...) -> Int32Array   (blocks the caller; state-transition's synchronous
 *     verifySignatureSet.  verifyOnMainThread uses verifyJobs on the latency engine)
 *   registerPubkeys(engine, keys: Uint8Array, keySize: 48 | 96, validate: boolean)
 *     -> {first: number, status: Int32Array}   (lb_pubkey_table_append: the index2pubkey cache)
 *   tableSize(engine) -> number
 *   g1Decompress(engine, keys48: Uint8Array) -> {out: Uint8Array, status: Int32Array}
 *   aggregateSignatures(engine, groupOffsets: Uint32Array, sigs: Uint8Array, sigSizes?, validate?)
 *     -> {out: Uint8Array (96 B per group), status: Int32Array}
 *   aggregatePubkeys(engine, setPkOffsets: Uint32Array, pubkeys: Uint8Array)
 *     -> {out: Uint8Array, status: Int32Array}
 *   errorName(code: number) -> string
 *   kzgLoadSetup(engine, g1: Uint8Array (48 B each), g2: Uint8Array (96 B each))   (throws on a bad point)
 *   g1Lincomb(engine, scalars32le: Uint8Array, points48?: Uint8Array) -> Uint8Array(48)
 *       (points omitted: the loaded setup's [tau^i] G1)
 *   kzgVerifyProof(engine, commitment48, z32le, y32le, proof48) -> boolean
 *   (the KZG calls are synchronous, as c-kzg's are; lodestar_amd/js/kzg.js builds the ckzg
 *   module surface of util/kzg.ts on them)
 */
#define NAPI_VERSION 4
#include <node_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lodestar_bls.h"

#define NAPI_CALL(env, call)                                      \
  do {                                                            \
    if ((call) != napi_ok) {                                      \
      napi_throw_error((env), NULL, "N-API call failed: " #call); \
      return NULL;                                                \
    }                                                             \
  } while (0)

struct verify_req;
typedef struct engine_box {
  lb_engine* e;
  int in_flight;       /* queued/running async requests holding e (JS thread only) */
  int destroy_pending; /* destroyEngine called while requests were in flight */
  /* the engine's request thread: a FIFO of verify_req, drained one at a time (an engine runs one
   * batch at a time anyway, lb_engine.mu), each settled through tsfn on the JS thread */
  int thr_started, thr_stop;
  pthread_t thr;
  pthread_mutex_t mu;
  pthread_cond_t cv;
  struct verify_req *head, *tail;
  napi_threadsafe_function tsfn;
} engine_box;

static void box_stop_thread(engine_box* b) {
  if (!b->thr_started) return;
  pthread_mutex_lock(&b->mu);
  b->thr_stop = 1;
  pthread_cond_signal(&b->cv);
  pthread_mutex_unlock(&b->mu);
  pthread_join(b->thr, NULL);
  napi_release_threadsafe_function(b->tsfn, napi_tsfn_abort);
  pthread_mutex_destroy(&b->mu);
  pthread_cond_destroy(&b->cv);
  b->thr_started = 0;
}

static void engine_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  engine_box* b = (engine_box*)data;
  /* the External is only collected once no request holds a reference to it */
  box_stop_thread(b);
  if (b->e) lb_engine_destroy(b->e);
  free(b);
}

/* ---------------------------------------------------------------- pinned request buffers */
/* Free lists of pinned buffers by power-of-two size class (4 KiB .. 2 GiB).  Only the JS thread
 * allocates and frees (request parse / completion), so no lock is needed. */
#define POOL_CLASSES 20
#define POOL_KEEP 8
typedef struct pin_hdr {
  struct pin_hdr* next;
  int cls;
} pin_hdr;
static pin_hdr* g_pool[POOL_CLASSES];
static int g_pool_n[POOL_CLASSES];

static void* pin_alloc(size_t bytes) {
  int cls = 0;
  size_t cap = 4096;
  while (cap < bytes + 64 && cls < POOL_CLASSES - 1) {
    cap <<= 1;
    cls++;
  }
  if (cap < bytes + 64) return NULL;
  pin_hdr* h = g_pool[cls];
  if (h) {
    g_pool[cls] = h->next;
    g_pool_n[cls]--;
  } else {
    h = (pin_hdr*)lb_host_alloc(cap);
    if (!h) return NULL;
    h->cls = cls;
  }
  return (uint8_t*)h + 64; /* 64-byte aligned payload */
}

static void pin_free(void* p) {
  if (!p) return;
  pin_hdr* h = (pin_hdr*)((uint8_t*)p - 64);
  if (g_pool_n[h->cls] >= POOL_KEEP) {
    lb_host_free(h);
    return;
  }
  h->next = g_pool[h->cls];
  g_pool[h->cls] = h;
  g_pool_n[h->cls]++;
}

static napi_value throw_code(napi_env env, int32_t code) {
  napi_throw_error(env, NULL, lb_error_name(code));
  return NULL;
}

static napi_value create_engine(napi_env env, napi_callback_info info) {
  static int queues_set = 0;
  size_t argc = 2;
  napi_value argv[2];
  int32_t device = 0;
  uint32_t flags = 0;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc >= 1) NAPI_CALL(env, napi_get_value_int32(env, argv[0], &device));
  if (argc >= 2) NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &flags));
  if (!queues_set) {
    /* HIP reads GPU_MAX_HW_QUEUES once, at runtime initialisation (the first engine): each
     * engine drives three streams, and with the default 4 queues the streams of concurrent
     * engines would share hardware queues (false dependencies between independent batches).
     * A value of 16 or more set by the operator wins; the cap of 32 is the pool's limit. */
    const char* v = getenv("GPU_MAX_HW_QUEUES");
    if (!v || !*v || atoi(v) < 16) setenv("GPU_MAX_HW_QUEUES", "16", 1);
    queues_set = 1;
  }
  engine_box* b = (engine_box*)calloc(1, sizeof(engine_box));
  int32_t st = lb_engine_create_ex(device, flags, &b->e);
  if (st != LB_OK) {
    free(b);
    return throw_code(env, st);
  }
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, b, engine_finalize, NULL, &ext));
  return ext;
}

static napi_value destroy_engine(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  NAPI_CALL(env, napi_get_value_external(env, argv[0], (void**)&b));
  if (b && b->e) {
    if (b->in_flight > 0) {
      b->destroy_pending = 1; /* the last completing request destroys it */
    } else {
      box_stop_thread(b);
      lb_engine_destroy(b->e);
      b->e = NULL;
    }
  }
  return NULL;
}

/* A typed array view: kind, element count and data pointer (null/undefined -> n = 0, data NULL). */
typedef struct {
  int present;
  napi_typedarray_type type;
  size_t n;
  void* data;
} tview;

static int get_view(napi_env env, napi_value v, tview* out) {
  napi_valuetype t;
  memset(out, 0, sizeof(*out));
  if (napi_typeof(env, v, &t) != napi_ok) return 0;
  if (t == napi_null || t == napi_undefined) return 1;
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return 0;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &out->type, &out->n, &out->data, &ab, &off) != napi_ok) return 0;
  out->present = 1;
  return 1;
}

/* pinned copy of the first `bytes` bytes of a view */
static void* pin_copy(const tview* v, size_t bytes) {
  void* p = pin_alloc(bytes ? bytes : 1);
  if (p && bytes) memcpy(p, v->data, bytes);
  return p;
}

typedef struct verify_req {
  struct verify_req* next; /* engine thread FIFO */
  napi_deferred deferred;
  napi_ref engine_ref;
  engine_box* box;
  lb_engine* e;
  uint32_t n_jobs;
  int indexed;
  uint32_t *job_off, *pk_off, *sig_sizes, *pk_idx;
  uint8_t *pks, *roots, *sigs;
  int32_t* out;
  int32_t status;
} verify_req;

static void free_req(verify_req* r) {
  pin_free(r->job_off);
  pin_free(r->pk_off);
  pin_free(r->sig_sizes);
  pin_free(r->pk_idx);
  pin_free(r->pks);
  pin_free(r->roots);
  pin_free(r->sigs);
  free(r->out);
  free(r);
}

static verify_req* arg_error(napi_env env, verify_req* r, const char* msg) {
  if (r) free_req(r);
  napi_throw_type_error(env, NULL, msg);
  return NULL;
}

/* (engine, jobOffsets, setPkOffsets, pubkeys | pkIndices, roots, sigs, sigSizes?) -> request.
 * Every length is checked against what the offsets imply before anything is copied or queued. */
static verify_req* parse_verify(napi_env env, napi_callback_info info, napi_value* engine_val) {
  size_t argc = 7;
  napi_value argv[7];
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 6)
    return arg_error(env, NULL, "verifyJobs(engine, jobOffsets, setPkOffsets, pubkeys|pkIndices, roots, sigs, sigSizes?)");
  engine_box* b = NULL;
  if (napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e || b->destroy_pending) {
    napi_throw_error(env, NULL, "engine destroyed");
    return NULL;
  }
  if (engine_val) *engine_val = argv[0];
  tview jo, po, pk, rt, sg, sz;
  memset(&sz, 0, sizeof(sz));
  if (!get_view(env, argv[1], &jo) || !get_view(env, argv[2], &po) || !get_view(env, argv[3], &pk) ||
      !get_view(env, argv[4], &rt) || !get_view(env, argv[5], &sg) || (argc >= 7 && !get_view(env, argv[6], &sz)))
    return arg_error(env, NULL, "expected typed array arguments");
  if (!jo.present || jo.type != napi_uint32_array || jo.n < 1)
    return arg_error(env, NULL, "jobOffsets must be a non-empty Uint32Array");
  if (!po.present || po.type != napi_uint32_array || po.n < 1)
    return arg_error(env, NULL, "setPkOffsets must be a non-empty Uint32Array");
  const uint32_t* jof = (const uint32_t*)jo.data;
  const uint32_t* pof = (const uint32_t*)po.data;
  const uint32_t n_jobs = (uint32_t)(jo.n - 1);
  if (jof[0] != 0) return arg_error(env, NULL, "jobOffsets[0] must be 0");
  for (uint32_t j = 0; j < n_jobs; j++)
    if (jof[j + 1] < jof[j]) return arg_error(env, NULL, "jobOffsets must be non-decreasing");
  const uint32_t n_sets = jof[n_jobs];
  if (po.n != (size_t)n_sets + 1) return arg_error(env, NULL, "setPkOffsets must have jobOffsets[nJobs] + 1 entries");
  if (pof[0] != 0) return arg_error(env, NULL, "setPkOffsets[0] must be 0");
  for (uint32_t i = 0; i < n_sets; i++)
    if (pof[i + 1] < pof[i]) return arg_error(env, NULL, "setPkOffsets must be non-decreasing");
  const size_t n_pks = pof[n_sets];
  const int indexed = pk.present && pk.type == napi_uint32_array;
  if (pk.present && !indexed && pk.type != napi_uint8_array)
    return arg_error(env, NULL, "pubkeys must be a Uint8Array (96 B per key) or a Uint32Array of table indices");
  if (indexed ? pk.n < n_pks : (n_pks && (!pk.present || pk.n < n_pks * 96)))
    return arg_error(env, NULL, "pubkeys shorter than setPkOffsets[nSets] keys");
  if (!rt.present || rt.type != napi_uint8_array || rt.n < (size_t)n_sets * 32)
    return arg_error(env, NULL, "signingRoots must be a Uint8Array of 32 B per set");
  if (!sg.present || sg.type != napi_uint8_array || sg.n < (size_t)n_sets * 96)
    return arg_error(env, NULL, "signatures must be a Uint8Array of 96 B per set");
  if (sz.present && (sz.type != napi_uint32_array || sz.n < n_sets))
    return arg_error(env, NULL, "sigSizes must be a Uint32Array with one entry per set");
  verify_req* r = (verify_req*)calloc(1, sizeof(verify_req));
  r->box = b;
  r->e = b->e;
  r->n_jobs = n_jobs;
  r->indexed = indexed;
  r->job_off = (uint32_t*)pin_copy(&jo, (size_t)(n_jobs + 1) * 4);
  r->pk_off = (uint32_t*)pin_copy(&po, (size_t)(n_sets + 1) * 4);
  if (indexed)
    r->pk_idx = (uint32_t*)pin_copy(&pk, n_pks * 4);
  else
    r->pks = (uint8_t*)pin_copy(&pk, n_pks * 96);
  r->roots = (uint8_t*)pin_copy(&rt, (size_t)n_sets * 32);
  r->sigs = (uint8_t*)pin_copy(&sg, (size_t)n_sets * 96);
  if (sz.present) r->sig_sizes = (uint32_t*)pin_copy(&sz, (size_t)n_sets * 4);
  r->out = (int32_t*)calloc(n_jobs ? n_jobs : 1, sizeof(int32_t));
  if (!r->job_off || !r->pk_off || !r->roots || !r->sigs || !r->out || (indexed ? !r->pk_idx : !r->pks) ||
      (sz.present && !r->sig_sizes)) {
    free_req(r);
    napi_throw_error(env, NULL, "out of pinned host memory");
    return NULL;
  }
  return r;
}

static void run_verify(verify_req* r) {
  if (r->indexed)
    r->status = lb_verify_jobs_indexed(r->e, r->n_jobs, r->job_off, r->pk_off, r->pk_idx, r->roots, r->sigs,
                                       r->sig_sizes, NULL, r->out);
  else
    r->status = lb_verify_jobs(r->e, r->n_jobs, r->job_off, r->pk_off, r->pks, r->roots, r->sigs, r->sig_sizes,
                               NULL, r->out);
}

static napi_value result_array(napi_env env, verify_req* r) {
  napi_value ab, arr;
  void* data;
  if (napi_create_arraybuffer(env, (size_t)r->n_jobs * 4, &data, &ab) != napi_ok) return NULL;
  if (r->n_jobs) memcpy(data, r->out, (size_t)r->n_jobs * 4);
  if (napi_create_typedarray(env, napi_int32_array, r->n_jobs, ab, 0, &arr) != napi_ok) return NULL;
  return arr;
}

/* JS thread: settle the request's promise, release the engine reference */
static void complete_verify(napi_env env, napi_value js_cb, void* context, void* data) {
  (void)js_cb;
  (void)context;
  verify_req* r = (verify_req*)data;
  engine_box* b = r->box;
  if (env) { /* NULL env: the function is being torn down (napi_tsfn_abort) */
    if (r->status != LB_OK) {
      napi_value msg, err;
      napi_create_string_utf8(env, lb_error_name(r->status), NAPI_AUTO_LENGTH, &msg);
      napi_create_error(env, NULL, msg, &err);
      napi_reject_deferred(env, r->deferred, err);
    } else {
      napi_resolve_deferred(env, r->deferred, result_array(env, r));
    }
    if (--b->in_flight == 0) {
      napi_unref_threadsafe_function(env, b->tsfn); /* an idle engine does not keep Node alive */
      if (b->destroy_pending && b->e) {
        box_stop_thread(b);
        lb_engine_destroy(b->e);
        b->e = NULL;
      }
    }
    if (r->engine_ref) napi_delete_reference(env, r->engine_ref);
  }
  free_req(r);
}

static void* engine_thread(void* arg) {
  engine_box* b = (engine_box*)arg;
  for (;;) {
    pthread_mutex_lock(&b->mu);
    while (!b->head && !b->thr_stop) pthread_cond_wait(&b->cv, &b->mu);
    if (!b->head) { /* stop, queue drained */
      pthread_mutex_unlock(&b->mu);
      return NULL;
    }
    verify_req* r = b->head;
    b->head = r->next;
    if (!b->head) b->tail = NULL;
    pthread_mutex_unlock(&b->mu);
    run_verify(r);
    napi_call_threadsafe_function(b->tsfn, r, napi_tsfn_blocking);
  }
}

static int box_start_thread(napi_env env, engine_box* b) {
  if (b->thr_started) return 1;
  napi_value name;
  if (napi_create_string_utf8(env, "lodestar_bls.verifyJobs", NAPI_AUTO_LENGTH, &name) != napi_ok ||
      napi_create_threadsafe_function(env, NULL, NULL, name, 0, 1, NULL, NULL, b, complete_verify, &b->tsfn) != napi_ok)
    return 0;
  napi_unref_threadsafe_function(env, b->tsfn);
  pthread_mutex_init(&b->mu, NULL);
  pthread_cond_init(&b->cv, NULL);
  b->thr_stop = 0;
  b->head = b->tail = NULL;
  if (pthread_create(&b->thr, NULL, engine_thread, b) != 0) {
    napi_release_threadsafe_function(b->tsfn, napi_tsfn_abort);
    return 0;
  }
  b->thr_started = 1;
  return 1;
}

static napi_value verify_jobs(napi_env env, napi_callback_info info) {
  napi_value engine_val;
  verify_req* r = parse_verify(env, info, &engine_val);
  if (!r) return NULL;
  engine_box* b = r->box;
  if (!box_start_thread(env, b)) {
    free_req(r);
    napi_throw_error(env, NULL, "cannot start the engine thread");
    return NULL;
  }
  napi_value promise;
  if (napi_create_promise(env, &r->deferred, &promise) != napi_ok) {
    free_req(r);
    napi_throw_error(env, NULL, "N-API call failed: napi_create_promise");
    return NULL;
  }
  napi_create_reference(env, engine_val, 1, &r->engine_ref); /* keep the engine alive while in flight */
  if (b->in_flight++ == 0) napi_ref_threadsafe_function(env, b->tsfn); /* pending work keeps Node alive */
  pthread_mutex_lock(&b->mu);
  r->next = NULL;
  if (b->tail) b->tail->next = r;
  else b->head = r;
  b->tail = r;
  pthread_cond_signal(&b->cv);
  pthread_mutex_unlock(&b->mu);
  return promise;
}

static napi_value verify_jobs_sync(napi_env env, napi_callback_info info) {
  verify_req* r = parse_verify(env, info, NULL);
  if (!r) return NULL;
  run_verify(r);
  napi_value out = NULL;
  if (r->status != LB_OK)
    throw_code(env, r->status);
  else
    out = result_array(env, r);
  free_req(r);
  return out;
}

static napi_value aggregate_pubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  if (argc < 3 || napi_get_value_external(env, argv[0], (void**)&b) != napi_ok) {
    napi_throw_type_error(env, NULL, "aggregatePubkeys(engine, setPkOffsets: Uint32Array, pubkeys: Uint8Array)");
    return NULL;
  }
  if (!b || !b->e) return throw_code(env, LB_ERR_ARGUMENT);
  tview off, pk;
  if (!get_view(env, argv[1], &off) || !get_view(env, argv[2], &pk) || !off.present ||
      off.type != napi_uint32_array || off.n < 1 || (pk.present && pk.type != napi_uint8_array)) {
    napi_throw_type_error(env, NULL, "aggregatePubkeys(engine, setPkOffsets: Uint32Array, pubkeys: Uint8Array)");
    return NULL;
  }
  const uint32_t* o = (const uint32_t*)off.data;
  const uint32_t n = (uint32_t)(off.n - 1);
  if (o[0] != 0) {
    napi_throw_type_error(env, NULL, "setPkOffsets[0] must be 0");
    return NULL;
  }
  for (uint32_t i = 0; i < n; i++)
    if (o[i + 1] < o[i]) {
      napi_throw_type_error(env, NULL, "setPkOffsets must be non-decreasing");
      return NULL;
    }
  if ((size_t)o[n] * 96 > (pk.present ? pk.n : 0)) {
    napi_throw_type_error(env, NULL, "pubkeys shorter than setPkOffsets[nSets] keys");
    return NULL;
  }
  napi_value ab_o, ab_s, out_o, out_s, obj;
  void *po, *ps;
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 96, &po, &ab_o));
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 4, &ps, &ab_s));
  int32_t st = lb_aggregate_pubkeys(b->e, n, o, (const uint8_t*)pk.data, (uint8_t*)po, (int32_t*)ps);
  if (st != LB_OK) return throw_code(env, st);
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, (size_t)n * 96, ab_o, 0, &out_o));
  NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, n, ab_s, 0, &out_s));
  NAPI_CALL(env, napi_create_object(env, &obj));
  NAPI_CALL(env, napi_set_named_property(env, obj, "out", out_o));
  NAPI_CALL(env, napi_set_named_property(env, obj, "status", out_s));
  return obj;
}

static napi_value register_pubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  if (argc < 3 || napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e) {
    napi_throw_type_error(env, NULL, "registerPubkeys(engine, keys: Uint8Array, keySize: 48 | 96, validate?)");
    return NULL;
  }
  tview k;
  uint32_t key_size = 0;
  bool validate = false;
  if (!get_view(env, argv[1], &k) || !k.present || k.type != napi_uint8_array ||
      napi_get_value_uint32(env, argv[2], &key_size) != napi_ok || (key_size != 48 && key_size != 96) ||
      k.n % key_size) {
    napi_throw_type_error(env, NULL, "keys must be a Uint8Array of 48- or 96-byte keys");
    return NULL;
  }
  if (argc >= 4) napi_get_value_bool(env, argv[3], &validate);
  const uint32_t n = (uint32_t)(k.n / key_size);
  napi_value ab_s, out_s, obj, first_v;
  void* ps;
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)(n ? n : 1) * 4, &ps, &ab_s));
  uint32_t first = 0;
  int32_t st = lb_pubkey_table_append(b->e, n, (const uint8_t*)k.data, key_size, validate ? 1 : 0, (int32_t*)ps,
                                      &first);
  if (st != LB_OK) return throw_code(env, st);
  NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, n, ab_s, 0, &out_s));
  NAPI_CALL(env, napi_create_uint32(env, first, &first_v));
  NAPI_CALL(env, napi_create_object(env, &obj));
  NAPI_CALL(env, napi_set_named_property(env, obj, "first", first_v));
  NAPI_CALL(env, napi_set_named_property(env, obj, "status", out_s));
  return obj;
}

/* aggregateSignatures(engine, groupOffsets: Uint32Array, sigs: Uint8Array (96 B each),
 *                     sigSizes: Uint32Array | null, validate: boolean)
 *   -> {out: Uint8Array (96 B per group), status: Int32Array}   (lb_aggregate_signatures) */
static napi_value aggregate_signatures(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  tview off, sg, sz;
  memset(&sz, 0, sizeof(sz));
  bool validate = true;
  if (argc < 3 || napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e ||
      !get_view(env, argv[1], &off) || !off.present || off.type != napi_uint32_array || off.n < 1 ||
      !get_view(env, argv[2], &sg) || (sg.present && sg.type != napi_uint8_array) ||
      (argc >= 4 && !get_view(env, argv[3], &sz)) || (sz.present && sz.type != napi_uint32_array)) {
    napi_throw_type_error(env, NULL, "aggregateSignatures(engine, groupOffsets, sigs, sigSizes?, validate?)");
    return NULL;
  }
  if (argc >= 5) napi_get_value_bool(env, argv[4], &validate);
  const uint32_t* o = (const uint32_t*)off.data;
  const uint32_t ng = (uint32_t)(off.n - 1);
  if (o[0] != 0) {
    napi_throw_type_error(env, NULL, "groupOffsets[0] must be 0");
    return NULL;
  }
  for (uint32_t g = 0; g < ng; g++)
    if (o[g + 1] < o[g]) {
      napi_throw_type_error(env, NULL, "groupOffsets must be non-decreasing");
      return NULL;
    }
  const size_t n = o[ng];
  if (n * 96 > (sg.present ? sg.n : 0) || (sz.present && sz.n < n)) {
    napi_throw_type_error(env, NULL, "sigs / sigSizes shorter than groupOffsets[nGroups] signatures");
    return NULL;
  }
  napi_value ab_o, ab_s, out_o, out_s, obj;
  void *po, *ps;
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)ng * 96, &po, &ab_o));
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)ng * 4, &ps, &ab_s));
  int32_t st = lb_aggregate_signatures(b->e, ng, o, (const uint8_t*)sg.data, sz.present ? (const uint32_t*)sz.data : NULL,
                                       validate ? 1 : 0, (uint8_t*)po, (int32_t*)ps);
  if (st != LB_OK) return throw_code(env, st);
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, (size_t)ng * 96, ab_o, 0, &out_o));
  NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, ng, ab_s, 0, &out_s));
  NAPI_CALL(env, napi_create_object(env, &obj));
  NAPI_CALL(env, napi_set_named_property(env, obj, "out", out_o));
  NAPI_CALL(env, napi_set_named_property(env, obj, "status", out_s));
  return obj;
}

/* g1Decompress(engine, keys48: Uint8Array) -> {out: Uint8Array (96 B per key), status: Int32Array} */
static napi_value g1_decompress(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  tview k;
  if (argc < 2 || napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e ||
      !get_view(env, argv[1], &k) || !k.present || k.type != napi_uint8_array || k.n % 48) {
    napi_throw_type_error(env, NULL, "g1Decompress(engine, keys48: Uint8Array of 48-byte keys)");
    return NULL;
  }
  const uint32_t n = (uint32_t)(k.n / 48);
  napi_value ab_o, ab_s, out_o, out_s, obj;
  void *po, *ps;
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 96, &po, &ab_o));
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 4, &ps, &ab_s));
  int32_t st = lb_g1_decompress(b->e, n, (const uint8_t*)k.data, (uint8_t*)po, (int32_t*)ps, 0);
  if (st != LB_OK) return throw_code(env, st);
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, (size_t)n * 96, ab_o, 0, &out_o));
  NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, n, ab_s, 0, &out_s));
  NAPI_CALL(env, napi_create_object(env, &obj));
  NAPI_CALL(env, napi_set_named_property(env, obj, "out", out_o));
  NAPI_CALL(env, napi_set_named_property(env, obj, "status", out_s));
  return obj;
}

/* merkleize(engine, chunkOffsets: Uint32Array (nTrees + 1), chunks: Uint8Array (32 B each),
 *            depths: Uint32Array (nTrees), mixLengths: BigUint64Array (nTrees; 2^64 - 1 = no mix))
 *   -> Uint8Array (32-byte roots): lb_merkleize, the SSZ hashing of signing-root production
 *   (getBlockSignatureSets -> computeSigningRoot, state-transition/src/util/signingRoot.ts:7-13);
 *   synchronous, one launch per call (js/signing_roots.js batches every tree of one level). */
static napi_value merkleize(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  tview off, ch, dep, mix;
  if (argc < 5 || napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e ||
      !get_view(env, argv[1], &off) || !off.present || off.type != napi_uint32_array || off.n < 1 ||
      !get_view(env, argv[2], &ch) || !ch.present || ch.type != napi_uint8_array || ch.n % 32 ||
      !get_view(env, argv[3], &dep) || !dep.present || dep.type != napi_uint32_array || dep.n != off.n - 1 ||
      !get_view(env, argv[4], &mix) || !mix.present || mix.type != napi_biguint64_array || mix.n != off.n - 1) {
    napi_throw_type_error(env, NULL,
                          "merkleize(engine, chunkOffsets: Uint32Array, chunks: Uint8Array, depths: Uint32Array, "
                          "mixLengths: BigUint64Array)");
    return NULL;
  }
  const uint32_t n = (uint32_t)dep.n;
  const uint32_t* o = (const uint32_t*)off.data;
  if (o[0] != 0 || (size_t)o[n] * 32 != ch.n) {
    napi_throw_type_error(env, NULL, "merkleize: chunk offsets do not match the chunk bytes");
    return NULL;
  }
  for (uint32_t t = 0; t < n; t++)
    if (o[t + 1] < o[t] || ((const uint32_t*)dep.data)[t] > 63 ||
        (uint64_t)(o[t + 1] - o[t]) > (1ull << ((const uint32_t*)dep.data)[t])) {
      napi_throw_type_error(env, NULL, "merkleize: a tree has more chunks than 2^depth");
      return NULL;
    }
  napi_value ab, out;
  void* po;
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)(n ? n : 1) * 32, &po, &ab));
  if (n) {
    const int32_t st = lb_merkleize(b->e, n, o, (const uint8_t*)ch.data, (const uint32_t*)dep.data,
                                    (const uint64_t*)mix.data, (uint8_t*)po);
    if (st != LB_OK) return throw_code(env, st);
  }
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, (size_t)n * 32, ab, 0, &out));
  return out;
}

/* KZG group work (util/kzg.ts ckzg calls; synchronous, like c-kzg's) */
static napi_value kzg_load_setup(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  tview g1, g2;
  if (argc < 3 || napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e ||
      !get_view(env, argv[1], &g1) || !g1.present || g1.type != napi_uint8_array || !g1.n || g1.n % 48 ||
      !get_view(env, argv[2], &g2) || !g2.present || g2.type != napi_uint8_array || g2.n < 192 || g2.n % 96) {
    napi_throw_type_error(env, NULL, "kzgLoadSetup(engine, g1: Uint8Array of 48-byte points, g2: Uint8Array of >= 2 96-byte points)");
    return NULL;
  }
  const uint32_t n1 = (uint32_t)(g1.n / 48);
  int32_t* st = (int32_t*)malloc((size_t)n1 * 4);
  if (!st) return throw_code(env, LB_ERR_ARGUMENT);
  const int32_t r = lb_kzg_load_setup(b->e, (const uint8_t*)g1.data, n1, (const uint8_t*)g2.data,
                                      (uint32_t)(g2.n / 96), st);
  free(st);
  if (r != LB_OK) return throw_code(env, r);
  napi_value u;
  NAPI_CALL(env, napi_get_undefined(env, &u));
  return u;
}

static napi_value g1_lincomb(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  tview sc, pts;
  memset(&pts, 0, sizeof(pts));
  if (argc < 2 || napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e ||
      !get_view(env, argv[1], &sc) || !sc.present || sc.type != napi_uint8_array || sc.n % 32 ||
      (argc >= 3 && !get_view(env, argv[2], &pts)) ||
      (pts.present && (pts.type != napi_uint8_array || pts.n != sc.n / 32 * 48))) {
    napi_throw_type_error(env, NULL, "g1Lincomb(engine, scalars32le: Uint8Array, points48?: Uint8Array)");
    return NULL;
  }
  napi_value ab, out;
  void* po;
  NAPI_CALL(env, napi_create_arraybuffer(env, 48, &po, &ab));
  const int32_t r = lb_g1_lincomb(b->e, (uint32_t)(sc.n / 32), pts.present ? (const uint8_t*)pts.data : NULL,
                                  (const uint8_t*)sc.data, (uint8_t*)po);
  if (r != LB_OK) return throw_code(env, r);
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, 48, ab, 0, &out));
  return out;
}

static napi_value kzg_verify_proof(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  tview c, z, y, pr;
  if (argc < 5 || napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e ||
      !get_view(env, argv[1], &c) || !c.present || c.n != 48 || !get_view(env, argv[2], &z) || !z.present ||
      z.n != 32 || !get_view(env, argv[3], &y) || !y.present || y.n != 32 || !get_view(env, argv[4], &pr) ||
      !pr.present || pr.n != 48) {
    napi_throw_type_error(env, NULL, "kzgVerifyProof(engine, commitment48, z32le, y32le, proof48)");
    return NULL;
  }
  int32_t ok = 0;
  const int32_t r = lb_kzg_verify_proof(b->e, (const uint8_t*)c.data, (const uint8_t*)z.data,
                                        (const uint8_t*)y.data, (const uint8_t*)pr.data, &ok);
  if (r != LB_OK) return throw_code(env, r);
  if (ok < 0) return throw_code(env, -ok);
  napi_value v;
  NAPI_CALL(env, napi_get_boolean(env, ok == 1, &v));
  return v;
}

static napi_value table_size(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], v;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  engine_box* b = NULL;
  NAPI_CALL(env, napi_get_value_external(env, argv[0], (void**)&b));
  NAPI_CALL(env, napi_create_uint32(env, b && b->e ? lb_pubkey_table_size(b->e) : 0, &v));
  return v;
}

static napi_value hw_queues(napi_env env, napi_callback_info info) {
  (void)info;
  const char* v = getenv("GPU_MAX_HW_QUEUES");
  napi_value r;
  NAPI_CALL(env, napi_create_int32(env, v && *v ? atoi(v) : 4, &r));
  return r;
}

static napi_value error_name(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], s;
  int32_t code = 0;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  NAPI_CALL(env, napi_get_value_int32(env, argv[0], &code));
  NAPI_CALL(env, napi_create_string_utf8(env, lb_error_name(code), NAPI_AUTO_LENGTH, &s));
  return s;
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"createEngine", NULL, create_engine, NULL, NULL, NULL, napi_default, NULL},
      {"destroyEngine", NULL, destroy_engine, NULL, NULL, NULL, napi_default, NULL},
      {"verifyJobs", NULL, verify_jobs, NULL, NULL, NULL, napi_default, NULL},
      {"verifyJobsSync", NULL, verify_jobs_sync, NULL, NULL, NULL, napi_default, NULL},
      {"aggregatePubkeys", NULL, aggregate_pubkeys, NULL, NULL, NULL, napi_default, NULL},
      {"registerPubkeys", NULL, register_pubkeys, NULL, NULL, NULL, napi_default, NULL},
      {"tableSize", NULL, table_size, NULL, NULL, NULL, napi_default, NULL},
      {"g1Decompress", NULL, g1_decompress, NULL, NULL, NULL, napi_default, NULL},
      {"aggregateSignatures", NULL, aggregate_signatures, NULL, NULL, NULL, napi_default, NULL},
      {"errorName", NULL, error_name, NULL, NULL, NULL, napi_default, NULL},
      {"hwQueues", NULL, hw_queues, NULL, NULL, NULL, napi_default, NULL},
      {"merkleize", NULL, merkleize, NULL, NULL, NULL, napi_default, NULL},
      {"kzgLoadSetup", NULL, kzg_load_setup, NULL, NULL, NULL, napi_default, NULL},
      {"g1Lincomb", NULL, g1_lincomb, NULL, NULL, NULL, napi_default, NULL},
      {"kzgVerifyProof", NULL, kzg_verify_proof, NULL, NULL, NULL, napi_default, NULL},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

NAPI_MODULE(lodestar_bls, init)
