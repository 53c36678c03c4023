/*
 * lb_napi.c — thin N-API (C) addon over the C ABI in include/lodestar_bls.h.
 *
 * This is the binding a Lodestar maintainer adds next to packages/beacon-node/src/chain/bls
 * (INTEGRATION.md).  It replaces two boundaries of the reference: the JS -> native one inside
 * @chainsafe/blst (node-gyp addon under maybeBatch.ts:18-37) and the worker_threads one
 * (structured clone of BlsWorkReq[], multithread/index.ts:330):
 *   - inputs are COPIED out of the JS typed arrays before the call returns, so JS may reuse
 *     its buffers at once (the reference structured-clones them);
 *   - GPU work runs on a libuv worker thread (napi_async_work), never on the event loop, and
 *     settles a Promise on the JS thread;
 *   - errors come back as codes and become Error objects whose message is the blst error
 *     string ("BLST_INVALID_SIZE", ...), as @chainsafe/blst throws them.
 *
 * Exports:
 *   createEngine(device: number) -> External
 *   destroyEngine(engine)
 *   verifyJobs(engine, jobOffsets: Uint32Array, setPkOffsets: Uint32Array, pubkeys: Uint8Array,
 *              signingRoots: Uint8Array, signatures: Uint8Array, sigSizes: Uint32Array | null)
 *     -> Promise<Int32Array>   (per job: 1 valid, 0 invalid, -code rejects)
 *   verifyJobsSync(...same...) -> Int32Array   (verifyOnMainThread path; blocks like the reference)
 *   aggregatePubkeys(engine, setPkOffsets: Uint32Array, pubkeys: Uint8Array)
 *     -> {out: Uint8Array, status: Int32Array}
 *   errorName(code: number) -> string
 */
#include <node_api.h>
#include <stdint.h>
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

typedef struct {
  lb_engine* e;
} engine_box;

static void engine_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  engine_box* b = (engine_box*)data;
  if (b->e) lb_engine_destroy(b->e);
  free(b);
}

static napi_value throw_code(napi_env env, int32_t code) {
  napi_throw_error(env, NULL, lb_error_name(code));
  return NULL;
}

static napi_value create_engine(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  int32_t device = 0;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc >= 1) NAPI_CALL(env, napi_get_value_int32(env, argv[0], &device));
  engine_box* b = (engine_box*)calloc(1, sizeof(engine_box));
  int32_t st = lb_engine_create(device, &b->e);
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
    lb_engine_destroy(b->e);
    b->e = NULL;
  }
  return NULL;
}

/* copy a typed array's bytes (null/undefined -> NULL) */
static int copy_typed(napi_env env, napi_value v, void** out, size_t* nbytes, size_t elem) {
  napi_valuetype t;
  *out = NULL;
  *nbytes = 0;
  if (napi_typeof(env, v, &t) != napi_ok) return 0;
  if (t == napi_null || t == napi_undefined) return 1;
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (!is_ta) return 0;
  napi_typedarray_type tt;
  size_t len, off;
  void* data;
  napi_value ab;
  if (napi_get_typedarray_info(env, v, &tt, &len, &data, &ab, &off) != napi_ok) return 0;
  size_t bytes = len * elem;
  *out = malloc(bytes ? bytes : 1);
  if (bytes) memcpy(*out, data, bytes);
  *nbytes = bytes;
  return 1;
}

typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref engine_ref;
  lb_engine* e;
  uint32_t n_jobs;
  uint32_t *job_off, *pk_off, *sig_sizes;
  uint8_t *pks, *roots, *sigs;
  int32_t* out;
  int32_t status;
} verify_req;

static void free_req(verify_req* r) {
  free(r->job_off);
  free(r->pk_off);
  free(r->sig_sizes);
  free(r->pks);
  free(r->roots);
  free(r->sigs);
  free(r->out);
  free(r);
}

/* (engine, jobOffsets, setPkOffsets, pubkeys, roots, sigs, sigSizes?) -> request */
static verify_req* parse_verify(napi_env env, napi_callback_info info, napi_value* engine_val) {
  size_t argc = 7;
  napi_value argv[7];
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 6) {
    napi_throw_type_error(env, NULL, "verifyJobs(engine, jobOffsets, setPkOffsets, pubkeys, roots, sigs, sigSizes?)");
    return NULL;
  }
  engine_box* b = NULL;
  if (napi_get_value_external(env, argv[0], (void**)&b) != napi_ok || !b || !b->e) {
    napi_throw_error(env, NULL, "engine destroyed");
    return NULL;
  }
  if (engine_val) *engine_val = argv[0];
  verify_req* r = (verify_req*)calloc(1, sizeof(verify_req));
  r->e = b->e;
  size_t nb;
  int ok = copy_typed(env, argv[1], (void**)&r->job_off, &nb, 4);
  r->n_jobs = nb >= 4 ? (uint32_t)(nb / 4 - 1) : 0;
  ok &= copy_typed(env, argv[2], (void**)&r->pk_off, &nb, 4);
  ok &= copy_typed(env, argv[3], (void**)&r->pks, &nb, 1);
  ok &= copy_typed(env, argv[4], (void**)&r->roots, &nb, 1);
  ok &= copy_typed(env, argv[5], (void**)&r->sigs, &nb, 1);
  if (argc >= 7) ok &= copy_typed(env, argv[6], (void**)&r->sig_sizes, &nb, 4);
  if (!ok || !r->job_off || !r->pk_off) {
    free_req(r);
    napi_throw_type_error(env, NULL, "expected Uint32Array / Uint8Array arguments");
    return NULL;
  }
  r->out = (int32_t*)calloc(r->n_jobs ? r->n_jobs : 1, sizeof(int32_t));
  return r;
}

static void run_verify(verify_req* r) {
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

static void exec_verify(napi_env env, void* data) {
  (void)env;
  run_verify((verify_req*)data);
}

static void complete_verify(napi_env env, napi_status status, void* data) {
  verify_req* r = (verify_req*)data;
  if (status != napi_ok || r->status != LB_OK) {
    napi_value msg, err;
    napi_create_string_utf8(env, lb_error_name(status != napi_ok ? LB_ERR_DEVICE : r->status), NAPI_AUTO_LENGTH,
                            &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, r->deferred, err);
  } else {
    napi_resolve_deferred(env, r->deferred, result_array(env, r));
  }
  napi_delete_async_work(env, r->work);
  if (r->engine_ref) napi_delete_reference(env, r->engine_ref);
  free_req(r);
}

static napi_value verify_jobs(napi_env env, napi_callback_info info) {
  napi_value engine_val;
  verify_req* r = parse_verify(env, info, &engine_val);
  if (!r) return NULL;
  napi_create_reference(env, engine_val, 1, &r->engine_ref); /* keep the engine alive while in flight */
  napi_value promise, name;
  NAPI_CALL(env, napi_create_promise(env, &r->deferred, &promise));
  NAPI_CALL(env, napi_create_string_utf8(env, "lodestar_bls.verifyJobs", NAPI_AUTO_LENGTH, &name));
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, exec_verify, complete_verify, r, &r->work));
  NAPI_CALL(env, napi_queue_async_work(env, r->work));
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
  NAPI_CALL(env, napi_get_value_external(env, argv[0], (void**)&b));
  if (!b || !b->e) return throw_code(env, LB_ERR_ARGUMENT);
  uint32_t* off = NULL;
  uint8_t* pks = NULL;
  size_t nb_off, nb_pk;
  if (argc < 3 || !copy_typed(env, argv[1], (void**)&off, &nb_off, 4) ||
      !copy_typed(env, argv[2], (void**)&pks, &nb_pk, 1) || nb_off < 4) {
    free(off);
    free(pks);
    napi_throw_type_error(env, NULL, "aggregatePubkeys(engine, setPkOffsets: Uint32Array, pubkeys: Uint8Array)");
    return NULL;
  }
  uint32_t n = (uint32_t)(nb_off / 4 - 1);
  napi_value ab_o, ab_s, out_o, out_s, obj;
  void *po, *ps;
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 96, &po, &ab_o));
  NAPI_CALL(env, napi_create_arraybuffer(env, (size_t)n * 4, &ps, &ab_s));
  int32_t st = lb_aggregate_pubkeys(b->e, n, off, pks, (uint8_t*)po, (int32_t*)ps);
  free(off);
  free(pks);
  if (st != LB_OK) return throw_code(env, st);
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, (size_t)n * 96, ab_o, 0, &out_o));
  NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, n, ab_s, 0, &out_s));
  NAPI_CALL(env, napi_create_object(env, &obj));
  NAPI_CALL(env, napi_set_named_property(env, obj, "out", out_o));
  NAPI_CALL(env, napi_set_named_property(env, obj, "status", out_s));
  return obj;
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
      {"errorName", NULL, error_name, NULL, NULL, NULL, napi_default, NULL},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

NAPI_MODULE(lodestar_bls, init)
