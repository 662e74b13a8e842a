/*
 * sift_napi.c -- Node N-API addon over the C ABI of libsift_hip.so.
 *
 * This is the FFI a maintainer of the reference (browser/Node JS) binds: a
 * thin, zero-copy layer that hands ImageData-shaped Float32Array buffers to
 * include/sift_hip.h and returns typed arrays.  The JS module ../js/sift.mjs
 * builds the reference's call surface (src/worker.js / background.js) on it.
 * Heavy calls exist in a synchronous form and, for the one-call detector, an
 * async form on the libuv pool (napi_create_async_work) that resolves a
 * Promise, so the JS thread is not blocked -- the role the reference's Web
 * Worker plays.
 */
#define NAPI_VERSION 7  /* napi_detach_arraybuffer (releaseBuffer); Node >= 12.16 */
#include <execinfo.h>
#include <node_api.h>
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include "../../include/sift_hip.h"

#define NAPI_CALL(env, call)                                              \
  do {                                                                    \
    if ((call) != napi_ok) {                                              \
      napi_throw_error((env), NULL, "N-API call failed: " #call);        \
      return NULL;                                                        \
    }                                                                     \
  } while (0)

static napi_value throw_sift(napi_env env, struct sift_ctx *ctx, int rc, const char *what) {
  char buf[512];
  snprintf(buf, sizeof buf, "%s failed (%d): %s", what, rc, ctx ? sift_last_error(ctx) : "");
  napi_value msg, err, code;
  napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &msg);
  napi_create_error(env, NULL, msg, &err);
  napi_create_int32(env, rc, &code);
  napi_set_named_property(env, err, "siftCode", code);
  napi_throw(env, err);
  return NULL;
}

/* The JS handle of a context.  A sift_ctx is not re-entrant (include/sift_hip.h):
 * while a detectAsync job runs on the libuv pool the context is `busy` and
 * every other call on it is rejected instead of racing the worker thread. */
typedef struct ctx_box {
  struct sift_ctx *ctx;
  int busy;
  int flags;       /* sift_params.flags of the last build / load through this handle */
  double d2h_ms;   /* host wall time of this context's last keypoint copy (JS thread only) */
  napi_ref weak;   /* weak reference to the JS handle (no finalizer: see pool_rec) */
  struct ctx_box *next;
} ctx_box;

static ctx_box *get_box(napi_env env, napi_value v) {
  void *p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "expected a sift context");
    return NULL;
  }
  ctx_box *b = (ctx_box *)p;
  if (b->busy) {
    napi_throw_error(env, "SIFT_E_BUSY", "sift context busy: a detectAsync job is still running on it");
    return NULL;
  }
  return b;
}

static struct sift_ctx *get_ctx(napi_env env, napi_value v) {
  ctx_box *b = get_box(env, v);
  return b ? b->ctx : NULL;
}

static int get_i32_prop(napi_env env, napi_value obj, const char *name, int def) {
  bool has = false;
  napi_value v;
  int32_t r = def;
  if (napi_has_named_property(env, obj, name, &has) == napi_ok && has &&
      napi_get_named_property(env, obj, name, &v) == napi_ok) {
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_number) napi_get_value_int32(env, v, &r);
  }
  return r;
}

static double get_f64_prop(napi_env env, napi_value obj, const char *name, double def) {
  bool has = false;
  napi_value v;
  double r = def;
  if (napi_has_named_property(env, obj, name, &has) == napi_ok && has &&
      napi_get_named_property(env, obj, name, &v) == napi_ok) {
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_number) napi_get_value_double(env, v, &r);
  }
  return r;
}

/* params object with the C field names (the JS module maps worker.js names). */
static void read_params(napi_env env, napi_value obj, sift_params *p) {
  sift_params_default(p);
  p->num_octaves = get_i32_prop(env, obj, "num_octaves", p->num_octaves);
  p->scales_per_octave = get_i32_prop(env, obj, "scales_per_octave", p->scales_per_octave);
  p->min_blur = get_f64_prop(env, obj, "min_blur", p->min_blur);
  p->assumed_blur = get_f64_prop(env, obj, "assumed_blur", p->assumed_blur);
  p->min_interpixel_distance = get_f64_prop(env, obj, "min_interpixel_distance", p->min_interpixel_distance);
  p->flags = get_i32_prop(env, obj, "flags", 0);
}

static void *typed_data(napi_env env, napi_value v, napi_typedarray_type want, size_t *len) {
  bool is = false;
  napi_is_typedarray(env, v, &is);
  if (!is) return NULL;
  napi_typedarray_type t;
  size_t n;
  void *data;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, &n, &data, &ab, &off) != napi_ok || t != want) return NULL;
  if (len) *len = n;
  return data;
}

static napi_value make_typed(napi_env env, napi_typedarray_type t, size_t n, size_t elem, void **data) {
  napi_value ab, arr;
  void *p = NULL;
  if (napi_create_arraybuffer(env, n * elem, &p, &ab) != napi_ok) return NULL;
  if (napi_create_typedarray(env, t, n, ab, 0, &arr) != napi_ok) return NULL;
  if (data) *data = p;
  return arr;
}

/* Recycled host buffers for large results (planes, typed keypoint fields).
 * A fresh ArrayBuffer's pages fault on first touch: 10-19 GB/s into fresh
 * pages however many threads copy, against 56 GB/s of DMA into touched pages
 * (profiles/r4p_d2h_probe.txt).  Buffers of >= 1 MiB are external
 * ArrayBuffers that go back to this pool when V8 collects them, so their
 * pages stay mapped; the external-memory accounting tells V8 to collect.
 * Finalizers run on their environment's JS thread, detectAsync takes buffers
 * on the libuv pool: one lock.
 *
 * Size classes: a request is served from a buffer of its class (2 MiB units,
 * rounded up to 3 significant bits: at most 1/8 slack), so keypoint fields
 * whose counts differ from image to image still reuse each other's buffers.
 * A full pool evicts its least recently returned buffers (unmapped,
 * unregistered) instead of refusing the new one, so the sizes in current
 * use stay pooled whatever passed through before. */
#define POOL_MIN_BYTES ((size_t)1 << 20)
#define POOL_SLOTS 256
static struct {
  void *p;
  size_t bytes; /* the class size (the mapping's length) */
  unsigned long long stamp;
} g_pool[POOL_SLOTS];
static int g_pool_n = 0;
static size_t g_pool_bytes = 0;
static unsigned long long g_pool_clock = 0;
static size_t g_pool_cap = (size_t)6 << 30;  /* bytes kept for reuse (SIFT_NAPI_POOL_MB) */
static size_t g_reg_cap = (size_t)4 << 30;   /* bytes kept page-locked (SIFT_NAPI_PIN_MB) */
static pthread_mutex_t g_pool_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_once_t g_pool_once = PTHREAD_ONCE_INIT;

static void pool_caps(void) {
  const char *e = getenv("SIFT_NAPI_POOL_MB");
  if (e && *e) g_pool_cap = (size_t)strtoull(e, NULL, 10) << 20;
  e = getenv("SIFT_NAPI_PIN_MB");
  if (e && *e) g_reg_cap = (size_t)strtoull(e, NULL, 10) << 20;
}

/* The class of a request of >= POOL_MIN_BYTES bytes. */
static size_t pool_class(size_t bytes) {
  const size_t G = (size_t)2 << 20;
  size_t n = (bytes + G - 1) / G;
  int e = 0;
  while ((n >> e) >= 16) ++e;
  const size_t u = (size_t)1 << e;
  return (n + u - 1) / u * u * G;
}

/* Large buffers are anonymous mappings advised as transparent huge pages:
 * a fresh buffer then faults once per 2 MiB instead of once per 4 KiB
 * (first-touch memset 11 -> 18 GB/s, profiles/r4p_d2h_probe.txt). */
static void *big_alloc(size_t bytes) {
  void *p = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return NULL;
#ifdef MADV_HUGEPAGE
  madvise(p, bytes, MADV_HUGEPAGE);
#endif
  return p;
}

/* Recycled buffers are page-locked for the device (sift_host_register, on
 * their first reuse: registering a fresh buffer costs what its first touch
 * does, so one-shot results stay unregistered), up to g_reg_cap bytes: plane
 * and keypoint reads into them are one DMA (56 GB/s against 33 GB/s staged,
 * profiles/r4ak_plane_readback_probe.json).  g_reg lists them (pool lock);
 * the registration itself runs outside the lock. */
static struct {
  void *p;
  size_t bytes;
} g_reg[2 * POOL_SLOTS];
static int g_reg_n = 0;
static size_t g_reg_bytes = 0;

static int reg_find(void *p) {
  for (int i = 0; i < g_reg_n; ++i)
    if (g_reg[i].p == p) return i;
  return -1;
}

/* Unmap a class buffer (unregistering it first); small ones are malloc'ed. */
static void big_free(void *p, size_t bytes) {
  if (!p) return;
  if (bytes >= POOL_MIN_BYTES) {
    pthread_mutex_lock(&g_pool_mu);
    const int i = reg_find(p);
    if (i >= 0) {
      g_reg_bytes -= g_reg[i].bytes;
      g_reg[i] = g_reg[--g_reg_n];
    }
    pthread_mutex_unlock(&g_pool_mu);
    if (i >= 0) (void)sift_host_unregister(p);
    munmap(p, bytes);
  } else {
    free(p);
  }
}

/* A buffer for a request of `bytes` (class size pool_class(bytes) when large). */
static void *pool_take(size_t bytes) {
  if (bytes < POOL_MIN_BYTES) {
    void *p = NULL;
    return posix_memalign(&p, 4096, bytes ? bytes : 1) ? NULL : p;
  }
  const size_t cls = pool_class(bytes);
  void *p = NULL;
  int do_reg = 0;
  pthread_once(&g_pool_once, pool_caps);
  pthread_mutex_lock(&g_pool_mu);
  int best = -1;
  for (int i = 0; i < g_pool_n; ++i)  /* the most recently returned buffer of the class */
    if (g_pool[i].bytes == cls && (best < 0 || g_pool[i].stamp > g_pool[best].stamp)) best = i;
  if (best >= 0) {
    p = g_pool[best].p;
    g_pool[best] = g_pool[--g_pool_n];
    g_pool_bytes -= cls;
    do_reg = reg_find(p) < 0 && g_reg_n < 2 * POOL_SLOTS && g_reg_bytes + cls <= g_reg_cap;
    if (do_reg) {  /* reserve the record; filled in below */
      g_reg[g_reg_n].p = NULL;
      g_reg[g_reg_n].bytes = cls;
      g_reg_n++;
      g_reg_bytes += cls;
    }
  }
  pthread_mutex_unlock(&g_pool_mu);
  if (!p) return big_alloc(cls);
  if (do_reg) {  /* first reuse: page-lock it, outside the lock */
    const int ok = sift_host_register(p, cls) == SIFT_OK;
    pthread_mutex_lock(&g_pool_mu);
    for (int i = g_reg_n - 1; i >= 0; --i)
      if (g_reg[i].p == NULL && g_reg[i].bytes == cls) {
        if (ok) {
          g_reg[i].p = p;
        } else {
          g_reg_bytes -= cls;
          g_reg[i] = g_reg[--g_reg_n];
        }
        break;
      }
    pthread_mutex_unlock(&g_pool_mu);
  }
  return p;
}

/* Return a buffer of a `bytes` request (the class is recomputed). */
static void pool_give(void *p, size_t bytes) {
  if (!p) return;
  if (bytes < POOL_MIN_BYTES) {
    free(p);
    return;
  }
  const size_t cls = pool_class(bytes);
  void *evict[POOL_SLOTS];
  size_t evict_b[POOL_SLOTS];
  int ne = 0;
  pthread_once(&g_pool_once, pool_caps);
  pthread_mutex_lock(&g_pool_mu);
  if (cls <= g_pool_cap) {
    /* make room: the least recently returned buffers go */
    while (g_pool_n > 0 && (g_pool_n >= POOL_SLOTS || g_pool_bytes + cls > g_pool_cap)) {
      int old = 0;
      for (int i = 1; i < g_pool_n; ++i)
        if (g_pool[i].stamp < g_pool[old].stamp) old = i;
      evict[ne] = g_pool[old].p;
      evict_b[ne++] = g_pool[old].bytes;
      g_pool_bytes -= g_pool[old].bytes;
      g_pool[old] = g_pool[--g_pool_n];
    }
    g_pool[g_pool_n].p = p;
    g_pool[g_pool_n].bytes = cls;
    g_pool[g_pool_n].stamp = ++g_pool_clock;
    g_pool_n++;
    g_pool_bytes += cls;
    p = NULL;
  }
  pthread_mutex_unlock(&g_pool_mu);
  for (int i = 0; i < ne; ++i) big_free(evict[i], evict_b[i]);
  if (p) big_free(p, cls);
}

typedef struct env_state env_state;
static env_state *get_state(napi_env env);
static void pool_sweep(napi_env env, env_state *st);

/* Pool state for the tests: buffers, bytes, page-locked buffers, bytes. */
static napi_value js_pool_stats(napi_env env, napi_callback_info info) {
  (void)info;
  pool_sweep(env, get_state(env));  /* collected results count as pooled */
  pthread_mutex_lock(&g_pool_mu);
  const double v[4] = {(double)g_pool_n, (double)g_pool_bytes, (double)g_reg_n, (double)g_reg_bytes};
  pthread_mutex_unlock(&g_pool_mu);
  napi_value arr;
  NAPI_CALL(env, napi_create_array_with_length(env, 4, &arr));
  for (uint32_t i = 0; i < 4; ++i) {
    napi_value x;
    NAPI_CALL(env, napi_create_double(env, v[i], &x));
    NAPI_CALL(env, napi_set_element(env, arr, i, x));
  }
  return arr;
}

/* Result-buffer ownership.  Node 12 defers every N-API finalizer that a
 * collection triggers to a native immediate, and its environment teardown
 * can run those after the napi_env is gone (a fault opening a HandleScope,
 * profiles/r5ag_node12_exit_finalizer.txt) or meet an external ArrayBuffer
 * whose finalizer is still queued (`ArrayBufferReference::Finalize`
 * assertion).  So no object this addon hands out carries a finalizer: a
 * pooled result is an external ArrayBuffer WITHOUT one, and this record --
 * the single owner of its memory -- holds a weak reference to it.  A record
 * whose ArrayBuffer V8 has collected is swept (memory back to the pool, V8's
 * external-memory count lowered) whenever the environment makes a new pooled
 * result, and at the environment's cleanup hook.  Records are touched on
 * their environment's JS thread only. */
typedef struct pool_rec {
  void *p;
  size_t bytes;
  napi_ref weak;         /* weak reference to the ArrayBuffer (no finalizer) */
  int released;          /* the memory went back early (releaseBuffer) */
  int borrows;           /* detectAsync jobs reading this memory on the libuv pool */
  int give_pending;      /* released while borrowed: give when the last borrow ends */
  struct pool_rec *next;
} pool_rec;

/* Per-environment state (napi_set_instance_data): main thread and every
 * worker_threads Worker have their own. */
struct env_state {
  pool_rec *live;        /* result buffers handed to JS and not yet swept */
  ctx_box *ctxs;         /* contexts handed to JS and not yet swept */
  int closing;           /* this environment's cleanup hook has run */
};

static env_state *get_state(napi_env env) {
  void *d = NULL;
  if (napi_get_instance_data(env, &d) != napi_ok) return NULL;
  return (env_state *)d;
}

/* The memory of a record goes back to the pool (once, and not while a job reads it). */
static void rec_give(pool_rec *r) {
  if (r->borrows > 0) {
    r->give_pending = 1;
    return;
  }
  r->give_pending = 0;
  if (r->p) pool_give(r->p, r->bytes);
  r->p = NULL;
}

/* Sweep the records whose ArrayBuffers V8 has collected. */
static void pool_sweep(napi_env env, env_state *st) {
  if (!st || st->closing) return;
  napi_handle_scope scope;
  if (napi_open_handle_scope(env, &scope) != napi_ok) return;
  int64_t freed = 0;
  for (pool_rec **pp = &st->live; *pp;) {
    pool_rec *r = *pp;
    napi_value v = NULL;
    if (r->borrows == 0 && napi_get_reference_value(env, r->weak, &v) == napi_ok && v == NULL) {
      *pp = r->next;
      napi_delete_reference(env, r->weak);
      if (!r->released) {
        freed += (int64_t)r->bytes;
        rec_give(r);
      }
      free(r);
    } else {
      pp = &r->next;
    }
  }
  napi_close_handle_scope(env, scope);
  if (freed) {
    int64_t adj;
    napi_adjust_external_memory(env, -freed, &adj);
  }
}

/* The live, unreleased record whose memory starts at p (NULL: not a pooled result). */
static pool_rec *pool_find(env_state *st, const void *p) {
  if (!st || !p) return NULL;
  for (pool_rec *r = st->live; r; r = r->next)
    if (!r->released && r->p == p) return r;
  return NULL;
}

/* An external ArrayBuffer over a pool buffer (takes ownership of p, also on failure). */
static napi_value pool_arraybuffer(napi_env env, void *p, size_t bytes) {
  env_state *st = get_state(env);
  pool_sweep(env, st);
  napi_value ab;
  pool_rec *r = (pool_rec *)calloc(1, sizeof(pool_rec));
  if (!st || !r) {
    free(r);
    pool_give(p, bytes);
    return NULL;
  }
  r->p = p;
  r->bytes = bytes;
  if (napi_create_external_arraybuffer(env, p, bytes, NULL, NULL, &ab) != napi_ok ||
      napi_create_reference(env, ab, 0, &r->weak) != napi_ok) {
    free(r);
    pool_give(p, bytes);
    return NULL;
  }
  r->next = st->live;
  st->live = r;
  int64_t adj;
  napi_adjust_external_memory(env, (int64_t)bytes, &adj);
  return ab;
}

/* The pooled result an ArrayBuffer is (NULL for any other buffer). */
static pool_rec *pool_rec_of(napi_env env, napi_value ab) {
  bool isab = false;
  void *data = NULL;
  size_t len = 0;
  if (napi_is_arraybuffer(env, ab, &isab) != napi_ok || !isab) return NULL;
  if (napi_get_arraybuffer_info(env, ab, &data, &len) != napi_ok) return NULL;
  pool_rec *r = pool_find(get_state(env), data);
  return r && r->bytes == len ? r : NULL;
}

/* releaseBuffer(arrayBuffer) -> bool: hand a pooled result buffer (a plane or
 * a typed keypoint field of >= 1 MiB) back before V8 collects it: the
 * ArrayBuffer is detached (its views read as empty from then on) and the
 * memory returns to the pool -- at once, or, while a detectAsync job still
 * reads it as its input image, when that job completes -- so the next result
 * of its size class reuses it (page-locked on reuse) instead of faulting in
 * fresh pages.  false for any other buffer and for one released before (left
 * untouched). */
static napi_value js_release_buffer(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], res;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bool ok = false;
  pool_rec *r = argc > 0 ? pool_rec_of(env, argv[0]) : NULL;
  if (r && napi_detach_arraybuffer(env, argv[0]) == napi_ok) {
    r->released = 1;
    int64_t adj;
    napi_adjust_external_memory(env, -(int64_t)r->bytes, &adj);
    rec_give(r);
    ok = true;
  }
  NAPI_CALL(env, napi_get_boolean(env, ok, &res));
  return res;
}

/* make_typed over a recycled buffer (large results). */
static napi_value make_typed_pooled(napi_env env, napi_typedarray_type t, size_t n, size_t elem, void **data) {
  const size_t bytes = n * elem;
  if (bytes < POOL_MIN_BYTES) return make_typed(env, t, n, elem, data);
  pool_sweep(env, get_state(env));  /* collected results first, so this request can reuse one */
  void *p = pool_take(bytes);
  if (!p) return NULL;
  napi_value ab = pool_arraybuffer(env, p, bytes), arr;
  if (!ab || napi_create_typedarray(env, t, n, ab, 0, &arr) != napi_ok) return NULL;
  if (data) *data = p;
  return arr;
}

/* poolBuffer(bytes) -> Float32Array over a pooled buffer (test hook: the
 * result-buffer lifetime without a device). */
static napi_value js_pool_buffer(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  double b = 0;
  if (argc > 0) napi_get_value_double(env, argv[0], &b);
  if (!(b >= 4)) {
    napi_throw_range_error(env, NULL, "poolBuffer: bytes >= 4");
    return NULL;
  }
  float *d = NULL;
  napi_value arr = make_typed_pooled(env, napi_float32_array, (size_t)b / 4, 4, (void **)&d);
  if (!arr) {
    napi_throw_error(env, NULL, "poolBuffer: allocation failed");
    return NULL;
  }
  return arr;
}

/* Destroy the contexts whose JS handles V8 has collected (a busy one is
 * still referenced by its job, so it is never collected). */
static void ctx_sweep(napi_env env, env_state *st) {
  if (!st || st->closing) return;
  napi_handle_scope scope;
  if (napi_open_handle_scope(env, &scope) != napi_ok) return;
  for (ctx_box **pp = &st->ctxs; *pp;) {
    ctx_box *b = *pp;
    napi_value v = NULL;
    if (!b->busy && napi_get_reference_value(env, b->weak, &v) == napi_ok && v == NULL) {
      *pp = b->next;
      napi_delete_reference(env, b->weak);
      if (b->ctx) sift_ctx_destroy(b->ctx);
      free(b);
    } else {
      pp = &b->next;
    }
  }
  napi_close_handle_scope(env, scope);
}

/* createContext(device) -> external */
static napi_value js_create_context(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int32_t dev = 0;
  if (argc > 0) napi_get_value_int32(env, argv[0], &dev);
  struct sift_ctx *ctx = NULL;
  int rc = sift_ctx_create(dev, &ctx);
  if (rc) return throw_sift(env, NULL, rc, "sift_ctx_create (is a HIP device visible?)");
  ctx_box *b = (ctx_box *)calloc(1, sizeof(ctx_box));
  if (!b) {
    sift_ctx_destroy(ctx);
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  b->ctx = ctx;
  env_state *st = get_state(env);
  ctx_sweep(env, st);
  napi_value ext;
  if (!st || napi_create_external(env, b, NULL, NULL, &ext) != napi_ok ||
      napi_create_reference(env, ext, 0, &b->weak) != napi_ok) {
    sift_ctx_destroy(ctx);
    free(b);
    napi_throw_error(env, NULL, "napi_create_external failed");
    return NULL;
  }
  b->next = st->ctxs;
  st->ctxs = b;
  return ext;
}

/* octaveDims(width, height, numOctaves) -> Int32Array(2*O) */
static napi_value js_octave_dims(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int32_t w = 0, h = 0, o = 0;
  napi_get_value_int32(env, argv[0], &w);
  napi_get_value_int32(env, argv[1], &h);
  napi_get_value_int32(env, argv[2], &o);
  if (o < 1 || o > 64) {
    napi_throw_range_error(env, NULL, "numOctaves out of range");
    return NULL;
  }
  int32_t *d;
  napi_value arr = make_typed(env, napi_int32_array, 2 * (size_t)o, 4, (void **)&d);
  int rc = sift_octave_dims(w, h, o, d);
  if (rc) return throw_sift(env, NULL, rc, "sift_octave_dims");
  return arr;
}

/* buildScaleSpace(ctx, Float32Array img, width, height, params, Float64Array|null sigmas) */
static napi_value js_build(napi_env env, napi_callback_info info) {
  size_t argc = 6;
  napi_value argv[6];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  size_t n = 0;
  const float *img = (const float *)typed_data(env, argv[1], napi_float32_array, &n);
  int32_t w = 0, h = 0;
  napi_get_value_int32(env, argv[2], &w);
  napi_get_value_int32(env, argv[3], &h);
  if (!img || (size_t)w * (size_t)h > n) {
    napi_throw_type_error(env, NULL, "image must be a Float32Array of width*height gray values");
    return NULL;
  }
  sift_params p;
  read_params(env, argv[4], &p);
  const double *sig = NULL;
  if (argc > 5) sig = (const double *)typed_data(env, argv[5], napi_float64_array, NULL);
  int rc = sift_build_scale_space(ctx, img, w, h, (size_t)w, &p, sig);
  if (rc) return throw_sift(env, ctx, rc, "sift_build_scale_space");
  get_box(env, argv[0])->flags = p.flags;
  return NULL;
}

/* getPlane(ctx, kind, octave, scale) -> Float32Array */
static napi_value js_get_plane(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t kind = 0, o = 0, s = 0, rows = 0, cols = 0;
  napi_get_value_int32(env, argv[1], &kind);
  napi_get_value_int32(env, argv[2], &o);
  napi_get_value_int32(env, argv[3], &s);
  int rc = sift_get_dims(ctx, o, &rows, &cols);
  if (rc) return throw_sift(env, ctx, rc, "sift_get_dims");
  float *dst;
  napi_value arr = make_typed_pooled(env, napi_float32_array, (size_t)rows * cols, 4, (void **)&dst);
  if (!arr) return throw_sift(env, ctx, SIFT_E_ARG, "plane buffer allocation");
  rc = sift_get_plane(ctx, kind, o, s, dst, (size_t)rows * cols);
  if (rc) return throw_sift(env, ctx, rc, "sift_get_plane");
  return arr;
}

/* getDims(ctx, octave) -> [rows, cols] */
static napi_value js_get_dims(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t o = 0, r = 0, c = 0;
  napi_get_value_int32(env, argv[1], &o);
  int rc = sift_get_dims(ctx, o, &r, &c);
  if (rc) return throw_sift(env, ctx, rc, "sift_get_dims");
  napi_value arr, a, b;
  napi_create_array_with_length(env, 2, &arr);
  napi_create_int32(env, r, &a);
  napi_create_int32(env, c, &b);
  napi_set_element(env, arr, 0, a);
  napi_set_element(env, arr, 1, b);
  return arr;
}

/* loadDog / loadScaleSpace(ctx, Float32Array flat, width, height, params) */
static napi_value load_common(napi_env env, napi_callback_info info, int which) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  size_t len = 0;
  const float *flat = (const float *)typed_data(env, argv[1], napi_float32_array, &len);
  if (!flat) {
    napi_throw_type_error(env, NULL, "planes must be a Float32Array");
    return NULL;
  }
  int32_t w = 0, h = 0;
  napi_get_value_int32(env, argv[2], &w);
  napi_get_value_int32(env, argv[3], &h);
  sift_params p;
  read_params(env, argv[4], &p);
  /* The C entry points copy sum_o rows_o*cols_o*(S+2) (or S+3) floats: the
   * array must hold exactly that many, or the copy would read past its end. */
  if (w < 1 || h < 1 || p.num_octaves < 1 || p.num_octaves > 64 || p.scales_per_octave < 1) {
    napi_throw_range_error(env, NULL, "bad pyramid geometry");
    return NULL;
  }
  int32_t dims[128];
  if (sift_octave_dims(w, h, p.num_octaves, dims) != SIFT_OK) {
    napi_throw_range_error(env, NULL, "bad pyramid geometry");
    return NULL;
  }
  size_t px = 0;
  for (int o = 0; o < p.num_octaves; ++o) px += (size_t)dims[2 * o] * (size_t)dims[2 * o + 1];
  const size_t want = px * (size_t)(p.scales_per_octave + (which ? 3 : 2));
  if (len != want) {
    char buf[160];
    snprintf(buf, sizeof buf, "pyramid holds %zu values, the geometry needs %zu", len, want);
    napi_throw_range_error(env, NULL, buf);
    return NULL;
  }
  int rc = which ? sift_load_scale_space(ctx, flat, w, h, &p) : sift_load_dog(ctx, flat, w, h, &p);
  if (rc) return throw_sift(env, ctx, rc, which ? "sift_load_scale_space" : "sift_load_dog");
  get_box(env, argv[0])->flags = p.flags;
  return NULL;
}
static napi_value js_load_dog(napi_env env, napi_callback_info info) { return load_common(env, info, 0); }
static napi_value js_load_ss(napi_env env, napi_callback_info info) { return load_common(env, info, 1); }

/* extremum records -> {ints: Int32Array(4n) [o,s,x,y], values: Float64Array(n)} set on `out` as ints/values
 * (or lowInts/lowValues) */
static void extrema_to_js(napi_env env, const sift_extremum *e, size_t n, napi_value out, const char *ki,
                          const char *kv) {
  int32_t *ints;
  double *vals;
  napi_value ia = make_typed(env, napi_int32_array, 4 * n, 4, (void **)&ints);
  napi_value va = make_typed(env, napi_float64_array, n, 8, (void **)&vals);
  for (size_t i = 0; i < n; ++i) {
    ints[4 * i] = e[i].octave;
    ints[4 * i + 1] = e[i].scale;
    ints[4 * i + 2] = e[i].x;
    ints[4 * i + 3] = e[i].y;
    vals[i] = e[i].value;
  }
  napi_set_named_property(env, out, ki, ia);
  napi_set_named_property(env, out, kv, va);
}

/* findExtrema(ctx, wantLow) -> {ints: Int32Array(4n) [o,s,x,y], values: Float64Array(n), lowContrast,
 *                               lowInts?, lowValues? (the low-contrast list, wantLow)} */
static napi_value js_find_extrema(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box *box = get_box(env, argv[0]);
  if (!box) return NULL;
  struct sift_ctx *ctx = box->ctx;
  bool want_low = false;
  if (argc > 1) napi_get_value_bool(env, argv[1], &want_low);
  size_t n = 0, low = 0;
  if (want_low) {
    /* the pyramid's flags + SIFT_F_LOW_CONTRAST_LIST for this extrema stage */
    sift_set_flags(ctx, box->flags | SIFT_F_LOW_CONTRAST_LIST);
  }
  int rc = sift_find_extrema(ctx, NULL, 0, &n, &low);
  if (want_low) sift_set_flags(ctx, box->flags);
  if (rc) return throw_sift(env, ctx, rc, "sift_find_extrema");
  sift_extremum *tmp = (sift_extremum *)malloc(sizeof(sift_extremum) * (n ? n : 1));
  rc = sift_copy_candidates(ctx, tmp, n, &n);
  if (rc) {
    free(tmp);
    return throw_sift(env, ctx, rc, "sift_copy_candidates");
  }
  napi_value out, lv;
  napi_create_object(env, &out);
  extrema_to_js(env, tmp, n, out, "ints", "values");
  free(tmp);
  napi_create_double(env, (double)low, &lv);
  napi_set_named_property(env, out, "lowContrast", lv);
  if (want_low) {
    size_t nl = 0;
    rc = sift_copy_low_contrast(ctx, NULL, 0, &nl);
    if (rc) return throw_sift(env, ctx, rc, "sift_copy_low_contrast");
    sift_extremum *lt = (sift_extremum *)malloc(sizeof(sift_extremum) * (nl ? nl : 1));
    rc = sift_copy_low_contrast(ctx, lt, nl, &nl);
    if (rc) {
      free(lt);
      return throw_sift(env, ctx, rc, "sift_copy_low_contrast");
    }
    extrema_to_js(env, lt, nl, out, "lowInts", "lowValues");
    free(lt);
  }
  return out;
}

/* setCandidates(ctx, Int32Array(4n) [o,s,x,y], Float64Array(n)) */
static napi_value js_set_candidates(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  size_t ni = 0, nv = 0;
  const int32_t *ints = (const int32_t *)typed_data(env, argv[1], napi_int32_array, &ni);
  const double *vals = (const double *)typed_data(env, argv[2], napi_float64_array, &nv);
  if (!ints || !vals || ni != 4 * nv) {
    napi_throw_type_error(env, NULL, "expected Int32Array(4n) and Float64Array(n)");
    return NULL;
  }
  sift_extremum *c = (sift_extremum *)malloc(sizeof(sift_extremum) * (nv ? nv : 1));
  for (size_t i = 0; i < nv; ++i) {
    c[i].octave = ints[4 * i];
    c[i].scale = ints[4 * i + 1];
    c[i].x = ints[4 * i + 2];
    c[i].y = ints[4 * i + 3];
    c[i].value = vals[i];
  }
  int rc = sift_set_candidates(ctx, c, nv);
  free(c);
  if (rc) return throw_sift(env, ctx, rc, "sift_set_candidates");
  return NULL;
}

/* setRefineParams(ctx, minBlurLevel, minInterpixelDistance) */
static napi_value js_refine_params(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  double mb = 0.8, mid = 0.5;
  napi_get_value_double(env, argv[1], &mb);
  napi_get_value_double(env, argv[2], &mid);
  int rc = sift_refine_params(ctx, mb, mid);
  if (rc) return throw_sift(env, ctx, rc, "sift_refine_params");
  return NULL;
}

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e3 + (double)t.tv_nsec * 1e-6;
}

/* The last keypoints as two malloc'd field arrays (sift_copy_keypoints_soa:
 * one DMA into the context's pinned staging, one host pass); *ms = host wall
 * time of that copy.  On error both are NULL. */
typedef struct {
  int32_t *ints;
  double *reals;
  size_t n;
} kp_soa;

static int copy_keypoints_host(struct sift_ctx *ctx, size_t n, kp_soa *out, double *ms) {
  out->n = n;
  out->ints = (int32_t *)pool_take(sizeof(int32_t) * 4 * (n ? n : 1));
  out->reals = (double *)pool_take(sizeof(double) * 4 * (n ? n : 1));
  const double t0 = now_ms();
  int rc = (out->ints && out->reals) ? sift_copy_keypoints_soa(ctx, out->ints, out->reals, n, &out->n) : SIFT_E_ARG;
  *ms = now_ms() - t0;
  if (rc) {
    pool_give(out->ints, sizeof(int32_t) * 4 * (n ? n : 1));
    pool_give(out->reals, sizeof(double) * 4 * (n ? n : 1));
    out->ints = NULL;
    out->reals = NULL;
  }
  out->n = n;  /* the buffers' size (sift_copy_keypoints_soa returns the same count) */
  return rc;
}

/* JS typed arrays over the field arrays (external pool buffers: no copy; takes ownership). */
static napi_value keypoint_arrays(napi_env env, kp_soa *k, size_t singular) {
  napi_value iab, dab, ia, da;
  const size_t n = k->n;
  iab = pool_arraybuffer(env, k->ints, sizeof(int32_t) * 4 * (n ? n : 1));
  k->ints = NULL;  /* owned by the array buffer (or released) now */
  if (!iab) {
    pool_give(k->reals, sizeof(double) * 4 * (n ? n : 1));
    k->reals = NULL;
    return NULL;
  }
  dab = pool_arraybuffer(env, k->reals, sizeof(double) * 4 * (n ? n : 1));
  k->reals = NULL;
  if (!dab) return NULL;
  napi_create_typedarray(env, napi_int32_array, 4 * n, iab, 0, &ia);
  napi_create_typedarray(env, napi_float64_array, 4 * n, dab, 0, &da);
  napi_value out, sv;
  napi_create_object(env, &out);
  napi_set_named_property(env, out, "ints", ia);      /* octave, scaleLevel, localX, localY */
  napi_set_named_property(env, out, "doubles", da);   /* absoluteSigma, absoluteX, absoluteY, interpolatedValue */
  napi_create_double(env, (double)singular, &sv);
  napi_set_named_property(env, out, "singular", sv);
  return out;
}

static napi_value keypoints_to_js(napi_env env, ctx_box *box, size_t n, size_t singular) {
  kp_soa k;
  int rc = copy_keypoints_host(box->ctx, n, &k, &box->d2h_ms);
  if (rc) return throw_sift(env, box->ctx, rc, "sift_copy_keypoints_soa");
  return keypoint_arrays(env, &k, singular);
}

/* refine(ctx) -> {ints, doubles, singular} (singular > 0: caller mirrors the reference's TypeError) */
static napi_value js_refine(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box *box = get_box(env, argv[0]);
  if (!box) return NULL;
  struct sift_ctx *ctx = box->ctx;
  if (!ctx) return NULL;
  size_t n = 0, sing = 0;
  int rc = sift_refine(ctx, NULL, 0, &n, &sing);
  if (rc && rc != SIFT_E_SINGULAR) return throw_sift(env, ctx, rc, "sift_refine");
  return keypoints_to_js(env, box, n, sing);
}

/* detect(ctx, img, width, height, params) -> {ints, doubles, singular} */
static napi_value js_detect(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box *box = get_box(env, argv[0]);
  if (!box) return NULL;
  struct sift_ctx *ctx = box->ctx;
  if (!ctx) return NULL;
  size_t len = 0;
  const float *img = (const float *)typed_data(env, argv[1], napi_float32_array, &len);
  int32_t w = 0, h = 0;
  napi_get_value_int32(env, argv[2], &w);
  napi_get_value_int32(env, argv[3], &h);
  if (!img || (size_t)w * (size_t)h > len) {
    napi_throw_type_error(env, NULL, "image must be a Float32Array of width*height gray values");
    return NULL;
  }
  sift_params p;
  read_params(env, argv[4], &p);
  size_t n = 0;
  int rc = sift_detect(ctx, img, w, h, (size_t)w, &p, NULL, 0, &n);
  if (rc && rc != SIFT_E_SINGULAR) return throw_sift(env, ctx, rc, "sift_detect");
  size_t sing = 0;
  sift_last_counts(ctx, NULL, NULL, NULL, &sing, NULL);
  return keypoints_to_js(env, box, n, sing);
}

/* detectBatch(ctx, Float32Array of n images back to back, n, w, h, params) ->
 * {ints, doubles, singular, counts}: one batched detection (sift_detect_batch),
 * keypoints image-major, counts[b] = keypoints of image b. */
static napi_value js_detect_batch(napi_env env, napi_callback_info info) {
  size_t argc = 6;
  napi_value argv[6];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box *box = get_box(env, argv[0]);
  if (!box) return NULL;
  struct sift_ctx *ctx = box->ctx;
  if (!ctx) return NULL;
  size_t len = 0;
  const float *img = (const float *)typed_data(env, argv[1], napi_float32_array, &len);
  int32_t nimg = 0, w = 0, h = 0;
  napi_get_value_int32(env, argv[2], &nimg);
  napi_get_value_int32(env, argv[3], &w);
  napi_get_value_int32(env, argv[4], &h);
  if (!img || nimg < 1 || w < 1 || h < 1 || (size_t)nimg * (size_t)w * (size_t)h > len) {
    napi_throw_type_error(env, NULL, "images must be a Float32Array of n*width*height gray values");
    return NULL;
  }
  sift_params p;
  read_params(env, argv[5], &p);
  size_t n = 0;
  int rc = sift_detect_batch(ctx, img, nimg, (size_t)w * (size_t)h, w, h, (size_t)w, &p, NULL, 0, &n);
  if (rc && rc != SIFT_E_SINGULAR) return throw_sift(env, ctx, rc, "sift_detect_batch");
  size_t sing = 0;
  sift_last_counts(ctx, NULL, NULL, NULL, &sing, NULL);
  napi_value out = keypoints_to_js(env, box, n, sing);
  if (!out) return NULL;
  int nb = 0;
  sift_last_block_counts(ctx, NULL, 0, &nb);
  int64_t *blk = (int64_t *)calloc((size_t)(nb > 0 ? nb : 1), sizeof(int64_t));
  sift_last_block_counts(ctx, blk, nb, &nb);
  double *cnt;
  napi_value ca = make_typed(env, napi_float64_array, (size_t)nimg, 8, (void **)&cnt);
  const int per = nb / nimg;
  for (int b = 0; b < nimg; ++b) {
    double c = 0;
    for (int q = 0; q < per; ++q) c += (double)blk[b * per + q];
    cnt[b] = c;
  }
  free(blk);
  napi_set_named_property(env, out, "counts", ca);
  return out;
}

/* ---- detectAsync: the one-call path on the libuv pool, returns a Promise ---- */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref img_ref;
  napi_ref ctx_ref;
  ctx_box *box;
  struct sift_ctx *ctx;
  const float *img;
  int w, h, rc;
  sift_params p;
  size_t n;
  kp_soa kp;          /* host field arrays, copied on the worker thread */
  pool_rec *borrowed; /* the input image is a pooled result: held against release until completion */
  double d2h_ms;      /* their copy's wall time, published to the context on the JS thread */
} detect_job;

static void detect_execute(napi_env env, void *data) {
  (void)env;
  detect_job *j = (detect_job *)data;
  j->rc = sift_detect(j->ctx, j->img, j->w, j->h, (size_t)j->w, &j->p, NULL, 0, &j->n);
  if (j->rc == SIFT_OK || j->rc == SIFT_E_SINGULAR) {
    const int rc = copy_keypoints_host(j->ctx, j->n, &j->kp, &j->d2h_ms);
    if (rc) j->rc = rc;
  }
}

static void detect_complete(napi_env env, napi_status status, void *data) {
  detect_job *j = (detect_job *)data;
  j->box->busy = 0;
  j->box->d2h_ms = j->d2h_ms;
  if (status == napi_ok && (j->rc == SIFT_OK || j->rc == SIFT_E_SINGULAR)) {
    size_t sing = 0;
    sift_last_counts(j->ctx, NULL, NULL, NULL, &sing, NULL);
    napi_value res = keypoint_arrays(env, &j->kp, sing);
    if (res) {
      napi_resolve_deferred(env, j->deferred, res);
    } else {
      napi_value exc;
      napi_get_and_clear_last_exception(env, &exc);
      napi_reject_deferred(env, j->deferred, exc);
    }
  } else {
    char buf[512];
    snprintf(buf, sizeof buf, "sift_detect failed (%d): %s", j->rc, sift_last_error(j->ctx));
    napi_value msg, err;
    napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, j->deferred, err);
  }
  {
    const size_t n = j->kp.n ? j->kp.n : 1;  /* still ours on an error path: back to the pool */
    if (j->kp.ints) pool_give(j->kp.ints, sizeof(int32_t) * 4 * n);
    if (j->kp.reals) pool_give(j->kp.reals, sizeof(double) * 4 * n);
  }
  if (j->borrowed && --j->borrowed->borrows == 0 && j->borrowed->give_pending) rec_give(j->borrowed);
  napi_delete_reference(env, j->img_ref);
  napi_delete_reference(env, j->ctx_ref);
  napi_delete_async_work(env, j->work);
  free(j);
}

static napi_value js_detect_async(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box *box = get_box(env, argv[0]);
  if (!box) return NULL;
  struct sift_ctx *ctx = box->ctx;
  size_t len = 0;
  const float *img = (const float *)typed_data(env, argv[1], napi_float32_array, &len);
  int32_t w = 0, h = 0;
  napi_get_value_int32(env, argv[2], &w);
  napi_get_value_int32(env, argv[3], &h);
  if (!img || (size_t)w * (size_t)h > len) {
    napi_throw_type_error(env, NULL, "image must be a Float32Array of width*height gray values");
    return NULL;
  }
  detect_job *j = (detect_job *)calloc(1, sizeof(detect_job));
  j->box = box;
  j->ctx = ctx;
  j->img = img;
  j->w = w;
  j->h = h;
  read_params(env, argv[4], &j->p);
  napi_value promise, name;
  NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
  NAPI_CALL(env, napi_create_reference(env, argv[1], 1, &j->img_ref));  /* keep the buffer alive */
  NAPI_CALL(env, napi_create_reference(env, argv[0], 1, &j->ctx_ref));
  napi_create_string_utf8(env, "sift_detect", NAPI_AUTO_LENGTH, &name);
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, detect_execute, detect_complete, j, &j->work));
  NAPI_CALL(env, napi_queue_async_work(env, j->work));
  box->busy = 1;  /* until detect_complete (JS thread) */
  {
    /* an input that is a pooled result (a plane handed out earlier) stays
     * ours until the job is done: releaseBuffer then defers its give */
    napi_typedarray_type t;
    size_t n, off;
    void *d;
    napi_value ab;
    if (napi_get_typedarray_info(env, argv[1], &t, &n, &d, &ab, &off) == napi_ok) {
      j->borrowed = pool_rec_of(env, ab);
      if (j->borrowed) j->borrowed->borrows++;
    }
  }
  return promise;
}

static napi_value js_counts(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  size_t v[5] = {0, 0, 0, 0, 0};
  sift_last_counts(ctx, &v[0], &v[1], &v[2], &v[3], &v[4]);
  const char *names[5] = {"candidates", "lowContrast", "keypoints", "singular", "exact"};
  napi_value out;
  napi_create_object(env, &out);
  for (int i = 0; i < 5; ++i) {
    napi_value x;
    napi_create_double(env, (double)v[i], &x);
    napi_set_named_property(env, out, names[i], x);
  }
  return out;
}

/* timings(ctx) -> device stage times of the last call chain (sift_last_timings)
 * and the host wall time of the last keypoint copy to the host, ms */
static napi_value js_timings(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box *box = get_box(env, argv[0]);
  if (!box) return NULL;
  struct sift_ctx *ctx = box->ctx;
  sift_timings t;
  memset(&t, 0, sizeof t);
  int rc = sift_last_timings(ctx, &t);
  if (rc) return throw_sift(env, ctx, rc, "sift_last_timings");
  const char *names[6] = {"gaussDogMs", "extremaMs", "refineMs", "h2dMs", "gaussOct0Ms", "d2hMs"};
  const double v[6] = {t.gauss_dog_ms, t.extrema_ms, t.refine_ms, t.h2d_ms, t.gauss_oct0_ms, box->d2h_ms};
  napi_value out;
  napi_create_object(env, &out);
  for (int i = 0; i < 6; ++i) {
    napi_value x;
    napi_create_double(env, v[i], &x);
    napi_set_named_property(env, out, names[i], x);
  }
  return out;
}

static napi_value js_abi_version(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value v;
  napi_create_int32(env, sift_abi_version(), &v);
  return v;
}

/* ---- image products (ABI >= 4): RGBA ImageData in, preview ImageData out ---- */
static const uint8_t *rgba_data(napi_env env, napi_value v, size_t *len) {
  const uint8_t *d = (const uint8_t *)typed_data(env, v, napi_uint8_clamped_array, len);
  if (!d) d = (const uint8_t *)typed_data(env, v, napi_uint8_array, len);
  return d;
}

static const uint8_t *rgba_args(napi_env env, napi_value *argv, int32_t *w, int32_t *h) {
  size_t len = 0;
  const uint8_t *rgba = rgba_data(env, argv[1], &len);
  napi_get_value_int32(env, argv[2], w);
  napi_get_value_int32(env, argv[3], h);
  if (!rgba || *w <= 0 || *h <= 0 || (size_t)*w * (size_t)*h * 4 > len) {
    napi_throw_type_error(env, NULL, "image data must be a Uint8ClampedArray of width*height RGBA pixels");
    return NULL;
  }
  return rgba;
}

/* rgbaToGray(ctx, rgba, width, height, wantAlpha) -> {gray: Float32Array, alpha?: Float32Array} */
static napi_value js_rgba_to_gray(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t w = 0, h = 0;
  const uint8_t *rgba = rgba_args(env, argv, &w, &h);
  if (!rgba) return NULL;
  bool want_alpha = false;
  if (argc > 4) napi_get_value_bool(env, argv[4], &want_alpha);
  float *g = NULL, *a = NULL;
  napi_value out, garr, aarr = NULL;
  garr = make_typed(env, napi_float32_array, (size_t)w * h, 4, (void **)&g);
  if (want_alpha) aarr = make_typed(env, napi_float32_array, (size_t)w * h, 4, (void **)&a);
  int rc = sift_rgba_to_gray(ctx, rgba, w, h, (size_t)w * 4, g, a);
  if (rc) return throw_sift(env, ctx, rc, "sift_rgba_to_gray");
  napi_create_object(env, &out);
  napi_set_named_property(env, out, "gray", garr);
  if (aarr) napi_set_named_property(env, out, "alpha", aarr);
  return out;
}

/* buildScaleSpaceRgba(ctx, rgba, width, height, params, Float64Array|null sigmas) */
static napi_value js_build_rgba(napi_env env, napi_callback_info info) {
  size_t argc = 6;
  napi_value argv[6];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t w = 0, h = 0;
  const uint8_t *rgba = rgba_args(env, argv, &w, &h);
  if (!rgba) return NULL;
  sift_params p;
  read_params(env, argv[4], &p);
  const double *sig = NULL;
  if (argc > 5) sig = (const double *)typed_data(env, argv[5], napi_float64_array, NULL);
  int rc = sift_build_scale_space_rgba(ctx, rgba, w, h, (size_t)w * 4, &p, sig);
  if (rc) return throw_sift(env, ctx, rc, "sift_build_scale_space_rgba");
  get_box(env, argv[0])->flags = p.flags;
  return NULL;
}

/* detectRgba(ctx, rgba, width, height, params) -> keypoints */
static napi_value js_detect_rgba(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box *box = get_box(env, argv[0]);
  if (!box) return NULL;
  struct sift_ctx *ctx = box->ctx;
  if (!ctx) return NULL;
  int32_t w = 0, h = 0;
  const uint8_t *rgba = rgba_args(env, argv, &w, &h);
  if (!rgba) return NULL;
  sift_params p;
  read_params(env, argv[4], &p);
  size_t n = 0;
  int rc = sift_detect_rgba(ctx, rgba, w, h, (size_t)w * 4, &p, NULL, 0, &n);
  if (rc && rc != SIFT_E_SINGULAR) return throw_sift(env, ctx, rc, "sift_detect_rgba");
  size_t sing = 0;
  sift_last_counts(ctx, NULL, NULL, NULL, &sing, NULL);
  return keypoints_to_js(env, box, n, sing);
}

/* planeImage(ctx, kind, octave, scale, mode, coefficient) -> Uint8ClampedArray(rows*cols*4) */
static napi_value js_plane_image(napi_env env, napi_callback_info info) {
  size_t argc = 6;
  napi_value argv[6];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  struct sift_ctx *ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t kind = 0, o = 0, s = 0, mode = 0, rows = 0, cols = 0;
  double coef = 1.0;
  napi_get_value_int32(env, argv[1], &kind);
  napi_get_value_int32(env, argv[2], &o);
  napi_get_value_int32(env, argv[3], &s);
  napi_get_value_int32(env, argv[4], &mode);
  if (argc > 5) napi_get_value_double(env, argv[5], &coef);
  int rc = sift_get_dims(ctx, o, &rows, &cols);
  if (rc) return throw_sift(env, ctx, rc, "sift_get_dims");
  uint8_t *dst;
  const size_t bytes = (size_t)rows * cols * 4;
  napi_value arr = make_typed(env, napi_uint8_clamped_array, bytes, 1, (void **)&dst);
  rc = sift_plane_image(ctx, kind, o, s, mode, coef, dst, bytes);
  if (rc) return throw_sift(env, ctx, rc, "sift_plane_image");
  return arr;
}

/* SIFT_NAPI_SEGV_TRACE=1 (diagnostics): a fatal signal prints the native
 * stack to stderr before the default action. */
static void segv_trace(int sig) {
  void *bt[64];
  const int n = backtrace(bt, 64);
  static const char msg[] = "sift_napi: fatal signal, native stack:\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(bt, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

/* The environment is going away (process exit or a Worker ending; no JS runs
 * from here on): its result buffers go back to the pool and its contexts are
 * destroyed, except what an unfinished detectAsync job still uses. */
static void on_env_cleanup(void *arg) {
  napi_env env = (napi_env)arg;
  env_state *st = get_state(env);
  if (!st) return;
  st->closing = 1;
  for (pool_rec *r = st->live, *nx; r; r = nx) {
    nx = r->next;
    napi_delete_reference(env, r->weak);
    if (r->borrows > 0) continue;  /* its job's memory: left as it is */
    if (!r->released || r->give_pending) {
      r->borrows = 0;
      rec_give(r);
    }
    free(r);
  }
  st->live = NULL;
  for (ctx_box *b = st->ctxs, *nx; b; b = nx) {
    nx = b->next;
    napi_delete_reference(env, b->weak);
    if (b->busy) continue;
    if (b->ctx) sift_ctx_destroy(b->ctx);
    free(b);
  }
  st->ctxs = NULL;
}

/* At exit (before the HIP runtime's own teardown, whose handlers were
 * registered earlier): the pooled buffers are unpinned while it still runs. */
static void pool_atexit(void) {
  pthread_mutex_lock(&g_pool_mu);
  const int n = g_reg_n;
  void *p[2 * POOL_SLOTS];
  for (int i = 0; i < n; ++i) p[i] = g_reg[i].p;
  g_reg_n = 0;
  g_reg_bytes = 0;
  pthread_mutex_unlock(&g_pool_mu);
  for (int i = 0; i < n; ++i)
    if (p[i]) (void)sift_host_unregister(p[i]);
}

static napi_value init(napi_env env, napi_value exports) {
  {
    env_state *st = (env_state *)calloc(1, sizeof(env_state));
    if (!st || napi_set_instance_data(env, st, NULL, NULL) != napi_ok) {
      free(st);
      napi_throw_error(env, NULL, "sift_napi: per-environment state");
      return NULL;
    }
    napi_add_env_cleanup_hook(env, on_env_cleanup, env);
  }
  {
    static int once = 0;
    if (!once) {
      once = 1;
      atexit(pool_atexit);
    }
  }
  {
    const char *t = getenv("SIFT_NAPI_SEGV_TRACE");
    if (t && atoi(t)) {
      signal(SIGSEGV, segv_trace);
      signal(SIGBUS, segv_trace);
      signal(SIGABRT, segv_trace);
    }
  }
  napi_property_descriptor props[] = {
      {"abiVersion", 0, js_abi_version, 0, 0, 0, napi_enumerable, 0},
      {"createContext", 0, js_create_context, 0, 0, 0, napi_enumerable, 0},
      {"octaveDims", 0, js_octave_dims, 0, 0, 0, napi_enumerable, 0},
      {"buildScaleSpace", 0, js_build, 0, 0, 0, napi_enumerable, 0},
      {"getPlane", 0, js_get_plane, 0, 0, 0, napi_enumerable, 0},
      {"getDims", 0, js_get_dims, 0, 0, 0, napi_enumerable, 0},
      {"loadDog", 0, js_load_dog, 0, 0, 0, napi_enumerable, 0},
      {"loadScaleSpace", 0, js_load_ss, 0, 0, 0, napi_enumerable, 0},
      {"findExtrema", 0, js_find_extrema, 0, 0, 0, napi_enumerable, 0},
      {"setCandidates", 0, js_set_candidates, 0, 0, 0, napi_enumerable, 0},
      {"refine", 0, js_refine, 0, 0, 0, napi_enumerable, 0},
      {"setRefineParams", 0, js_refine_params, 0, 0, 0, napi_enumerable, 0},
      {"detect", 0, js_detect, 0, 0, 0, napi_enumerable, 0},
      {"detectAsync", 0, js_detect_async, 0, 0, 0, napi_enumerable, 0},
      {"poolStats", 0, js_pool_stats, 0, 0, 0, napi_enumerable, 0},
      {"releaseBuffer", 0, js_release_buffer, 0, 0, 0, napi_enumerable, 0},
      {"poolBuffer", 0, js_pool_buffer, 0, 0, 0, napi_enumerable, 0},
      {"detectBatch", 0, js_detect_batch, 0, 0, 0, napi_enumerable, 0},
      {"counts", 0, js_counts, 0, 0, 0, napi_enumerable, 0},
      {"timings", 0, js_timings, 0, 0, 0, napi_enumerable, 0},
      {"rgbaToGray", 0, js_rgba_to_gray, 0, 0, 0, napi_enumerable, 0},
      {"buildScaleSpaceRgba", 0, js_build_rgba, 0, 0, 0, napi_enumerable, 0},
      {"detectRgba", 0, js_detect_rgba, 0, 0, 0, napi_enumerable, 0},
      {"planeImage", 0, js_plane_image, 0, 0, 0, napi_enumerable, 0},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
