/*
 * sentinel_oracle.c — TEST INFRASTRUCTURE ONLY (see sentinel_oracle.h).
 *
 * Single-threaded C restatement of the reference Java path.  Citations are
 * relative to /root/reference with these abbreviations:
 *   CORE = sentinel-core/src/main/java/com/alibaba/csp/sentinel
 *   PF   = sentinel-extension/sentinel-parameter-flow-control/src/main/java/com/alibaba/csp/sentinel
 *   CS   = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster
 *
 * Faithfulness rules: object structure follows the Java (lazy LeapArray
 * buckets, null slots, Occupiable borrow arrays, per-call currentWindow()
 * rolls); Java numerics are reproduced exactly (saturating casts,
 * Math.round, Math.nextUp, wrapping long arithmetic, no FMA contraction —
 * built with -ffp-contract=off).  Concurrency artefacts (CAS retry loops,
 * Thread.yield) are single-threaded no-ops.  Thread.sleep() does not
 * advance the mocked clock; the duration is reported as a wait.
 *
 * ParameterMetric's maps (ConcurrentLinkedHashMap LRUs of capacity
 * min(4000*durationInSec, 200000), ParameterMetric.java:37-39,99) are exact
 * unbounded maps by default, as in the engine's exact table; so_set_param_lru
 * bounds them like the reference (CacheMap section below).  The two agree
 * while no rule's map sees more distinct keys than its capacity; where they
 * differ, the LRU mode is the reference's behaviour (SURVEY.md §7 part 6).
 */
#include "sentinel_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================
 * Mocked clock — CORE/util/TimeUtil.java:222-224 (mockStatic in tests)
 * ==================================================================== */
static _Thread_local int64_t g_now = 0;  /* per thread: oracle/sharded.py replays shards on threads */
static int64_t g_stat_max_rt = 5000;   /* CORE/config/SentinelConfig.java:69,247 */

void so_set_time(int64_t t) { g_now = t; }
int64_t so_now(void) { return g_now; }
void so_set_statistic_max_rt(int64_t rt) { g_stat_max_rt = rt; }

/* ======================================================================
 * Java numeric semantics
 * ==================================================================== */
int32_t so_java_d2i(double a) {                 /* JLS 5.1.3 */
    if (a != a) return 0;
    if (a >= 2147483647.0) return INT32_MAX;
    if (a <= -2147483648.0) return INT32_MIN;
    return (int32_t)a;
}
int64_t so_java_d2l(double a) {
    if (a != a) return 0;
    if (a >= 9223372036854775807.0) return INT64_MAX;   /* == 2^63 */
    if (a <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)a;
}
/* java.lang.Math.round(double) (JDK 8+): round half up, computed exactly. */
int64_t so_java_round(double a) {
    int64_t bits;
    memcpy(&bits, &a, 8);
    int64_t biased_exp = (bits & 0x7ff0000000000000LL) >> 52;
    int64_t shift = (52 - 1 + 1023) - biased_exp;
    if ((shift & -64) == 0) {
        int64_t r = (bits & 0x000fffffffffffffLL) | (0x000fffffffffffffLL + 1);
        if (bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    return so_java_d2l(a);
}
double so_java_next_up(double a) { return nextafter(a, INFINITY); }
static int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static int64_t jmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
static int64_t jdiv(int64_t a, int64_t b) {      /* b != 0 checked by callers */
    if (a == INT64_MIN && b == -1) return INT64_MIN;
    return a / b;
}
static int32_t iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }

/* ======================================================================
 * Exact hash map  (Object value -> long), used for ParameterMetric and
 * ClusterParamMetric buckets.  Key = Java equals() identity (tag, bits).
 * ==================================================================== */
typedef struct {
    uint8_t* used; uint8_t* tag; uint64_t* bits; int64_t* val;
    uint32_t cap, size;
} so_map;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}
static void map_init(so_map* m, uint32_t cap) {
    m->cap = cap; m->size = 0;
    m->used = calloc(cap, 1); m->tag = calloc(cap, 1);
    m->bits = calloc(cap, 8); m->val = calloc(cap, 8);
}
static void map_free(so_map* m) { free(m->used); free(m->tag); free(m->bits); free(m->val); memset(m, 0, sizeof *m); }
static void map_clear(so_map* m) { memset(m->used, 0, m->cap); m->size = 0; }
static uint32_t map_slot(const so_map* m, uint8_t tag, uint64_t bits) {
    return (uint32_t)(mix64(bits * 31 + tag) & (m->cap - 1));
}
static int64_t* map_find(so_map* m, uint8_t tag, uint64_t bits) {
    uint32_t i = map_slot(m, tag, bits);
    while (m->used[i]) {
        if (m->tag[i] == tag && m->bits[i] == bits) return &m->val[i];
        i = (i + 1) & (m->cap - 1);
    }
    return NULL;
}
static void map_grow(so_map* m);
static int64_t* map_insert(so_map* m, uint8_t tag, uint64_t bits, int64_t v) {
    if ((m->size + 1) * 2 > m->cap) map_grow(m);
    uint32_t i = map_slot(m, tag, bits);
    while (m->used[i]) i = (i + 1) & (m->cap - 1);
    m->used[i] = 1; m->tag[i] = tag; m->bits[i] = bits; m->val[i] = v; m->size++;
    return &m->val[i];
}
static void map_grow(so_map* m) {
    so_map n; map_init(&n, m->cap * 2);
    for (uint32_t i = 0; i < m->cap; i++)
        if (m->used[i]) map_insert(&n, m->tag[i], m->bits[i], m->val[i]);
    map_free(m); *m = n;
}
static void map_remove(so_map* m, uint8_t tag, uint64_t bits) {  /* backward-shift delete */
    uint32_t i = map_slot(m, tag, bits);
    while (m->used[i] && !(m->tag[i] == tag && m->bits[i] == bits)) i = (i + 1) & (m->cap - 1);
    if (!m->used[i]) return;
    m->used[i] = 0; m->size--;
    uint32_t j = i;
    for (;;) {
        j = (j + 1) & (m->cap - 1);
        if (!m->used[j]) break;
        uint32_t k = map_slot(m, m->tag[j], m->bits[j]);
        if ((j > i && (k <= i || k > j)) || (j < i && (k <= i && k > j))) {
            m->used[i] = 1; m->tag[i] = m->tag[j]; m->bits[i] = m->bits[j]; m->val[i] = m->val[j];
            m->used[j] = 0; i = j;
        }
    }
}

/* ======================================================================
 * Buckets
 * ==================================================================== */
/* MetricEvent ordinals: CORE/slots/statistic/MetricEvent.java:21-39 */
enum { EV_PASS = 0, EV_BLOCK, EV_EXCEPTION, EV_SUCCESS, EV_RT, EV_OCCUPIED_PASS, EV_COUNT };
/* ClusterFlowEvent ordinals: CS/flow/statistic/data/ClusterFlowEvent.java:22-52 */
enum { CE_PASS = 0, CE_BLOCK, CE_PASS_REQUEST, CE_BLOCK_REQUEST, CE_OCCUPIED_PASS,
       CE_OCCUPIED_BLOCK, CE_WAITING, CE_COUNT };

typedef struct { int64_t c[EV_COUNT]; int64_t min_rt; } mbucket;   /* MetricBucket.java:28-142 */
typedef struct { int64_t c[CE_COUNT]; } cbucket;                   /* ClusterMetricBucket.java:24-50 */
typedef struct { int64_t v; } ubucket;                              /* LongAdder (UnaryLeapArray) */

static void mb_init(mbucket* b) { memset(b->c, 0, sizeof b->c); b->min_rt = g_stat_max_rt; } /* MetricBucket.java:37-58 */
static void mb_reset_from(mbucket* b, const mbucket* src) {          /* MetricBucket.java:46-53 */
    for (int e = 0; e < EV_COUNT; e++) b->c[e] = src->c[e];
    b->min_rt = g_stat_max_rt;
}
static void mb_reset(mbucket* b) { mb_init(b); }                     /* MetricBucket.java:64-70 */
static void mb_add_rt(mbucket* b, int64_t rt) {                      /* MetricBucket.java:129-136 */
    b->c[EV_RT] = jadd(b->c[EV_RT], rt);
    if (rt < b->min_rt) b->min_rt = rt;
}

/* ======================================================================
 * LeapArray — CORE/slots/statistic/base/LeapArray.java:41-445
 * ==================================================================== */
#define SO_LA_CLUSTER_PARAM 5   /* ClusterParameterLeapArray (internal) */

struct so_wrap { int64_t window_length; int64_t window_start; void* value; };

struct so_leap_array {
    int kind;
    int window_length, sample_count, interval_ms;
    double interval_sec;
    so_wrap** array;                 /* AtomicReferenceArray<WindowWrap<T>>; NULL = absent */
    so_leap_array* borrow;           /* OccupiableBucketLeapArray.java:31 borrowArray       */
    int64_t occupy[CE_COUNT];        /* ClusterMetricLeapArray.java:31 occupyCounter        */
    int has_occupied;                /* ClusterMetricLeapArray.java:32                      */
    so_wrap* throwaway;              /* LeapArray.java:220-223 windows not stored           */
};

static size_t value_size(int kind) {
    switch (kind) {
    case SO_LA_CLUSTER: return sizeof(cbucket);
    case SO_LA_UNARY: return sizeof(ubucket);
    case SO_LA_CLUSTER_PARAM: return sizeof(so_map);
    default: return sizeof(mbucket);
    }
}
static void value_free(int kind, void* v) {
    if (!v) return;
    if (kind == SO_LA_CLUSTER_PARAM) map_free((so_map*)v);
    free(v);
}

static so_wrap* la_window_value(so_leap_array* a, int64_t t);

/* newEmptyBucket(time) per subclass */
static void* la_new_empty_bucket(so_leap_array* a, int64_t time) {
    void* v = calloc(1, value_size(a->kind));
    switch (a->kind) {
    case SO_LA_OCCUPIABLE: {                       /* OccupiableBucketLeapArray.java:40-49 */
        mbucket* b = v; mb_init(b);
        so_wrap* bw = la_window_value(a->borrow, time);
        if (bw) mb_reset_from(b, (mbucket*)bw->value);
        break;
    }
    case SO_LA_BUCKET: case SO_LA_FUTURE:          /* BucketLeapArray.java:35-38; FutureBucketLeapArray.java:36-39 */
        mb_init((mbucket*)v); break;
    case SO_LA_CLUSTER_PARAM:                      /* ClusterParameterLeapArray.java:40-42 */
        map_init((so_map*)v, 16); break;
    default: break;                                /* ClusterMetricBucket / LongAdder: zero */
    }
    return v;
}
/* resetWindowTo(w, startTime) per subclass */
static so_wrap* la_reset_window_to(so_leap_array* a, so_wrap* w, int64_t start) {
    w->window_start = start;                       /* WindowWrap.resetTo (WindowWrap.java:78-81) */
    switch (a->kind) {
    case SO_LA_OCCUPIABLE: {                       /* OccupiableBucketLeapArray.java:52-64 */
        so_wrap* bw = la_window_value(a->borrow, start);
        mbucket* b = w->value;
        mb_reset(b);
        if (bw) b->c[EV_PASS] = jadd(b->c[EV_PASS], (int64_t)(int32_t)((mbucket*)bw->value)->c[EV_PASS]);
        break;
    }
    case SO_LA_BUCKET: case SO_LA_FUTURE:
        mb_reset((mbucket*)w->value); break;
    case SO_LA_UNARY:                              /* UnaryLeapArray.java:33-38 */
        ((ubucket*)w->value)->v = 0; break;
    case SO_LA_CLUSTER: {                          /* ClusterMetricLeapArray.java:45-71 */
        cbucket* b = w->value;
        memset(b, 0, sizeof *b);
        if (a->has_occupied) {
            b->c[CE_OCCUPIED_PASS] += a->occupy[CE_PASS];
            b->c[CE_PASS] += a->occupy[CE_PASS]; a->occupy[CE_PASS] = 0;
            b->c[CE_PASS_REQUEST] += a->occupy[CE_PASS_REQUEST]; a->occupy[CE_PASS_REQUEST] = 0;
            a->has_occupied = 0;
        }
        break;
    }
    case SO_LA_CLUSTER_PARAM:                      /* ClusterParameterLeapArray.java:44-48 */
        map_clear((so_map*)w->value); break;
    }
    return w;
}
/* isWindowDeprecated(time, w) — LeapArray.java:294-296; Future inverts it (FutureBucketLeapArray.java:49-52) */
static int la_is_deprecated(const so_leap_array* a, int64_t time, const so_wrap* w) {
    if (a->kind == SO_LA_FUTURE) return time >= w->window_start;
    return jsub(time, w->window_start) > a->interval_ms;
}

so_leap_array* so_la_new(int kind, int sample_count, int interval_ms) {   /* LeapArray.java:70-87 */
    if (sample_count <= 0 || interval_ms <= 0 || interval_ms % sample_count != 0) return NULL;
    so_leap_array* a = calloc(1, sizeof *a);
    a->kind = kind;
    a->window_length = interval_ms / sample_count;
    a->interval_ms = interval_ms;
    a->interval_sec = interval_ms / 1000.0;
    a->sample_count = sample_count;
    a->array = calloc((size_t)sample_count, sizeof(so_wrap*));
    if (kind == SO_LA_OCCUPIABLE) a->borrow = so_la_new(SO_LA_FUTURE, sample_count, interval_ms);
    return a;
}
static void wrap_free(int kind, so_wrap* w) { if (w) { value_free(kind, w->value); free(w); } }
void so_la_free(so_leap_array* a) {
    if (!a) return;
    for (int i = 0; i < a->sample_count; i++) wrap_free(a->kind, a->array[i]);
    wrap_free(a->kind, a->throwaway);
    free(a->array);
    so_la_free(a->borrow);
    free(a);
}
static int la_time_idx(const so_leap_array* a, int64_t t) {          /* LeapArray.java:110-115 */
    int64_t time_id = t / a->window_length;
    return (int)(time_id % a->sample_count);
}
static int64_t la_window_start(const so_leap_array* a, int64_t t) {  /* LeapArray.java:117-119 */
    return t - t % a->window_length;
}
static so_wrap* new_wrap(so_leap_array* a, int64_t ws, int64_t t) {
    so_wrap* w = calloc(1, sizeof *w);
    w->window_length = a->window_length; w->window_start = ws;
    w->value = la_new_empty_bucket(a, t);
    return w;
}
/* currentWindow(long) — LeapArray.java:128-225 */
so_wrap* so_la_current_window(so_leap_array* a, int64_t t) {
    if (t < 0) return NULL;
    int idx = la_time_idx(a, t);
    int64_t ws = la_window_start(a, t);
    so_wrap* old = a->array[idx];
    if (old == NULL) {                                   /* :164-174 create + CAS */
        a->array[idx] = new_wrap(a, ws, t);
        return a->array[idx];
    } else if (ws == old->window_start) {                /* :175-183 */
        return old;
    } else if (ws > old->window_start) {                 /* :184-213 tryLock + reset */
        return la_reset_window_to(a, old, ws);
    }
    /* :214-222 should not go through here: a window that is never stored */
    wrap_free(a->kind, a->throwaway);
    a->throwaway = new_wrap(a, ws, t);
    return a->throwaway;
}
so_wrap* so_la_current_window_now(so_leap_array* a) { return so_la_current_window(a, g_now); } /* :89-91 */

/* getPreviousWindow(long) — LeapArray.java:234-251; deprecation reads TimeUtil (:242) */
so_wrap* so_la_previous_window(so_leap_array* a, int64_t t) {
    if (t < 0) return NULL;
    int idx = la_time_idx(a, t - a->window_length);
    t = t - a->window_length;
    so_wrap* w = a->array[idx];
    if (w == NULL || la_is_deprecated(a, g_now, w)) return NULL;
    if (w->window_start + a->window_length < t) return NULL;
    return w;
}
/* getWindowValue(long) — LeapArray.java:268-281 (+ WindowWrap.isTimeInWindow :87-89) */
static so_wrap* la_window_value(so_leap_array* a, int64_t t) {
    if (t < 0) return NULL;
    int idx = la_time_idx(a, t);
    so_wrap* w = a->array[idx];
    if (w == NULL || !(w->window_start <= t && t < w->window_start + a->window_length)) return NULL;
    return w;
}
so_wrap* so_la_window_value(so_leap_array* a, int64_t t) { return la_window_value(a, t); }
/* getValidHead(long) — LeapArray.java:378-388; deprecation reads TimeUtil (:383) */
so_wrap* so_la_valid_head(so_leap_array* a, int64_t t) {
    int idx = la_time_idx(a, t + a->window_length);
    so_wrap* w = a->array[idx];
    if (w == NULL || la_is_deprecated(a, g_now, w)) return NULL;
    return w;
}
/* values(long) — LeapArray.java:353-369 (returns the wraps of the values) */
int so_la_values(so_leap_array* a, int64_t t, so_wrap** out, int cap) {
    int n = 0;
    if (t < 0) return 0;
    for (int i = 0; i < a->sample_count; i++) {
        so_wrap* w = a->array[i];
        if (w == NULL || la_is_deprecated(a, t, w)) continue;
        if (n < cap) out[n] = w;
        n++;
    }
    return n;
}
/* list(long) — LeapArray.java:308-322 (same filter as values) */
int so_la_list_now(so_leap_array* a, so_wrap** out, int cap) { return so_la_values(a, g_now, out, cap); }

/* OccupiableBucketLeapArray.currentWaiting — :67-76 */
int64_t so_la_current_waiting(so_leap_array* a) {
    if (a->kind != SO_LA_OCCUPIABLE) return 0;             /* LeapArray.java:436-438 */
    so_la_current_window(a->borrow, g_now);
    int64_t waiting = 0;
    so_wrap* vals[SF_MAX_SAMPLE_COUNT * 4];
    int n = so_la_values(a->borrow, g_now, vals, SF_MAX_SAMPLE_COUNT * 4);
    for (int i = 0; i < n; i++) waiting = jadd(waiting, ((mbucket*)vals[i]->value)->c[EV_PASS]);
    return waiting;
}
/* OccupiableBucketLeapArray.addWaiting — :79-83 */
void so_la_add_waiting(so_leap_array* a, int64_t t, int32_t c) {
    so_wrap* w = so_la_current_window(a->borrow, t);
    mbucket* b = w->value;
    b->c[EV_PASS] = jadd(b->c[EV_PASS], c);
}
int64_t so_wrap_start(const so_wrap* w) { return w ? w->window_start : SF_WS_ABSENT; }
int64_t so_wrap_length(const so_wrap* w) { return w->window_length; }
int64_t so_wrap_get(const so_wrap* w, int event) {
    return ((const int64_t*)w->value)[event];     /* mbucket/cbucket/ubucket all begin with int64 counters */
}
void so_wrap_add(so_wrap* w, int event, int64_t n) {
    int64_t* c = (int64_t*)w->value; c[event] = jadd(c[event], n);
}
int64_t so_wrap_min_rt(const so_wrap* w) { return ((const mbucket*)w->value)->min_rt; }
void so_wrap_add_rt(so_wrap* w, int64_t rt) { mb_add_rt((mbucket*)w->value, rt); }

/* ======================================================================
 * ArrayMetric — CORE/slots/statistic/metric/ArrayMetric.java:36-346
 * ==================================================================== */
struct so_array_metric { so_leap_array* data; };
#define AM_MAXV 64

so_array_metric* so_am_new(int sample_count, int interval_ms, int enable_occupy) { /* :40-58 */
    so_array_metric* m = calloc(1, sizeof *m);
    m->data = so_la_new(enable_occupy ? SO_LA_OCCUPIABLE : SO_LA_BUCKET, sample_count, interval_ms);
    return m;
}
void so_am_free(so_array_metric* m) { if (m) { so_la_free(m->data); free(m); } }

static int64_t am_sum(so_array_metric* m, int event) {   /* pass()/block()/... :117-126 etc. */
    so_la_current_window(m->data, g_now);
    so_wrap* v[AM_MAXV];
    int n = so_la_values(m->data, g_now, v, AM_MAXV);
    int64_t s = 0;
    for (int i = 0; i < n; i++) s = jadd(s, ((mbucket*)v[i]->value)->c[event]);
    return s;
}
int64_t so_am_pass(so_array_metric* m) { return am_sum(m, EV_PASS); }
int64_t so_am_block(so_array_metric* m) { return am_sum(m, EV_BLOCK); }
int64_t so_am_success(so_array_metric* m) { return am_sum(m, EV_SUCCESS); }
int64_t so_am_exception(so_array_metric* m) { return am_sum(m, EV_EXCEPTION); }
int64_t so_am_rt(so_array_metric* m) { return am_sum(m, EV_RT); }
int64_t so_am_occupied_pass(so_array_metric* m) { return am_sum(m, EV_OCCUPIED_PASS); }
int64_t so_am_min_rt(so_array_metric* m) {               /* :151-162 */
    so_la_current_window(m->data, g_now);
    int64_t rt = g_stat_max_rt;
    so_wrap* v[AM_MAXV];
    int n = so_la_values(m->data, g_now, v, AM_MAXV);
    for (int i = 0; i < n; i++) if (((mbucket*)v[i]->value)->min_rt < rt) rt = ((mbucket*)v[i]->value)->min_rt;
    return rt > 1 ? rt : 1;
}
int64_t so_am_max_success(so_array_metric* m) {          /* :81-92 */
    so_la_current_window(m->data, g_now);
    int64_t s = 0;
    so_wrap* v[AM_MAXV];
    int n = so_la_values(m->data, g_now, v, AM_MAXV);
    for (int i = 0; i < n; i++) if (((mbucket*)v[i]->value)->c[EV_SUCCESS] > s) s = ((mbucket*)v[i]->value)->c[EV_SUCCESS];
    return s > 1 ? s : 1;
}
int64_t so_am_previous_window_pass(so_array_metric* m) {  /* :279-286 */
    so_la_current_window(m->data, g_now);
    so_wrap* w = so_la_previous_window(m->data, g_now);
    return w ? ((mbucket*)w->value)->c[EV_PASS] : 0;
}
int64_t so_am_previous_window_block(so_array_metric* m) { /* :270-277 */
    so_la_current_window(m->data, g_now);
    so_wrap* w = so_la_previous_window(m->data, g_now);
    return w ? ((mbucket*)w->value)->c[EV_BLOCK] : 0;
}
int64_t so_am_window_pass(so_array_metric* m, int64_t t) { /* getWindowPass :324-330 */
    so_wrap* w = la_window_value(m->data, t);
    return w ? ((mbucket*)w->value)->c[EV_PASS] : 0;
}
int64_t so_am_waiting(so_array_metric* m) { return so_la_current_waiting(m->data); } /* :333-335 */
void so_am_add(so_array_metric* m, int event, int32_t n) {  /* addPass/addBlock/... :222-261 */
    so_wrap* w = so_la_current_window(m->data, g_now);
    mbucket* b = w->value;
    b->c[event] = jadd(b->c[event], n);
}
void so_am_add_rt(so_array_metric* m, int64_t rt) {        /* :256-260 */
    so_wrap* w = so_la_current_window(m->data, g_now);
    mb_add_rt((mbucket*)w->value, rt);
}
void so_am_add_waiting(so_array_metric* m, int64_t t, int32_t c) { so_la_add_waiting(m->data, t, c); } /* :236-238 */

/* details()/detailsOnCondition() — :192-220 ; fromBucket :198-212 */
int so_am_details(so_array_metric* m, int filter, int64_t lo, sf_metric_row* out, int cap) {
    so_la_current_window(m->data, g_now);
    so_wrap* v[AM_MAXV];
    int n = so_la_values(m->data, g_now, v, AM_MAXV), k = 0;
    for (int i = 0; i < n; i++) {
        if (filter && !(v[i]->window_start >= lo)) continue;
        mbucket* b = v[i]->value;
        if (k < cap) {
            sf_metric_row* r = &out[k];
            memset(r, 0, sizeof *r);
            r->block_qps = b->c[EV_BLOCK]; r->exception_qps = b->c[EV_EXCEPTION];
            r->pass_qps = b->c[EV_PASS]; r->success_qps = b->c[EV_SUCCESS];
            r->rt = b->c[EV_SUCCESS] != 0 ? jdiv(b->c[EV_RT], b->c[EV_SUCCESS]) : b->c[EV_RT];
            r->timestamp = v[i]->window_start; r->occupied_pass_qps = b->c[EV_OCCUPIED_PASS];
        }
        k++;
    }
    return k;
}

/* ======================================================================
 * StatisticNode — CORE/node/StatisticNode.java:90-347
 * ==================================================================== */
static int g_sample_count = 2;        /* SampleCountProperty.SAMPLE_COUNT (SampleCountProperty.java:39) */
static int g_interval = 1000;         /* IntervalProperty.INTERVAL (IntervalProperty.java:41)          */
static int g_occupy_timeout = 500;    /* OccupyTimeoutProperty (OccupyTimeoutProperty.java:41)        */

struct so_node {
    so_array_metric* second;          /* :97-98 rollingCounterInSecond */
    so_array_metric* minute;          /* :105 rollingCounterInMinute   */
    int64_t cur_thread_num;           /* :111 LongAdder                */
    int64_t last_fetch_time;          /* :116                          */
};
so_node* so_node_new(void) {
    so_node* n = calloc(1, sizeof *n);
    n->second = so_am_new(g_sample_count, g_interval, 1);
    n->minute = so_am_new(60, 60 * 1000, 0);
    n->last_fetch_time = -1;
    return n;
}
void so_node_free(so_node* n) { if (n) { so_am_free(n->second); so_am_free(n->minute); free(n); } }
static double sec_interval(so_node* n) { return n->second->data->interval_sec; }
double so_node_pass_qps(so_node* n) { return (double)so_am_pass(n->second) / sec_interval(n); }     /* :205-208 */
double so_node_block_qps(so_node* n) { return (double)so_am_block(n->second) / sec_interval(n); }   /* :169-171 */
double so_node_success_qps(so_node* n) { return (double)so_am_success(n->second) / sec_interval(n); }
double so_node_previous_pass_qps(so_node* n) { return (double)so_am_previous_window_pass(n->minute); } /* :179-181 */
double so_node_max_success_qps(so_node* n) {                                                      /* :221-224 */
    return (double)so_am_max_success(n->second) * n->second->data->sample_count / sec_interval(n);
}
double so_node_avg_rt(so_node* n) {                                                               /* :232-240 */
    int64_t sc = so_am_success(n->second);
    if (sc == 0) return 0;
    return (double)so_am_rt(n->second) * 1.0 / (double)sc;
}
double so_node_min_rt(so_node* n) { return (double)so_am_min_rt(n->second); }                     /* :243-245 */
int32_t so_node_cur_thread_num(so_node* n) { return (int32_t)n->cur_thread_num; }                 /* :248-250 */
void so_node_add_pass_request(so_node* n, int32_t c) {                                            /* :253-256 */
    so_am_add(n->second, EV_PASS, c); so_am_add(n->minute, EV_PASS, c);
}
void so_node_add_rt_and_success(so_node* n, int64_t rt, int32_t c) {                              /* :259-265 */
    so_am_add(n->second, EV_SUCCESS, c); so_am_add_rt(n->second, rt);
    so_am_add(n->minute, EV_SUCCESS, c); so_am_add_rt(n->minute, rt);
}
void so_node_increase_block_qps(so_node* n, int32_t c) {                                          /* :268-271 */
    so_am_add(n->second, EV_BLOCK, c); so_am_add(n->minute, EV_BLOCK, c);
}
void so_node_increase_exception_qps(so_node* n, int32_t c) {                                      /* :274-277 */
    so_am_add(n->second, EV_EXCEPTION, c); so_am_add(n->minute, EV_EXCEPTION, c);
}
void so_node_increase_thread_num(so_node* n) { n->cur_thread_num++; }                             /* :280-282 */
void so_node_decrease_thread_num(so_node* n) { n->cur_thread_num--; }                             /* :285-287 */
/* tryOccupyNext — :295-330 */
int64_t so_node_try_occupy_next(so_node* n, int64_t now, int32_t c, double threshold) {
    double max_count = threshold * g_interval / 1000;
    int64_t current_borrow = so_am_waiting(n->second);
    if ((double)current_borrow >= max_count) return g_occupy_timeout;
    int window_length = g_interval / g_sample_count;
    int64_t earliest = now - now % window_length + window_length - g_interval;
    int idx = 0;
    int64_t current_pass = so_am_pass(n->second);
    while (earliest < now) {
        int64_t wait = (int64_t)idx * window_length + window_length - now % window_length;
        if (wait >= g_occupy_timeout) break;
        int64_t window_pass = so_am_window_pass(n->second, earliest);
        if ((double)(current_pass + current_borrow + c - window_pass) <= max_count) return wait;
        earliest += window_length;
        current_pass -= window_pass;
        idx++;
    }
    return g_occupy_timeout;
}
int64_t so_node_waiting(so_node* n) { return so_am_waiting(n->second); }                           /* :333-335 */
void so_node_add_waiting_request(so_node* n, int64_t future, int32_t c) { so_am_add_waiting(n->second, future, c); } /* :338-340 */
void so_node_add_occupied_pass(so_node* n, int32_t c) {                                           /* :343-346 */
    so_am_add(n->minute, EV_OCCUPIED_PASS, c); so_am_add(n->minute, EV_PASS, c);
}
static void read_bucket(const so_wrap* w, sf_bucket* b) {
    if (!w) { memset(b, 0, sizeof *b); b->window_start = SF_WS_ABSENT; return; }
    const mbucket* m = w->value;
    b->window_start = w->window_start;
    b->pass = m->c[EV_PASS]; b->block = m->c[EV_BLOCK]; b->exception = m->c[EV_EXCEPTION];
    b->success = m->c[EV_SUCCESS]; b->rt = m->c[EV_RT]; b->occupied_pass = m->c[EV_OCCUPIED_PASS];
    b->min_rt = m->min_rt;
}
void so_node_read(so_node* n, sf_node_state* out) {
    memset(out, 0, sizeof *out);
    for (int i = 0; i < SF_MAX_SAMPLE_COUNT; i++) {
        out->second[i].window_start = SF_WS_ABSENT; out->borrow_ws[i] = SF_WS_ABSENT;
    }
    for (int i = 0; i < SF_MINUTE_BUCKETS; i++) out->minute[i].window_start = SF_WS_ABSENT;
    if (!n) return;
    so_leap_array* s = n->second->data;
    for (int i = 0; i < s->sample_count && i < SF_MAX_SAMPLE_COUNT; i++) {
        read_bucket(s->array[i], &out->second[i]);
        so_wrap* bw = s->borrow->array[i];
        out->borrow_ws[i] = bw ? bw->window_start : SF_WS_ABSENT;
        out->borrow_pass[i] = bw ? ((mbucket*)bw->value)->c[EV_PASS] : 0;
    }
    for (int i = 0; i < SF_MINUTE_BUCKETS; i++) read_bucket(n->minute->data->array[i], &out->minute[i]);
    out->cur_thread_num = n->cur_thread_num;
}

/* ======================================================================
 * Traffic shaping controllers — CORE/slots/block/flow/controller/ (all)
 * ==================================================================== */
enum { CT_DEFAULT, CT_WARM_UP, CT_RATE_LIMITER, CT_WARM_UP_RATE_LIMITER };
struct so_controller {
    int type;
    double count; int grade;                        /* DefaultController.java:33-41 */
    int cold_factor, warning_token, max_token;      /* WarmUpController.java:76-96 */
    double slope;
    int64_t stored_tokens, last_filled_time;        /* AtomicLong(0), AtomicLong(0) */
    int max_queueing_time_ms;                       /* RateLimiterController.java:32-35 */
    int64_t latest_passed_time;                     /* AtomicLong(-1) */
};

/* Node reads dispatched to a real StatisticNode or a Mockito-style mock. */
static double nd_pass_qps(so_node* n, const so_mock_node* m) { return m ? m->pass_qps : so_node_pass_qps(n); }
static double nd_prev_qps(so_node* n, const so_mock_node* m) { return m ? m->previous_pass_qps : so_node_previous_pass_qps(n); }
static int32_t nd_threads(so_node* n, const so_mock_node* m) { return m ? m->cur_thread_num : so_node_cur_thread_num(n); }

so_controller* so_ctrl_default(double count, int grade) {
    so_controller* c = calloc(1, sizeof *c);
    c->type = CT_DEFAULT; c->count = count; c->grade = grade;
    c->latest_passed_time = -1;        /* unused by this controller; reads like the RateLimiter initial */
    return c;
}
static void warm_up_construct(so_controller* c, double count, int period, int cold_factor) { /* WarmUpController.java:113-139 */
    c->count = count;
    c->cold_factor = cold_factor;
    c->warning_token = so_java_d2i(period * count) / (cold_factor - 1);
    c->max_token = c->warning_token + so_java_d2i(2 * period * count / (1.0 + cold_factor));
    c->slope = (cold_factor - 1.0) / count / (c->max_token - c->warning_token);
    c->stored_tokens = 0; c->last_filled_time = 0;
}
so_controller* so_ctrl_warm_up(double count, int period_sec, int cold_factor) {
    if (cold_factor <= 1) return NULL;                              /* :114-116 IllegalArgumentException */
    so_controller* c = calloc(1, sizeof *c);
    c->type = CT_WARM_UP; warm_up_construct(c, count, period_sec, cold_factor);
    c->latest_passed_time = -1;        /* unused by this controller */
    return c;
}
so_controller* so_ctrl_rate_limiter(int timeout_ms, double count) {
    so_controller* c = calloc(1, sizeof *c);
    c->type = CT_RATE_LIMITER; c->max_queueing_time_ms = timeout_ms; c->count = count;
    c->latest_passed_time = -1;
    return c;
}
so_controller* so_ctrl_warm_up_rate_limiter(double count, int period_sec, int timeout_ms, int cold_factor) {
    if (cold_factor <= 1) return NULL;
    so_controller* c = calloc(1, sizeof *c);
    c->type = CT_WARM_UP_RATE_LIMITER; warm_up_construct(c, count, period_sec, cold_factor);
    c->max_queueing_time_ms = timeout_ms; c->latest_passed_time = -1;
    return c;
}
void so_ctrl_free(so_controller* c) { free(c); }
int32_t so_ctrl_warning_token(const so_controller* c) { return c->warning_token; }
int32_t so_ctrl_max_token(const so_controller* c) { return c->max_token; }
double so_ctrl_slope(const so_controller* c) { return c->slope; }
void so_ctrl_state(const so_controller* c, sf_rule_state* out) {
    out->stored_tokens = c->stored_tokens;
    out->last_filled_time = c->last_filled_time;
    out->latest_passed_time = c->latest_passed_time;
}

/* WarmUpController.coolDownTokens — :217-232 */
static int64_t cool_down_tokens(so_controller* c, int64_t current_time, int64_t pass_qps) {
    int64_t old_value = c->stored_tokens;
    int64_t new_value = old_value;
    if (old_value < c->warning_token) {
        new_value = so_java_d2l((double)old_value + (double)(current_time - c->last_filled_time) * c->count / 1000);
    } else if (old_value > c->warning_token) {
        if (pass_qps < so_java_d2i(c->count) / c->cold_factor) {
            new_value = so_java_d2l((double)old_value + (double)(current_time - c->last_filled_time) * c->count / 1000);
        }
    }
    return new_value < c->max_token ? new_value : c->max_token;
}
/* WarmUpController.syncToken — :178-197 */
static void sync_token(so_controller* c, int64_t pass_qps) {
    int64_t current_time = g_now;
    current_time = current_time - current_time % 1000;
    int64_t old_last_fill = c->last_filled_time;
    if (current_time <= old_last_fill) return;
    int64_t new_value = cool_down_tokens(c, current_time, pass_qps);
    c->stored_tokens = new_value;                              /* compareAndSet succeeds single-threaded */
    int64_t current_value = (c->stored_tokens = jsub(c->stored_tokens, pass_qps));
    if (current_value < 0) c->stored_tokens = 0;
    c->last_filled_time = current_time;
}

int so_ctrl_can_pass(so_controller* c, so_node* node, const so_mock_node* mock,
                     int32_t acquire, int prioritized, int64_t* wait_ms, int* prio_wait) {
    *wait_ms = 0; *prio_wait = 0;
    switch (c->type) {
    case CT_DEFAULT: {                                           /* DefaultController.java:50-89 */
        int32_t cur = (node == NULL && mock == NULL) ? 0
            : (c->grade == SF_GRADE_THREAD ? nd_threads(node, mock) : so_java_d2i(nd_pass_qps(node, mock)));
        if ((double)iadd(cur, acquire) > c->count) {
            if (prioritized && c->grade == SF_GRADE_QPS && node != NULL) {
                int64_t now = g_now;
                int64_t wait = so_node_try_occupy_next(node, now, acquire, c->count);
                if (wait < g_occupy_timeout) {
                    so_node_add_waiting_request(node, now + wait, acquire);
                    so_node_add_occupied_pass(node, acquire);
                    *wait_ms = wait; *prio_wait = 1;             /* sleep + PriorityWaitException */
                    return 1;
                }
            }
            return 0;
        }
        return 1;
    }
    case CT_WARM_UP: {                                           /* WarmUpController.java:147-175 */
        int64_t pass_qps = so_java_d2l(nd_pass_qps(node, mock));
        int64_t previous_qps = so_java_d2l(nd_prev_qps(node, mock));
        sync_token(c, previous_qps);
        int64_t rest = c->stored_tokens;
        if (rest >= c->warning_token) {
            int64_t above = rest - c->warning_token;
            double warning_qps = so_java_next_up(1.0 / ((double)above * c->slope + 1.0 / c->count));
            if ((double)(pass_qps + acquire) <= warning_qps) return 1;
        } else {
            if ((double)(pass_qps + acquire) <= c->count) return 1;
        }
        return 0;
    }
    case CT_RATE_LIMITER: {                                      /* RateLimiterController.java:48-102 */
        if (acquire <= 0) return 1;
        if (c->count <= 0) return 0;
        int64_t current_time = g_now;
        int64_t cost = so_java_round(1.0 * acquire / c->count * 1000);
        int64_t expected = cost + c->latest_passed_time;
        if (expected <= current_time) {
            c->latest_passed_time = current_time;
            return 1;
        }
        int64_t wait = cost + c->latest_passed_time - g_now;
        if (wait > c->max_queueing_time_ms) return 0;
        int64_t old_time = (c->latest_passed_time += cost);
        wait = old_time - g_now;
        if (wait > c->max_queueing_time_ms) { c->latest_passed_time -= cost; return 0; }
        if (wait > 0) *wait_ms = wait;
        return 1;
    }
    case CT_WARM_UP_RATE_LIMITER: {                              /* WarmUpRateLimiterController.java:43-87 */
        int64_t previous_qps = so_java_d2l(nd_prev_qps(node, mock));
        sync_token(c, previous_qps);
        int64_t current_time = g_now;
        int64_t rest = c->stored_tokens;
        int64_t cost;
        if (rest >= c->warning_token) {
            int64_t above = rest - c->warning_token;
            double warming_qps = so_java_next_up(1.0 / ((double)above * c->slope + 1.0 / c->count));
            cost = so_java_round(1.0 * acquire / warming_qps * 1000);
        } else {
            cost = so_java_round(1.0 * acquire / c->count * 1000);
        }
        int64_t expected = cost + c->latest_passed_time;
        if (expected <= current_time) {
            c->latest_passed_time = current_time;
            return 1;
        }
        int64_t wait = cost + c->latest_passed_time - current_time;
        if (wait > c->max_queueing_time_ms) return 0;
        int64_t old_time = (c->latest_passed_time += cost);
        wait = old_time - g_now;
        if (wait > c->max_queueing_time_ms) { c->latest_passed_time -= cost; return 0; }
        if (wait > 0) *wait_ms = wait;
        return 1;
    }
    }
    return 1;
}

/* ======================================================================
 * CacheMap (PF/slots/statistic/cache/CacheMap.java) — the maps ParameterMetric
 * keeps per rule and per parameter index.  Two modes:
 *   exact: an unbounded map, as in the engine (the default);
 *   LRU:   ConcurrentLinkedHashMapWrapper (ConcurrentLinkedHashMapWrapper.java:
 *          35-44): com.googlecode.concurrentlinkedhashmap 1.4.2 (not vendored;
 *          sentinel-parameter-flow-control/pom.xml:26-30) with
 *          maximumWeightedCapacity(size) and the singleton weigher.  Restated
 *          from its published algorithm, single-threaded: get / putIfAbsent of
 *          a present key record a read in the thread's read buffer (afterRead);
 *          a buffer holding 32 undrained reads is drained, and every write
 *          (putIfAbsent of an absent key -> AddTask, put of a present key,
 *          remove -> RemovalTask) drains the read buffer first and then its
 *          task (drainBuffers: drainReadBuffers, drainWriteBuffer).  A drained
 *          read moves its node to the back of the eviction deque (applyRead,
 *          a node no longer in the deque is skipped); AddTask appends the new
 *          node and evicts from the front while weightedSize > capacity.  Since
 *          every add drains all pending reads before it evicts, the deque at
 *          each eviction is ordered by last access (read or insert): the map is
 *          a strict LRU of `cap` entries, which is what this restates.
 * ==================================================================== */
#define SO_NIL 0xffffffffu
typedef struct {
    so_map ix;                          /* (tag, bits) -> node index            */
    uint64_t cap;                       /* maximumWeightedCapacity (entries)    */
    uint32_t n, pool, head, tail, free_list;   /* head: least recently used     */
    uint32_t *prev, *next; uint8_t* tag; uint64_t* bits; int64_t* val;
    uint64_t evictions;
} so_lru;
typedef struct { so_map map; so_lru* lru; } so_cmap;   /* lru NULL: exact */

static so_lru* lru_new(uint64_t cap) {
    so_lru* m = calloc(1, sizeof *m);
    map_init(&m->ix, 16);
    m->cap = cap; m->head = m->tail = m->free_list = SO_NIL;
    return m;
}
static void lru_free(so_lru* m) {
    if (!m) return;
    map_free(&m->ix);
    free(m->prev); free(m->next); free(m->tag); free(m->bits); free(m->val); free(m);
}
static void lru_unlink(so_lru* m, uint32_t x) {
    if (m->prev[x] != SO_NIL) m->next[m->prev[x]] = m->next[x]; else m->head = m->next[x];
    if (m->next[x] != SO_NIL) m->prev[m->next[x]] = m->prev[x]; else m->tail = m->prev[x];
}
static void lru_append(so_lru* m, uint32_t x) {
    m->prev[x] = m->tail; m->next[x] = SO_NIL;
    if (m->tail != SO_NIL) m->next[m->tail] = x; else m->head = x;
    m->tail = x;
}
static void lru_touch(so_lru* m, uint32_t x) {           /* applyRead: moveToBack */
    if (m->tail == x) return;
    lru_unlink(m, x); lru_append(m, x);
}
static void lru_drop(so_lru* m, uint32_t x) {            /* remove from map + deque */
    map_remove(&m->ix, m->tag[x], m->bits[x]);
    lru_unlink(m, x);
    m->next[x] = m->free_list; m->free_list = x; m->n--;
}
static int64_t* lru_get(so_lru* m, uint8_t tag, uint64_t bits, int touch) {
    int64_t* x = map_find(&m->ix, tag, bits);
    if (!x) return NULL;
    if (touch) lru_touch(m, (uint32_t)*x);
    return &m->val[*x];
}
/* putIfAbsent: the present entry (a read), or NULL after adding `v` (AddTask:
 * append, then evict from the front while the map holds more than cap). */
static int64_t* lru_put_if_absent(so_lru* m, uint8_t tag, uint64_t bits, int64_t v) {
    int64_t* have = lru_get(m, tag, bits, 1);
    if (have) return have;
    uint32_t x = m->free_list;
    if (x != SO_NIL) m->free_list = m->next[x];
    else {
        if (m->n == m->pool) {
            uint32_t np = m->pool ? m->pool * 2 : 64;
            m->prev = realloc(m->prev, np * 4ull); m->next = realloc(m->next, np * 4ull);
            m->tag = realloc(m->tag, np); m->bits = realloc(m->bits, np * 8ull); m->val = realloc(m->val, np * 8ull);
            for (uint32_t k = np; k-- > m->pool;) { m->next[k] = m->free_list; m->free_list = k; }
            m->pool = np;
        }
        x = m->free_list; m->free_list = m->next[x];
    }
    m->tag[x] = tag; m->bits[x] = bits; m->val[x] = v; m->n++;
    map_insert(&m->ix, tag, bits, x);
    lru_append(m, x);
    while (m->n > m->cap) { lru_drop(m, m->head); m->evictions++; }   /* evict() */
    return NULL;
}

static void cm_init(so_cmap* c, uint64_t lru_cap) {
    memset(c, 0, sizeof *c);
    if (lru_cap) c->lru = lru_new(lru_cap); else map_init(&c->map, 16);
}
static void cm_free(so_cmap* c) { if (c->lru) lru_free(c->lru); else map_free(&c->map); memset(c, 0, sizeof *c); }
/* CacheMap.get: an access (afterRead) */
static int64_t* cm_get(so_cmap* c, uint8_t tag, uint64_t bits) {
    return c->lru ? lru_get(c->lru, tag, bits, 1) : map_find(&c->map, tag, bits);
}
/* a look without an access (state readers for tests) */
static int64_t* cm_peek(so_cmap* c, uint8_t tag, uint64_t bits) {
    return c->lru ? lru_get(c->lru, tag, bits, 0) : map_find(&c->map, tag, bits);
}
/* CacheMap.putIfAbsent: the present value (an access), or NULL after the insert */
static int64_t* cm_put_if_absent(so_cmap* c, uint8_t tag, uint64_t bits, int64_t v) {
    if (c->lru) return lru_put_if_absent(c->lru, tag, bits, v);
    int64_t* have = map_find(&c->map, tag, bits);
    if (have) return have;
    map_insert(&c->map, tag, bits, v);
    return NULL;
}
/* CacheMap.put over a present or absent key: the value set, an access */
static void cm_put(so_cmap* c, uint8_t tag, uint64_t bits, int64_t v) {
    int64_t* have = cm_put_if_absent(c, tag, bits, v);
    if (have) *have = v;
}
static void cm_remove(so_cmap* c, uint8_t tag, uint64_t bits) {
    if (!c->lru) { map_remove(&c->map, tag, bits); return; }
    int64_t* x = map_find(&c->lru->ix, tag, bits);
    if (x) lru_drop(c->lru, (uint32_t)*x);
}

/* ======================================================================
 * ParameterMetric + ParamFlowChecker — PF/slots/block/flow/param/ (all)
 * ==================================================================== */
typedef struct { int key; int present; so_cmap map; } rule_map;   /* Map<ParamFlowRule, CacheMap<Object,AtomicLong>> entry */
typedef struct { int idx; so_cmap map; } thread_map;              /* Map<Integer, CacheMap<Object,AtomicInteger>> entry */
struct so_param_metric {
    rule_map* time_counters; int n_time, cap_time;       /* ruleTimeCounters  ParameterMetric.java:46 */
    rule_map* token_counters; int n_token, cap_token;    /* ruleTokenCounter  :50 */
    thread_map* thread_counts; int n_thread, cap_thread; /* threadCountMap    :54 */
    int lru;                                             /* CacheMaps are CLHM LRUs (else exact) */
    uint64_t spins;                                      /* evicted-token spins reached (never, see below) */
};
so_param_metric* so_pm_new_mode(int lru) {
    so_param_metric* pm = calloc(1, sizeof(so_param_metric));
    pm->lru = lru;
    return pm;
}
so_param_metric* so_pm_new(void) { return so_pm_new_mode(0); }
void so_pm_free(so_param_metric* pm) {
    if (!pm) return;
    for (int i = 0; i < pm->n_time; i++) cm_free(&pm->time_counters[i].map);
    for (int i = 0; i < pm->n_token; i++) cm_free(&pm->token_counters[i].map);
    for (int i = 0; i < pm->n_thread; i++) cm_free(&pm->thread_counts[i].map);
    free(pm->time_counters); free(pm->token_counters); free(pm->thread_counts); free(pm);
}
/* LRU evictions so far over all of the metric's maps (LRU mode) */
uint64_t so_pm_evictions(so_param_metric* pm) {
    uint64_t n = 0;
    if (!pm) return 0;
    for (int i = 0; i < pm->n_time; i++) if (pm->time_counters[i].map.lru) n += pm->time_counters[i].map.lru->evictions;
    for (int i = 0; i < pm->n_token; i++) if (pm->token_counters[i].map.lru) n += pm->token_counters[i].map.lru->evictions;
    for (int i = 0; i < pm->n_thread; i++) if (pm->thread_counts[i].map.lru) n += pm->thread_counts[i].map.lru->evictions;
    return n;
}
static so_cmap* rule_map_get(rule_map* arr, int n, int key) {
    for (int i = 0; i < n; i++) if (arr[i].key == key) return &arr[i].map;
    return NULL;
}
static so_cmap* thread_map_get(so_param_metric* pm, int idx) {
    for (int i = 0; i < pm->n_thread; i++) if (pm->thread_counts[i].idx == idx) return &pm->thread_counts[i].map;
    return NULL;
}
/* ParameterMetric.initialize — :99-121.  LRU capacities: BASE_PARAM_MAX_CAPACITY
 * (4000) x durationInSec capped at TOTAL_MAX_CAPACITY (200000) for the rule
 * maps, THREAD_COUNT_MAX_CAPACITY (4000) for the thread maps (:37-39). */
void so_pm_initialize(so_param_metric* pm, int key, const sf_param_rule* rule) {
    uint64_t cap = 0, tcap = 0;
    if (pm->lru) {
        int64_t c = jmul(4000, rule->duration_in_sec);
        cap = (uint64_t)(c < 200000 ? c : 200000);
        tcap = 4000;
        if (c <= 0) cap = 1;   /* invalid rules never get here (ParamFlowRuleUtil.isValidRule) */
    }
    if (!rule_map_get(pm->time_counters, pm->n_time, key)) {
        if (pm->n_time == pm->cap_time) { pm->cap_time = pm->cap_time ? pm->cap_time * 2 : 4;
            pm->time_counters = realloc(pm->time_counters, sizeof(rule_map) * pm->cap_time); }
        rule_map* r = &pm->time_counters[pm->n_time++]; r->key = key; r->present = 1; cm_init(&r->map, cap);
    }
    if (!rule_map_get(pm->token_counters, pm->n_token, key)) {
        if (pm->n_token == pm->cap_token) { pm->cap_token = pm->cap_token ? pm->cap_token * 2 : 4;
            pm->token_counters = realloc(pm->token_counters, sizeof(rule_map) * pm->cap_token); }
        rule_map* r = &pm->token_counters[pm->n_token++]; r->key = key; r->present = 1; cm_init(&r->map, cap);
    }
    if (!thread_map_get(pm, rule->param_idx)) {
        if (pm->n_thread == pm->cap_thread) { pm->cap_thread = pm->cap_thread ? pm->cap_thread * 2 : 4;
            pm->thread_counts = realloc(pm->thread_counts, sizeof(thread_map) * pm->cap_thread); }
        thread_map* t = &pm->thread_counts[pm->n_thread++]; t->idx = rule->param_idx; cm_init(&t->map, tcap);
    }
}
/* addThreadCount / decreaseThreadCount for one (index, value) — :184-239, :125-181 */
void so_pm_add_thread(so_param_metric* pm, int idx, uint8_t tag, uint64_t bits) {
    so_cmap* m = thread_map_get(pm, idx);
    if (!m || tag == SF_TAG_NULL) return;
    int64_t* v = cm_put_if_absent(m, tag, bits, 0);            /* putIfAbsent(new AtomicInteger()) */
    if (v) (*v) = (int32_t)((uint32_t)*v + 1u);                /* incrementAndGet */
    else cm_put(m, tag, bits, 1);                              /* put(value, new AtomicInteger(1)) */
}
void so_pm_dec_thread(so_param_metric* pm, int idx, uint8_t tag, uint64_t bits) {
    so_cmap* m = thread_map_get(pm, idx);
    if (!m || tag == SF_TAG_NULL) return;
    int64_t* v = cm_put_if_absent(m, tag, bits, 0);            /* putIfAbsent(new AtomicInteger()) */
    if (!v) return;
    int32_t cur = (int32_t)((uint32_t)*v - 1u);                /* decrementAndGet */
    *v = cur;
    if (cur <= 0) cm_remove(m, tag, bits);
}
/* getThreadCount — :242-250 (cacheMap.get: an access) */
int64_t so_pm_thread_count(so_param_metric* pm, int idx, uint8_t tag, uint64_t bits) {
    so_cmap* m = thread_map_get(pm, idx);
    if (!m) return 0;
    int64_t* v = cm_get(m, tag, bits);
    return v ? *v : 0;
}
int64_t so_pm_thread_peek(so_param_metric* pm, int idx, uint8_t tag, uint64_t bits) {
    so_cmap* m = thread_map_get(pm, idx);
    if (!m) return 0;
    int64_t* v = cm_peek(m, tag, bits);
    return v ? *v : 0;
}
int so_pm_read(so_param_metric* pm, int key, uint8_t tag, uint64_t bits,
               int64_t* time_value, int64_t* tokens, int* has_tokens) {
    so_cmap* tm = rule_map_get(pm->time_counters, pm->n_time, key);
    so_cmap* km = rule_map_get(pm->token_counters, pm->n_token, key);
    int64_t* t = tm ? cm_peek(tm, tag, bits) : NULL;
    int64_t* k = km ? cm_peek(km, tag, bits) : NULL;
    *time_value = t ? *t : 0; *tokens = k ? *k : 0; *has_tokens = k != NULL;
    return t != NULL;
}

static const sf_hot_item* hot_item(const sf_param_rule* rule, const sf_hot_item* items, uint8_t tag, uint64_t bits) {
    for (uint32_t i = 0; i < rule->item_count; i++) {
        const sf_hot_item* it = &items[rule->item_offset + i];
        if (it->tag == tag && it->bits == bits) return it;
    }
    return NULL;
}

/* ParamFlowChecker.passDefaultLocalCheck — ParamFlowChecker.java:139-219.
 * The map operations are the reference's, in its order (each an LRU access). */
static int pass_default_local(so_param_metric* pm, int key, const sf_param_rule* rule,
                              const sf_hot_item* items, int32_t acquire, uint8_t tag, uint64_t bits) {
    so_cmap* token_counters = rule_map_get(pm->token_counters, pm->n_token, key);
    so_cmap* time_counters = rule_map_get(pm->time_counters, pm->n_time, key);
    if (!token_counters || !time_counters) return 1;
    int64_t token_count = so_java_d2l(rule->count);
    const sf_hot_item* hi = tag == SF_TAG_NULL ? NULL : hot_item(rule, items, tag, bits);   /* no null hot item */
    if (hi) token_count = hi->count;
    if (token_count == 0) return 0;
    int64_t max_count = jadd(token_count, rule->burst_count);
    if (acquire > max_count) return 0;
    if (tag == SF_TAG_NULL) return 2;       /* timeCounters.putIfAbsent(null): NullPointerException */
    int64_t current_time = g_now;
    int64_t* last_add = cm_put_if_absent(time_counters, tag, bits, current_time);   /* :165 */
    if (!last_add) {                                                                 /* :166-169 */
        cm_put_if_absent(token_counters, tag, bits, max_count - acquire);
        return 1;
    }
    int64_t pass_time = current_time - *last_add;
    if (pass_time > jmul(rule->duration_in_sec, 1000)) {                              /* :173-195 */
        int64_t* old_qps = cm_put_if_absent(token_counters, tag, bits, max_count - acquire);
        if (!old_qps) {
            *last_add = current_time;
            return 1;
        }
        int64_t rest = *old_qps;
        int64_t to_add = jdiv(jmul(pass_time, token_count), jmul(rule->duration_in_sec, 1000));
        int64_t new_qps = jadd(to_add, rest) > max_count ? (max_count - acquire)
                                                          : jsub(jadd(rest, to_add), acquire);
        if (new_qps < 0) return 0;
        *old_qps = new_qps;                                     /* CAS succeeds */
        *last_add = current_time;
        return 1;
    }
    int64_t* old_qps = cm_get(token_counters, tag, bits);                             /* :196-215 */
    if (old_qps) {
        int64_t v = *old_qps;
        if (v - acquire >= 0) { *old_qps = v - acquire; return 1; }
        return 0;
    }
    /* Time entry present, token entry absent: the reference yields and loops
     * (:204-217) until a later clock passes the duration -- under the mocked
     * clock, forever.  Single-threaded it is unreachable even in LRU mode: the
     * two maps of a rule have one capacity and see the same operations in the
     * same order (putIfAbsent / get of the same key, every call above), so they
     * hold the same keys at all times.  Recorded, and answered as a block. */
    pm->spins++;
    return 0;
}
/* ParamFlowChecker.passThrottleLocalCheck — :222-273 */
static int pass_throttle_local(so_param_metric* pm, int key, const sf_param_rule* rule,
                               const sf_hot_item* items, int32_t acquire, uint8_t tag, uint64_t bits,
                               int64_t* wait_ms) {
    so_cmap* time_recorder = rule_map_get(pm->time_counters, pm->n_time, key);
    if (!time_recorder) return 1;
    int64_t token_count = so_java_d2l(rule->count);
    const sf_hot_item* hi = tag == SF_TAG_NULL ? NULL : hot_item(rule, items, tag, bits);
    if (hi) token_count = hi->count;
    if (token_count == 0) return 0;
    if (tag == SF_TAG_NULL) return 2;       /* timeRecorderMap.putIfAbsent(null): NullPointerException */
    int64_t cost = so_java_round(1.0 * 1000 * acquire * (double)rule->duration_in_sec / (double)token_count);
    int64_t current_time = g_now;
    int64_t* rec = cm_put_if_absent(time_recorder, tag, bits, current_time);
    if (!rec) return 1;
    int64_t last_pass = *rec;
    int64_t expected = last_pass + cost;
    if (expected <= current_time || expected - current_time < rule->max_queueing_time_ms) {
        rec = cm_get(time_recorder, tag, bits);                 /* timeRecorderMap.get(value) :255 */
        *rec = current_time;
        int64_t wait = expected - current_time;
        if (wait > 0) { *rec = expected; *wait_ms = wait; }
        return 1;
    }
    return 0;
}
/* ParamFlowChecker.passSingleValueCheck — :114-137.  1 pass, 0 block; 2 for a
 * null element of a collection: the parameter maps throw NullPointerException
 * (ConcurrentLinkedHashMap takes no null key) after the checks before them,
 * and passLocalCheck catches it (:108-110): the value passes, its loop ends. */
int so_param_pass_single(so_param_metric* pm, int key, const sf_param_rule* rule,
                         const sf_hot_item* items, int32_t acquire, uint8_t tag, uint64_t bits,
                         int64_t* wait_ms) {
    *wait_ms = 0;
    if (rule->grade == SF_GRADE_QPS) {
        if (rule->control_behavior == SF_BEHAVIOR_RATE_LIMITER)
            return pass_throttle_local(pm, key, rule, items, acquire, tag, bits, wait_ms);
        return pass_default_local(pm, key, rule, items, acquire, tag, bits);
    } else if (rule->grade == SF_GRADE_THREAD) {
        if (tag == SF_TAG_NULL) return 2;   /* getThreadCount: cacheMap.get(null) */
        int64_t thread_count = so_pm_thread_count(pm, rule->param_idx, tag, bits);
        const sf_hot_item* hi = hot_item(rule, items, tag, bits);
        if (hi) return ++thread_count <= hi->count;
        int64_t threshold = so_java_d2l(rule->count);
        return ++thread_count <= threshold;
    }
    return 1;
}

/* ======================================================================
 * Cluster server metrics — CS/flow/statistic/ (all)
 * ==================================================================== */
struct so_cluster_metric { so_leap_array* la; };                   /* ClusterMetric.java:28-37 */
so_cluster_metric* so_cm_new(int sample_count, int interval_ms) {
    so_cluster_metric* m = calloc(1, sizeof *m);
    m->la = so_la_new(SO_LA_CLUSTER, sample_count, interval_ms);
    return m;
}
void so_cm_free(so_cluster_metric* m) { if (m) { so_la_free(m->la); free(m); } }
void so_cm_add(so_cluster_metric* m, int event, int64_t n) {      /* :39-41 */
    so_wrap* w = so_la_current_window(m->la, g_now);
    ((cbucket*)w->value)->c[event] = jadd(((cbucket*)w->value)->c[event], n);
}
int64_t so_cm_sum(so_cluster_metric* m, int event) {              /* :47-55 */
    so_la_current_window(m->la, g_now);
    so_wrap* v[AM_MAXV];
    int n = so_la_values(m->la, g_now, v, AM_MAXV);
    int64_t s = 0;
    for (int i = 0; i < n; i++) s = jadd(s, ((cbucket*)v[i]->value)->c[event]);
    return s;
}
double so_cm_avg(so_cluster_metric* m, int event) {               /* :57-59 */
    return (double)so_cm_sum(m, event) / m->la->interval_sec;
}
/* tryOccupyNext — :69-79 ; canOccupy :81-86 ; getFirstCountOfWindow ClusterMetricLeapArray.java:83-92 */
int32_t so_cm_try_occupy_next(so_cluster_metric* m, int event, int32_t c, double threshold) {
    double latest_qps = so_cm_avg(m, CE_PASS);
    so_wrap* head = so_la_valid_head(m->la, g_now);
    int64_t head_pass = head ? ((cbucket*)head->value)->c[event] : 0;
    int64_t occupied = m->la->occupy[event];
    if (!(latest_qps + (double)(c + occupied) - (double)head_pass <= threshold)) return 0;
    m->la->occupy[CE_PASS] += c;                                  /* addOccupyPass :74-78 */
    m->la->occupy[CE_PASS_REQUEST] += 1;
    m->la->has_occupied = 1;
    so_cm_add(m, CE_WAITING, c);
    return 1000 / m->la->sample_count;
}

struct so_cluster_param_metric { so_leap_array* la; };             /* ClusterParamMetric.java:35-46 */
so_cluster_param_metric* so_cpm_new(int sample_count, int interval_ms) {
    so_cluster_param_metric* m = calloc(1, sizeof *m);
    m->la = so_la_new(SO_LA_CLUSTER_PARAM, sample_count, interval_ms);
    return m;
}
void so_cpm_free(so_cluster_param_metric* m) { if (m) { so_la_free(m->la); free(m); } }
int64_t so_cpm_sum(so_cluster_param_metric* m, uint8_t tag, uint64_t bits) {  /* :52-66 */
    if (tag == SF_TAG_NULL) return 0;
    so_la_current_window(m->la, g_now);
    so_wrap* v[AM_MAXV];
    int n = so_la_values(m->la, g_now, v, AM_MAXV);
    int64_t s = 0;
    for (int i = 0; i < n; i++) { int64_t* c = map_find((so_map*)v[i]->value, tag, bits); if (c) s = jadd(s, *c); }
    return s;
}
void so_cpm_add_value(so_cluster_param_metric* m, uint8_t tag, uint64_t bits, int32_t c) { /* :72-84 */
    if (tag == SF_TAG_NULL) return;
    so_map* data = (so_map*)so_la_current_window(m->la, g_now)->value;
    int64_t* cur = map_find(data, tag, bits);
    if (cur) *cur = jadd(*cur, c); else map_insert(data, tag, bits, c);
}
double so_cpm_avg(so_cluster_param_metric* m, uint8_t tag, uint64_t bits) {   /* :86-88 */
    return (double)so_cpm_sum(m, tag, bits) / m->la->interval_sec;
}

struct so_request_limiter { double qps_allowed; so_leap_array* data; };      /* RequestLimiter.java:29-45 */
so_request_limiter* so_rl_new(double qps_allowed) {
    so_request_limiter* l = calloc(1, sizeof *l);
    l->qps_allowed = qps_allowed; l->data = so_la_new(SO_LA_UNARY, 10, 1000);
    return l;
}
void so_rl_free(so_request_limiter* l) { if (l) { so_la_free(l->data); free(l); } }
int64_t so_rl_sum(so_request_limiter* l) {                                    /* :55-63 */
    so_la_current_window(l->data, g_now);
    so_wrap* v[AM_MAXV];
    int n = so_la_values(l->data, g_now, v, AM_MAXV);
    int64_t s = 0;
    for (int i = 0; i < n; i++) s = jadd(s, ((ubucket*)v[i]->value)->v);
    return s;
}
void so_rl_add(so_request_limiter* l, int32_t x) {                          /* :51-53 */
    ubucket* b = (ubucket*)so_la_current_window(l->data, g_now)->value;
    b->v = jadd(b->v, x);
}
int so_rl_can_pass(so_request_limiter* l) {                                   /* :72-74 */
    return (double)so_rl_sum(l) / l->data->interval_sec + 1 <= l->qps_allowed;
}
int so_rl_try_pass(so_request_limiter* l) {                                   /* :81-87 */
    if (so_rl_can_pass(l)) {
        ((ubucket*)so_la_current_window(l->data, g_now)->value)->v += 1;
        return 1;
    }
    return 0;
}

/* ======================================================================
 * Replay engine: StatisticSlot + SystemSlot + ParamFlowSlot + FlowSlot
 * per event, one ClusterNode per resource.
 * ==================================================================== */
typedef struct {
    sf_flow_rule rule;
    so_controller* ctrl;              /* FlowRuleUtil.generateRater :132-152 */
    int64_t ref_local;                /* RELATE: refResource's local id (-1: never a ClusterNode) */
} flow_rule_rt;

/* a StatisticNode keyed by an origin or a context name id */
typedef struct { uint32_t id; so_node* node; } keyed_node;

typedef struct {
    sf_param_rule rule;               /* param_idx mutated by applyRealParamIdx */
} param_rule_rt;

typedef struct {
    so_node* node;                    /* ClusterNode (null until first entry) */
    int* flow_rules; int n_flow;      /* indices into e->flow (list order)    */
    int* param_rules; int n_param;
    so_param_metric* pm;              /* ParameterMetricStorage entry          */
    int* cbs; int n_cb;               /* circuit breakers (indices into e->cb, rule list order) */
    /* ClusterNode.originCountMap (ClusterNode.java:101-120) and the resource's
     * DefaultNodes by context name (NodeSelectorSlot), kept for the resources
     * whose rules read them (the engine's set, sentinel_flow.h) */
    keyed_node* onodes; int n_on;
    keyed_node* dnodes; int n_dn;
} res_rt;

/* One CircuitBreaker (DegradeRuleManager.newCircuitBreakerFrom, :206-219) with
 * its LeapArray(1, statIntervalMs) counter (ResponseTimeCircuitBreaker.java:48-56,
 * ExceptionCircuitBreaker.java:47-56, AbstractCircuitBreaker.java:47-55). */
typedef struct {
    sf_degrade_rule rule;
    int64_t max_rt;                   /* Math.round(count) (ResponseTimeCircuitBreaker :52) */
    double threshold;                 /* slowRatioThreshold (RT) / count */
    int64_t recovery;                 /* timeWindow * 1000 */
    int state;                        /* SF_CB_* */
    int64_t next_retry;
    int has_bucket; int64_t ws, hit, total;
} so_breaker;

typedef struct {                      /* cluster flow / param rule state */
    int64_t flow_id; int is_param; double count; int threshold_type; uint32_t ns;
    uint32_t item_offset, item_count;
    so_cluster_metric* cm; so_cluster_param_metric* cpm;
} cluster_rt;

typedef struct { uint32_t id; int32_t connected; double max_qps; so_request_limiter* limiter; } ns_rt;

struct so_engine {
    sf_config cfg;
    res_rt* res; uint32_t n_res;
    flow_rule_rt* flow; uint32_t n_flow;
    param_rule_rt* param; uint32_t n_param;
    sf_hot_item* items; uint32_t n_items;
    /* SystemRuleManager static state :68-101 */
    int check_system_status;
    double highest_system_load, highest_cpu_usage, qps;
    int64_t max_rt, max_thread;
    int load_set, cpu_set;
    double cur_load, cur_cpu;
    so_node* entry_node;              /* Constants.ENTRY_NODE (Constants.java:66) */
    int report_set;                   /* so_set_report_entry_node: the ENTRY_NODE the metric log reports */
    sf_node_state report;
    /* entries of the batch being replayed */
    uint8_t* entry_blocked; uint32_t cap_entries;
    const uint8_t* forced;            /* so_submit_forced: planned SystemRule verdicts, ENTRY_NODE untouched */
    so_breaker* cb; uint32_t n_cb;    /* DegradeRuleManager's circuit breakers, load order of the valid rules */
    /* cluster */
    cluster_rt* cl; uint32_t n_cl;
    sf_hot_item* cl_items; uint32_t n_cl_items;
    ns_rt* ns; uint32_t n_ns;
    int param_lru;                    /* so_set_param_lru: ParameterMetric CacheMaps as CLHM LRUs */
};

/* ParameterMetric's CacheMaps bounded like the reference's (exact by default).
 * Takes effect for the metrics created afterwards: call before the first batch. */
int so_set_param_lru(so_engine* e, int on) { e->param_lru = on != 0; return 0; }
int so_param_lru_stats(so_engine* e, uint64_t* evictions, uint64_t* spins) {
    uint64_t ev = 0, sp = 0;
    for (uint32_t r = 0; r < e->n_res; r++)
        if (e->res[r].pm) { ev += so_pm_evictions(e->res[r].pm); sp += e->res[r].pm->spins; }
    *evictions = ev; *spins = sp;
    return 0;
}

static void apply_statics(const sf_config* cfg) {
    g_sample_count = cfg->sample_count; g_interval = cfg->interval_ms;
    g_occupy_timeout = cfg->occupy_timeout_ms; g_stat_max_rt = cfg->statistic_max_rt;
}

so_engine* so_create(const sf_config* cfg) {
    so_engine* e = calloc(1, sizeof *e);
    e->cfg = *cfg;
    if (e->cfg.shard_count == 0) e->cfg.shard_count = 1;
    e->n_res = cfg->max_resources;
    e->res = calloc(e->n_res ? e->n_res : 1, sizeof(res_rt));
    apply_statics(cfg);
    e->entry_node = so_node_new();
    e->highest_system_load = e->highest_cpu_usage = e->qps = 1.7976931348623157e308;
    e->max_rt = e->max_thread = INT64_MAX;
    return e;
}
static so_node* keyed_get(keyed_node** arr, int* n, uint32_t id, int create) {
    for (int k = 0; k < *n; k++) if ((*arr)[k].id == id) return (*arr)[k].node;
    if (!create) return NULL;
    *arr = realloc(*arr, sizeof(keyed_node) * (size_t)(*n + 1));
    (*arr)[*n].id = id; (*arr)[*n].node = so_node_new();
    return (*arr)[(*n)++].node;
}
static void clear_flow(so_engine* e) {
    for (uint32_t i = 0; i < e->n_flow; i++) so_ctrl_free(e->flow[i].ctrl);
    free(e->flow); e->flow = NULL; e->n_flow = 0;
    for (uint32_t r = 0; r < e->n_res; r++) { free(e->res[r].flow_rules); e->res[r].flow_rules = NULL; e->res[r].n_flow = 0; }
}
static void clear_param(so_engine* e) {
    free(e->param); e->param = NULL; e->n_param = 0;
    free(e->items); e->items = NULL; e->n_items = 0;
    for (uint32_t r = 0; r < e->n_res; r++) {
        free(e->res[r].param_rules); e->res[r].param_rules = NULL; e->res[r].n_param = 0;
        so_pm_free(e->res[r].pm); e->res[r].pm = NULL;
    }
}
void so_destroy(so_engine* e) {
    free(e->cb);
    for (uint32_t r = 0; e->res && r < e->n_res; r++) free(e->res[r].cbs);
    if (!e) return;
    clear_flow(e); clear_param(e);
    for (uint32_t r = 0; r < e->n_res; r++) {
        so_node_free(e->res[r].node);
        for (int k = 0; k < e->res[r].n_on; k++) so_node_free(e->res[r].onodes[k].node);
        for (int k = 0; k < e->res[r].n_dn; k++) so_node_free(e->res[r].dnodes[k].node);
        free(e->res[r].onodes); free(e->res[r].dnodes);
    }
    free(e->res);
    so_node_free(e->entry_node);
    free(e->entry_blocked);
    for (uint32_t i = 0; i < e->n_cl; i++) { so_cm_free(e->cl[i].cm); so_cpm_free(e->cl[i].cpm); }
    free(e->cl); free(e->cl_items);
    for (uint32_t i = 0; i < e->n_ns; i++) so_rl_free(e->ns[i].limiter);
    free(e->ns);
    free(e);
}
static int local_id(so_engine* e, uint32_t res, uint32_t* out) {
    if (res % e->cfg.shard_count != e->cfg.shard_index) return 0;
    uint32_t l = res / e->cfg.shard_count;
    if (l >= e->n_res) return 0;
    *out = l; return 1;
}
/* FlowRuleManager.loadRules -> FlowRuleUtil.buildFlowRuleMap (rules arrive in
 * Java iteration order; invalid rules are skipped as isValidRule does). */
int so_load_flow_rules(so_engine* e, const sf_flow_rule* rules, uint32_t n) {
    apply_statics(&e->cfg);
    clear_flow(e);
    e->flow = calloc(n ? n : 1, sizeof(flow_rule_rt));
    for (uint32_t i = 0; i < n; i++) {
        const sf_flow_rule* r = &rules[i];
        uint32_t l;
        if (!local_id(e, r->resource, &l)) return SF_ERR_INVALID;
        /* FlowRuleUtil.isValidRule :170-185 + checkControlBehaviorField :233-246 */
        int valid = r->count >= 0 && r->grade >= 0 && r->strategy >= 0 && r->control_behavior >= 0;
        /* checkStrategyField :236-241 (QPS grade only) */
        if (valid && r->grade == SF_GRADE_QPS && (r->strategy == SF_STRATEGY_RELATE || r->strategy == SF_STRATEGY_CHAIN) &&
            r->ref_resource == SF_REF_NONE)
            valid = 0;
        if (valid && r->grade == SF_GRADE_QPS) {
            if (r->control_behavior == SF_BEHAVIOR_WARM_UP) valid = r->warm_up_period_sec > 0;
            else if (r->control_behavior == SF_BEHAVIOR_RATE_LIMITER) valid = r->max_queueing_time_ms > 0;
            else if (r->control_behavior == SF_BEHAVIOR_WARM_UP_RATE_LIMITER)
                valid = r->warm_up_period_sec > 0 && r->max_queueing_time_ms > 0;
        } else if (valid && r->grade != SF_GRADE_THREAD) valid = 0;
        if (!valid) continue;
        flow_rule_rt* f = &e->flow[e->n_flow];
        f->rule = *r;
        f->ref_local = -1;
        if (r->strategy == SF_STRATEGY_RELATE && r->ref_resource != SF_REF_NONE) {
            if (r->ref_resource % e->cfg.shard_count != e->cfg.shard_index) return SF_ERR_UNSUPPORTED;
            if (r->ref_resource / e->cfg.shard_count < e->n_res) f->ref_local = r->ref_resource / e->cfg.shard_count;
        }
        /* generateRater :132-152 */
        if (r->grade == SF_GRADE_QPS && r->control_behavior == SF_BEHAVIOR_WARM_UP)
            f->ctrl = so_ctrl_warm_up(r->count, r->warm_up_period_sec, e->cfg.cold_factor);
        else if (r->grade == SF_GRADE_QPS && r->control_behavior == SF_BEHAVIOR_RATE_LIMITER)
            f->ctrl = so_ctrl_rate_limiter(r->max_queueing_time_ms, r->count);
        else if (r->grade == SF_GRADE_QPS && r->control_behavior == SF_BEHAVIOR_WARM_UP_RATE_LIMITER)
            f->ctrl = so_ctrl_warm_up_rate_limiter(r->count, r->warm_up_period_sec, r->max_queueing_time_ms, e->cfg.cold_factor);
        else
            f->ctrl = so_ctrl_default(r->count, r->grade);
        res_rt* rr = &e->res[l];
        rr->flow_rules = realloc(rr->flow_rules, sizeof(int) * (rr->n_flow + 1));
        rr->flow_rules[rr->n_flow++] = (int)e->n_flow;
        e->n_flow++;
    }
    return SF_OK;
}
int so_load_param_rules(so_engine* e, const sf_param_rule* rules, uint32_t n,
                        const sf_hot_item* items, uint32_t n_items) {
    clear_param(e);
    e->items = malloc(sizeof(sf_hot_item) * (n_items ? n_items : 1));
    if (n_items) memcpy(e->items, items, sizeof(sf_hot_item) * n_items);
    e->n_items = n_items;
    e->param = calloc(n ? n : 1, sizeof(param_rule_rt));
    for (uint32_t i = 0; i < n; i++) {
        uint32_t l;
        if (!local_id(e, rules[i].resource, &l)) return SF_ERR_INVALID;
        e->param[e->n_param].rule = rules[i];
        res_rt* rr = &e->res[l];
        rr->param_rules = realloc(rr->param_rules, sizeof(int) * (rr->n_param + 1));
        rr->param_rules[rr->n_param++] = (int)e->n_param;
        e->n_param++;
    }
    return SF_OK;
}
/* SystemRuleManager.SystemPropertyListener.configUpdate :173-196, loadSystemConf :267-289 */
int so_load_system_rules(so_engine* e, const sf_system_rule* rules, uint32_t n) {
    e->check_system_status = 0;
    e->highest_system_load = e->highest_cpu_usage = e->qps = 1.7976931348623157e308;
    e->max_rt = e->max_thread = INT64_MAX;
    e->load_set = e->cpu_set = 0;
    for (uint32_t i = 0; i < n; i++) {
        const sf_system_rule* r = &rules[i];
        int check = 0;
        if (r->highest_system_load >= 0) { e->highest_system_load = fmin(e->highest_system_load, r->highest_system_load); e->load_set = 1; check = 1; }
        if (r->highest_cpu_usage >= 0 && r->highest_cpu_usage <= 1) { e->highest_cpu_usage = fmin(e->highest_cpu_usage, r->highest_cpu_usage); e->cpu_set = 1; check = 1; }
        if (r->avg_rt >= 0) { if (r->avg_rt < e->max_rt) e->max_rt = r->avg_rt; check = 1; }
        if (r->max_thread >= 0) { if (r->max_thread < e->max_thread) e->max_thread = r->max_thread; check = 1; }
        if (r->qps >= 0) { e->qps = fmin(e->qps, r->qps); check = 1; }
        e->check_system_status = check;
    }
    return SF_OK;
}
/* ---- DegradeSlot (DegradeSlot.java:42-94) ---------------------------------
 * DegradeRuleManager.isValidRule :183-204 */
static int cb_valid(const sf_degrade_rule* r) {
    if (!(r->count >= 0) || r->time_window_s <= 0) return 0;
    if (r->min_request_amount <= 0 || r->stat_interval_ms <= 0) return 0;
    if (r->grade == SF_DEGRADE_GRADE_RT) return r->slow_ratio_threshold >= 0 && r->slow_ratio_threshold <= 1;
    if (r->grade == SF_DEGRADE_GRADE_EXCEPTION_RATIO) return r->count <= 1;
    return r->grade == SF_DEGRADE_GRADE_EXCEPTION_COUNT;
}
static int same_double(double a, double b) {   /* Double.compare(a, b) == 0 */
    if (a != a || b != b) return a != a && b != b;
    return memcmp(&a, &b, sizeof a) == 0;
}
/* DegradeRule.equals (DegradeRule.java:153-164) */
static int cb_rule_equal(const sf_degrade_rule* a, const sf_degrade_rule* b) {
    return a->resource == b->resource && a->grade == b->grade && same_double(a->count, b->count) &&
           a->time_window_s == b->time_window_s && a->min_request_amount == b->min_request_amount &&
           same_double(a->slow_ratio_threshold, b->slow_ratio_threshold) && a->stat_interval_ms == b->stat_interval_ms;
}

/* buildCircuitBreakers (:236-265) with getExistingSameCbOrNew (:151-163): an
 * equal rule of the resource keeps its breaker and state (two equal new rules
 * sharing one breaker are refused, like the engine). */
int so_load_degrade_rules(so_engine* e, const sf_degrade_rule* rules, uint32_t n, uint32_t* n_loaded) {
    so_breaker* nb = calloc(n ? n : 1, sizeof *nb);
    uint8_t* taken = calloc(e->n_cb ? e->n_cb : 1, 1);
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++) {
        const sf_degrade_rule* r = &rules[i];
        uint32_t l;
        if (!cb_valid(r)) continue;
        if (!local_id(e, r->resource, &l)) { free(nb); free(taken); return SF_ERR_INVALID; }
        int reuse = -1;
        for (uint32_t o = 0; o < e->n_cb; o++)
            if (cb_rule_equal(&e->cb[o].rule, r)) {
                if (taken[o]) { free(nb); free(taken); return SF_ERR_UNSUPPORTED; }
                reuse = (int)o; taken[o] = 1; break;
            }
        if (reuse >= 0) {
            nb[k] = e->cb[reuse];
        } else {
            so_breaker* b = &nb[k];
            b->rule = *r;
            b->max_rt = so_java_round(r->count);
            b->threshold = r->grade == SF_DEGRADE_GRADE_RT ? r->slow_ratio_threshold : r->count;
            b->recovery = (int64_t)r->time_window_s * 1000;
            b->state = SF_CB_CLOSED;
        }
        k++;
    }
    free(taken);
    free(e->cb);
    e->cb = nb; e->n_cb = k;
    for (uint32_t r = 0; r < e->n_res; r++) { free(e->res[r].cbs); e->res[r].cbs = NULL; e->res[r].n_cb = 0; }
    for (uint32_t c = 0; c < k; c++) {
        uint32_t l = 0;
        local_id(e, e->cb[c].rule.resource, &l);
        res_rt* rr = &e->res[l];
        rr->cbs = realloc(rr->cbs, (size_t)(rr->n_cb + 1) * sizeof(int));
        rr->cbs[rr->n_cb++] = (int)c;
    }
    if (n_loaded) *n_loaded = k;
    return SF_OK;
}

int so_read_breaker(so_engine* e, uint32_t k, sf_breaker_state* out) {
    if (k >= e->n_cb) return SF_ERR_INVALID;
    const so_breaker* b = &e->cb[k];
    memset(out, 0, sizeof *out);
    out->state = b->state; out->next_retry_ms = b->next_retry;
    out->window_start = b->has_bucket ? b->ws : SF_WS_ABSENT;
    out->hit_count = b->hit; out->total_count = b->total;
    return SF_OK;
}

/* LeapArray(1, interval).currentWindow(now) of the breaker's counter */
static void cb_current(so_breaker* b) {
    const int64_t ws = g_now - g_now % b->rule.stat_interval_ms;
    if (!b->has_bucket || ws > b->ws) { b->has_bucket = 1; b->ws = ws; b->hit = 0; b->total = 0; }
}
static void cb_to_open(so_breaker* b) {          /* transformToOpen + updateNextRetryTimestamp (:93-95) */
    b->state = SF_CB_OPEN;
    b->next_retry = g_now + b->recovery;
}
/* onRequestComplete + handleStateChangeWhenThresholdExceeded
 * (ResponseTimeCircuitBreaker.java:64-130, ExceptionCircuitBreaker.java:64-119) */
static void cb_on_complete(so_breaker* b, int64_t rt, int error) {
    cb_current(b);
    const int hit = b->rule.grade == SF_DEGRADE_GRADE_RT ? rt > b->max_rt : error != 0;
    b->hit += hit;
    b->total += 1;
    if (b->state == SF_CB_OPEN) return;
    if (b->state == SF_CB_HALF_OPEN) {
        if (hit) cb_to_open(b);                                           /* fromHalfOpenToOpen */
        else { b->state = SF_CB_CLOSED; cb_current(b); b->hit = b->total = 0; }   /* fromHalfOpenToClose + resetStat */
        return;
    }
    if (b->total < b->rule.min_request_amount) return;
    if (b->rule.grade == SF_DEGRADE_GRADE_RT) {
        const double ratio = b->hit * 1.0 / b->total;
        if (ratio > b->threshold || (ratio == b->threshold && b->threshold == 1.0)) cb_to_open(b);
    } else {
        const double cur = b->rule.grade == SF_DEGRADE_GRADE_EXCEPTION_RATIO ? b->hit * 1.0 / b->total : (double)b->hit;
        if (cur > b->threshold) cb_to_open(b);
    }
}
/* DegradeSlot.performChecking (:50-61): tryPass of each breaker
 * (AbstractCircuitBreaker.tryPass :67-82); the breakers the entry moved to
 * HALF_OPEN go back to OPEN when a later one refuses (whenTerminate :113-129).
 * Returns the refusing breaker's position in the resource list or -1. */
static int cb_check(so_engine* e, res_rt* rr) {
    int moved[SF_MAX_BREAKERS_PER_RESOURCE], n_moved = 0;
    for (int k = 0; k < rr->n_cb; k++) {
        so_breaker* b = &e->cb[rr->cbs[k]];
        if (b->state == SF_CB_CLOSED) continue;
        if (b->state == SF_CB_OPEN && g_now >= b->next_retry) {
            b->state = SF_CB_HALF_OPEN;
            if (n_moved < SF_MAX_BREAKERS_PER_RESOURCE) moved[n_moved++] = rr->cbs[k];
            continue;
        }
        for (int q = 0; q < n_moved; q++)
            if (e->cb[moved[q]].state == SF_CB_HALF_OPEN) e->cb[moved[q]].state = SF_CB_OPEN;
        return k;
    }
    return -1;
}

int so_set_system_status(so_engine* e, double load, double cpu) { e->cur_load = load; e->cur_cpu = cpu; return SF_OK; }

/* SystemRuleManager.checkSystem :291-340 ; checkBbr :342-348.  Returns -1 pass or the reason. */
static int check_system(so_engine* e, int32_t count) {
    if (!e->check_system_status) return -1;
    double current_qps = so_node_pass_qps(e->entry_node);
    if (current_qps + count > e->qps) return 0;
    int32_t current_thread = so_node_cur_thread_num(e->entry_node);
    if (current_thread > e->max_thread) return 1;
    double rt = so_node_avg_rt(e->entry_node);
    if (rt > (double)e->max_rt) return 2;
    if (e->load_set && e->cur_load > e->highest_system_load) {
        if (current_thread > 1 && current_thread > so_node_max_success_qps(e->entry_node) * so_node_min_rt(e->entry_node) / 1000)
            return 3;
    }
    if (e->cpu_set && e->cur_cpu > e->highest_cpu_usage) return 4;
    return -1;
}

static void arg_of(const sf_event_batch* in, uint32_t i, uint32_t slot, uint8_t* tag, uint64_t* bits) {
    *tag = in->arg_tag[(size_t)slot * in->n + i];
    *bits = in->arg_bits[(size_t)slot * in->n + i];
}
static uint32_t nargs_of(const sf_event_batch* in, uint32_t i) {
    if (in->arg_slots == 0 || !in->arg_tag) return 0;
    return in->n_args ? in->n_args[i] : in->arg_slots;
}

/* ParamFlowChecker.passLocalCheck — :84-112: the value, or every element of a
 * Collection / array in iteration order (earlier elements' tokens stay
 * consumed when a later one fails); a thrown exception passes the value. */
static int param_pass_value(so_param_metric* pm, int key, const sf_param_rule* rule, const sf_hot_item* items,
                            int32_t acquire, const sf_event_batch* in, uint32_t i, uint32_t slot, int64_t* wait_ms) {
    uint8_t tg; uint64_t bt; arg_of(in, i, slot, &tg, &bt);
    if (tg != SF_TAG_COLLECTION) return so_param_pass_single(pm, key, rule, items, acquire, tg, bt, wait_ms) != 0;
    *wait_ms = 0;
    const uint64_t k = (uint64_t)slot * in->n + i;
    for (uint32_t e = in->arg_elem_off[k]; e < in->arg_elem_off[k + 1]; e++) {
        int64_t w = 0;
        int ok = so_param_pass_single(pm, key, rule, items, acquire, in->elem_tag[e], in->elem_bits[e], &w);
        if (ok == 0) return 0;
        if (ok == 2) return 1;
        *wait_ms += w;
    }
    return 1;
}
/* ParameterMetric.addThreadCount / decreaseThreadCount — :125-239 over every
 * arg: null skipped, collections element by element; a null element throws
 * and ends the whole callback (one try around the loop over the args). */
static void pm_thread_event(so_param_metric* pm, const sf_event_batch* in, uint32_t i, uint32_t na, int add) {
    for (uint32_t s = 0; s < na; s++) {
        uint8_t tg; uint64_t bt; arg_of(in, i, s, &tg, &bt);
        if (tg != SF_TAG_COLLECTION) {
            if (add) so_pm_add_thread(pm, (int)s, tg, bt); else so_pm_dec_thread(pm, (int)s, tg, bt);
            continue;
        }
        if (!thread_map_get(pm, (int)s)) continue;
        const uint64_t k = (uint64_t)s * in->n + i;
        for (uint32_t e = in->arg_elem_off[k]; e < in->arg_elem_off[k + 1]; e++) {
            if (in->elem_tag[e] == SF_TAG_NULL) return;
            if (add) so_pm_add_thread(pm, (int)s, in->elem_tag[e], in->elem_bits[e]);
            else so_pm_dec_thread(pm, (int)s, in->elem_tag[e], in->elem_bits[e]);
        }
    }
}

/* FlowRuleManager.isOtherOrigin (FlowRuleManager.java:132-148): "" is never other */
static int is_other_origin(so_engine* e, const res_rt* rr, uint32_t origin) {
    if (origin == SF_ORIGIN_NONE) return 0;
    for (int k = 0; k < rr->n_flow; k++)
        if (e->flow[rr->flow_rules[k]].rule.limit_app == origin) return 0;
    return 1;
}
/* FlowRuleChecker.selectReferenceNode (:93-115) */
static int select_reference(const flow_rule_rt* f, uint32_t ctx) {
    if (f->rule.ref_resource == SF_REF_NONE) return SO_SEL_NONE;           /* StringUtil.isEmpty */
    if (f->rule.strategy == SF_STRATEGY_RELATE) return SO_SEL_REF;
    if (f->rule.strategy == SF_STRATEGY_CHAIN) return f->rule.ref_resource == ctx ? SO_SEL_CONTEXT : SO_SEL_NONE;
    return SO_SEL_NONE;
}
/* FlowRuleChecker.selectNodeByRequesterAndStrategy (:129-161); filterOrigin :117-120 */
static int select_node(so_engine* e, const res_rt* rr, const flow_rule_rt* f, uint32_t origin, uint32_t ctx) {
    const uint32_t app = f->rule.limit_app;
    const int direct = f->rule.strategy == SF_STRATEGY_DIRECT;
    if (origin != SF_ORIGIN_NONE && app == origin && origin != SF_APP_DEFAULT && origin != SF_APP_OTHER)
        return direct ? SO_SEL_ORIGIN : select_reference(f, ctx);
    if (app == SF_APP_DEFAULT) return direct ? SO_SEL_CLUSTER : select_reference(f, ctx);
    if (app == SF_APP_OTHER && is_other_origin(e, rr, origin)) return direct ? SO_SEL_ORIGIN : select_reference(f, ctx);
    return SO_SEL_NONE;
}
int so_select_node(so_engine* e, uint32_t rule_index, uint32_t origin, uint32_t context) {
    if (rule_index >= e->n_flow) return -1;
    uint32_t l = 0;
    if (!local_id(e, e->flow[rule_index].rule.resource, &l)) return -1;
    return select_node(e, &e->res[l], &e->flow[rule_index], origin, context);
}

int so_submit(so_engine* e, const sf_event_batch* in, sf_verdicts* out) {
    so_node* const en = e->forced ? NULL : e->entry_node;      /* the node-wide rounds update it themselves */
    apply_statics(&e->cfg);
    if (in->mem != SF_MEM_HOST || out->mem != SF_MEM_HOST) return SF_ERR_INVALID;
    if (in->n > e->cap_entries) {
        free(e->entry_blocked); e->cap_entries = in->n;
        e->entry_blocked = malloc(in->n ? in->n : 1);
    }
    for (uint32_t i = 0; i < in->n; i++) {
        g_now = in->ts_ms[i];                                   /* mocked TimeUtil for the whole event */
        uint32_t l;
        if (!local_id(e, in->res_id[i], &l)) return SF_ERR_INVALID;
        res_rt* rr = &e->res[l];
        int32_t count = in->count[i];
        uint8_t fl = in->flags[i];
        int is_in = (fl & SF_EV_IN) != 0;
        uint32_t na = nargs_of(in, i);
        uint8_t status = SF_V_PASS; int64_t wait = 0; int rule_idx = 0;
        /* Context: origin and name (ContextUtil.enter).  ClusterBuilderSlot
         * creates the origin node of every entry with an origin
         * (ClusterBuilderSlot.java:107-110: clusterNode.getOrCreateOriginNode);
         * the DefaultNode of (context, resource) is kept while a CHAIN rule of the
         * resource names the context (DESIGN.md §2 divergences) */
        const uint32_t origin = in->origin ? in->origin[i] : SF_ORIGIN_NONE;
        const uint32_t ctx = in->context ? in->context[i] : 0u;
        int want_dn = 0;
        for (int k = 0; k < rr->n_flow; k++) {
            const sf_flow_rule* fr = &e->flow[rr->flow_rules[k]].rule;
            if (fr->strategy == SF_STRATEGY_CHAIN && fr->ref_resource == ctx) want_dn = 1;
        }
        so_node* on = origin != SF_ORIGIN_NONE ? keyed_get(&rr->onodes, &rr->n_on, origin, 1) : NULL;
        so_node* dn = want_dn ? keyed_get(&rr->dnodes, &rr->n_dn, ctx, 1) : NULL;

        if (fl & SF_EV_EXIT) {
            /* StatisticSlot.exit :134-165 */
            int64_t ref = in->entry_ref ? in->entry_ref[i] : -1;
            int64_t create_ts;
            int blocked;
            if (ref >= 0) {
                if ((uint64_t)ref >= i) return SF_ERR_INVALID;
                blocked = e->entry_blocked[ref];
                create_ts = in->ts_ms[ref];
            } else {
                blocked = ref == -2;                            /* the entry was blocked in an earlier batch */
                create_ts = in->create_ts ? in->create_ts[i] : g_now;
            }
            if (!blocked) {
                if (!rr->node) rr->node = so_node_new();
                int64_t rt = g_now - create_ts;
                int err = (fl & SF_EV_ERROR) != 0;
                /* recordCompleteFor(DefaultNode -> ClusterNode), recordCompleteFor(originNode) :150-151, :167-178 */
                if (dn) { so_node_add_rt_and_success(dn, rt, count); so_node_decrease_thread_num(dn); if (err) so_node_increase_exception_qps(dn, count); }
                so_node_add_rt_and_success(rr->node, rt, count);
                so_node_decrease_thread_num(rr->node);
                if (err) so_node_increase_exception_qps(rr->node, count);
                if (on) { so_node_add_rt_and_success(on, rt, count); so_node_decrease_thread_num(on); if (err) so_node_increase_exception_qps(on, count); }
                if (is_in && en) {
                    so_node_add_rt_and_success(en, rt, count);
                    so_node_decrease_thread_num(en);
                    if (err) so_node_increase_exception_qps(en, count);
                }
                /* ParamFlowStatisticExitCallback.onExit -> decreaseThreadCount(args) */
                if (rr->pm) pm_thread_event(rr->pm, in, i, na, 0);
                /* DegradeSlot.exit :72-91: onRequestComplete of every breaker */
                for (int k = 0; k < rr->n_cb; k++) cb_on_complete(&e->cb[rr->cbs[k]], rt, err);
                status = SF_V_EXIT;
            } else {
                status = SF_V_EXIT_IGNORED;
            }
            e->entry_blocked[i] = 0;
            out->status[i] = status;
            if (out->wait_ms) out->wait_ms[i] = 0;
            if (out->rule_idx) out->rule_idx[i] = 0;
            continue;
        }

        /* ClusterBuilderSlot: ClusterNode created on the first entry */
        if (!rr->node) rr->node = so_node_new();
        int blocked = 0, prio_wait = 0;

        /* A slot StatisticSlot wraps but the engine does not run (AuthoritySlot,
         * order -6000 < SystemSlot -5000, Constants.java:80-84) threw a
         * BlockException: StatisticSlot counts it (StatisticSlot.java:102-124),
         * no later slot runs */
        if (fl & SF_EV_BLOCKED) { blocked = 1; status = SF_V_BLOCK_OTHER; }
        /* SystemSlot -> SystemRuleManager.checkSystem */
        if (is_in && !blocked) {
            int reason = e->forced ? (e->forced[i] == 0xFF ? -1 : (int)e->forced[i]) : check_system(e, count);
            if (reason >= 0) { blocked = 1; status = SF_V_BLOCK_SYSTEM; rule_idx = reason; }
        }
        /* ParamFlowSlot.checkFlow :82-103 (args never null from SphU.entry) */
        if (!blocked && rr->n_param > 0) {
            if (!rr->pm) rr->pm = so_pm_new_mode(e->param_lru);
            for (int k = 0; k < rr->n_param && !blocked; k++) {
                sf_param_rule* pr = &e->param[rr->param_rules[k]].rule;
                /* applyRealParamIdx :56-66 (mutates the rule) */
                if (pr->param_idx < 0) {
                    if (-pr->param_idx <= (int)na) pr->param_idx = (int)na + pr->param_idx;
                    else pr->param_idx = -pr->param_idx;
                }
                so_pm_initialize(rr->pm, rr->param_rules[k], pr);
                /* ParamFlowChecker.passCheck :48-67 */
                if ((int)na <= pr->param_idx) continue;
                uint8_t tg; uint64_t bt; arg_of(in, i, (uint32_t)pr->param_idx, &tg, &bt);
                if (tg == SF_TAG_NULL) continue;
                int64_t w = 0;
                if (!param_pass_value(rr->pm, rr->param_rules[k], pr, e->items, count, in, i, (uint32_t)pr->param_idx, &w)) {
                    blocked = 1; status = SF_V_BLOCK_PARAM; rule_idx = k;
                } else if (w > 0) {
                    wait += w;                                  /* throttle sleep inside the slot */
                }
            }
        }
        /* FlowSlot -> FlowRuleChecker.checkFlow :44-59 */
        if (!blocked) {
            for (int k = 0; k < rr->n_flow; k++) {
                flow_rule_rt* f = &e->flow[rr->flow_rules[k]];
                int64_t w = 0; int pw = 0;
                /* canPassCheck :66-80: a cluster rule finds no TokenService (ClusterStateManager not
                 * started, pickClusterService :195-203) -> fallbackToLocalOrPass :184-193 */
                if (f->rule.cluster_mode && !f->rule.cluster_fallback) continue;
                /* passLocalCheck :82-91 -> selectNodeByRequesterAndStrategy; no node -> pass */
                so_node* sel = NULL;
                switch (select_node(e, rr, f, origin, ctx)) {
                case SO_SEL_CLUSTER: sel = rr->node; break;
                case SO_SEL_ORIGIN: sel = on; break;
                case SO_SEL_CONTEXT: sel = dn; break;
                case SO_SEL_REF: sel = f->ref_local >= 0 ? e->res[f->ref_local].node : NULL; break;  /* getClusterNode */
                default: break;
                }
                if (!sel) continue;
                int ok = so_ctrl_can_pass(f->ctrl, sel, NULL, count, (fl & SF_EV_PRIO) != 0, &w, &pw);
                if (pw) { prio_wait = 1; wait += w; rule_idx = k; break; }  /* PriorityWaitException */
                if (!ok) { blocked = 1; status = SF_V_BLOCK_FLOW; rule_idx = k; break; }
                wait += w;
            }
        }
        /* DegradeSlot.entry (DegradeSlot.java:42-61), the last slot: not reached
         * after a block or a PriorityWaitException from FlowSlot */
        if (!blocked && !prio_wait && rr->n_cb) {
            const int k = cb_check(e, rr);
            if (k >= 0) { blocked = 1; status = SF_V_BLOCK_DEGRADE; rule_idx = k; }
        }
        /* StatisticSlot.entry accounting :64-123 (DefaultNode -> ClusterNode, origin node) */
        if (blocked) {
            if (dn) so_node_increase_block_qps(dn, count);
            so_node_increase_block_qps(rr->node, count);
            if (on) so_node_increase_block_qps(on, count);
            if (is_in && en) so_node_increase_block_qps(en, count);
        } else if (prio_wait) {
            if (dn) so_node_increase_thread_num(dn);
            so_node_increase_thread_num(rr->node);
            if (on) so_node_increase_thread_num(on);
            if (is_in && en) so_node_increase_thread_num(en);
            if (rr->pm) pm_thread_event(rr->pm, in, i, na, 1);
            status = SF_V_PRIORITY_WAIT;
        } else {
            if (dn) { so_node_increase_thread_num(dn); so_node_add_pass_request(dn, count); }
            so_node_increase_thread_num(rr->node);
            so_node_add_pass_request(rr->node, count);
            if (on) { so_node_increase_thread_num(on); so_node_add_pass_request(on, count); }
            if (is_in && en) { so_node_increase_thread_num(en); so_node_add_pass_request(en, count); }
            if (rr->pm) pm_thread_event(rr->pm, in, i, na, 1);
            status = wait > 0 ? SF_V_PASS_WAIT : SF_V_PASS;
        }
        e->entry_blocked[i] = (uint8_t)blocked;
        out->status[i] = status;
        if (out->wait_ms) out->wait_ms[i] = (int32_t)wait;
        if (out->rule_idx) out->rule_idx[i] = (uint16_t)rule_idx;
    }
    return SF_OK;
}

/* The node-wide SystemRule rounds of a sharded node (include/sentinel_flow.h:
 * sf_system_plan / sf_submit_forced / sf_entry_node_add), restated one IN event
 * per round: the plan of merged[p] is checkSystem on the ENTRY_NODE as every
 * earlier IN event of the node left it (SystemRuleManager.checkSystem
 * :291-348; StatisticSlot.java:64-165 the updates). */
int so_system_plan(so_engine* e, const sf_event_batch* in, const uint8_t* status, uint32_t p, uint32_t* q,
                   uint8_t* sys_mask) {
    (void)status;
    if (p >= in->n) return SF_ERR_INVALID;
    apply_statics(&e->cfg);
    g_now = in->ts_ms[p];
    const uint8_t f = in->flags[p];
    int reason = -1;
    if ((f & SF_EV_IN) && !(f & (SF_EV_EXIT | SF_EV_BLOCKED))) reason = check_system(e, in->count[p]);
    sys_mask[p] = reason < 0 ? 0xFF : (uint8_t)reason;
    *q = p + 1;
    return SF_OK;
}

int so_submit_forced(so_engine* e, const sf_event_batch* in, sf_verdicts* out, const uint8_t* sys_mask) {
    e->forced = sys_mask;
    const int rc = so_submit(e, in, out);
    e->forced = NULL;
    return rc;
}

int so_entry_node_add(so_engine* e, const sf_event_batch* in, const uint8_t* status) {
    apply_statics(&e->cfg);
    so_node* en = e->entry_node;
    for (uint32_t i = 0; i < in->n; i++) {
        const uint8_t f = in->flags[i], v = status[i];
        if (!(f & SF_EV_IN)) continue;
        g_now = in->ts_ms[i];
        const int32_t c = in->count[i];
        if (f & SF_EV_EXIT) {
            if (v != SF_V_EXIT) continue;
            const int64_t ref = in->entry_ref ? in->entry_ref[i] : -1;
            const int64_t cts = ref >= 0 ? in->ts_ms[ref] : (in->create_ts ? in->create_ts[i] : g_now);
            so_node_add_rt_and_success(en, g_now - cts, c);
            so_node_decrease_thread_num(en);
            if (f & SF_EV_ERROR) so_node_increase_exception_qps(en, c);
        } else if (v == SF_V_PASS || v == SF_V_PASS_WAIT) {
            so_node_increase_thread_num(en);
            so_node_add_pass_request(en, c);
        } else if (v == SF_V_PRIORITY_WAIT) {
            so_node_increase_thread_num(en);
        } else {
            so_node_increase_block_qps(en, c);
        }
    }
    return SF_OK;
}

int so_read_node(so_engine* e, uint32_t res, sf_node_state* out) {
    uint32_t l;
    if (!local_id(e, res, &l)) return SF_ERR_INVALID;
    so_node_read(e->res[l].node, out);
    return SF_OK;
}
int so_read_entry_node(so_engine* e, sf_node_state* out) { so_node_read(e->entry_node, out); return SF_OK; }
int so_read_origin_node(so_engine* e, uint32_t res, uint32_t origin, sf_node_state* out) {
    uint32_t l;
    if (!local_id(e, res, &l)) return SF_ERR_INVALID;
    so_node* n = keyed_get(&e->res[l].onodes, &e->res[l].n_on, origin, 0);
    if (!n) return SF_ERR_INVALID;
    so_node_read(n, out);
    return SF_OK;
}
int so_read_context_node(so_engine* e, uint32_t context, uint32_t res, sf_node_state* out) {
    uint32_t l;
    if (!local_id(e, res, &l)) return SF_ERR_INVALID;
    so_node* n = keyed_get(&e->res[l].dnodes, &e->res[l].n_dn, context, 0);
    if (!n) return SF_ERR_INVALID;
    so_node_read(n, out);
    return SF_OK;
}
int so_read_rule_state(so_engine* e, uint32_t idx, sf_rule_state* out) {
    if (idx >= e->n_flow) return SF_ERR_INVALID;
    so_ctrl_state(e->flow[idx].ctrl, out);
    return SF_OK;
}
/* Whole-engine state comparison (bench.py steady-state check, tests): one
 * FNV-1a digest per local resource row over its canonical sf_node_state words
 * -- for i < sample_count: second[i] (window_start, pass, block, exception,
 * success, rt, occupied_pass, min_rt), borrow_ws[i], borrow_pass[i]; then the
 * 60 minute buckets; then cur_thread_num -- the same word order
 * include/sentinel_flow.h sf_node_digests gives the engine's rows. */
static uint64_t fnv_words(uint64_t h, const int64_t* w, int n) {
    for (int i = 0; i < n; i++) { h ^= (uint64_t)w[i]; h *= 0x100000001b3ull; }
    return h;
}
uint64_t so_node_digest(const sf_node_state* s, int sample_count) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (int i = 0; i < sample_count; i++) {
        h = fnv_words(h, &s->second[i].window_start, 8);
        h = fnv_words(h, &s->borrow_ws[i], 1);
        h = fnv_words(h, &s->borrow_pass[i], 1);
    }
    for (int i = 0; i < SF_MINUTE_BUCKETS; i++) h = fnv_words(h, &s->minute[i].window_start, 8);
    return fnv_words(h, &s->cur_thread_num, 1);
}
int so_node_digests(so_engine* e, uint64_t* out, uint32_t n) {
    sf_node_state st;
    for (uint32_t l = 0; l < n; l++) {
        so_node_read(l < e->n_res ? e->res[l].node : NULL, &st);
        out[l] = so_node_digest(&st, e->cfg.sample_count);
    }
    return SF_OK;
}
int so_read_rule_states(so_engine* e, uint32_t first, uint32_t n, sf_rule_state* out) {
    if ((uint64_t)first + n > e->n_flow) return SF_ERR_INVALID;
    for (uint32_t i = 0; i < n; i++) so_ctrl_state(e->flow[first + i].ctrl, &out[i]);
    return SF_OK;
}
int so_read_param(so_engine* e, uint32_t pidx, uint8_t tag, uint64_t bits,
                  int64_t* time_value, int64_t* tokens, int* has_tokens) {
    if (pidx >= e->n_param) return SF_ERR_INVALID;
    uint32_t l;
    if (!local_id(e, e->param[pidx].rule.resource, &l)) return SF_ERR_INVALID;
    if (!e->res[l].pm) { *time_value = 0; *tokens = 0; *has_tokens = 0; return 0; }
    return so_pm_read(e->res[l].pm, (int)pidx, tag, bits, time_value, tokens, has_tokens);
}
int32_t so_param_rule_idx(so_engine* e, uint32_t pidx) {
    return pidx < e->n_param ? e->param[pidx].rule.param_idx : INT32_MIN;
}
int64_t so_param_thread(so_engine* e, uint32_t res, int idx, uint8_t tag, uint64_t bits) {
    uint32_t l;
    if (!local_id(e, res, &l) || !e->res[l].pm) return 0;
    return so_pm_thread_peek(e->res[l].pm, idx, tag, bits);
}
/* StatisticNode.metrics() :120-137 of one node: rows appended at out[*k] */
static void node_metrics(so_node* n, int64_t now, uint32_t resource, sf_metric_row* out, uint32_t cap, uint32_t* k) {
    int64_t current_time = now - now % 1000;
    sf_metric_row rows[64];
    int nr = so_am_details(n->minute, 0, 0, rows, 64);
    int64_t new_last = n->last_fetch_time;
    for (int j = 0; j < nr && j < 64; j++) {
        sf_metric_row* r = &rows[j];
        int in_time = r->timestamp > n->last_fetch_time && r->timestamp < current_time;     /* isNodeInTime :144-146 */
        int valid = r->pass_qps > 0 || r->block_qps > 0 || r->success_qps > 0 || r->exception_qps > 0
                    || r->rt > 0 || r->occupied_pass_qps > 0;                                /* isValidMetricNode :148-151 */
        if (in_time && valid) {
            r->resource = resource;
            if (*k < cap) out[*k] = *r;
            (*k)++;
            if (r->timestamp > new_last) new_last = r->timestamp;
        }
    }
    n->last_fetch_time = new_last;
}

/* StatisticNode.metrics() per ClusterNode :120-137 (MetricTimerListener.java:40-69) */
int so_snapshot(so_engine* e, int64_t now, sf_metric_row* out, uint32_t cap, uint32_t* n_out) {
    uint32_t k = 0;
    g_now = now;
    for (uint32_t l = 0; l < e->n_res; l++)
        if (e->res[l].node) node_metrics(e->res[l].node, now, l * e->cfg.shard_count + e->cfg.shard_index, out, cap, &k);
    *n_out = k;
    return k <= cap ? SF_OK : SF_ERR_CAPACITY;
}

/* ---- metrics.log lines ------------------------------------------------
 * MetricNode.toFatString (CORE/node/metric/MetricNode.java:213-229):
 * timestamp|yyyy-MM-dd HH:mm:ss|name('|'->'_')|pass|block|success|exception|rt|occupiedPass|concurrency|classification\n
 * SimpleDateFormat in a fixed zone of tz_offset_ms (no DST). */
static const char* const ENTRY_NAME = "__total_inbound_traffic__";   /* Constants.java:45 */

static size_t fat_line(const sf_metric_row* r, const char* name, size_t name_len, int32_t cls, int64_t tz,
                       char* buf, size_t cap) {
    int64_t t = r->timestamp + tz;
    int64_t days = t / 86400000, msd = t % 86400000;
    if (msd < 0) { msd += 86400000; days--; }
    /* civil date of a day count (proleptic Gregorian, as java.util.GregorianCalendar after 1582) */
    int64_t z = days + 719468, era = (z >= 0 ? z : z - 146096) / 146097;
    int64_t doe = z - era * 146097, yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t y = yoe + era * 400, doy = doe - (365 * yoe + yoe / 4 - yoe / 100), mp = (5 * doy + 2) / 153;
    int64_t d = doy - (153 * mp + 2) / 5 + 1, m = mp < 10 ? mp + 3 : mp - 9;
    if (m <= 2) y++;
    char nm[4096];
    size_t nl = name_len < sizeof nm - 1 ? name_len : sizeof nm - 1;
    for (size_t i = 0; i < nl; i++) nm[i] = name[i] == '|' ? '_' : name[i];
    nm[nl] = 0;
    int w = snprintf(buf, cap, "%lld|%04lld-%02lld-%02lld %02lld:%02lld:%02lld|%s|%lld|%lld|%lld|%lld|%lld|%lld|%d|%d\n",
                     (long long)r->timestamp, (long long)y, (long long)m, (long long)d, (long long)(msd / 3600000),
                     (long long)(msd / 60000 % 60), (long long)(msd / 1000 % 60), nm, (long long)r->pass_qps,
                     (long long)r->block_qps, (long long)r->success_qps, (long long)r->exception_qps,
                     (long long)r->rt, (long long)r->occupied_pass_qps, (int)r->concurrency, (int)cls);
    return w < 0 ? 0 : (size_t)w;
}

static void row_name(const so_names* nt, uint32_t res, const char** name, size_t* len, int32_t* cls, char* tmp) {
    *cls = 0;
    if (res == SF_RES_ENTRY_NODE) { *name = ENTRY_NAME; *len = strlen(ENTRY_NAME); return; }
    if (nt && res < nt->n) {
        *name = nt->bytes + nt->offsets[res]; *len = (size_t)(nt->offsets[res + 1] - nt->offsets[res]);
        if (nt->types) *cls = nt->types[res];
        return;
    }
    *len = (size_t)sprintf(tmp, "%u", res); *name = tmp;    /* no name loaded: the resource id */
}

int so_format_fat(const so_names* nt, const sf_metric_row* rows, uint32_t n, int64_t tz_offset_ms, char* out,
                  uint64_t cap, uint64_t* len_out) {
    uint64_t o = 0;
    char line[8192], tmp[16];
    for (uint32_t i = 0; i < n; i++) {
        const char* nm; size_t nl; int32_t cls;
        row_name(nt, rows[i].resource, &nm, &nl, &cls, tmp);
        size_t w = fat_line(&rows[i], nm, nl, cls, tz_offset_ms, line, sizeof line);
        if (o + w <= cap) memcpy(out + o, line, w);
        o += w;
    }
    *len_out = o;
    return o <= cap ? SF_OK : SF_ERR_CAPACITY;
}

/* MetricTimerListener.run (CORE/node/metric/MetricTimerListener.java:40-69):
 * every ClusterNode's metrics() (resources in id order: the reference walks a
 * HashMap, whose order is not reproducible), then ENTRY_NODE's, grouped by
 * second in a TreeMap; MetricWriter.write(time, nodes) (MetricWriter.java:120-170)
 * appends each node's toFatString in list order. */
typedef struct { int64_t ts; uint32_t pos; } ts_pos;
static int cmp_ts(const void* a, const void* b) {
    const ts_pos *x = a, *y = b;
    if (x->ts != y->ts) return x->ts < y->ts ? -1 : 1;
    return x->pos < y->pos ? -1 : x->pos > y->pos;    /* list position: stable */
}
/* A node holding the given windows (restated state: each stored WindowWrap
 * with its counters), for the reported ENTRY_NODE. */
static so_node* node_from_state(const sf_node_state* st) {
    so_node* n = so_node_new();
    so_leap_array* m = n->minute->data;
    for (int i = 0; i < SF_MINUTE_BUCKETS; i++) {
        const sf_bucket* b = &st->minute[i];
        if (b->window_start == SF_WS_ABSENT) continue;
        so_wrap* w = new_wrap(m, b->window_start, b->window_start);
        mbucket* v = w->value;
        v->c[EV_PASS] = b->pass; v->c[EV_BLOCK] = b->block; v->c[EV_EXCEPTION] = b->exception;
        v->c[EV_SUCCESS] = b->success; v->c[EV_RT] = b->rt; v->c[EV_OCCUPIED_PASS] = b->occupied_pass;
        v->min_rt = b->min_rt;
        m->array[i] = w;
    }
    n->cur_thread_num = st->cur_thread_num;
    return n;
}
int so_set_report_entry_node(so_engine* e, const sf_node_state* node) {
    e->report_set = node != NULL;
    if (node) e->report = *node;
    return SF_OK;
}
int so_metric_log(so_engine* e, const so_names* nt, int64_t now, int64_t tz_offset_ms, int include_entry_node,
                  char* out, uint64_t cap, uint64_t* len_out, uint32_t* n_lines) {
    uint32_t k = 0, cap_rows = 1024;
    sf_metric_row* rows = malloc(cap_rows * sizeof *rows);
    g_now = now;
    /* MetricTimerListener reads Constants.ENTRY_NODE: on a sharded node the
     * node-wide merge, when set (lastFetchTime stays this engine's) */
    so_node* rep = NULL;
    if (include_entry_node && e->report_set) {
        rep = node_from_state(&e->report);
        rep->last_fetch_time = e->entry_node->last_fetch_time;
    }
    for (uint32_t l = 0; l <= e->n_res; l++) {
        so_node* n = l < e->n_res ? e->res[l].node : (include_entry_node ? (rep ? rep : e->entry_node) : NULL);
        if (!n) continue;
        if (k + 64 > cap_rows) { cap_rows = 2 * (k + 64); rows = realloc(rows, cap_rows * sizeof *rows); }
        node_metrics(n, now, l < e->n_res ? l * e->cfg.shard_count + e->cfg.shard_index : SF_RES_ENTRY_NODE,
                     rows, cap_rows, &k);
    }
    ts_pos* order = malloc((k ? k : 1) * sizeof *order);
    sf_metric_row* sorted = malloc((k ? k : 1) * sizeof *sorted);
    for (uint32_t i = 0; i < k; i++) { order[i].ts = rows[i].timestamp; order[i].pos = i; }
    qsort(order, k, sizeof *order, cmp_ts);
    for (uint32_t i = 0; i < k; i++) sorted[i] = rows[order[i].pos];
    if (rep) { e->entry_node->last_fetch_time = rep->last_fetch_time; so_node_free(rep); }
    int rc = so_format_fat(nt, sorted, k, tz_offset_ms, out, cap, len_out);
    free(rows); free(order); free(sorted);
    *n_lines = k;
    return rc;
}

/* ---- cluster token server: DefaultTokenService / ClusterFlowChecker ---- */
int so_load_namespaces(so_engine* e, const sf_namespace* ns, uint32_t n) {
    for (uint32_t i = 0; i < e->n_ns; i++) so_rl_free(e->ns[i].limiter);
    free(e->ns);
    e->ns = calloc(n ? n : 1, sizeof(ns_rt)); e->n_ns = n;
    for (uint32_t i = 0; i < n; i++) {
        e->ns[i].id = ns[i].namespace_id; e->ns[i].connected = ns[i].connected_count;
        e->ns[i].max_qps = ns[i].max_allowed_qps;
        /* GlobalRequestLimiter.initIfAbsent :36-41 */
        e->ns[i].limiter = ns[i].max_allowed_qps >= 0 ? so_rl_new(ns[i].max_allowed_qps) : NULL;
    }
    return SF_OK;
}
int so_load_cluster_rules(so_engine* e, const sf_cluster_flow_rule* flow, uint32_t n_flow,
                          const sf_cluster_param_rule* param, uint32_t n_param,
                          const sf_hot_item* items, uint32_t n_items) {
    for (uint32_t i = 0; i < e->n_cl; i++) { so_cm_free(e->cl[i].cm); so_cpm_free(e->cl[i].cpm); }
    free(e->cl); free(e->cl_items);
    e->n_cl = n_flow + n_param;
    e->cl = calloc(e->n_cl ? e->n_cl : 1, sizeof(cluster_rt));
    e->cl_items = malloc(sizeof(sf_hot_item) * (n_items ? n_items : 1));
    if (n_items) memcpy(e->cl_items, items, sizeof(sf_hot_item) * n_items);
    e->n_cl_items = n_items;
    for (uint32_t i = 0; i < n_flow; i++) {
        cluster_rt* c = &e->cl[i];
        c->flow_id = flow[i].flow_id; c->count = flow[i].count; c->threshold_type = flow[i].threshold_type;
        c->ns = flow[i].namespace_id;
        c->cm = so_cm_new(flow[i].sample_count, flow[i].window_interval_ms);   /* ClusterFlowRuleManager.java:361-362 */
    }
    for (uint32_t i = 0; i < n_param; i++) {
        cluster_rt* c = &e->cl[n_flow + i];
        c->flow_id = param[i].flow_id; c->count = param[i].count; c->threshold_type = param[i].threshold_type;
        c->ns = param[i].namespace_id; c->is_param = 1;
        c->item_offset = param[i].item_offset; c->item_count = param[i].item_count;
        c->cpm = so_cpm_new(param[i].sample_count, param[i].window_interval_ms); /* ClusterParamFlowRuleManager.java:354-355 */
    }
    return SF_OK;
}
static ns_rt* find_ns(so_engine* e, uint32_t id) {
    for (uint32_t i = 0; i < e->n_ns; i++) if (e->ns[i].id == id) return &e->ns[i];
    return NULL;
}
static cluster_rt* find_cl(so_engine* e, int64_t id, int is_param) {
    for (uint32_t i = 0; i < e->n_cl; i++) if (e->cl[i].flow_id == id && e->cl[i].is_param == is_param) return &e->cl[i];
    return NULL;
}
int64_t so_cluster_sum(so_engine* e, int64_t flow_id, int event, int64_t now) {
    cluster_rt* c = find_cl(e, flow_id, 0);
    if (!c) return 0;
    g_now = now;
    return so_cm_sum(c->cm, event);
}
int so_request_tokens(so_engine* e, const sf_token_batch* in, sf_token_results* out) {
    if (in->mem != SF_MEM_HOST || out->mem != SF_MEM_HOST) return SF_ERR_INVALID;
    for (uint32_t i = 0; i < in->n; i++) {
        g_now = in->ts_ms[i];
        int64_t id = in->flow_id[i];
        int32_t count = in->count[i];
        int is_param = (in->flags[i] & SF_TOK_PARAM) != 0;
        int prio = (in->flags[i] & SF_TOK_PRIORITIZED) != 0;
        int8_t st; int32_t remaining = 0, wait = 0;
        if (id <= 0 || count <= 0) {                                   /* DefaultTokenService.notValidRequest :70-72 */
            st = SF_TOKEN_BAD_REQUEST;
        } else if (is_param && (!in->param_tag || !in->param_bits ||
                                (in->param_off && in->param_off[i + 1] == in->param_off[i]))) {
            st = SF_TOKEN_BAD_REQUEST;                                  /* params == null || isEmpty :52-54 */
        } else {
            cluster_rt* c = find_cl(e, id, is_param);
            if (!c) st = SF_TOKEN_NO_RULE_EXISTS;
            else {
                ns_rt* ns = find_ns(e, c->ns);
                /* allowProceed -> GlobalRequestLimiter.tryPass :46-55 (namespace not null) */
                int allow = (ns == NULL || ns->limiter == NULL) ? 1 : so_rl_try_pass(ns->limiter);
                int connected = ns ? ns->connected : 0;
                if (!allow) st = SF_TOKEN_TOO_MANY_REQUEST;
                else if (!is_param) {
                    /* ClusterFlowChecker.acquireClusterToken :55-112 */
                    so_cluster_metric* m = c->cm;
                    double latest_qps = so_cm_avg(m, CE_PASS);
                    double global_threshold = (c->threshold_type == SF_THRESHOLD_GLOBAL ? c->count : c->count * connected)
                                              * e->cfg.exceed_count;
                    double next_remaining = global_threshold - latest_qps - count;
                    if (next_remaining >= 0) {
                        so_cm_add(m, CE_PASS, count); so_cm_add(m, CE_PASS_REQUEST, 1);
                        if (prio) so_cm_add(m, CE_OCCUPIED_PASS, count);
                        st = SF_TOKEN_OK; remaining = so_java_d2i(next_remaining);
                    } else {
                        int waited = 0;
                        if (prio) {
                            double occupy_avg = so_cm_avg(m, CE_WAITING);
                            if (occupy_avg <= e->cfg.max_occupy_ratio * global_threshold) {
                                int32_t w = so_cm_try_occupy_next(m, CE_PASS, count, global_threshold);
                                if (w > 0) { st = SF_TOKEN_SHOULD_WAIT; wait = w; waited = 1; }
                            }
                        }
                        if (!waited) {
                            so_cm_add(m, CE_BLOCK, count); so_cm_add(m, CE_BLOCK_REQUEST, 1);
                            if (prio) so_cm_add(m, CE_OCCUPIED_BLOCK, count);
                            st = SF_TOKEN_BLOCKED;
                        }
                    }
                } else {
                    /* ClusterParamFlowChecker.acquireClusterToken :42-87: every value
                     * must have room (the first without stops the check), then all are added */
                    const uint32_t v0 = in->param_off ? in->param_off[i] : i;
                    const uint32_t v1 = in->param_off ? in->param_off[i + 1] : i + 1;
                    double rem = -1;
                    int passed = 1;
                    for (uint32_t v = v0; v < v1; v++) {
                        uint8_t tg = in->param_tag[v]; uint64_t bt = in->param_bits[v];
                        double latest_qps = so_cpm_avg(c->cpm, tg, bt);
                        double raw = c->count;                              /* getRawThreshold :110-117 */
                        for (uint32_t k = 0; k < c->item_count; k++) {
                            const sf_hot_item* it = &e->cl_items[c->item_offset + k];
                            if (it->tag == tg && it->bits == bt) { raw = it->count; break; }
                        }
                        double threshold = c->threshold_type == SF_THRESHOLD_GLOBAL ? raw : raw * connected;
                        rem = threshold - latest_qps - count;
                        if (rem < 0) { passed = 0; break; }
                    }
                    if (passed) {
                        for (uint32_t v = v0; v < v1; v++) so_cpm_add_value(c->cpm, in->param_tag[v], in->param_bits[v], count);
                        if (v1 - v0 > 1) rem = -1;                          /* remaining unsupported for multi-values */
                        st = SF_TOKEN_OK; remaining = so_java_d2i(rem);
                    } else {
                        st = SF_TOKEN_BLOCKED;
                    }
                }
            }
        }
        out->status[i] = st;
        if (out->remaining) out->remaining[i] = remaining;
        if (out->wait_ms) out->wait_ms[i] = wait;
    }
    return SF_OK;
}

/* ======================================================================
 * Token-server wire path (C1 frames).  Restates, per connection and in
 * order, the server pipeline of CS/server/NettyTransportServer.java:84-101:
 *   LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2)  (netty 4.1: 2-byte
 *     big-endian length, frameLength = length + 2, frames above 1024 bytes
 *     discarded with TooLongFrameException, length field stripped)
 *   NettyRequestDecoder (ByteToMessageDecoder, CS/server/codec/netty/
 *     NettyRequestDecoder.java:36-49): decodes while bytes remain; bytes a
 *     decode leaves unread stay in the cumulation for the next frame
 *   DefaultRequestEntityDecoder.java:42-63, FlowRequestDataDecoder.java:37-48,
 *   ParamFlowRequestDataDecoder.java:35-90 (ClusterConstants PARAM_TYPE_*)
 *   TokenServerHandler.channelRead :61-82 -> FlowRequestProcessor :36-52 /
 *     ParamFlowRequestProcessor :38-54 -> DefaultTokenService :39-64
 *   DefaultResponseEntityWriter.java:35-52, FlowResponseDataWriter.java:30-33,
 *     LengthFieldPrepender(2).
 * The stream stops (SF_WIRE_HOST) at the first frame whose outcome is not a
 * pure function of the frame and the token state (PING, a type without a
 * decoder, a body not consumed exactly): the C-ABI contract in
 * sentinel_flow.h.  A PARAM_FLOW frame's parameters are one Collection
 * (ParamFlowRequestDataDecoder.java:49-58 builds an ArrayList).
 * ====================================================================== */
enum { WF_NONE = 0, WF_REQ = 1, WF_BAD = 2, WF_HOST = 3 };

static uint32_t wbe32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
static uint64_t wbe64(const uint8_t* p) { return ((uint64_t)wbe32(p) << 32) | wbe32(p + 4); }
static void wput32(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v; }

uint64_t so_string_key(const uint8_t* b, uint32_t len) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (uint32_t i = 0; i < len; i++) { h ^= b[i]; h *= 0x100000001b3ULL; }
    return h;
}

typedef struct {
    int32_t xid; int8_t type; uint8_t prio;
    int64_t flow_id; int32_t count;
    int param; uint32_t v0, nv;               /* values at vtag/vbits[v0 .. v0 + nv) */
} so_wire_req;

/* One frame body through NettyRequestDecoder + DefaultRequestEntityDecoder +
 * the request processor.  WF_NONE: no response (empty frame, or the
 * processor's NullPointerException on null data). */
static int so_wire_decode(const uint8_t* b, uint32_t L, so_wire_req* r, uint8_t* vtag, uint64_t* vbits, uint32_t v0) {
    memset(r, 0, sizeof *r);
    r->v0 = v0;
    if (L == 0) return WF_NONE;                      /* callDecode: nothing readable */
    if (L < 5) return WF_HOST;                       /* decode() returns null, bytes stay cumulated */
    r->xid = (int32_t)wbe32(b);
    r->type = (int8_t)b[4];                          /* int type = source.readByte() */
    const uint8_t* q = b + 5;
    const uint32_t rem = L - 5;
    if (r->type == 1) {                              /* MSG_TYPE_FLOW */
        if (rem == 0) return WF_NONE;                /* data null -> NPE in FlowRequestProcessor :39 */
        if (rem < 12 || rem > 13) return WF_HOST;    /* data bytes left unread */
        r->flow_id = (int64_t)wbe64(q);
        r->count = (int32_t)wbe32(q + 8);
        r->prio = rem == 13 ? (q[12] != 0) : 0;      /* readBoolean */
        return WF_REQ;
    }
    if (r->type == 2) {                              /* MSG_TYPE_PARAM_FLOW */
        if (rem == 0) return WF_NONE;
        if (rem < 16) return WF_HOST;
        r->flow_id = (int64_t)wbe64(q);
        r->count = (int32_t)wbe32(q + 8);
        const int32_t amount = (int32_t)wbe32(q + 12);
        uint32_t p = 16;
        if (amount <= 0) return rem == 16 ? WF_NONE : WF_HOST;   /* decode() returns null */
        if ((uint32_t)amount > rem - 16) return WF_HOST;          /* every parameter reads >= 1 byte */
        int n = 0;
        for (int32_t k = 0; k < amount; k++) {
            if (p + 1 > rem) return WF_HOST;         /* IndexOutOfBoundsException */
            const uint8_t ty = q[p++];
            uint8_t tag = 0; uint64_t bits = 0; int ok = 1;
            switch (ty) {
            case 0: if (p + 4 > rem) return WF_HOST; tag = SF_TAG_INT; bits = (uint64_t)(int64_t)(int32_t)wbe32(q + p); p += 4; break;
            case 7: {                                /* PARAM_TYPE_STRING */
                if (p + 4 > rem) return WF_HOST;
                const int32_t len = (int32_t)wbe32(q + p); p += 4;
                if (len < 0 || (uint32_t)len > rem - p) return WF_HOST;
                tag = SF_TAG_STRING; bits = so_string_key(q + p, (uint32_t)len); p += (uint32_t)len; break;
            }
            case 6: if (p + 1 > rem) return WF_HOST; tag = SF_TAG_BOOL; bits = q[p] != 0; p += 1; break;
            case 3: {                                /* readDouble; Double.equals: doubleToLongBits */
                if (p + 8 > rem) return WF_HOST;
                uint64_t v = wbe64(q + p); p += 8;
                if ((v & 0x7ff0000000000000ULL) == 0x7ff0000000000000ULL && (v & 0x000fffffffffffffULL)) v = 0x7ff8000000000000ULL;
                tag = SF_TAG_DOUBLE; bits = v; break;
            }
            case 1: if (p + 8 > rem) return WF_HOST; tag = SF_TAG_LONG; bits = wbe64(q + p); p += 8; break;
            case 4: {                                /* readFloat; Float.equals: floatToIntBits */
                if (p + 4 > rem) return WF_HOST;
                uint32_t v = wbe32(q + p); p += 4;
                if ((v & 0x7f800000u) == 0x7f800000u && (v & 0x007fffffu)) v = 0x7fc00000u;
                tag = SF_TAG_FLOAT; bits = v; break;
            }
            case 2: if (p + 1 > rem) return WF_HOST; tag = SF_TAG_BYTE; bits = (uint64_t)(int64_t)(int8_t)q[p]; p += 1; break;
            case 5: if (p + 2 > rem) return WF_HOST; tag = SF_TAG_SHORT; bits = (uint64_t)(int64_t)(int16_t)(((uint32_t)q[p] << 8) | q[p + 1]); p += 2; break;
            default: ok = 0;                         /* decodeParam returns false, nothing added */
            }
            if (ok) { vtag[v0 + n] = tag; vbits[v0 + n] = bits; n++; }
        }
        if (p != rem) return WF_HOST;                /* bytes left in the cumulation */
        if (n == 0) return WF_BAD;                   /* requestParamToken: params.isEmpty() -> badRequest */
        r->nv = (uint32_t)n;
        r->param = 1;
        return WF_REQ;
    }
    if (rem == 0 && r->type != 0) return WF_NONE;    /* no decoder: null message, nothing left */
    return WF_HOST;                                  /* PING, or no decoder with bytes left */
}

int so_serve_frames(so_engine* e, const sf_wire_batch* in, sf_wire_out* out) {
    const uint32_t S = in->n_streams;
    const uint64_t total = in->stream_off[S];
    so_wire_req* reqs = (so_wire_req*)malloc(sizeof(so_wire_req) * (total / 2 + 1));
    uint8_t* kind = (uint8_t*)malloc(total / 2 + 1);
    uint32_t* rstream = (uint32_t*)malloc(sizeof(uint32_t) * (total / 2 + 1));
    uint64_t nr = 0, nframes = 0;
    uint8_t* vtag = (uint8_t*)malloc(total + 1);             /* every parameter takes >= 1 byte */
    uint64_t* vbits = (uint64_t*)malloc(8 * (total + 1));
    uint32_t nvals = 0;
    for (uint32_t s = 0; s < S; s++) {
        uint64_t p = in->stream_off[s];
        const uint64_t end = in->stream_off[s + 1];
        uint8_t stop = SF_WIRE_DONE;
        while (p < end) {
            if (end - p < 2) { stop = SF_WIRE_PARTIAL; break; }
            const uint32_t L = ((uint32_t)in->bytes[p] << 8) | in->bytes[p + 1];
            if (p + 2 + L > end) { stop = SF_WIRE_PARTIAL; break; }
            if (L + 2 > SF_WIRE_MAX_FRAME) { p += 2 + L; nframes++; continue; }   /* TooLongFrameException */
            so_wire_req r;
            const int k = so_wire_decode(in->bytes + p + 2, L, &r, vtag, vbits, nvals);
            if (k == WF_HOST) { stop = SF_WIRE_HOST; break; }
            nframes++;
            if (k != WF_NONE) { reqs[nr] = r; kind[nr] = (uint8_t)k; rstream[nr] = s; nr++; }
            if (k == WF_REQ) nvals += r.nv;
            p += 2 + L;
        }
        out->consumed[s] = p - in->stream_off[s];
        out->stop[s] = stop;
    }
    /* the token service, in (stream, frame) order */
    uint64_t nq = 0;
    for (uint64_t i = 0; i < nr; i++) nq += kind[i] == WF_REQ;
    int64_t* fid = (int64_t*)calloc(nq + 1, 8); int32_t* cnt = (int32_t*)calloc(nq + 1, 4);
    uint8_t* fl = (uint8_t*)calloc(nq + 1, 1); int64_t* ts = (int64_t*)calloc(nq + 1, 8);
    uint8_t* tg = (uint8_t*)calloc(nvals + nq + 1, 1); uint64_t* bt = (uint64_t*)calloc(nvals + nq + 1, 8);
    uint32_t* po = (uint32_t*)calloc(nq + 1, 4);
    int8_t* st = (int8_t*)calloc(nq + 1, 1); int32_t* rm = (int32_t*)calloc(nq + 1, 4); int32_t* wt = (int32_t*)calloc(nq + 1, 4);
    for (uint64_t i = 0, j = 0; i < nr; i++) {
        if (kind[i] != WF_REQ) continue;
        fid[j] = reqs[i].flow_id; cnt[j] = reqs[i].count; ts[j] = in->now_ms;
        fl[j] = (uint8_t)((reqs[i].prio ? SF_TOK_PRIORITIZED : 0) | (reqs[i].param ? SF_TOK_PARAM : 0));
        for (uint32_t v = 0; v < reqs[i].nv; v++) { tg[po[j] + v] = vtag[reqs[i].v0 + v]; bt[po[j] + v] = vbits[reqs[i].v0 + v]; }
        po[j + 1] = po[j] + reqs[i].nv;
        j++;
    }
    int rc = SF_OK;
    if (nq) {
        sf_token_batch b = {(uint32_t)nq, SF_MEM_HOST, fid, cnt, fl, ts, tg, bt, po};
        sf_token_results o = {SF_MEM_HOST, st, rm, wt};
        rc = so_request_tokens(e, &b, &o);
    }
    /* responses: LengthFieldPrepender(2) + xid, type, status, FlowTokenResponseData */
    const uint64_t need = nr * SF_WIRE_RESP_BYTES;
    uint32_t s_cur = 0;
    out->resp_off[0] = 0;
    for (uint64_t i = 0, j = 0; i < nr && rc == SF_OK; i++) {
        while (s_cur < rstream[i]) out->resp_off[++s_cur] = i * SF_WIRE_RESP_BYTES;
        if (need > out->cap) continue;
        uint8_t* o = out->resp + i * SF_WIRE_RESP_BYTES;
        int8_t status = SF_TOKEN_BAD_REQUEST; int32_t remaining = 0, wait = 0;
        if (kind[i] == WF_REQ) {
            status = st[j]; remaining = rm[j];
            wait = reqs[i].param ? 0 : wt[j];        /* ParamFlowRequestProcessor: setWaitInMs(0) */
            j++;
        }
        o[0] = 0; o[1] = 14;
        wput32(o + 2, (uint32_t)reqs[i].xid);
        o[6] = (uint8_t)reqs[i].type;
        o[7] = (uint8_t)status;
        wput32(o + 8, (uint32_t)remaining);
        wput32(o + 12, (uint32_t)wait);
    }
    while (s_cur < S) out->resp_off[++s_cur] = nr * SF_WIRE_RESP_BYTES;
    out->n_frames = nframes; out->n_requests = nq; out->n_responses = nr;
    free(reqs); free(kind); free(rstream);
    free(fid); free(cnt); free(fl); free(ts); free(tg); free(bt); free(st); free(rm); free(wt);
    free(po); free(vtag); free(vbits);
    if (rc == SF_OK && need > out->cap) return SF_ERR_CAPACITY;
    return rc;
}
