/*
 * sentinel_flow.h — C-ABI of the MI355X batch flow-check engine.
 *
 * This is the drop-in boundary for Sentinel's statistics-and-check hot path
 * (SURVEY.md §8b).  A Java shim binds these symbols through JNI / Panama FFM
 *  from behind two existing SPIs:
 *
 *   - SlotChainBuilder / ProcessorSlot   (in-process SphU.entry path)
 *       replaces  StatisticSlot.entry/exit + SystemSlot + ParamFlowSlot +
 *       FlowSlot of the default chain:
 *         sentinel-core/.../slotchain/SlotChainBuilder.java:25-33
 *         sentinel-core/.../slotchain/ProcessorSlot.java:28-77
 *         sentinel-core/.../slots/statistic/StatisticSlot.java:55-178
 *         sentinel-core/.../slots/block/flow/FlowSlot.java:162-174
 *         sentinel-parameter-flow-control/.../param/ParamFlowSlot.java:38-104
 *         sentinel-core/.../slots/system/SystemSlot.java:37-42
 *   - TokenService                        (cluster token server)
 *       replaces  DefaultTokenService.requestToken/requestParamToken:
 *         sentinel-core/.../cluster/TokenService.java:26-63
 *         sentinel-cluster-server-default/.../flow/DefaultTokenService.java:39-64
 *
 * Plain C: no exceptions cross the ABI, no torch / HIP types in signatures.
 * Every function returning int returns SF_OK (0) or a negative SF_ERR_* code;
 * sf_last_error() gives a human-readable message for the calling thread.
 *
 * Threading: one engine instance serialises sf_submit / sf_request_tokens
 * internally (a submit lock).  The Java shim batches from many application
 * threads into one flusher thread (SURVEY.md §8b "Threading").
 *
 * Ownership: the caller owns all input/output arrays; the engine owns every
 * byte of device state.  Rules are copied at load.
 */
#ifndef SENTINEL_FLOW_H
#define SENTINEL_FLOW_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SF_ABI_VERSION 1

/* ---- return codes ------------------------------------------------------ */
#define SF_OK               0
#define SF_ERR_INVALID     -1   /* bad argument / inconsistent batch        */
#define SF_ERR_NOMEM       -2   /* host or device allocation failed         */
#define SF_ERR_DEVICE      -3   /* HIP runtime error / no usable GPU        */
#define SF_ERR_UNSUPPORTED -4   /* rule or event feature outside the engine */
#define SF_ERR_CAPACITY    -5   /* batch / table larger than configured     */

/* ---- Sentinel constants (RuleConstant.java:26-66) ------------------------ */
#define SF_GRADE_THREAD 0
#define SF_GRADE_QPS    1
#define SF_STRATEGY_DIRECT 0
#define SF_STRATEGY_RELATE 1
#define SF_STRATEGY_CHAIN  2
#define SF_BEHAVIOR_DEFAULT              0
#define SF_BEHAVIOR_WARM_UP              1
#define SF_BEHAVIOR_RATE_LIMITER         2
#define SF_BEHAVIOR_WARM_UP_RATE_LIMITER 3
/* ClusterRuleConstant.FLOW_THRESHOLD_AVG_LOCAL = 0, FLOW_THRESHOLD_GLOBAL = 1 */
#define SF_THRESHOLD_AVG_LOCAL 0
#define SF_THRESHOLD_GLOBAL    1

#define SF_MAX_SAMPLE_COUNT 16   /* second-window buckets supported          */
#define SF_MINUTE_BUCKETS   60   /* StatisticNode.java:105 ArrayMetric(60,60000) */
#define SF_MAX_RULES_PER_RESOURCE 8
#define SF_MAX_ARGS 4

/* ---- engine configuration (SentinelConfig / *Property defaults) -------- */
typedef struct sf_config {
    int32_t  sample_count;        /* SampleCountProperty.SAMPLE_COUNT = 2      */
    int32_t  interval_ms;         /* IntervalProperty.INTERVAL = 1000          */
    int32_t  occupy_timeout_ms;   /* OccupyTimeoutProperty = 500               */
    int32_t  cold_factor;         /* ColdFactorProperty.coldFactor = 3         */
    int64_t  statistic_max_rt;    /* SentinelConfig.statisticMaxRt = 5000      */
    uint32_t max_resources;       /* resource ids of this shard: [0, max)      */
    uint32_t max_batch;           /* largest sf_submit / sf_request_tokens n   */
    uint32_t param_capacity;      /* exact hot-param table entries             */
    uint32_t shard_count;         /* resource sharding: res % shard_count ==   */
    uint32_t shard_index;         /*   shard_index; local id = res/shard_count */
    int32_t  device;              /* HIP device ordinal                        */
    /* cluster token server (ServerFlowConfig.java:26-31) */
    int32_t  cluster_sample_count;/* 10 */
    int32_t  cluster_interval_ms; /* 1000 */
    double   exceed_count;        /* 1.0 */
    double   max_occupy_ratio;    /* 1.0 */
    uint32_t max_flow_ids;        /* capacity of the flowId table              */
    uint32_t heavy_min_events;    /* resource segments longer than this use the
                                     window/skip algorithms (0 = engine default) */
    uint32_t aux_capacity;        /* origin nodes (one per (resource, origin) of
                                     the traffic) + context nodes of CHAIN rules
                                     (0 = 65536)                               */
    uint32_t pad;
} sf_config;

/* Fill *cfg with the reference defaults listed above. */
void sf_config_default(sf_config* cfg);

/* ---- rules ------------------------------------------------------------- */
/* Origins and context names are interned by the caller into one id space:
 * 0 is the string "default", 1 is "other" (RuleConstant.LIMIT_APP_DEFAULT /
 * LIMIT_APP_OTHER), any other origin name is an id >= 2, and the empty origin
 * "" (no ContextUtil.enter origin) is SF_ORIGIN_NONE.  Context names are a
 * separate id space (0 is whatever name the host interns first, normally
 * "sentinel_default_context").                                              */
#define SF_APP_DEFAULT 0u
#define SF_APP_OTHER   1u
#define SF_ORIGIN_NONE 0xFFFFFFFFu
#define SF_REF_NONE    0xFFFFFFFFu   /* blank refResource                       */

/* One FlowRule (FlowRule.java:36-241); the caller passes rules already in the
 * order Java iterates them (FlowRuleUtil.buildFlowRuleMap: HashSet order +
 * stable FlowRuleComparator sort, FlowRuleUtil.java:83-130; sf_flow_rule_order).
 * Rules of one resource keep array order.  FlowRuleChecker.
 * selectNodeByRequesterAndStrategy (FlowRuleChecker.java:129-161) picks the
 * node a rule checks:
 *   limit_app == the event's origin (not "default"/"other") or limit_app
 *   "other" with an origin no rule of the resource names
 *       DIRECT -> the origin node of (resource, origin)
 *   limit_app "default"  DIRECT -> the resource's ClusterNode
 *   RELATE (any matching limit_app) -> the ClusterNode of ref_resource (a
 *       resource id; none until that resource's first entry -> pass);
 *       ref_resource must live on the same shard (res % shard_count)
 *   CHAIN -> the resource's DefaultNode of context ref_resource (a context id)
 *       when the event's context is that one, else pass
 *   anything else -> no node -> pass.
 * cluster_mode: ClusterStateManager is not started in the engine's process
 * (pickClusterService() == null, FlowRuleChecker.java:163-203), so a cluster
 * rule is checked locally when cluster_fallback (fallbackToLocalWhenFail,
 * ClusterFlowConfig default true) is set and passes otherwise.  Cluster
 * token rules themselves go to sf_load_cluster_rules (the token server).   */
typedef struct sf_flow_rule {
    uint32_t resource;            /* resource id (interned name)               */
    int32_t  grade;               /* SF_GRADE_*                                */
    double   count;
    int32_t  strategy;            /* SF_STRATEGY_*                             */
    int32_t  control_behavior;    /* SF_BEHAVIOR_*                             */
    int32_t  warm_up_period_sec;  /* default 10                                */
    int32_t  max_queueing_time_ms;/* default 500                               */
    int32_t  cluster_mode;        /* FlowRule.clusterMode                      */
    uint32_t ref_resource;        /* RELATE: resource id; CHAIN: context id    */
    uint32_t limit_app;           /* SF_APP_DEFAULT (also a blank limitApp), SF_APP_OTHER, or an origin id */
    int32_t  cluster_fallback;    /* ClusterFlowConfig.fallbackToLocalWhenFail */
} sf_flow_rule;

/* Param value identity = Java equals(): (type tag, 64-bit payload); strings
 * are interned by the caller (ParamFlowChecker.java:126-155).            */
#define SF_TAG_NULL   0
#define SF_TAG_INT    1
#define SF_TAG_LONG   2
#define SF_TAG_STRING 3
#define SF_TAG_DOUBLE 4
#define SF_TAG_BOOL   5
#define SF_TAG_OTHER  6
#define SF_TAG_BYTE   7   /* java.lang.Byte  (wire PARAM_TYPE_BYTE)  */
#define SF_TAG_SHORT  8   /* java.lang.Short (wire PARAM_TYPE_SHORT) */
#define SF_TAG_FLOAT  9   /* java.lang.Float (wire PARAM_TYPE_FLOAT), bits = floatToIntBits */
/* An argument that is a java.util.Collection or an array: its elements are
 * listed separately (sf_event_batch.arg_elem_off / sf_token_batch.param_off). */
#define SF_TAG_COLLECTION 0x40

typedef struct sf_hot_item {      /* ParamFlowItem parsed (ParamFlowRuleUtil.java:188-240) */
    uint8_t  tag;
    uint8_t  pad[3];
    int32_t  count;
    uint64_t bits;
} sf_hot_item;

/* One ParamFlowRule (ParamFlowRule.java:45-83). */
typedef struct sf_param_rule {
    uint32_t resource;
    int32_t  grade;               /* SF_GRADE_QPS (default) / SF_GRADE_THREAD  */
    int32_t  param_idx;           /* may be negative: ParamFlowSlot.applyRealParamIdx */
    int32_t  control_behavior;    /* SF_BEHAVIOR_DEFAULT / SF_BEHAVIOR_RATE_LIMITER */
    double   count;
    int32_t  max_queueing_time_ms;/* default 0 */
    int32_t  burst_count;         /* default 0 */
    int64_t  duration_in_sec;     /* default 1 */
    uint32_t item_offset;         /* hot items: items[item_offset .. +item_count) */
    uint32_t item_count;
} sf_param_rule;

/* SystemRule thresholds (SystemRuleManager.java:291-348); negative = unset. */
typedef struct sf_system_rule {
    double  highest_system_load;
    double  highest_cpu_usage;
    double  qps;
    int64_t avg_rt;
    int64_t max_thread;
} sf_system_rule;

/* ---- events (time-ordered, SoA) ----------------------------------------- */
#define SF_EV_EXIT   0x01u   /* EXIT event (Entry.exit), else ENTRY            */
#define SF_EV_IN     0x02u   /* EntryType.IN (feeds ENTRY_NODE / SystemRule)   */
#define SF_EV_PRIO   0x04u   /* prioritized entry                              */
#define SF_EV_ERROR  0x08u   /* EXIT: business exception recorded (Tracer)     */
/* ENTRY blocked by a slot that StatisticSlot wraps but the engine does not run
 * (AuthoritySlot, order -6000, between StatisticSlot -7000 and SystemSlot
 * -5000: Constants.java:80-84).  StatisticSlot.entry catches its
 * BlockException (AuthorityException) like any other (StatisticSlot.java:102-124):
 * block += count on the resource's ClusterNode and, for EntryType.IN, on
 * ENTRY_NODE; no SystemRule / ParamFlowRule / FlowRule / breaker sees the
 * entry; its EXIT records nothing (blockError set, :139).  Verdict
 * SF_V_BLOCK_OTHER.                                                         */
#define SF_EV_BLOCKED 0x10u

#define SF_MEM_HOST   0
#define SF_MEM_DEVICE 1

typedef struct sf_event_batch {
    uint32_t        n;
    int32_t         mem;          /* SF_MEM_HOST or SF_MEM_DEVICE (all arrays) */
    const uint32_t* res_id;       /* [n] resource id                          */
    const int64_t*  ts_ms;        /* [n] mocked TimeUtil clock, non-decreasing */
    const int32_t*  count;        /* [n] acquireCount (EXIT: the entry's count) */
    const uint8_t*  flags;        /* [n] SF_EV_*                               */
    /* EXIT only: index (in this batch) of the ENTRY being exited, or -1 when
     * that entry passed in an earlier batch (then create_ts supplies rt).   */
    const int64_t*  entry_ref;    /* [n] or NULL when the batch has no EXIT   */
    const int64_t*  create_ts;    /* [n] or NULL; read only where entry_ref<0 */
    /* args: n_args[i] values for event i, stored [slot][n] (slot-major).   */
    uint32_t        arg_slots;    /* 0..SF_MAX_ARGS                            */
    const uint8_t*  n_args;       /* [n] or NULL (= arg_slots for every event) */
    const uint8_t*  arg_tag;      /* [arg_slots*n]                             */
    const uint64_t* arg_bits;     /* [arg_slots*n]                             */
    /* Collection / array arguments (ParamFlowChecker.passLocalCheck :84-112,
     * ParameterMetric.addThreadCount / decreaseThreadCount :125-239): the
     * argument k = slot*n + i whose arg_tag[k] is SF_TAG_COLLECTION holds the
     * elements elem_tag / elem_bits[arg_elem_off[k] .. arg_elem_off[k+1]) in
     * iteration order.  Every element must pass each rule in turn; the tokens
     * of the elements before a failing one stay consumed.  A null element
     * (SF_TAG_NULL) ends the loop as the reference's NullPointerException in
     * the parameter maps does (the value then passes that rule), after the
     * checks that come first (a zero threshold, acquireCount > max tokens).
     * NULL arg_elem_off: no argument is a collection.                         */
    const uint32_t* arg_elem_off; /* [arg_slots*n + 1] or NULL                 */
    const uint8_t*  elem_tag;     /* [n_elems]                                 */
    const uint64_t* elem_bits;    /* [n_elems]                                 */
    uint32_t        n_elems;
    /* Context of each event (ContextUtil.enter(name, origin)): origin id
     * (SF_ORIGIN_NONE = "") and context-name id; an EXIT carries its entry's.
     * NULL: no origin / context 0 for every event.  Read only for resources
     * whose flow rules select an origin or context node (sf_flow_rule).     */
    const uint32_t* origin;       /* [n] or NULL                               */
    const uint32_t* context;      /* [n] or NULL                               */
} sf_event_batch;

/* ---- verdicts ---------------------------------------------------------- */
#define SF_V_PASS          0   /* entry passed                                   */
#define SF_V_PASS_WAIT     1   /* passed after Thread.sleep(wait_ms) (rate limiter) */
#define SF_V_PRIORITY_WAIT 2   /* PriorityWaitException(wait_ms): passed, borrowed */
#define SF_V_BLOCK_FLOW    3   /* FlowException (rule_idx = index in resource list) */
#define SF_V_BLOCK_PARAM   4   /* ParamFlowException                             */
#define SF_V_BLOCK_SYSTEM  5   /* SystemBlockException (rule_idx: 0 qps 1 thread 2 rt 3 load 4 cpu) */
#define SF_V_EXIT          6   /* exit of a passed entry: recorded               */
#define SF_V_EXIT_IGNORED  7   /* exit of a blocked entry: nothing recorded      */

typedef struct sf_verdicts {
    int32_t  mem;                 /* SF_MEM_HOST or SF_MEM_DEVICE             */
    uint8_t* status;              /* [n] SF_V_*  (required)                    */
    int32_t* wait_ms;             /* [n] or NULL                               */
    uint16_t* rule_idx;           /* [n] or NULL                               */
} sf_verdicts;

/* ---- cluster token service (TokenService.java:26-63) -------------------- */
/* TokenResultStatus.java:27-69 */
#define SF_TOKEN_OK                0
#define SF_TOKEN_BLOCKED           1
#define SF_TOKEN_SHOULD_WAIT       2
#define SF_TOKEN_NO_RULE_EXISTS    3
#define SF_TOKEN_BAD_REQUEST      -4
#define SF_TOKEN_TOO_MANY_REQUEST -2
#define SF_TOKEN_FAIL             -1

typedef struct sf_cluster_flow_rule {   /* cluster-mode FlowRule + ClusterFlowConfig */
    int64_t  flow_id;
    double   count;
    int32_t  threshold_type;      /* SF_THRESHOLD_*                            */
    uint32_t namespace_id;
    int32_t  sample_count;        /* ClusterFlowConfig default 10              */
    int32_t  window_interval_ms;  /* default 1000                              */
} sf_cluster_flow_rule;

typedef struct sf_cluster_param_rule {  /* cluster-mode ParamFlowRule */
    int64_t  flow_id;
    double   count;
    int32_t  threshold_type;
    uint32_t namespace_id;
    int32_t  sample_count;
    int32_t  window_interval_ms;
    uint32_t item_offset;         /* hot items (exclusive thresholds) */
    uint32_t item_count;
} sf_cluster_param_rule;

typedef struct sf_namespace {
    uint32_t namespace_id;
    int32_t  connected_count;     /* ConnectionManager.getConnectedCount       */
    double   max_allowed_qps;     /* GlobalRequestLimiter; < 0: no limiter     */
} sf_namespace;

#define SF_TOK_PRIORITIZED 0x01u
#define SF_TOK_PARAM       0x02u  /* requestParamToken                          */

typedef struct sf_token_batch {
    uint32_t        n;
    int32_t         mem;
    const int64_t*  flow_id;      /* [n] rule id (Long ruleId)                 */
    const int32_t*  count;        /* [n] acquireCount                          */
    const uint8_t*  flags;        /* [n] SF_TOK_*                              */
    const int64_t*  ts_ms;        /* [n] server clock at request, non-decreasing */
    const uint8_t*  param_tag;    /* [n] or NULL (param_off: [param_off[n]])   */
    const uint64_t* param_bits;   /* [n] or NULL (param_off: [param_off[n]])   */
    /* requestParamToken(Long, int, Collection<Object> params): with param_off,
     * request i's params are param_tag / param_bits[param_off[i] ..
     * param_off[i+1]) in iteration order (ClusterParamFlowChecker.java:42-87:
     * every value must have room before any is added; remaining is -1 for
     * more than one value; an empty collection is BAD_REQUEST,
     * DefaultTokenService.java:53-56).  NULL: one value per request.        */
    const uint32_t* param_off;    /* [n + 1] or NULL                           */
} sf_token_batch;

typedef struct sf_token_results {
    int32_t  mem;
    int8_t*  status;              /* [n] SF_TOKEN_*                            */
    int32_t* remaining;           /* [n] or NULL                               */
    int32_t* wait_ms;             /* [n] or NULL                               */
} sf_token_results;

/* ---- state read-back (parity tests, metric snapshot) -------------------- */
#define SF_WS_ABSENT INT64_MIN    /* bucket slot never created (Java null)     */

typedef struct sf_bucket {       /* WindowWrap<MetricBucket> (MetricBucket.java:28-142) */
    int64_t window_start;
    int64_t pass, block, exception, success, rt, occupied_pass;
    int64_t min_rt;
} sf_bucket;

typedef struct sf_node_state {    /* ClusterNode of one resource (StatisticNode.java:97-105) */
    sf_bucket second[SF_MAX_SAMPLE_COUNT];
    int64_t   borrow_ws[SF_MAX_SAMPLE_COUNT];    /* FutureBucketLeapArray */
    int64_t   borrow_pass[SF_MAX_SAMPLE_COUNT];
    sf_bucket minute[SF_MINUTE_BUCKETS];
    int64_t   cur_thread_num;
} sf_node_state;

typedef struct sf_rule_state {    /* controller state (WarmUp / RateLimiter) */
    int64_t stored_tokens;
    int64_t last_filled_time;
    int64_t latest_passed_time;
} sf_rule_state;

typedef struct sf_metric_row {    /* MetricNode (MetricNode.java:160-229) */
    uint32_t resource;            /* global resource id, or SF_RES_ENTRY_NODE  */
    int32_t  concurrency;         /* MetricNode.concurrency: metrics() never sets it (ArrayMetric.fromBucket :199-214), so 0 in snapshots */
    int64_t  timestamp;
    int64_t  pass_qps, block_qps, success_qps, exception_qps, rt, occupied_pass_qps;
} sf_metric_row;

typedef struct sf_stats {         /* device-clock timings, summed over sf_submit calls while timing is on */
    double   total_ms;
    double   sort_ms;             /* keys + radix sort + segment heads + gather + classify */
    double   decide_ms;           /* light and heavy decision kernels (two streams) up to the join */
    double   scatter_ms;
    uint64_t n_events;            /* of the last call */
    uint64_t n_segments;          /* resources touched by the last call */
    uint64_t n_launches;
    double   light_ms;            /* k_decide_light alone (stream A) */
    double   heavy_decide_ms;     /* k_heavy_decide alone (stream B) */
    double   heavy_fill_ms;       /* k_heavy_fill alone (stream B) */
    double   classify_ms;         /* k_classify alone */
    double   stream_ms;           /* k_heavy_stream alone (stream C: THREAD-grade and RateLimiter heavy segments) */
    double   metric_scan_ms;      /* last sf_metric_log: k_mlog_count alone (every node's minute row) */
    double   metric_log_ms;       /* last sf_metric_log: all its kernels, before the copy to the host */
    double   wire_ms;             /* last sf_serve_frames: device time from framing to encoded responses (host syncs included) */
    uint64_t sys_rounds;          /* SystemRule sub-batches (planner rounds) over the sf_submit calls */
    uint64_t aux_nodes;           /* origin / context nodes kept (pool slots in use) */
    uint64_t aux_capacity;        /* pool slots backed by device memory (grows by chunks between batches) */
    uint64_t aux_index_grows;     /* times the pool's index table was rebuilt larger */
    uint64_t param_table_grows;   /* times the exact ParamFlow table was rebuilt larger (before a batch) */
    /* the wave walk of long one-resource xflow segments (k_decide_xw): chunks
     * settled by the exact solve, chunks on the serial path, solve rounds,
     * events the serial part walked */
    uint64_t xw_chunks_exact, xw_chunks_serial, xw_rounds, xw_serial_events;
    uint64_t sys_exchanges;       /* all-gathers of sf_submit_node's per-window exchange (SF_SYSX_MSG_BYTES each, plan step) */
} sf_stats;

typedef struct sf_heavy_profile { /* diagnostics: one heavy segment of the last sf_submit */
    uint32_t resource;            /* local resource index on this shard        */
    uint32_t events;              /* events of the resource in the batch       */
    uint32_t mode;                /* heavy algorithm (DESIGN.md "Kernels")     */
    uint32_t start;               /* k_heavy_stream segments: start after the launch's first segment start (100 MHz ticks) */
    uint64_t ticks;               /* time of the segment in its kernel, 100 MHz device clock */
} sf_heavy_profile;

/* ---- API ------------------------------------------------------------- */
typedef struct sf_engine sf_engine;

int  sf_abi_version(void);
int  sf_create(const sf_config* cfg, sf_engine** out);
void sf_destroy(sf_engine* e);
const char* sf_last_error(void);

int  sf_load_flow_rules (sf_engine* e, const sf_flow_rule* rules, uint32_t n);
int  sf_load_param_rules(sf_engine* e, const sf_param_rule* rules, uint32_t n,
                         const sf_hot_item* items, uint32_t n_items);
int  sf_load_system_rules(sf_engine* e, const sf_system_rule* rules, uint32_t n);
/* JMX load / cpu inputs of SystemRule (fixed inputs in a replay). */
int  sf_set_system_status(sf_engine* e, double avg_load, double cpu_usage);

/* Decide a time-ordered batch: per-event verdicts, state updated in place.
 * Returns when the verdicts are written (and checked). */
int  sf_submit(sf_engine* e, const sf_event_batch* in, sf_verdicts* out);
/* Same, enqueued only (batch and verdict arrays in HBM, SF_MEM_DEVICE): the
 * engine sorts batch k+1 while it decides batch k (two internal Work sets).
 * Batches are decided in submission order, exactly as by sf_submit; the
 * arrays must stay valid until sf_sync, which waits for every enqueued batch
 * and reports the first error any of them raised.  Host-memory batches and
 * timing mode fall back to sf_submit. */
int  sf_submit_async(sf_engine* e, const sf_event_batch* in, sf_verdicts* out);

/* ---- compact batches (the PCIe form: 8 bytes per event) -----------------
 * For a host that submits from its own memory (the Java shim's EventBatcher):
 * one uint64 per event instead of 17-25 bytes of SoA, so the batch crosses
 * PCIe 2-3x faster, and with sf_submit_packed_async the copy of batch k+1,
 * the decision of batch k and the copy back of the verdicts of batch k-1
 * overlap (host arrays in page-locked memory from sf_host_alloc; pageable
 * memory works, without the overlap).
 *   bits  0..31  resource id
 *   bits 32..51  ts_ms - ts_base (0 .. 2^20-1 ms; time-ordered as in sf_event_batch)
 *   bits 52..58  acquireCount 1..127; 0: the next value of count_ext
 *   bits 59..63  flags (SF_EV_EXIT | SF_EV_IN | SF_EV_PRIO | SF_EV_ERROR | SF_EV_BLOCKED)
 * exit_ref / exit_cts hold, for the EXIT events in batch order, what
 * entry_ref / create_ts hold for them in sf_event_batch (create_ts read where
 * exit_ref < 0; NULL: 0).  origin (per event) as in sf_event_batch.
 * The verdicts are sf_verdicts in the same memory kind as the batch.
 *
 * The narrow form (4 bytes per event; ev NULL, ev4 set) for resource ids below
 * 2^24: the time leaves the word for a table of the batch's milliseconds,
 *   ev4 bits  0..23  resource id
 *       bits 24..26  acquireCount 1..7; 0: the next value of count_ext
 *       bits 27..31  flags
 *   ms_end[m] = the number of events with ts_ms - ts_base <= m (m < n_ms,
 *   non-decreasing, ms_end[n_ms - 1] == n; else SF_ERR_INVALID at sync), so
 *   event i is at ts_base + the first m with ms_end[m] > i.  n_ms <= 2^20.
 * A config-3 batch (2^27 events over 4 s) crosses PCIe in 0.63 GB instead of
 * 1.16 GB.                                                                 */
#define SF_PK_COUNT_SHIFT 52
#define SF_PK_FLAGS_SHIFT 59
#define SF_PK4_COUNT_SHIFT 24
#define SF_PK4_FLAGS_SHIFT 27
#define SF_PK4_MAX_MS 1048576u
typedef struct sf_packed_batch {
    uint32_t        n;
    int32_t         mem;          /* SF_MEM_HOST or SF_MEM_DEVICE (all arrays)  */
    int64_t         ts_base;
    const uint64_t* ev;           /* [n]                                        */
    const int64_t*  exit_ref;     /* [n_exit] or NULL when the batch has no EXIT */
    const int64_t*  exit_cts;     /* [n_exit] or NULL                           */
    const int32_t*  count_ext;    /* [n_count_ext] or NULL                      */
    const uint32_t* origin;       /* [n] or NULL                                */
    uint32_t        n_exit;
    uint32_t        n_count_ext;
    const uint32_t* ev4;          /* [n]: the narrow form (ev NULL), or NULL    */
    const uint32_t* ms_end;       /* [n_ms]: the narrow form's time table       */
    uint32_t        n_ms;
    uint32_t        pad0;
} sf_packed_batch;
int  sf_submit_packed(sf_engine* e, const sf_packed_batch* in, sf_verdicts* out);
/* Enqueued only; sf_sync waits and reports the first error.  Host arrays
 * (batch and verdicts) must stay untouched until sf_sync.                   */
int  sf_submit_packed_async(sf_engine* e, const sf_packed_batch* in, sf_verdicts* out);
/* Sparse host verdicts of a packed batch: the copy back is 1 byte per event
 * plus the exceptions.  status [n] as in sf_verdicts; the events whose
 * wait_ms is not 0 (queued passes) as (index << 32 | (uint32_t)wait_ms) in
 * waits, the events whose rule_idx is not 0 (blocks by a resource's later
 * rule) as (index << 32 | rule_idx) in rules, each list in any order, its
 * length in counts[0] / counts[1].  waits and rules hold n entries; the first
 * `prefetch` of each list come back with the status bytes, the rest (if any)
 * at sf_sync_packed_sparse.  Every wait / rule not listed is 0. */
typedef struct sf_sparse_verdicts {
    uint8_t*  status;             /* [n]                                       */
    uint64_t* waits;              /* [n]                                       */
    uint64_t* rules;              /* [n]                                       */
    uint32_t* counts;             /* [2]                                       */
    uint32_t  prefetch;
    uint32_t  pad;
} sf_sparse_verdicts;
int  sf_submit_packed_sparse_async(sf_engine* e, const sf_packed_batch* in, sf_sparse_verdicts* out);
/* Waits for that batch (like sf_sync_packed) and completes its lists. */
int  sf_sync_packed_sparse(sf_engine* e, const sf_sparse_verdicts* out);
/* Waits for ONE sf_submit_packed_async batch with host verdicts -- the one
 * whose verdicts go to out->status -- and returns that batch's error; the
 * batch enqueued after it keeps running.  With two host verdict buffers used
 * in turn, a caller double-buffers: enqueue k+1, sf_sync_packed(k), hand out
 * k's verdicts, enqueue k+2 into k's buffers ...  (the Java flusher,
 * EventBatcher.java).  SF_OK when that batch was already collected. */
int  sf_sync_packed(sf_engine* e, const sf_verdicts* out);

/* SystemRules on a resource-sharded node (shard_count > 1).
 * SystemRuleManager.checkSystem (SystemRuleManager.java:291-348) reads the
 * node-wide ENTRY_NODE, which every earlier IN event of every resource (every
 * shard) updates, so a sharded engine with SystemRules refuses sf_submit and
 * is driven by rounds instead (sentinel_amd/system_shard.py does it over
 * torch.distributed):
 *   1. the ranks all-gather the IN events of the batch (global submission
 *      order; an exit's entry_ref indexes this merged stream, -1 for an entry
 *      of an earlier batch) -- every rank holds the same merged stream;
 *   2. sf_system_plan(merged, verdicts of merged[0, p), p) -> q and the forced
 *      SystemBlockException of every IN entry of merged[p, q) (SYS_NONE = 0xFF
 *      for none; else 0 qps, 1 thread, 2 rt, 3 load, 4 cpu), identical on every
 *      rank (same inputs, same ENTRY_NODE);
 *   3. each rank decides its own events before merged[q] in global order with
 *      sf_submit_forced (sys_mask per event; an exit whose entry lay in an
 *      earlier sub-batch carries entry_ref -1 and its create_ts when the entry
 *      passed, -2 when it was blocked);
 *   4. the ranks combine the verdicts of merged[p, q) (each event is decided by
 *      exactly one rank) and every rank adds them to its ENTRY_NODE with
 *      sf_entry_node_add; p = q.
 * Host arrays; calls of one batch use increasing p.  A call with p > 0 and
 * the same event arrays (addresses and n) as the call before continues that
 * merged stream: its events are not copied to the device again, nor the
 * verdicts already passed (only those added since the call before), so the
 * arrays must not change within a batch except by appending verdicts. */
int  sf_system_plan(sf_engine* e, const sf_event_batch* in_events, const uint8_t* status, uint32_t p,
                    uint32_t* q, uint8_t* sys_mask);
int  sf_submit_forced(sf_engine* e, const sf_event_batch* in, sf_verdicts* out, const uint8_t* sys_mask);
int  sf_entry_node_add(sf_engine* e, const sf_event_batch* in_events, const uint8_t* status);

/* Cluster token server (DefaultTokenService). */
int  sf_load_namespaces(sf_engine* e, const sf_namespace* ns, uint32_t n);
int  sf_load_cluster_rules(sf_engine* e, const sf_cluster_flow_rule* flow, uint32_t n_flow,
                           const sf_cluster_param_rule* param, uint32_t n_param,
                           const sf_hot_item* items, uint32_t n_items);
int  sf_request_tokens(sf_engine* e, const sf_token_batch* in, sf_token_results* out);
/* Token server over the GPUs of a node: one engine per GPU,
 * each loaded with ALL cluster rules and namespaces, with shard_count /
 * shard_index of its sf_config; a request is decided by its owner shard only
 * (another shard's request makes sf_request_tokens fail with SF_ERR_INVALID).
 * The owner of a flowId is flow_id % shard_count, except that every rule of a
 * namespace with a GlobalRequestLimiter (max_allowed_qps >= 0) is pinned to
 * namespace_id % shard_count: the limiter is one sequential gate over the
 * namespace (GlobalRequestLimiter.java:46-55).  Requests with flow_id <= 0
 * belong to shard 0.  sf_token_shard computes the owners of a batch from the
 * rule tables (host only: no engine, no GPU), for the front-end that routes
 * requests; ClusterMetric state stays on the owner (sf_cluster_sum).
 * sf_serve_frames needs shard_count == 1 (its front-end routes decoded frames). */
int  sf_token_shard(const sf_cluster_flow_rule* flow, uint32_t n_flow, const sf_cluster_param_rule* param,
                    uint32_t n_param, const sf_namespace* ns, uint32_t n_ns, uint32_t shard_count,
                    const int64_t* flow_id, const uint8_t* flags, uint32_t n, uint32_t* out_shard);
/* ---- token-server wire path (C1 frames) ------------
 * Replaces the server pipeline of NettyTransportServer.java:84-101 up to the
 * TokenService call and back:
 *   LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2)  -> NettyRequestDecoder
 *   -> DefaultRequestEntityDecoder.java:42-63 (xid:int32, type:int8)
 *   -> FlowRequestDataDecoder.java:37-48 / ParamFlowRequestDataDecoder.java:35-90
 *   -> TokenServerHandler.channelRead (:61-82) -> Flow/ParamFlowRequestProcessor
 *   -> DefaultTokenService (sf_request_tokens)
 *   -> DefaultResponseEntityWriter.java:35-52 + FlowResponseDataWriter.java:30-33
 *   -> LengthFieldPrepender(2).
 * The input is the raw inbound bytes of n_streams connections, concatenated
 * (stream s = in[stream_off[s], stream_off[s+1])); all big-endian, as Netty.
 * Every request decided in one call is stamped now_ms and decided in (stream,
 * frame) order.  Per stream the engine handles the longest prefix of frames it
 * decides exactly like the reference and stops at:
 *   - an incomplete frame at the end              -> SF_WIRE_PARTIAL
 *   - a frame the host must run through the reference pipeline -> SF_WIRE_HOST:
 *     PING (ConnectionManager bookkeeping; its connected count takes effect at
 *     the next call), a type with no decoder, or a frame whose body the
 *     decoder does not consume exactly (Netty's cumulation would carry the
 *     rest into the next frame).  The parameters of a PARAM_FLOW frame are
 *     one Collection (requestParamToken with every decoded value).
 * consumed[s] = bytes of stream s handled (the stopping frame starts there).
 * Frames longer than 1024 bytes are skipped without a response (Netty's
 * TooLongFrameException); a FLOW / PARAM_FLOW frame with no data gets no
 * response (the processor's NullPointerException), as in the reference.
 * Responses of stream s: out[resp_off[s] .. resp_off[s+1]), SF_WIRE_RESP_BYTES
 * each (2-B length 14, xid, type, status, remaining, waitInMs).
 * String parameters are keyed by sf_string_key() of their bytes: a rule's
 * String hot items must be loaded with SF_TAG_STRING bits = sf_string_key(). */
#define SF_WIRE_DONE    0
#define SF_WIRE_PARTIAL 1
#define SF_WIRE_HOST    2
#define SF_WIRE_RESP_BYTES 16
#define SF_WIRE_MAX_FRAME 1024      /* LengthFieldBasedFrameDecoder maxFrameLength */

typedef struct sf_wire_batch {
    int32_t         mem;            /* SF_MEM_HOST / SF_MEM_DEVICE: bytes and stream_off */
    uint32_t        n_streams;
    const uint8_t*  bytes;
    const uint64_t* stream_off;     /* [n_streams + 1], non-decreasing, total < 2^31 */
    int64_t         now_ms;         /* server clock (TimeUtil) of every request   */
} sf_wire_batch;

typedef struct sf_wire_out {        /* host memory */
    uint8_t*  resp;                 /* response bytes                               */
    uint64_t  cap;                  /* capacity of resp in bytes                    */
    uint64_t* resp_off;             /* [n_streams + 1] byte offsets into resp       */
    uint64_t* consumed;             /* [n_streams]                                  */
    uint8_t*  stop;                 /* [n_streams] SF_WIRE_*                        */
    uint64_t  n_frames;             /* out: complete frames found                   */
    uint64_t  n_requests;           /* out: requests decided by the token service   */
    uint64_t  n_responses;          /* out: responses written                       */
} sf_wire_out;

/* 64-bit key of a wire String parameter (FNV-1a 64 of its bytes). */
uint64_t sf_string_key(const uint8_t* bytes, uint32_t len);
int  sf_serve_frames(sf_engine* e, const sf_wire_batch* in, sf_wire_out* out);

/* ClusterMetric.getSum(event) of a cluster flow rule at time now_ms
 * (ClusterMetric.java:47-55; rolls the current bucket like the reference).
 * event: ClusterFlowEvent ordinal (PASS 0, BLOCK 1, PASS_REQUEST 2,
 * BLOCK_REQUEST 3, OCCUPIED_PASS 4, OCCUPIED_BLOCK 5, WAITING 6). */
int  sf_cluster_sum(sf_engine* e, int64_t flow_id, int event, int64_t now_ms, int64_t* out);

/* State read-back and the per-second metric snapshot (StatisticNode.metrics). */
int  sf_read_node(sf_engine* e, uint32_t resource, sf_node_state* out);
int  sf_read_entry_node(sf_engine* e, sf_node_state* out);
int  sf_read_rule_state(sf_engine* e, uint32_t rule_index, sf_rule_state* out);
/* Bulk forms of the two reads above, for whole-engine state comparison.
 * sf_node_digests: out[l] for local rows l < n_rows (row l holds resource
 * l * shard_count + shard_index) = FNV-1a 64 (h ^= word; h *= 0x100000001b3,
 * seed 0xcbf29ce484222325) over the row's sf_node_state as sf_read_node gives
 * it, word by word: for i < sample_count second[i] (window_start, pass, block,
 * exception, success, rt, occupied_pass, min_rt), borrow_ws[i],
 * borrow_pass[i]; then the SF_MINUTE_BUCKETS minute buckets; then
 * cur_thread_num.  sf_read_rule_states: rules first .. first + n - 1. */
int  sf_node_digests(sf_engine* e, uint64_t* out, uint32_t n_rows);
int  sf_read_rule_states(sf_engine* e, uint32_t first, uint32_t n, sf_rule_state* out);
/* The origin node of (resource, origin) (ClusterNode.getOrCreateOriginNode,
 * ClusterNode.java:101-120) and the DefaultNode of (context, resource)
 * (NodeSelectorSlot), for the resources whose rules read them.  The engine
 * keeps an origin node while the resource has a DIRECT rule with a limit_app
 * other than "default", a context node while it has a CHAIN rule naming that
 * context (statistics start when such a rule is loaded: DESIGN.md §2
 * divergences); SF_ERR_INVALID for a node it does not keep. */
int  sf_read_origin_node(sf_engine* e, uint32_t resource, uint32_t origin, sf_node_state* out);
int  sf_read_context_node(sf_engine* e, uint32_t context, uint32_t resource, sf_node_state* out);
int  sf_snapshot(sf_engine* e, int64_t now_ms, sf_metric_row* out, uint32_t cap, uint32_t* n_out);

/* metrics.log (MetricTimerListener -> MetricWriter) ------------------------
 * Resource names and types (ResourceWrapper.getName / getResourceType) for
 * the log lines: name of resource id i = bytes[offsets[i], offsets[i+1]),
 * types[i] (ResourceTypeConstants, or NULL = COMMON 0); copied to HBM.
 * A resource without a loaded name is written as its decimal id. */
#define SF_RES_ENTRY_NODE 0xFFFFFFFFu   /* Constants.ENTRY_NODE, "__total_inbound_traffic__" */
int  sf_load_resource_names(sf_engine* e, const char* bytes, const uint64_t* offsets, const int32_t* types,
                            uint32_t n);
/* One MetricTimerListener.run (MetricTimerListener.java:40-69) over this
 * shard at now_ms: StatisticNode.metrics() of every ClusterNode (resource id
 * order) and, if include_entry_node, of ENTRY_NODE (last within a second),
 * grouped by second ascending (the TreeMap), each row written as
 * MetricNode.toFatString (MetricNode.java:213-229) the way MetricWriter.write
 * appends it (MetricWriter.java:120-170); the date in a fixed zone of
 * tz_offset_ms.  Updates every node's lastFetchTime, like the reference.
 * *len_out = bytes needed; SF_ERR_CAPACITY if > cap (state still advanced). */
int  sf_metric_log(sf_engine* e, int64_t now_ms, int64_t tz_offset_ms, int include_entry_node, char* out,
                   uint64_t cap, uint64_t* len_out, uint32_t* n_lines);
/* MetricNode.toFatString of caller rows (formatting alone, on the GPU). */
int  sf_format_metric_rows(sf_engine* e, const sf_metric_row* rows, uint32_t n, int64_t tz_offset_ms, char* out,
                           uint64_t cap, uint64_t* len_out);

/* SystemRules on a resource-sharded node, the per-window exchange (DESIGN.md
 * §5; replaces SystemSlot's reads of Constants.ENTRY_NODE,
 * SystemRuleManager.checkSystem SystemRuleManager.java:291-348, when the node's
 * resources are split over engines).  Every rank calls it with its shard's
 * events of the same node batch, in submission order, and `seq` = their
 * global sequence numbers (increasing; time non-decreasing in them).  The
 * ranks exchange per-window aggregates only (a rank's ENTRY_NODE contribution
 * and a 128-bin histogram of its undecided IN entries per level, 4.2 KB): with
 * `allgather` NULL over the engine's RCCL communicator (sf_comm_init; device
 * buffers, stream-ordered), else through the callback, which must return
 * rank 0's `bytes`, rank 1's, ... in `recv` (0 = success; host buffers).  The
 * verdicts, and every rank's ENTRY_NODE, equal one engine deciding the whole
 * node batch.  SF_ERR_UNSUPPORTED (every rank alike) when a loaded SystemRule
 * has thread / average-RT / BBR checks or an IN entry has acquireCount < 0:
 * use the event all-gather protocol (sf_system_plan, sf_submit_forced,
 * sf_entry_node_add).  Without SystemRules it is sf_submit. */
typedef int (*sf_allgather_fn)(void* ctx, const void* send, void* recv, uint64_t bytes);
#define SF_SYSX_MSG_BYTES 4224     /* one rank's message of a plan level (sf_sysx.h SX_WORDS * 8) */
int  sf_submit_node(sf_engine* e, const sf_event_batch* in, const int64_t* seq, sf_verdicts* out,
                    sf_allgather_fn allgather, void* ctx);

/* Node-wide Constants.ENTRY_NODE over the resource shards of a node: one
 * engine per GPU, joined by RCCL (xGMI).  Rank 0 creates the id, the host
 * distributes it (any channel), every rank calls sf_comm_init.  The merge is
 * exact: per bucket slot the node-wide latest window (all-reduce MAX), then
 * SUM of its counters, MIN of minRt, SUM of curThreadNum (sentinel_amd/dist.py). */
int  sf_comm_unique_id(uint8_t* out, size_t len /* >= 128 */);
int  sf_comm_init(sf_engine* e, int nranks, int rank, const uint8_t* id, size_t len);
int  sf_entry_node_allreduce(sf_engine* e, sf_node_state* out);
/* The ENTRY_NODE whose "__total_inbound_traffic__" line sf_metric_log writes
 * (MetricTimerListener.java:40-69 reads Constants.ENTRY_NODE, the node-wide
 * node): NULL = this engine's own (its shard's inbound traffic, the default);
 * else a copy of *node -- on the rank that writes the node's metrics.log, the
 * node-wide merge sf_entry_node_allreduce returned, set before each fetch.
 * Its windows are reported; lastFetchTime stays this engine's.  Decisions
 * (SystemRule) never read it. */
int  sf_set_report_entry_node(sf_engine* e, const sf_node_state* node);

/* ---- DegradeSlot circuit breakers -----------------
 * Replaces DegradeSlot.performChecking / exit (DegradeSlot.java:50-94) and
 * the breakers behind DegradeRuleManager.getCircuitBreakers
 * (DegradeRuleManager.java:236-265): ResponseTimeCircuitBreaker
 * (ResponseTimeCircuitBreaker.java:64-130) and ExceptionCircuitBreaker
 * (ExceptionCircuitBreaker.java:64-119) over AbstractCircuitBreaker's
 * CLOSED/OPEN/HALF_OPEN machine (AbstractCircuitBreaker.java:67-173).
 * sf_degrade_submit runs a degrade-only chain: ENTRY -> tryPass of each
 * breaker of the resource in rule order (first refusal = DegradeException;
 * a breaker moved OPEN->HALF_OPEN by this entry falls back to OPEN through
 * the whenTerminate hook, :113-129); EXIT of a passed entry ->
 * onRequestComplete of every breaker with rt = exit ts - create ts and the
 * SF_EV_ERROR flag (Tracer error).  A reload keeps the breaker (and its
 * state) of every rule equal to a loaded one on the same resource
 * (DegradeRuleManager.getExistingSameCbOrNew :151-163; two equal new rules
 * that would share one breaker are refused with SF_ERR_UNSUPPORTED); a
 * failed load leaves the loaded rules in place.  Event times must be
 * non-decreasing within a batch and across batches (SF_ERR_INVALID).
 * With degrade rules loaded, sf_submit runs DegradeSlot last in its chain
 * (after SystemSlot, ParamFlowSlot, FlowSlot): the same breakers, a
 * DegradeException counted as a block by StatisticSlot, entries blocked
 * earlier (or PriorityWaitException) never checked, and only exits of
 * entries that passed the chain completing requests.  Both calls share the
 * breaker state.                                                          */
#define SF_DEGRADE_GRADE_RT              0   /* RuleConstant.DEGRADE_GRADE_RT */
#define SF_DEGRADE_GRADE_EXCEPTION_RATIO 1
#define SF_DEGRADE_GRADE_EXCEPTION_COUNT 2
#define SF_V_BLOCK_DEGRADE 8   /* DegradeException (rule_idx = breaker index in the resource's list) */
#define SF_V_BLOCK_OTHER   9   /* SF_EV_BLOCKED entry (AuthorityException): counted as a block, no check ran */
#define SF_CB_CLOSED    0
#define SF_CB_OPEN      1
#define SF_CB_HALF_OPEN 2
#define SF_MAX_BREAKERS_PER_RESOURCE 64

typedef struct sf_degrade_rule {   /* DegradeRule (DegradeRule.java) */
    uint32_t resource;
    int32_t  grade;                /* SF_DEGRADE_GRADE_* */
    double   count;                /* RT: max allowed rt (Math.round); ratio / count threshold */
    int32_t  time_window_s;        /* recovery timeout = time_window_s * 1000 */
    int32_t  min_request_amount;   /* default 5 */
    double   slow_ratio_threshold; /* RT grade only, default 1.0 */
    int32_t  stat_interval_ms;     /* default 1000 */
    int32_t  pad;
} sf_degrade_rule;

typedef struct sf_breaker_state {  /* one circuit breaker after the last batch */
    int32_t  state;                /* SF_CB_* */
    int32_t  pad;
    int64_t  next_retry_ms;        /* nextRetryTimestamp */
    int64_t  window_start;         /* its single stat bucket (LeapArray(1, statIntervalMs)) */
    int64_t  hit_count;            /* slowCount (RT) / errorCount (exception) */
    int64_t  total_count;
} sf_breaker_state;

/* Invalid rules (DegradeRuleManager.isValidRule :183-204) are skipped like
 * the reference; *n_loaded (may be NULL) = breakers installed, whose
 * indices (load order of the valid rules) sf_read_breaker takes. */
int  sf_load_degrade_rules(sf_engine* e, const sf_degrade_rule* rules, uint32_t n, uint32_t* n_loaded);
int  sf_degrade_submit(sf_engine* e, const sf_event_batch* in, sf_verdicts* out);
int  sf_read_breaker(sf_engine* e, uint32_t breaker_index, sf_breaker_state* out);

/* ---- rule-list order (host only, no engine) -----------------------------
 * The order in which the reference's managers hold a resource's rules:
 * FlowRuleUtil.buildFlowRuleMap (FlowRuleUtil.java:83-130) drops invalid
 * rules, collapses equal ones in a java.util.HashSet, lists the set in its
 * (JDK 8 HashMap) iteration order and sorts it stably with FlowRuleComparator
 * (FlowRuleComparator.java:27-57: cluster-mode rules last, limitApp
 * "default" after specific origins); ParamFlowRuleUtil.buildParamRuleMap
 * (ParamFlowRuleUtil.java:138-186) the same without the sort.  Rule order
 * decides which rule blocks (and which ParamFlow rules consumed tokens), so a
 * host that loads rules from a Java rule list passes them to sf_load_*_rules
 * in this order.  The String fields enter through their Java hash codes:    */
typedef struct sf_rule_key {
    int32_t  resource_hash;   /* getResource().hashCode()                          */
    uint32_t limit_app_id;    /* 0 "default" (also a blank limitApp), 1 "other", >1 an origin */
    int32_t  limit_app_hash;  /* getLimitApp().hashCode() (unused when id is 0)    */
    int32_t  extra_hash;      /* flow: refResource.hashCode() (0 for null);
                                 param: paramFlowItemList.hashCode()               */
    int32_t  cluster_hash;    /* flow: clusterConfig.hashCode() (0 for null, the local
                                 rule); equal rules must have equal values here      */
} sf_rule_key;
/* order[0 .. *n_out): indices of the kept rules, resources in order of first
 * appearance, each resource's rules in the manager's order.  Validity is
 * FlowRuleUtil.isValidRule (:170-254) / ParamFlowRuleUtil.isValidRule (:46-52)
 * on the struct fields; a cluster-mode or RELATE/CHAIN flow rule is taken to
 * carry a valid clusterConfig / non-blank refResource.
 * SF_ERR_UNSUPPORTED if a HashMap bin would be treeified (>8 equal-bucket
 * rules of one resource in a 64-slot table): not modelled.                   */
int  sf_flow_rule_order(const sf_flow_rule* rules, const sf_rule_key* keys, uint32_t n, uint32_t* order,
                        uint32_t* n_out);
int  sf_param_rule_order(const sf_param_rule* rules, const sf_rule_key* keys, uint32_t n, const sf_hot_item* items,
                         uint32_t n_items, uint32_t* order, uint32_t* n_out);

/* Device helpers so hosts without a GPU framework can stage HBM inputs. */
int  sf_device_alloc(sf_engine* e, size_t bytes, void** ptr);
int  sf_device_free(sf_engine* e, void* ptr);
int  sf_memcpy(sf_engine* e, void* dst, const void* src, size_t bytes, int kind /*0 H2D 1 D2H 2 D2D*/);
/* Page-locked host memory (hipHostMalloc): batch and verdict arrays of an
 * SF_MEM_HOST sf_submit placed here move over PCIe by DMA at full rate
 * instead of through pageable staging (the Java flusher's off-heap buffers). */
int  sf_host_alloc(sf_engine* e, size_t bytes, void** ptr);
int  sf_host_free(sf_engine* e, void* ptr);
int  sf_sync(sf_engine* e);      /* waits for sf_submit_async batches; their first error */
int  sf_get_stats(sf_engine* e, sf_stats* out);
int  sf_set_timing(sf_engine* e, int enabled);
/* diagnostics: the exact hot-parameter table (ParameterMetric maps): occupied
 * slots, capacity, and the longest probe distance from a key's home slot
 * (at most 4096: an insert that would go farther is SF_ERR_CAPACITY). */
int  sf_param_table_stats(sf_engine* e, uint64_t* used, uint64_t* capacity, uint32_t* max_probe);
/* ParameterMetric.getThreadCount(paramIdx, value) (ParameterMetric.java:241-253)
 * of a resource's ParamFlow statistics: the live thread count of one typed
 * parameter value (tag, bits as in sf_event_batch), 0 when it has none. */
int  sf_read_param_thread(sf_engine* e, uint32_t resource, int param_idx, uint8_t tag, uint64_t bits, int64_t* out);
/* diagnostics: per heavy segment of the last sf_submit (timing must be on) */
int  sf_heavy_profile_read(sf_engine* e, sf_heavy_profile* out, uint32_t cap, uint32_t* n_out);

#ifdef __cplusplus
}
#endif
#endif /* SENTINEL_FLOW_H */
