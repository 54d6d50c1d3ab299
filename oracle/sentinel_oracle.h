/*
 * sentinel_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A single-threaded, line-faithful C restatement of the reference's
 * statistics-and-check path (fan1994song/Sentinel @ 1.8.6-SNAPSHOT, Java).
 * It is the parity checker for the HIP engine and the "port" CPU baseline.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product (sentinel_amd/, libsentinel_flow.so) never links it.
 *
 * Parity pinning: the reference is Java and no JDK exists here, so the
 * reference cannot be run.  This restatement is pinned by transcribing the
 * reference's own deterministic unit tests (mocked TimeUtil clock) as
 * known-answer tests: tests/test_oracle_kat.py (SURVEY.md §8c list).
 *
 * Every TimeUtil.currentTimeMillis() call of the reference reads the mocked
 * clock so_set_time() (TimeUtil.java:222-224, AbstractTimeBasedTest).
 */
#ifndef SENTINEL_ORACLE_H
#define SENTINEL_ORACLE_H

#include <stdint.h>
#include "../include/sentinel_flow.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- mocked clock ---- */
void    so_set_time(int64_t t);
int64_t so_now(void);
void    so_set_statistic_max_rt(int64_t rt);

/* ---- Java numeric helpers (exposed for tests) ---- */
int64_t so_java_round(double a);          /* Math.round(double)         */
double  so_java_next_up(double a);        /* Math.nextUp(double)        */
int32_t so_java_d2i(double a);            /* (int) double               */
int64_t so_java_d2l(double a);            /* (long) double              */

/* ---- LeapArray family (object API for the window-core KATs) ---- */
#define SO_LA_BUCKET      0   /* BucketLeapArray                */
#define SO_LA_OCCUPIABLE  1   /* OccupiableBucketLeapArray      */
#define SO_LA_FUTURE      2   /* FutureBucketLeapArray          */
#define SO_LA_UNARY       3   /* UnaryLeapArray (LongAdder)     */
#define SO_LA_CLUSTER     4   /* ClusterMetricLeapArray         */

typedef struct so_leap_array so_leap_array;
typedef struct so_wrap so_wrap;

so_leap_array* so_la_new(int kind, int sample_count, int interval_ms);
void     so_la_free(so_leap_array* a);
so_wrap* so_la_current_window(so_leap_array* a, int64_t t);     /* currentWindow(long) */
so_wrap* so_la_current_window_now(so_leap_array* a);            /* currentWindow()     */
so_wrap* so_la_previous_window(so_leap_array* a, int64_t t);    /* getPreviousWindow(long) */
so_wrap* so_la_valid_head(so_leap_array* a, int64_t t);         /* getValidHead(long)  */
so_wrap* so_la_window_value(so_leap_array* a, int64_t t);       /* getWindowValue(long) (wrap of it) */
/* values(t) / list(t): writes up to cap wraps, returns the count */
int      so_la_values(so_leap_array* a, int64_t t, so_wrap** out, int cap);
int      so_la_list_now(so_leap_array* a, so_wrap** out, int cap);
int64_t  so_la_current_waiting(so_leap_array* a);               /* Occupiable          */
void     so_la_add_waiting(so_leap_array* a, int64_t t, int32_t c);
int64_t  so_wrap_start(const so_wrap* w);
int64_t  so_wrap_length(const so_wrap* w);
/* MetricBucket counters: event = MetricEvent ordinal (PASS..OCCUPIED_PASS);
 * cluster buckets: ClusterFlowEvent ordinal; unary: event ignored */
int64_t  so_wrap_get(const so_wrap* w, int event);
void     so_wrap_add(so_wrap* w, int event, int64_t n);
int64_t  so_wrap_min_rt(const so_wrap* w);
void     so_wrap_add_rt(so_wrap* w, int64_t rt);

/* ---- ArrayMetric over an occupiable or plain array ---- */
typedef struct so_array_metric so_array_metric;
so_array_metric* so_am_new(int sample_count, int interval_ms, int enable_occupy);
void    so_am_free(so_array_metric* m);
int64_t so_am_pass(so_array_metric* m);
int64_t so_am_block(so_array_metric* m);
int64_t so_am_success(so_array_metric* m);
int64_t so_am_exception(so_array_metric* m);
int64_t so_am_rt(so_array_metric* m);
int64_t so_am_min_rt(so_array_metric* m);
int64_t so_am_max_success(so_array_metric* m);
int64_t so_am_occupied_pass(so_array_metric* m);
int64_t so_am_previous_window_pass(so_array_metric* m);
int64_t so_am_previous_window_block(so_array_metric* m);
int64_t so_am_window_pass(so_array_metric* m, int64_t t);
int64_t so_am_waiting(so_array_metric* m);
void    so_am_add(so_array_metric* m, int event, int32_t n);  /* addPass/addBlock/... */
void    so_am_add_rt(so_array_metric* m, int64_t rt);
void    so_am_add_waiting(so_array_metric* m, int64_t t, int32_t c);
/* details(): MetricNode rows of the minute-style array, filtered by
 * (ts >= lo) when filter != 0.  Returns row count. */
int     so_am_details(so_array_metric* m, int filter, int64_t lo, sf_metric_row* out, int cap);

/* ---- StatisticNode ---- */
typedef struct so_node so_node;
so_node* so_node_new(void);
void     so_node_free(so_node* n);
double   so_node_pass_qps(so_node* n);
double   so_node_block_qps(so_node* n);
double   so_node_previous_pass_qps(so_node* n);
double   so_node_avg_rt(so_node* n);
double   so_node_min_rt(so_node* n);
double   so_node_success_qps(so_node* n);
double   so_node_max_success_qps(so_node* n);
int32_t  so_node_cur_thread_num(so_node* n);
void     so_node_add_pass_request(so_node* n, int32_t c);
void     so_node_increase_block_qps(so_node* n, int32_t c);
void     so_node_add_rt_and_success(so_node* n, int64_t rt, int32_t c);
void     so_node_increase_exception_qps(so_node* n, int32_t c);
void     so_node_increase_thread_num(so_node* n);
void     so_node_decrease_thread_num(so_node* n);
int64_t  so_node_try_occupy_next(so_node* n, int64_t now, int32_t c, double threshold);
int64_t  so_node_waiting(so_node* n);
void     so_node_add_waiting_request(so_node* n, int64_t future, int32_t c);
void     so_node_add_occupied_pass(so_node* n, int32_t c);
void     so_node_read(so_node* n, sf_node_state* out);

/* A mocked Node (Mockito in the controller tests): fixed readings. */
typedef struct so_mock_node {
    double  pass_qps;
    double  previous_pass_qps;
    int32_t cur_thread_num;
} so_mock_node;

/* ---- traffic shaping controllers ---- */
typedef struct so_controller so_controller;
so_controller* so_ctrl_default(double count, int grade);
so_controller* so_ctrl_warm_up(double count, int period_sec, int cold_factor);
so_controller* so_ctrl_rate_limiter(int timeout_ms, double count);
so_controller* so_ctrl_warm_up_rate_limiter(double count, int period_sec, int timeout_ms, int cold_factor);
void so_ctrl_free(so_controller* c);
/* canPass against a real node (node != NULL) or a mock (mock != NULL).
 * Returns 1 pass / 0 block.  *wait_ms: Thread.sleep the reference would do;
 * *prio_wait: 1 when the reference throws PriorityWaitException. */
int  so_ctrl_can_pass(so_controller* c, so_node* node, const so_mock_node* mock,
                      int32_t acquire, int prioritized, int64_t* wait_ms, int* prio_wait);
void so_ctrl_state(const so_controller* c, sf_rule_state* out);
/* WarmUp internals exposed for KATs */
int32_t so_ctrl_warning_token(const so_controller* c);
int32_t so_ctrl_max_token(const so_controller* c);
double  so_ctrl_slope(const so_controller* c);

/* ---- ParamFlowChecker (object level) ---- */
typedef struct so_param_metric so_param_metric;      /* ParameterMetric */
so_param_metric* so_pm_new(void);
so_param_metric* so_pm_new_mode(int lru);   /* lru: CacheMaps as ConcurrentLinkedHashMap LRUs */
uint64_t so_pm_evictions(so_param_metric* pm);
int64_t so_pm_thread_peek(so_param_metric* pm, int param_idx, uint8_t tag, uint64_t bits);
void so_pm_free(so_param_metric* pm);
/* passSingleValueCheck(rule, acquireCount, value); rule_key identifies the
 * rule's counter maps inside pm (ParameterMetric maps keyed by rule).      */
int  so_param_pass_single(so_param_metric* pm, int rule_key, const sf_param_rule* rule,
                          const sf_hot_item* items, int32_t acquire,
                          uint8_t tag, uint64_t bits, int64_t* wait_ms);
void so_pm_initialize(so_param_metric* pm, int rule_key, const sf_param_rule* rule);
void so_pm_add_thread(so_param_metric* pm, int param_idx, uint8_t tag, uint64_t bits);
void so_pm_dec_thread(so_param_metric* pm, int param_idx, uint8_t tag, uint64_t bits);
int64_t so_pm_thread_count(so_param_metric* pm, int param_idx, uint8_t tag, uint64_t bits);
/* token / time counter read-back: returns 1 when present */
int  so_pm_read(so_param_metric* pm, int rule_key, uint8_t tag, uint64_t bits,
                int64_t* last_add_or_pass_time, int64_t* tokens, int* has_tokens);

/* ---- cluster server objects ---- */
typedef struct so_cluster_metric so_cluster_metric;
so_cluster_metric* so_cm_new(int sample_count, int interval_ms);
void    so_cm_free(so_cluster_metric* m);
void    so_cm_add(so_cluster_metric* m, int event, int64_t n);
int64_t so_cm_sum(so_cluster_metric* m, int event);
double  so_cm_avg(so_cluster_metric* m, int event);
int32_t so_cm_try_occupy_next(so_cluster_metric* m, int event, int32_t c, double threshold);

typedef struct so_cluster_param_metric so_cluster_param_metric;
so_cluster_param_metric* so_cpm_new(int sample_count, int interval_ms);
void    so_cpm_free(so_cluster_param_metric* m);
void    so_cpm_add_value(so_cluster_param_metric* m, uint8_t tag, uint64_t bits, int32_t c);
int64_t so_cpm_sum(so_cluster_param_metric* m, uint8_t tag, uint64_t bits);
double  so_cpm_avg(so_cluster_param_metric* m, uint8_t tag, uint64_t bits);

typedef struct so_request_limiter so_request_limiter;
so_request_limiter* so_rl_new(double qps_allowed);
void    so_rl_free(so_request_limiter* l);
int     so_rl_try_pass(so_request_limiter* l);
int64_t so_rl_sum(so_request_limiter* l);
int     so_rl_can_pass(so_request_limiter* l);
void    so_rl_add(so_request_limiter* l, int32_t x);

/* ---- replay engine: same ABI shapes as the product (host memory only) ---- */
typedef struct so_engine so_engine;
so_engine* so_create(const sf_config* cfg);
int  so_set_param_lru(so_engine* e, int on);
int  so_param_lru_stats(so_engine* e, uint64_t* evictions, uint64_t* spins);
void so_destroy(so_engine* e);
int  so_load_flow_rules(so_engine* e, const sf_flow_rule* rules, uint32_t n);
int  so_load_param_rules(so_engine* e, const sf_param_rule* rules, uint32_t n,
                         const sf_hot_item* items, uint32_t n_items);
int  so_load_system_rules(so_engine* e, const sf_system_rule* rules, uint32_t n);
int  so_set_system_status(so_engine* e, double load, double cpu);
int  so_submit(so_engine* e, const sf_event_batch* in, sf_verdicts* out);
int  so_system_plan(so_engine* e, const sf_event_batch* in, const uint8_t* status, uint32_t p, uint32_t* q,
                    uint8_t* sys_mask);
int  so_submit_forced(so_engine* e, const sf_event_batch* in, sf_verdicts* out, const uint8_t* sys_mask);
int  so_entry_node_add(so_engine* e, const sf_event_batch* in, const uint8_t* status);
int  so_load_degrade_rules(so_engine* e, const sf_degrade_rule* rules, uint32_t n, uint32_t* n_loaded);
int  so_read_breaker(so_engine* e, uint32_t k, sf_breaker_state* out);
int  so_read_node(so_engine* e, uint32_t res, sf_node_state* out);
int  so_read_origin_node(so_engine* e, uint32_t res, uint32_t origin, sf_node_state* out);
int  so_read_context_node(so_engine* e, uint32_t context, uint32_t res, sf_node_state* out);
/* FlowRuleChecker.selectNodeByRequesterAndStrategy of loaded rule rule_index
 * for a Context (origin, name): SO_SEL_* (-1: bad index). */
enum { SO_SEL_NONE = 0, SO_SEL_CLUSTER = 1, SO_SEL_ORIGIN = 2, SO_SEL_CONTEXT = 3, SO_SEL_REF = 4 };
int  so_select_node(so_engine* e, uint32_t rule_index, uint32_t origin, uint32_t context);
int  so_read_entry_node(so_engine* e, sf_node_state* out);
int  so_read_rule_state(so_engine* e, uint32_t rule_index, sf_rule_state* out);
uint64_t so_node_digest(const sf_node_state* s, int sample_count);
int  so_node_digests(so_engine* e, uint64_t* out, uint32_t n_rows);      /* one per local row l < n_rows */
int  so_read_rule_states(so_engine* e, uint32_t first, uint32_t n, sf_rule_state* out);
int  so_read_param(so_engine* e, uint32_t param_rule_index, uint8_t tag, uint64_t bits,
                   int64_t* time_value, int64_t* tokens, int* has_tokens);
int32_t so_param_rule_idx(so_engine* e, uint32_t param_rule_index);
int64_t so_param_thread(so_engine* e, uint32_t res, int param_idx, uint8_t tag, uint64_t bits);
int  so_snapshot(so_engine* e, int64_t now, sf_metric_row* out, uint32_t cap, uint32_t* n_out);
/* metrics.log lines (MetricTimerListener / MetricWriter / MetricNode.toFatString) */
typedef struct so_names { const char* bytes; const uint64_t* offsets; const int32_t* types; uint32_t n; } so_names;
int  so_format_fat(const so_names* nt, const sf_metric_row* rows, uint32_t n, int64_t tz_offset_ms, char* out,
                   uint64_t cap, uint64_t* len_out);
int  so_set_report_entry_node(so_engine* e, const sf_node_state* node);
int  so_metric_log(so_engine* e, const so_names* nt, int64_t now, int64_t tz_offset_ms, int include_entry_node,
                   char* out, uint64_t cap, uint64_t* len_out, uint32_t* n_lines);
int  so_load_namespaces(so_engine* e, const sf_namespace* ns, uint32_t n);
int  so_load_cluster_rules(so_engine* e, const sf_cluster_flow_rule* flow, uint32_t n_flow,
                           const sf_cluster_param_rule* param, uint32_t n_param,
                           const sf_hot_item* items, uint32_t n_items);
int  so_request_tokens(so_engine* e, const sf_token_batch* in, sf_token_results* out);
int64_t so_cluster_sum(so_engine* e, int64_t flow_id, int event, int64_t now);
/* token-server wire path (sf_serve_frames contract, sentinel_flow.h) */
uint64_t so_string_key(const uint8_t* b, uint32_t len);
int  so_serve_frames(so_engine* e, const sf_wire_batch* in, sf_wire_out* out);

#ifdef __cplusplus
}
#endif
#endif
