// sf_token.h — device state and launch interface of the batched cluster
// token server (product code): DefaultTokenService.requestToken /
// requestParamToken for a time-ordered batch of requests.
//
// Reference (CS = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster):
//   DefaultTokenService          CS/flow/DefaultTokenService.java:39-72
//   ClusterFlowChecker           CS/flow/ClusterFlowChecker.java:38-112
//   ClusterParamFlowChecker      CS/flow/ClusterParamFlowChecker.java:42-120
//   ClusterMetric                CS/flow/statistic/metric/ClusterMetric.java:39-98
//   ClusterMetricLeapArray       CS/flow/statistic/metric/ClusterMetricLeapArray.java:34-92
//   ClusterParamMetric           CS/flow/statistic/metric/ClusterParamMetric.java:52-88
//   ClusterParameterLeapArray    CS/flow/statistic/metric/ClusterParameterLeapArray.java:39-49
//   GlobalRequestLimiter         CS/flow/statistic/limit/GlobalRequestLimiter.java:46-55
//   RequestLimiter               CS/flow/statistic/limit/RequestLimiter.java:51-87
//
// HBM layout:
//   rules   [n_flow + n_param]  ClRule: flow rules first, then param rules
//   fstate  [n_flow]            ClFlowState: the ClusterMetricLeapArray of one flowId
//   idtab   open-addressed      flow_id -> (flow rule index, param rule index)
//   ns / lim [n_ns]             namespace table and its RequestLimiter (UnaryLeapArray(10, 1000))
//   cptab   open-addressed      (param rule, value) -> per-value window counts
#pragma once
#include "sf_internal.h"

namespace sf {

constexpr int CL_MAXS = 16;                  // sampleCount of a cluster rule (ClusterFlowConfig, default 10)
constexpr int CE_PASS = 0, CE_BLOCK = 1, CE_PASS_REQUEST = 2, CE_BLOCK_REQUEST = 3, CE_OCCUPIED_PASS = 4,
              CE_OCCUPIED_BLOCK = 5, CE_WAITING = 6, CE_COUNT = 7;   // ClusterFlowEvent.java ordinals
constexpr int LIM_S = 10, LIM_WL = 100, LIM_INTERVAL = 1000;        // RequestLimiter: UnaryLeapArray(10, 1000)

struct ClRule {                  // 56 B
    double count;
    int64_t flow_id;
    int32_t threshold_type, ns;  // ns: namespace index, -1 when the namespace is not loaded
    int32_t S, wl;
    int32_t interval, is_param;
    uint32_t item_off, item_cnt;
    uint32_t owner, pad;         // shard deciding this rule's requests (sf_token_shard)
};
struct ClBucket { int64_t ws; int64_t c[CE_COUNT]; };          // WindowWrap<ClusterMetricBucket>, 64 B
struct ClFlowState {                                            // ClusterMetricLeapArray, 1056 B
    ClBucket b[CL_MAXS];
    int64_t occ_pass, occ_req;                                  // occupyCounter[PASS], [PASS_REQUEST]
    int64_t has_occ, pad;
};
struct ClNs { int32_t connected, has_limiter; double max_qps; };
struct LimState { int64_t ws[LIM_S]; int64_t v[LIM_S]; };
struct IdSlot { int64_t id; int32_t flow, param; };             // id == 0: empty (valid ids are > 0)
struct CpSlot {                  // (param rule, value): one value's column of ClusterParameterLeapArray
    uint64_t hi, lo;             // hi: (rule + 1) << 32 | tag, bit 63 while being claimed; 0 empty
    int64_t ws[CL_MAXS];         // window each count belongs to (WS_NONE: never)
    int64_t cnt[CL_MAXS];
};
constexpr uint64_t CP_CLAIM = 1ull << 63;

struct TokState {
    uint32_t n_flow, n_rules, n_ns;
    const ClRule* rules;
    ClFlowState* fstate;
    const IdSlot* idtab; uint64_t id_mask;
    const ClNs* ns; LimState* lim;
    CpSlot* cptab; uint64_t cp_mask;
    const DevHotItem* items;
    double exceed_count, max_occupy_ratio;
    int32_t* err;
    uint8_t* rmulti;             // [n_rules] per call: a param rule with a multi-value request (serial group)
    uint32_t shard_count, shard_index;
};

struct TokBatch {
    uint32_t n;
    const int64_t* flow_id; const int32_t* count; const uint8_t* flags; const int64_t* ts;
    const uint8_t* ptag; const uint64_t* pbits;
    const uint32_t* poff;        // [n+1] Collection<Object> params (values at [poff[i], poff[i+1])), or null
};
struct TokOut { int8_t* status; int32_t* remaining; int32_t* wait; };

struct TokWork {                 // sized for cfg.max_batch requests
    uint8_t* nskey_in; uint8_t* nskey_out;
    uint32_t* idx_in; uint32_t* idx_out;
    uint64_t* key_in; uint64_t* key_out;
    uint32_t* rule_of;           // [n] rule index of a request (valid where pending)
    uint8_t* pending;            // [n] 1: reached the checker
    uint32_t* head; uint32_t* head_scan;
    uint32_t* seg_start; uint32_t* n_seg;
    void* sort8_tmp; size_t sort8_bytes;
    void* sort64_tmp; size_t sort64_bytes;
    void* scan_tmp; size_t scan_bytes;
};

hipError_t tok_query_temp(uint32_t max_n, size_t* sort8, size_t* sort64, size_t* scan);
hipError_t tok_launch(const TokState& ts, TokWork& w, const TokBatch& b, const TokOut& out, hipStream_t s);
hipError_t tok_init_flow_state(ClFlowState* fs, uint32_t n, hipStream_t s);
// ClusterMetric.getSum(event) at time now (rolls the current window like the reference)
hipError_t tok_cluster_sum(const TokState& ts, uint32_t rule, int event, int64_t now, int64_t* d_out, hipStream_t s);

}  // namespace sf
