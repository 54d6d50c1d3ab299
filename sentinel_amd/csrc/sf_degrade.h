// DegradeSlot circuit breakers on the GPU.
// Device layout and launchers shared by sf_degrade.hip and sf_engine.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "../../include/sentinel_flow.h"

// Constants of one breaker, precomputed at load (ResponseTimeCircuitBreaker.java:48-56,
// ExceptionCircuitBreaker.java:47-56, AbstractCircuitBreaker.java:47-55).  40 B.
struct DevBreakerRule {
    int32_t grade;       // SF_DEGRADE_GRADE_*
    int32_t min_req;     // minRequestAmount
    int64_t max_rt;      // Math.round(count) (RT grade)
    double  thr;         // slowRatioThreshold (RT) or count (exception grades)
    int64_t recovery;    // timeWindow * 1000
    int64_t interval;    // statIntervalMs (LeapArray(1, interval))
};

// Breaker state lives in HBM as sf_breaker_state (40 B); window_start ==
// DG_WS_NONE means the single bucket was never created.
constexpr int64_t DG_WS_NONE = INT64_MIN;

struct DegradeDev {
    uint32_t n_rres = 0;                 // resources with at least one breaker (dense ids)
    uint32_t key_bits = 1;
    const uint32_t* rr_of = nullptr;     // [R] local resource -> dense id, n_rres if none
    const uint32_t* off = nullptr;       // [n_rres+1] breakers of dense resource k: [off[k], off[k+1])
    const DevBreakerRule* rules = nullptr;
    sf_breaker_state* state = nullptr;
};

struct DegradeBatch {
    uint32_t n;
    const uint32_t* res; const int64_t* ts; const uint8_t* flags;
    const int64_t* eref; const int64_t* cts;
    uint32_t shard_count, shard_index, R;
    int64_t* last_ts;                          // engine clock (non-decreasing across batches)
};

struct alignas(16) DgEv {                      // sorted event of a breaker resource, 32 B
    int64_t t, cr;                             // ts, entry create ts (exits)
    uint32_t idx, fl;                          // submission index, flags | bad << 8
    uint32_t ref, refpos;                      // entry_ref (~0 = none) and its sorted position
};

struct DegradeWork {
    uint32_t cap = 0;
    uint32_t *keys_in = nullptr, *keys_out = nullptr, *idx_in = nullptr, *idx_out = nullptr;
    uint32_t *beg = nullptr, *end = nullptr;   // [n_rres] sorted segment of each breaker resource
    uint32_t beg_cap = 0;
    void* sort_tmp = nullptr; size_t sort_tmp_bytes = 0;
    int* err = nullptr;                        // events outside the shard / bad refs
    uint32_t* heavy = nullptr;                 // [n_rres] long segments for the wave walk
    uint32_t* n_heavy = nullptr;
    DgEv* sev = nullptr;                       // [cap]
    uint32_t* inv = nullptr;                   // [cap] submission index -> sorted position
};

hipError_t dg_sort_bytes(uint32_t n, uint32_t key_bits, size_t* bytes);
// One sf_degrade_submit on stream s: keys + default verdicts, stable sort by
// breaker resource, segment bounds, then the per-resource state-machine walk.
hipError_t dg_launch(const DegradeDev& d, DegradeWork& w, const DegradeBatch& b, uint8_t* status,
                     uint16_t* rule, int32_t* wait, hipStream_t s);
