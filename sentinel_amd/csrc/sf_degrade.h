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

#ifndef SF_HD
#define SF_HD __host__ __device__ __forceinline__
#endif

// ---- one breaker's state machine (host + device: the sf_submit lane walk,
// the degrade-only kernels and tests/hostsim share it)
SF_HD void dg_roll(sf_breaker_state& s, const DevBreakerRule& r, int64_t t) {
    // LeapArray(1, interval).currentWindow(t): create, keep, or reset the single bucket (LeapArray.java:128-225)
    if (t >= 0 && s.window_start != DG_WS_NONE && t >= s.window_start && t - s.window_start < r.interval)
        return;                                // same window: no 64-bit modulo on the serial chain
    const int64_t ws = t - t % r.interval;
    if (s.window_start == DG_WS_NONE || ws > s.window_start) {
        s.window_start = ws;
        s.hit_count = 0;
        s.total_count = 0;
    }
}

SF_HD void dg_open(sf_breaker_state& s, const DevBreakerRule& r, int64_t t) {
    s.state = SF_CB_OPEN;
    s.next_retry_ms = t + r.recovery;          // updateNextRetryTimestamp (AbstractCircuitBreaker.java:93-95)
}

// onRequestComplete + handleStateChangeWhenThresholdExceeded of one breaker
// (ResponseTimeCircuitBreaker.java:64-130, ExceptionCircuitBreaker.java:64-119).
SF_HD void dg_complete(sf_breaker_state& s, const DevBreakerRule& r, int64_t t, int64_t rt, bool error) {
    dg_roll(s, r, t);
    const bool hit = r.grade == SF_DEGRADE_GRADE_RT ? rt > r.max_rt : error;
    s.hit_count += hit;
    s.total_count += 1;
    if (s.state == SF_CB_OPEN) return;
    if (s.state == SF_CB_HALF_OPEN) {
        if (hit) {
            dg_open(s, r, t);                  // fromHalfOpenToOpen
        } else {
            s.state = SF_CB_CLOSED;            // fromHalfOpenToClose -> resetStat (current bucket)
            s.hit_count = 0;
            s.total_count = 0;
        }
        return;
    }
    if (s.total_count < r.min_req) return;
    const double cur = (r.grade == SF_DEGRADE_GRADE_EXCEPTION_COUNT) ? (double)s.hit_count
                                                                      : (double)s.hit_count * 1.0 / (double)s.total_count;
    if (cur > r.thr) {
        dg_open(s, r, t);
    } else if (r.grade == SF_DEGRADE_GRADE_RT && cur == r.thr && r.thr == 1.0) {
        dg_open(s, r, t);                      // ResponseTimeCircuitBreaker.java:126-129
    }
}

// DegradeSlot.performChecking (DegradeSlot.java:50-61): tryPass of the
// resource's breakers [c0, c1) in list order, the first refusal blocks
// (AbstractCircuitBreaker.tryPass :67-82).  A breaker the entry moved OPEN ->
// HALF_OPEN goes back to OPEN when a later breaker refuses it (the
// whenTerminate hook of fromOpenToHalfOpen, :113-129, fires at the blocked
// entry's exit).  Returns the refusing breaker's index in the list, or -1.
SF_HD int dg_entry_check(sf_breaker_state* S, uint32_t c0, uint32_t c1, int64_t t) {
    uint64_t moved = 0;
    int blocked = -1;
    for (uint32_t c = c0; c < c1; c++) {
        const int st = S[c].state;
        if (st == SF_CB_CLOSED) continue;
        if (st == SF_CB_OPEN && t >= S[c].next_retry_ms) {   // retryTimeoutArrived && fromOpenToHalfOpen
            S[c].state = SF_CB_HALF_OPEN;
            moved |= 1ull << (c - c0);
            continue;
        }
        blocked = (int)(c - c0);
        break;
    }
    if (blocked >= 0)
        for (uint32_t q = 0; q < c1 - c0; q++)
            if (((moved >> q) & 1) && S[c0 + q].state == SF_CB_HALF_OPEN) S[c0 + q].state = SF_CB_OPEN;
    return blocked;
}

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
