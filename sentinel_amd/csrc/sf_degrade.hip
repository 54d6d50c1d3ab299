// DegradeSlot circuit breakers on the GPU.
//
// Reference (sentinel-core/.../slots/block/degrade/):
//   DegradeSlot.performChecking / exit           DegradeSlot.java:50-94
//   AbstractCircuitBreaker tryPass + transitions circuitbreaker/AbstractCircuitBreaker.java:67-173
//   ResponseTimeCircuitBreaker.onRequestComplete circuitbreaker/ResponseTimeCircuitBreaker.java:64-130
//   ExceptionCircuitBreaker.onRequestComplete    circuitbreaker/ExceptionCircuitBreaker.java:64-119
//
// A breaker's state is a strict function of its resource's event order, so
// the batch is split by resource (stable radix sort of the events of
// resources that have breakers, keyed by a dense id) and each such resource's
// events are walked in time order by one lane, breaker state in HBM
// (sf_breaker_state, 40 B).  Events of resources without breakers get their
// verdict in the first, fully coalesced pass and are never touched again.
#include <cstring>
#include <rocprim/rocprim.hpp>
#include "sf_degrade.h"

namespace {

constexpr int BLK = 256;

__global__ void __launch_bounds__(BLK) k_dg_keys(DegradeDev d, DegradeBatch b, uint32_t* keys, uint32_t* idx,
                                                 uint8_t* status, uint16_t* rule, int32_t* wait, int* err) {
    const uint32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= b.n) return;
    const uint32_t r = b.res[i];
    const uint8_t f = b.flags[i];
    uint32_t key = d.n_rres;
    if (r % b.shard_count != b.shard_index || r / b.shard_count >= b.R) {
        atomicOr(err, 1);
    } else if (d.n_rres) {               // rr_of exists once degrade rules were loaded
        key = d.rr_of[r / b.shard_count];
    }
    keys[i] = key;
    idx[i] = i;
    // no breaker (or not yet decided): entries pass the degrade check, exits record
    status[i] = (f & SF_EV_EXIT) ? SF_V_EXIT : SF_V_PASS;
    if (rule) rule[i] = 0;
    if (wait) wait[i] = 0;
}

__global__ void __launch_bounds__(BLK) k_dg_bounds(const uint32_t* keys, uint32_t n, uint32_t none, uint32_t* beg,
                                                   uint32_t* end) {
    const uint32_t j = blockIdx.x * BLK + threadIdx.x;
    if (j >= n) return;
    const uint32_t k = keys[j];
    if (k >= none) return;
    if (j == 0 || keys[j - 1] != k) beg[k] = j;
    if (j == n - 1 || keys[j + 1] != k) end[k] = j + 1;
}

__device__ __forceinline__ void dg_roll(sf_breaker_state& s, const DevBreakerRule& r, int64_t t) {
    // LeapArray(1, interval).currentWindow(t): create, keep, or reset the single bucket (LeapArray.java:128-225)
    const int64_t ws = t - t % r.interval;
    if (s.window_start == DG_WS_NONE || ws > s.window_start) {
        s.window_start = ws;
        s.hit_count = 0;
        s.total_count = 0;
    }
}

__device__ __forceinline__ void dg_open(sf_breaker_state& s, const DevBreakerRule& r, int64_t t) {
    s.state = SF_CB_OPEN;
    s.next_retry_ms = t + r.recovery;          // updateNextRetryTimestamp (AbstractCircuitBreaker.java:93-95)
}

// onRequestComplete + handleStateChangeWhenThresholdExceeded of one breaker.
__device__ __forceinline__ void dg_complete(sf_breaker_state& s, const DevBreakerRule& r, int64_t t, int64_t rt,
                                            bool error) {
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

// One lane walks one breaker resource's events in time order.
__global__ void __launch_bounds__(BLK) k_dg_walk(DegradeDev d, DegradeBatch b, const uint32_t* perm,
                                                 const uint32_t* beg, const uint32_t* end, uint8_t* status,
                                                 uint16_t* rule, int* err) {
    const uint32_t k = blockIdx.x * BLK + threadIdx.x;
    if (k >= d.n_rres) return;
    const uint32_t j0 = beg[k], j1 = end[k];
    if (j0 >= j1) return;
    const uint32_t c0 = d.off[k], c1 = d.off[k + 1];
    const DevBreakerRule* R = d.rules;
    sf_breaker_state* S = d.state;
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t i = perm[j];
        const int64_t t = b.ts[i];
        const uint8_t f = b.flags[i];
        if (!(f & SF_EV_EXIT)) {
            // DegradeSlot.performChecking: tryPass of each breaker, first refusal blocks
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
            if (blocked >= 0) {
                // whenTerminate hook of the probes this entry opened: HALF_OPEN -> OPEN, retry time kept
                while (moved) {
                    const int q = __builtin_ctzll(moved);
                    moved &= moved - 1;
                    if (S[c0 + q].state == SF_CB_HALF_OPEN) S[c0 + q].state = SF_CB_OPEN;
                }
                status[i] = SF_V_BLOCK_DEGRADE;
                if (rule) rule[i] = (uint16_t)blocked;
            }
            continue;
        }
        // EXIT: DegradeSlot.exit -> onRequestComplete of every breaker (passed entries only)
        int64_t created;
        const int64_t ref = b.eref ? b.eref[i] : -1;
        if (ref >= 0) {
            if ((uint64_t)ref >= b.n) { atomicOr(err, 2); continue; }
            if (status[ref] == SF_V_BLOCK_DEGRADE) { status[i] = SF_V_EXIT_IGNORED; continue; }
            created = b.ts[ref];
        } else {
            if (!b.cts) { atomicOr(err, 2); continue; }
            created = b.cts[i];
        }
        const int64_t rt = t - created;
        const bool error = (f & SF_EV_ERROR) != 0;
        for (uint32_t c = c0; c < c1; c++) {
            sf_breaker_state s = S[c];
            dg_complete(s, R[c], t, rt, error);
            S[c] = s;
        }
    }
}

inline uint32_t blocks(uint32_t n) { return (n + BLK - 1) / BLK; }

}  // namespace

hipError_t dg_sort_bytes(uint32_t n, uint32_t key_bits, size_t* bytes) {
    return rocprim::radix_sort_pairs(nullptr, *bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (uint32_t*)nullptr, n, 0u, key_bits);
}

hipError_t dg_launch(const DegradeDev& d, DegradeWork& w, const DegradeBatch& b, uint8_t* status, uint16_t* rule,
                     int32_t* wait, hipStream_t s) {
    if (b.n == 0) return hipSuccess;
    k_dg_keys<<<blocks(b.n), BLK, 0, s>>>(d, b, w.keys_in, w.idx_in, status, rule, wait, w.err);
    if (d.n_rres == 0) return hipGetLastError();
    size_t bytes = w.sort_tmp_bytes;
    hipError_t e = rocprim::radix_sort_pairs(w.sort_tmp, bytes, w.keys_in, w.keys_out, w.idx_in, w.idx_out, b.n, 0u,
                                             d.key_bits, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(w.end, 0, (size_t)d.n_rres * 4, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(w.beg, 0, (size_t)d.n_rres * 4, s);
    if (e != hipSuccess) return e;
    k_dg_bounds<<<blocks(b.n), BLK, 0, s>>>(w.keys_out, b.n, d.n_rres, w.beg, w.end);
    k_dg_walk<<<blocks(d.n_rres), BLK, 0, s>>>(d, b, w.idx_out, w.beg, w.end, status, rule, w.err);
    return hipGetLastError();
}
