// sf_decide.h — the per-resource decision interpreter (product code).
//
// One lane owns one resource segment of a time-sorted batch and replays the
// reference semantics event by event against that resource's ClusterNode
// state, which it keeps in registers for the length of the segment:
//   second window (OccupiableBucketLeapArray + borrow FutureBucketLeapArray),
//   the current minute bucket (cached; others read on demand), curThreadNum,
//   the controller states of its flow rules.
// Every TimeUtil.currentTimeMillis() of the reference reads the event time.
//
// Reference citations (CORE = sentinel-core/src/main/java/com/alibaba/csp/sentinel,
// PF = sentinel-extension/sentinel-parameter-flow-control/src/main/java/com/alibaba/csp/sentinel):
//   LeapArray.currentWindow            CORE/slots/statistic/base/LeapArray.java:128-225
//   OccupiableBucketLeapArray          CORE/slots/statistic/metric/occupy/OccupiableBucketLeapArray.java:40-83
//   FutureBucketLeapArray              .../occupy/FutureBucketLeapArray.java:36-52
//   ArrayMetric                        CORE/slots/statistic/metric/ArrayMetric.java:117-330
//   StatisticNode                      CORE/node/StatisticNode.java:205-346
//   StatisticSlot.entry/exit           CORE/slots/statistic/StatisticSlot.java:55-178
//   FlowRuleChecker.checkFlow          CORE/slots/block/flow/FlowRuleChecker.java:44-59
//   Default/WarmUp/RateLimiter/WarmUpRateLimiter controllers  CORE/slots/block/flow/controller/
//   ParamFlowSlot.checkFlow            PF/slots/block/flow/param/ParamFlowSlot.java:56-104
//   ParamFlowChecker                   PF/slots/block/flow/param/ParamFlowChecker.java:48-273
//   ParameterMetric thread counts      PF/slots/block/flow/param/ParameterMetric.java:125-250
//
// This header compiles for the device (the product kernel) and, for the CPU
// unit tests of the kernel logic only, for the host (tests/hostsim).
#pragma once
#include "sf_internal.h"

#ifndef SF_HD
#define SF_HD __host__ __device__ __forceinline__
#endif

namespace sf {

// ---------------------------------------------------------------- Java numerics
SF_HD int64_t d_bits(double x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __double_as_longlong(x);
#else
    int64_t b; __builtin_memcpy(&b, &x, 8); return b;
#endif
}
SF_HD double d_from_bits(int64_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __longlong_as_double(b);
#else
    double x; __builtin_memcpy(&x, &b, 8); return x;
#endif
}
SF_HD int32_t j_d2i(double a) {                        // (int) double, JLS 5.1.3
    if (a != a) return 0;
    if (a >= 2147483647.0) return INT32_MAX;
    if (a <= -2147483648.0) return INT32_MIN;
    return (int32_t)a;
}
SF_HD int64_t j_d2l(double a) {                        // (long) double
    if (a != a) return 0;
    if (a >= 9223372036854775807.0) return INT64_MAX;
    if (a <= -9223372036854775807.0 - 1.0) return INT64_MIN;
    return (int64_t)a;
}
SF_HD int64_t j_round(double a) {                      // Math.round(double), exact half-up
    int64_t bits = d_bits(a);
    int64_t be = (bits & 0x7ff0000000000000LL) >> 52;
    int64_t shift = (52 - 1 + 1023) - be;
    if ((shift & -64) == 0) {
        int64_t r = (bits & 0x000fffffffffffffLL) | (0x000fffffffffffffLL + 1);
        if (bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    return j_d2l(a);
}
SF_HD double j_next_up(double x) {                     // Math.nextUp(double)
    if (x != x || x == __builtin_inf()) return x;
    if (x == 0.0) return d_from_bits(1);
    int64_t b = d_bits(x);
    return d_from_bits(x > 0 ? b + 1 : b - 1);
}
SF_HD int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
SF_HD int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
SF_HD int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
SF_HD int64_t jdiv(int64_t a, int64_t b) { return (a == INT64_MIN && b == -1) ? INT64_MIN : a / b; }

SF_HD uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}

SF_HD Bucket fresh_bucket(int64_t ws, int64_t max_rt) {  // new/reset MetricBucket (MetricBucket.java:37-70)
    Bucket b; b.ws = ws; b.pass = b.block = b.exc = b.succ = b.rt = b.occ = 0; b.min_rt = max_rt; return b;
}

// ============================================================ node state
// MAXS: compile-time capacity of the second window.  With MAXS == 2 every
// bucket access is a branch on a constant index, so the window lives in VGPRs.
template <int MAXS>
struct NodeWin {
    Bucket sec[MAXS];
    Borrow bor[MAXS];
    // LeapArray.java:220-223 hands out a throwaway window for a time older
    // than the slot's bucket; what is added to it is lost, so the interpreter
    // drops those writes instead of keeping a scratch bucket (no lane-private
    // memory: everything stays in VGPRs).
    int64_t threads;
    // minute window: row in HBM + one cached bucket
    Bucket* gmin;
    Bucket mb; int32_t mi; int32_t mdirty;
    int64_t m_ws = INT64_MIN;                  // window start of mb's slot for the last time looked up
    int32_t S, wl, interval;
    int64_t max_rt;
    double interval_sec;
    // last window looked up: events come in time order, so most lookups hit
    // it and skip the 64-bit division by the runtime window length
    int64_t c_ws = INT64_MIN; int32_t c_idx = 0;
    int32_t bdirty = 0;                        // a borrow bucket changed (written back only then)

    // window start and slot of time t (t - t % wl, (t / wl) % S), cached
    SF_HD int64_t win_of(int64_t t, int& idx) {
        if (!(t >= c_ws && t < c_ws + (int64_t)wl)) {
            const int64_t q = t / wl;
            c_ws = t - (t - q * wl);
            c_idx = (int)(q % S);
        }
        idx = c_idx;
        return c_ws;
    }

    template <class F> SF_HD void visit(int idx, F f) {
        if constexpr (MAXS == 1) { f(sec[0]); }
        else if constexpr (MAXS == 2) { if (idx == 0) f(sec[0]); else f(sec[1]); }
        else { f(sec[idx]); }
    }
    template <class F> SF_HD void visit_bor(int idx, F f) {
        if constexpr (MAXS == 1) { f(bor[0]); }
        else if constexpr (MAXS == 2) { if (idx == 0) f(bor[0]); else f(bor[1]); }
        else { f(bor[idx]); }
    }

    // ---- FutureBucketLeapArray (borrowArray) ----
    // getWindowValue(t) -> pass of the bucket containing t, or -1 when null (LeapArray.java:268-281)
    SF_HD int64_t borrow_value(int64_t t) {
        int idx;
        win_of(t, idx);
        int64_t v = -1;
        visit_bor(idx, [&](Borrow& b) { if (b.ws <= t && t < b.ws + wl) v = b.pass; });
        return v;
    }
    // currentWindow(t): returns idx, or -1 for a throwaway window
    SF_HD int borrow_current(int64_t t) {
        int idx;
        const int64_t ws = win_of(t, idx);
        int r = idx;
        visit_bor(idx, [&](Borrow& b) {
            if (b.ws == ws) return;
            if (ws > b.ws) { b.ws = ws; b.pass = 0; bdirty = 1; return; }   // FutureBucketLeapArray.resetWindowTo :41-46
            r = -1;
        });
        return r;
    }
    // OccupiableBucketLeapArray.currentWaiting (:67-76)
    SF_HD int64_t current_waiting(int64_t now) {
        borrow_current(now);
        int64_t w = 0;
        for (int i = 0; i < S; i++)
            visit_bor(i, [&](Borrow& b) { if (!(now >= b.ws)) w = wadd(w, b.pass); });   // Future deprecation :49-52
        return w;
    }
    SF_HD void add_waiting(int64_t t, int32_t c) {                       // :79-83
        int i = borrow_current(t);
        if (i < 0) return;                                               // throwaway window
        visit_bor(i, [&](Borrow& b) { b.pass = wadd(b.pass, c); });
        bdirty = 1;
    }

    // ---- OccupiableBucketLeapArray main window ----
    // currentWindow(t): returns idx or -1 (throwaway window, LeapArray.java:220-223)
    SF_HD int sec_current(int64_t t) {
        int idx;
        const int64_t ws = win_of(t, idx);
        int r = idx;
        bool reset = false;
        visit(idx, [&](Bucket& b) {
            if (b.ws == ws) return;
            if (ws > b.ws) { reset = true; return; }
            r = -1;
        });
        if (reset) {
            int64_t bp = borrow_value(ws);
            Bucket nb = fresh_bucket(ws, max_rt);
            if (bp >= 0) nb.pass = (int64_t)(int32_t)bp;                // resetWindowTo :52-64
            visit(idx, [&](Bucket& b) { b = nb; });
        }
        return r;
    }
    template <class F> SF_HD void sec_apply(int64_t t, F f) {
        int i = sec_current(t);
        if (i >= 0) visit(i, f);                                       // throwaway: the add is lost
    }
    SF_HD int64_t sec_sum_pass(int64_t now) {            // ArrayMetric.pass() :117-126
        sec_current(now);
        int64_t s = 0;
        for (int i = 0; i < S; i++)
            visit(i, [&](Bucket& b) { if (!(wsub(now, b.ws) > interval)) s = wadd(s, b.pass); });
        return s;
    }
    // ArrayMetric sums / extremes over the valid buckets, after the roll (ArrayMetric.java:68-162)
    template <class G> SF_HD int64_t sec_sum(int64_t now, G get) {
        sec_current(now);
        int64_t s = 0;
        for (int i = 0; i < S; i++)
            visit(i, [&](Bucket& b) { if (!(wsub(now, b.ws) > interval)) s = wadd(s, get(b)); });
        return s;
    }
    SF_HD int64_t sec_min_rt(int64_t now) {              // ArrayMetric.minRt :151-162
        sec_current(now);
        int64_t rt = max_rt;
        for (int i = 0; i < S; i++)
            visit(i, [&](Bucket& b) { if (!(wsub(now, b.ws) > interval) && b.min_rt < rt) rt = b.min_rt; });
        return rt > 1 ? rt : 1;
    }
    SF_HD int64_t sec_max_success(int64_t now) {         // ArrayMetric.maxSuccess :81-92
        sec_current(now);
        int64_t m = 0;
        for (int i = 0; i < S; i++)
            visit(i, [&](Bucket& b) { if (!(wsub(now, b.ws) > interval) && b.succ > m) m = b.succ; });
        return m > 1 ? m : 1;
    }
    SF_HD int64_t sec_window_pass(int64_t t) {            // ArrayMetric.getWindowPass :324-330
        int idx;
        win_of(t, idx);
        int64_t v = 0;
        visit(idx, [&](Bucket& b) { if (b.ws <= t && t < b.ws + wl) v = b.pass; });
        return v;
    }

    // ---- BucketLeapArray(60, 60000): minute window ----
    SF_HD void min_flush() {
        if (mdirty) { gmin[mi] = mb; mdirty = 0; }
    }
    // currentWindow(t): true when the cached bucket is the live one, false
    // for a throwaway window (older than the slot's bucket)
    // (the slot and window start of the last second looked up are cached:
    // events come in time order, so most lookups skip the 64-bit division)
    SF_HD bool min_current(int64_t t) {
        if (!(t >= m_ws && t < m_ws + 1000)) {
            const int idx = (int)((t / 1000) % MINUTE);
            m_ws = t - t % 1000;
            if (idx != mi) { min_flush(); mb = gmin[idx]; mi = idx; }
        }
        const int64_t ws = m_ws;
        if (mb.ws == ws) return true;
        if (ws > mb.ws) { mb = fresh_bucket(ws, max_rt); mdirty = 1; return true; }
        return false;
    }
    template <class F> SF_HD void min_apply(int64_t t, F f) {
        if (min_current(t)) { f(mb); mdirty = 1; }
    }
    // ArrayMetric.previousWindowPass (:279-286) -> getPreviousWindow (LeapArray.java:234-251).
    // The answer is fixed within a second: the previous second's bucket is a
    // slot this walk no longer writes (its own is the current second's), and
    // both deprecation tests give the same result at every time of the second
    // -- so it is read once per second, not at every WarmUp check.
    int64_t pp_sec = INT64_MIN, pp_val = 0;
    SF_HD int64_t min_previous_pass(int64_t now) {
        min_current(now);
        if (m_ws == pp_sec) return pp_val;
        int64_t tp = now - 1000;
        int idx = (int)((tp / 1000) % MINUTE);
        Bucket b = (idx == mi) ? mb : gmin[idx];
        int64_t v = b.pass;
        if (wsub(now, b.ws) > 60000) v = 0;              // isWindowDeprecated (TimeUtil now)
        if (b.ws + 1000 < tp) v = 0;
        pp_sec = m_ws; pp_val = v;
        return v;
    }

    // ---- StatisticNode ----
    SF_HD double pass_qps(int64_t now) { return (double)sec_sum_pass(now) / interval_sec; }   // :205-208
    SF_HD double previous_pass_qps(int64_t now) { return (double)min_previous_pass(now); }   // :179-181
    SF_HD void add_pass(int64_t now, int32_t c) {                                            // :253-256
        sec_apply(now, [&](Bucket& b) { b.pass = wadd(b.pass, c); });
        min_apply(now, [&](Bucket& m) { m.pass = wadd(m.pass, c); });
    }
    SF_HD void add_block(int64_t now, int32_t c) {                                           // :268-271
        sec_apply(now, [&](Bucket& b) { b.block = wadd(b.block, c); });
        min_apply(now, [&](Bucket& m) { m.block = wadd(m.block, c); });
    }
    SF_HD void add_exception(int64_t now, int32_t c) {                                       // :274-277
        sec_apply(now, [&](Bucket& b) { b.exc = wadd(b.exc, c); });
        min_apply(now, [&](Bucket& m) { m.exc = wadd(m.exc, c); });
    }
    SF_HD void add_rt_success(int64_t now, int64_t rt, int32_t c) {                          // :259-265
        auto f = [&](Bucket& b) {                                                            // MetricBucket.addRT :129-136
            b.succ = wadd(b.succ, c); b.rt = wadd(b.rt, rt); if (rt < b.min_rt) b.min_rt = rt;
        };
        sec_apply(now, f);
        min_apply(now, f);
    }
    SF_HD void add_occupied_pass(int64_t now, int32_t c) {                                   // :343-346
        min_apply(now, [&](Bucket& m) { m.occ = wadd(m.occ, c); });
        min_apply(now, [&](Bucket& m) { m.pass = wadd(m.pass, c); });
    }
    // tryOccupyNext :295-330 (IntervalProperty / SampleCountProperty statics)
    SF_HD int64_t try_occupy_next(int64_t now, int32_t c, double threshold, int32_t occupy_timeout) {
        double max_count = threshold * interval / 1000;
        int64_t current_borrow = current_waiting(now);
        if ((double)current_borrow >= max_count) return occupy_timeout;
        int32_t window_length = interval / S;
        int64_t earliest = now - now % window_length + window_length - interval;
        int idx = 0;
        int64_t current_pass = sec_sum_pass(now);
        while (earliest < now) {
            int64_t wait = (int64_t)(idx * window_length + window_length) - now % window_length;
            if (wait >= occupy_timeout) break;
            int64_t window_pass = sec_window_pass(earliest);
            if ((double)(current_pass + current_borrow + c - window_pass) <= max_count) return wait;
            earliest += window_length;
            current_pass -= window_pass;
            idx++;
        }
        return occupy_timeout;
    }
};

SF_HD DevRuleState fresh_rule_state() {     // AtomicLong(0), AtomicLong(0), AtomicLong(-1)
    DevRuleState s{}; s.stored_tokens = 0; s.last_filled = 0; s.latest_passed = -1; return s;
}

// ============================================================ controllers
// WarmUpController.syncToken :178-197 + coolDownTokens :217-232
SF_HD void warm_sync(const DevRule& r, DevRuleState& s, int64_t now, int64_t pass_qps) {
    int64_t current_time = now - now % 1000;
    if (current_time <= s.last_filled) return;
    int64_t old_value = s.stored_tokens, new_value = old_value;
    if (old_value < r.warning_token) {
        new_value = j_d2l((double)old_value + (double)(current_time - s.last_filled) * r.count / 1000);
    } else if (old_value > r.warning_token) {
        if (pass_qps < j_d2i(r.count) / r.cold_factor)
            new_value = j_d2l((double)old_value + (double)(current_time - s.last_filled) * r.count / 1000);
    }
    if (new_value > r.max_token) new_value = r.max_token;
    s.stored_tokens = wsub(new_value, pass_qps);
    if (s.stored_tokens < 0) s.stored_tokens = 0;
    s.last_filled = current_time;
}

// canPass: returns 1 pass / 0 block; *prio_wait set on PriorityWaitException.
template <int MAXS>
SF_HD int can_pass(const DevRule& r, DevRuleState& s, NodeWin<MAXS>& nd, int64_t now, int32_t acq,
                   bool prio, int32_t occupy_timeout, int64_t* wait, bool* prio_wait) {
    switch (r.kind) {
    case CT_DEFAULT: {                                             // DefaultController.java:50-89
        int32_t cur = r.grade == SF_GRADE_THREAD ? (int32_t)nd.threads : j_d2i(nd.pass_qps(now));
        if ((double)(int32_t)((uint32_t)cur + (uint32_t)acq) > r.count) {
            if (prio && r.grade == SF_GRADE_QPS) {
                int64_t w = nd.try_occupy_next(now, acq, r.count, occupy_timeout);
                if (w < occupy_timeout) {
                    nd.add_waiting(now + w, acq);
                    nd.add_occupied_pass(now, acq);
                    *wait = w; *prio_wait = true;
                    return 1;
                }
            }
            return 0;
        }
        return 1;
    }
    case CT_WARM_UP: {                                             // WarmUpController.java:147-175
        int64_t pass_qps = j_d2l(nd.pass_qps(now));
        int64_t previous_qps = j_d2l(nd.previous_pass_qps(now));
        warm_sync(r, s, now, previous_qps);
        int64_t rest = s.stored_tokens;
        if (rest >= r.warning_token) {
            int64_t above = rest - r.warning_token;
            double warning_qps = j_next_up(1.0 / ((double)above * r.slope + 1.0 / r.count));
            return (double)(pass_qps + acq) <= warning_qps;
        }
        return (double)(pass_qps + acq) <= r.count;
    }
    case CT_RATE_LIMITER:                                          // RateLimiterController.java:48-102
    case CT_WARM_UP_RATE_LIMITER: {                                // WarmUpRateLimiterController.java:43-87
        int64_t cost;
        if (r.kind == CT_RATE_LIMITER) {
            if (acq <= 0) return 1;
            if (r.count <= 0) return 0;
            cost = j_round(1.0 * acq / r.count * 1000);
        } else {
            int64_t previous_qps = j_d2l(nd.previous_pass_qps(now));
            warm_sync(r, s, now, previous_qps);
            int64_t rest = s.stored_tokens;
            if (rest >= r.warning_token) {
                int64_t above = rest - r.warning_token;
                double warming_qps = j_next_up(1.0 / ((double)above * r.slope + 1.0 / r.count));
                cost = j_round(1.0 * acq / warming_qps * 1000);
            } else {
                cost = j_round(1.0 * acq / r.count * 1000);
            }
        }
        int64_t expected = cost + s.latest_passed;
        if (expected <= now) { s.latest_passed = now; return 1; }
        int64_t w = cost + s.latest_passed - now;
        if (w > r.max_queue_ms) return 0;
        s.latest_passed += cost;
        w = s.latest_passed - now;
        if (w > r.max_queue_ms) { s.latest_passed -= cost; return 0; }
        if (w > 0) *wait = w;
        return 1;
    }
    }
    return 1;
}

// ============================================================ param table
// Open addressing with linear probing, at most PT_MAX_PROBE slots from a
// key's home: a key is never placed farther, so a lookup stops there too, and
// an insert that finds no free slot in reach is SF_ERR_CAPACITY (the table is
// too full for the configured param_capacity) instead of a scan of the table.
constexpr uint64_t PT_MAX_PROBE = 4096;
struct ParamTable {
    ParamSlot* slots; uint64_t mask; int32_t* err;
    // inserts counted (the host grows the table between batches, sf_engine.cpp
    // param_reserve): 256 counters 64 B apart, one per workgroup residue
    unsigned int* ins = nullptr;
    SF_HD static uint64_t hash(uint64_t hi, uint64_t lo) { return mix64(hi ^ mix64(lo + 0x9e3779b97f4a7c15ULL)); }
    // find slot of key; returns nullptr if absent
    SF_HD ParamSlot* find(uint64_t hi, uint64_t lo) const {
        uint64_t i = hash(hi, lo) & mask;
        const uint64_t reach = mask < PT_MAX_PROBE ? mask : PT_MAX_PROBE;
        for (uint64_t probe = 0; probe <= reach; probe++) {
#ifdef __HIP_DEVICE_COMPILE__
            uint64_t h = __hip_atomic_load(&slots[i].hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
            uint64_t h = slots[i].hi;
#endif
            if (h == 0) return nullptr;
            if (h == hi && slots[i].lo == lo) return &slots[i];
            i = (i + 1) & mask;
        }
        return nullptr;
    }
    // insert a key known to be absent (only the owning lane ever inserts a given key)
    SF_HD ParamSlot* insert(uint64_t hi, uint64_t lo) const {
        uint64_t i = hash(hi, lo) & mask;
        const uint64_t reach = mask < PT_MAX_PROBE ? mask : PT_MAX_PROBE;
        for (uint64_t probe = 0; probe <= reach; probe++) {
#ifdef __HIP_DEVICE_COMPILE__
            unsigned long long expected = 0;
            if (__hip_atomic_compare_exchange_strong((unsigned long long*)&slots[i].hi, &expected,
                    (unsigned long long)hi, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                slots[i].lo = lo; slots[i].a = 0; slots[i].b = 0;
                if (ins) atomicAdd(&ins[(blockIdx.x & 255u) * 16u], 1u);
                return &slots[i];
            }
#else
            if (slots[i].hi == 0) { slots[i].hi = hi; slots[i].lo = lo; slots[i].a = 0; slots[i].b = 0; return &slots[i]; }
#endif
            i = (i + 1) & mask;
        }
        *err = SF_ERR_CAPACITY;
        return nullptr;
    }
};
SF_HD uint64_t pkey_hi(uint32_t res, uint64_t kind, uint32_t idx, uint32_t tag) {
    return ((uint64_t)(res + 1u) << 32) | (kind << 24) | ((uint64_t)(idx & 0xffff) << 8) | (tag & 0xff);
}

// ParameterMetric.addThreadCount / decreaseThreadCount for one value (:184-239, :125-181).
// delta > 0: that many addThreadCount calls (heavy_param adds a value's passes
// of a 64-event group at once); delta < 0: one decreaseThreadCount.
SF_HD void pm_thread_add(const ParamTable& pt, uint32_t res, int idx, uint32_t tag, uint64_t bits, int delta) {
    if (tag == SF_TAG_NULL) return;
    uint64_t hi = pkey_hi(res, PK_THREAD, (uint32_t)idx, tag);
    ParamSlot* s = pt.find(hi, bits);
    if (delta > 0) {
        if (!s) { s = pt.insert(hi, bits); if (s) s->a = delta; }
        else s->a = (int32_t)((uint32_t)s->a + (uint32_t)delta);
    } else {
        if (!s) { pt.insert(hi, bits); return; }              // putIfAbsent(new AtomicInteger())
        int32_t cur = (int32_t)((uint32_t)s->a - 1u);
        s->a = cur <= 0 ? 0 : cur;                            // remove at <= 0 == reads as 0
    }
}
SF_HD int64_t pm_thread_get(const ParamTable& pt, uint32_t res, int idx, uint32_t tag, uint64_t bits) {
    ParamSlot* s = pt.find(pkey_hi(res, PK_THREAD, (uint32_t)idx, tag), bits);
    return s ? s->a : 0;
}

// ParamFlowChecker.passSingleValueCheck :114-137 (+ default :139-219, throttle :222-273).
// Returns 1 pass, 0 block, 2 for a null element of a collection: the checks
// before the first map access run, then the map throws NullPointerException,
// which passLocalCheck catches (:108-110): the value passes, its loop ends.
SF_HD int param_pass_single(const ParamTable& pt, uint32_t res, int rule_k, const DevParamRule& r,
                            const DevHotItem* items, int64_t now, int32_t acq, uint32_t tag, uint64_t bits,
                            int64_t* wait) {
    int64_t token_count = j_d2l(r.count);
    if (tag == SF_TAG_NULL) {                                // no hot item is null (ParamFlowRuleUtil.parseHotItems)
        if (r.grade == SF_GRADE_QPS) {
            if (token_count == 0) return 0;                  // :156-158 / :236-238
            if (r.behavior != SF_BEHAVIOR_RATE_LIMITER && acq > wadd(token_count, r.burst)) return 0;   // :160-163
        }
        return 2;                                            // putIfAbsent(null) / get(null)
    }
    bool hot = false; int32_t hot_count = 0;
    for (int k = 0; k < r.item_cnt; k++) {
        const DevHotItem& it = items[r.item_off + k];
        if (it.tag == tag && it.bits == bits) { hot = true; hot_count = it.count; break; }
    }
    if (r.grade == SF_GRADE_QPS) {
        if (hot) token_count = hot_count;
        if (token_count == 0) return 0;
        uint64_t hi = pkey_hi(res, PK_RULE, (uint32_t)rule_k, tag);
        if (r.behavior == SF_BEHAVIOR_RATE_LIMITER) {
            int64_t cost = j_round(1.0 * 1000 * acq * (double)r.duration_sec / (double)token_count);
            ParamSlot* s = pt.find(hi, bits);
            if (!s) { s = pt.insert(hi, bits); if (s) s->a = now; return 1; }
            int64_t last = s->a, expected = last + cost;
            if (expected <= now || expected - now < r.max_queue_ms) {
                s->a = now;
                int64_t w = expected - now;
                if (w > 0) { s->a = expected; *wait = w; }
                return 1;
            }
            return 0;
        }
        int64_t max_count = wadd(token_count, r.burst);
        if (acq > max_count) return 0;
        ParamSlot* s = pt.find(hi, bits);
        if (!s) {                                          // first sight :165-169
            s = pt.insert(hi, bits);
            if (s) { s->a = now; s->b = max_count - acq; }
            return 1;
        }
        int64_t pass_time = now - s->a;
        if (pass_time > wmul(r.duration_sec, 1000)) {      // refill :173-195
            int64_t rest = s->b;
            int64_t to_add = jdiv(wmul(pass_time, token_count), wmul(r.duration_sec, 1000));
            int64_t new_qps = wadd(to_add, rest) > max_count ? (max_count - acq) : wsub(wadd(rest, to_add), acq);
            if (new_qps < 0) return 0;
            s->b = new_qps; s->a = now;
            return 1;
        }
        if (s->b - acq >= 0) { s->b -= acq; return 1; }    // :196-215
        return 0;
    } else if (r.grade == SF_GRADE_THREAD) {
        int64_t thread_count = pm_thread_get(pt, res, r.param_idx, tag, bits);
        if (hot) return ++thread_count <= hot_count;
        return ++thread_count <= token_count;
    }
    return 1;
}

// One QPS-grade rule (default or throttle behaviour) over the occurrences of
// one value, in order, with the (rule, value) state in registers: exactly
// param_pass_single applied occurrence by occurrence (ParamFlowChecker
// :139-219 / :222-273), one table find before and one write after.  `live`
// (bit o: occurrence o reaches this rule) loses the occurrences it blocks;
// now_of / acq_of / wait_of index the occurrences.
template <class NOW, class ACQ, class WAIT>
SF_HD uint64_t param_run_rule(const ParamTable& pt, uint32_t res, int rule_k, const DevParamRule& r,
                              const DevHotItem* items, uint32_t tag, uint64_t bits, uint64_t live, NOW now_of,
                              ACQ acq_of, WAIT wait_of) {
    int64_t token_count = j_d2l(r.count);
    for (int k = 0; k < r.item_cnt; k++) {
        const DevHotItem& it = items[r.item_off + k];
        if (it.tag == tag && it.bits == bits) { token_count = it.count; break; }
    }
    const uint64_t hi = pkey_hi(res, PK_RULE, (uint32_t)rule_k, tag);
    ParamSlot* sl = pt.find(hi, bits);
    bool ex = sl != nullptr, dirty = false;
    int64_t A = ex ? sl->a : 0, B = ex ? sl->b : 0;
    const bool rl = r.behavior == SF_BEHAVIOR_RATE_LIMITER;
    const int64_t max_count = wadd(token_count, r.burst);
    for (uint64_t m = live; m; m &= m - 1) {
        const int o = __builtin_ctzll(m);
        const int64_t now = now_of(o);
        const int32_t acq = acq_of(o);
        bool ok;
        if (token_count == 0) ok = false;
        else if (rl) {
            const int64_t cost = j_round(1.0 * 1000 * acq * (double)r.duration_sec / (double)token_count);
            if (!ex) { ex = true; A = now; ok = true; }
            else {
                const int64_t expected = A + cost;
                ok = expected <= now || expected - now < r.max_queue_ms;
                if (ok) {
                    A = now;
                    const int64_t w = expected - now;
                    if (w > 0) { A = expected; wait_of(o, w); }
                }
            }
        } else if (acq > max_count) ok = false;
        else if (!ex) { ex = true; A = now; B = max_count - acq; ok = true; }
        else {
            const int64_t pass_time = now - A;
            if (pass_time > wmul(r.duration_sec, 1000)) {
                const int64_t to_add = jdiv(wmul(pass_time, token_count), wmul(r.duration_sec, 1000));
                const int64_t nq = wadd(to_add, B) > max_count ? (max_count - acq) : wsub(wadd(B, to_add), acq);
                ok = nq >= 0;
                if (ok) { B = nq; A = now; }
            } else {
                ok = B - acq >= 0;
                if (ok) B -= acq;
            }
        }
        if (ok) dirty = true;
        else live &= ~(1ull << o);
    }
    if (dirty) {
        if (!sl) sl = pt.insert(hi, bits);
        if (sl) { sl->a = A; sl->b = B; }
    }
    return live;
}

// ============================================================ the segment
struct SegIO {          // sorted-order batch arrays
    const int64_t* ts; const int32_t* cnt; const uint8_t* flags;
    const int64_t* eref; const int64_t* cts;
    uint32_t arg_slots; const uint8_t* nargs; const uint8_t* atag; const uint64_t* abits; uint32_t n;
    // collection / array arguments: a sorted arg with tag SF_TAG_COLLECTION has
    // abits = its index k into the batch's CSR (elements [aoff[k], aoff[k+1]))
    const uint32_t* aoff; const uint8_t* etag; const uint64_t* ebits;
    uint8_t* v_status; int32_t* v_wait; uint16_t* v_rule;     // sorted order (read back by exits)
    const uint32_t* perm;                                       // sorted -> submission index, or null
    uint8_t* o_status; int32_t* o_wait; uint16_t* o_rule;       // the caller's verdicts (submission order)
    // xflow walk (sf_xflow.h): resource id, origin and context of each event in
    // submission order (read through perm; origin / context may be null)
    const uint32_t* ev_res; const uint32_t* ev_origin; const uint32_t* ev_ctx;
    uint32_t shard_count;
};

// final verdict of sorted event j, straight into the caller's arrays
// (the status itself stays in sorted order, v_status: launch_scatter moves all
// of them to submission order in bucketed passes after the decide phase)
SF_HD void emit_verdict(const SegIO& io, uint32_t j, uint8_t status, int32_t wait, uint16_t rule) {
    (void)status;
    const bool w = io.o_wait && wait, r = io.o_rule && rule;
    if (!io.perm || !(w || r)) return;
    const uint32_t i = io.perm[j];
    if (w) io.o_wait[i] = wait;                          // (cleared before the decide phase)
    if (r) io.o_rule[i] = rule;
}

// ParamFlowChecker.passLocalCheck (:84-112): one value, or every element of a
// collection / array in order (the tokens of the elements before a failing one
// stay consumed).  Waits of throttled elements add up (each sleeps).
SF_HD int param_pass_value(const ParamTable& pt, uint32_t res, int rule_k, const DevParamRule& r,
                           const DevHotItem* items, int64_t now, int32_t acq, uint32_t tag, uint64_t bits,
                           const SegIO& io, int64_t* wait) {
    if (tag != SF_TAG_COLLECTION) return param_pass_single(pt, res, rule_k, r, items, now, acq, tag, bits, wait) != 0;
    for (uint32_t e = io.aoff[bits], e1 = io.aoff[bits + 1]; e < e1; e++) {
        int64_t w = 0;
        const int ok = param_pass_single(pt, res, rule_k, r, items, now, acq, io.etag[e], io.ebits[e], &w);
        if (ok == 0) return 0;
        if (ok == 2) return 1;
        if (w > 0) *wait += w;
    }
    return 1;
}

// ParameterMetric.addThreadCount / decreaseThreadCount (:125-239) over the
// event's args with a thread map (pm_init): a null arg is skipped, a
// collection counts each element; a null element throws, which ends the whole
// callback (the outer try around every index).
SF_HD void pm_thread_event(const ParamTable& pt, uint32_t res, uint8_t pm_init, const SegIO& io, uint32_t j,
                           uint32_t na, int delta) {
    for (uint32_t a = 0; a < na && a < 8; a++) {
        if (!((pm_init >> a) & 1)) continue;
        const uint32_t tg = io.atag[(size_t)a * io.n + j];
        const uint64_t bt = io.abits[(size_t)a * io.n + j];
        if (tg != SF_TAG_COLLECTION) { pm_thread_add(pt, res, (int)a, tg, bt, delta); continue; }
        for (uint32_t e = io.aoff[bt], e1 = io.aoff[bt + 1]; e < e1; e++) {
            if (io.etag[e] == SF_TAG_NULL) return;
            pm_thread_add(pt, res, (int)a, io.etag[e], io.ebits[e], delta);
        }
    }
}

// A lane's resource row into / out of a NodeWin: second-window buckets,
// borrow buckets (only once a prioritized entry has been submitted: before
// that every borrow bucket is the initial empty one, st.prio_seen), thread
// count, minute row (buckets loaded on demand)
template <int MAXS>
SF_HD void nw_load_row(NodeWin<MAXS>& nd, const DevState& st, uint32_t res) {
    nd.S = st.S; nd.wl = st.wl; nd.interval = st.interval; nd.max_rt = st.max_rt;
    nd.interval_sec = st.interval / 1000.0;
    const bool bor = *st.prio_seen != 0;
    for (int i = 0; i < MAXS; i++) {
        if (i < st.S) nd.sec[i] = st.second[(size_t)res * st.S + i];
        else nd.sec[i] = fresh_bucket(WS_NONE, st.max_rt);
        if (i < st.S && bor) nd.bor[i] = st.borrow[(size_t)res * st.S + i];
        else { nd.bor[i].ws = WS_NONE; nd.bor[i].pass = 0; }
    }
    nd.threads = st.threads[res];
    nd.gmin = st.minute + (size_t)res * MINUTE;
    nd.mi = -1; nd.mdirty = 0;
    nd.mb = fresh_bucket(WS_NONE, st.max_rt);
}
template <int MAXS>
SF_HD void nw_store_row(NodeWin<MAXS>& nd, const DevState& st, uint32_t res) {
    for (int i = 0; i < MAXS; i++)
        if (i < st.S) {
            st.second[(size_t)res * st.S + i] = nd.sec[i];
            if (nd.bdirty) st.borrow[(size_t)res * st.S + i] = nd.bor[i];
        }
    nd.min_flush();
    st.threads[res] = nd.threads;
}

SF_HD bool v_blocked(uint8_t v) {
    return v == SF_V_BLOCK_FLOW || v == SF_V_BLOCK_PARAM || v == SF_V_BLOCK_SYSTEM || v == SF_V_BLOCK_DEGRADE ||
           v == SF_V_BLOCK_OTHER;
}
// verdict of an entry carrying EVF_SYSBLK: a planned SystemBlockException
// (reason 0..4 in rule_idx) or an SF_EV_BLOCKED entry (SYSR_OTHER)
SF_HD uint8_t sysblk_status(uint8_t fl) {
    return ((fl >> EVF_SYSREASON_SHIFT) & 7) == SYSR_OTHER ? (uint8_t)SF_V_BLOCK_OTHER : (uint8_t)SF_V_BLOCK_SYSTEM;
}
SF_HD int sysblk_rule(uint8_t fl) {
    const int r = (fl >> EVF_SYSREASON_SHIFT) & 7;
    return r == SYSR_OTHER ? 0 : r;
}

// the resource's circuit breakers [*b0, *b1) (DegradeRuleManager's list order)
SF_HD void breakers_of(const DevState& st, uint32_t res, uint32_t* b0, uint32_t* b1) {
    *b0 = *b1 = 0;
    if (!st.dg_rr_of) return;
    const uint32_t k = st.dg_rr_of[res];
    if (k < st.dg_n) { *b0 = st.dg_off[k]; *b1 = st.dg_off[k + 1]; }
}

// SystemRules: a SystemBlockException of an IN entry is decided by the
// planner (sf_system.h) and arrives as EVF_SYSBLK on the event.
#ifndef SF_EV_CH
#define SF_EV_CH 8
#endif
// PF false: the engine has no ParamFlow and no degrade rules loaded (the host
// knows it per launch), so that code is compiled out of the lane (fewer live
// registers, more wavefronts per SIMD)
template <int MAXS, uint32_t EV_CH = SF_EV_CH, bool PF = true>
SF_HD void decide_segment(const DevState& st, const SegIO& io, uint32_t res, uint32_t lo, uint32_t hi) {
    NodeWin<MAXS> nd;
    nw_load_row(nd, st, res);
    const RDesc rd = st.rdesc[res];
    const uint32_t r0 = rd.r0;
    const int nrules = rd.nrules;
    // controller state of the first rule stays in registers; further rules of
    // the resource (rare) are read-modified-written in place in HBM, which
    // is exact because this lane owns the resource (a DefaultController keeps none)
    DevRuleState rs0 = (rd.flags & RD_STATE0) ? st.rstate[r0] : fresh_rule_state();
    uint32_t p0 = 0, p1 = 0;
    if (PF && (rd.flags & RD_PRULE)) { p0 = st.prule_off[res]; p1 = st.prule_off[res + 1]; }
    const int nprules = (int)(p1 - p0);
    uint8_t pm_init = nprules ? st.pm_init[res] : 0;
    bool pm_exists = pm_init != 0;
    ParamTable pt{st.ptab, st.pcap_mask, st.err, st.pins};
    uint32_t cb0 = 0, cb1 = 0;                                 // DegradeSlot breakers (this lane owns them)
    if (PF && (rd.flags & RD_BRK)) breakers_of(st, res, &cb0, &cb1);

    // The lane's events are read EV_CH at a time with all loads in flight together
    // (each cache line of the sorted arrays is then fetched once, not once per
    // event after the lines of the other lanes' segments evicted it), and picked
    // out of registers by unrolled selects (no dynamic register indexing).
    int64_t t_[EV_CH]; int32_t c_[EV_CH]; uint8_t f_[EV_CH];
    // statuses out eight at a time (decide_qps_segment)
    uint32_t sblk = lo & ~7u;
    uint64_t sbuf = 0;
    auto st_flush = [&](uint32_t jend) {
        if (sblk >= lo && jend == sblk + 8) { __builtin_memcpy(io.v_status + sblk, &sbuf, 8); return; }
        for (uint32_t q = sblk > lo ? sblk : lo; q < jend; q++) io.v_status[q] = (uint8_t)(sbuf >> (8 * (q - sblk)));
    };
    auto st_put = [&](uint32_t j, uint8_t status) {
        sbuf |= (uint64_t)status << (8 * (j - sblk));
        if ((j & 7u) == 7u) { st_flush(j + 1); sblk = j + 1; sbuf = 0; }
    };
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t k_ = (j - lo) % EV_CH;
        if (k_ == 0) {
#pragma unroll
            for (uint32_t q = 0; q < EV_CH; q++) {
                const uint32_t jj = j + q < hi ? j + q : hi - 1;
                t_[q] = io.ts[jj]; c_[q] = io.cnt[jj]; f_[q] = io.flags[jj];
            }
        }
        int64_t now = t_[0]; int32_t c = c_[0]; uint8_t fl = f_[0];
#pragma unroll
        for (uint32_t q = 1; q < EV_CH; q++)
            if (k_ == q) { now = t_[q]; c = c_[q]; fl = f_[q]; }
        const uint32_t na = io.arg_slots ? (io.nargs ? io.nargs[j] : io.arg_slots) : 0;
        uint8_t status; int64_t wait = 0; int rule_idx = 0;

        if (fl & SF_EV_EXIT) {                                  // StatisticSlot.exit :134-165
            int64_t ref = io.eref ? io.eref[j] : -1;
            bool blocked; int64_t create_ts;
            if (ref >= 0) {
                if ((ref < (int64_t)lo || ref >= (int64_t)j || (io.flags[ref] & SF_EV_EXIT))) {   // entry of another resource / order
                    *st.err = SF_ERR_INVALID;
#if !defined(__HIP_DEVICE_COMPILE__) && defined(SF_HOST_DEBUG)
                    printf("bad ref j=%u ref=%lld lo=%u flags=%d\n", j, (long long)ref, lo, ref>=0? io.flags[ref]:-1);
#endif
                    ref = j;   // treat as this exit's own slot: reads as not blocked below
                }
                const uint8_t est = ref >= (int64_t)sblk ? (uint8_t)(sbuf >> (8 * (uint32_t)(ref - sblk))) : io.v_status[ref];
                blocked = ref == (int64_t)j ? true : v_blocked(est);
                create_ts = io.ts[ref];
            }
            else { blocked = ref == EREF_DEAD; create_ts = io.cts ? io.cts[j] : now; }
            if (!blocked) {
                int64_t rt = now - create_ts;
                nd.add_rt_success(now, rt, c);                  // recordCompleteFor :167-178
                nd.threads--;
                if (fl & SF_EV_ERROR) nd.add_exception(now, c);
                if (pm_exists) pm_thread_event(pt, res, pm_init, io, j, na, -1);   // ParamFlowStatisticExitCallback
                for (uint32_t cb = cb0; cb < cb1; cb++) {        // DegradeSlot.exit :72-91 (after StatisticSlot.exit)
                    sf_breaker_state bs = st.dg_state[cb];
                    dg_complete(bs, st.dg_rules[cb], now, rt, (fl & SF_EV_ERROR) != 0);
                    st.dg_state[cb] = bs;
                }
                status = SF_V_EXIT;
            } else {
                status = SF_V_EXIT_IGNORED;
            }
            st_put(j, status);
            emit_verdict(io, j, status, 0, 0);
            continue;
        }

        bool blocked = false, prio_wait = false;
        status = SF_V_PASS;
        if (fl & EVF_SYSBLK) {        // SF_EV_BLOCKED (AuthoritySlot) or a planned SystemBlockException (sf_system.h)
            blocked = true; status = sysblk_status(fl); rule_idx = sysblk_rule(fl);
        }
        // ParamFlowSlot.checkFlow :82-103
        if (!blocked && nprules) {
            pm_exists = true;
            for (int k = 0; k < nprules && !blocked; k++) {
                DevParamRule& pr = st.prules[p0 + k];
                if (pr.param_idx < 0) {                          // applyRealParamIdx :56-66
                    if (-pr.param_idx <= (int)na) pr.param_idx = (int)na + pr.param_idx;
                    else pr.param_idx = -pr.param_idx;
                }
                if (pr.param_idx < 8) pm_init |= (uint8_t)(1u << pr.param_idx);   // initParamMetricsFor
                if ((int)na <= pr.param_idx) continue;             // passCheck :53-56
                uint32_t tg = io.atag[(size_t)pr.param_idx * io.n + j];
                uint64_t bt = io.abits[(size_t)pr.param_idx * io.n + j];
                if (tg == SF_TAG_NULL) continue;
                int64_t w = 0;
                if (!param_pass_value(pt, res, k, pr, st.items, now, c, tg, bt, io, &w)) {
                    blocked = true; status = SF_V_BLOCK_PARAM; rule_idx = k;
                } else if (w > 0) {
                    wait += w;
                }
            }
        }
        // FlowSlot -> FlowRuleChecker.checkFlow :44-59
        if (!blocked) {
            for (int k = 0; k < nrules; k++) {
                int64_t w = 0; bool pw = false;
                int ok = can_pass<MAXS>(st.rules[r0 + k], k == 0 ? rs0 : st.rstate[r0 + k], nd, now, c,
                                        (fl & SF_EV_PRIO) != 0, st.occupy_timeout, &w, &pw);
                if (pw) { prio_wait = true; wait += w; rule_idx = k; break; }
                if (!ok) { blocked = true; status = SF_V_BLOCK_FLOW; rule_idx = k; break; }
                wait += w;
            }
        }
        // DegradeSlot.entry (DegradeSlot.java:42-61), last in the chain; a
        // PriorityWaitException from FlowSlot never reaches it
        if (!blocked && !prio_wait && cb1 > cb0) {
            const int k = dg_entry_check(st.dg_state, cb0, cb1, now);
            if (k >= 0) { blocked = true; status = SF_V_BLOCK_DEGRADE; rule_idx = k; }
        }
        // StatisticSlot.entry accounting :64-123
        if (blocked) {
            nd.add_block(now, c);
        } else {
            nd.threads++;
            if (prio_wait) status = SF_V_PRIORITY_WAIT;
            else {
                nd.add_pass(now, c); status = wait > 0 ? SF_V_PASS_WAIT : SF_V_PASS;
            }
            if (pm_exists) pm_thread_event(pt, res, pm_init, io, j, na, +1);
        }
        st_put(j, status);                                   // (exits of this segment read it back)
        emit_verdict(io, j, status, (int32_t)wait, (uint16_t)rule_idx);
    }
    if (hi > sblk) st_flush(hi);

    // write back (borrow and the first rule's controller state only when they can have changed)
    nw_store_row(nd, st, res);
    if (rd.flags & RD_STATE0) st.rstate[r0] = rs0;           // DefaultController keeps no state
    if (nprules) st.pm_init[res] = pm_init;
}

// The lean lane walk of a segment whose resource has exactly one rule, a
// QPS-grade DefaultController, and nothing else in the chain (no ParamFlow
// rules, no breakers) and whose entries are neither prioritized nor blocked by
// a planned SystemBlockException (k_classify routes on the segment flags).
// This is exactly decide_segment's path for such a segment
// (DefaultController.canPass :50-72, StatisticSlot entry / exit accounting
// :55-178) with a fraction of its live registers (no controller state, params,
// breakers, occupy path), so more wavefronts fit per SIMD.
template <int MAXS>
SF_HD void decide_qps_segment(const DevState& st, const SegIO& io, uint32_t res, uint32_t lo, uint32_t hi) {
    NodeWin<MAXS> nd;
    nw_load_row(nd, st, res);
    const double count = st.rdesc[res].count0;
    // events read QC at a time with every load in flight together (time,
    // acquireCount and flags), picked out of registers by
    // unrolled selects: a lane walking a long segment then waits for memory
    // once per chunk instead of once per event
#ifndef SF_QPS_CH
#define SF_QPS_CH 16
#endif
    constexpr uint32_t QC = SF_QPS_CH;
    static_assert(QC % 4 == 0, "flags are packed four to a register");
    // times as 32-bit offsets from the chunk's first (a chunk spanning 2^31 ms
    // or more falls back to per-event loads), flags four to a register
    int64_t t0_ = 0; uint32_t td_[QC]; int32_t c_[QC]; uint32_t f4_[QC / 4];
    bool wide_ = false;
    uint32_t sblk = lo & ~7u;                                  // 8-aligned block of the buffered statuses
    uint64_t sbuf = 0;
    auto st_flush = [&](uint32_t jend) {                       // statuses [max(lo, sblk), jend)
        if (sblk >= lo && jend == sblk + 8) { __builtin_memcpy(io.v_status + sblk, &sbuf, 8); return; }
        for (uint32_t q = sblk > lo ? sblk : lo; q < jend; q++) io.v_status[q] = (uint8_t)(sbuf >> (8 * (q - sblk)));
    };
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t k_ = (j - lo) % QC;
        if (k_ == 0) {
            int64_t tt[QC]; uint8_t ff[QC];
#pragma unroll
            for (uint32_t q = 0; q < QC; q++) {
                const uint32_t jj = j + q < hi ? j + q : hi - 1;
                tt[q] = io.ts[jj]; c_[q] = io.cnt[jj]; ff[q] = io.flags[jj];
            }
            t0_ = tt[0];
            wide_ = tt[QC - 1] - t0_ >= (int64_t)0x7fffffff;
#pragma unroll
            for (uint32_t q = 0; q < QC; q++) td_[q] = (uint32_t)(tt[q] - t0_);
#pragma unroll
            for (uint32_t q = 0; q < QC / 4; q++)
                f4_[q] = (uint32_t)ff[4 * q] | ((uint32_t)ff[4 * q + 1] << 8) | ((uint32_t)ff[4 * q + 2] << 16) |
                         ((uint32_t)ff[4 * q + 3] << 24);
        }
        uint32_t td = td_[0]; int32_t c = c_[0]; uint32_t fw = f4_[0];
#pragma unroll
        for (uint32_t q = 1; q < QC; q++)
            if (k_ == q) { td = td_[q]; c = c_[q]; }
#pragma unroll
        for (uint32_t q = 1; q < QC / 4; q++)
            if (k_ / 4 == q) fw = f4_[q];
        const uint8_t fl = (uint8_t)(fw >> (8 * (k_ % 4)));
        const int64_t now = wide_ ? io.ts[j] : t0_ + (int64_t)td;
        uint8_t status;
        if (fl & SF_EV_EXIT) {                                  // StatisticSlot.exit :134-165
            int64_t ref = io.eref ? io.eref[j] : -1;
            bool blocked; int64_t create_ts;
            if (ref >= 0) {
                if (ref < (int64_t)lo || ref >= (int64_t)j || (io.flags[ref] & SF_EV_EXIT)) { *st.err = SF_ERR_INVALID; ref = j; }
                // the entry's status: still in the store buffer, or stored
                const uint8_t est = ref >= (int64_t)sblk ? (uint8_t)(sbuf >> (8 * (uint32_t)(ref - sblk))) : io.v_status[ref];
                blocked = ref == (int64_t)j ? true : v_blocked(est);
                create_ts = io.ts[ref];
            } else {
                blocked = ref == EREF_DEAD; create_ts = io.cts ? io.cts[j] : now;
            }
            if (!blocked) {
                nd.add_rt_success(now, now - create_ts, c);
                nd.threads--;
                if (fl & SF_EV_ERROR) nd.add_exception(now, c);
                status = SF_V_EXIT;
            } else {
                status = SF_V_EXIT_IGNORED;
            }
        } else {
            const int32_t cur = j_d2i(nd.pass_qps(now));
            if ((double)(int32_t)((uint32_t)cur + (uint32_t)c) > count) {
                nd.add_block(now, c); status = SF_V_BLOCK_FLOW;
            } else {
                nd.threads++; nd.add_pass(now, c); status = SF_V_PASS;
            }
        }
        // statuses go out eight at a time (one aligned 8-byte store per block of
        // the segment's own; byte stores at its ends): a byte store per event
        // costs a partial-line write each
        sbuf |= (uint64_t)status << (8 * (j - sblk));
        if ((j & 7u) == 7u) { st_flush(j + 1); sblk = j + 1; sbuf = 0; }
    }
    if (hi > sblk) st_flush(hi);
    nw_store_row(nd, st, res);
}

// k_classify: the lean walk applies to this segment (SM_LIGHTQ)
constexpr uint32_t SEGF_PRIO_ = 1u, SEGF_SYS_ = 4u;   // = SEGF_PRIO / SEGF_SYS (sf_heavy.h)
SF_HD bool qps_lean(const DevState& st, uint32_t res, uint32_t segflags) {
    if (segflags & (SEGF_PRIO_ | SEGF_SYS_)) return false;
    return (st.rdesc[res].flags & RD_LEAN) != 0;
}

// the resource's RDesc from the rule tables (k_rdesc; the host simulator's refresh)
SF_HD RDesc make_rdesc(const DevState& st, uint32_t res) {
    RDesc d{};
    const uint32_t r0 = st.rule_off[res], n = st.rule_off[res + 1] - r0;
    d.r0 = r0;
    d.nrules = (uint8_t)n;
    const bool prule = st.prule_off[res + 1] != st.prule_off[res];
    const bool brk = st.dg_rr_of && st.dg_rr_of[res] < st.dg_n;
    d.flags = (uint8_t)((prule ? RD_PRULE : 0) | (brk ? RD_BRK : 0));
    if (n) {
        const DevRule& r = st.rules[r0];
        d.count0 = r.count;
        if (r.kind != CT_DEFAULT) d.flags |= RD_STATE0;
        if (n == 1 && !prule && !brk && r.kind == CT_DEFAULT && r.grade == SF_GRADE_QPS) d.flags |= RD_LEAN;
    }
    return d;
}

// ============================================================ rule tables (host side)
// FlowRuleUtil.isValidRule (FlowRuleUtil.java:170-185) + checkStrategyField (:236-241)
// + checkControlBehaviorField (:243-254); a cluster rule's ClusterFlowConfig is
// taken to be valid (checkClusterField :210-230: the ABI does not carry it)
inline bool valid_flow_rule(const sf_flow_rule& r) {
    if (!(r.count >= 0) || r.grade < 0 || r.strategy < 0 || r.control_behavior < 0) return false;
    if (r.grade == SF_GRADE_QPS) {
        if ((r.strategy == SF_STRATEGY_RELATE || r.strategy == SF_STRATEGY_CHAIN) && r.ref_resource == SF_REF_NONE)
            return false;
        switch (r.control_behavior) {
        case SF_BEHAVIOR_WARM_UP: return r.warm_up_period_sec > 0;
        case SF_BEHAVIOR_RATE_LIMITER: return r.max_queueing_time_ms > 0;
        case SF_BEHAVIOR_WARM_UP_RATE_LIMITER: return r.warm_up_period_sec > 0 && r.max_queueing_time_ms > 0;
        default: return true;
        }
    }
    return r.grade == SF_GRADE_THREAD;
}
// FlowRuleUtil.generateRater (:132-152) + WarmUpController.construct (WarmUpController.java:113-139)
// ref_local: RELATE's referenced resource as a local id (XNONE: none); CHAIN keeps the context id
inline DevRule make_dev_rule(const sf_flow_rule& r, int cold_factor, int host_index, uint32_t ref_local = XNONE) {
    DevRule d{};
    d.grade = (uint8_t)r.grade; d.count = r.count; d.max_queue_ms = r.max_queueing_time_ms;
    d.cold_factor = cold_factor; d.host_index = host_index;
    d.strategy = (uint8_t)(r.strategy <= SF_STRATEGY_CHAIN ? r.strategy : 3);   // 3+: no reference node
    d.limit_app = r.limit_app;
    d.ref = r.strategy == SF_STRATEGY_RELATE ? ref_local : r.ref_resource;
    d.always_pass = (r.cluster_mode && !r.cluster_fallback) ? 1 : 0;
    d.kind = CT_DEFAULT;
    if (r.grade == SF_GRADE_QPS) {
        if (r.control_behavior == SF_BEHAVIOR_WARM_UP) d.kind = CT_WARM_UP;
        else if (r.control_behavior == SF_BEHAVIOR_RATE_LIMITER) d.kind = CT_RATE_LIMITER;
        else if (r.control_behavior == SF_BEHAVIOR_WARM_UP_RATE_LIMITER) d.kind = CT_WARM_UP_RATE_LIMITER;
    }
    if (d.kind == CT_WARM_UP || d.kind == CT_WARM_UP_RATE_LIMITER) {
        int period = r.warm_up_period_sec;
        d.warning_token = j_d2i(period * r.count) / (cold_factor - 1);
        d.max_token = d.warning_token + j_d2i(2 * period * r.count / (1.0 + cold_factor));
        d.slope = (cold_factor - 1.0) / r.count / (double)(d.max_token - d.warning_token);
    }
    return d;
}
// DegradeRuleManager.isValidRule (DegradeRuleManager.java:183-204)
inline bool dg_valid(const sf_degrade_rule& r) {
    if (!(r.count >= 0) || r.time_window_s <= 0) return false;
    if (r.min_request_amount <= 0 || r.stat_interval_ms <= 0) return false;
    switch (r.grade) {
        case SF_DEGRADE_GRADE_RT: return r.slow_ratio_threshold >= 0 && r.slow_ratio_threshold <= 1;
        case SF_DEGRADE_GRADE_EXCEPTION_RATIO: return r.count <= 1;
        case SF_DEGRADE_GRADE_EXCEPTION_COUNT: return true;
        default: return false;
    }
}
// a breaker's constants (ResponseTimeCircuitBreaker.java:48-56, ExceptionCircuitBreaker.java:47-56,
// AbstractCircuitBreaker.java:47-55)
inline DevBreakerRule make_dev_breaker_rule(const sf_degrade_rule& r) {
    DevBreakerRule d{};
    d.grade = r.grade;
    d.min_req = r.min_request_amount;
    d.max_rt = j_round(r.count);                             // Math.round (ResponseTimeCircuitBreaker.java:52)
    d.thr = r.grade == SF_DEGRADE_GRADE_RT ? r.slow_ratio_threshold : r.count;
    d.recovery = (int64_t)r.time_window_s * 1000;
    d.interval = r.stat_interval_ms;
    return d;
}
inline DevParamRule make_dev_param_rule(const sf_param_rule& r, int host_index) {
    DevParamRule d{};
    d.grade = r.grade; d.param_idx = r.param_idx; d.behavior = r.control_behavior;
    d.max_queue_ms = r.max_queueing_time_ms; d.count = r.count; d.duration_sec = r.duration_in_sec;
    d.burst = r.burst_count; d.item_off = (int32_t)r.item_offset; d.item_cnt = (int32_t)r.item_count;
    d.host_index = host_index;
    return d;
}

}  // namespace sf
