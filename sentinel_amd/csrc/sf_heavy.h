// sf_heavy.h — decision algorithms for heavy resource segments (product code).
//
// A Zipf(1.1) batch puts ~12 % of all events on one resource; replaying such
// a segment event by event in one lane is a latency-bound serial chain.  For
// the common single-rule classes the reference semantics admit a description
// whose size is proportional to the number of WINDOWS and PASSES, not events:
//
//  QPS DefaultController / WarmUpController (no prioritized entries):
//    inside one bucket window (LeapArray hw of length interval/sampleCount)
//    the threshold and passQps of the other buckets are constant, so the pass
//    set is the greedy prefix of the entries' acquireCount prefix sums plus at
//    most a few tail passes (DefaultController.java:50-89,
//    WarmUpController.java:147-175; WarmUp syncToken runs once per second).
//  RateLimiterController: an entry passes iff t >= latestPassedTime +
//    cost(c) - maxQueueingTimeMs (RateLimiterController.java:48-102), so the
//    next pass is found by a search over the time-sorted segment.
//
// One wavefront (a "team", QPS / WarmUp) or workgroup (k_heavy_stream: RL,
// THREAD) runs the decision chain for one segment and sets one PASS BIT per
// passed entry (RateLimiter waits go straight into v_wait).  Device-wide
// kernels then write every verdict from the bits, reduce the per-window
// counters, and apply them to the LeapArray state in time order (bucket reset
// semantics of LeapArray.currentWindow).
#pragma once
#include "sf_decide.h"

namespace sf {

// segment modes (seg_mode[s])
enum : uint8_t { SM_LIGHT = 0, SM_GENERIC = 1, SM_QPS = 2, SM_WARM = 3, SM_RL = 4, SM_NORULE = 5, SM_THREAD = 6,
                 SM_PARAM = 7, SM_XFLOW = 8,
                 SM_LIGHTQ = 9 };   // short light segment of a lone QPS DefaultController rule (decide_qps_segment)
constexpr uint32_t SEGF_PRIO = SEGF_PRIO_, SEGF_NONPOS = 2u, SEGF_SYS = SEGF_SYS_, SEGF_EXIT = 8u, SEGF_COLL = 16u;
constexpr uint32_t SEGF_ORIGIN = 32u;   // (tests/hostsim's routing model only: an event carries an origin)
constexpr uint32_t SEGF_BIGC = 64u;     // a checked entry with acquireCount > THR_CBIG (k_thr_heads; THREAD run mode off)

struct Acc {            // per (segment, window) counter deltas
    unsigned long long pass, block, succ, rt, exc, n_pass, n_exit, n_touch;
    long long min_rt;
};

static_assert(sizeof(Acc) == ACC_BYTES, "Acc layout must match the engine allocation");

// Segment routing (k_classify): the window/skip algorithms cover single-rule
// QPS / WarmUp / RateLimiter resources (and resources without rules) when no
// entry is prioritized or has acquireCount <= 0 and IntervalProperty is 1 s.
SF_HD uint8_t heavy_mode(const DevState& st, uint32_t res, uint32_t segflags, int64_t first_ts) {
    // circuit breakers (DegradeSlot) feed back into the node's pass / block
    // counts event by event: the generic lane walk (decide_segment) only
    if (st.dg_rr_of && st.dg_rr_of[res] < st.dg_n) return SM_GENERIC;
    // a borrowed (prioritized) pass waiting for a window of this batch would be
    // copied into that window when it is created: keep such resources exact
    // on the generic path (OccupiableBucketLeapArray.java:40-64)
    const int64_t ws_first = first_ts - first_ts % st.wl;
    for (int i = 0; i < st.S; i++)
        if (st.borrow[(size_t)res * st.S + i].ws >= ws_first) return SM_GENERIC;
    const uint32_t nr = st.rule_off[res + 1] - st.rule_off[res];
    const uint32_t np = st.prule_off[res + 1] - st.prule_off[res];
    // (EVF_SYSBLK entries, SEGF_SYS, are blocks no controller sees: the window
    // paths skip them as candidates and k_heavy_fill counts them as blocks)
    if ((segflags & SEGF_NONPOS) || st.interval != 1000) return SM_GENERIC;
    if (np != 0) {
        // ParamFlow-only resources whose decisions are independent per parameter
        // value (QPS-grade rules on one argument index, no exits, no collection
        // arguments): k_heavy_decide's wavefront path by value (heavy_param)
        if (st.rule_off[res + 1] != st.rule_off[res] || (segflags & (SEGF_EXIT | SEGF_COLL))) return SM_GENERIC;
        const uint32_t p0 = st.prule_off[res];
        const int32_t idx = st.prules[p0].param_idx;
        if (idx < 0 || idx >= 8 || (st.pm_init[res] & ~(1u << idx))) return SM_GENERIC;
        for (uint32_t k = p0; k < p0 + np; k++) {
            const DevParamRule& pr = st.prules[k];
            if (pr.param_idx != idx || pr.grade != SF_GRADE_QPS ||
                (pr.behavior != SF_BEHAVIOR_DEFAULT && pr.behavior != SF_BEHAVIOR_RATE_LIMITER)) return SM_GENERIC;
        }
        return SM_PARAM;
    }
    if (nr == 0) return SM_NORULE;
    if (nr != 1 || (segflags & SEGF_PRIO)) return SM_GENERIC;
    const DevRule& r = st.rules[st.rule_off[res]];
    if (r.kind == CT_DEFAULT && r.grade == SF_GRADE_QPS) return SM_QPS;
    if (r.kind == CT_WARM_UP) return SM_WARM;
    if (r.kind == CT_RATE_LIMITER) return SM_RL;
    if (r.kind == CT_DEFAULT && r.grade == SF_GRADE_THREAD && r.count < 2147483647.0) return SM_THREAD;
    return SM_GENERIC;
}

struct HeavyCtx {
    const uint32_t* seg_start; const uint32_t* seg_res; const uint8_t* seg_mode;
    const uint32_t* heavy_list; const uint32_t* n_heavy;  // n_heavy[0] front count, n_heavy[3] back count
    uint32_t seg_cap;
    const int64_t* pcg;                // inclusive prefix of entry acquireCount over the sorted batch
    Acc* acc_hw; Acc* acc_sec; const uint32_t* acc_hw_base; const uint32_t* acc_sec_base;
    const int64_t* seg_hw0; const int64_t* seg_sec0;    // first window index of the segment
    uint64_t* hticks;                                   // per heavy-list entry, or null
    unsigned long long* passbits;                       // [n/64+2] bit j: entry j passed (QPS/WarmUp/RL/THREAD)
    const uint32_t* exit_of;                            // [n] sorted index of an entry's exit (or ~0)
    unsigned long long* lxfar;                          // [n/64+2] live exits beyond the LDS ring (SM_THREAD)
    const uint2* thr_rec;                               // [n] SM_THREAD window-walk event records (k_thr_rec)
    // THREAD run mode (sf_stream.h thr_runs_segment; k_thr_rid / k_thr_rec)
    uint32_t* rid;                                      // [n] global run id of each SM_THREAD event
    uint32_t* run_start;                                // [runs] first sorted position of each run
    uint32_t* run_pre;                                  // [runs] live exits of a run not marked by the walk
    uint2* rrec;                                        // [n] entry records: (run id of the exit or ~0, acquireCount)
    uint32_t* seg_rb; uint32_t* seg_re;                 // [segments] run id range of a SM_THREAD segment
    const uint32_t* segflag;                            // [segments] SEGF_* flags
};

// A THREAD segment is decided run by run when its runs are long on average
// (few kind changes); the decision needs only the prepared tables, so both the
// record preparation (k_thr_rec) and the stream kernel take it the same way.
#ifndef SF_THR_RUN_AVG
#define SF_THR_RUN_AVG 16
#endif
SF_HD bool thr_run_mode(const HeavyCtx& hc, uint32_t s, uint32_t lo, uint32_t hi, uint32_t segflag) {
    const uint32_t nr = hc.seg_re[s] - hc.seg_rb[s];
    return !(segflag & SEGF_BIGC) && (uint64_t)(hi - lo) >= (uint64_t)SF_THR_RUN_AVG * nr;
}

SF_HD bool pass_bit(const unsigned long long* pb, uint32_t j) { return (pb[j >> 6] >> (j & 63)) & 1ull; }

// ------------------------------------------------------------------ team
#if defined(__HIP__)
struct Team {           // one wavefront: lock-step, reductions by cross-lane shuffles
    int rank;
    static constexpr int size = 64;
    __device__ long long min(long long v) {
        for (int o = 32; o > 0; o >>= 1) { long long w = __shfl_xor(v, o); v = w < v ? w : v; }
        return v;
    }
    __device__ bool leader() const { return rank == 0; }
};
#else
struct Team {
    int rank = 0;
    static constexpr int size = 1;
    long long min(long long v) { return v; }
    bool leader() const { return true; }
};
#endif

// First j in [lo, hi) with pred(j) true (pred monotone false..true); hi if none.
template <class P>
SF_HD uint32_t team_first_true(Team& tm, uint32_t lo, uint32_t hi, P pred) {
    if (tm.size == 1) {                                   // host build / tiny teams: binary search
        uint32_t a = lo, b = hi;
        while (a < b) { uint32_t m = a + (b - a) / 2; if (pred(m)) b = m; else a = m + 1; }
        return a;
    }
    while (lo < hi) {
        uint64_t n = hi - lo;
        if (n <= (uint64_t)tm.size) {
            long long cand = (tm.rank < (int)n && pred(lo + (uint32_t)tm.rank)) ? (long long)tm.rank : (long long)n;
            long long r = tm.min(cand);
            return lo + (uint32_t)r;
        }
        uint64_t step = (n + tm.size - 1) / tm.size;
        uint64_t last = (uint64_t)(tm.rank + 1) * step;
        if (last > n) last = n;
        long long cand = (tm.rank * step < n && pred(lo + (uint32_t)(last - 1))) ? (long long)tm.rank : (long long)tm.size;
        long long c = tm.min(cand);
        if (c >= tm.size) return hi;
        uint64_t nlo = c * step, nhi = (c + 1) * step;
        if (nhi > n) nhi = n;
        hi = lo + (uint32_t)nhi;
        lo = lo + (uint32_t)nlo;
    }
    return lo;
}

// First j in [lo, hi) with pred(j) true, pred arbitrary: forward scan, one
// team-wide chunk per step (cheap when the answer is near lo).
template <class P>
SF_HD uint32_t team_next(Team& tm, uint32_t lo, uint32_t hi, P pred) {
    for (uint32_t q = lo; q < hi; q += (uint32_t)tm.size) {
        const uint32_t j = q + (uint32_t)tm.rank;
        const long long cand = (j < hi && pred(j)) ? (long long)j : (long long)hi;
        const long long r = tm.min(cand);
        if (r < (long long)hi) return (uint32_t)r;
    }
    return hi;
}

SF_HD bool is_entry(uint8_t f) { return (f & SF_EV_EXIT) == 0; }
// an entry the controllers decide (not blocked before them: EVF_SYSBLK)
SF_HD bool is_checked_entry(uint8_t f) { return (f & (SF_EV_EXIT | EVF_SYSBLK)) == 0; }

// Σ acquireCount of entries in [a, b] inclusive (a <= b), from the global prefix
SF_HD int64_t csum(const int64_t* pcg, uint32_t a, uint32_t b) { return pcg[b] - (a ? pcg[a - 1] : 0); }

// pass bits: decided entries are one bit each in hc.passbits (k_heavy_fill
// turns them into verdicts); words at segment edges are shared, hence atomic
SF_HD void or_bits(unsigned long long* w, unsigned long long m) {
#if defined(__HIP_DEVICE_COMPILE__)
    atomicOr(w, m);
#else
    *w |= m;
#endif
}
// entries [a, b) passed: the team sets the words in parallel
SF_HD void set_pass_range(Team& tm, unsigned long long* pb, uint32_t a, uint32_t b) {
    if (a >= b) return;
    const uint32_t w0 = a >> 6, w1 = (b - 1) >> 6;
    for (uint32_t w = w0 + (uint32_t)tm.rank; w <= w1; w += (uint32_t)Team::size) {
        unsigned long long m = ~0ull;
        if (w == w0) m &= ~0ull << (a & 63);
        if (w == w1) m &= ~0ull >> (63 - ((b - 1) & 63));
        or_bits(pb + w, m);
    }
}

// ---------------------------------------------------------- QPS / WarmUp
// Runs uniformly on every lane of the team; only the leader writes.
// Only (windowStart, pass) of the second-window buckets matter here (the
// deltas are applied by heavy_apply); MAXS bounds the sample count at compile
// time and every bucket access is an unrolled compare-select (no lane memory).
template <int MAXS>
SF_HD void heavy_qps(Team& tm, const DevState& st, const SegIO& io, const HeavyCtx& hc, uint32_t s,
                     uint32_t res, uint32_t lo, uint32_t hi, bool warm) {
    const int S = st.S, wl = st.wl;
    int64_t sws[MAXS], spass[MAXS], bws[MAXS], bpass[MAXS];
#pragma unroll
    for (int i = 0; i < MAXS; i++) {
        if (i < S) {
            sws[i] = st.second[(size_t)res * S + i].ws; spass[i] = st.second[(size_t)res * S + i].pass;
            bws[i] = st.borrow[(size_t)res * S + i].ws; bpass[i] = st.borrow[(size_t)res * S + i].pass;
        } else { sws[i] = WS_NONE; spass[i] = 0; bws[i] = WS_NONE; bpass[i] = 0; }
    }
    const uint32_t r0 = st.rule_off[res];
    const DevRule rule = st.rules[r0];
    DevRuleState rs = st.rstate[r0];
    const Bucket* gmin = st.minute + (size_t)res * MINUTE;
    // per-second pass totals of the minute window (for previousPassQps)
    int64_t cur_sec = INT64_MIN, cur_sec_pass = 0, prev_sec_pass_known = INT64_MIN, prev_sec_pass = 0;
    int64_t last_sync_sec = INT64_MIN;

    uint32_t p = lo;
    while (p < hi) {
        const int64_t t0 = io.ts[p];
        const int64_t h = t0 / wl, ws = h * wl, hw_end = ws + wl;
        const uint32_t b = team_first_true(tm, p, hi, [&](uint32_t j) { return io.ts[j] >= hw_end; });
        // second-window roll at t0 (OccupiableBucketLeapArray.currentWindow)
        const int idx = (int)(h % S);
        int64_t cur_pass = 0, p_prev = 0;
#pragma unroll
        for (int i = 0; i < MAXS; i++) {
            if (i == idx) {
                if (sws[i] != ws) {                    // roll: reset / create (resetWindowTo :52-64)
                    const int64_t bw = bws[i], bp = bpass[i];   // borrow slot of ws is the same index
                    sws[i] = ws;
                    spass[i] = (bw <= ws && ws < bw + wl) ? (int64_t)(int32_t)bp : 0;
                }
                cur_pass = spass[i];
            }
        }
#pragma unroll
        for (int i = 0; i < MAXS; i++)
            if (i < S && i != idx && !(wsub(t0, sws[i]) > st.interval)) p_prev = wadd(p_prev, spass[i]);
        const int64_t base = p_prev + cur_pass;
        // minute-window bookkeeping for this hw's second
        const int64_t sn = t0 / 1000;
        if (sn != cur_sec) {
            // pass of the minute bucket for second sn before this batch's passes
            const Bucket& mb = gmin[(int)(sn % MINUTE)];
            int64_t init = (mb.ws == sn * 1000) ? mb.pass : 0;
            if (cur_sec != INT64_MIN) { prev_sec_pass_known = cur_sec; prev_sec_pass = cur_sec_pass; }
            cur_sec = sn; cur_sec_pass = init;
        }
        // entries of [p, b)
        const bool has_entry = csum(hc.pcg, p, b - 1) > 0;
        double thr = rule.count;
        if (warm && has_entry) {
            if (sn > last_sync_sec) {
                int64_t prev_qps;                 // previousPassQps: minute bucket (sn-1)
                if (prev_sec_pass_known == sn - 1) prev_qps = prev_sec_pass;
                else {
                    const Bucket& pb = gmin[(int)((sn - 1) % MINUTE)];
                    prev_qps = (pb.ws == (sn - 1) * 1000) ? pb.pass : 0;
                }
                warm_sync(rule, rs, t0, prev_qps);
                last_sync_sec = sn;
            }
            int64_t rest = rs.stored_tokens;
            if (rest >= rule.warning_token) {
                int64_t above = rest - rule.warning_token;
                thr = j_next_up(1.0 / ((double)above * rule.slope + 1.0 / rule.count));
            }
        }
        int64_t passed = 0;
        if (has_entry) {
            const int64_t* pcg = hc.pcg;
            const int64_t pc0 = p ? pcg[p - 1] : 0;
            // first failing entry: (double)(base + Σc[p..j]) > thr  (DefaultController: (int)passQps + c > count)
            const uint32_t f = team_first_true(tm, p, b, [&](uint32_t j) {
                return (double)(base + (pcg[j] - pc0)) > thr;
            });
            if (f > p) { passed = (f ? pcg[f - 1] : 0) - pc0; set_pass_range(tm, hc.passbits, p, f); }
            // tail: remaining entries with small acquireCount may still fit
            uint32_t j = f + 1;
            while (j < b && (double)(base + passed + 1) <= thr) {      // else no c >= 1 can pass any more
                j = team_next(tm, j, b, [&](uint32_t k) {
                    return is_checked_entry(io.flags[k]) && (double)(base + passed + io.cnt[k]) <= thr;
                });
                if (j >= b) break;
                passed += io.cnt[j];
                if (tm.leader()) or_bits(hc.passbits + (j >> 6), 1ull << (j & 63));
                j++;
            }
        }
#pragma unroll
        for (int i = 0; i < MAXS; i++)
            if (i == idx) spass[i] = wadd(spass[i], passed);
        cur_sec_pass = wadd(cur_sec_pass, passed);
        p = b;
    }
    if (tm.leader()) st.rstate[r0] = rs;
    (void)s;
}

// ---------------------------------------------------------- RateLimiter
SF_HD void heavy_rl(Team& tm, const DevState& st, const SegIO& io, const HeavyCtx& hc, uint32_t s,
                    uint32_t res, uint32_t lo, uint32_t hi) {
    const uint32_t r0 = st.rule_off[res];
    const DevRule rule = st.rules[r0];
    DevRuleState rs = st.rstate[r0];
    if (rule.count > 0) {
        const int64_t cost1 = j_round(1.0 * 1 / rule.count * 1000);
        int64_t L = rs.latest_passed;
        uint32_t p = lo;
        while (p < hi) {
            const int64_t thr = L + cost1 - rule.max_queue_ms;
            // entries before thr cannot pass (cost >= cost1 for c >= 1); first candidate chunk checked directly
            uint32_t j = (p < hi && io.ts[p] >= thr) ? p
                         : team_first_true(tm, p, hi, [&](uint32_t k) { return io.ts[k] >= thr; });
            j = team_next(tm, j, hi, [&](uint32_t k) {
                if (!is_checked_entry(io.flags[k])) return false;
                const int32_t c = io.cnt[k];
                const int64_t ck = c == 1 ? cost1 : j_round(1.0 * c / rule.count * 1000);
                return io.ts[k] >= L + ck - rule.max_queue_ms;
            });
            if (j >= hi) break;
            const int32_t cj = io.cnt[j];
            const int64_t cost = cj == 1 ? cost1 : j_round(1.0 * cj / rule.count * 1000);
            const int64_t t = io.ts[j];
            int32_t wait = 0;
            if (L + cost <= t) L = t;
            else { L += cost; wait = (int32_t)(L - t); }
            if (tm.leader()) {
                or_bits(hc.passbits + (j >> 6), 1ull << (j & 63));
                if (io.v_wait) io.v_wait[j] = wait;
            }
            p = j + 1;
        }
        rs.latest_passed = L;
    }
    if (tm.leader()) st.rstate[r0] = rs;
    (void)s;
}


// ---------------------------------------------------------- THREAD grade
// DefaultController, FLOW_GRADE_THREAD (DefaultController.java:50-89): an
// entry passes iff (int)curThreadNum + c <= count; a pass adds one thread
// (StatisticSlot.java:64-65), the exit of a passed entry removes it (:157).
// The exit of an entry decided in this batch is live iff that entry passed.
// Output: one bit per passed entry in hc.passbits; k_heavy_fill turns the
// bits into verdicts and window counters.
#if !defined(__HIP__)
// host build (tests/hostsim): one event at a time; the GPU runs k_heavy_stream
inline void heavy_thread(Team&, const DevState& st, const SegIO& io, const HeavyCtx& hc, uint32_t, uint32_t res,
                         uint32_t lo, uint32_t hi, unsigned long long*, unsigned long long*) {
    const double M = st.rules[st.rule_off[res]].count;
    int64_t T = st.threads[res];
    for (uint32_t j = lo; j < hi; j++) {
        if (is_entry(io.flags[j])) {
            if (!(io.flags[j] & EVF_SYSBLK) && (double)(int32_t)((uint32_t)(int32_t)T + (uint32_t)io.cnt[j]) <= M) {
                T++;
                hc.passbits[j >> 6] |= 1ull << (j & 63);
            }
        } else {
            const int64_t r = io.eref ? io.eref[j] : -1;
            if (r == -1 || (r >= (int64_t)lo && r < (int64_t)j && pass_bit(hc.passbits, (uint32_t)r))) T--;
        }
    }
}
#endif

// Apply the per-window deltas of one heavy segment to its node state in
// time order (LeapArray.currentWindow reset semantics; MetricBucket adds).
SF_HD void heavy_apply(const DevState& st, const HeavyCtx& hc, uint32_t s, uint32_t res, uint32_t n_hw,
                       uint32_t n_sec) {
    const int S = st.S, wl = st.wl;
    const int64_t h0 = hc.seg_hw0[s], s0 = hc.seg_sec0[s];
    int64_t threads = st.threads[res];
    for (uint32_t k = 0; k < n_hw; k++) {
        const Acc& a = hc.acc_hw[hc.acc_hw_base[s] + k];
        if (!a.n_touch) continue;
        const int64_t h = h0 + k, ws = h * wl;
        Bucket& b = st.second[(size_t)res * S + (int)(h % S)];
        if (b.ws != ws) {
            Bucket nb = fresh_bucket(ws, st.max_rt);
            const Borrow& bw = st.borrow[(size_t)res * S + (int)(h % S)];
            if (bw.ws <= ws && ws < bw.ws + wl) nb.pass = (int64_t)(int32_t)bw.pass;
            b = nb;
        }
        b.pass = wadd(b.pass, (int64_t)a.pass); b.block = wadd(b.block, (int64_t)a.block);
        b.succ = wadd(b.succ, (int64_t)a.succ); b.rt = wadd(b.rt, (int64_t)a.rt); b.exc = wadd(b.exc, (int64_t)a.exc);
        if (a.min_rt < b.min_rt) b.min_rt = a.min_rt;
        threads += (int64_t)a.n_pass - (int64_t)a.n_exit;
    }
    for (uint32_t k = 0; k < n_sec; k++) {
        const Acc& a = hc.acc_sec[hc.acc_sec_base[s] + k];
        if (!a.n_touch) continue;
        const int64_t sn = s0 + k, ws = sn * 1000;
        Bucket& b = st.minute[(size_t)res * MINUTE + (int)(sn % MINUTE)];
        if (b.ws != ws) b = fresh_bucket(ws, st.max_rt);
        b.pass = wadd(b.pass, (int64_t)a.pass); b.block = wadd(b.block, (int64_t)a.block);
        b.succ = wadd(b.succ, (int64_t)a.succ); b.rt = wadd(b.rt, (int64_t)a.rt); b.exc = wadd(b.exc, (int64_t)a.exc);
        if (a.min_rt < b.min_rt) b.min_rt = a.min_rt;
    }
    st.threads[res] = threads;
}

// verdict + accounting contribution of event j of a heavy segment decided
// into pass bits (QPS / WarmUp / RL / THREAD; no-rule segments pass every
// entry).  RateLimiter waits were written into v_wait when the entry passed.
struct EvContrib { uint8_t status; int32_t wait; bool touch, passed, live_exit; int64_t c, rt; bool err; };
SF_HD EvContrib heavy_event(const HeavyCtx& hc, const SegIO& io, uint32_t lo, uint8_t mode, uint32_t j) {
    EvContrib r{};
    const uint8_t f = io.flags[j];
    r.c = io.cnt[j];
    const bool all = mode == SM_NORULE;
    if (is_entry(f)) {
        const bool sysb = (f & EVF_SYSBLK) != 0;
        r.passed = !sysb && (all || pass_bit(hc.passbits, j));
        r.wait = (mode == SM_RL && r.passed && io.v_wait) ? io.v_wait[j] : 0;
        r.status = r.passed ? (r.wait > 0 ? SF_V_PASS_WAIT : SF_V_PASS) : (sysb ? sysblk_status(f) : SF_V_BLOCK_FLOW);
        r.touch = true;
    } else {
        const int64_t ref = io.eref ? io.eref[j] : -1;
        r.live_exit = ref == -1 || (ref >= (int64_t)lo && ref < (int64_t)j && !(io.flags[ref] & EVF_SYSBLK) &&
                                    (all || pass_bit(hc.passbits, (uint32_t)ref)));
        r.status = r.live_exit ? SF_V_EXIT : SF_V_EXIT_IGNORED;
        r.touch = r.live_exit;
        r.rt = io.ts[j] - (ref >= 0 ? io.ts[ref] : (io.cts ? io.cts[j] : io.ts[j]));
        r.err = (f & SF_EV_ERROR) != 0;
    }
    return r;
}

}  // namespace sf
