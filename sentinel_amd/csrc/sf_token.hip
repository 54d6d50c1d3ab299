// sf_token.hip — gfx950 kernels of one sf_request_tokens (product code).
//
// A batch of token requests, time-ordered, as the Netty workers of the
// reference token server would hand them to DefaultTokenService one by one.
// Decisions are bit-exact with the reference replayed in batch order.
//
//   k_tok_prep      DefaultTokenService.notValidRequest / rule lookup
//                   (BAD_REQUEST, NO_RULE_EXISTS), namespace of each request
//   namespace gate  GlobalRequestLimiter.tryPass: requests radix-sorted by
//                   namespace (stable: time order kept); one wavefront per
//                   namespace walks its 100-ms windows.  Inside a window the
//                   limiter sum of the other buckets is constant, so the
//                   passes are the first K requests (TOO_MANY_REQUEST after)
//   k_tok_keys      key of a request that reached the checker: the flow rule
//                   index, or the exact (param rule, value) table slot
//   radix sort      (key, index): requests grouped per flowId / per value
//   k_tok_decide    one lane per group replays ClusterFlowChecker (the
//                   flowId's ClusterMetricLeapArray staged in LDS) or
//                   ClusterParamFlowChecker (one value's window counts)
//
// Param values of one rule are independent: ClusterParamMetric.getSum(value)
// only counts the value's own adds in the buckets that values() keeps, and a
// bucket reset by any value's currentWindow() only clears windows the value
// could not count any more (time-ordered requests).  So each (rule, value)
// keeps its own column of (window start, count) pairs, and different values
// are decided in parallel.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "sf_decide.h"
#include "sf_token.h"

namespace sf {

constexpr uint8_t NS_NONE = 0xff;
constexpr uint64_t KEY_NONE = ~0ull;
constexpr uint64_t KEY_PARAM = 1ull << 63;
constexpr uint64_t KEY_SERIAL = 1ull << 62;     // every request of one param rule, in time order
constexpr int8_t TOK_PENDING = 100;

static inline unsigned tblocks(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

__device__ __forceinline__ uint64_t id_hash(int64_t id) { return mix64((uint64_t)id * 0x9e3779b97f4a7c15ULL); }

__device__ int32_t id_lookup(const TokState& ts, int64_t id, bool param) {
    uint64_t i = id_hash(id) & ts.id_mask;
    for (uint64_t p = 0; p <= ts.id_mask; p++) {
        const IdSlot& s = ts.idtab[i];
        if (s.id == 0) return -1;
        if (s.id == id) return param ? s.param : s.flow;
        i = (i + 1) & ts.id_mask;
    }
    return -1;
}

// DefaultTokenService.requestToken / requestParamToken up to the checker
__global__ void k_tok_prep(TokState ts, TokBatch b, TokWork w, TokOut out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    const int64_t id = b.flow_id[i];
    const int32_t c = b.count[i];
    const bool param = (b.flags[i] & SF_TOK_PARAM) != 0;
    const int32_t r = id > 0 ? id_lookup(ts, id, param) : -1;
    // sharded token server: only the owner shard decides (sf_token_shard)
    const uint32_t owner = id <= 0 ? 0u : (r >= 0 ? ts.rules[r].owner : (uint32_t)((uint64_t)id % ts.shard_count));
    if (owner != ts.shard_index) *ts.err = SF_ERR_INVALID;
    int8_t st = TOK_PENDING;
    uint8_t nk = NS_NONE;
    const uint32_t nv = (param && b.poff) ? b.poff[i + 1] - b.poff[i] : 1u;
    if (id <= 0 || c <= 0 || (param && (!b.ptag || !b.pbits || nv == 0))) {
        st = SF_TOKEN_BAD_REQUEST;                          // notValidRequest / params empty :66-72
    } else if (r < 0) {
        st = SF_TOKEN_NO_RULE_EXISTS;                       // getFlowRuleById == null :45-47
    } else {
        w.rule_of[i] = (uint32_t)r;
        // a request with several values couples them (all must pass before any is
        // added): that rule's requests are decided by one lane in time order
        if (nv > 1) ts.rmulti[r] = 1;
        const int32_t ns = ts.rules[r].ns;
        if (ns >= 0 && ts.ns[ns].has_limiter) nk = (uint8_t)ns;   // else GlobalRequestLimiter passes
    }
    w.pending[i] = st == TOK_PENDING;
    w.nskey_in[i] = nk;
    w.idx_in[i] = i;
    out.status[i] = st == TOK_PENDING ? 0 : st;
    out.remaining[i] = 0;
    out.wait[i] = 0;
}

// namespace ranges in the namespace-sorted order
__global__ void k_ns_bounds(const uint8_t* nsk, uint32_t n, uint32_t* lo, uint32_t* hi) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint8_t k = nsk[j];
    if (k == NS_NONE) return;
    if (j == 0 || nsk[j - 1] != k) lo[k] = j;
    if (j == n - 1 || nsk[j + 1] != k) hi[k] = j + 1;
}

// GlobalRequestLimiter.tryPass (RequestLimiter.canPass: sum / 1.0 + 1 <= qpsAllowed,
// then add 1 to the current bucket), one wavefront per namespace.
__global__ void __launch_bounds__(64) k_ns_limit(TokState ts, TokBatch b, TokWork w, TokOut out, const uint32_t* nlo,
                                                 const uint32_t* nhi) {
    const uint32_t ns = blockIdx.x;
    const uint32_t lo = nlo[ns], hi = nhi[ns];
    if (hi <= lo) return;
    const int lane = (int)threadIdx.x;
    const double qps = ts.ns[ns].max_qps;
    LimState L = ts.lim[ns];
    uint32_t p = lo;
    while (p < hi) {
        const int64_t t0 = b.ts[w.idx_out[p]];
        const int64_t ws = t0 - t0 % LIM_WL, wend = ws + LIM_WL;
        // end of this window: wave-wide 64-ary search over the sorted times
        uint32_t a = p, e = hi;
        while (e - a > 64) {
            const uint32_t step = (e - a + 63) / 64;
            const uint32_t last = min(a + (uint32_t)(lane + 1) * step, e) - 1;
            const bool ge = a + (uint32_t)lane * step < e && b.ts[w.idx_out[last]] >= wend;
            const unsigned long long m = __ballot(ge);
            if (!m) { a = e; break; }
            const uint32_t k = (uint32_t)(__ffsll((long long)m) - 1);
            const uint32_t na = a + k * step;
            e = min(a + (k + 1) * step, e);
            a = na;
        }
        uint32_t bnd = e;
        if (a < e) {
            const unsigned long long m = __ballot(a + (uint32_t)lane < e && b.ts[w.idx_out[a + lane]] >= wend);
            bnd = m ? a + (uint32_t)(__ffsll((long long)m) - 1) : e;
        }
        // currentWindow(t0) then values(t0): other buckets' validity is constant inside the window
        const int cur = (int)((t0 / LIM_WL) % LIM_S);
        int64_t sum = 0, cur_v = 0;
        for (int k = 0; k < LIM_S; k++) {
            if (k == cur) cur_v = L.ws[k] == ws ? L.v[k] : 0;
            else if (L.ws[k] != WS_NONE && !(t0 - L.ws[k] > LIM_INTERVAL)) sum = wadd(sum, L.v[k]);
        }
        sum = wadd(sum, cur_v);
        // request k of the window passes iff (sum + k) / 1.0 + 1 <= qps (monotone in k)
        const uint32_t nw = bnd - p;
        uint32_t klo = 0, khi = nw;                      // first failing k
        while (klo < khi) {
            const uint32_t mid = (klo + khi) / 2;
            if ((double)wadd(sum, (int64_t)mid) / 1.0 + 1 <= qps) klo = mid + 1;
            else khi = mid;
        }
        const uint32_t K = klo;
        for (uint32_t j = p + K + (uint32_t)lane; j < bnd; j += 64) {
            const uint32_t i = w.idx_out[j];
            w.pending[i] = 0;
            out.status[i] = SF_TOKEN_TOO_MANY_REQUEST;
        }
        L.ws[cur] = ws;
        L.v[cur] = wadd(cur_v, (int64_t)K);
        p = bnd;
    }
    if (lane == 0) ts.lim[ns] = L;
}

// exact (param rule, value) slot: find, or claim an empty one.  A slot being
// claimed (CP_CLAIM) is re-read until its owner publishes the key; the owner
// finishes without waiting on anyone, so the wait is bounded.
__device__ uint32_t cp_find_or_insert(const TokState& ts, uint64_t hi, uint64_t lo) {
    uint64_t i = mix64(hi ^ mix64(lo + 0x9e3779b97f4a7c15ULL)) & ts.cp_mask;
    uint64_t probes = 0;
    const uint64_t reach = ts.cp_mask < PT_MAX_PROBE ? ts.cp_mask : PT_MAX_PROBE;   // as ParamTable (sf_decide.h)
    while (probes <= reach) {
        CpSlot& s = ts.cptab[i];
        const uint64_t h = __hip_atomic_load(&s.hi, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (h == 0) {
            uint64_t expected = 0;
            if (__hip_atomic_compare_exchange_strong(&s.hi, &expected, hi | CP_CLAIM, __ATOMIC_ACQUIRE,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                s.lo = lo;
                for (int k = 0; k < CL_MAXS; k++) { s.ws[k] = WS_NONE; s.cnt[k] = 0; }
                __hip_atomic_store(&s.hi, hi, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                return (uint32_t)i;
            }
            continue;                                   // lost the race: look at this slot again
        }
        if (h & CP_CLAIM) { __builtin_amdgcn_s_sleep(1); continue; }
        if (h == hi && s.lo == lo) return (uint32_t)i;
        i = (i + 1) & ts.cp_mask;
        probes++;
    }
    *ts.err = SF_ERR_CAPACITY;
    return 0xffffffffu;
}

__global__ void k_tok_keys(TokState ts, TokBatch b, TokWork w, TokOut out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    uint64_t key = KEY_NONE;
    if (w.pending[i]) {
        const uint32_t r = w.rule_of[i];
        const ClRule& rule = ts.rules[r];
        const uint32_t v0 = b.poff ? b.poff[i] : i;
        if (!rule.is_param) key = r;
        else if (ts.rmulti[r]) key = KEY_SERIAL | r;
        else if (b.ptag[v0] == SF_TAG_NULL) {
            // a null value has no metric: getSum(null) == 0 and addValue(null) adds nothing
            // (ClusterParamMetric.java:52-55,72-75), so the decision needs no state
            const int32_t connected = rule.ns >= 0 ? ts.ns[rule.ns].connected : 0;
            double raw = rule.count;
            for (uint32_t k = 0; k < rule.item_cnt; k++)
                if (ts.items[rule.item_off + k].tag == SF_TAG_NULL) { raw = ts.items[rule.item_off + k].count; break; }
            const double thr = rule.threshold_type == SF_THRESHOLD_GLOBAL ? raw : raw * connected;
            const double next = thr - 0.0 - b.count[i];
            out.status[i] = next >= 0 ? SF_TOKEN_OK : SF_TOKEN_BLOCKED;
            out.remaining[i] = next >= 0 ? j_d2i(next) : 0;
            out.wait[i] = 0;
        } else {
            const uint64_t hi = ((uint64_t)(r + 1) << 32) | b.ptag[v0];
            const uint32_t slot = cp_find_or_insert(ts, hi, b.pbits[v0]);
            if (slot != 0xffffffffu) key = KEY_PARAM | slot;
        }
    }
    w.key_in[i] = key;
    w.idx_in[i] = i;
}

__global__ void k_tok_heads(const uint64_t* key, uint32_t n, uint32_t* head) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    head[j] = (key[j] != KEY_NONE && (j == 0 || key[j] != key[j - 1])) ? 1u : 0u;
}
__global__ void k_tok_segments(const uint64_t* key, const uint32_t* head, const uint32_t* pos, uint32_t n,
                               uint32_t* seg_start, uint32_t* n_seg) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    if (head[j]) seg_start[pos[j]] = j;
    // the last segment ends where KEY_NONE starts (sorted last) or at n
    const bool last_valid = key[j] != KEY_NONE && (j == n - 1 || key[j + 1] == KEY_NONE);
    if (last_valid) { const uint32_t ns = pos[j] + head[j]; *n_seg = ns; seg_start[ns] = j + 1; }
}

// ---------------------------------------------------------------- ClusterMetric (one flowId, in LDS)
struct ClMetric {
    ClFlowState* s;
    int S, wl, I;
    double isec;
    // LeapArray.currentWindow(t) with ClusterMetricLeapArray.resetWindowTo (:45-71); -1: throwaway
    __device__ int cur(int64_t t) {
        const int idx = (int)((t / wl) % S);
        const int64_t ws = t - t % wl;
        ClBucket& b = s->b[idx];
        if (b.ws == WS_NONE) {                                   // newEmptyBucket: no transfer
            b.ws = ws;
            for (int k = 0; k < CE_COUNT; k++) b.c[k] = 0;
            return idx;
        }
        if (b.ws == ws) return idx;
        if (ws > b.ws) {
            b.ws = ws;
            for (int k = 0; k < CE_COUNT; k++) b.c[k] = 0;
            if (s->has_occ) {                                    // transferOccupyToBucket :54-60
                b.c[CE_OCCUPIED_PASS] = wadd(b.c[CE_OCCUPIED_PASS], s->occ_pass);
                b.c[CE_PASS] = wadd(b.c[CE_PASS], s->occ_pass); s->occ_pass = 0;
                b.c[CE_PASS_REQUEST] = wadd(b.c[CE_PASS_REQUEST], s->occ_req); s->occ_req = 0;
                s->has_occ = 0;
            }
            return idx;
        }
        return -1;
    }
    __device__ int64_t sum(int ev, int64_t t) {                  // ClusterMetric.getSum :47-55
        cur(t);
        int64_t r = 0;
        for (int k = 0; k < S; k++) {
            const ClBucket& b = s->b[k];
            if (b.ws != WS_NONE && !(wsub(t, b.ws) > I)) r = wadd(r, b.c[ev]);
        }
        return r;
    }
    __device__ double avg(int ev, int64_t t) { return (double)sum(ev, t) / isec; }
    __device__ void add(int ev, int64_t n, int64_t t) {
        const int k = cur(t);
        if (k >= 0) s->b[k].c[ev] = wadd(s->b[k].c[ev], n);
    }
    __device__ int64_t head_pass(int64_t t) {                    // getFirstCountOfWindow -> getValidHead
        const int idx = (int)(((t + wl) / wl) % S);
        const ClBucket& b = s->b[idx];
        if (b.ws == WS_NONE || wsub(t, b.ws) > I) return 0;
        return b.c[CE_PASS];
    }
};

// ClusterFlowChecker.acquireClusterToken (:55-112) for one request that passed the namespace gate
__device__ void flow_decide(ClMetric& m, const ClRule& r, const TokState& ts, int32_t connected, int64_t t, int32_t c,
                            bool prio, int8_t* st, int32_t* rem, int32_t* wt) {
    const double latest = m.avg(CE_PASS, t);
    const double thr = (r.threshold_type == SF_THRESHOLD_GLOBAL ? r.count : r.count * connected) * ts.exceed_count;
    const double next = thr - latest - c;
    if (next >= 0) {
        m.add(CE_PASS, c, t); m.add(CE_PASS_REQUEST, 1, t);
        if (prio) m.add(CE_OCCUPIED_PASS, c, t);
        *st = SF_TOKEN_OK; *rem = j_d2i(next); *wt = 0;
        return;
    }
    if (prio) {
        const double occ_avg = m.avg(CE_WAITING, t);
        if (occ_avg <= ts.max_occupy_ratio * thr) {
            // ClusterMetric.tryOccupyNext :69-79, canOccupy :81-86
            const double latest2 = m.avg(CE_PASS, t);
            const int64_t head = m.head_pass(t);
            const int64_t occupied = m.s->occ_pass;
            if (latest2 + (double)((int64_t)c + occupied) - (double)head <= thr) {
                m.s->occ_pass = wadd(m.s->occ_pass, c);          // addOccupyPass :74-78
                m.s->occ_req = wadd(m.s->occ_req, 1);
                m.s->has_occ = 1;
                m.add(CE_WAITING, c, t);
                const int32_t w = 1000 / m.S;
                if (w > 0) { *st = SF_TOKEN_SHOULD_WAIT; *rem = 0; *wt = w; return; }
            }
        }
    }
    m.add(CE_BLOCK, c, t); m.add(CE_BLOCK_REQUEST, 1, t);
    if (prio) m.add(CE_OCCUPIED_BLOCK, c, t);
    *st = SF_TOKEN_BLOCKED; *rem = 0; *wt = 0;
}

// one value's column of ClusterParameterLeapArray: getSum(value) at t (:52-66)
// and addValue(value, c) (:72-84) -- only the value's own adds are counted
__device__ __forceinline__ int64_t cp_sum(const CpSlot& s, int S, int wl, int I, int64_t t) {
    const int idx = (int)((t / wl) % S);
    const int64_t ws = t - t % wl;
    int64_t sum = 0;
    for (int k = 0; k < S; k++) {
        if (k == idx) { if (s.ws[k] == ws) sum = wadd(sum, s.cnt[k]); }
        else if (s.ws[k] != WS_NONE && !(wsub(t, s.ws[k]) > I)) sum = wadd(sum, s.cnt[k]);
    }
    return sum;
}
__device__ __forceinline__ void cp_add(CpSlot& s, int S, int wl, int64_t t, int32_t c) {
    const int idx = (int)((t / wl) % S);
    const int64_t ws = t - t % wl;
    if (s.ws[idx] != ws) {
        if (ws < s.ws[idx]) return;                              // throwaway window
        s.ws[idx] = ws; s.cnt[idx] = 0;
    }
    s.cnt[idx] = wadd(s.cnt[idx], c);
}
// getRawThreshold (:110-117) + calcGlobalThreshold (:97-108)
__device__ __forceinline__ double cp_threshold(const TokState& ts, const ClRule& rule, int32_t connected, uint8_t tag,
                                               uint64_t bits) {
    double raw = rule.count;
    for (uint32_t k = 0; k < rule.item_cnt; k++) {
        const DevHotItem& it = ts.items[rule.item_off + k];
        if (it.tag == tag && it.bits == bits) { raw = it.count; break; }
    }
    return rule.threshold_type == SF_THRESHOLD_GLOBAL ? raw : raw * connected;
}

// ClusterParamFlowChecker.acquireClusterToken (:42-87) for every request of one
// param rule that has multi-value requests in this batch, in time order: each
// value needs room (the first without stops the check), then every value is
// added; remaining is -1 for more than one value.  Value columns are found /
// claimed in the exact table as the single-value path does.
__device__ void tok_serial_rule(const TokState& ts, const TokBatch& b, const TokWork& w, const TokOut& out, uint32_t r,
                                uint32_t lo, uint32_t hi) {
    const ClRule rule = ts.rules[r];
    const int32_t connected = rule.ns >= 0 ? ts.ns[rule.ns].connected : 0;
    const double isec = rule.interval / 1000.0;
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t i = w.idx_out[j];
        const int64_t t = b.ts[i];
        const int32_t c = b.count[i];
        const uint32_t v0 = b.poff ? b.poff[i] : i, v1 = b.poff ? b.poff[i + 1] : i + 1;
        double rem = -1;
        bool passed = true;
        for (uint32_t v = v0; v < v1; v++) {
            const uint8_t tg = b.ptag[v];
            int64_t sum = 0;
            if (tg != SF_TAG_NULL) {                             // getSum(null) == 0
                const uint32_t sl = cp_find_or_insert(ts, ((uint64_t)(r + 1) << 32) | tg, b.pbits[v]);
                if (sl == 0xffffffffu) { passed = false; break; }
                sum = cp_sum(ts.cptab[sl], rule.S, rule.wl, rule.interval, t);
            }
            rem = cp_threshold(ts, rule, connected, tg, b.pbits[v]) - (double)sum / isec - c;
            if (rem < 0) { passed = false; break; }
        }
        if (passed) {
            for (uint32_t v = v0; v < v1; v++) {
                if (b.ptag[v] == SF_TAG_NULL) continue;          // addValue(null) adds nothing
                const uint32_t sl = cp_find_or_insert(ts, ((uint64_t)(r + 1) << 32) | b.ptag[v], b.pbits[v]);
                if (sl != 0xffffffffu) cp_add(ts.cptab[sl], rule.S, rule.wl, t, c);
            }
            if (v1 - v0 > 1) rem = -1;
            out.status[i] = SF_TOKEN_OK; out.remaining[i] = j_d2i(rem);
        } else {
            out.status[i] = SF_TOKEN_BLOCKED; out.remaining[i] = 0;
        }
        out.wait[i] = 0;
    }
}

constexpr int TD_T = 64;     // lanes per workgroup of k_tok_decide (LDS: one ClFlowState per lane)

__global__ void __launch_bounds__(TD_T) k_tok_decide(TokState ts, TokBatch b, TokWork w, TokOut out) {
    __shared__ ClFlowState lds[TD_T];
    const uint32_t sg = blockIdx.x * blockDim.x + threadIdx.x;
    if (sg >= *w.n_seg) return;
    const uint32_t lo = w.seg_start[sg], hi = w.seg_start[sg + 1];
    const uint64_t key = w.key_out[lo];
    if (key & KEY_SERIAL) { tok_serial_rule(ts, b, w, out, (uint32_t)(key & 0xffffffffu), lo, hi); return; }
    if (!(key & KEY_PARAM)) {
        const uint32_t r = (uint32_t)key;
        const ClRule rule = ts.rules[r];
        const int32_t connected = rule.ns >= 0 ? ts.ns[rule.ns].connected : 0;
        ClFlowState* st = &lds[threadIdx.x];
        *st = ts.fstate[r];
        ClMetric m{st, rule.S, rule.wl, rule.interval, rule.interval / 1000.0};
        for (uint32_t j = lo; j < hi; j++) {
            const uint32_t i = w.idx_out[j];
            int8_t s; int32_t rem, wt;
            flow_decide(m, rule, ts, connected, b.ts[i], b.count[i], (b.flags[i] & SF_TOK_PRIORITIZED) != 0, &s, &rem, &wt);
            out.status[i] = s; out.remaining[i] = rem; out.wait[i] = wt;
        }
        ts.fstate[r] = *st;
        return;
    }
    // ClusterParamFlowChecker.acquireClusterToken (:42-87), one value per request
    CpSlot& slot = ts.cptab[key & ~KEY_PARAM];
    const uint32_t r = (uint32_t)((slot.hi >> 32) & 0x7fffffffu) - 1u;
    const uint8_t tag = (uint8_t)(slot.hi & 0xff);
    const uint64_t bits = slot.lo;
    const ClRule rule = ts.rules[r];
    const int32_t connected = rule.ns >= 0 ? ts.ns[rule.ns].connected : 0;
    const double thr = cp_threshold(ts, rule, connected, tag, bits);
    const int S = rule.S, wl = rule.wl, I = rule.interval;
    const double isec = rule.interval / 1000.0;
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t i = w.idx_out[j];
        const int64_t t = b.ts[i];
        const int32_t c = b.count[i];
        const double next = thr - (double)cp_sum(slot, S, wl, I, t) / isec - c;   // getSum(value)
        if (next >= 0) {
            cp_add(slot, S, wl, t, c);                           // addValue :72-84
            out.status[i] = SF_TOKEN_OK; out.remaining[i] = j_d2i(next);
        } else {
            out.status[i] = SF_TOKEN_BLOCKED; out.remaining[i] = 0;
        }
        out.wait[i] = 0;
    }
}

__global__ void k_tok_init_flow(ClFlowState* fs, uint32_t n) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    ClFlowState s;
    for (int k = 0; k < CL_MAXS; k++) { s.b[k].ws = WS_NONE; for (int e = 0; e < CE_COUNT; e++) s.b[k].c[e] = 0; }
    s.occ_pass = s.occ_req = s.has_occ = s.pad = 0;
    fs[r] = s;
}

__global__ void k_tok_cluster_sum(TokState ts, uint32_t r, int ev, int64_t now, int64_t* out) {
    const ClRule rule = ts.rules[r];
    ClMetric m{&ts.fstate[r], rule.S, rule.wl, rule.interval, rule.interval / 1000.0};
    *out = m.sum(ev, now);
}

hipError_t tok_init_flow_state(ClFlowState* fs, uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_tok_init_flow, dim3(tblocks(n, 256)), dim3(256), 0, s, fs, n);
    return hipGetLastError();
}

hipError_t tok_cluster_sum(const TokState& ts, uint32_t rule, int event, int64_t now, int64_t* d_out, hipStream_t s) {
    hipLaunchKernelGGL(k_tok_cluster_sum, dim3(1), dim3(1), 0, s, ts, rule, event, now, d_out);
    return hipGetLastError();
}

hipError_t tok_query_temp(uint32_t max_n, size_t* sort8, size_t* sort64, size_t* scan) {
    hipError_t e = rocprim::radix_sort_pairs(nullptr, *sort8, (uint8_t*)nullptr, (uint8_t*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, max_n, 0u, 8u);
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(nullptr, *sort64, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, max_n, 0u, 64u);
    if (e != hipSuccess) return e;
    return rocprim::exclusive_scan(nullptr, *scan, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)max_n,
                                   rocprim::plus<uint32_t>());
}

hipError_t tok_launch(const TokState& ts, TokWork& w, const TokBatch& b, const TokOut& out, hipStream_t s) {
    const uint32_t n = b.n;
    if (!n) return hipSuccess;
    const unsigned T = 256;
    hipMemsetAsync(ts.rmulti, 0, ts.n_rules ? ts.n_rules : 1, s);
    hipLaunchKernelGGL(k_tok_prep, dim3(tblocks(n, T)), dim3(T), 0, s, ts, b, w, out);
    bool any_limiter = false;   // known on the host through n_ns (the table may have none with a limiter)
    any_limiter = ts.n_ns > 0;
    if (any_limiter) {
        hipError_t e = rocprim::radix_sort_pairs(w.sort8_tmp, w.sort8_bytes, w.nskey_in, w.nskey_out, w.idx_in,
                                                 w.idx_out, n, 0u, 8u, s);
        if (e != hipSuccess) return e;
        uint32_t* nlo = w.head;              // scratch: 256 + 256 words (head is reused below)
        uint32_t* nhi = w.head + 256;
        hipMemsetAsync(nlo, 0, 512 * sizeof(uint32_t), s);
        hipLaunchKernelGGL(k_ns_bounds, dim3(tblocks(n, T)), dim3(T), 0, s, w.nskey_out, n, nlo, nhi);
        hipLaunchKernelGGL(k_ns_limit, dim3(ts.n_ns), dim3(64), 0, s, ts, b, w, out, nlo, nhi);
    }
    hipLaunchKernelGGL(k_tok_keys, dim3(tblocks(n, T)), dim3(T), 0, s, ts, b, w, out);
    hipError_t e = rocprim::radix_sort_pairs(w.sort64_tmp, w.sort64_bytes, w.key_in, w.key_out, w.idx_in, w.idx_out,
                                             n, 0u, 64u, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tok_heads, dim3(tblocks(n, T)), dim3(T), 0, s, w.key_out, n, w.head);
    e = rocprim::exclusive_scan(w.scan_tmp, w.scan_bytes, w.head, w.head_scan, 0u, (size_t)n,
                                rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    hipMemsetAsync(w.n_seg, 0, sizeof(uint32_t), s);
    hipLaunchKernelGGL(k_tok_segments, dim3(tblocks(n, T)), dim3(T), 0, s, w.key_out, w.head, w.head_scan, n,
                       w.seg_start, w.n_seg);
    hipLaunchKernelGGL(k_tok_decide, dim3(tblocks(n, TD_T)), dim3(TD_T), 0, s, ts, b, w, out);
    return hipGetLastError();
}

}  // namespace sf
