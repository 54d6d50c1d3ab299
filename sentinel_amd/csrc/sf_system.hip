// sf_system.hip — the SystemRule safe-prefix planner on the GPU (product code).
//
// One sys_plan call plans the events from p: it finds the ENTRY_NODE bucket
// window of event p, bounds the ENTRY_NODE statistics at every IN entry of
// [p, min(window end, p + SP_CAP)) (sf_system.h), writes the forced system
// verdict of every entry whose five checks are all certain (mask: reason, or
// SYS_NONE for a certain pass) and returns q, the first IN entry whose
// outcome depends on undecided events (or the end of that range).
//
// The bounds are prefix sums in submission order: an exit-side prefix
// (independent of any classification) and an entry-side prefix (entries not
// certainly blocked, which depends on the exit side only).  Three passes of
// 4096-event blocks: A sums the exit side per block, B sums the entry side
// (classifying with A's prefix), C classifies every entry with both.  A
// block's prefix is the sum of the earlier blocks' totals (at most SP_NB
// partials, summed by the block itself: no separate scan launch).
#include "sf_sysx.h"

namespace sf {

constexpr int SP_T = 256, SP_RUN = 16, SP_BLK = SP_T * SP_RUN;   // 4096 events per block
constexpr uint32_t SP_NB = SYS_PLAN_BLOCKS;                       // blocks per plan
constexpr uint32_t SP_CAP = SP_NB * SP_BLK;                       // 2 Mi events per plan
static_assert(SP_CAP == SYS_PLAN_CAP, "sf_system.h SYS_PLAN_CAP");

struct SysPlanArgs {
    const int64_t* ts; const int32_t* cnt; const uint8_t* flags; const int64_t* eref; const int64_t* cts;
    const uint8_t* vstatus;                 // verdicts of the whole batch (events before p are decided)
    uint8_t* mask;                          // out: forced reason / SYS_NONE per IN entry of [p, q)
    uint32_t n, p;
    SysRule r;
    int32_t S, wl, interval;
    int64_t max_rt;                         // statisticMaxRt (empty-window minRt)
    double interval_sec;
    SysPlanDev* plan;
    SysExitQ* pa; SysEntQ* pb;              // [SP_NB] block totals
    // inert entries (sf_system.h param_inert): the engine's state and the
    // batch (args) to probe; exact: sys_plan_fix (every event of [p, lim)
    // decided, verdicts in vstatus / ostatus)
    bool inert, exact;
    DevState st;
    DevBatch b;
    uint8_t* ostatus; uint16_t* orule;
    uint8_t* ibuf;                          // [SP_CAP] param_inert of event p + k (k_sp_inert)
    uint32_t qcap;                          // limit the plan to qcap x the qps budget (k_sp_init; 0: off)
};

__global__ void k_sp_init(SysPlanArgs a, const EntryNode* en) {
    if (threadIdx.x != 0) return;
    SysPlanDev& pl = *a.plan;
    const int64_t t = a.ts[a.p];
    const int64_t end = t - t % a.wl + a.wl;
    uint32_t lo = a.p, hi = a.n;                 // first index with ts >= end
    while (lo < hi) { const uint32_t m = lo + (hi - lo) / 2; if (a.ts[m] >= end) hi = m; else lo = m + 1; }
    pl.wend = lo;
    pl.lim = min(lo, a.p + SP_CAP);
    pl.first_unc = pl.lim;
    pl.n_inert = 0;
    pl.base = sys_base(en->second, a.S, a.wl, a.interval, a.max_rt, en->threads, t);
    // A plan ends at its first entry whose qps check can go either way, which
    // comes within about B = qps * intervalSec - P passing entries of p while
    // the budget B is at least 1: plan only that far (2 B + 64 Ki events) instead
    // of the window's end.  Near a window's crossing B is small, and the
    // planner's passes over up to 2 Mi events were most of a round's cost.  A
    // plan cut short only costs one more round (every event before lim is
    // classified as before).
    if (a.qcap) {
        const double B = a.r.qps * a.interval_sec - (double)pl.base.P;
        // (B < 1: every entry with acquireCount >= 1 certainly fires until the
        // window ends -- a long round, not capped)
        if (B >= 1.0 && B < (double)SP_CAP) {
            const uint64_t cap = (uint64_t)a.p + (uint64_t)a.qcap * (uint64_t)B + 65536ull;
            if (cap < pl.lim) { pl.lim = (uint32_t)cap; pl.first_unc = pl.lim; }
        }
    }
}
// sys_plan_fix: the range is the decided sub-batch [p, q); base is still ENTRY_NODE at p
__global__ void k_sp_fix_init(SysPlanDev* pl) {
    if (threadIdx.x == 0) pl->lim = pl->q;
}

// block-wide inclusive scan of a struct with clear()/add() (Hillis-Steele in LDS)
template <class Q>
__device__ Q block_scan_incl(Q v, Q* lds) {
    const int t = threadIdx.x;
    lds[t] = v;
    __syncthreads();
    for (int d = 1; d < SP_T; d <<= 1) {
        Q o;
        o.clear();
        if (t >= d) o = lds[t - d];
        __syncthreads();
        if (t >= d) { v.add(o); lds[t] = v; }
        __syncthreads();
    }
    return v;
}

// sum of the totals of the blocks before block k
template <class Q>
__device__ Q block_prefix(const Q* tot, uint32_t k, Q* lds) {
    Q v;
    v.clear();
    for (uint32_t j = threadIdx.x; j < k; j += SP_T) v.add(tot[j]);
    v = block_scan_incl(v, lds);
    __shared__ Q res;
    if (threadIdx.x == SP_T - 1) res = v;
    __syncthreads();
    Q r = res;
    __syncthreads();
    return r;
}

__device__ __forceinline__ SysExitQ exit_q(const SysPlanArgs& a, uint32_t i) {
    // (exact: every entry before lim is decided)
    return sys_exit_q(a.ts, a.cnt, a.flags, a.eref, a.cts, a.vstatus, a.exact ? a.plan->lim : a.p, i, a.r.max_rt);
}
__device__ __forceinline__ bool inert_at(const SysPlanArgs& a, uint32_t i) {
    return a.inert && a.ibuf[i - a.p] != 0;
}
// one thread per event of [p, lim): the table probes of param_inert, all in
// flight at once (the passes read the flags)
__global__ void k_sp_inert(SysPlanArgs a) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x, i = a.p + k;
    if (i >= a.plan->lim) return;
    const uint8_t f = a.flags[i];
    const bool in = (f & SF_EV_IN) && !(f & (SF_EV_EXIT | SF_EV_BLOCKED));
    a.ibuf[k] = (in && param_inert(a.st, a.b, i, a.cnt[i], a.ts[i])) ? 1 : 0;
}
// IN entries that reach SystemSlot (an SF_EV_BLOCKED entry was blocked by
// AuthoritySlot before it: certainly blocked, no system verdict)
__device__ __forceinline__ bool in_entry(const SysPlanArgs& a, uint32_t i) {
    const uint8_t f = a.flags[i];
    return (f & SF_EV_IN) && !(f & (SF_EV_EXIT | SF_EV_BLOCKED));
}

__global__ void __launch_bounds__(SP_T) k_sp_a(SysPlanArgs a) {
    __shared__ SysExitQ lds[SP_T];
    const SysPlanDev& pl = *a.plan;
    const uint32_t b0 = a.p + blockIdx.x * SP_BLK;
    if (b0 >= pl.lim) return;
    const uint32_t r0 = b0 + threadIdx.x * SP_RUN, r1 = min(r0 + SP_RUN, pl.lim);
    SysExitQ v;
    v.clear();
    for (uint32_t i = r0; i < r1; i++) v.add(exit_q(a, i));
    v = block_scan_incl(v, lds);
    if (threadIdx.x == SP_T - 1) a.pa[blockIdx.x] = v;
}

// entry-side contribution of IN entry i with exit-side prefix x
__device__ __forceinline__ SysEntQ ent_q(const SysPlanArgs& a, const SysBase& base, const SysExitQ& x, uint32_t i) {
    SysEntQ e;
    e.clear();
    const int32_t c = a.cnt[i];
    SysEntQ none;
    none.clear();
    if (a.exact) {                                          // decided: the entries that passed, signed counts
        if (!v_blocked_any(a.vstatus[i])) { e.nb = 1; e.nb_c = c; }
        return e;
    }
    bool fire = false;
    sys_classify(a.r, base, a.S, a.interval_sec, x, none, c, &fire);
    if (!fire && inert_at(a, i)) fire = true;               // never passes either way
    if (!fire) { e.nb = 1; e.nb_c = c > 0 ? c : 0; e.nb_neg = c < 0 ? 1 : 0; }
    return e;
}

__global__ void __launch_bounds__(SP_T) k_sp_b(SysPlanArgs a) {
    __shared__ SysExitQ ldsx[SP_T];
    __shared__ SysEntQ ldse[SP_T];
    const SysPlanDev& pl = *a.plan;
    const uint32_t b0 = a.p + blockIdx.x * SP_BLK;
    if (b0 >= pl.lim) return;
    const SysBase base = pl.base;
    const uint32_t r0 = b0 + threadIdx.x * SP_RUN, r1 = min(r0 + SP_RUN, pl.lim);
    SysExitQ x = block_prefix(a.pa, blockIdx.x, ldsx);
    SysExitQ run;
    run.clear();
    for (uint32_t i = r0; i < r1; i++) run.add(exit_q(a, i));
    SysExitQ incl = block_scan_incl(run, ldsx);
    // exclusive prefix of this thread's run: block prefix + (inclusive - own)
    SysExitQ ex;
    ex.clear();
    if (threadIdx.x > 0) ex = ldsx[threadIdx.x - 1];
    __syncthreads();
    x.add(ex);
    (void)incl;
    SysEntQ e;
    e.clear();
    for (uint32_t i = r0; i < r1; i++) {
        if (in_entry(a, i)) e.add(ent_q(a, base, x, i));
        x.add(exit_q(a, i));
    }
    e = block_scan_incl(e, ldse);
    if (threadIdx.x == SP_T - 1) a.pb[blockIdx.x] = e;
}

__global__ void __launch_bounds__(SP_T) k_sp_c(SysPlanArgs a) {
    __shared__ SysExitQ ldsx[SP_T];
    __shared__ SysEntQ ldse[SP_T];
    SysPlanDev& pl = *a.plan;
    const uint32_t b0 = a.p + blockIdx.x * SP_BLK;
    if (b0 >= pl.lim) return;
    const SysBase base = pl.base;
    const uint32_t r0 = b0 + threadIdx.x * SP_RUN, r1 = min(r0 + SP_RUN, pl.lim);
    SysExitQ x = block_prefix(a.pa, blockIdx.x, ldsx);
    SysEntQ en = block_prefix(a.pb, blockIdx.x, ldse);
    SysExitQ run;
    run.clear();
    for (uint32_t i = r0; i < r1; i++) run.add(exit_q(a, i));
    block_scan_incl(run, ldsx);
    SysExitQ ex;
    ex.clear();
    if (threadIdx.x > 0) ex = ldsx[threadIdx.x - 1];
    __syncthreads();
    x.add(ex);
    // entry-side run partial, then its exclusive prefix
    SysExitQ xw = x;
    SysEntQ erun;
    erun.clear();
    for (uint32_t i = r0; i < r1; i++) {
        if (in_entry(a, i)) erun.add(ent_q(a, base, xw, i));
        xw.add(exit_q(a, i));
    }
    block_scan_incl(erun, ldse);
    SysEntQ eex;
    eex.clear();
    if (threadIdx.x > 0) eex = ldse[threadIdx.x - 1];
    __syncthreads();
    en.add(eex);
    // classify
    uint32_t n_inert = 0;
    for (uint32_t i = r0; i < r1; i++) {
        if (in_entry(a, i)) {
            const int32_t c = a.cnt[i];
            if (a.exact) {
                // sys_plan_fix: everything before i decided, so the bounds are one
                // value (the passes folded into the base); an inert entry's system
                // verdict, settled
                if (a.mask[i] == SYS_INERT) {
                    SysBase be = base;
                    be.P = wadd(base.P, en.nb_c); be.T = base.T + en.nb;
                    SysExitQ xx = x;
                    xx.nneg = 0;
                    SysEntQ none;
                    none.clear();
                    bool f2 = false;
                    const int res = sys_classify(a.r, be, a.S, a.interval_sec, xx, none, c, &f2);
                    if (res == -1 || a.ostatus[i] != SF_V_BLOCK_PARAM) *a.st.err = SF_ERR_INVALID;   // (cannot happen)
                    else if (res >= 0) {
                        a.ostatus[i] = SF_V_BLOCK_SYSTEM;
                        if (a.orule) a.orule[i] = (uint16_t)res;
                    }
                } else if (!v_blocked_any(a.vstatus[i])) {
                    en.nb++; en.nb_c = wadd(en.nb_c, c);
                }
                x.add(exit_q(a, i));
                continue;
            }
            bool fire = false;
            const int res = sys_classify(a.r, base, a.S, a.interval_sec, x, en, c, &fire);
            bool counts = !fire;
            if (res == -1) {
                if (!inert_at(a, i)) { atomicMin(&pl.first_unc, i); break; }
                a.mask[i] = SYS_INERT;                     // never passes: settled after the sub-batch
                n_inert++;
                counts = false;
            } else {
                a.mask[i] = res >= 0 ? (uint8_t)res : SYS_NONE;
                if (counts && inert_at(a, i)) counts = false;
            }
            if (counts) { en.nb++; en.nb_c = wadd(en.nb_c, c > 0 ? c : 0); en.nb_neg += c < 0 ? 1 : 0; }
        } else if (!a.exact && (a.flags[i] & (SF_EV_IN | SF_EV_EXIT | SF_EV_BLOCKED)) == (SF_EV_IN | SF_EV_BLOCKED)) {
            a.mask[i] = SYS_NONE;                          // blocked before SystemSlot: no system verdict
        }
        x.add(exit_q(a, i));
    }
    if (n_inert) atomicAdd(&pl.n_inert, n_inert);
}

__global__ void k_sp_done(SysPlanDev* pl) {
    if (threadIdx.x == 0) pl->q = min(pl->first_unc, pl->lim);
}

static SysPlanArgs plan_args(const DevState& st, const DevBatch& b, const uint8_t* vstatus, uint8_t* mask,
                             const SysRule& r, uint32_t p, SysPlanDev* plan, SysExitQ* pa, SysEntQ* pb,
                             uint8_t* ibuf) {
    SysPlanArgs a{};
    a.ts = b.ts; a.cnt = b.cnt; a.flags = b.flags; a.eref = b.eref; a.cts = b.cts;
    a.vstatus = vstatus; a.mask = mask; a.n = b.n; a.p = p; a.r = r;
    a.S = st.S; a.wl = st.wl; a.interval = st.interval; a.max_rt = st.max_rt;
    a.interval_sec = st.interval / 1000.0;
    a.plan = plan; a.pa = pa; a.pb = pb;
    a.st = st; a.b = b;
    a.ibuf = ibuf;
    return a;
}

hipError_t sys_plan(const DevState& st, const DevBatch& b, const uint8_t* vstatus, uint8_t* mask, const SysRule& r,
                    const EntryNode* en, uint32_t p, SysPlanDev* plan, SysExitQ* pa, SysEntQ* pb, hipStream_t s,
                    uint8_t* ibuf) {
    SysPlanArgs a = plan_args(st, b, vstatus, mask, r, p, plan, pa, pb, ibuf);
    a.inert = ibuf && st.n_prule != 0;
    static const uint32_t qcap = [] { const char* x = getenv("SF_PLAN_QCAP"); return x ? (uint32_t)atoi(x) : 2u; }();
    a.qcap = qcap;
    const uint32_t nb = (uint32_t)std::min<uint64_t>(SP_NB, ((uint64_t)(b.n - p) + SP_BLK - 1) / SP_BLK);
    hipLaunchKernelGGL(k_sp_init, dim3(1), dim3(64), 0, s, a, en);
    if (a.inert) hipLaunchKernelGGL(k_sp_inert, dim3(nb * (SP_BLK / 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_sp_a, dim3(nb), dim3(SP_T), 0, s, a);
    hipLaunchKernelGGL(k_sp_b, dim3(nb), dim3(SP_T), 0, s, a);
    hipLaunchKernelGGL(k_sp_c, dim3(nb), dim3(SP_T), 0, s, a);
    hipLaunchKernelGGL(k_sp_done, dim3(1), dim3(64), 0, s, plan);
    return hipGetLastError();
}

hipError_t sys_plan_fix(const DevState& st, const DevBatch& b, const DevVerdicts& out, const uint8_t* mask,
                        const SysRule& r, uint32_t p, uint32_t q, SysPlanDev* plan, SysExitQ* pa, SysEntQ* pb,
                        hipStream_t s) {
    if (q <= p) return hipSuccess;
    SysPlanArgs a = plan_args(st, b, out.status, (uint8_t*)mask, r, p, plan, pa, pb, nullptr);
    a.exact = true;
    a.ostatus = out.status; a.orule = out.rule;
    const uint32_t nb = (uint32_t)(((uint64_t)(q - p) + SP_BLK - 1) / SP_BLK);
    hipLaunchKernelGGL(k_sp_fix_init, dim3(1), dim3(64), 0, s, plan);
    hipLaunchKernelGGL(k_sp_a, dim3(nb), dim3(SP_T), 0, s, a);
    hipLaunchKernelGGL(k_sp_b, dim3(nb), dim3(SP_T), 0, s, a);
    hipLaunchKernelGGL(k_sp_c, dim3(nb), dim3(SP_T), 0, s, a);
    return hipGetLastError();
}

}  // namespace sf

// ------------------------------------------------------------------ the per-window exchange (sf_sysx.h)
namespace sf {

__device__ __forceinline__ bool sx_in_entry(const DevBatch& b, uint32_t i) {
    const uint8_t f = b.flags[i];
    return (f & SF_EV_IN) && !(f & (SF_EV_EXIT | SF_EV_BLOCKED));
}
__device__ __forceinline__ int64_t sx_cell(int64_t t, int64_t g) { return t >= 0 ? t / g : -((-t + g - 1) / g); }
// first i in [lo, hi) with seq[i] >= key
__device__ uint32_t sx_lower(const int64_t* seq, uint32_t lo, uint32_t hi, int64_t key) {
    while (lo < hi) { const uint32_t m = lo + (hi - lo) / 2; if (seq[m] >= key) hi = m; else lo = m + 1; }
    return lo;
}

__global__ void k_sx_header(SxArgs a, int64_t* out) {
    const uint32_t n = a.b.n;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[0] = n ? sx_cell(a.b.ts[0], a.g) : INT64_MAX;
        out[1] = n ? sx_cell(a.b.ts[n - 1], a.g) : INT64_MIN;
        out[2] = n ? a.seq[n - 1] + 1 : INT64_MIN;
        out[4] = n;
    }
    bool neg = false;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        neg |= sx_in_entry(a.b, i) && a.b.cnt[i] < 0;
    if (__ballot(neg) && (threadIdx.x & 63) == 0) atomicOr((unsigned long long*)&out[3], 1ull);
}
__global__ void k_sx_fill(int64_t* p, uint32_t n, int64_t v) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void k_sx_winfirst(SxArgs a, int64_t* out, uint32_t nw) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.b.n) return;
    const int64_t c = sx_cell(a.b.ts[i], a.g);
    if (i > 0 && sx_cell(a.b.ts[i - 1], a.g) == c) return;
    const int64_t k = c - a.c0;
    if (k >= 0 && k < (int64_t)nw) out[k] = a.seq[i];
}
hipError_t sx_header(const SxArgs& a, int64_t* out, hipStream_t s) {
    hipMemsetAsync(out, 0, 5 * sizeof(int64_t), s);
    const uint32_t nb = (uint32_t)std::min<uint64_t>(1024, ((uint64_t)a.b.n + 255) / 256 + 1);
    hipLaunchKernelGGL(k_sx_header, dim3(nb), dim3(256), 0, s, a, out);
    return hipGetLastError();
}
hipError_t sx_winfirst(const SxArgs& a, int64_t* out, uint32_t nw, hipStream_t s) {
    hipLaunchKernelGGL(k_sx_fill, dim3((nw + 255) / 256), dim3(256), 0, s, out, nw, INT64_MAX);
    if (a.b.n) hipLaunchKernelGGL(k_sx_winfirst, dim3((a.b.n + 255) / 256), dim3(256), 0, s, a, out, nw);
    return hipGetLastError();
}

__global__ void k_sx_clear(int64_t* msg, bool keep_delta) {
    const int i = threadIdx.x + blockIdx.x * blockDim.x;
    if (i < SX_DELTA) { if (!keep_delta) msg[i] = i == SXD_KEY ? -1 : 0; }
    else if (i < SXM_CMIN) msg[i] = 0;
    else if (i < SXM_CMAX) msg[i] = INT64_MAX;
    else if (i < SX_WORDS) msg[i] = INT64_MIN;
}
hipError_t sx_nodelta(int64_t* msg, hipStream_t s) {
    hipLaunchKernelGGL(k_sx_clear, dim3((SX_WORDS + 255) / 256), dim3(256), 0, s, msg, false);
    return hipGetLastError();
}

constexpr int SX_T = 256;
// One thread per contiguous run of the level's local events (sequence
// numbers increase, so a run's bin changes rarely): sums in registers, one set
// of atomics per (run, bin).
__global__ void __launch_bounds__(SX_T) k_sx_stats(SxArgs a, uint32_t lp, bool level0, int64_t lo, int64_t hi,
                                                   int64_t w) {
    __shared__ uint32_t rng[2];
    if (threadIdx.x == 0) {
        rng[0] = sx_lower(a.seq, lp, a.b.n, lo);
        rng[1] = sx_lower(a.seq, rng[0], a.b.n, hi);
    }
    __syncthreads();
    const uint32_t i0 = rng[0], i1 = rng[1];
    const uint64_t nth = (uint64_t)gridDim.x * SX_T, len = i1 - i0;
    const uint32_t per = (uint32_t)((len + nth - 1) / nth);
    const uint64_t t = (uint64_t)blockIdx.x * SX_T + threadIdx.x;
    const uint64_t r0 = (uint64_t)i0 + t * per;
    const uint32_t r1 = (uint32_t)std::min<uint64_t>(r0 + per, i1);
    int64_t bin = -1, u = 0, n = 0, cmn = INT64_MAX, cmx = INT64_MIN;
    auto flush = [&]() {
        if (bin < 0 || !n) return;
        atomicAdd((unsigned long long*)&a.msg[SXM_U + bin], (unsigned long long)u);
        atomicAdd((unsigned long long*)&a.msg[SXM_N + bin], (unsigned long long)n);
        atomicMin((long long*)&a.msg[SXM_CMIN + bin], (long long)cmn);
        atomicMax((long long*)&a.msg[SXM_CMAX + bin], (long long)cmx);
    };
    for (uint64_t i = r0; i < r1; i++) {
        if (!sx_in_entry(a.b, (uint32_t)i)) continue;
        const int32_t c = a.b.cnt[i];
        bool inert;
        if (level0) {
            inert = a.ibuf && param_inert(a.st, a.b, (uint32_t)i, c, a.b.ts[i]);
            if (a.ibuf) a.ibuf[i] = inert ? 1 : 0;
        } else {
            inert = a.ibuf && a.ibuf[i];
        }
        const int64_t k = (a.seq[i] - lo) / w;
        if (k != bin) { flush(); bin = k; u = 0; n = 0; cmn = INT64_MAX; cmx = INT64_MIN; }
        if (!inert && c > 0) u = sx_sat(u, c);
        n++;
        if (c < cmn) cmn = c;
        if (c > cmx) cmx = c;
    }
    flush();
}
hipError_t sx_stats(const SxArgs& a, const SxPlan& pl, uint32_t lp, bool level0, hipStream_t s) {
    hipLaunchKernelGGL(k_sx_clear, dim3((SX_WORDS + 255) / 256), dim3(256), 0, s, a.msg, level0);
    if (pl.done) return hipGetLastError();
    const uint64_t rest = a.b.n > lp ? a.b.n - lp : 0;
    const uint32_t nb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, (rest + 16 * SX_T - 1) / (16 * SX_T)));
    hipLaunchKernelGGL(k_sx_stats, dim3(nb), dim3(SX_T), 0, s, a, lp, level0, pl.lo, pl.hi, pl.w);
    return hipGetLastError();
}

// this rank's first event with seq >= q (batches whose sequence numbers are in HBM)
__global__ void k_sx_locate(SxArgs a, uint32_t lp, int64_t q, uint32_t* out) {
    if (threadIdx.x == 0) *out = sx_lower(a.seq, lp, a.b.n, q);
}
hipError_t sx_locate(const SxArgs& a, uint32_t lp, int64_t q, uint32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_sx_locate, dim3(1), dim3(64), 0, s, a, lp, q, out);
    return hipGetLastError();
}

__global__ void k_sx_mask(SxArgs a, uint8_t* mask, uint32_t lp, uint32_t lq, int64_t P) {
    const uint32_t i = lp + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= lq) return;
    mask[i] = sx_in_entry(a.b, i) ? sx_reason(a.r, P, a.interval_sec, a.b.cnt[i]) : SYS_NONE;
}
hipError_t sx_mask(const SxArgs& a, uint8_t* mask, uint32_t lp, uint32_t lq, int64_t P, hipStream_t s) {
    if (lq > lp) hipLaunchKernelGGL(k_sx_mask, dim3((lq - lp + 255) / 256), dim3(256), 0, s, a, mask, lp, lq, P);
    return hipGetLastError();
}

}  // namespace sf
