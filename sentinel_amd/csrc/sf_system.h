// sf_system.h — SystemRule (SystemRuleManager.checkSystem, SystemRuleManager.java:291-348)
// on the parallel pipeline: the safe-prefix planner (product code; host-
// compilable for the CPU tests in tests/hostsim).
//
// checkSystem reads the global ENTRY_NODE (Constants.java:66), which every
// earlier EntryType.IN event updates: every IN entry depends on every earlier
// one, across resources.  Instead of replaying the batch in one lane, the
// engine cuts it into sub-batches [p, q) whose system verdicts are all known
// before the sub-batch is decided:
//
//  - ENTRY_NODE is exact at p (all events before p are decided and reduced);
//  - a sub-batch stays inside one bucket window of the ENTRY_NODE second
//    array, so the valid buckets are fixed and only the current one grows;
//  - for every IN entry i of [p, lim) the planner bounds the ENTRY_NODE
//    statistics the reference would read at i over every outcome of the
//    undecided events in [p, i): pass count P in [P_p, P_p + sum of the
//    acquireCounts of IN entries not certainly blocked], thread count in
//    [T_p - certain live exits, + those entries], RT/success sums with the
//    certainly live exits (earlier batches, or entries decided before p) plus
//    any subset of the exits of entries inside [p, i);
//  - each of the five checks (qps, thread, rt, load/BBR, cpu; that order) is
//    then certainly passed, certainly failed, or unknown; an entry whose first
//    non-passed check is certainly failed is a certain SystemBlockException
//    with that reason, an entry passing all five a certain pass, anything else
//    ends the sub-batch (q = the first unknown IN entry).
//
// The event at p always has exact bounds, so every sub-batch holds at least
// one event.  The sub-batch is then decided by the ordinary per-resource
// pipeline with the certain blocks forced (an event flag), and ENTRY_NODE is
// reduced over it, exactly as for a batch without SystemRules.  A system
// block is invisible to its resource's controllers (only the block counters,
// which no controller reads), so the forced verdicts and the per-resource
// decisions compose exactly.
#pragma once
#include "sf_decide.h"

namespace sf {

// ENTRY_NODE at p, restricted to what the checks read inside the window.
struct SysBase {
    int64_t W;              // window start of the current bucket
    int64_t P;              // pass sum over the valid buckets (current included)
    int64_t T;              // curThreadNum
    int64_t RT, SU;         // rt / success sums over the valid buckets
    int64_t cur_succ;       // success of the current bucket (maxSuccess bound)
    int64_t other_max_succ; // max success over the other valid buckets (0 if none)
    int64_t min_rt;         // min of min_rt over the valid buckets (statisticMaxRt if none)
    int32_t valid_other;    // number of valid non-current buckets
    int32_t pad;
};

SF_HD SysBase sys_base(const Bucket* sec, int S, int wl, int interval, int64_t max_rt, int64_t threads, int64_t t) {
    SysBase b{};
    b.W = t - t % wl;
    const int idx = (int)((t / wl) % S);
    b.T = threads;
    b.min_rt = max_rt;
    for (int i = 0; i < S; i++) {
        const Bucket& k = sec[i];
        if (i == idx) {
            if (k.ws != b.W) continue;                       // reset at the first read of the window
            b.P = wadd(b.P, k.pass); b.RT = wadd(b.RT, k.rt); b.SU = wadd(b.SU, k.succ);
            b.cur_succ = k.succ;
            if (k.min_rt < b.min_rt) b.min_rt = k.min_rt;
            continue;
        }
        if (k.ws == WS_NONE || wsub(t, k.ws) > interval) continue;   // deprecated at every t of the window
        b.P = wadd(b.P, k.pass); b.RT = wadd(b.RT, k.rt); b.SU = wadd(b.SU, k.succ);
        if (k.succ > b.other_max_succ) b.other_max_succ = k.succ;
        if (k.min_rt < b.min_rt) b.min_rt = k.min_rt;
        b.valid_other++;
    }
    return b;
}

// Per-event prefix quantities (IN events only).  Exits: "certain" = live for
// sure (entry of an earlier batch, or decided before p and not blocked);
// "unc" = the entry is inside [p, i) (live iff it passes).
// Also the raw count of IN entries and of IN entries with acquireCount < 0
// (independent of any classification, so the "certainly fails" side of every
// check depends on these quantities only).
struct SysExitQ {
    int64_t xc, xc_c, xc_rt;     // certain live exits: count, sum acquireCount, sum rt
    int64_t xu, xu_c, xu_pos;    // uncertain exits: count, sum acquireCount, sum max(0, rt - M c)
    int64_t xu_bad;              // uncertain exits with acquireCount <= 0 (no rt bound)
    int64_t xc_min, xu_min;      // min rt
    int64_t ne, nneg;            // IN entries, IN entries with acquireCount < 0
    SF_HD void clear() { xc = xc_c = xc_rt = xu = xu_c = xu_pos = xu_bad = ne = nneg = 0; xc_min = xu_min = INT64_MAX; }
    SF_HD void add(const SysExitQ& o) {
        xc += o.xc; xc_c = wadd(xc_c, o.xc_c); xc_rt = wadd(xc_rt, o.xc_rt);
        xu += o.xu; xu_c = wadd(xu_c, o.xu_c); xu_pos = (o.xu_pos > INT64_MAX - xu_pos) ? INT64_MAX : xu_pos + o.xu_pos; xu_bad += o.xu_bad;
        if (o.xc_min < xc_min) xc_min = o.xc_min;
        if (o.xu_min < xu_min) xu_min = o.xu_min;
        ne += o.ne; nneg += o.nneg;
    }
};
struct SysEntQ {
    int64_t nb, nb_c, nb_neg;    // IN entries not certainly blocked: count, sum max(c, 0), count with c < 0
    SF_HD void clear() { nb = nb_c = nb_neg = 0; }
    SF_HD void add(const SysEntQ& o) { nb += o.nb; nb_c = wadd(nb_c, o.nb_c); nb_neg += o.nb_neg; }
};

enum : int { CK_PASS = 0, CK_FIRE = 1, CK_UNKNOWN = 2 };

// The five checks of one IN entry with acquireCount c, given the prefix
// bounds; returns -2 certain pass, -1 unknown, else the certain block reason.
// *any_fire: some check certainly fails (the entry is certainly blocked); it
// depends on the exit-side prefix x only, so the entry-side prefix (which
// counts the entries that are not certainly blocked) is a plain prefix sum.
SF_HD int sys_classify(const SysRule& r, const SysBase& b, int S, double interval_sec, const SysExitQ& x,
                       const SysEntQ& en, int32_t c, bool* any_fire) {
    int st[5];
    // qps: passQps + c > qps; passQps = P / intervalSec with P in [P_p, P_p + en.nb_c]
    // (an earlier entry with acquireCount < 0 could lower P: no certain failure then)
    {
        const double lo = (double)b.P / interval_sec, hi = (double)wadd(b.P, en.nb_c) / interval_sec;
        const bool fire = x.nneg == 0 && lo + c > r.qps, pass = !(hi + c > r.qps);
        st[0] = fire ? CK_FIRE : (pass ? CK_PASS : CK_UNKNOWN);
    }
    // thread: (int) curThreadNum > maxThread, T in [T_p - xc, T_p - xc + entries]
    const int64_t t_lo = b.T - x.xc, t_hi = b.T + en.nb - x.xc, t_top = b.T + x.ne - x.xc;
    const bool t_ok = t_lo >= INT32_MIN && t_top <= INT32_MAX;          // no int wrap: monotone
    {
        const bool fire = t_ok && t_lo > r.max_thread, pass = t_ok && !(t_hi > r.max_thread);
        st[1] = fire ? CK_FIRE : (pass ? CK_PASS : CK_UNKNOWN);
    }
    // rt: avgRt = RT * 1.0 / SU (0 when SU == 0) > maxRt
    const int64_t RTc = wadd(b.RT, x.xc_rt), SUc = wadd(b.SU, x.xc_c);
    if (r.max_rt == INT64_MAX) st[2] = CK_PASS;                         // unset: no double exceeds 2^63
    else if (x.xu == 0) {
        const double avg = SUc == 0 ? 0.0 : (double)RTc * 1.0 / (double)SUc;
        st[2] = avg > (double)r.max_rt ? CK_FIRE : CK_PASS;
    } else if (x.xu_bad == 0 && RTc >= 0 && SUc >= 0 && r.max_rt >= 0) {
        // every subset: RT - M*SU <= 0 exactly => avg <= M in exact reals => the rounded quotient too
        const __int128 worst = (__int128)RTc - (__int128)r.max_rt * (__int128)SUc + (__int128)x.xu_pos;
        st[2] = worst <= 0 ? CK_PASS : CK_UNKNOWN;
    } else {
        st[2] = CK_UNKNOWN;
    }
    // load: highestSystemLoad exceeded -> checkBbr(currentThread) (:342-348):
    // block iff th > 1 && th > maxSuccessQps * minRt / 1000, monotone in th, maxSuccess and minRt
    if (!(r.load_set && r.cur_load > r.highest_load)) st[3] = CK_PASS;
    else if (!t_ok || x.xu_bad) st[3] = CK_UNKNOWN;
    else {
        const int64_t cur_lo = wadd(b.cur_succ, x.xc_c), cur_hi = wadd(cur_lo, x.xu_c);
        int64_t ms_lo = cur_lo > b.other_max_succ ? cur_lo : b.other_max_succ;
        int64_t ms_hi = cur_hi > b.other_max_succ ? cur_hi : b.other_max_succ;
        ms_lo = ms_lo > 1 ? ms_lo : 1; ms_hi = ms_hi > 1 ? ms_hi : 1;
        int64_t mr_hi = b.min_rt < x.xc_min ? b.min_rt : x.xc_min;           // certain exits only
        int64_t mr_lo = mr_hi < x.xu_min ? mr_hi : x.xu_min;                  // every exit
        mr_hi = mr_hi > 1 ? mr_hi : 1; mr_lo = mr_lo > 1 ? mr_lo : 1;
        const double rhs_lo = (double)ms_lo * S / interval_sec * (double)mr_lo / 1000;
        const double rhs_hi = (double)ms_hi * S / interval_sec * (double)mr_hi / 1000;
        const int32_t th_lo = (int32_t)t_lo, th_hi = (int32_t)t_hi;
        const bool fire = th_lo > 1 && th_lo > rhs_hi;
        const bool pass = !(th_hi > 1 && th_hi > rhs_lo);
        st[3] = fire ? CK_FIRE : (pass ? CK_PASS : CK_UNKNOWN);
    }
    // cpu: a fixed input of the replay
    st[4] = (r.cpu_set && r.cur_cpu > r.highest_cpu) ? CK_FIRE : CK_PASS;
    *any_fire = st[0] == CK_FIRE || st[1] == CK_FIRE || st[2] == CK_FIRE || st[3] == CK_FIRE || st[4] == CK_FIRE;
    for (int k = 0; k < 5; k++) {
        if (st[k] == CK_PASS) continue;
        return st[k] == CK_FIRE ? k : -1;
    }
    return -2;
}

SF_HD bool v_blocked_any(uint8_t v) { return v_blocked(v); }

// Exit-side contribution of event i (submission index) when planning from p:
// ts / cnt / flags / eref / cts are the whole batch's arrays, vstatus its
// verdicts (decided before p).
SF_HD SysExitQ sys_exit_q(const int64_t* ts, const int32_t* cnt, const uint8_t* flags, const int64_t* eref,
                          const int64_t* cts, const uint8_t* vstatus, uint32_t p, uint32_t i, int64_t max_rt) {
    SysExitQ q;
    q.clear();
    const uint8_t f = flags[i];
    if (!(f & SF_EV_IN)) return q;
    const int32_t c = cnt[i];
    if (!(f & SF_EV_EXIT)) {
        q.ne = 1;
        q.nneg = c < 0 ? 1 : 0;
        return q;
    }
    const int64_t ref = eref ? eref[i] : -1;
    const int64_t t = ts[i];
    if (ref == EREF_DEAD) return q;                      // the entry was blocked earlier: nothing recorded
    if (ref < 0) {                                       // entry passed in an earlier batch
        const int64_t rt = t - (cts ? cts[i] : t);
        q.xc = 1; q.xc_c = c; q.xc_rt = rt; q.xc_min = rt;
    } else if (ref < (int64_t)p) {                       // entry decided before p
        if (!v_blocked_any(vstatus[ref])) {
            const int64_t rt = t - ts[ref];
            q.xc = 1; q.xc_c = c; q.xc_rt = rt; q.xc_min = rt;
        }
    } else if (flags[ref] & SF_EV_BLOCKED) {             // entry blocked before SystemSlot: nothing recorded
        return q;
    } else {                                             // entry inside the plan: live iff it passes
        const int64_t rt = t - ts[ref];
        q.xu = 1; q.xu_c = c; q.xu_min = rt;
        if (c <= 0) q.xu_bad = 1;
        else if (max_rt != INT64_MAX) {
            const __int128 d = (__int128)rt - (__int128)max_rt * c;
            q.xu_pos = d <= 0 ? 0 : (d > (__int128)INT64_MAX ? INT64_MAX : (int64_t)d);
        }
    }
    return q;
}

// Inert entries.  Between SystemSlot and FlowSlot sits ParamFlowSlot
// (ParamFlowSlot.checkFlow :82-103): an IN entry that passes SystemSlot is
// checked by its resource's ParamFlow rules in order.  When the first one is a
// QPS rule with the default behaviour whose value's token counter already
// exists, holds fewer tokens than the entry asks for, and is not due for a
// refill at the entry's time (ParamFlowChecker.passDefaultLocalCheck :139-219:
// without a refill the counter only falls, and a refill is due at no earlier
// event when none is due at this one), that rule certainly blocks the entry
// whatever the undecided events before it do.  Blocked by SystemSlot or by that
// rule, the entry then changes nothing but the block counters, which count it
// either way (StatisticSlot.entry :107-123), so it never adds to a pass or
// thread bound, and its own system verdict can be settled once the sub-batch is
// decided (sys_plan_fix).  param_inert tells, from the table as it is at p
// (the events before p are decided and no event at or after p has run).  The
// batch is this engine's (a sharded engine's own events under sf_sysx.h).
SF_HD bool param_inert(const DevState& st, const DevBatch& b, uint32_t i, int32_t acq, int64_t now) {
    if (!st.rdesc || !b.atag) return false;
    const uint32_t l = b.res[i] / st.shard_count;             // (this engine's events: res % shards == index)
    if (l >= st.R || (st.xmap && st.xmap[l] != XNONE)) return false;
    if (!(st.rdesc[l].flags & RD_PRULE)) return false;
    const DevParamRule& r = st.prules[st.prule_off[l]];
    if (r.grade != SF_GRADE_QPS || r.behavior == SF_BEHAVIOR_RATE_LIMITER || r.param_idx < 0) return false;
    const uint32_t na = b.nargs ? b.nargs[i] : b.arg_slots;
    if ((uint32_t)r.param_idx >= na || (uint32_t)r.param_idx >= b.arg_slots) return false;   // passCheck :53-56
    const uint32_t tag = b.atag[(size_t)r.param_idx * b.arg_stride + i];
    if (tag == SF_TAG_NULL || tag == SF_TAG_COLLECTION) return false;
    const uint64_t bits = b.abits[(size_t)r.param_idx * b.arg_stride + i];
    int64_t token_count = j_d2l(r.count);
    for (int k = 0; k < r.item_cnt; k++) {
        const DevHotItem& it = st.items[r.item_off + k];
        if (it.tag == tag && it.bits == bits) { token_count = it.count; break; }
    }
    if (token_count == 0) return true;                       // :156-158
    if (acq > wadd(token_count, r.burst)) return true;       // :160-163
    const ParamTable pt{st.ptab, st.pcap_mask, st.err, nullptr};
    const ParamSlot* sl = pt.find(pkey_hi(l, PK_RULE, 0u, tag), bits);
    if (!sl) return false;                                   // first sight passes
    if (wsub(now, sl->a) > wmul(r.duration_sec, 1000)) return false;   // a refill is due
    return sl->b - acq < 0;                                  // :196-215
}

// planner state in HBM (one per engine)
struct SysPlanDev {
    SysBase base;
    uint32_t wend, lim, first_unc, q;
    uint32_t n_inert, pad;         // IN entries planned SYS_INERT (read with q)
};

// Plan the events from p of batch b (whole batch, base 0): mask[i] for the
// IN entries of [p, q), plan->q.  vstatus: the batch's verdicts (before p).
// ibuf ([SYS_PLAN_CAP] scratch, or null): this engine decides the entries (not
// a merged node stream), so an unknown entry its first ParamFlow rule certainly
// blocks is planned SYS_INERT instead of ending the sub-batch (param_inert).
hipError_t sys_plan(const DevState& st, const DevBatch& b, const uint8_t* vstatus, uint8_t* mask, const SysRule& r,
                    const EntryNode* en, uint32_t p, SysPlanDev* plan, SysExitQ* pa, SysEntQ* pb, hipStream_t s,
                    uint8_t* ibuf = nullptr);
// After [p, q) is decided (verdicts in out, ENTRY_NODE still at p): the exact
// system verdict of every SYS_INERT entry of [p, q); a fired check turns its
// ParamFlow block into the SystemBlockException SystemSlot threw first.
hipError_t sys_plan_fix(const DevState& st, const DevBatch& b, const DevVerdicts& out, const uint8_t* mask,
                        const SysRule& r, uint32_t p, uint32_t q, SysPlanDev* plan, SysExitQ* pa, SysEntQ* pb,
                        hipStream_t s);
constexpr uint32_t SYS_PLAN_BLOCKS = 512;       // SP_NB (sf_system.hip): size of pa / pb
constexpr uint32_t SYS_PLAN_CAP = SYS_PLAN_BLOCKS * 4096;   // events per plan (size of ibuf)

}  // namespace sf
