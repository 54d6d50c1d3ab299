// sf_xflow.h — the xflow walk: flow rules that check a node other than the
// resource's own ClusterNode (product code).
//
// FlowRuleChecker.selectNodeByRequesterAndStrategy (FlowRuleChecker.java:129-161)
// picks, per rule and per event, the node the rule's controller reads:
//   limitApp == origin (not "default"/"other")  DIRECT -> origin node   (Context.getOriginNode)
//   limitApp "default"                          DIRECT -> ClusterNode
//   limitApp "other", origin no rule names      DIRECT -> origin node   (FlowRuleManager.isOtherOrigin :132-148)
//   any of the three with RELATE -> ClusterNode of refResource (ClusterBuilderSlot.getClusterNode: null
//       until that resource's first entry), CHAIN -> the DefaultNode of (context, resource) when the
//       context name is refResource (selectReferenceNode :93-115); no node -> the rule passes.
// StatisticSlot then accounts every entry / exit on the DefaultNode (which
// forwards to the ClusterNode, DefaultNode.java:110-143) and on the origin
// node (StatisticSlot.java:64-178).
//
// Resources with such rules, and the resources their RELATE rules read, are
// grouped (connected by RELATE references) and each group's events are sorted
// into ONE segment (k_keys_packed maps every member to the group key), so one
// lane replays the group in submission order — a RELATE check reads the other
// resource's ClusterNode exactly as the events before it left it.  All node
// state of the walk lives in HBM (held in NodeWins while consecutive events
// use the same node, stored back on a switch); origin and context nodes sit in
// a pool indexed by an exact hash table.
// This is the rare path: the common DIRECT/"default" rules never come here,
// and neither do origin nodes no rule reads (ClusterBuilderSlot creates one
// for every entry with an origin): those are written after the verdicts by
// the origin-node pass (sf_origin.hip).
#pragma once
#include <vector>

#include "sf_decide.h"

namespace sf {

constexpr uint64_t PK_AUX = 3;
constexpr uint32_t AX_ORIGIN = 1, AX_CTX = 2;
enum : int { XS_NONE = 0, XS_CLUSTER = 1, XS_ORIGIN = 2, XS_CTX = 3, XS_REF = 4 };

// the four arrays of one statistic node (a resource row or a pool slot)
struct NodeRows { Bucket* sec; Borrow* bor; Bucket* min; int64_t* thr; };

SF_HD NodeRows cluster_rows(const DevState& st, uint32_t l) {
    return NodeRows{st.second + (size_t)l * st.S, st.borrow + (size_t)l * st.S, st.minute + (size_t)l * MINUTE,
                    st.threads + l};
}
SF_HD NodeRows aux_rows(const DevState& st, uint32_t k) {
    const AuxChunk& c = st.ax_chunks[k >> AX_SHIFT];
    const size_t i = k & (AX_CHUNK - 1);
    return NodeRows{c.sec + i * st.S, c.bor + i * st.S, c.min + i * MINUTE, c.thr + i};
}
template <int MAXS>
SF_HD void nw_load(NodeWin<MAXS>& nd, const DevState& st, const NodeRows& r) {
    nd.S = st.S; nd.wl = st.wl; nd.interval = st.interval; nd.max_rt = st.max_rt;
    nd.interval_sec = st.interval / 1000.0;
    for (int i = 0; i < MAXS; i++) {
        if (i < st.S) { nd.sec[i] = r.sec[i]; nd.bor[i] = r.bor[i]; }
        else { nd.sec[i] = fresh_bucket(WS_NONE, st.max_rt); nd.bor[i].ws = WS_NONE; nd.bor[i].pass = 0; }
    }
    nd.threads = *r.thr;
    nd.gmin = r.min; nd.mi = -1; nd.mdirty = 0; nd.mb = fresh_bucket(WS_NONE, st.max_rt);
    nd.c_ws = INT64_MIN; nd.c_idx = 0; nd.bdirty = 0; nd.m_ws = INT64_MIN; nd.pp_sec = INT64_MIN;
}
template <int MAXS>
SF_HD void nw_store(NodeWin<MAXS>& nd, const DevState& st, const NodeRows& r) {
    for (int i = 0; i < MAXS; i++)
        if (i < st.S) { r.sec[i] = nd.sec[i]; r.bor[i] = nd.bor[i]; }
    nd.min_flush();
    *r.thr = nd.threads;
}
// ClusterBuilderSlot creates a resource's ClusterNode at its first entry, which
// always rolls a second-window bucket (pass, block and the occupy path all do)
SF_HD bool node_created(const DevState& st, const NodeRows& r) {
    for (int i = 0; i < st.S; i++)
        if (r.sec[i].ws != WS_NONE) return true;
    return false;
}

// the pool slot of origin / context node (kind, id) of local resource l.  The
// sort phase's index pass (sf_origin.hip k_ox_index) has inserted every key a
// batch can ask for and the host has grown the pool to cover them, so on the
// device this is a find; the insert below serves the host build (tests/hostsim)
SF_HD uint32_t aux_get(const DevState& st, uint32_t l, uint32_t kind, uint32_t id) {
    ParamTable t{st.xtab, st.xcap_mask, st.err};
    const uint64_t hi = pkey_hi(l, PK_AUX, kind, 0);
    ParamSlot* s = t.find(hi, id);
    if (s) return (uint32_t)s->a;
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t k = atomicAdd(st.ax_count, 1u);
    if (k >= st.ax_cap) { atomicSub(st.ax_count, 1u); *st.err = SF_ERR_CAPACITY; return XNONE; }   // (saturates)
#else
    const uint32_t k = *st.ax_count;
    if (k >= st.ax_cap) { *st.err = SF_ERR_CAPACITY; return XNONE; }
    (*st.ax_count)++;
#endif
    s = t.insert(hi, id);
    if (!s) return XNONE;
    s->a = k;
    return k;
}

// FlowRuleManager.isOtherOrigin (FlowRuleManager.java:132-148) over the resource's rules
SF_HD bool other_origin(const DevState& st, uint32_t r0, uint32_t r1, uint32_t origin) {
    if (origin == SF_ORIGIN_NONE) return false;
    for (uint32_t k = r0; k < r1; k++)
        if (st.rules[k].limit_app == origin) return false;
    return true;
}
// FlowRuleChecker.selectReferenceNode (:93-115)
SF_HD int ref_select(const DevRule& r, uint32_t ctx) {
    if (r.ref == XNONE) return XS_NONE;                               // StringUtil.isEmpty(refResource)
    if (r.strategy == SF_STRATEGY_RELATE) return XS_REF;
    if (r.strategy == SF_STRATEGY_CHAIN) return ctx == r.ref ? XS_CTX : XS_NONE;
    return XS_NONE;
}
// FlowRuleChecker.selectNodeByRequesterAndStrategy (:129-161); filterOrigin :117-120
SF_HD int xflow_select(const DevState& st, const DevRule& r, uint32_t r0, uint32_t r1, uint32_t origin, uint32_t ctx) {
    const uint32_t app = r.limit_app;
    const bool direct = r.strategy == SF_STRATEGY_DIRECT;
    if (origin != SF_ORIGIN_NONE && app == origin && origin != SF_APP_DEFAULT && origin != SF_APP_OTHER)
        return direct ? XS_ORIGIN : ref_select(r, ctx);
    if (app == SF_APP_DEFAULT) return direct ? XS_CLUSTER : ref_select(r, ctx);
    if (app == SF_APP_OTHER && other_origin(st, r0, r1, origin)) return direct ? XS_ORIGIN : ref_select(r, ctx);
    return XS_NONE;
}

// One event j of a group segment starting at lo: SystemSlot (forced verdict)
// -> ParamFlowSlot -> FlowSlot with per-rule node selection -> DegradeSlot,
// then StatisticSlot's accounting.  cn / on / dn hold the nodes cl / oi / di
// (XNONE: none held); a switch stores the held node back first.
template <int MAXS>
SF_HD void xg_event(const DevState& st, const SegIO& io, const ParamTable& pt, uint32_t lo, uint32_t j,
                    NodeWin<MAXS>& cn, NodeWin<MAXS>& on, NodeWin<MAXS>& dn, uint32_t& cl, uint32_t& oi,
                    uint32_t& di) {
    const uint32_t i = io.perm[j];
    const uint32_t gres = io.ev_res[i];
    const uint32_t l = gres / io.shard_count;
    const uint32_t origin = io.ev_origin ? io.ev_origin[i] : SF_ORIGIN_NONE;
    const uint32_t ctx = io.ev_ctx ? io.ev_ctx[i] : 0u;
    const int64_t now = io.ts[j];
    const int32_t c = io.cnt[j];
    const uint8_t fl = io.flags[j];
    const uint32_t na = io.arg_slots ? (io.nargs ? io.nargs[j] : io.arg_slots) : 0;
    const uint32_t r0 = st.rule_off[l], r1 = st.rule_off[l + 1];
    // the origin node of every entry with an origin (ClusterBuilderSlot.java:107-110:
    // getOrCreateOriginNode whatever the rules); a context DefaultNode while a CHAIN
    // rule of the resource names the context (DESIGN.md §2 divergences)
    const bool want_on = origin != SF_ORIGIN_NONE;
    bool want_dn = false;
    for (uint32_t k = r0; k < r1; k++) {
        const DevRule& r = st.rules[k];
        if (r.strategy == SF_STRATEGY_CHAIN && r.ref == ctx) want_dn = true;
    }
    if (l != cl) {
        if (cl != XNONE) nw_store(cn, st, cluster_rows(st, cl));
        nw_load(cn, st, cluster_rows(st, l));
        cl = l;
    }
    {
        const uint32_t k = want_on ? aux_get(st, l, AX_ORIGIN, origin) : XNONE;
        if (k != oi) {
            if (oi != XNONE) nw_store(on, st, aux_rows(st, oi));
            if (k != XNONE) nw_load(on, st, aux_rows(st, k));
            oi = k;
        }
        const uint32_t m = want_dn ? aux_get(st, l, AX_CTX, ctx) : XNONE;
        if (m != di) {
            if (di != XNONE) nw_store(dn, st, aux_rows(st, di));
            if (m != XNONE) nw_load(dn, st, aux_rows(st, m));
            di = m;
        }
    }
    const uint32_t p0 = st.prule_off[l], p1 = st.prule_off[l + 1];
    const int nprules = (int)(p1 - p0);
    uint8_t pm_init = nprules ? st.pm_init[l] : 0;
    bool pm_exists = pm_init != 0;
    uint32_t cb0, cb1;
    breakers_of(st, l, &cb0, &cb1);
    uint8_t status; int64_t wait = 0; int rule_idx = 0;

    if (fl & SF_EV_EXIT) {                                  // StatisticSlot.exit :134-165
        int64_t ref = io.eref ? io.eref[j] : -1;
        bool blocked; int64_t create_ts;
        if (ref >= 0) {
            if (ref < (int64_t)lo || ref >= (int64_t)j || (io.flags[ref] & SF_EV_EXIT) ||
                io.ev_res[io.perm[ref]] != gres) {
                *st.err = SF_ERR_INVALID;
                ref = j;
            }
            blocked = ref == (int64_t)j ? true : v_blocked(io.v_status[ref]);
            create_ts = io.ts[ref];
        } else {
            blocked = ref == EREF_DEAD; create_ts = io.cts ? io.cts[j] : now;
        }
        if (!blocked) {
            const int64_t rt = now - create_ts;
            const bool er = (fl & SF_EV_ERROR) != 0;
            // recordCompleteFor(DefaultNode -> ClusterNode), recordCompleteFor(originNode) :150-151
            if (di != XNONE) { dn.add_rt_success(now, rt, c); dn.threads--; if (er) dn.add_exception(now, c); }
            cn.add_rt_success(now, rt, c); cn.threads--; if (er) cn.add_exception(now, c);
            if (oi != XNONE) { on.add_rt_success(now, rt, c); on.threads--; if (er) on.add_exception(now, c); }
            if (pm_exists) pm_thread_event(pt, l, pm_init, io, j, na, -1);
            for (uint32_t cb = cb0; cb < cb1; cb++) {
                sf_breaker_state bs = st.dg_state[cb];
                dg_complete(bs, st.dg_rules[cb], now, rt, er);
                st.dg_state[cb] = bs;
            }
            status = SF_V_EXIT;
        } else {
            status = SF_V_EXIT_IGNORED;
        }
    } else {
        bool blocked = false, prio_wait = false;
        status = SF_V_PASS;
        if (fl & EVF_SYSBLK) {    // SF_EV_BLOCKED (AuthoritySlot) or a planned SystemBlockException
            blocked = true; status = sysblk_status(fl); rule_idx = sysblk_rule(fl);
        }
        if (!blocked && nprules) {                          // ParamFlowSlot.checkFlow :82-103
            pm_exists = true;
            for (int k = 0; k < nprules && !blocked; k++) {
                DevParamRule& pr = st.prules[p0 + k];
                if (pr.param_idx < 0) {                     // applyRealParamIdx :56-66
                    if (-pr.param_idx <= (int)na) pr.param_idx = (int)na + pr.param_idx;
                    else pr.param_idx = -pr.param_idx;
                }
                if (pr.param_idx < 8) pm_init |= (uint8_t)(1u << pr.param_idx);
                if ((int)na <= pr.param_idx) continue;
                const uint32_t tg = io.atag[(size_t)pr.param_idx * io.n + j];
                const uint64_t bt = io.abits[(size_t)pr.param_idx * io.n + j];
                if (tg == SF_TAG_NULL) continue;
                int64_t w = 0;
                if (!param_pass_value(pt, l, k, pr, st.items, now, c, tg, bt, io, &w)) {
                    blocked = true; status = SF_V_BLOCK_PARAM; rule_idx = k;
                } else if (w > 0) {
                    wait += w;
                }
            }
        }
        if (!blocked) {                                     // FlowRuleChecker.checkFlow :44-59
            const bool prio = (fl & SF_EV_PRIO) != 0;
            for (uint32_t k = 0; k < r1 - r0; k++) {
                const DevRule& r = st.rules[r0 + k];
                if (r.always_pass) continue;                // cluster rule, no fallback (:184-193)
                const int sel = xflow_select(st, r, r0, r1, origin, ctx);
                if (sel == XS_NONE) continue;
                DevRuleState rs = st.rstate[r0 + k];
                int64_t w = 0; bool pw = false; int ok = 1;
                if (sel == XS_CLUSTER || (sel == XS_REF && r.ref == l)) {
                    ok = can_pass<MAXS>(r, rs, cn, now, c, prio, st.occupy_timeout, &w, &pw);
                } else if (sel == XS_ORIGIN) {
                    if (oi != XNONE) ok = can_pass<MAXS>(r, rs, on, now, c, prio, st.occupy_timeout, &w, &pw);
                } else if (sel == XS_CTX) {
                    if (di != XNONE) ok = can_pass<MAXS>(r, rs, dn, now, c, prio, st.occupy_timeout, &w, &pw);
                } else {                                    // RELATE: another resource of the group
                    const NodeRows rr = cluster_rows(st, r.ref);
                    if (node_created(st, rr)) {
                        NodeWin<MAXS> rn;
                        nw_load(rn, st, rr);
                        ok = can_pass<MAXS>(r, rs, rn, now, c, prio, st.occupy_timeout, &w, &pw);
                        nw_store(rn, st, rr);
                    }
                }
                st.rstate[r0 + k] = rs;
                if (pw) { prio_wait = true; wait += w; rule_idx = (int)k; break; }
                if (!ok) { blocked = true; status = SF_V_BLOCK_FLOW; rule_idx = (int)k; break; }
                wait += w;
            }
        }
        if (!blocked && !prio_wait && cb1 > cb0) {          // DegradeSlot.entry (DegradeSlot.java:42-61)
            const int k = dg_entry_check(st.dg_state, cb0, cb1, now);
            if (k >= 0) { blocked = true; status = SF_V_BLOCK_DEGRADE; rule_idx = k; }
        }
        // StatisticSlot.entry accounting :64-123 (DefaultNode -> ClusterNode, origin node)
        if (blocked) {
            if (di != XNONE) dn.add_block(now, c);
            cn.add_block(now, c);
            if (oi != XNONE) on.add_block(now, c);
        } else {
            if (di != XNONE) dn.threads++;
            cn.threads++;
            if (oi != XNONE) on.threads++;
            if (prio_wait) {
                status = SF_V_PRIORITY_WAIT;
            } else {
                if (di != XNONE) dn.add_pass(now, c);
                cn.add_pass(now, c);
                if (oi != XNONE) on.add_pass(now, c);
                status = wait > 0 ? SF_V_PASS_WAIT : SF_V_PASS;
            }
            if (pm_exists) pm_thread_event(pt, l, pm_init, io, j, na, +1);
        }
    }
    if (nprules) st.pm_init[l] = pm_init;
    io.v_status[j] = status;
    emit_verdict(io, j, status, (int32_t)wait, (uint16_t)rule_idx);
}

// One group segment [lo, hi) (events of several resources, submission order).
// The current resource's ClusterNode and the last origin / context node stay
// in registers while consecutive events use them (a group of one resource
// keeps its node for the whole segment); a switch stores the old node back
// first, so a RELATE read of another member always sees HBM up to date.
template <int MAXS>
SF_HD void decide_xgroup(const DevState& st, const SegIO& io, uint32_t lo, uint32_t hi) {
    const ParamTable pt{st.ptab, st.pcap_mask, st.err, st.pins};
    NodeWin<MAXS> cn, on, dn;
    uint32_t cl = XNONE, oi = XNONE, di = XNONE;          // nodes held in cn / on / dn
    for (uint32_t j = lo; j < hi; j++) xg_event<MAXS>(st, io, pt, lo, j, cn, on, dn, cl, oi, di);
    if (cl != XNONE) nw_store(cn, st, cluster_rows(st, cl));
    if (oi != XNONE) nw_store(on, st, aux_rows(st, oi));
    if (di != XNONE) nw_store(dn, st, aux_rows(st, di));
}

// ============================================================ wave walk eligibility
enum : uint8_t { XWF_ON = 1, XWF_THREAD = 2 };
constexpr uint32_t XW_MIN = 256;               // shorter xflow segments stay on k_decide_x's lanes
// a segment of resource l (its own group) with all-DIRECT rules, no ParamFlow
// rule and no circuit breaker, at least XW_MIN events: k_decide_xw
SF_HD bool xw_take(const DevState& st, uint32_t l, uint32_t len) {
    if (len < XW_MIN || !st.xw || !(st.xw[l] & XWF_ON)) return false;
    if (st.prule_off[l + 1] != st.prule_off[l]) return false;
    uint32_t b0, b1;
    breakers_of(st, l, &b0, &b1);
    return b0 == b1;
}

// ============================================================ groups (host side)
// xw[l] for the resources of one-member groups whose rules all check DIRECT
// (their ClusterNode or an origin node: no RELATE / CHAIN)
inline void build_xw(const DevRule* dr, const uint32_t* off, uint32_t R, const std::vector<uint32_t>& xmap,
                     std::vector<uint8_t>& xw) {
    xw.assign(R, 0);
    std::vector<uint32_t> members(R, 0);
    for (uint32_t l = 0; l < R; l++)
        if (xmap[l] != XNONE) members[xmap[l]]++;
    for (uint32_t l = 0; l < R; l++) {
        if (xmap[l] != l || members[l] != 1) continue;
        uint8_t f = XWF_ON;
        for (uint32_t k = off[l]; k < off[l + 1]; k++) {
            if (dr[k].strategy != SF_STRATEGY_DIRECT) { f = 0; break; }
            if (dr[k].grade == SF_GRADE_THREAD) f |= XWF_THREAD;
        }
        xw[l] = f;
    }
}

// A rule runs on the xflow walk unless it is limitApp "default" + DIRECT and
// not a cluster rule without fallback.
inline bool rule_is_ext(const DevRule& r) {
    return r.strategy != SF_STRATEGY_DIRECT || r.limit_app != SF_APP_DEFAULT || r.always_pass;
}
// xmap[l] = key of l's group (its smallest member; members: resources with an
// extended rule and the resources RELATE rules read, joined by RELATE), XNONE
// elsewhere.  Returns false (xmap untouched) when no rule is extended.
inline bool build_xmap(const DevRule* dr, const uint32_t* off, uint32_t R, std::vector<uint32_t>& xmap) {
    bool any = false;
    for (uint32_t k = 0; k < off[R] && !any; k++) any = rule_is_ext(dr[k]);
    if (!any) return false;
    std::vector<uint32_t> par(R, XNONE);
    auto find = [&](uint32_t x) {
        while (par[x] != x) { par[x] = par[par[x]]; x = par[x]; }
        return x;
    };
    auto join = [&](uint32_t a, uint32_t b) {
        a = find(a); b = find(b);
        if (a != b) { if (a < b) par[b] = a; else par[a] = b; }   // the root is the smallest member
    };
    for (uint32_t l = 0; l < R; l++)
        for (uint32_t k = off[l]; k < off[l + 1]; k++) {
            const DevRule& r = dr[k];
            if (!rule_is_ext(r)) continue;
            if (par[l] == XNONE) par[l] = l;
            if (r.strategy == SF_STRATEGY_RELATE && r.ref != XNONE && r.ref < R) {
                if (par[r.ref] == XNONE) par[r.ref] = r.ref;
                join(l, r.ref);
            }
        }
    xmap.assign(R, XNONE);
    for (uint32_t l = 0; l < R; l++)
        if (par[l] != XNONE) xmap[l] = find(l);
    return true;
}

}  // namespace sf
