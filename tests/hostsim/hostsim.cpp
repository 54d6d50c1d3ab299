// TEST-ONLY host build of the engine's decision code (sf_decide.h, sf_heavy.h).
//
// Runs the exact device algorithms on the CPU (heavy teams of size 1) with the
// same routing as the HIP pipeline, so the CPU suite can check the kernel
// logic against the oracle.  Never loaded by the product: libsentinel_flow.so
// has no path to it, and sf_create fails without a gfx950 device.
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "../../sentinel_amd/csrc/sf_heavy.h"
#include "../../sentinel_amd/csrc/sf_xflow.h"
#include "../../sentinel_amd/csrc/sf_sysx.h"

using namespace sf;

struct hs_engine {
    sf_config cfg;
    DevState st{};
    std::vector<Bucket> second, minute;
    std::vector<Borrow> borrow;
    std::vector<int64_t> threads;
    std::vector<uint32_t> rule_off, prule_off;
    std::vector<DevRule> rules;
    std::vector<DevRuleState> rstate;
    std::vector<uint32_t> flow_pos;
    std::vector<DevParamRule> prules;
    std::vector<DevHotItem> items;
    std::vector<uint8_t> pm_init;
    std::vector<RDesc> rdesc;
    int32_t prio_seen = 0;                         // (k_segs: any prioritized entry submitted so far)
    std::vector<ParamSlot> ptab;
    std::vector<uint32_t> dg_rr, dg_off;
    std::vector<DevBreakerRule> dg_rules;
    std::vector<sf_breaker_state> dg_state;
    std::vector<uint32_t> dg_pos;                  // load order -> position
    // xflow walk: group keys, origin / context node pool and its index table
    std::vector<uint32_t> xmap;
    std::vector<ParamSlot> xtab;
    std::vector<Bucket> ax_second, ax_minute;
    std::vector<Borrow> ax_borrow;
    std::vector<int64_t> ax_threads;
    std::vector<AuxChunk> ax_chunks;          // the device's chunk directory over the contiguous host pool
    uint32_t ax_count = 0;
    int32_t err = 0;
    uint32_t R;
    uint32_t heavy_min;
    uint64_t n_heavy_segments = 0, n_heavy_item_segments = 0, mode_count[8] = {};
    void refresh(bool rules_changed = true) {
        st.second = second.data(); st.borrow = borrow.data(); st.minute = minute.data();
        st.threads = threads.data(); st.rule_off = rule_off.data(); st.rules = rules.data();
        st.rstate = rstate.data(); st.prule_off = prule_off.data(); st.prules = prules.data();
        st.items = items.data(); st.pm_init = pm_init.data(); st.ptab = ptab.data();
        st.pcap_mask = ptab.size() - 1; st.err = &err;
        st.dg_n = dg_off.empty() ? 0 : (uint32_t)dg_off.size() - 1;
        st.dg_rr_of = st.dg_n ? dg_rr.data() : nullptr;
        st.dg_off = dg_off.data(); st.dg_rules = dg_rules.data(); st.dg_state = dg_state.data();
        st.xmap = xmap.empty() ? nullptr : xmap.data();
        st.xtab = xtab.data(); st.xcap_mask = xtab.empty() ? 0 : xtab.size() - 1;
        ax_chunks.clear();
        const size_t S_ = st.S;
        for (size_t c = 0; c * AX_CHUNK < ax_threads.size(); c++)
            ax_chunks.push_back(AuxChunk{ax_second.data() + c * AX_CHUNK * S_, ax_borrow.data() + c * AX_CHUNK * S_,
                                         ax_minute.data() + c * AX_CHUNK * MINUTE, ax_threads.data() + c * AX_CHUNK});
        st.ax_chunks = ax_chunks.data(); st.ax_count = &ax_count; st.ax_cap = (uint32_t)ax_threads.size();
        st.prio_seen = &prio_seen;
        if (rules_changed) {
            rdesc.resize(R);
            st.rdesc = rdesc.data();
            for (uint32_t r = 0; r < R; r++) rdesc[r] = make_rdesc(st, r);
        }
    }
};

extern "C" {

hs_engine* hs_create(const sf_config* c) {
    hs_engine* e = new hs_engine();
    e->cfg = *c;
    e->R = c->max_resources;
    e->heavy_min = c->heavy_min_events ? c->heavy_min_events : 512;
    size_t R = e->R, S = c->sample_count;
    e->second.assign(R * S, fresh_bucket(WS_NONE, c->statistic_max_rt));
    e->borrow.assign(R * S, Borrow{WS_NONE, 0});
    e->minute.assign(R * MINUTE, fresh_bucket(WS_NONE, c->statistic_max_rt));
    e->threads.assign(R, 0);
    e->rule_off.assign(R + 1, 0); e->prule_off.assign(R + 1, 0);
    e->rules.resize(1); e->rstate.resize(1); e->prules.resize(1); e->items.resize(1);
    e->pm_init.assign(R, 0);
    size_t pcap = 16; while (pcap < c->param_capacity) pcap <<= 1;
    e->ptab.assign(pcap, ParamSlot{0, 0, 0, 0});
    DevState& st = e->st;
    st.S = c->sample_count; st.wl = c->interval_ms / c->sample_count; st.interval = c->interval_ms;
    st.occupy_timeout = c->occupy_timeout_ms; st.max_rt = c->statistic_max_rt; st.R = e->R;
    st.shard_count = c->shard_count;
    e->refresh();
    return e;
}
void hs_destroy(hs_engine* e) { delete e; }

static bool local_of(hs_engine* e, uint32_t res, uint32_t* l) {
    if (res % e->cfg.shard_count != e->cfg.shard_index) return false;
    *l = res / e->cfg.shard_count; return *l < e->R;
}

// the origin / context node pool (lives as long as the engine)
static void ensure_pool(hs_engine* e) {
    if (!e->ax_threads.empty()) return;
    size_t cap = e->cfg.aux_capacity ? e->cfg.aux_capacity : 65536;
    const size_t S = e->cfg.sample_count;
    cap = (cap + AX_CHUNK - 1) / AX_CHUNK * AX_CHUNK;          // whole chunks (sf_internal.h AuxChunk)
    size_t tcap = 16; while (tcap < 2 * cap) tcap <<= 1;
    e->xtab.assign(tcap, ParamSlot{0, 0, 0, 0});
    e->ax_second.assign(cap * S, fresh_bucket(WS_NONE, e->cfg.statistic_max_rt));
    e->ax_borrow.assign(cap * S, Borrow{WS_NONE, 0});
    e->ax_minute.assign(cap * MINUTE, fresh_bucket(WS_NONE, e->cfg.statistic_max_rt));
    e->ax_threads.assign(cap, 0);
}

int hs_load_flow_rules(hs_engine* e, const sf_flow_rule* rules, uint32_t n) {
    std::vector<uint32_t> counts(e->R + 1, 0), loc, refl;
    std::vector<const sf_flow_rule*> valid;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t l; if (!local_of(e, rules[i].resource, &l)) return SF_ERR_INVALID;
        if (!valid_flow_rule(rules[i])) continue;
        uint32_t ref = XNONE;
        if (rules[i].strategy == SF_STRATEGY_RELATE && rules[i].ref_resource != SF_REF_NONE) {
            if (rules[i].ref_resource % e->cfg.shard_count != e->cfg.shard_index) return SF_ERR_UNSUPPORTED;
            if (rules[i].ref_resource / e->cfg.shard_count < e->R) ref = rules[i].ref_resource / e->cfg.shard_count;
        }
        if (++counts[l] > SF_MAX_RULES_PER_RESOURCE) return SF_ERR_UNSUPPORTED;
        valid.push_back(&rules[i]); loc.push_back(l); refl.push_back(ref);
    }
    for (uint32_t r = 0; r < e->R; r++) e->rule_off[r + 1] = e->rule_off[r] + counts[r];
    std::vector<uint32_t> fill(e->rule_off.begin(), e->rule_off.end() - 1);
    e->rules.assign(std::max<size_t>(1, valid.size()), DevRule{});
    e->rstate.assign(std::max<size_t>(1, valid.size()), fresh_rule_state());
    e->flow_pos.assign(valid.size(), 0);
    for (size_t k = 0; k < valid.size(); k++) {
        uint32_t pos = fill[loc[k]]++;
        e->flow_pos[k] = pos;
        e->rules[pos] = make_dev_rule(*valid[k], e->cfg.cold_factor, (int)k, refl[k]);
    }
    std::vector<uint32_t> xm;
    if (build_xmap(e->rules.data(), e->rule_off.data(), e->R, xm)) {
        e->xmap = xm;
        ensure_pool(e);
    } else {
        e->xmap.clear();
    }
    e->refresh();
    return SF_OK;
}

int hs_load_param_rules(hs_engine* e, const sf_param_rule* rules, uint32_t n, const sf_hot_item* items, uint32_t ni) {
    std::vector<uint32_t> counts(e->R + 1, 0), loc(n);
    for (uint32_t i = 0; i < n; i++) { if (!local_of(e, rules[i].resource, &loc[i])) return SF_ERR_INVALID; counts[loc[i]]++; }
    for (uint32_t r = 0; r < e->R; r++) e->prule_off[r + 1] = e->prule_off[r] + counts[r];
    std::vector<uint32_t> fill(e->prule_off.begin(), e->prule_off.end() - 1);
    e->prules.assign(std::max<uint32_t>(1, n), DevParamRule{});
    for (uint32_t i = 0; i < n; i++) e->prules[fill[loc[i]]++] = make_dev_param_rule(rules[i], (int)i);
    e->items.assign(std::max<uint32_t>(1, ni), DevHotItem{});
    for (uint32_t i = 0; i < ni; i++) { e->items[i].bits = items[i].bits; e->items[i].count = items[i].count; e->items[i].tag = items[i].tag; }
    std::fill(e->pm_init.begin(), e->pm_init.end(), 0);
    std::fill(e->ptab.begin(), e->ptab.end(), ParamSlot{0, 0, 0, 0});
    e->refresh();
    return SF_OK;
}

// DegradeSlot rules (fresh breakers; list order per resource)
int hs_load_degrade_rules(hs_engine* e, const sf_degrade_rule* rules, uint32_t n, uint32_t* n_loaded) {
    std::vector<uint32_t> loc, valid;
    for (uint32_t i = 0; i < n; i++) {
        if (!dg_valid(rules[i])) continue;
        uint32_t l; if (!local_of(e, rules[i].resource, &l)) return SF_ERR_INVALID;
        valid.push_back(i); loc.push_back(l);
    }
    const uint32_t nv = (uint32_t)valid.size();
    std::vector<uint32_t> order(nv);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return loc[a] < loc[b]; });
    e->dg_rr.assign(e->R, 0); e->dg_off.clear(); e->dg_rules.assign(std::max<uint32_t>(1, nv), DevBreakerRule{});
    e->dg_state.assign(std::max<uint32_t>(1, nv), sf_breaker_state{SF_CB_CLOSED, 0, 0, DG_WS_NONE, 0, 0});
    e->dg_pos.assign(nv, 0);
    for (uint32_t p = 0; p < nv; p++) {
        const uint32_t v = order[p];
        if (p == 0 || loc[order[p - 1]] != loc[v]) e->dg_off.push_back(p);
        e->dg_rules[p] = make_dev_breaker_rule(rules[valid[v]]);
        e->dg_pos[v] = p;
    }
    const uint32_t nr = (uint32_t)e->dg_off.size();
    if (nv) e->dg_off.push_back(nv);
    for (auto& x : e->dg_rr) x = nr;
    for (uint32_t k = 0; k < nr; k++) e->dg_rr[loc[order[e->dg_off[k]]]] = k;
    e->refresh();
    if (n_loaded) *n_loaded = nv;
    return SF_OK;
}
int hs_read_breaker(hs_engine* e, uint32_t k, sf_breaker_state* out) {
    if (k >= e->dg_pos.size()) return SF_ERR_INVALID;
    *out = e->dg_state[e->dg_pos[k]];
    if (out->window_start == DG_WS_NONE) out->window_start = SF_WS_ABSENT;
    return SF_OK;
}

int hs_submit(hs_engine* e, const sf_event_batch* in, sf_verdicts* out) {
    if (in->origin) { ensure_pool(e); e->refresh(false); }        // origin nodes of every entry with an origin
    const uint32_t n = in->n;
    e->err = 0;
    std::vector<uint32_t> key(n), perm(n), inv(n);
    for (uint32_t i = 0; i < n; i++) {
        if (!local_of(e, in->res_id[i], &key[i])) return SF_ERR_INVALID;
        if (!e->xmap.empty() && e->xmap[key[i]] != XNONE) key[i] = e->xmap[key[i]];   // xflow group segment
    }
    std::iota(perm.begin(), perm.end(), 0u);
    std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
    std::vector<int64_t> ts(n), eref(n, -1), cts(n, 0), pcg(n);
    std::vector<int32_t> cnt(n);
    std::vector<uint8_t> fl(n), nargs(n), atag((size_t)n * in->arg_slots), vs(n);
    std::vector<uint64_t> abits((size_t)n * in->arg_slots);
    std::vector<int32_t> vw(n); std::vector<uint16_t> vr(n);
    for (uint32_t j = 0; j < n; j++) {
        uint32_t i = perm[j]; inv[i] = j;
        ts[j] = in->ts_ms[i]; cnt[j] = in->count[i];
        fl[j] = in->flags[i] & 0x0Fu;                            // k_keys_packed's internal flags
        if ((in->flags[i] & (SF_EV_BLOCKED | SF_EV_EXIT)) == SF_EV_BLOCKED)
            fl[j] |= EVF_SYSBLK | (uint8_t)(SYSR_OTHER << EVF_SYSREASON_SHIFT);
        if (in->n_args) nargs[j] = in->n_args[i];
        for (uint32_t a = 0; a < in->arg_slots; a++) {
            atag[(size_t)a * n + j] = in->arg_tag[(size_t)a * n + i];
            abits[(size_t)a * n + j] = atag[(size_t)a * n + j] == SF_TAG_COLLECTION ? (uint64_t)a * n + i
                                                                                  : in->arg_bits[(size_t)a * n + i];
        }
        pcg[j] = (j ? pcg[j - 1] : 0) + ((fl[j] & (SF_EV_EXIT | EVF_SYSBLK)) ? 0 : (int64_t)cnt[j]);
    }
    if (in->entry_ref)
        for (uint32_t j = 0; j < n; j++) {
            int64_t r = in->entry_ref[perm[j]];
            eref[j] = r >= 0 ? (int64_t)inv[r] : (r == EREF_DEAD ? EREF_DEAD : (int64_t)-1);
            cts[j] = in->create_ts ? in->create_ts[perm[j]] : 0;
        }
    SegIO io{ts.data(), cnt.data(), fl.data(), in->entry_ref ? eref.data() : nullptr,
             in->entry_ref ? cts.data() : nullptr, in->arg_slots, in->n_args ? nargs.data() : nullptr,
             atag.data(), abits.data(), n, in->arg_elem_off, in->elem_tag, in->elem_bits,
             vs.data(), vw.data(), vr.data()};
    // light / generic segments emit their verdicts through the identity permutation
    // into the sorted-order arrays (the final loop below scatters them)
    std::vector<uint32_t> ident(n);
    std::iota(ident.begin(), ident.end(), 0u);
    io.perm = ident.data(); io.o_status = vs.data(); io.o_wait = vw.data(); io.o_rule = vr.data();
    std::vector<uint32_t> sres(n), sorigin(n), sctx(n);          // xflow walk: sorted order (perm is the identity)
    for (uint32_t j = 0; j < n; j++) {
        sres[j] = in->res_id[perm[j]];
        sorigin[j] = in->origin ? in->origin[perm[j]] : SF_ORIGIN_NONE;
        sctx[j] = in->context ? in->context[perm[j]] : 0u;
    }
    io.ev_res = sres.data(); io.ev_origin = sorigin.data(); io.ev_ctx = sctx.data(); io.shard_count = e->cfg.shard_count;
    // segments + routing (k_segments / k_classify)
    std::vector<uint32_t> seg_start, seg_res, segflag;
    for (uint32_t j = 0; j < n; j++) {
        if (j == 0 || key[perm[j]] != key[perm[j - 1]]) { seg_start.push_back(j); seg_res.push_back(key[perm[j]]); segflag.push_back(0); }
        if (in->origin && in->origin[perm[j]] != SF_ORIGIN_NONE) segflag.back() |= SEGF_ORIGIN;
        if (!(fl[j] & SF_EV_EXIT) && ((fl[j] & (SF_EV_PRIO | EVF_SYSBLK)) || cnt[j] <= 0)) {
            if (fl[j] & SF_EV_PRIO) e->prio_seen = 1;           // (sticky, as k_segs sets it)
            segflag.back() |= ((fl[j] & SF_EV_PRIO) ? SEGF_PRIO : 0u) | (cnt[j] <= 0 ? SEGF_NONPOS : 0u) |
                              ((fl[j] & EVF_SYSBLK) ? SEGF_SYS : 0u);
        }
    }
    const uint32_t ns = (uint32_t)seg_start.size();
    seg_start.push_back(n);
    std::vector<uint8_t> mode(ns);
    std::vector<uint32_t> hwb(ns), secb(ns), nhw(ns), nsec(ns);
    std::vector<int64_t> hw0(ns), sec0(ns);
    std::vector<Acc> acc_hw, acc_sec;
    for (uint32_t s = 0; s < ns; s++) {
        uint32_t lo = seg_start[s], hi = seg_start[s + 1];
        if ((!e->xmap.empty() && e->xmap[seg_res[s]] != XNONE) || (segflag[s] & SEGF_ORIGIN)) { mode[s] = SM_XFLOW; continue; }
        if (hi - lo <= e->heavy_min) { mode[s] = SM_LIGHT; continue; }
        e->n_heavy_segments++;
        mode[s] = heavy_mode(e->st, seg_res[s], segflag[s], ts[lo]);
        if (mode[s] == SM_PARAM) mode[s] = SM_GENERIC;          // (the wavefront param path is GPU-only)
        e->mode_count[mode[s] & 7]++;
        if (mode[s] != SM_GENERIC) {
            e->n_heavy_item_segments++;
            hw0[s] = ts[lo] / e->st.wl; sec0[s] = ts[lo] / 1000;
            nhw[s] = (uint32_t)(ts[hi - 1] / e->st.wl - hw0[s] + 1); nsec[s] = (uint32_t)(ts[hi - 1] / 1000 - sec0[s] + 1);
            hwb[s] = (uint32_t)acc_hw.size(); secb[s] = (uint32_t)acc_sec.size();
            Acc z{}; z.min_rt = INT64_MAX;
            acc_hw.resize(acc_hw.size() + nhw[s], z); acc_sec.resize(acc_sec.size() + nsec[s], z);
        }
    }
    std::vector<unsigned long long> passbits(n / 64 + 2, 0ull);
    HeavyCtx hc{seg_start.data(), seg_res.data(), mode.data(), nullptr, nullptr, 0u, pcg.data(),
                acc_hw.data(), acc_sec.data(), hwb.data(), secb.data(), hw0.data(), sec0.data(),
                nullptr, passbits.data()};
    for (uint32_t s = 0; s < ns; s++) {
        uint32_t lo = seg_start[s], hi = seg_start[s + 1], res = seg_res[s];
        Team tm;
        switch (mode[s]) {
        case SM_QPS:
        case SM_WARM:
            if (e->st.S <= 2) heavy_qps<2>(tm, e->st, io, hc, s, res, lo, hi, mode[s] == SM_WARM);
            else heavy_qps<SF_MAX_SAMPLE_COUNT>(tm, e->st, io, hc, s, res, lo, hi, mode[s] == SM_WARM);
            break;
        case SM_RL: heavy_rl(tm, e->st, io, hc, s, res, lo, hi); break;
        case SM_THREAD: heavy_thread(tm, e->st, io, hc, s, res, lo, hi, nullptr, nullptr); break;
        case SM_NORULE: break;                    // every entry passes (fill)
        case SM_XFLOW:
            if (e->st.S <= 2) decide_xgroup<2>(e->st, io, lo, hi);
            else decide_xgroup<SF_MAX_SAMPLE_COUNT>(e->st, io, lo, hi);
            break;
        default: {
            // the lean QPS walk of short segments (k_classify's SM_LIGHTQ routing)
            if (mode[s] == SM_LIGHT && qps_lean(e->st, res, segflag[s])) {
                if (e->st.S <= 2) decide_qps_segment<2>(e->st, io, res, lo, hi);
                else decide_qps_segment<SF_MAX_SAMPLE_COUNT>(e->st, io, res, lo, hi);
                break;
            }
            if (e->st.S <= 2) decide_segment<2>(e->st, io, res, lo, hi);
            else decide_segment<SF_MAX_SAMPLE_COUNT>(e->st, io, res, lo, hi);
        }
        }
    }
    // k_heavy_fill
    for (uint32_t s = 0; s < ns; s++) {
        if (mode[s] < SM_QPS || mode[s] == SM_XFLOW) continue;
        for (uint32_t j = seg_start[s]; j < seg_start[s + 1]; j++) {
            EvContrib c = heavy_event(hc, io, seg_start[s], mode[s], j);
            vs[j] = c.status; vw[j] = c.wait; vr[j] = 0;
            if (!c.touch) continue;
            for (int t = 0; t < 2; t++) {
                Acc& a = t == 0 ? acc_hw[hwb[s] + (ts[j] / e->st.wl - hw0[s])] : acc_sec[secb[s] + (ts[j] / 1000 - sec0[s])];
                a.n_touch++;
                if (c.live_exit) {
                    a.succ += c.c; a.rt += c.rt; a.n_exit++; if (c.err) a.exc += c.c;
                    if (c.rt < a.min_rt) a.min_rt = c.rt;
                } else if (c.passed) { a.pass += c.c; a.n_pass++; }
                else a.block += c.c;
            }
        }
    }
    // k_heavy_apply
    for (uint32_t s = 0; s < ns; s++)
        if (mode[s] >= SM_QPS && mode[s] != SM_XFLOW) heavy_apply(e->st, hc, s, seg_res[s], nhw[s], nsec[s]);
    for (uint32_t j = 0; j < n; j++) {
        uint32_t i = perm[j];
        ((uint8_t*)out->status)[i] = vs[j];
        if (out->wait_ms) out->wait_ms[i] = vw[j];
        if (out->rule_idx) out->rule_idx[i] = vr[j];
    }
    return e->err;
}

void hs_heavy_stats(hs_engine* e, uint64_t* heavy, uint64_t* items) { *heavy = e->n_heavy_segments; *items = e->n_heavy_item_segments; }
void hs_mode_counts(hs_engine* e, uint64_t* out8) { for (int i = 0; i < 8; i++) out8[i] = e->mode_count[i]; }

int hs_read_node(hs_engine* e, uint32_t res, sf_node_state* out) {
    uint32_t l; if (!local_of(e, res, &l)) return SF_ERR_INVALID;
    std::memset(out, 0, sizeof *out);
    for (int i = 0; i < SF_MAX_SAMPLE_COUNT; i++) { out->second[i].window_start = SF_WS_ABSENT; out->borrow_ws[i] = SF_WS_ABSENT; }
    auto conv = [](const Bucket& d, sf_bucket* o) {
        if (d.ws == WS_NONE) { std::memset(o, 0, sizeof *o); o->window_start = SF_WS_ABSENT; return; }
        o->window_start = d.ws; o->pass = d.pass; o->block = d.block; o->exception = d.exc; o->success = d.succ;
        o->rt = d.rt; o->occupied_pass = d.occ; o->min_rt = d.min_rt;
    };
    int S = e->cfg.sample_count;
    for (int i = 0; i < S; i++) {
        conv(e->second[(size_t)l * S + i], &out->second[i]);
        const Borrow& b = e->borrow[(size_t)l * S + i];
        out->borrow_ws[i] = b.ws == WS_NONE ? SF_WS_ABSENT : b.ws;
        out->borrow_pass[i] = b.ws == WS_NONE ? 0 : b.pass;
    }
    for (int i = 0; i < MINUTE; i++) conv(e->minute[(size_t)l * MINUTE + i], &out->minute[i]);
    out->cur_thread_num = e->threads[l];
    return SF_OK;
}

static void read_rows(hs_engine* e, const NodeRows& r, sf_node_state* out) {
    std::memset(out, 0, sizeof *out);
    for (int i = 0; i < SF_MAX_SAMPLE_COUNT; i++) { out->second[i].window_start = SF_WS_ABSENT; out->borrow_ws[i] = SF_WS_ABSENT; }
    auto conv = [](const Bucket& d, sf_bucket* o) {
        if (d.ws == WS_NONE) { std::memset(o, 0, sizeof *o); o->window_start = SF_WS_ABSENT; return; }
        o->window_start = d.ws; o->pass = d.pass; o->block = d.block; o->exception = d.exc; o->success = d.succ;
        o->rt = d.rt; o->occupied_pass = d.occ; o->min_rt = d.min_rt;
    };
    for (int i = 0; i < e->cfg.sample_count; i++) {
        conv(r.sec[i], &out->second[i]);
        out->borrow_ws[i] = r.bor[i].ws == WS_NONE ? SF_WS_ABSENT : r.bor[i].ws;
        out->borrow_pass[i] = r.bor[i].ws == WS_NONE ? 0 : r.bor[i].pass;
    }
    for (int i = 0; i < MINUTE; i++) conv(r.min[i], &out->minute[i]);
    out->cur_thread_num = *r.thr;
}
static int read_aux(hs_engine* e, uint32_t res, uint32_t kind, uint32_t id, sf_node_state* out) {
    uint32_t l; if (!local_of(e, res, &l) || e->xtab.empty()) return SF_ERR_INVALID;
    const ParamTable t{e->xtab.data(), e->xtab.size() - 1, &e->err};
    const ParamSlot* s = t.find(pkey_hi(l, PK_AUX, kind, 0), id);
    if (!s) return SF_ERR_INVALID;
    read_rows(e, aux_rows(e->st, (uint32_t)s->a), out);
    return SF_OK;
}
int hs_read_origin_node(hs_engine* e, uint32_t res, uint32_t origin, sf_node_state* out) {
    return read_aux(e, res, AX_ORIGIN, origin, out);
}
int hs_read_context_node(hs_engine* e, uint32_t context, uint32_t res, sf_node_state* out) {
    return read_aux(e, res, AX_CTX, context, out);
}

int hs_read_rule_state(hs_engine* e, uint32_t idx, sf_rule_state* out) {
    if (idx >= e->flow_pos.size()) return SF_ERR_INVALID;
    const DevRuleState& s = e->rstate[e->flow_pos[idx]];
    out->stored_tokens = s.stored_tokens; out->last_filled_time = s.last_filled; out->latest_passed_time = s.latest_passed;
    return SF_OK;
}

// the per-window exchange's plan step (sf_sysx.h sx_reduce) on host arrays
void hs_sx_reduce(const int64_t* msgs, int N, SxPlan* pl, double qps, double interval_sec) {
    SysRule r{};
    r.qps = qps;
    sx_reduce(msgs, N, pl, r, interval_sec);
}

}  // extern "C"
