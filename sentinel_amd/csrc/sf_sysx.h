// sf_sysx.h — SystemRule on a resource-sharded node: the per-window exchange
// (product code; host-compilable for the CPU tests in tests/hostsim).
//
// SystemRuleManager.checkSystem (SystemRuleManager.java:291-348) reads the
// node-wide Constants.ENTRY_NODE.  With the resources hash-sharded over the
// GPUs of a node, rank r decides only its events, but an IN entry's system
// verdict depends on the passes of every earlier IN entry of the node.  For the
// inbound-QPS check (`passQps + acquireCount > qps`, :303-307; passQps =
// ENTRY_NODE's pass sum over the valid buckets / intervalSec,
// StatisticNode.java:205-214) the node-wide state an entry reads is one
// number, P(i) = P_p + (passes of IN entries of the node in [p, i)), so the
// ranks exchange per-window aggregates instead of events:
//
//  - the node's events carry global sequence numbers (submission order; time
//    is non-decreasing in it); a *plan window* is a run of events inside one
//    g-ms cell, g = gcd(bucket length, 1000), so it lies inside one
//    ENTRY_NODE second bucket and one minute bucket;
//  - ENTRY_NODE is identical on every rank and exact at seq s_p (every event
//    of the node before s_p is decided);
//  - each rank bins its undecided IN entries of [lo, hi) (seq space, SX_B
//    bins): u = sum of acquireCounts of the entries that can still pass (an
//    entry its first ParamFlow rule certainly blocks, sf_system.h
//    param_inert, counts 0), n = entries, min / max acquireCount;
//  - after an all-gather of those messages every rank holds the node-wide
//    prefix of u at every bin boundary, so it classifies whole bins the same
//    way: all entries certainly fire the QPS check (P_p / intervalSec + cmin >
//    qps: P only grows), all certainly pass it (even if every entry counted in
//    u before the bin's end passed), or the bin is the crossing bin, which the
//    next level splits into SX_B bins; a one-sequence-number bin is exact;
//  - q = the first crossing entry (or the window end): every IN entry of the
//    node in [s_p, q) has a certain system verdict, each rank decides its own
//    events before q with the verdicts forced (the ordinary pipeline), packs
//    its ENTRY_NODE contribution of them (one second and one minute bucket,
//    SX_DELTA words), and the next round's first message carries it: every
//    rank adds the node's sum and ENTRY_NODE is exact at q.
//
// The entry at s_p is always classified (its prefix is exact), so each round
// progresses.  Per round the exchange is SX_WORDS * 8 B per rank per level
// (<= 4.3 KB; about three levels per round).  Eligible SystemRules read only
// the QPS check (and the CPU check, a fixed input): no thread, average-RT or
// BBR check can fire.  The other kinds stay on the event all-gather protocol
// (sentinel_amd/system_shard.py submit_node_gather).
#pragma once
#include "sf_system.h"

namespace sf {

constexpr int SX_B = 128;                 // bins per level
constexpr int SX_DELTA = 16;              // int64 words of a rank's ENTRY_NODE contribution
constexpr int SX_WORDS = SX_DELTA + 4 * SX_B;
static_assert(SX_WORDS * 8 == SF_SYSX_MSG_BYTES, "sentinel_flow.h SF_SYSX_MSG_BYTES");
// message words: delta [0, 16): key (plan window index, -1: none), second
// bucket (pass, block, succ, rt, exc, touched), minute bucket (same), minRt of
// each, threads; then u[SX_B], n[SX_B], cmin[SX_B], cmax[SX_B]
enum : int { SXD_KEY = 0, SXD_SEC = 1, SXD_MIN = 7, SXD_MRS = 13, SXD_MRM = 14, SXD_THR = 15 };
enum : int { SXM_U = SX_DELTA, SXM_N = SX_DELTA + SX_B, SXM_CMIN = SX_DELTA + 2 * SX_B, SXM_CMAX = SX_DELTA + 3 * SX_B };

// one round's plan (host; identical on every rank)
struct SxPlan {
    int64_t lo, hi, w;            // level range [lo, hi) of sequence numbers, bin width
    int64_t ub;                   // node-wide u over [s_p, lo)
    int64_t P;                    // ENTRY_NODE pass sum the QPS check reads in this window (at s_p)
    int64_t q;                    // result: the sub-batch is [s_p, q)
    int32_t done, level;
};

// SystemRules whose verdicts the exchange decides: the QPS check and the CPU
// check only (SystemRuleManager.java:303-340: maxThread / maxRt unset, the
// load check's BBR never reached)
SF_HD bool sx_rule_ok(const SysRule& r) {
    return r.max_thread == INT64_MAX && r.max_rt == INT64_MAX && !(r.load_set && r.cur_load > r.highest_load);
}

SF_HD int64_t sx_sat(int64_t a, int64_t b) {            // (a, b >= 0)
    return a > INT64_MAX - b ? INT64_MAX : a + b;
}

// The system verdict of an IN entry of [s_p, q) with acquireCount c: the
// classification made it certain, so the QPS check fires iff it fires at the
// exact P_p (sys_classify's order: qps first, then the fixed CPU check).
SF_HD uint8_t sx_reason(const SysRule& r, int64_t P, double interval_sec, int32_t c) {
    if ((double)P / interval_sec + c > r.qps) return 0;
    if (r.cpu_set && r.cur_cpu > r.highest_cpu) return 4;
    return SYS_NONE;
}

SF_HD void sx_begin(SxPlan* pl, int64_t lo, int64_t hi) {
    pl->lo = lo; pl->hi = hi;
    pl->w = hi > lo ? (hi - lo + SX_B - 1) / SX_B : 1;
    pl->ub = 0; pl->q = hi; pl->done = hi <= lo ? 1 : 0; pl->level = 0;
}

// One level: the node-wide bins (N messages of SX_WORDS words, rank order)
// -> the crossing bin, the next level's range, or q.  pl->P is set.
SF_HD void sx_reduce(const int64_t* msgs, int N, SxPlan* pl, const SysRule& r, double interval_sec) {
    if (pl->done) return;
    int64_t G = pl->ub;
    const double base = (double)pl->P / interval_sec;
    for (int b = 0; b < SX_B; b++) {
        const int64_t lo_b = pl->lo + (int64_t)b * pl->w;
        if (lo_b >= pl->hi) break;
        int64_t U = 0, n = 0, cmn = INT64_MAX, cmx = INT64_MIN;
        for (int k = 0; k < N; k++) {
            const int64_t* m = msgs + (size_t)k * SX_WORDS;
            U = sx_sat(U, m[SXM_U + b]); n += m[SXM_N + b];
            if (m[SXM_CMIN + b] < cmn) cmn = m[SXM_CMIN + b];
            if (m[SXM_CMAX + b] > cmx) cmx = m[SXM_CMAX + b];
        }
        if (n == 0) continue;                                   // (u == 0)
        const bool fire_all = base + (double)cmn > r.qps;     // (the batch has no acquireCount < 0)
        if (!fire_all) {
            // the largest P an entry of the bin can read: every counted entry
            // before it passed (a bin of one sequence number: exactly its prefix)
            const int64_t top = sx_sat(sx_sat(pl->P < 0 ? 0 : pl->P, G), pl->w == 1 ? 0 : U);
            const bool pass_all = !((double)top / interval_sec + (double)cmx > r.qps);
            if (!pass_all) {
                if (pl->w == 1) { pl->q = lo_b; pl->done = 1; return; }
                pl->ub = G;
                pl->lo = lo_b;
                pl->hi = lo_b + pl->w < pl->hi ? lo_b + pl->w : pl->hi;
                pl->w = (pl->hi - pl->lo + SX_B - 1) / SX_B;
                pl->level++;
                return;
            }
        }
        G = sx_sat(G, U);
    }
    pl->q = pl->hi;
    pl->done = 1;
}

// ENTRY_NODE += the node's contribution of the last sub-batch (the sum of the
// ranks' deltas of one plan window: adds commute inside one bucket), with
// LeapArray.currentWindow's reset rule (a bucket of an older window is reset;
// ENTRY_NODE never borrows).
SF_HD void sx_merge(Bucket& bk, int64_t ws, const int64_t* s, int64_t minrt, int64_t max_rt) {
    if (bk.ws != ws) {
        if (bk.ws != WS_NONE && ws < bk.ws) return;        // older than the slot: a throwaway window
        bk = fresh_bucket(ws, max_rt);
    }
    bk.pass = wadd(bk.pass, s[0]); bk.block = wadd(bk.block, s[1]);
    bk.succ = wadd(bk.succ, s[2]); bk.rt = wadd(bk.rt, s[3]); bk.exc = wadd(bk.exc, s[4]);
    if (minrt < bk.min_rt) bk.min_rt = minrt;
}
SF_HD void sx_apply_delta(const int64_t* msgs, int N, EntryNode* en, int64_t ws_sec, int S, int wl, int64_t ws_min,
                          int64_t max_rt) {
    int64_t sec[6] = {0, 0, 0, 0, 0, 0}, mn[6] = {0, 0, 0, 0, 0, 0}, mrs = INT64_MAX, mrm = INT64_MAX, thr = 0;
    bool any = false;
    for (int k = 0; k < N; k++) {
        const int64_t* d = msgs + (size_t)k * SX_WORDS;
        if (d[SXD_KEY] < 0) continue;
        any = true;
        for (int f = 0; f < 6; f++) { sec[f] = wadd(sec[f], d[SXD_SEC + f]); mn[f] = wadd(mn[f], d[SXD_MIN + f]); }
        if (d[SXD_MRS] < mrs) mrs = d[SXD_MRS];
        if (d[SXD_MRM] < mrm) mrm = d[SXD_MRM];
        thr = wadd(thr, d[SXD_THR]);
    }
    if (!any) return;
    if (sec[5]) sx_merge(en->second[(int)((ws_sec / wl) % S)], ws_sec, sec, mrs, max_rt);
    if (mn[5]) sx_merge(en->minute[(int)((ws_min / 1000) % MINUTE)], ws_min, mn, mrm, max_rt);
    en->threads = wadd(en->threads, thr);
}

}  // namespace sf

#ifndef SF_HOSTSIM
namespace sf {
// ---- launchers (sf_system.hip; sf_entry.hip for the delta) ----
struct SxArgs {
    DevBatch b;                   // this rank's whole batch (base 0)
    const int64_t* seq;           // its global sequence numbers (increasing)
    int64_t* msg;                 // this rank's message [SX_WORDS]
    SysRule r;
    int S, wl, interval;
    int64_t max_rt;
    double interval_sec;
    DevState st;                  // (param_inert probes)
    uint8_t* ibuf;                // [n] inert flags of the round (written at level 0)
    int64_t g, c0;                // plan-window cell length, the node's first cell
};
// per batch: out[0..4] = first cell, last cell, last seq + 1, any IN entry with acquireCount < 0, n
hipError_t sx_header(const SxArgs& a, int64_t* out, hipStream_t s);
// per batch: out[k] = the first sequence number of this rank's events in plan window k (INT64_MAX: none)
hipError_t sx_winfirst(const SxArgs& a, int64_t* out, uint32_t nw, hipStream_t s);
// one level: clear this rank's bins (level 0 keeps the delta) and bin its IN entries of the plan's range
hipError_t sx_stats(const SxArgs& a, const SxPlan& pl, uint32_t lp, bool level0, hipStream_t s);
// *out = this rank's first event from lp with seq >= q
hipError_t sx_locate(const SxArgs& a, uint32_t lp, int64_t q, uint32_t* out, hipStream_t s);
// forced system verdicts of this rank's events [lp, lq) (P: ENTRY_NODE's pass sum at s_p)
hipError_t sx_mask(const SxArgs& a, uint8_t* mask, uint32_t lp, uint32_t lq, int64_t P, hipStream_t s);
// no delta in the message (key -1)
hipError_t sx_nodelta(int64_t* msg, hipStream_t s);
// the delta of a decided view (one plan window, `key`) into msg
hipError_t launch_entry_delta(const DevState& st, const DevBatch& v, const uint8_t* vstatus, EntryAcc* acc,
                              int64_t* msg, int64_t key, hipStream_t s);
}  // namespace sf
#endif
