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

namespace sf_dg {

constexpr int BLK = 256;
constexpr uint32_t HEAVY = 64;      // segments longer than this are walked by a whole wave
constexpr uint32_t MAXC = 4;        // breakers per resource held in registers by the wave walk

__global__ void __launch_bounds__(BLK) k_dg_keys(DegradeDev d, DegradeBatch b, uint32_t* keys, uint32_t* idx,
                                                 uint8_t* status, uint16_t* rule, int32_t* wait, int* err) {
    const uint32_t i = blockIdx.x * BLK + threadIdx.x;
    if (i >= b.n) return;
    const uint32_t r = b.res[i];
    const uint8_t f = b.flags[i];
    uint32_t key = d.n_rres;
    if (b.ts[i] < (i ? b.ts[i - 1] : *b.last_ts)) atomicOr(err, 4);   // the clock never goes back
    if (r % b.shard_count != b.shard_index || r / b.shard_count >= b.R) {
        atomicOr(err, 1);
    } else if (d.n_rres) {               // rr_of exists once degrade rules were loaded
        key = d.rr_of[r / b.shard_count];
    }
    // an entry blocked by an earlier slot (SF_EV_BLOCKED) never reaches
    // DegradeSlot, and its exit returns early there (blockError set,
    // DegradeSlot.java:72-77); so does the exit of an entry blocked in an
    // earlier batch (entry_ref -2): none of them is walked
    bool skip = false;
    uint8_t st = (f & SF_EV_EXIT) ? SF_V_EXIT : SF_V_PASS;
    if (!(f & SF_EV_EXIT)) {
        if (f & SF_EV_BLOCKED) { skip = true; st = SF_V_BLOCK_OTHER; }
    } else if (b.eref) {
        const int64_t ref = b.eref[i];
        if (ref == -2 || (ref >= 0 && ref < (int64_t)i && (b.flags[ref] & (SF_EV_BLOCKED | SF_EV_EXIT)) == SF_EV_BLOCKED)) {
            skip = true; st = SF_V_EXIT_IGNORED;
        }
    }
    keys[i] = skip ? d.n_rres : key;
    idx[i] = i;
    // no breaker (or not yet decided): entries pass the degrade check, exits record
    status[i] = st;
    if (rule) rule[i] = 0;
    if (wait) wait[i] = 0;
}

// a refused batch (bad shard, clock, refs) does not advance the engine clock
__global__ void k_dg_clock(DegradeBatch b, const int* err) { if (*err == 0) *b.last_ts = b.ts[b.n - 1]; }

__global__ void __launch_bounds__(BLK) k_dg_bounds(const uint32_t* keys, uint32_t n, uint32_t none, uint32_t* beg,
                                                   uint32_t* end) {
    const uint32_t j = blockIdx.x * BLK + threadIdx.x;
    if (j >= n) return;
    const uint32_t k = keys[j];
    if (k >= none) return;
    if (j == 0 || keys[j - 1] != k) beg[k] = j;
    if (j == n - 1 || keys[j + 1] != k) end[k] = j + 1;
}

__device__ __forceinline__ int64_t rl64(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Sorted event payload of every breaker-resource event (keys < none come
// first after the sort): the wave walk then reads one coalesced 32-B record per
// lane instead of a chain of dependent gathers.
__global__ void __launch_bounds__(BLK) k_dg_inv(uint32_t n, const uint32_t* keys, const uint32_t* perm,
                                                uint32_t none, uint32_t* inv) {
    const uint32_t j = blockIdx.x * BLK + threadIdx.x;
    if (j < n && keys[j] < none) inv[perm[j]] = j;
}

__global__ void __launch_bounds__(BLK) k_dg_gather(DegradeBatch b, const uint32_t* keys, const uint32_t* perm,
                                                   uint32_t none, const uint32_t* inv, DgEv* sev) {
    const uint32_t j = blockIdx.x * BLK + threadIdx.x;
    if (j >= b.n || keys[j] >= none) return;
    const uint32_t idx = perm[j];
    DgEv ev;
    ev.idx = idx;
    ev.t = b.ts[idx];
    uint32_t fl = b.flags[idx], bad = 0;
    ev.ref = 0xFFFFFFFFu;
    ev.refpos = 0xFFFFFFFFu;
    ev.cr = 0;
    if (fl & SF_EV_EXIT) {
        const int64_t ref = b.eref ? b.eref[idx] : -1;
        if (ref >= 0) {
            // the entry: earlier in this batch, same resource, an ENTRY (its sorted position is then valid)
            if (ref < (int64_t)idx && b.res[ref] == b.res[idx] && !(b.flags[ref] & SF_EV_EXIT)) {
                ev.cr = b.ts[ref];
                ev.ref = (uint32_t)ref;
                ev.refpos = inv[ref];        // the entry's sorted position (same resource)
            } else {
                bad = 1;
            }
        } else if (b.cts) {
            ev.cr = b.cts[idx];
        } else {
            bad = 1;
        }
    }
    ev.fl = fl | (bad << 8);
    sev[j] = ev;
}

// value of the lane below (lane 0: its own)
__device__ __forceinline__ int64_t rl64_up(int64_t v) {
    const int lane = threadIdx.x;
    const int src = lane == 0 ? 0 : lane - 1;
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)v >> 32), src);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// One wave per long breaker segment (<= MAXC breakers).  Chunks of 64 events:
// every lane gathers one event (index, ts, flags, entry ref, create ts) and the
// verdict of an entry decided in an earlier chunk, the next chunk's events are
// fetched while this one is walked, and the walk itself runs wave-uniform on
// readlane'd values with the breaker state in registers -- the per-event chain
// has no memory access.  A reference to an entry of the current or previous
// chunk is a bit of that chunk's blocked mask, found from the entry's sorted
// position (k_dg_inv / k_dg_gather).  Before the serial walk, a bulk
// prefix decides lane-parallel every event up to the first one that can change
// a breaker's state: entries refused by an OPEN (retry not reached) or
// HALF_OPEN breaker or passed by CLOSED ones, and exits that only count
// (window rolls by a segmented ballot count; a CLOSED breaker's trip point is
// found from each lane's running counts).
__global__ void __launch_bounds__(64) k_dg_wave(DegradeDev d, DegradeBatch b, const DgEv* __restrict__ sev,
                                                const uint32_t* beg, const uint32_t* end, uint8_t* status,
                                                uint16_t* rule, int* err, const uint32_t* heavy,
                                                const uint32_t* n_heavy) {
    const int lane = threadIdx.x;
    const uint32_t nh = *n_heavy;
    for (uint32_t h = blockIdx.x; h < nh; h += gridDim.x) {
        const uint32_t k = heavy[h];
        const uint32_t j0 = beg[k], j1 = end[k];
        const uint32_t c0 = d.off[k];
        const uint32_t nc = d.off[k + 1] - c0;
        sf_breaker_state S[MAXC];
        DevBreakerRule R[MAXC];
#pragma unroll
        for (uint32_t c = 0; c < MAXC; c++) {
            if (c < nc) { S[c] = d.state[c0 + c]; R[c] = d.rules[c0 + c]; }
        }
        // the lane's event of chunk [j, j+64) (sorted payload of k_dg_gather: one coalesced 32-B load)
        auto load_rec = [&](uint32_t j, uint32_t& idx, int64_t& t, uint32_t& fl, int64_t& ref, uint32_t& rp,
                            int64_t& cr, bool& bad) {
            const uint32_t p = j + lane;
            idx = 0xFFFFFFFFu; t = 0; fl = 0; ref = -1; rp = 0xFFFFFFFFu; cr = 0; bad = false;
            if (p < j1) {
                const DgEv ev = sev[p];
                idx = ev.idx; t = ev.t; fl = ev.fl & 0xFFu; cr = ev.cr; rp = ev.refpos;
                ref = ev.ref == 0xFFFFFFFFu ? -1 : (int64_t)ev.ref;
                bad = (ev.fl >> 8) != 0u;
            }
        };
        // verdict of the event's entry when that entry sits before sorted position `bound`
        // (stored and fenced by this wave, or outside the segment)
        auto load_old = [&](uint32_t fl, bool bad, int64_t ref, uint32_t rp, uint32_t bound) -> bool {
            return (fl & SF_EV_EXIT) && !bad && ref >= 0 && rp < bound && status[ref] == SF_V_BLOCK_DEGRADE;
        };
        // records are fetched two chunks ahead, older-entry verdicts one chunk ahead
        uint32_t idx, fl, rp, idx1 = 0xFFFFFFFFu, fl1 = 0, rp1 = 0xFFFFFFFFu, idx2 = 0xFFFFFFFFu, fl2 = 0,
                 rp2 = 0xFFFFFFFFu;
        int64_t t, ref, cr, t1 = 0, ref1 = -1, cr1 = 0, t2 = 0, ref2 = -1, cr2 = 0;
        bool bad, old_blk, bad1 = false, old1 = false, bad2 = false;
        load_rec(j0, idx, t, fl, ref, rp, cr, bad);
        old_blk = load_old(fl, bad, ref, rp, j0);
        if (j0 + 64 < j1) load_rec(j0 + 64, idx1, t1, fl1, ref1, rp1, cr1, bad1);
        uint64_t pblk = 0;                              // previous chunk: blocked entries
        for (uint32_t j = j0; j < j1; j += 64) {
            const uint32_t cnt = min(64u, j1 - j);
            const uint32_t pj = j - 64;                 // previous chunk's start (unused in the first chunk)
            if (bad) atomicOr(err, 2);
            const uint64_t badm = __ballot(bad), oldm = __ballot(old_blk);
            if (j + 128 < j1) load_rec(j + 128, idx2, t2, fl2, ref2, rp2, cr2, bad2);
            // the next chunk's older-entry verdicts are those stored before this chunk
            if (j + 64 < j1) old1 = load_old(fl1, bad1, ref1, rp1, j);
            uint8_t my_st = (fl & SF_EV_EXIT) ? SF_V_EXIT : SF_V_PASS;
            uint16_t my_rule = 0;
            // ---- bulk prefix: the events before the first state change, decided lane-parallel
            const bool valid = (uint32_t)lane < cnt;
            const bool is_en = valid && !(fl & SF_EV_EXIT);
            const bool is_ex = valid && (fl & SF_EV_EXIT) && !bad;
            // an entry changes nothing while the first non-CLOSED breaker refuses it without a retry
            int bstar = -1;
            bool any_half = false;
#pragma unroll
            for (uint32_t c = 0; c < MAXC; c++) {
                if (c < nc) {
                    any_half |= S[c].state == SF_CB_HALF_OPEN;
                    if (bstar < 0 && S[c].state != SF_CB_CLOSED) bstar = (int)c;
                }
            }
            bool inv_blk = false, inv = true;
            if (bstar >= 0) {
                int64_t retry = 0;
                int st = 0;
#pragma unroll
                for (uint32_t c = 0; c < MAXC; c++)
                    if ((int)c == bstar) { retry = S[c].next_retry_ms; st = S[c].state; }
                inv = st == SF_CB_HALF_OPEN || t < retry;
                inv_blk = inv;
            }
            const uint64_t N = __ballot(is_en && !inv), BI = __ballot(is_en && inv_blk);
            bool ign = false;
            if (is_ex && ref >= 0) {
                if (rp >= j && rp < j + 64) ign = (BI >> (rp - j)) & 1ull;
                else if (j > j0 && rp >= pj && rp < j) ign = (pblk >> (rp - pj)) & 1ull;
                else ign = old_blk;
            }
            const uint64_t E = __ballot(is_ex && !ign);
            const uint64_t le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
            uint64_t T = any_half ? E : 0ull;
            int64_t wsv[MAXC];
            uint64_t Hm[MAXC];
#pragma unroll
            for (uint32_t c = 0; c < MAXC; c++) {
                wsv[c] = 0; Hm[c] = 0;
                if (c < nc) {
                    const int64_t L = R[c].interval, ws0 = S[c].window_start;
                    // the current window needs no 64-bit modulo (lanes past a window boundary take it)
                    const int64_t ws = (t >= 0 && ws0 != DG_WS_NONE && t >= ws0 && t - ws0 < L) ? ws0 : t - t % L;
                    wsv[c] = ws;
                    const bool h = R[c].grade == SF_DEGRADE_GRADE_RT ? (t - cr) > R[c].max_rt : (fl & SF_EV_ERROR) != 0;
                    Hm[c] = __ballot(is_ex && !ign && h);
                    if (S[c].state == SF_CB_CLOSED) {
                        const int64_t pws = rl64_up(ws);
                        const uint64_t B = __ballot(valid && (lane == 0 || ws != pws));
                        const uint64_t bl = B & le;
                        const int start = bl ? 63 - __builtin_clzll(bl) : 0;
                        const uint64_t run = le & ~((1ull << start) - 1);
                        const bool same = ws == S[c].window_start;
                        const int64_t tot = __builtin_popcountll(E & run) + (same ? S[c].total_count : 0);
                        const int64_t hh = __builtin_popcountll(Hm[c] & run) + (same ? S[c].hit_count : 0);
                        bool cond = false;
                        if (((E >> lane) & 1ull) && tot >= R[c].min_req) {
                            const double cur = R[c].grade == SF_DEGRADE_GRADE_EXCEPTION_COUNT
                                                   ? (double)hh : (double)hh * 1.0 / (double)tot;
                            cond = cur > R[c].thr ||
                                   (R[c].grade == SF_DEGRADE_GRADE_RT && cur == R[c].thr && R[c].thr == 1.0);
                        }
                        T |= __ballot(cond);
                    }
                }
            }
            const uint64_t stop = (T | N) & (cnt == 64 ? ~0ull : ((1ull << cnt) - 1));
            const uint32_t cut = stop ? (uint32_t)__builtin_ctzll(stop) : cnt;
            const uint64_t below = cut >= 64 ? ~0ull : ((1ull << cut) - 1);
#pragma unroll
            for (uint32_t c = 0; c < MAXC; c++) {
                const uint64_t eb = E & below;
                if (c < nc && eb) {
                    const int m = 63 - __builtin_clzll(eb);
                    const int64_t W = rl64(wsv[c], m);
                    const uint64_t inW = __ballot(wsv[c] == W) & eb;
                    const int64_t nW = __builtin_popcountll(inW), hW = __builtin_popcountll(inW & Hm[c]);
                    if (S[c].window_start == DG_WS_NONE || W > S[c].window_start) {
                        S[c].window_start = W; S[c].total_count = nW; S[c].hit_count = hW;
                    } else {
                        S[c].total_count += nW; S[c].hit_count += hW;
                    }
                }
            }
            if ((uint32_t)lane < cut) {
                if (is_en && inv_blk) { my_st = SF_V_BLOCK_DEGRADE; my_rule = (uint16_t)bstar; }
                else if (is_ex && ign) my_st = SF_V_EXIT_IGNORED;
            }
            uint64_t blkm = BI & below;
            for (uint32_t q = cut; q < cnt; q++) {
                const int64_t tq = rl64(t, q);
                const uint32_t fq = (uint32_t)__builtin_amdgcn_readlane((int)fl, q);
                if (!(fq & SF_EV_EXIT)) {
                    uint32_t moved = 0;
                    int blocked = -1;
#pragma unroll
                    for (uint32_t c = 0; c < MAXC; c++) {
                        if (c < nc && blocked < 0 && S[c].state != SF_CB_CLOSED) {
                            if (S[c].state == SF_CB_OPEN && tq >= S[c].next_retry_ms) {
                                S[c].state = SF_CB_HALF_OPEN;
                                moved |= 1u << c;
                            } else {
                                blocked = (int)c;
                            }
                        }
                    }
                    if (blocked >= 0) {
#pragma unroll
                        for (uint32_t c = 0; c < MAXC; c++)
                            if (((moved >> c) & 1u) && S[c].state == SF_CB_HALF_OPEN) S[c].state = SF_CB_OPEN;
                        blkm |= 1ull << q;
                        if ((uint32_t)lane == q) { my_st = SF_V_BLOCK_DEGRADE; my_rule = (uint16_t)blocked; }
                    }
                    continue;
                }
                if ((badm >> q) & 1ull) continue;
                const int64_t rq = rl64(ref, q);
                const uint32_t rpq = (uint32_t)__builtin_amdgcn_readlane((int)rp, q);
                bool ign;
                if (rq < 0) ign = false;
                else if (rpq >= j && rpq < j + 64) ign = (blkm >> (rpq - j)) & 1ull;
                else if (j > j0 && rpq >= pj && rpq < j) ign = (pblk >> (rpq - pj)) & 1ull;
                else ign = (oldm >> q) & 1ull;
                if (ign) {
                    if ((uint32_t)lane == q) my_st = SF_V_EXIT_IGNORED;
                    continue;
                }
                const int64_t rt = tq - rl64(cr, q);
                const bool error = (fq & SF_EV_ERROR) != 0;
#pragma unroll
                for (uint32_t c = 0; c < MAXC; c++)
                    if (c < nc) dg_complete(S[c], R[c], tq, rt, error);
            }
            if ((uint32_t)lane < cnt) {
                status[idx] = my_st;
                if (rule) rule[idx] = my_rule;
            }
            // verdicts visible to this wave's loads from the next chunk on (one wave owns the segment)
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            pblk = blkm;
            idx = idx1; t = t1; fl = fl1; ref = ref1; rp = rp1; cr = cr1; bad = bad1; old_blk = old1;
            idx1 = idx2; t1 = t2; fl1 = fl2; ref1 = ref2; rp1 = rp2; cr1 = cr2; bad1 = bad2;
        }
        if (lane == 0) {
#pragma unroll
            for (uint32_t c = 0; c < MAXC; c++)
                if (c < nc) d.state[c0 + c] = S[c];
        }
    }
}

// One lane walks one breaker resource's events in time order (short segments).
__global__ void __launch_bounds__(BLK) k_dg_walk(DegradeDev d, DegradeBatch b, const uint32_t* perm,
                                                 const uint32_t* beg, const uint32_t* end, uint8_t* status,
                                                 uint16_t* rule, int* err, uint32_t* heavy, uint32_t* n_heavy) {
    const uint32_t k = blockIdx.x * BLK + threadIdx.x;
    if (k >= d.n_rres) return;
    const uint32_t j0 = beg[k], j1 = end[k];
    if (j0 >= j1) return;
    const uint32_t c0 = d.off[k], c1 = d.off[k + 1];
    if (j1 - j0 > HEAVY && c1 - c0 <= MAXC) {               // k_dg_wave's segment
        heavy[atomicAdd(n_heavy, 1u)] = k;
        return;
    }
    const DevBreakerRule* R = d.rules;
    sf_breaker_state* S = d.state;
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t i = perm[j];
        const int64_t t = b.ts[i];
        const uint8_t f = b.flags[i];
        if (!(f & SF_EV_EXIT)) {
            const int blocked = dg_entry_check(S, c0, c1, t);   // DegradeSlot.performChecking
            if (blocked >= 0) {
                status[i] = SF_V_BLOCK_DEGRADE;
                if (rule) rule[i] = (uint16_t)blocked;
            }
            continue;
        }
        // EXIT: DegradeSlot.exit -> onRequestComplete of every breaker (passed entries only)
        int64_t created;
        const int64_t ref = b.eref ? b.eref[i] : -1;
        if (ref >= 0) {
            if (ref >= (int64_t)i || b.res[ref] != b.res[i] || (b.flags[ref] & SF_EV_EXIT)) { atomicOr(err, 2); continue; }
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

}  // namespace sf_dg

using namespace sf_dg;

hipError_t dg_sort_bytes(uint32_t n, uint32_t key_bits, size_t* bytes) {
    return rocprim::radix_sort_pairs(nullptr, *bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (uint32_t*)nullptr, n, 0u, key_bits);
}

hipError_t dg_launch(const DegradeDev& d, DegradeWork& w, const DegradeBatch& b, uint8_t* status, uint16_t* rule,
                     int32_t* wait, hipStream_t s) {
    if (b.n == 0) return hipSuccess;
    k_dg_keys<<<blocks(b.n), BLK, 0, s>>>(d, b, w.keys_in, w.idx_in, status, rule, wait, w.err);
    k_dg_clock<<<1, 1, 0, s>>>(b, w.err);
    if (d.n_rres == 0) return hipGetLastError();
    size_t bytes = w.sort_tmp_bytes;
    hipError_t e = rocprim::radix_sort_pairs(w.sort_tmp, bytes, w.keys_in, w.keys_out, w.idx_in, w.idx_out, b.n, 0u,
                                             d.key_bits, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(w.end, 0, (size_t)d.n_rres * 4, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(w.beg, 0, (size_t)d.n_rres * 4, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(w.n_heavy, 0, 4, s);
    if (e != hipSuccess) return e;
    k_dg_bounds<<<blocks(b.n), BLK, 0, s>>>(w.keys_out, b.n, d.n_rres, w.beg, w.end);
    k_dg_walk<<<blocks(d.n_rres), BLK, 0, s>>>(d, b, w.idx_out, w.beg, w.end, status, rule, w.err, w.heavy,
                                               w.n_heavy);
    const uint32_t waves = min(d.n_rres, 2048u);
    k_dg_inv<<<blocks(b.n), BLK, 0, s>>>(b.n, w.keys_out, w.idx_out, d.n_rres, w.inv);
    k_dg_gather<<<blocks(b.n), BLK, 0, s>>>(b, w.keys_out, w.idx_out, d.n_rres, w.inv, w.sev);
    k_dg_wave<<<waves, 64, 0, s>>>(d, b, w.sev, w.beg, w.end, status, rule, w.err, w.heavy, w.n_heavy);
    return hipGetLastError();
}
