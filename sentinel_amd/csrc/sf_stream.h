// sf_stream.h — heavy THREAD-grade and RateLimiter segments, one 256-thread
// workgroup per segment (product code, device only).
//
// Both controllers are serial per resource: every decision reads the state
// the previous one left (curThreadNum for DefaultController THREAD grade,
// latestPassedTime for RateLimiterController).  One wavefront runs that chain;
// the other three keep it fed.  The segment streams through LDS in chunks of
// HS_CH events, double-buffered: while wave 0 decides chunk k out of LDS, all
// four waves have the global loads of chunk k+1 in flight (coalesced, 8 events
// per lane), then write them into the other buffer and meet at a barrier.
//
//  THREAD (DefaultController.java:50-89, StatisticSlot.java:64-65,157): an
//    entry passes iff (int)(curThreadNum + acquireCount) <= count; a pass adds
//    one thread, the exit of a passed entry removes it.  Each event is packed
//    into a 32-bit code in LDS (entry: acquireCount; exit: distance back to
//    its entry).  Wave 0 decides 64-event windows with ballots, keeping the
//    pass bits of the last RING_BITS events in an LDS ring for exit liveness.
//  RATE LIMITER (RateLimiterController.java:48-102): an entry passes iff
//    t >= latestPassedTime + cost(c) - maxQueueingTimeMs.  Wave 0 jumps to the
//    first event at or after the lower bound latest + cost(1) - maxQueue with
//    a search over the chunk's LDS timestamps, then takes the first candidate
//    of a 64-event ballot.  Work is proportional to passes plus chunks.
#pragma once
#include "sf_heavy.h"

namespace sf {

constexpr int HS_T = 256;                 // threads per workgroup
constexpr int HS_PL = 8;                  // events per lane per chunk
constexpr int HS_CH = HS_T * HS_PL;       // events per chunk (2048)
// LDS: THREAD codes 2 x 8 KiB + pass ring 16 KiB; RL timestamps 2 x 16 KiB + counts 2 x 8 KiB
constexpr int HS_LDS_WORDS = (2 * HS_CH * 8 + 2 * HS_CH * 4) / 8;   // 48 KiB as u64 words
constexpr uint32_t CODE_EXIT = 0x80000000u;
constexpr uint32_t CODE_DEAD = 0x7fffffffu;   // exit distance field: entry not in this segment (never live)

struct StreamCtx {
    const uint32_t* list; const uint32_t* n_list;   // n_list[0] front count, n_list[1] back count
    uint32_t seg_cap;
    uint64_t* sticks;
};

__device__ __forceinline__ bool stream_at(const StreamCtx& sc, uint32_t b, uint32_t* s) {
    const uint32_t nf = sc.n_list[0], nb = sc.n_list[1];
    if (b < nf) { *s = sc.list[b]; return true; }
    if (b < nf + nb) { *s = sc.list[sc.seg_cap - 1 - (b - nf)]; return true; }
    return false;
}

// ------------------------------------------------------------------ THREAD
// DefaultController, FLOW_GRADE_THREAD (DefaultController.java:50-89,
// StatisticSlot.java:64-65,157): an entry passes iff (int)(curThreadNum +
// acquireCount) <= count; a pass adds one thread, the exit of a passed entry
// removes one.  An exit's liveness is settled when its entry passes: the pass
// sets the exit's bit in a live-exit bitmap, an LDS ring over the next
// LX_WORDS * 64 events (farther exits go to a bitmap in HBM that the chunk
// loader folds back in).  Exits of entries of earlier batches are always live
// and enter the ring when their chunk is prepared.
//
// Waves 1-3 prepare chunk k+1 (THR_WPC windows of 64 events) while wave 0
// decides chunk k.  Per window they precompute the entry mask, cumulative
// masks of entries with acquireCount <= m (m = 1..7), the in-window exits of
// the window's own entries, max over entries of (rank + acquireCount), and
// every entry's exit position (exit_of, written by k_gather_exit).  Wave 0
// then needs one LDS word of live exits per window:
//   - no room even with every live exit first: every entry blocks;
//   - every entry fits even at T + rank: all pass, their exits marked live;
//   - else a scalar walk over the events that change the thread count (the
//     next live exit, or the next entry that fits at the current room).
// Work is proportional to windows plus passes, not to events.
constexpr uint32_t LX_WORDS = 2048;               // live-exit ring: 128 Ki events ahead (16 KiB)
constexpr int THR_WPC = 24;                       // windows per chunk (8 per helper wave)
constexpr uint32_t THR_CH = THR_WPC * 64;          // events per chunk
constexpr uint32_t XO_NONE = 0xffffffffu;
constexpr int32_t THR_CSMALL = 8;                  // scalar walk for acquireCount <= 8
constexpr int32_t THR_CBIG = 1 << 20;              // integer compares exact below this (no int wrap)

struct ThrWin {                                    // 24 B per window
    unsigned long long ent;                        // entries
    unsigned long long inw;                        // exits whose entry is in this window
    int32_t maxrc;                                 // bound of max over entries of rank + acquireCount
    uint32_t flags;                                // bit 0: an acquireCount > 8, bit 1: > THR_CBIG
};

struct ThrLds {
    unsigned long long lx[LX_WORDS];               // live exits of window (pos - lo) / 64 at word % LX_WORDS
    ThrWin win[2][THR_WPC];
    uint32_t xo[2][THR_CH];                        // exit position (sorted index) of each entry, or XO_NONE
    int32_t cn[2][THR_CH];                         // acquireCount (exact path)
};
static_assert(sizeof(ThrLds) <= HS_LDS_WORDS * 8, "THREAD LDS layout exceeds the stream kernel's LDS");

__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long v) {
    return (unsigned long long)uniform64((int64_t)v);
}

// Helper wave h (1..3): prepare windows h-1, h+2, ... of the chunk starting at q0.
// Every load of the wave's windows is issued before any is used (one memory
// round trip per chunk; indices clamped into the segment instead of branches).
constexpr int THR_WPW = THR_WPC / 3;              // windows per helper wave
__device__ void thr_prepare(ThrLds& L, int buf, const SegIO& io, const uint32_t* exit_of,
                            const unsigned long long* lxfar, uint32_t q0, uint32_t lo, uint32_t hi, int h) {
    const int lane = (int)(threadIdx.x & 63);
    uint8_t fa[THR_WPW]; int32_t ca[THR_WPW]; int64_t ra[THR_WPW]; uint32_t xa[THR_WPW];
    unsigned long long f0a[THR_WPW], f1a[THR_WPW];
#pragma unroll
    for (int k = 0; k < THR_WPW; k++) {
        const uint32_t q = q0 + 64u * (uint32_t)(h - 1 + 3 * k);
        const uint32_t jc = min(q + (uint32_t)lane, hi - 1);
        fa[k] = io.flags[jc];
        ca[k] = io.cnt[jc];
        ra[k] = io.eref ? io.eref[jc] : -1;
        xa[k] = exit_of[jc];
        const uint32_t g = min(q, hi - 1) >> 6;
        f0a[k] = __hip_atomic_load(lxfar + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        f1a[k] = __hip_atomic_load(lxfar + g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int k = 0; k < THR_WPW; k++) {
        const int wl = h - 1 + 3 * k;
        const uint32_t q = q0 + 64u * (uint32_t)wl;
        if (q >= hi) break;
        const uint32_t j = q + (uint32_t)lane;
        const bool valid = j < hi;
        const uint8_t f = fa[k];
        const int32_t c = ca[k];
        const int64_t ref = ra[k];
        const bool ent = valid && !(f & SF_EV_EXIT);
        const bool ex = valid && (f & SF_EV_EXIT);
        ThrWin wn;
        wn.ent = __ballot(ent);
        wn.inw = __ballot(ex && ref >= (int64_t)q && ref < (int64_t)j);
        const bool gt1 = __ballot(ent && c > 1) != 0ull, gt8 = __ballot(ent && c > THR_CSMALL) != 0ull;
        wn.flags = (gt8 ? 1u : 0u) | (__ballot(ent && c > THR_CBIG) ? 2u : 0u);
        // bound of max(rank + acquireCount): (entries - 1) + (1, or 8 when some count is 2..8)
        wn.maxrc = gt8 ? INT32_MAX : (int32_t)__popcll(wn.ent) - 1 + (gt1 ? THR_CSMALL : 1);
        L.xo[buf][64 * wl + lane] = ent ? xa[k] : XO_NONE;
        L.cn[buf][64 * wl + lane] = c;
        const unsigned long long mo = __ballot(ex && ref < 0);        // entry of an earlier batch: live
        if (lane == 0) {
            L.win[buf][wl] = wn;
            // live exits of far-away entries (written into HBM when those entries passed)
            const uint32_t sh = q & 63;
            const unsigned long long far = sh ? (f0a[k] >> sh) | (f1a[k] << (64 - sh)) : f0a[k];
            const unsigned long long add = (mo | far) & (q + 64 <= hi ? ~0ull : ((1ull << (hi - q)) - 1ull));
            if (add) atomicOr(&L.lx[((q - lo) >> 6) % LX_WORDS], add);
        }
    }
}

// mark the exit at sorted position x live (its entry just passed); q = current window
__device__ __forceinline__ bool thr_mark_exit(ThrLds& L, unsigned long long* lxfar, uint32_t x, uint32_t q,
                                              uint32_t lo) {
    if (x - q < (LX_WORDS - 1) * 64u) { atomicOr(&L.lx[((x - lo) >> 6) % LX_WORDS], 1ull << ((x - lo) & 63)); return false; }
    atomicOr(lxfar + (x >> 6), 1ull << (x & 63));
    return true;
}

// Wave 0: decide the windows of one prepared chunk.  The window summaries of
// the chunk are read into registers once (lane w <-> window w) and used with
// readlane.  The live-exit word of a window is read from the LDS ring after
// the previous window's exits were marked (one LDS op per window, in order).
// While saturated (no room) a run of windows without live exits blocks
// entirely: one vector read of their ring words finds the next one.  Inside a
// window, only events that change the thread count are visited; the exits of
// the window's passed entries are marked in one vector step after it.
__device__ __forceinline__ unsigned long long rl64(unsigned long long v, int l) {
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((unsigned long long)b << 32) | a;
}

__device__ void thr_decide(ThrLds& L, int buf, unsigned long long* lxfar, uint32_t q0, uint32_t lo, uint32_t hi,
                           double M, int64_t IM, int64_t& T, unsigned long long* pbits) {
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t nwin = min((hi - q0 + 63) / 64, (uint32_t)THR_WPC);
    bool far_marked = false;
    T = uniform64(T);
    const int wl = lane < THR_WPC ? lane : 0;
    const unsigned long long r_ent = L.win[buf][wl].ent;
    const int32_t r_maxrc = L.win[buf][wl].maxrc;
    const uint32_t r_flags = L.win[buf][wl].flags;
    const uint32_t slot0 = (q0 - lo) >> 6;
    uint32_t w = 0;
    while (w < nwin) {
        const uint32_t q = q0 + 64 * w;
        const uint32_t slot = (slot0 + w) % LX_WORDS;
        const unsigned long long me = rl64(r_ent, (int)w);
        const uint32_t flags = (uint32_t)__builtin_amdgcn_readlane((int)r_flags, (int)w);
        const int64_t room0 = IM - T;
        const bool tsmall = T >= (int64_t)INT32_MIN + 64 && T + (int64_t)THR_CBIG + 64 <= (int64_t)INT32_MAX;
        if (room0 <= 0 && tsmall) {
            // saturated: skip the windows with no live exit (all their entries block)
            const uint32_t wn_ = w + (uint32_t)lane;
            const bool inr = wn_ < nwin;
            const unsigned long long v = inr ? L.lx[(slot0 + wn_) % LX_WORDS] : 0ull;
            const uint32_t fl = (uint32_t)__shfl((int)r_flags, inr ? (int)wn_ : 0);
            const unsigned long long stop = __ballot(inr && (v != 0ull || (fl & 2u)));
            if (!stop) { w = nwin; break; }
            const uint32_t k = (uint32_t)(__ffsll((long long)stop) - 1);
            if (k > 0) { w += k; continue; }
        }
        unsigned long long ml = uniform_u64(L.lx[slot]);     // live exits of this window
        const int32_t maxrc = __builtin_amdgcn_readlane(r_maxrc, (int)w);
        unsigned long long pmask = 0;
        const bool nowrap = !(flags & 2u) && tsmall;
        if (me == 0) {
            T -= __popcll(ml);
        } else if (nowrap && room0 + (int64_t)__popcll(ml) < 1) {
            // even with every live exit first, no entry fits (acquireCount >= 1):
            // all entries block, so no exit of this window's entries turns live
            T -= __popcll(ml);
        } else if (nowrap && room0 >= (int64_t)maxrc) {
            // the thread count before an entry is <= T + (entries before it): all fit
            pmask = me;
            ml |= uniform_u64(L.win[buf][w].inw);        // exits of this window's entries, inside it
            T += (int64_t)__popcll(me) - (int64_t)__popcll(ml);
        } else {
            const uint32_t xo = L.xo[buf][64 * w + lane];
            const int32_t c = L.cn[buf][64 * w + lane];
            const bool small = nowrap && !(flags & 1u);
            // in-window exit of each entry lane: bit position, or 64
            const uint32_t inpos = (xo != XO_NONE && xo - q < 64u && xo > q + (uint32_t)lane) ? xo - q : 64u;
            const bool ent = (me >> lane) & 1ull;
            int cursor = 0;
            while (cursor < 64) {
                unsigned long long fm = 0;
                if (small) {
                    // without int wrap (int)(T + c) <= count  <=>  c <= floor(count) - T
                    const int64_t room = IM - T;
                    if (room >= THR_CSMALL) fm = me;
                    else if (room > 0) fm = __ballot(ent && (int64_t)c <= room);
                } else {
                    fm = __ballot(ent && (double)(int32_t)((uint32_t)(int32_t)T + (uint32_t)c) <= M);
                }
                const unsigned long long cand = (fm | ml) & (~0ull << cursor);
                if (!cand) break;
                const int kk = __ffsll((long long)cand) - 1;
                const unsigned long long bit = 1ull << kk;
                if (me & bit) {
                    T += 1; pmask |= bit;
                    const uint32_t ip = (uint32_t)__builtin_amdgcn_readlane((int)inpos, kk);
                    if (ip < 64u) ml |= 1ull << ip;
                } else {
                    T -= 1;
                }
                cursor = kk + 1;
            }
        }
        T = uniform64(T);
        if (pmask) {
            // exits of the passed entries beyond this window turn live (one vector step)
            const uint32_t xo = L.xo[buf][64 * w + lane];
            const bool mk = ((pmask >> lane) & 1ull) && xo != XO_NONE && xo < hi && xo >= q + 64;
            bool fm2 = false;
            if (mk) fm2 = thr_mark_exit(L, lxfar, xo, q, lo);
            far_marked |= __ballot(fm2) != 0;
            if (lane == 0) {
                const uint32_t sh = q & 63;
                atomicOr(pbits + (q >> 6), pmask << sh);
                if (sh) atomicOr(pbits + (q >> 6) + 1, pmask >> (64 - sh));
            }
        }
        if (lane == 0) L.lx[slot] = 0ull;                  // consumed: reused LX_WORDS windows later
        w++;
    }
    if (far_marked) {                                      // far exits must be in HBM before a loader reads them
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        __builtin_amdgcn_s_waitcnt(0);
    }
}

// ------------------------------------------------------------------ RateLimiter
struct RlRegs { int64_t ts[HS_PL]; int32_t c[HS_PL]; };

__device__ __forceinline__ void rl_load(RlRegs& r, const SegIO& io, uint32_t q0, uint32_t hi) {
    uint8_t f[HS_PL];
#pragma unroll
    for (int i = 0; i < HS_PL; i++) {
        const uint32_t j = min(q0 + (uint32_t)(i * HS_T) + threadIdx.x, hi - 1);
        r.ts[i] = io.ts[j];
        r.c[i] = io.cnt[j];
        f[i] = io.flags[j];
    }
#pragma unroll
    for (int i = 0; i < HS_PL; i++) {
        const bool v = q0 + (uint32_t)(i * HS_T) + threadIdx.x < hi;
        r.ts[i] = v ? r.ts[i] : INT64_MAX;
        r.c[i] = (v && !(f[i] & SF_EV_EXIT)) ? r.c[i] : 0;        // 0: exit / padding (never a candidate)
    }
}
__device__ __forceinline__ void rl_store(const RlRegs& r, int64_t* tsb, int32_t* cb) {
#pragma unroll
    for (int i = 0; i < HS_PL; i++) { tsb[i * HS_T + threadIdx.x] = r.ts[i]; cb[i * HS_T + threadIdx.x] = r.c[i]; }
}

// first index in [a, n) of the sorted LDS timestamps with ts >= x (n if none)
__device__ __forceinline__ uint32_t lds_first_ge(const int64_t* tsb, uint32_t a, uint32_t n, int64_t x) {
    const int lane = (int)(threadIdx.x & 63);
    while (n - a > 64) {
        const uint32_t step = (n - a + 63) / 64;
        const uint32_t last = min(a + (uint32_t)(lane + 1) * step, n) - 1;
        const bool ge = a + (uint32_t)lane * step < n && tsb[last] >= x;
        const unsigned long long m = __ballot(ge);
        if (!m) return n;
        const uint32_t k = (uint32_t)(__ffsll((long long)m) - 1);
        const uint32_t na = a + k * step;
        n = min(a + (k + 1) * step, n);
        a = na;
    }
    const unsigned long long m = __ballot(a + (uint32_t)lane < n && tsb[a + lane] >= x);
    return m ? a + (uint32_t)(__ffsll((long long)m) - 1) : n;
}

__device__ __forceinline__ void rl_decide_chunk(const int64_t* tsb, const int32_t* cb, uint32_t q0, uint32_t hi,
                                                const DevRule& rule, int64_t cost1, int64_t& L, ItemWriter& iw) {
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t n = min(hi - q0, (uint32_t)HS_CH);
    uint32_t p = 0;
    while (p < n) {
        // cost(c) >= cost(1) for c >= 1: nothing before this time can pass
        p = lds_first_ge(tsb, p, n, L + cost1 - rule.max_queue_ms);
        if (p >= n) break;
        const uint32_t k = p + (uint32_t)lane;
        bool cand = false;
        if (k < n) {
            const int32_t c = cb[k];
            if (c > 0) {
                const int64_t cost = c == 1 ? cost1 : j_round(1.0 * c / rule.count * 1000);
                cand = tsb[k] >= L + cost - rule.max_queue_ms;
            }
        }
        const unsigned long long m = __ballot(cand);
        if (!m) { p += 64; continue; }
        const uint32_t jj = p + (uint32_t)(__ffsll((long long)m) - 1);
        const int32_t cj = cb[jj];
        const int64_t cost = cj == 1 ? cost1 : j_round(1.0 * cj / rule.count * 1000);
        const int64_t t = tsb[jj];
        int32_t wait = 0;
        if (L + cost <= t) L = t;                           // expectedTime <= currentTime
        else { L += cost; wait = (int32_t)(L - t); }        // queued: sleep(wait), then pass
        iw.push(lane == 0, q0 + jj, q0 + jj + 1, wait);
        p = jj + 1;
    }
}

__global__ void __launch_bounds__(HS_T) k_heavy_stream(DevState st, SegIO io, HeavyCtx hc, StreamCtx sc) {
    __shared__ unsigned long long smem[HS_LDS_WORDS];
    uint32_t s;
    if (!stream_at(sc, blockIdx.x, &s)) return;
    const uint64_t t_start = sc.sticks ? wall_clock64() : 0;
    const uint32_t lo = hc.seg_start[s], hi = hc.seg_start[s + 1], res = hc.seg_res[s];
    const uint32_t r0 = st.rule_off[res];
    const DevRule rule = st.rules[r0];
    const bool wave0 = threadIdx.x < 64;
    const uint32_t nch = (hi - lo + HS_CH - 1) / HS_CH;
    if (hc.seg_mode[s] == SM_THREAD) {
        ThrLds& L = *reinterpret_cast<ThrLds*>(smem);
        for (uint32_t i = threadIdx.x; i < LX_WORDS; i += HS_T) L.lx[i] = 0ull;
        __syncthreads();
        const double M = rule.count;
        const int64_t IM = (int64_t)floor(M);
        int64_t T = st.threads[res];
        const int h = (int)(threadIdx.x >> 6);
        const uint32_t ntc = (hi - lo + THR_CH - 1) / THR_CH;
        if (h > 0) thr_prepare(L, 0, io, hc.exit_of, hc.lxfar, lo, lo, hi, h);
        __syncthreads();
#ifdef SF_STREAM_PROF
        uint64_t t_work = 0, t_bar = 0;
#endif
        for (uint32_t k = 0; k < ntc; k++) {
            const uint32_t q0 = lo + k * THR_CH;
#ifdef SF_STREAM_PROF
            const uint64_t c0 = __builtin_amdgcn_s_memtime();
#endif
            if (h == 0) thr_decide(L, k & 1, hc.lxfar, q0, lo, hi, M, IM, T, hc.passbits);
            else if (k + 1 < ntc) thr_prepare(L, (k + 1) & 1, io, hc.exit_of, hc.lxfar, q0 + THR_CH, lo, hi, h);
#ifdef SF_STREAM_PROF
            const uint64_t c1 = __builtin_amdgcn_s_memtime();
#endif
            __syncthreads();
#ifdef SF_STREAM_PROF
            t_work += c1 - c0; t_bar += __builtin_amdgcn_s_memtime() - c1;
#endif
        }
#ifdef SF_STREAM_PROF
        if ((threadIdx.x & 63) == 0)
            printf("SF_STREAM_PROF seg %u wave %d events %u chunks %u: work %lu barrier %lu cycles\n", s, h, hi - lo,
                   ntc, (unsigned long)t_work, (unsigned long)t_bar);
#endif
    } else {                                                     // SM_RL
        int64_t* tsb = (int64_t*)smem;                           // [2][HS_CH]
        int32_t* cb = (int32_t*)(smem + 2 * HS_CH);              // [2][HS_CH]
        DevRuleState rs = st.rstate[r0];
        ItemWriter iw{hc.item_lo, hc.item_hi, hc.item_wait, lo, 0};
        if (rule.count > 0) {
            const int64_t cost1 = j_round(1.0 * 1 / rule.count * 1000);
            int64_t L = rs.latest_passed;
            RlRegs r;
            rl_load(r, io, lo, hi);
            rl_store(r, tsb, cb);
            __syncthreads();
            for (uint32_t k = 0; k < nch; k++) {
                const uint32_t q0 = lo + k * HS_CH;
                const bool more = k + 1 < nch;
                if (more) rl_load(r, io, q0 + HS_CH, hi);
                if (wave0) rl_decide_chunk(tsb + (k & 1) * HS_CH, cb + (k & 1) * HS_CH, q0, hi, rule, cost1, L, iw);
                if (more) rl_store(r, tsb + ((k + 1) & 1) * HS_CH, cb + ((k + 1) & 1) * HS_CH);
                __syncthreads();
            }
            rs.latest_passed = L;
        }
        if (threadIdx.x == 0) { hc.n_items[s] = iw.n; st.rstate[r0] = rs; }
    }
    if (sc.sticks && threadIdx.x == 0) sc.sticks[blockIdx.x] = wall_clock64() - t_start;
}

}  // namespace sf
