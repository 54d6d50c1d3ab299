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
struct ThrRegs { uint32_t code[HS_PL]; };

__device__ __forceinline__ void thr_load(ThrRegs& r, const SegIO& io, uint32_t q0, uint32_t lo, uint32_t hi) {
    // every load of the chunk issued before any is used (one memory round trip):
    // indices are clamped into the segment instead of branching around loads
    uint8_t f[HS_PL]; int32_t cn[HS_PL]; int64_t rf[HS_PL];
#pragma unroll
    for (int i = 0; i < HS_PL; i++) {
        const uint32_t j = min(q0 + (uint32_t)(i * HS_T) + threadIdx.x, hi - 1);
        f[i] = io.flags[j];
        cn[i] = io.cnt[j];
    }
    if (io.eref) {
#pragma unroll
        for (int i = 0; i < HS_PL; i++) rf[i] = io.eref[min(q0 + (uint32_t)(i * HS_T) + threadIdx.x, hi - 1)];
    } else {
#pragma unroll
        for (int i = 0; i < HS_PL; i++) rf[i] = -1;
    }
#pragma unroll
    for (int i = 0; i < HS_PL; i++) {
        const uint32_t j = q0 + (uint32_t)(i * HS_T) + threadIdx.x;
        uint32_t c = 0;
        if (f[i] & SF_EV_EXIT) {
            const int64_t ref = rf[i];
            uint32_t d;
            if (ref < 0) d = 0;                                                  // entry of an earlier batch: live
            else if (ref < (int64_t)lo || ref >= (int64_t)j) d = CODE_DEAD;     // bad ref (k_heavy_fill flags it)
            else d = (uint32_t)((int64_t)j - ref);
            c = CODE_EXIT | d;
        } else {
            c = (uint32_t)cn[i];                                                 // >= 1 (heavy_mode)
        }
        r.code[i] = j < hi ? c : 0u;
    }
}
__device__ __forceinline__ void thr_store(const ThrRegs& r, uint32_t* buf) {
#pragma unroll
    for (int i = 0; i < HS_PL; i++) buf[i * HS_T + threadIdx.x] = r.code[i];
}

// Ring word a lane needs for its exit when the exit's entry lies two or more
// windows back (windows are 64-event blocks counted from the segment start
// lo): read ahead of time, since the ring holds every window up to the one
// before the current.  0 when not needed.
__device__ __forceinline__ unsigned long long thr_ring_word(const unsigned long long* ring, uint32_t code, int lane,
                                                            uint32_t q, uint32_t lo) {
    // branch-free: always one LDS read (clamped address), the word kept only when needed
    const uint32_t d = code & ~CODE_EXIT;
    const bool need = (code & CODE_EXIT) && d != 0 && d != CODE_DEAD && d > (uint32_t)lane + 64 && d < RING_BITS - 64;
    const uint32_t b = (q + (uint32_t)lane - (need ? d : 0u) - lo) % RING_BITS;
    const unsigned long long wd = ring[b >> 6];
    return need ? wd : 0ull;
}

__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ unsigned long long lane_mask64(const uint32_t vlo, const uint32_t vhi, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)vlo, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)vhi, lane);
    return ((unsigned long long)hi << 32) | lo;
}

// Wave 0: decide the 64-event windows of one chunk.  T = curThreadNum
// (wave-uniform, kept in SGPRs); prev = pass mask of the window before.
// Software-pipelined: the code of window w+2 and the ring words of window
// w+1 are read from LDS while window w is decided; liveness of an exit whose
// entry is in window w-1 comes from `prev`, in window w from the mask being
// built, further back from the ring, beyond the ring from the pass bits in HBM.
//
// Per window: all-block and all-pass are decided from a few ballots.  Else a
// scalar walk visits only the events that change the thread count; the
// entries that fit at a given room IM - T are precomputed as cumulative
// ballots by acquireCount (lane m of cum holds the mask of entries with c <= m).
constexpr int32_t THR_CSMALL = 8;            // scalar walk for acquireCount <= 8
constexpr int32_t THR_CBIG = 1 << 20;        // integer compares exact below this (no int wrap)

__device__ __forceinline__ void thr_decide_chunk(const uint32_t* buf, unsigned long long* ring, uint32_t q0,
                                                 uint32_t lo, uint32_t hi, double M, int64_t IM, int64_t& T,
                                                 unsigned long long& prev, unsigned long long* pbits) {
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t nwin = (min(hi - q0, (uint32_t)HS_CH) + 63) / 64;
    uint32_t code_c = buf[lane];
    uint32_t code_n = nwin > 1 ? buf[64 + lane] : 0u;
    unsigned long long rw_c = thr_ring_word(ring, code_c, lane, q0, lo);
    T = uniform64(T);
    for (uint32_t w = 0; w < nwin; w++) {
        const uint32_t q = q0 + 64 * w;
        // read ahead (LDS ops of one wave complete in order)
        const uint32_t code_nn = w + 2 < nwin ? buf[64 * (w + 2) + lane] : 0u;
        const unsigned long long rw_n = w + 1 < nwin ? thr_ring_word(ring, code_n, lane, q + 64, lo) : 0ull;

        const uint32_t code = code_c;
        const bool valid = q + (uint32_t)lane < hi;
        const bool ex = valid && (code & CODE_EXIT);
        const bool ent = valid && !(code & CODE_EXIT);
        const uint32_t d = code & ~CODE_EXIT;
        const int32_t c = (int32_t)code;
        // exit liveness without branches: entry of an earlier batch (d == 0), this
        // window (in-window: decided below), the previous window, the LDS ring
        const bool exr = ex && d != CODE_DEAD && d != 0;
        const uint32_t sh = (uint32_t)(lane - (int)d) & 63u;
        const bool inwin = exr && d <= (uint32_t)lane;
        const bool in_prev = exr && d > (uint32_t)lane && d <= (uint32_t)lane + 64;
        const bool in_ring = exr && d > (uint32_t)lane + 64 && d < RING_BITS - 64;
        bool live = (ex && d == 0) || (in_prev && ((prev >> sh) & 1ull)) || (in_ring && ((rw_c >> sh) & 1ull));
        const bool in_hbm = exr && d >= RING_BITS - 64;
        if (__builtin_expect(__ballot(in_hbm) != 0, 0)) {
            // older than the ring: this wave's own bits, back from L2
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_s_waitcnt(0);
            if (in_hbm) {
                const uint32_t r = q + (uint32_t)lane - d;
                const unsigned long long wd =
                    __hip_atomic_load(pbits + (r >> 6), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                live = (wd >> (r & 63)) & 1ull;
            }
        }
        const unsigned long long m_ent = __ballot(ent);
        unsigned long long m_live = __ballot(live);
        const unsigned long long m_inwin = __ballot(inwin);
        const int n_live = (int)__popcll(m_live);
        const int n_ent = (int)__popcll(m_ent);
        unsigned long long pmask = 0;
        const int64_t room0 = IM - T;
        // integer compares are exact while (int)(T + c) of the reference cannot wrap
        const bool small_t = T >= (int64_t)INT32_MIN + 64 && T + (int64_t)THR_CBIG + 64 <= (int64_t)INT32_MAX;
        const bool nowrap = small_t && !__ballot(ent && c > THR_CBIG);
        if (n_ent == 0) {
            T -= n_live;
        } else if (nowrap && room0 + n_live < 1) {
            // even with every earlier-window live exit first, no entry fits (c >= 1);
            // then this window's own entries all block and their exits are dead
            T -= n_live;
        } else if (nowrap && !__ballot(ent && (int64_t)c + (int64_t)__builtin_amdgcn_mbcnt_hi(
                                                  (uint32_t)(m_ent >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m_ent, 0u))
                                                  > room0)) {
            // the thread count before an entry is <= T + (entries before it in the
            // window): every entry fits
            pmask = m_ent;
            T += (int64_t)n_ent - (int64_t)n_live - (int64_t)__popcll(m_inwin);
        } else if (nowrap && !__ballot(ent && c > THR_CSMALL)) {
            // scalar walk over the events that change the thread count
            uint32_t cum_lo = 0, cum_hi = 0;                 // lane m: entries with c <= m
#pragma unroll
            for (int m = 1; m < THR_CSMALL; m++) {
                const unsigned long long mm = __ballot(ent && c <= m);
                if (lane == m) { cum_lo = (uint32_t)mm; cum_hi = (uint32_t)(mm >> 32); }
            }
            int cursor = 0;
            while (cursor < 64) {
                const int64_t room = IM - T;
                const unsigned long long fm = room <= 0 ? 0ull
                                            : room >= THR_CSMALL ? m_ent
                                            : lane_mask64(cum_lo, cum_hi, (int)room);
                const unsigned long long cand = (fm | m_live) & (~0ull << cursor);
                if (!cand) break;
                const int kk = __ffsll((long long)cand) - 1;
                const unsigned long long bit = 1ull << kk;
                if (m_ent & bit) {
                    T += 1; pmask |= bit;
                    if (m_inwin) m_live |= __ballot(inwin && lane - (int)d == kk);   // its exit is now live
                } else {
                    T -= 1;
                }
                cursor = kk + 1;
            }
        } else {
            // general step loop in exact Java arithmetic (large acquireCount / int wrap)
            int cursor = 0;
            for (;;) {
                const bool fits = ent && (double)(int32_t)((uint32_t)(int32_t)T + (uint32_t)c) <= M;
                const bool lv = inwin ? ((pmask >> ((uint32_t)(lane - (int)d) & 63u)) & 1ull) != 0 : live;
                const unsigned long long m = __ballot(lane >= cursor && (fits || lv));
                if (!m) break;
                const int kk = __ffsll((long long)m) - 1;
                if ((m_ent >> kk) & 1ull) { T += 1; pmask |= 1ull << kk; } else { T -= 1; }
                cursor = kk + 1;
            }
        }
        T = uniform64(T);
        if (lane == 0) {
            ring[((q - lo) >> 6) % RING_WORDS] = pmask;                    // window q = ring word (q-lo)/64
            if (pmask) {
                const uint32_t sh = q & 63;
                atomicOr(pbits + (q >> 6), pmask << sh);
                if (sh) atomicOr(pbits + (q >> 6) + 1, pmask >> (64 - sh));
            }
        }
        prev = pmask;
        code_c = code_n; code_n = code_nn; rw_c = rw_n;
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
        uint32_t* codes = (uint32_t*)smem;                       // [2][HS_CH]
        unsigned long long* ring = smem + HS_CH;                 // after 16 KiB of codes: RING_WORDS words
        const double M = rule.count;
        const int64_t IM = (int64_t)floor(M);
        int64_t T = st.threads[res];
        unsigned long long prev = 0;
        ThrRegs r;
        thr_load(r, io, lo, lo, hi);
        thr_store(r, codes);
        __syncthreads();
#ifdef SF_STREAM_PROF
        uint64_t t_dec = 0, t_wait = 0, t_ld = 0;
#endif
        for (uint32_t k = 0; k < nch; k++) {
            const uint32_t q0 = lo + k * HS_CH;
            const bool more = k + 1 < nch;
#ifdef SF_STREAM_PROF
            const uint64_t c0 = __builtin_amdgcn_s_memtime();
#endif
            if (more) thr_load(r, io, q0 + HS_CH, lo, hi);
#ifdef SF_STREAM_PROF
            const uint64_t c1 = __builtin_amdgcn_s_memtime();
#endif
            if (wave0) thr_decide_chunk(codes + (k & 1) * HS_CH, ring, q0, lo, hi, M, IM, T, prev, hc.passbits);
#ifdef SF_STREAM_PROF
            const uint64_t c2 = __builtin_amdgcn_s_memtime();
#endif
            if (more) thr_store(r, codes + ((k + 1) & 1) * HS_CH);
            __syncthreads();
#ifdef SF_STREAM_PROF
            const uint64_t c3 = __builtin_amdgcn_s_memtime();
            t_ld += c1 - c0; t_dec += c2 - c1; t_wait += c3 - c2;
#endif
        }
#ifdef SF_STREAM_PROF
        if (threadIdx.x == 0)
            printf("SF_STREAM_PROF seg %u events %u chunks %u: issue %lu decide %lu store+barrier %lu cycles\n", s,
                   hi - lo, nch, (unsigned long)t_ld, (unsigned long)t_dec, (unsigned long)t_wait);
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
