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
// LDS: THREAD records 2 x 24 KiB + live-exit ring 16 KiB; RL timestamps 2 x 16 KiB + counts 2 x 8 KiB
constexpr int HS_LDS_WORDS = (2 * HS_CH * 8 + 2 * HS_CH * 4) / 8;   // RL: 48 KiB as u64 words
constexpr uint32_t CODE_EXIT = 0x80000000u;
constexpr uint32_t CODE_DEAD = 0x7fffffffu;   // exit distance field: entry not in this segment (never live)

struct StreamCtx {
    const uint32_t* list; const uint32_t* n_list;   // n_list[0] front count, n_list[1] back count
    uint32_t seg_cap;
    uint64_t* sticks;
    uint32_t* next;                                 // work queue head (k_heavy_stream)
};

__device__ __forceinline__ bool stream_at(const StreamCtx& sc, uint32_t b, uint32_t* s) {
    const uint32_t nf = sc.n_list[0], nb = sc.n_list[1];
    if (b < nf) { *s = sc.list[b]; return true; }
    if (b < nf + nb) { *s = sc.list[sc.seg_cap - 1 - (b - nf)]; return true; }
    return false;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not
// for its outstanding global stores and atomics (the pass bits are read by
// later kernels; far live exits are fenced explicitly where they are written).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
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
#ifndef SF_THR_WPC
#define SF_THR_WPC 48
#endif
constexpr int THR_WPC = SF_THR_WPC;               // windows per chunk (16 per helper wave, <= 64 lanes)
constexpr uint32_t THR_CH = THR_WPC * 64;          // events per chunk
constexpr uint32_t XO_NONE = 0xffffffffu;
constexpr int32_t THR_CSMALL = 8;                  // scalar walk for acquireCount <= 8
constexpr int32_t THR_CBIG = 1 << 20;              // integer compares exact below this (no int wrap)

struct ThrWin {                                    // 24 B per window
    unsigned long long ent;                        // entries
    unsigned long long inw;                        // exits whose entry is in this window
    int32_t maxrc;                                 // bound of max over entries of rank + acquireCount
    uint32_t flags;                                // bit 0: an acquireCount > 8, bit 1: > THR_CBIG, bit 2: > 1
};

// Event record (k_thr_rec, one per event of a window-walk THREAD segment, 8 B):
//   entry: x = sorted position of its exit (or XO_NONE), y = acquireCount (>= 1)
//   exit:  x = distance back to its entry in the segment (0: none), y = THR_REC_EXIT
//          (| THR_REC_LIVE: the entry was decided earlier, the exit is live)
constexpr uint32_t THR_REC_EXIT = 0x80000000u;
constexpr uint32_t THR_REC_LIVE = 1u;

struct ThrLds {
    unsigned long long lx[LX_WORDS];               // live exits of window (pos - lo) / 64 at word % LX_WORDS
    ThrWin win[2][THR_WPC];
    uint2 rec[2][THR_CH];                          // event records of the chunk
};
__device__ __forceinline__ uint32_t rec_xo(uint2 r) { return r.x; }                    // entries
__device__ __forceinline__ int32_t rec_c(uint2 r) { return (int32_t)r.y; }              // entries
__device__ __forceinline__ int rec_d(uint2 r) {                                         // exits: distance, or 0
    return (r.y & THR_REC_EXIT) && r.x < 65536u ? (int)r.x : 0;
}
static_assert(THR_WPC % 3 == 0 && THR_WPC <= 64, "one decider lane per window, windows split over 3 helpers");
// the kernel's LDS: the larger of the THREAD and RateLimiter layouts
constexpr int HS_SMEM_WORDS = (int)(sizeof(ThrLds) + 7) / 8 > HS_LDS_WORDS ? (int)(sizeof(ThrLds) + 7) / 8 : HS_LDS_WORDS;

__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t uniform64_at(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ unsigned long long rl64(unsigned long long v, int l) {
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((unsigned long long)b << 32) | a;
}

__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long v) {
    return (unsigned long long)uniform64((int64_t)v);
}

// Helper wave h (1..3): prepare windows h-1, h+2, ... of the chunk starting at
// q0.  Two steps, software-pipelined one chunk ahead: thr_issue puts every
// global load of the wave's windows in flight (indices clamped into the
// segment instead of branches), thr_finish (one chunk later, after the loads
// have landed) builds the window summaries in LDS.  Far live-exit words may be
// read that early: a far mark lands at least LX_WORDS - 1 windows past the
// entry that makes it, and the decider fences those before each barrier.
constexpr int THR_WPW = THR_WPC / 3;              // windows per helper wave
struct ThrPre {
    uint2 rec[THR_WPW];
    unsigned long long f0, f1;                     // far live-exit words of window k in lane k
};
__device__ __forceinline__ void thr_issue(ThrPre& P, const uint2* rec, const unsigned long long* lxfar,
                                          uint32_t q0, uint32_t hi, int h) {
    const int lane = (int)(threadIdx.x & 63);
#pragma unroll
    for (int k = 0; k < THR_WPW; k++) {
        const uint32_t q = min(q0, hi) + 64u * (uint32_t)(h - 1 + 3 * k);
        P.rec[k] = rec[min(q + (uint32_t)lane, hi - 1)];
    }
    // the two far-bitmap words under window k, loaded by lane k (two loads per chunk)
    const uint32_t qk = min(q0, hi) + 64u * (uint32_t)(h - 1 + 3 * min(lane, THR_WPW - 1));
    const uint32_t g = min(qk, hi - 1) >> 6;
    P.f0 = __hip_atomic_load(lxfar + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    P.f1 = __hip_atomic_load(lxfar + g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ void thr_finish(ThrLds& L, int buf, const ThrPre& P, uint32_t q0, uint32_t lo, uint32_t hi, int h) {
    const int lane = (int)(threadIdx.x & 63);
#pragma unroll
    for (int k = 0; k < THR_WPW; k++) {
        const int wl = h - 1 + 3 * k;
        const uint32_t q = q0 + 64u * (uint32_t)wl;
        if (q >= hi) break;
        const bool valid = q + (uint32_t)lane < hi;
        const uint2 r = P.rec[k];
        const bool ex = valid && (r.y & THR_REC_EXIT);
        const bool ent = valid && !(r.y & THR_REC_EXIT);
        const int32_t c = (int32_t)r.y;
        ThrWin wn;
        wn.ent = __ballot(ent);
        wn.inw = __ballot(ex && r.x >= 1u && r.x <= (uint32_t)lane);
        const bool gt1 = __ballot(ent && c > 1) != 0ull, gt8 = __ballot(ent && c > THR_CSMALL) != 0ull;
        wn.flags = (gt8 ? 1u : 0u) | (__ballot(ent && c > THR_CBIG) ? 2u : 0u) | (gt1 ? 4u : 0u);
        // bound of max(rank + acquireCount): (entries - 1) + (1, or 8 when some count is 2..8)
        wn.maxrc = gt8 ? INT32_MAX : (int32_t)__popcll(wn.ent) - 1 + (gt1 ? THR_CSMALL : 1);
        L.rec[buf][64 * wl + lane] = valid ? r : make_uint2(XO_NONE, THR_REC_EXIT);
        const unsigned long long mo = __ballot(ex && (r.y & THR_REC_LIVE));   // entry of an earlier batch: live
        const unsigned long long f0 = rl64(P.f0, k), f1 = rl64(P.f1, k);
        if (lane == 0) {
            L.win[buf][wl] = wn;
            // live exits of far-away entries (written into HBM when those entries passed)
            const uint32_t sh = q & 63;
            const unsigned long long far = sh ? (f0 >> sh) | (f1 << (64 - sh)) : f0;
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
// inclusive scans over the 64 lanes of a wavefront (DPP: row shifts, then row broadcasts)
__device__ __forceinline__ int wave_scan_add(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);     // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);     // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);     // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);     // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);     // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);     // row_bcast:31
    return v;
}
__device__ __forceinline__ int wave_scan_max(int v) {
    constexpr int ID = INT32_MIN;
    v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(ID, v, 0x143, 0xc, 0xf, false));
    return v;
}

// One window of a THREAD segment with every acquireCount in 1..8, no int
// wrap and room0 = floor(count) - T >= 0, decided in wavefront steps instead
// of a walk.  With entries of acquireCount 1 taken as attempted +1 steps and
// live exits as -1 steps, the thread count is the walk reflected at the cap
// (a blocked entry is an absorbed step): with V the prefix sum of the steps,
// the room before event k is  max(room0, max_{j<k} V_j (and 0)) - V_{k-1}.
// Entries with acquireCount > 1 are taken as blocked unless known to pass
// ("forced"), and exits of this window's own entries as dead unless known
// live.  A round is exact up to the first event where either guess is
// refuted: the first non-forced entry that has room for its acquireCount
// (it passes: forced), or the first exit whose entry passed (live).  Each
// refutation is a fact, so the rounds converge, to the serial outcome (every
// fixed point agrees with the serial decisions event by event).
__device__ __forceinline__ unsigned long long thr_window_solve(int room0, unsigned long long me,
                                                               unsigned long long& ml, int32_t c, int eln) {
    const int lane = (int)(threadIdx.x & 63);
    const bool ent = (me >> lane) & 1ull;
    const bool one = ent && c == 1, multi = ent && c > 1;
    const bool inx = eln < 64;
    const int el6 = eln & 63;
    unsigned long long forced = 0, pm = 0;
    while (true) {
        const bool live = (ml >> lane) & 1ull;
        const bool fo = (forced >> lane) & 1ull;
        const int x = (one || fo) ? 1 : (live ? -1 : 0);
        const int v = wave_scan_add(x);
        const int vex = v - x;
        const int room = max(room0, wave_scan_max(vex)) - vex;     // room before this event
        pm = __ballot((one && room >= 1) || fo);
        const unsigned long long mis = __ballot(multi && !fo && room >= c);
        const int j1 = mis ? __ffsll((long long)mis) - 1 : 64;
        const bool nx = inx && !live && ((pm >> el6) & 1ull);      // exit of a (guessed) passed entry
        const unsigned long long nw = __ballot(nx && eln < j1);
        const int ne = nw ? __ffsll((long long)nw) - 1 : 64;
        if (j1 == 64 && ne == 64) break;
        const int F = min(j1, ne);                                  // events before F are exact
        ml |= __ballot(nx && eln < F);
        if (j1 < ne) forced |= 1ull << j1;
    }
    return pm;
}

// Run mode: a chunk made of few long runs of entries and of exits (a
// saturated head resource whose events of each millisecond are its entries,
// then its exits) is decided run by run instead of window by window.
//   - a run of entries only adds threads: with room R = floor(count) - T, the
//     passes are the greedy left-to-right choice of entries with
//     acquireCount <= R, R falling by one per pass -- every entry of
//     acquireCount 1 up to the R-th one, plus the few larger counts that still
//     fit, found 64 entries at a time with ballots (no scan);
//   - a run of exits only releases threads: T falls by the number of live
//     exits in it, one vector read of its live-exit words and a wave sum.
// The exits of a run's passed entries are marked live before the next run is
// read (same wave, LDS order), so a run of exits always sees every entry
// before it.  Applies to chunks of at most THR_RUNS runs, without an
// acquireCount > THR_CBIG and with T far from int wrap; other chunks use the
// window walk below, which keeps the same state (T, the live-exit ring).
#ifndef SF_THR_RUNS
#define SF_THR_RUNS 40
#endif
constexpr int THR_RUNS = SF_THR_RUNS;

// Decide chunk [q0, q0 + 64 nwin) in run mode (thr_decide checked that it applies).
__device__ __forceinline__ void thr_decide_runs(ThrLds& L, int buf, unsigned long long* lxfar, uint32_t q0,
                                                uint32_t lo, uint32_t hi, int64_t IM, int64_t& T,
                                                unsigned long long r_ent, uint32_t nwin, uint32_t slot0,
                                                unsigned long long& pst, bool& far_marked) {
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t nev = min(hi - q0, 64u * nwin);
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t p = 0;
    while (p < nev) {
        const uint32_t w = p >> 6, b = p & 63;
        const bool is_ent = (rl64(r_ent, (int)w) >> b) & 1ull;
        // the run's end: the first later event of the other kind (or the chunk's end)
        unsigned long long x = (uint32_t)lane < nwin ? (is_ent ? ~r_ent : r_ent) : ~0ull;
        if ((uint32_t)lane < w) x = 0ull;
        else if ((uint32_t)lane == w) x &= ~0ull << b;
        const unsigned long long mw = __ballot(x != 0ull);
        const int l = __ffsll((long long)mw) - 1;
        const uint32_t e = min(64u * (uint32_t)l + (uint32_t)__builtin_ctzll(rl64(x, l)), nev);
        if (is_ent) {
            int64_t R = IM - T;
            for (uint32_t g = p; g < e && R > 0; g += 64) {
                const uint32_t k = g + (uint32_t)lane;
                const bool valid = k < e;
                const uint2 rc = valid ? L.rec[buf][k] : make_uint2(XO_NONE, 1u);
                const int32_t c = (int32_t)rc.y;
                const unsigned long long vm = __ballot(valid);
                const unsigned long long big = __ballot(valid && c > 1);
                const unsigned long long ones = vm & ~big;
                unsigned long long pm = 0;
                int from = 0;
                // every entry fits even after all earlier ones of the group passed
                const bool allfit = !__ballot(valid && c > THR_CSMALL) &&
                                    R >= (int64_t)__popcll(vm) - 1 + (big ? THR_CSMALL : 1);
                if (allfit) { pm = vm; R -= __popcll(vm); }
                else while (true) {
                    const unsigned long long bz = big & (from < 64 ? ~0ull << from : 0ull);
                    const int z = bz ? __ffsll((long long)bz) - 1 : 64;
                    const unsigned long long m1 = ones & (from < 64 ? ~0ull << from : 0ull) &
                                                  (z < 64 ? (1ull << z) - 1ull : ~0ull);
                    const int n1 = __popcll(m1);
                    if ((int64_t)n1 >= R) {                    // the first R of them pass, then R = 0
                        const int rank = __popcll(m1 & below);
                        pm |= __ballot(((m1 >> lane) & 1ull) && (int64_t)rank < R);
                        R = 0;
                        break;
                    }
                    pm |= m1; R -= n1;
                    if (z == 64) break;
                    if ((int64_t)__builtin_amdgcn_readlane(c, z) <= R) { pm |= 1ull << z; R -= 1; }
                    from = z + 1;
                    if (R == 0) break;
                }
                R = uniform64(R);
                if (pm) {
                    T += __popcll(pm);
                    const bool mk = ((pm >> lane) & 1ull) && rc.x != XO_NONE && rc.x < hi;
                    bool fm2 = false;
                    if (mk) fm2 = thr_mark_exit(L, lxfar, rc.x, q0, lo);
                    far_marked |= __ballot(fm2) != 0ull;
                    // pass bits staged per window (lane w <-> window w)
                    const uint32_t gw = g >> 6, sh = g & 63;
                    if ((uint32_t)lane == gw) pst |= pm << sh;
                    if (sh && (uint32_t)lane == gw + 1) pst |= pm >> (64 - sh);
                }
            }
            T = uniform64(T);
        } else {
            // live exits of [p, e): their ring words, edges masked
            int64_t nl = 0;
            for (uint32_t w0 = w; 64u * w0 < e; w0 += 64) {
                const uint32_t ww = w0 + (uint32_t)lane;
                unsigned long long v = 0;
                if (64u * ww < e) {
                    v = L.lx[(slot0 + ww) % LX_WORDS];
                    if (ww == w) v &= ~0ull << b;
                    const uint32_t lim = e - 64u * ww;             // events of this word inside the run
                    if (lim < 64u) v &= (1ull << lim) - 1ull;
                }
                const int s = wave_scan_add(__popcll(v));
                nl += __builtin_amdgcn_readlane(s, 63);
            }
            T = uniform64(T - nl);
        }
        p = e;
    }
    if ((uint32_t)lane < nwin) L.lx[(slot0 + (uint32_t)lane) % LX_WORDS] = 0ull;   // the chunk's words consumed
}

// THR_SW consecutive windows whose entries all fit are taken in one step.
constexpr int THR_SW = 4;
#ifndef SF_SOLVE_MIN_ROOM
#define SF_SOLVE_MIN_ROOM 0
#endif

__device__ void thr_decide(ThrLds& L, int buf, unsigned long long* lxfar, uint32_t q0, uint32_t lo, uint32_t hi,
                           double M, int64_t IM, int64_t& T, unsigned long long* pbits
#ifdef SF_STREAM_PROF
                           , uint64_t* prof
#endif
                           ) {
#ifdef SF_STREAM_PROF
    const uint64_t ta = __builtin_amdgcn_s_memtime();
#endif
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t nwin = min((hi - q0 + 63) / 64, (uint32_t)THR_WPC);
    bool far_marked = false;
    unsigned long long pst = 0;
    T = uniform64(T);
    const int wl = lane < THR_WPC ? lane : 0;
    const unsigned long long r_ent = L.win[buf][wl].ent;
    const int32_t r_maxrc = L.win[buf][wl].maxrc;
    const uint32_t r_flags = L.win[buf][wl].flags;
    const unsigned long long r_inw = L.win[buf][wl].inw;
    const unsigned long long bigm = __ballot((uint32_t)lane < nwin && (r_flags & 2u));   // windows needing the exact walk
    const uint32_t slot0 = (q0 - lo) >> 6;
    // live-exit words of the chunk's windows in registers (lane w <-> window w);
    // only this chunk's own passes can add to them (exits inside the chunk)
    unsigned long long r_lx = (uint32_t)lane < nwin ? L.lx[(slot0 + lane) % LX_WORDS] : 0ull;
    const uint32_t qend = q0 + 64u * nwin;
    uint32_t w = 0;
#ifdef SF_STREAM_PROF
    const uint64_t tb = __builtin_amdgcn_s_memtime();
#endif
    {
        // run mode (thr_decide_runs) for a chunk of few runs: count the runs
        // (kind changes between neighbouring events, inside and across words)
        const bool act = (uint32_t)lane < nwin;
        const unsigned long long b0 = __ballot(act && (r_ent & 1ull)), bt = __ballot(act && (r_ent >> 63));
        const int inner = wave_scan_add(act ? __popcll((r_ent ^ (r_ent << 1)) & ~1ull) : 0);
        const unsigned long long edge = nwin > 1 ? ((b0 >> 1) ^ bt) & ((1ull << (nwin - 1)) - 1ull) : 0ull;
        const int runs = 1 + __builtin_amdgcn_readlane(inner, 63) + __popcll(edge);
        const int64_t span = 64 * THR_WPC;
        if (!bigm && runs <= THR_RUNS && T >= (int64_t)INT32_MIN + span &&
            T + (int64_t)THR_CBIG + span <= (int64_t)INT32_MAX) {
            thr_decide_runs(L, buf, lxfar, q0, lo, hi, IM, T, r_ent, nwin, slot0, pst, far_marked);
            w = nwin;
#ifdef SF_STREAM_PROF
            prof[5]++;
#endif
        }
    }
    while (w < nwin) {
        const uint32_t q = q0 + 64 * w;
        const int64_t room0 = IM - T;
        const bool tsmall = T >= (int64_t)INT32_MIN + 64 && T + (int64_t)THR_CBIG + 64 <= (int64_t)INT32_MAX;
        {
            // a run of windows without entries: their live exits only release threads
            const unsigned long long noent = __ballot((uint32_t)lane < nwin && r_ent == 0ull) >> w;
            if (noent & 1ull) {
                const uint32_t e = min(w + (uint32_t)(__ffsll((long long)~noent) - 1), nwin);
                const bool in = (uint32_t)lane >= w && (uint32_t)lane < e;
                const int nl = wave_scan_add(in ? __popcll(r_lx) : 0);
                T = uniform64(T - (int64_t)__builtin_amdgcn_readlane(nl, 63));
                if (in) L.lx[(slot0 + (uint32_t)lane) % LX_WORDS] = 0ull;
                w = e;
#ifdef SF_STREAM_PROF
                prof[9]++;
#endif
                continue;
            }
        }
        if (room0 <= 0 && tsmall) {
            // saturated: skip the windows with no live exit (all their entries block)
            const unsigned long long stop = (__ballot((uint32_t)lane < nwin && r_lx != 0ull) | bigm) >> w;
#ifdef SF_STREAM_PROF
            prof[9]++;
#endif
            if (!stop) { w = nwin; break; }
            const uint32_t k = (uint32_t)(__ffsll((long long)stop) - 1);
            // The first window with live exits, x: when all of them follow its last
            // entry, its entries block too and the exits only release threads, as
            // do the live exits of the entry-free windows after it.  The skipped
            // run, x and that entry-free run are taken in this one step.
            const uint32_t x = w + k;
            const bool tail = r_lx != 0ull &&
                              (r_ent == 0ull || 63 - (int)__builtin_clzll(r_ent) < (int)__builtin_ctzll(r_lx));
            const unsigned long long tailm = __ballot((uint32_t)lane < nwin && tail) & ~bigm;
            if ((tailm >> x) & 1ull) {
                const unsigned long long ne = __ballot((uint32_t)lane < nwin && r_ent == 0ull) >> (x + 1);
                const uint32_t e = min(x + 1 + (uint32_t)(__ffsll((long long)~ne) - 1), nwin);
                const bool in = (uint32_t)lane >= x && (uint32_t)lane < e;
                const int nl = wave_scan_add(in ? __popcll(r_lx) : 0);
                T = uniform64(T - (int64_t)__builtin_amdgcn_readlane(nl, 63));
                if (in) L.lx[(slot0 + (uint32_t)lane) % LX_WORDS] = 0ull;
                w = e;
                continue;
            }
            if (k > 0) { w += k; continue; }
        }
        const unsigned long long me = rl64(r_ent, (int)w);
        const uint32_t flags = (uint32_t)__builtin_amdgcn_readlane((int)r_flags, (int)w);
        const uint32_t slot = (slot0 + w) % LX_WORDS;
        if (w + THR_SW <= nwin && tsmall && room0 >= 64 && !((bigm >> w) & ((1ull << THR_SW) - 1ull))) {
            // ---- THR_SW windows whose entries all fit even with every earlier entry
            // of them holding a thread: all pass, every exit of them inside is live
            const bool inr = (uint32_t)lane >= w && (uint32_t)lane < w + THR_SW;
            const int ne_ = wave_scan_add(inr ? __popcll(r_ent) : 0);
            const int sument = __builtin_amdgcn_readlane(ne_, 63);
            const unsigned long long f1 = __ballot(inr && (r_flags & 1u)), f4 = __ballot(inr && (r_flags & 4u));
            if (!f1 && room0 >= (int64_t)sument - 1 + (f4 ? THR_CSMALL : 1)) {
                const uint32_t qe = q + 64u * THR_SW;
                bool anyin = false;
#pragma unroll
                for (int k = 0; k < THR_SW; k++) {
                    const int pos = 64 * k + lane;
                    const uint2 rk = L.rec[buf][64 * (w + k) + lane];
                    const uint32_t xo_k = rec_xo(rk);
                    const int d = rec_d(rk);
                    const unsigned long long me_k = rl64(r_ent, (int)w + k);
                    const unsigned long long ml_k = rl64(r_lx, (int)w + k) | __ballot(d >= 1 && d <= pos);
                    T += (int64_t)__popcll(me_k) - (int64_t)__popcll(ml_k);
                    // exits beyond the superwindow of its passed entries turn live
                    const bool mk = ((me_k >> lane) & 1ull) && xo_k != XO_NONE && xo_k < hi && xo_k >= qe;
                    bool fm2 = false;
                    if (mk) fm2 = thr_mark_exit(L, lxfar, xo_k, q, lo);
                    far_marked |= __ballot(fm2) != 0;
                    anyin |= __ballot(mk && xo_k < qend) != 0ull;
                    if ((uint32_t)lane == w + (uint32_t)k) pst = me_k;
                }
                T = uniform64(T);
                if (anyin) r_lx |= ((uint32_t)lane >= w + THR_SW && (uint32_t)lane < nwin) ? L.lx[(slot0 + lane) % LX_WORDS] : 0ull;
                if (inr) L.lx[(slot0 + (uint32_t)lane) % LX_WORDS] = 0ull;
                w += THR_SW;
#ifdef SF_STREAM_PROF
                prof[4]++;
#endif
                continue;
            }
        }
        unsigned long long ml = rl64(r_lx, (int)w);            // live exits of this window
        const int32_t maxrc = __builtin_amdgcn_readlane(r_maxrc, (int)w);
        unsigned long long pmask = 0;
        const bool nowrap = !(flags & 2u) && tsmall;
        if (nowrap && room0 + (int64_t)__popcll(ml) < 1) {
            // even with every live exit first, no entry fits (acquireCount >= 1):
            // all entries block, so no exit of this window's entries turns live
            T -= __popcll(ml);
        } else {
            const uint2 rw = L.rec[buf][64 * w + lane];
            const uint32_t xo = rec_xo(rw);
            if (nowrap && room0 >= (int64_t)maxrc) {
                // the thread count before an entry is <= T + (entries before it): all fit
                pmask = me;
                ml |= rl64(r_inw, (int)w);                 // exits of this window's entries, inside it
                T += (int64_t)__popcll(me) - (int64_t)__popcll(ml);
            } else if (nowrap && !(flags & 1u) && room0 >= SF_SOLVE_MIN_ROOM) {
                const int32_t c = rec_c(rw);
                const int dd = rec_d(rw);
                const int eln = (dd >= 1 && dd <= lane) ? lane - dd : 255;   // in-window entry lane
                pmask = thr_window_solve((int)room0, me, ml, c, eln);
                T += (int64_t)__popcll(pmask) - (int64_t)__popcll(ml);
            } else {
                const int32_t c = rec_c(rw);
                const bool small = nowrap && !(flags & 1u);
                const bool ones = nowrap && !(flags & 4u);  // every acquireCount is 1: scalar candidates
                // in-window exit of each entry lane: bit position, or 64
                const uint32_t inpos = (xo != XO_NONE && xo - q < 64u && xo > q + (uint32_t)lane) ? xo - q : 64u;
                const bool ent = (me >> lane) & 1ull;
                int cursor = 0;
                while (cursor < 64) {
                    unsigned long long fm = 0;
                    if (ones) {
                        fm = IM - T > 0 ? me : 0ull;
                    } else if (small) {
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
                const bool mk = ((pmask >> lane) & 1ull) && xo != XO_NONE && xo < hi && xo >= q + 64;
                bool fm2 = false;
                if (mk) fm2 = thr_mark_exit(L, lxfar, xo, q, lo);
                far_marked |= __ballot(fm2) != 0;
                if ((uint32_t)lane == w) pst = pmask;      // pass bits staged: lane w <-> window w
                if (__ballot(mk && xo < qend))             // exits inside this chunk: refresh its words
                    r_lx |= ((uint32_t)lane > w && (uint32_t)lane < nwin) ? L.lx[(slot0 + lane) % LX_WORDS] : 0ull;
            }
        }
        T = uniform64(T);
        if (lane == 0) L.lx[slot] = 0ull;                  // consumed: reused LX_WORDS windows later
        w++;
#ifdef SF_STREAM_PROF
        prof[7]++;
#endif
    }
#ifdef SF_STREAM_PROF
    const uint64_t tc = __builtin_amdgcn_s_memtime();
#endif
    if (pst) {                                             // the chunk's pass bits: one vector step
        const uint32_t q = q0 + 64u * (uint32_t)lane, sh = q & 63;
        atomicOr(pbits + (q >> 6), pst << sh);
        if (sh) atomicOr(pbits + (q >> 6) + 1, pst >> (64 - sh));
    }
    if (far_marked) {                                      // far exits must be in HBM before a loader reads them
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        __builtin_amdgcn_s_waitcnt(0);
    }
#ifdef SF_STREAM_PROF
    const uint64_t td = __builtin_amdgcn_s_memtime();
    prof[0] += tb - ta; prof[1] += tc - tb; prof[2] += td - tc;
#endif
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
        r.c[i] = (v && !(f[i] & (SF_EV_EXIT | EVF_SYSBLK))) ? r.c[i] : 0;   // 0: exit / blocked before / padding
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

// Passes of the deciding wave, staged one per lane and written 64 at a time:
// one vector atomic into the pass bits and one scattered store of the waits
// (instead of single-lane memory ops on the serial chain).
struct PassStage {
    unsigned long long* pbits; int32_t* wait; uint32_t n;
    uint32_t spos; int32_t sw;
    __device__ __forceinline__ void flush() {
        const uint32_t k = n & 63u;
        if ((threadIdx.x & 63u) < (k ? k : 64u)) {
            atomicOr(pbits + (spos >> 6), 1ull << (spos & 63));
            wait[spos] = sw;
        }
    }
    __device__ __forceinline__ void push(uint32_t pos, int32_t w) {
        if ((threadIdx.x & 63u) == (n & 63u)) { spos = pos; sw = w; }
        n++;
        if ((n & 63u) == 0) flush();
    }
    __device__ __forceinline__ void finish() { if (n & 63u) flush(); }
};

__device__ __forceinline__ void rl_decide_chunk(const int64_t* tsb, const int32_t* cb, uint32_t q0, uint32_t hi,
                                                const DevRule& rule, int64_t cost1, int64_t& L, PassStage& iw) {
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t n = min(hi - q0, (uint32_t)HS_CH);
    uint32_t p = 0;
    while (p < n) {
        // cost(c) >= cost(1) for c >= 1: nothing before this time can pass
        p = lds_first_ge(tsb, p, n, L + cost1 - rule.max_queue_ms);
        if (p >= n) break;
        // 64 events into registers; L only grows, so an event that is not a
        // candidate now never becomes one: the window is settled in one visit
        const uint32_t k = p + (uint32_t)lane;
        const int32_t c = k < n ? cb[k] : 0;
        const int64_t t = k < n ? tsb[k] : 0;
        const int64_t cost = c == 1 ? cost1 : (c > 0 ? j_round(1.0 * c / rule.count * 1000) : 0);
        int from = 0;
        while (true) {
            const unsigned long long m = __ballot(c > 0 && lane >= from && t >= L + cost - rule.max_queue_ms);
            if (!m) break;
            const int jj = __ffsll((long long)m) - 1;
            const int64_t cj = uniform64_at(cost, jj), tj = uniform64_at(t, jj);
            int32_t wait = 0;
            if (L + cj <= tj) L = tj;                           // expectedTime <= currentTime
            else { L += cj; wait = (int32_t)(L - tj); }         // queued: sleep(wait), then pass
            iw.push(q0 + p + (uint32_t)jj, wait);
            from = jj + 1;
        }
        p += 64;
    }
}

// ------------------------------------------------------------ THREAD run mode
// A THREAD segment whose runs are long on average (thr_run_mode; the config-3
// head resource: every millisecond its entries, then its exits) is decided
// run by run from tables prepared ahead of it (k_thr_rid, k_thr_rec), by
// wave 0 alone:
//   - a run of exits releases the live exits in it: a counter per run (an LDS
//     ring of RUN_RC runs; farther ones in run_pre, with the exits whose entry
//     passed before this batch), so the run costs one LDS read whatever its length;
//   - a run of entries with room R = floor(count) - T > 0 passes entries
//     greedily (thr_group_passes), 64 at a time, until R is 0; each pass adds
//     one to the counter of its exit's run.  With no room the run is skipped.
// The run table (start, run_pre) is read 64 runs per load, two loads ahead;
// the first 64 entry records of each entry run of the next 64 runs are loaded
// into registers one table step ahead and parked in LDS, so the chain waits on
// global memory only when one run passes more than 64 entries.
constexpr uint32_t RUN_RC = 8192;                  // live-exit counters: runs ahead of the walk (32 KiB)
constexpr int THR_RG = 8;                          // groups of an entry run loaded together past the staged one
struct RunLds {
    uint32_t cnt[RUN_RC];
    uint2 stage[2][32][64];                        // first 64 records of each entry run of a table step
};
static_assert(sizeof(RunLds) <= sizeof(unsigned long long) * (size_t)HS_SMEM_WORDS, "run mode LDS");

// passes of one group of 64 entries (valid lanes) with room R > 0; R is lowered.
// The greedy walk runs on wave-uniform masks (scalar unit): every entry of
// acquireCount 1 before the next larger count passes while room is left; a
// larger count passes iff it fits.
__device__ __forceinline__ unsigned long long thr_group_passes(bool valid, int32_t c, int64_t& R) {
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long vm = __ballot(valid);
    const unsigned long long big = __ballot(valid && c > 1);
    const int nv = __popcll(vm);
    // every entry fits even after all earlier ones of the group passed
    if (!__ballot(valid && c > THR_CSMALL) && R >= (int64_t)nv - 1 + (big ? THR_CSMALL : 1)) {
        R -= nv;
        return vm;
    }
    const int r0 = __builtin_amdgcn_readfirstlane((int)(R < (1 << 30) ? R : (1 << 30)));
    int r = r0;
    const unsigned long long ones = vm & ~big;
    unsigned long long pm = 0, rest = vm;                  // entries not yet visited
    while (r > 0 && rest) {
        const unsigned long long bz = big & rest;
        const int z = bz ? __ffsll((long long)bz) - 1 : 64;
        const unsigned long long m1 = ones & rest & (z < 64 ? (1ull << z) - 1ull : ~0ull);
        const int n1 = __popcll(m1);
        if (n1 >= r) {                                     // the first r of them pass, then no room
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
            pm |= __ballot(((m1 >> lane) & 1ull) && (int)below < r);
            r = 0;
            break;
        }
        pm |= m1; r -= n1;
        if (z == 64) break;
        if (__builtin_amdgcn_readlane(c, z) <= r) { pm |= 1ull << z; r -= 1; }
        rest = z < 63 ? rest & (~0ull << (z + 1)) : 0ull;
    }
    R -= (int64_t)(r0 - r);
    return pm;
}

// the same with Java's int arithmetic, entry by entry: (int)(T + c) <= count
// (DefaultController.canPass); only when T may leave the int range
__device__ __forceinline__ unsigned long long thr_group_passes_exact(bool valid, int32_t c, int64_t T, double M) {
    unsigned long long vm = __ballot(valid), pm = 0;
    while (vm) {
        const int z = __ffsll((long long)vm) - 1;
        vm &= vm - 1;
        const int32_t cz = __builtin_amdgcn_readlane(c, z);
        if ((double)(int32_t)((uint32_t)(int32_t)T + (uint32_t)cz) <= M) { pm |= 1ull << z; T += 1; }
    }
    return pm;
}

template <bool EXACT>
__device__ void thr_runs_segment(const DevState& st, const SegIO& io, const HeavyCtx& hc, uint32_t s, uint32_t lo,
                                 uint32_t hi, uint32_t res, double M, RunLds& L) {
    constexpr bool wrapsafe = !EXACT;
    const int64_t IM = (int64_t)floor(M);
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t rb = hc.seg_rb[s], nr = hc.seg_re[s] - rb;
    // runs alternate kinds: run k holds entries iff (k & 1) == e0
    const uint32_t e0 = is_checked_entry(io.flags[lo]) ? 0u : 1u;
    int64_t T = uniform64(st.threads[res]);
    unsigned long long* pbits = hc.passbits;
    const uint2* rrec = hc.rrec;
    auto tbl = [&](uint32_t c, uint32_t& ts, uint32_t& tp) {
        const uint32_t k = 64u * c + (uint32_t)lane;
        ts = k < nr ? hc.run_start[rb + k] : hi;
        tp = k < nr ? __hip_atomic_load(hc.run_pre + rb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    };
    uint2 sr[32];                                  // staged first records of the entry runs of a table step
    auto stage_issue = [&](uint32_t ts) {
#pragma unroll
        for (int i = 0; i < 32; i++) {
            const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)ts, 2 * i + (int)e0);
            sr[i] = rrec[min(a + (uint32_t)lane, hi - 1)];
        }
    };
    auto stage_park = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 32; i++) L.stage[buf][i][lane] = sr[i];
    };
    const uint32_t nchunk = (nr + 63) / 64;
    uint32_t s0, p0, s1, p1, s2, p2;
    tbl(0, s0, p0);
    tbl(1, s1, p1);
    stage_issue(s0);
    stage_park(0);
    bool far = false;
#ifdef SF_STREAM_PROF
    uint64_t pf[8] = {0, 0, 0, 0, 0, 0, 0, 0};     // cycles: table steps, exit runs, entry runs; counts: exit runs, entry runs with room, groups
    const uint64_t pt0 = __builtin_amdgcn_s_memtime();
#endif
    for (uint32_t c = 0; c < nchunk; c++) {
#ifdef SF_STREAM_PROF
        const uint64_t pa = __builtin_amdgcn_s_memtime();
#endif
        if (far) {                                 // counters of far runs must be in HBM before their table loads
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
            __builtin_amdgcn_s_waitcnt(0);
            far = false;
        }
        tbl(c + 2, s2, p2);
        stage_issue(s1);
        const int buf = (int)(c & 1);
        const uint32_t kn = min(64u, nr - 64u * c);
        const uint32_t next0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)s1);
#ifdef SF_STREAM_PROF
        uint64_t pb = __builtin_amdgcn_s_memtime();
        pf[0] += pb - pa;
#endif
        for (uint32_t k = 0; k < kn; k++) {
            const uint32_t r = rb + 64u * c + k;                     // global run id
            const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)s0, (int)k);
            const uint32_t e = k + 1 < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)s0, (int)k + 1) : next0;
            if ((k & 1u) != e0) {
                // exits: release the live ones (marked by earlier passes, or from before the batch)
                const uint32_t slot = r % RUN_RC;
                const uint32_t cl = (uint32_t)__builtin_amdgcn_readfirstlane((int)L.cnt[slot]);
                const uint32_t nl = cl + (uint32_t)__builtin_amdgcn_readlane((int)p0, (int)k);
                if (lane == 0) L.cnt[slot] = 0u;
                T -= (int64_t)nl;
#ifdef SF_STREAM_PROF
                { const uint64_t pc = __builtin_amdgcn_s_memtime(); pf[1] += pc - pb; pb = pc; pf[3]++; }
#endif
                continue;
            }
            int64_t R = wrapsafe ? IM - T : 1;           // (exact path: every entry is tried)
#ifdef SF_STREAM_PROF
            if (R > 0) pf[4]++;
#endif
            // one group of 64 entries from g: passes, their exits' run counters, pass bits
            auto group = [&](uint2 rc, uint32_t g) {
                const bool valid = g + (uint32_t)lane < e;
                unsigned long long pm;
                if constexpr (!EXACT) pm = thr_group_passes(valid, (int32_t)rc.y, R);
                else pm = thr_group_passes_exact(valid, (int32_t)rc.y, T, M);   // (T + acquireCount may wrap)
#ifdef SF_STREAM_PROF
                pf[5]++;
#endif
                if (!pm) return;
                T += __popcll(pm);
                const bool mk = ((pm >> lane) & 1ull) && rc.x != XO_NONE;
                bool fm = false;
                if (mk) {
                    if (rc.x - r < RUN_RC - 1) atomicAdd(&L.cnt[rc.x % RUN_RC], 1u);
                    else { atomicAdd(hc.run_pre + rc.x, 1u); fm = true; }
                }
                far |= __ballot(fm) != 0ull;
                const uint32_t sh = g & 63;
                if (lane == 0) atomicOr(pbits + (g >> 6), pm << sh);
                if (lane == 1 && sh) atomicOr(pbits + (g >> 6) + 1, pm >> (64 - sh));
            };
            if (R > 0) group(L.stage[buf][k >> 1][lane], a);            // the staged first group
            // more room than the first group used: the rest of the run from HBM,
            // THR_RG groups per round with all their loads in flight
            for (uint32_t g = a + 64; g < e && R > 0; g += 64 * THR_RG) {
                uint2 nx[THR_RG];
#pragma unroll
                for (int i = 0; i < THR_RG; i++) nx[i] = rrec[min(g + 64u * (uint32_t)i + (uint32_t)lane, hi - 1)];
#pragma unroll
                for (int i = 0; i < THR_RG; i++) {
                    if (g + 64u * (uint32_t)i >= e || R <= 0) break;
                    group(nx[i], g + 64u * (uint32_t)i);
                }
            }
            T = uniform64(T);
#ifdef SF_STREAM_PROF
            { const uint64_t pc = __builtin_amdgcn_s_memtime(); pf[2] += pc - pb; pb = pc; }
#endif
        }
#ifdef SF_STREAM_PROF
        const uint64_t pd = __builtin_amdgcn_s_memtime();
#endif
        stage_park(buf ^ 1);
#ifdef SF_STREAM_PROF
        pf[0] += __builtin_amdgcn_s_memtime() - pd;
#endif
        s0 = s1; p0 = p1; s1 = s2; p1 = p2;
    }
#ifdef SF_STREAM_PROF
    if (lane == 0)
        printf("SF_RUN_PROF seg %u events %u runs %u: total %lu table %lu exit-runs %lu (%lu) entry-runs %lu (%lu with room, %lu groups)\n",
               s, hi - lo, nr, (unsigned long)(__builtin_amdgcn_s_memtime() - pt0), (unsigned long)pf[0],
               (unsigned long)pf[1], (unsigned long)pf[3], (unsigned long)pf[2], (unsigned long)pf[4], (unsigned long)pf[5]);
#endif
}

__device__ void stream_segment(const DevState& st, const SegIO& io, const HeavyCtx& hc, const StreamCtx& sc,
                               uint32_t s, uint32_t b, unsigned long long* smem) {
    const uint64_t t_start = sc.sticks ? wall_clock64() : 0;
    const uint32_t lo = hc.seg_start[s], hi = hc.seg_start[s + 1], res = hc.seg_res[s];
    const uint32_t r0 = st.rule_off[res];
    const DevRule rule = st.rules[r0];
    const bool wave0 = threadIdx.x < 64;
    const uint32_t nch = (hi - lo + HS_CH - 1) / HS_CH;
    // the deciding wave is the serial chain: it wins issue arbitration on its
    // SIMD against the memory-bound waves of the concurrent kernels
    if (wave0) __builtin_amdgcn_s_setprio(3);
    if (hc.seg_mode[s] == SM_THREAD && thr_run_mode(hc, s, lo, hi, hc.segflag[s])) {
        // (the run walk compares T + acquireCount with floor(count) in 64 bits,
        // exact while no int wrap can occur: T far from the int range; else
        // entry by entry in Java's int arithmetic)
        const int64_t T0 = st.threads[res], span = (int64_t)(hi - lo);
        const bool wrapsafe = T0 >= (int64_t)INT32_MIN + span && T0 + (int64_t)THR_CBIG + span <= (int64_t)INT32_MAX;
        RunLds& RL = *reinterpret_cast<RunLds*>(smem);
        for (uint32_t i = threadIdx.x; i < RUN_RC; i += HS_T) RL.cnt[i] = 0u;
        __syncthreads();
        if (wave0) {
            if (wrapsafe) thr_runs_segment<false>(st, io, hc, s, lo, hi, res, rule.count, RL);
            else thr_runs_segment<true>(st, io, hc, s, lo, hi, res, rule.count, RL);
        }
    } else if (hc.seg_mode[s] == SM_THREAD) {
        ThrLds& L = *reinterpret_cast<ThrLds*>(smem);
        for (uint32_t i = threadIdx.x; i < LX_WORDS; i += HS_T) L.lx[i] = 0ull;
        __syncthreads();
        const double M = rule.count;
        const int64_t IM = (int64_t)floor(M);
        int64_t T = st.threads[res];
        const int h = (int)(threadIdx.x >> 6);
        const uint32_t ntc = (hi - lo + THR_CH - 1) / THR_CH;
        // The two roles run separate loops with one barrier per chunk each, so the
        // helpers' code has straight-line load/consume order: their loads run two
        // chunks ahead, chunk c's records in register set c & 1 (loop unrolled by 2).
        if (h == 0) {
#ifdef SF_STREAM_PROF
            uint64_t tprof[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
            lds_barrier();
            for (uint32_t k = 0; k < ntc; k++) {
#ifdef SF_STREAM_PROF
                thr_decide(L, k & 1, hc.lxfar, lo + k * THR_CH, lo, hi, M, IM, T, hc.passbits, tprof);
#else
                thr_decide(L, k & 1, hc.lxfar, lo + k * THR_CH, lo, hi, M, IM, T, hc.passbits);
#endif
                lds_barrier();
            }
#ifdef SF_STREAM_PROF
            if ((threadIdx.x & 63) == 0)
                printf("SF_STREAM_PROF seg %u events %u chunks %u: prologue %lu loop %lu epilogue %lu; allfit-runs %lu single %lu skips %lu\n",
                       s, hi - lo, ntc, (unsigned long)tprof[0], (unsigned long)tprof[1], (unsigned long)tprof[2],
                       (unsigned long)tprof[4], (unsigned long)tprof[7], (unsigned long)tprof[9]);
#endif
        } else {
            // (loads past the segment are clamped into it, so every issue is
            // unconditional and the compiler's wait counts stay exact)
            ThrPre P0, P1;
            thr_issue(P0, hc.thr_rec, hc.lxfar, lo, hi, h);
            thr_issue(P1, hc.thr_rec, hc.lxfar, lo + THR_CH, hi, h);
            thr_finish(L, 0, P0, lo, lo, hi, h);
            thr_issue(P0, hc.thr_rec, hc.lxfar, lo + 2 * THR_CH, hi, h);
            lds_barrier();                                           // (no fence: the loads stay in flight)
            for (uint32_t k = 0; k < ntc; k += 2) {
                const uint32_t q1 = lo + (k + 1) * THR_CH;            // chunk k + 1 (odd: set P1, buffer 1)
                thr_finish(L, 1, P1, q1, lo, hi, h);
                thr_issue(P1, hc.thr_rec, hc.lxfar, q1 + 2 * THR_CH, hi, h);
                lds_barrier();
                if (k + 1 >= ntc) break;
                thr_finish(L, 0, P0, q1 + THR_CH, lo, hi, h);        // chunk k + 2 (even: set P0, buffer 0)
                thr_issue(P0, hc.thr_rec, hc.lxfar, q1 + 3 * THR_CH, hi, h);
                lds_barrier();
            }
            __builtin_amdgcn_s_waitcnt(0);                           // nothing in flight into the next segment
        }
    } else {                                                     // SM_RL
        int64_t* tsb = (int64_t*)smem;                           // [2][HS_CH]
        int32_t* cb = (int32_t*)(smem + 2 * HS_CH);              // [2][HS_CH]
        DevRuleState rs = st.rstate[r0];
        PassStage iw{hc.passbits, io.v_wait, 0, 0, 0};
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
                lds_barrier();
            }
            if (wave0) iw.finish();
            rs.latest_passed = L;
        }
        if (threadIdx.x == 0) st.rstate[r0] = rs;
    }
    if (sc.sticks && threadIdx.x == 0) {       // diagnostics: start (40 bits) and duration (24 bits)
        const uint64_t d = wall_clock64() - t_start;
        sc.sticks[b] = ((t_start & 0xffffffffffull) << 24) | (d < 0xffffffull ? d : 0xffffffull);
    }
    if (wave0) __builtin_amdgcn_s_setprio(0);
}

// Persistent: a grid sized to the chip takes the segments from a queue in
// list order (longest first).  Launched ahead of the light lanes, its
// workgroups hold their CU slots for the whole list instead of competing for
// them one segment at a time.  Every workgroup leaves when the queue is
// exhausted.
__global__ void __launch_bounds__(HS_T) k_heavy_stream(DevState st, SegIO io, HeavyCtx hc, StreamCtx sc) {
    __shared__ unsigned long long smem[HS_SMEM_WORDS];
    __shared__ uint32_t slot;
    while (true) {
        if (threadIdx.x == 0) slot = atomicAdd(sc.next, 1u);
        __syncthreads();
        const uint32_t b = slot;
        __syncthreads();
        uint32_t s;
        if (!stream_at(sc, b, &s)) break;
        stream_segment(st, io, hc, sc, s, b, smem);
        __syncthreads();                            // LDS is reused by the next segment
    }
}

}  // namespace sf
