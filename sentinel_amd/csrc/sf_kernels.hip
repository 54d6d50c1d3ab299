// sf_kernels.hip — gfx950 kernels of one sf_submit (product code).
//
// Sort phase (sort stream, one of two Work sets; overlaps the previous
// batch's decide phase):
//   k_keys_packed  validate + map resource ids to shard-local keys, 8-B payload
//   radix sort     stable (key, payload) sort by resource: per-resource time order
//                  is the input order (LeapArray semantics need it)
//   head scan      inclusive scan of segment-head flags (segment table written by k_unpack)
//   k_unpack       events into sorted order (SoA), per-segment flags
//   k_gather_exit  exits: sorted position of the entry (binary search in its segment), exit_of map
//   pc scan        inclusive prefix of entry acquireCount (heavy window budgets)
//   k_classify     light segments (by length class) -> lane interpreter; heavy -> window/skip algorithms
//   k_fill_tiles   fill tiles of the heavy segments of each class
// Decide phase (stateful, in batch order):
//   stream A:   k_heavy_stream  persistent; one 256-thread workgroup per heavy THREAD / RL segment (sf_stream.h)
//               k_heavy_fill / k_heavy_apply of its class
//   stream B:   k_heavy_decide  one wavefront per heavy QPS / WarmUp segment (sf_heavy.h)
//               k_heavy_fill    verdicts + per-window counter deltas from the pass bits
//               k_heavy_apply   deltas applied to the LeapArray state in time order
//   stream C:   k_decide_light  one lane per light segment (sf_decide.h)
// Every kernel writes its verdicts straight into the caller's arrays
// (submission order, through the sort permutation).
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "sf_rsort.h"
#include "sf_stream.h"
#include "sf_system.h"
#include "sf_xflow.h"

namespace sf {

__global__ void k_init_state(DevState st, size_t n_sec, size_t n_min) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = i; k < n_sec; k += stride) {
        st.second[k] = fresh_bucket(WS_NONE, st.max_rt);
        st.borrow[k].ws = WS_NONE; st.borrow[k].pass = 0;
    }
    for (size_t k = i; k < n_min; k += stride) st.minute[k] = fresh_bucket(WS_NONE, st.max_rt);
    for (size_t k = i; k < st.R; k += stride) st.threads[k] = 0;
}

// Sort payload: the radix sort carries each event's index, time offset from
// the batch's first event, flags and acquireCount packed into 8 bytes
// (PackedEv), so the sorted order is read back with coalesced loads instead of
// a random gather from the submission-order arrays; an offset or count that
// does not fit is read from the batch by k_unpack for that event only.
template <bool ORG>
__global__ void k_keys_packed(DevBatch b, uint32_t* keys, void* pvv, uint32_t shard_count, uint32_t shard_index,
                              uint32_t R, int32_t* err, const int64_t* last_ts, const uint32_t* xmap) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    uint32_t r = b.res[i];
    uint32_t l = r / shard_count;
    if (r % shard_count != shard_index || l >= R) { *err = SF_ERR_INVALID; l = 0; }
    if (xmap) {                                                  // an xflow group is one segment (sf_xflow.h)
        const uint32_t g = xmap[l];
        if (g != XNONE) l = g;
    }
    // the mocked clock never goes back: within the batch and across batches
    // (LeapArray would hand such an event a throwaway window)
    if (b.ts[i] < (i ? b.ts[i - 1] : *last_ts)) *err = SF_ERR_INVALID;
    keys[i] = l;
    const int64_t d = b.ts[i] - b.ts[0];
    const uint32_t dts = (d >= 0 && d < (int64_t)PV_DTS_FAR) ? (uint32_t)d : PV_DTS_FAR;
    const uint8_t f = b.flags[i];
    uint32_t fl = f & 0x0Fu;
    if ((f & (SF_EV_BLOCKED | SF_EV_EXIT)) == SF_EV_BLOCKED)     // blocked by AuthoritySlot (before SystemSlot)
        fl |= EVF_SYSBLK | ((uint32_t)SYSR_OTHER << EVF_SYSREASON_SHIFT);
    else if (b.sys && (f & SF_EV_IN) && !(f & SF_EV_EXIT)) {     // SystemBlockException forced by the planner
        const uint8_t sr = b.sys[i];
        if (sr < SYS_INERT) fl |= EVF_SYSBLK | ((uint32_t)sr << EVF_SYSREASON_SHIFT);   // (SYS_INERT / SYS_NONE: none)
    }
    const int32_t c = b.cnt[i];
    const uint32_t c8 = (c >= 1 && c <= 255) ? (uint32_t)c : 0u;
    const uint32_t meta = dts | (fl << 16) | (c8 << 24);
    if constexpr (ORG) {
        PackedEvO v; v.idx = i; v.meta = meta; v.origin = b.origin[i];
        ((PackedEvO*)pvv)[i] = v;
    } else {
        PackedEv v; v.idx = i; v.meta = meta;
        ((PackedEv*)pvv)[i] = v;
    }
}

// Also the segment table (segment id of sorted event j = inclusive count of
// segment heads up to j, minus one): start, resource and the segment count.
template <bool ORG>
__global__ void k_unpack(DevBatch b, const void* pvv, const uint32_t* keys, uint32_t* perm, int64_t* s_ts,
                         int32_t* s_cnt, uint8_t* s_flags, uint8_t* s_nargs, uint8_t* s_atag,
                         uint64_t* s_abits, const uint32_t* head_scan, uint32_t* seg_start, uint32_t* seg_res,
                         uint32_t* n_seg, uint32_t* segflag, int64_t* last_ts, const int32_t* err, bool exit_marks,
                         uint32_t* s_origin, int32_t* prio_seen) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= b.n) return;
    const uint32_t sid = head_scan[j] - 1;
    if (j == 0 || head_scan[j - 1] != head_scan[j]) { seg_start[sid] = j; seg_res[sid] = keys[j]; }
    if (j == b.n - 1) { *n_seg = sid + 1; seg_start[sid + 1] = b.n; }
    if (j == 0 && *err == 0) *last_ts = b.ts[b.n - 1];   // k_keys_packed of this batch has read the old value
    PackedEv v;
    if constexpr (ORG) {
        const PackedEvO vo = ((const PackedEvO*)pvv)[j];
        v.idx = vo.idx; v.meta = vo.meta;
        s_origin[j] = vo.origin;
    } else {
        v = ((const PackedEv*)pvv)[j];
    }
    const uint32_t i = v.idx;
    const uint32_t dts = v.meta & 0xffffu, c8 = v.meta >> 24;
    const int32_t c = c8 ? (int32_t)c8 : b.cnt[i];
    const uint8_t f = (uint8_t)(v.meta >> 16);
    perm[j] = i;
    s_ts[j] = dts != PV_DTS_FAR ? b.ts[0] + (int64_t)dts : b.ts[i]; s_cnt[j] = c; s_flags[j] = f;
    // segment flags (k_classify's routing): the exits (read only by the ParamFlow
    // routing, heavy_mode), prioritized / non-positive / blocked-before
    // entries; OR-ed per segment within the wavefront, one atomic per segment
    // and wavefront (origins need no flag: sf_origin.hip finds them per event)
    {
        uint32_t mine = 0;
        if (exit_marks && (f & SF_EV_EXIT)) mine |= SEGF_EXIT;
        if (!(f & SF_EV_EXIT))
            mine |= ((f & SF_EV_PRIO) ? SEGF_PRIO : 0u) | (c <= 0 ? SEGF_NONPOS : 0u) | ((f & EVF_SYSBLK) ? SEGF_SYS : 0u);
        const unsigned long long any = __ballot(mine != 0);
        if (any) {
            const int lane = (int)(threadIdx.x & 63);
            if (__ballot(mine & SEGF_PRIO) && lane == 0) atomicOr(prio_seen, 1);
            const int psid = __shfl_up((int)sid, 1);
            const unsigned long long heads = __ballot(lane == 0 || (uint32_t)psid != sid);
            const unsigned long long below = (1ull << lane) - 1ull;
            const unsigned long long after = heads & ~(below | (1ull << lane));
            const int nxt = after ? __ffsll((long long)after) - 1 : 64;
            const unsigned long long range = (nxt == 64 ? ~0ull : (1ull << nxt) - 1ull) & ~below;
            uint32_t acc = 0;
            const uint32_t kinds[4] = {SEGF_EXIT, SEGF_PRIO, SEGF_NONPOS, SEGF_SYS};
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (__ballot(mine & kinds[k]) & range) acc |= kinds[k];
            if (((heads >> lane) & 1ull) && acc) atomicOr(&segflag[sid], acc);
        }
    }
    if (b.arg_slots) {
        if (b.nargs) s_nargs[j] = b.nargs[i];
        for (uint32_t a = 0; a < b.arg_slots; a++) {
            const uint8_t tg = b.atag[(size_t)a * b.arg_stride + i];
            s_atag[(size_t)a * b.n + j] = tg;
            if (tg == SF_TAG_COLLECTION) atomicOr(&segflag[sid], SEGF_COLL);
            // a collection argument carries its index into the batch's element CSR
            s_abits[(size_t)a * b.n + j] = tg == SF_TAG_COLLECTION ? (uint64_t)a * b.arg_stride + (uint64_t)b.base + i
                                                                  : b.abits[(size_t)a * b.arg_stride + i];
        }
    }
}

// After the hand-written sort (sf_rsort.h), whose last pass wrote the sorted
// SoA: the segment table (segment id of sorted event j = inclusive count of
// segment heads up to j, minus one: start, resource, count), the engine clock,
// and the per-segment flags k_classify routes by.
__global__ void k_segs(DevBatch b, const int32_t* s_cnt, const uint8_t* s_flags, const uint8_t* s_atag,
                       const uint32_t* keys, const uint32_t* head_scan, uint32_t* seg_start, uint32_t* seg_res,
                       uint32_t* n_seg, uint32_t* segflag, int64_t* last_ts, const int32_t* err, bool exit_marks,
                       int32_t* prio_seen) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= b.n) return;
    const uint32_t sid = head_scan[j] - 1;
    if (j == 0 || head_scan[j - 1] != head_scan[j]) { seg_start[sid] = j; seg_res[sid] = keys[j]; }
    if (j == b.n - 1) { *n_seg = sid + 1; seg_start[sid + 1] = b.n; }
    if (j == 0 && *err == 0) *last_ts = b.ts[b.n - 1];   // the sort's first pass has read the old value
    const uint8_t f = s_flags[j];
    const int32_t c = s_cnt[j];
    uint32_t mine = 0;
    if (exit_marks && (f & SF_EV_EXIT)) mine |= SEGF_EXIT;
    if (!(f & SF_EV_EXIT))
        mine |= ((f & SF_EV_PRIO) ? SEGF_PRIO : 0u) | (c <= 0 ? SEGF_NONPOS : 0u) | ((f & EVF_SYSBLK) ? SEGF_SYS : 0u);
    for (uint32_t a = 0; a < b.arg_slots; a++)
        if (s_atag[(size_t)a * b.n + j] == SF_TAG_COLLECTION) mine |= SEGF_COLL;
    // OR-ed per segment within the wavefront, one atomic per segment and wavefront
    const unsigned long long any = __ballot(mine != 0);
    if (!any) return;
    const int lane = (int)(threadIdx.x & 63);
    if (__ballot(mine & SEGF_PRIO) && lane == 0) atomicOr(prio_seen, 1);   // (sticky: st.prio_seen)
    const int psid = __shfl_up((int)sid, 1);
    const unsigned long long heads = __ballot(lane == 0 || (uint32_t)psid != sid);
    const unsigned long long below = (1ull << lane) - 1ull;
    const unsigned long long after = heads & ~(below | (1ull << lane));
    const int nxt = after ? __ffsll((long long)after) - 1 : 64;
    const unsigned long long range = (nxt == 64 ? ~0ull : (1ull << nxt) - 1ull) & ~below;
    uint32_t acc = 0;
    const uint32_t kinds[5] = {SEGF_EXIT, SEGF_PRIO, SEGF_NONPOS, SEGF_SYS, SEGF_COLL};
#pragma unroll
    for (int k = 0; k < 5; k++)
        if (__ballot(mine & kinds[k]) & range) acc |= kinds[k];
    if (((heads >> lane) & 1ull) && acc) atomicOr(&segflag[sid], acc);
}

// ============================================================ segment table + prefixes (reduce, scan, rescan)
// The segment heads of the sorted keys and their inclusive count per
// position (head_scan = segment id + 1), the segment table (start, resource,
// flags) and, when the decide phase's window budgets need it, the inclusive
// prefix of the entries' acquireCounts (pcg: 0 for exits and EVF_SYSBLK
// entries; k_heavy_decide's greedy prefix) -- what the rocprim head scan,
// k_segs and the rocprim acquireCount scan wrote in three passes.  Three
// launches without any cross-workgroup waiting: per-tile totals, one
// workgroup scanning the tile totals, then every tile again from its prefix.
// (A decoupled look-back single pass measured 5 ms per batch on gfx950: its
// agent-scope release / acquire publishes write back and bypass the per-XCD
// L2 on every tile.)
constexpr int SL_T = 256, SL_K = 16, SL_TILE = SL_T * SL_K;       // 4096 positions per tile
size_t segs_lb_bytes(uint32_t max_n) { return ((size_t)max_n / SL_TILE + 2) * 16 + 64; }   // (sf_internal.h)

struct SegTile {                 // one thread's 16 positions
    uint32_t k[SL_K];
    int32_t c[SL_K];
    uint8_t f[SL_K];
    uint32_t hmask, heads;
    long long acq;
};
template <bool PCG>
__device__ __forceinline__ void seg_load(SegTile& t, const uint32_t* keys, const uint8_t* s_flags, const int32_t* s_cnt,
                                         uint32_t p0, uint32_t n) {
    if (p0 + SL_K <= n) {
        const uint4* kp = (const uint4*)(keys + p0);
#pragma unroll
        for (int q = 0; q < SL_K / 4; q++) { const uint4 v = kp[q]; t.k[4 * q] = v.x; t.k[4 * q + 1] = v.y; t.k[4 * q + 2] = v.z; t.k[4 * q + 3] = v.w; }
        const uint4 fv = *(const uint4*)(s_flags + p0);
        const uint32_t fw[4] = {fv.x, fv.y, fv.z, fv.w};
#pragma unroll
        for (int q = 0; q < SL_K; q++) t.f[q] = (uint8_t)(fw[q >> 2] >> (8 * (q & 3)));
        if (PCG) {
            const int4* cp = (const int4*)(s_cnt + p0);
#pragma unroll
            for (int q = 0; q < SL_K / 4; q++) { const int4 v = cp[q]; t.c[4 * q] = v.x; t.c[4 * q + 1] = v.y; t.c[4 * q + 2] = v.z; t.c[4 * q + 3] = v.w; }
        }
    } else {
#pragma unroll
        for (int q = 0; q < SL_K; q++) {
            const bool in = p0 + q < n;
            t.k[q] = in ? keys[p0 + q] : 0u;
            t.f[q] = in ? s_flags[p0 + q] : (uint8_t)SF_EV_EXIT;
            t.c[q] = (PCG && in) ? s_cnt[p0 + q] : 0;
        }
    }
    const uint32_t kprev = (p0 > 0 && p0 < n) ? keys[p0 - 1] : ~0u;
    t.hmask = 0; t.heads = 0; t.acq = 0;
#pragma unroll
    for (int q = 0; q < SL_K; q++) {
        const bool in = p0 + q < n;
        const bool h = in && (p0 + q == 0 || t.k[q] != (q ? t.k[q - 1] : kprev));
        t.hmask |= (h ? 1u : 0u) << q;
        t.heads += h;
        if (PCG) t.acq += (in && !(t.f[q] & (SF_EV_EXIT | EVF_SYSBLK))) ? (long long)t.c[q] : 0;
    }
}
// block-wide exclusive scan of (heads, acq) over the threads; totals out
__device__ __forceinline__ void seg_block_scan(uint32_t& hx, long long& ax, uint32_t* htot, long long* atot) {
    __shared__ uint32_t w_heads[SL_T / 64];
    __shared__ long long w_acq[SL_T / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t h0 = hx;
    const long long a0 = ax;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t h2 = __shfl_up(hx, d);
        const long long a2 = __shfl_up(ax, d);
        if (lane >= d) { hx += h2; ax += a2; }
    }
    if (lane == 63) { w_heads[wv] = hx; w_acq[wv] = ax; }
    __syncthreads();
    uint32_t hb = 0, ht = 0;
    long long ab = 0, at = 0;
#pragma unroll
    for (int w = 0; w < SL_T / 64; w++) {
        if (w < wv) { hb += w_heads[w]; ab += w_acq[w]; }
        ht += w_heads[w]; at += w_acq[w];
    }
    hx = hx - h0 + hb;
    ax = ax - a0 + ab;
    *htot = ht; *atot = at;
}

template <bool PCG>
__global__ void __launch_bounds__(SL_T) k_segs_red(const uint32_t* keys, const uint8_t* s_flags, const int32_t* s_cnt,
                                                   uint32_t n, uint32_t* t_heads, long long* t_acq) {
    SegTile t;
    seg_load<PCG>(t, keys, s_flags, s_cnt, blockIdx.x * SL_TILE + threadIdx.x * SL_K, n);
    uint32_t hx = t.heads, ht;
    long long ax = t.acq, at;
    seg_block_scan(hx, ax, &ht, &at);
    if (threadIdx.x == 0) { t_heads[blockIdx.x] = ht; t_acq[blockIdx.x] = at; }
}
// one workgroup: exclusive prefix of the tile totals, in place
__global__ void __launch_bounds__(1024) k_segs_tscan(uint32_t* t_heads, long long* t_acq, uint32_t tiles) {
    __shared__ uint32_t sh[1024];
    __shared__ long long sa[1024];
    const uint32_t per = (tiles + 1023) / 1024, i0 = threadIdx.x * per, i1 = min(i0 + per, tiles);
    uint32_t h = 0;
    long long a = 0;
    for (uint32_t i = i0; i < i1; i++) { h += t_heads[i]; a += t_acq[i]; }
    sh[threadIdx.x] = h; sa[threadIdx.x] = a;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const uint32_t h2 = threadIdx.x >= (unsigned)d ? sh[threadIdx.x - d] : 0u;
        const long long a2 = threadIdx.x >= (unsigned)d ? sa[threadIdx.x - d] : 0;
        __syncthreads();
        sh[threadIdx.x] += h2; sa[threadIdx.x] += a2;
        __syncthreads();
    }
    h = sh[threadIdx.x] - h; a = sa[threadIdx.x] - a;        // exclusive prefix of this thread's run
    for (uint32_t i = i0; i < i1; i++) {
        const uint32_t th = t_heads[i];
        const long long ta = t_acq[i];
        t_heads[i] = h; t_acq[i] = a;
        h += th; a += ta;
    }
}

template <bool PCG>
__global__ void __launch_bounds__(SL_T) k_segs_out(DevBatch b, const int32_t* s_cnt, const uint8_t* s_flags,
                                                   const uint8_t* s_atag, const uint32_t* keys, uint32_t* head_scan,
                                                   int64_t* pcg, uint32_t* seg_start, uint32_t* seg_res,
                                                   uint32_t* n_seg, uint32_t* segflag, int64_t* last_ts,
                                                   const int32_t* err, bool exit_marks, int32_t* prio_seen,
                                                   const uint32_t* t_heads, const long long* t_acq) {
    const uint32_t n = b.n, p0 = blockIdx.x * SL_TILE + threadIdx.x * SL_K;
    SegTile t;
    seg_load<PCG>(t, keys, s_flags, s_cnt, p0, n);
    uint32_t hx = t.heads, ht;
    long long ax = t.acq, at;
    seg_block_scan(hx, ax, &ht, &at);
    if (p0 >= n) return;
    uint32_t hs = t_heads[blockIdx.x] + hx;   // heads before this thread's first position
    long long run = PCG ? t_acq[blockIdx.x] + ax : 0;
    uint32_t hsv[SL_K];
    long long pv[SL_K];
    uint32_t acc = 0, prio = 0;
    int64_t cur = hs ? (int64_t)hs - 1 : -1;   // the segment of the position before this thread's first
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < SL_K; q++) {
        const uint32_t p = p0 + q;
        const bool in = p < n;
        if ((t.hmask >> q) & 1u) {
            if (acc && cur >= 0) atomicOr(&segflag[cur], acc);
            acc = 0;
            hs++;
            cur = (int64_t)hs - 1;
            seg_start[hs - 1] = p;
            seg_res[hs - 1] = t.k[q];
        }
        hsv[q] = hs;
        if (PCG) { run += (in && !(t.f[q] & (SF_EV_EXIT | EVF_SYSBLK))) ? (long long)t.c[q] : 0; pv[q] = run; }
        if (!in) continue;
        uint32_t mine = 0;
        if (exit_marks && (t.f[q] & SF_EV_EXIT)) mine |= SEGF_EXIT;
        if (!(t.f[q] & SF_EV_EXIT)) {
            const int32_t cq = PCG ? t.c[q] : s_cnt[p];
            mine |= ((t.f[q] & SF_EV_PRIO) ? SEGF_PRIO : 0u) | (cq <= 0 ? SEGF_NONPOS : 0u) |
                    ((t.f[q] & EVF_SYSBLK) ? SEGF_SYS : 0u);
        }
        for (uint32_t a = 0; a < b.arg_slots; a++)
            if (s_atag[(size_t)a * n + p] == SF_TAG_COLLECTION) mine |= SEGF_COLL;
        acc |= mine;
        prio |= mine & SEGF_PRIO;
        if (p == n - 1) { *n_seg = hs; seg_start[hs] = n; }
        if (p == 0 && *err == 0) *last_ts = b.ts[n - 1];      // the sort's first pass has read the old value
    }
    if (acc && cur >= 0) atomicOr(&segflag[cur], acc);
    if (__ballot(prio != 0) && lane == 0) atomicOr(prio_seen, 1);
    if (p0 + SL_K <= n) {
        uint4* hp = (uint4*)(head_scan + p0);
#pragma unroll
        for (int q = 0; q < SL_K / 4; q++) hp[q] = make_uint4(hsv[4 * q], hsv[4 * q + 1], hsv[4 * q + 2], hsv[4 * q + 3]);
        if (PCG) {
            longlong2* pp = (longlong2*)(pcg + p0);
#pragma unroll
            for (int q = 0; q < SL_K / 2; q++) pp[q] = make_longlong2(pv[2 * q], pv[2 * q + 1]);
        }
    } else {
        for (int q = 0; q < SL_K; q++) {
            if (p0 + q >= n) break;
            head_scan[p0 + q] = hsv[q];
            if (PCG) pcg[p0 + q] = pv[q];
        }
    }
}

template <bool PCG>
static void launch_segs3(const DevState& st, Work& w, const DevBatch& b, hipStream_t s) {
    const uint32_t n = b.n, tiles = (n + SL_TILE - 1) / SL_TILE;
    uint32_t* th = (uint32_t*)w.segs_lb;
    long long* ta = (long long*)((char*)w.segs_lb + (((size_t)tiles * 4 + 15) & ~(size_t)15));
    hipLaunchKernelGGL(k_segs_red<PCG>, dim3(tiles), dim3(SL_T), 0, s, w.keys_out, w.s_flags, w.s_cnt, n, th, ta);
    hipLaunchKernelGGL(k_segs_tscan, dim3(1), dim3(1024), 0, s, th, ta, tiles);
    hipLaunchKernelGGL(k_segs_out<PCG>, dim3(tiles), dim3(SL_T), 0, s, b, w.s_cnt, w.s_flags, w.s_atag, w.keys_out,
                       w.head_scan, w.pcg, w.seg_start, w.seg_res, w.n_seg, w.segflag, st.last_ts, st.err,
                       st.n_prule != 0, st.prio_seen, th, ta);
}

struct HeadFlag {       // 1 where a new resource segment starts in the sorted keys
    const uint32_t* keys;
    __device__ uint32_t operator()(uint32_t j) const { return (j == 0 || keys[j] != keys[j - 1]) ? 1u : 0u; }
};

// Exits only: the sorted position of each exit's entry.  The sort is stable
// and the segment holds one resource's events in submission order, so the
// entry is found by a binary search of the segment's submission indices (no
// inverse permutation scattered over the whole batch).  Forward map exit_of
// for THREAD-grade liveness; s_cts for entries of earlier batches.
__global__ void k_gather_exit(DevBatch b, const uint32_t* perm, const uint8_t* s_flags,
                              const uint32_t* head_scan, const uint32_t* seg_start, int64_t* s_eref,
                              int64_t* s_cts, uint32_t* exit_of, int32_t* err) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= b.n || !(s_flags[j] & SF_EV_EXIT)) return;
    const uint32_t i = perm[j];
    const int64_t raw = b.eref[i];
    // -1: the entry passed before this batch (live, create_ts gives its time);
    // EREF_DEAD: it was blocked before this batch (the exit is ignored)
    if (raw < 0) { s_eref[j] = raw == EREF_DEAD ? EREF_DEAD : -1; s_cts[j] = b.cts ? b.cts[i] : 0; return; }
    const int64_t r = raw - b.base;                                      // view-local index
    if (r < 0) {
        // the entry was decided in an earlier sub-batch of this batch: live
        // (-1, its time as create_ts) unless it was blocked (-2: the exit is ignored)
        if (!b.vprev || b.res[r] != b.res[i] || (b.flags[r] & SF_EV_EXIT)) {
            *err = SF_ERR_INVALID; s_eref[j] = -1; s_cts[j] = 0; return;
        }
        s_eref[j] = v_blocked_any(b.vprev[r]) ? -2 : -1;
        s_cts[j] = b.ts[r];
        return;
    }
    const uint32_t lo = seg_start[head_scan[j] - 1];          // entry in [segment start, j)
    if (r >= (int64_t)i) { *err = SF_ERR_INVALID; s_eref[j] = -1; s_cts[j] = 0; return; }
    // galloping back from j (an entry is usually a few of its resource's events
    // before its exit: the probes stay on the lines the neighbours read), then
    // a binary search of the bracket
    uint32_t a = lo, e = j;
    for (uint32_t step = 1; j - lo > step; step <<= 1) {
        const uint32_t m = j - step;
        if ((int64_t)perm[m] < r) { a = m + 1; break; }
        e = m;
        if ((int64_t)perm[m] == r) { a = m; break; }
    }
    while (a < e) { const uint32_t m = (a + e) >> 1; if ((int64_t)perm[m] < r) a = m + 1; else e = m; }
    if (a >= j || (int64_t)perm[a] != r) { *err = SF_ERR_INVALID; s_eref[j] = -1; s_cts[j] = 0; return; }
    s_eref[j] = a;
    exit_of[a] = j;
}

struct EntryCount {     // acquireCount of the entries the controllers see (input of the pc scan):
    const int32_t* cnt; const uint8_t* flags;    // 0 for exits and EVF_SYSBLK entries
    __device__ int64_t operator()(uint32_t j) const {
        return (flags[j] & (SF_EV_EXIT | EVF_SYSBLK)) ? 0 : (int64_t)cnt[j];
    }
};

// Append to a list with one atomic per wavefront (a single hot counter would
// otherwise serialise millions of atomics at one L2 channel).
__device__ uint32_t wave_append(uint32_t* counter, bool take) {
    const unsigned long long m = __ballot(take);
    if (!m) return 0;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// Route each segment: light lane interpreter, heavy window algorithms, or the
// heavy generic interpreter (one lane of a wavefront).
__global__ void k_classify(DevState st, Work w, const int64_t* s_ts) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = s < *w.n_seg;
    uint32_t lo = 0, hi = 0, res = 0;
    if (valid) { lo = w.seg_start[s]; hi = w.seg_start[s + 1]; res = w.seg_res[s]; }
    // an xflow group (sf_xflow.h) is decided by k_decide_x only; origins alone
    // do not route a segment there (their nodes: sf_origin.hip)
    const bool xs = valid && st.xmap && st.xmap[res] != XNONE;
    if (xs) w.seg_mode[s] = SM_XFLOW;
    {   // long xflow segments the wave walk can take (k_decide_xw)
        const bool xw = xs && xw_take(st, res, hi - lo);
        const uint32_t p = wave_append(&w.counters[12], xw);
        if (xw) w.xw_list[p] = s;
    }
    bool light = valid && !xs && hi - lo <= w.heavy_min;
    // a ParamFlow-only segment of more than 32 events is faster on the
    // wavefront-by-value path (SM_PARAM) than as one lane's serial table walk
    if (light && hi - lo > 32 && (st.rdesc[res].flags & RD_PRULE) &&
        heavy_mode(st, res, w.segflag[s], s_ts[lo]) == SM_PARAM)
        light = false;
    // light list slot: workgroup histogram of the length classes in LDS, one
    // global atomic per class and workgroup
    // (hcnt / hbase [0, LCLS): generic lane walk, [LCLS, 2 LCLS): lean QPS walk)
    __shared__ uint32_t hcnt[2 * LCLS], hbase[2 * LCLS];
    if (threadIdx.x < 2 * LCLS) hcnt[threadIdx.x] = 0;
    __syncthreads();
    // a segment of a resource whose only check is one QPS DefaultController rule
    // runs the lean lane walk (decide_qps_segment: k_decide_short_qps / k_decide_light_qps)
    const bool lean = light && qps_lean(st, res, w.segflag[s]);
    const int lc = (light && hi - lo > SHORT_MAX) ? light_class(hi - lo) : -1;
    const int hk = lc + (lean ? LCLS : 0);
    const uint32_t lrank = lc >= 0 ? atomicAdd(&hcnt[hk], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < 2 * LCLS)
        hbase[threadIdx.x] = hcnt[threadIdx.x] ? atomicAdd(&w.lcounts[threadIdx.x], hcnt[threadIdx.x]) : 0u;
    __syncthreads();
    if (light) {
        w.seg_mode[s] = lean ? SM_LIGHTQ : SM_LIGHT;
        if (lc >= 0) {
            if (lean) w.light_list[w.loff[lc] + w.lcap[lc] - 1 - (hbase[hk] + lrank)] = s;
            else w.light_list[w.loff[lc] + hbase[hk] + lrank] = s;
        }
    }
    // short segments (<= SHORT_MAX events) listed densely for k_decide_short /
    // k_decide_short_qps, in segment (resource) order within each workgroup,
    // one global atomic per workgroup and list: a deciding wavefront's lanes
    // hold neighbouring resource rows and no idle lanes for the segments of
    // the other kernel.  Class 0's light_list region (every segment fits)
    // holds both lists: generic from the front, lean QPS from the back.
    static_assert(SHORT_MAX >= 1, "class 0 (one-event segments) must be a short class");
    __shared__ uint32_t wsh[2][32], bsh[2];
    const bool shrt = light && hi - lo <= SHORT_MAX;
    const unsigned long long mg = __ballot(shrt && !lean), mq = __ballot(shrt && lean);
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6), nwv = (int)(blockDim.x >> 6);
    if (lane == 0) { wsh[0][wv] = (uint32_t)__popcll(mg); wsh[1][wv] = (uint32_t)__popcll(mq); }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint32_t acc = 0;
        for (int k = 0; k < nwv; k++) { const uint32_t c = wsh[threadIdx.x][k]; wsh[threadIdx.x][k] = acc; acc += c; }
        bsh[threadIdx.x] = acc ? atomicAdd(&w.counters[8 + threadIdx.x], acc) : 0u;
    }
    __syncthreads();
    if (shrt) {
        const unsigned long long below = (1ull << lane) - 1ull;
        if (lean) w.light_list[w.loff[0] + w.lcap[0] - 1 - (bsh[1] + wsh[1][wv] + (uint32_t)__popcll(mq & below))] = s;
        else w.light_list[w.loff[0] + bsh[0] + wsh[0][wv] + (uint32_t)__popcll(mg & below)] = s;
    }
    const bool heavy = valid && !light && !xs;
    if (!__ballot(heavy)) return;
    uint8_t mode = SM_GENERIC;
    if (heavy) {
        mode = heavy_mode(st, res, w.segflag[s], s_ts[lo]);
        if (mode != SM_GENERIC) {
            const int64_t h0 = s_ts[lo] / st.wl, h1 = s_ts[hi - 1] / st.wl;
            const int64_t s0 = s_ts[lo] / 1000, s1 = s_ts[hi - 1] / 1000;
            const int64_t nh = h1 - h0 + 1, ns = s1 - s0 + 1;
            if (nh > 65536 || ns > 65536) mode = SM_GENERIC;
            else {
                uint32_t bh = atomicAdd(&w.counters[2], (uint32_t)nh);
                uint32_t bs = atomicAdd(&w.counters[3], (uint32_t)ns);
                if ((uint64_t)bh + nh > w.acc_cap || (uint64_t)bs + ns > w.acc_cap) mode = SM_GENERIC;
                else {
                    w.acc_hw_base[s] = bh; w.acc_sec_base[s] = bs;
                    w.seg_hw0[s] = h0; w.seg_sec0[s] = s0; w.seg_nhw[s] = (uint32_t)nh; w.seg_nsec[s] = (uint32_t)ns;
                    Acc z{}; z.min_rt = INT64_MAX;
                    Acc* ah = (Acc*)w.acc_hw; Acc* as = (Acc*)w.acc_sec;
                    for (int64_t k = 0; k < nh; k++) ah[bh + k] = z;
                    for (int64_t k = 0; k < ns; k++) as[bs + k] = z;
                }
            }
        }
        w.seg_mode[s] = mode;
    }
    // THREAD-grade and RateLimiter segments go to k_heavy_stream, the rest to
    // k_heavy_decide.  Long-running segments first in each list, so that they
    // start first: [0, front) and [seg_cap - back, seg_cap)
    const bool strm = heavy && (mode == SM_THREAD || mode == SM_RL);
    const bool big = hi - lo > 65536u;
    const bool slow = heavy && !strm && (mode == SM_GENERIC || big);
    const uint32_t fpos = wave_append(&w.counters[1], slow);
    const uint32_t bpos = wave_append(&w.counters[4], heavy && !strm && !slow);
    if (slow) w.heavy_list[fpos] = s;
    else if (heavy && !strm) w.heavy_list[w.seg_cap - 1 - bpos] = s;
    const uint32_t sfp = wave_append(&w.counters[5], strm && big);
    const uint32_t sbp = wave_append(&w.counters[6], strm && !big);
    if (strm && big) w.stream_list[sfp] = s;
    else if (strm) w.stream_list[w.seg_cap - 1 - sbp] = s;
}

// heavy-list entry of workgroup b: front part, then the back part
// (k_heavy_apply walks both lists: every heavy item segment is in one of them)
__device__ __forceinline__ bool heavy_at(const HeavyCtx& hc, uint32_t b, uint32_t* s) {
    const uint32_t nf = hc.n_heavy[0], nb = hc.n_heavy[3];
    if (b < nf) { *s = hc.heavy_list[b]; return true; }
    if (b < nf + nb) { *s = hc.heavy_list[hc.seg_cap - 1 - (b - nf)]; return true; }
    return false;
}

struct LightLists { const uint32_t* list; const uint32_t* counts; uint32_t off[LCLS]; uint32_t cap[LCLS]; };

// One lane per light segment; thread t walks the length classes from the
// longest down, so a wavefront holds segments of one class (similar length)
// and the long ones are dispatched first.
#ifndef SF_LIGHT_MINB
#define SF_LIGHT_MINB 1
#endif
#ifndef SF_LIGHT_NOPF_MINB
#define SF_LIGHT_NOPF_MINB 1          // (3 wavefronts per SIMD: 96 B of spills, config 3 15.2 vs 14.1 ms)
#endif
template <int MAXS, bool PF>
__global__ void __launch_bounds__(128, PF ? SF_LIGHT_MINB : SF_LIGHT_NOPF_MINB) k_decide_light(DevState st, SegIO io, const uint32_t* seg_start,
                                                      const uint32_t* seg_res, LightLists ll) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    int c = LCLS - 1;
    for (; c >= 0; c--) {
        const uint32_t n = ll.counts[c];
        if (t < n) break;
        t -= n;
    }
    if (c < 0) return;
    const uint32_t s = ll.list[ll.off[c] + t];
    decide_segment<MAXS, SF_EV_CH, PF>(st, io, seg_res[s], seg_start[s], seg_start[s + 1]);
}

// The lean QPS light segments (SM_LIGHTQ, > SHORT_MAX events) from the back
// of each class region, longest class first (decide_qps_segment).
template <int MAXS>
__global__ void __launch_bounds__(128) k_decide_light_qps(DevState st, SegIO io, const uint32_t* seg_start,
                                                          const uint32_t* seg_res, LightLists ll) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    int c = LCLS - 1;
    for (; c >= 0; c--) {
        const uint32_t n = ll.counts[LCLS + c];
        if (t < n) break;
        t -= n;
    }
    if (c < 0) return;
    const uint32_t s = ll.list[ll.off[c] + ll.cap[c] - 1 - t];
    decide_qps_segment<MAXS>(st, io, seg_res[s], seg_start[s], seg_start[s + 1]);
}

// One lane per short light segment, from the dense short list (k_classify;
// see SHORT_MAX).
template <int MAXS, bool PF>
__global__ void __launch_bounds__(128, PF ? SF_LIGHT_MINB : SF_LIGHT_NOPF_MINB) k_decide_short(DevState st, SegIO io, const uint32_t* seg_start,
                                                      const uint32_t* seg_res, LightLists ll,
                                                      const uint32_t* n_short) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_short[0]) return;
    const uint32_t s = ll.list[ll.off[0] + t];
    decide_segment<MAXS, SF_EV_CH, PF>(st, io, seg_res[s], seg_start[s], seg_start[s + 1]);
}

// One lane per xflow group segment (sf_xflow.h): origin / context / RELATE
// rules (the long segments k_decide_xw takes excepted).
template <int MAXS>
__global__ void __launch_bounds__(64) k_decide_x(DevState st, SegIO io, const uint32_t* seg_start,
                                                 const uint32_t* seg_res, const uint8_t* seg_mode,
                                                 const uint32_t* n_seg) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= *n_seg || seg_mode[s] != SM_XFLOW) return;
    if (xw_take(st, seg_res[s], seg_start[s + 1] - seg_start[s])) return;
    decide_xgroup<MAXS>(st, io, seg_start[s], seg_start[s + 1]);
}

// ---- the wave walk of a long xflow segment (one resource, DIRECT rules)
// A wavefront takes the segment in chunks of at most 64 events that share
// one second-window bucket and one minute bucket.  Per chunk:
//  1. every lane checks its entry against the first rule that selects a node
//     (FlowRuleComparator order: origin-specific and `other` rules before
//     `default`), on the node and rule state as they stand at the chunk's
//     start.  Within one bucket a node's pass count and a RateLimiter's
//     latestPassedTime only grow, the WarmUp threshold is fixed for the second
//     (syncToken reads the previous second; on an origin node it waits until
//     the walk has synced the second, since the rule's tokens are shared by
//     every origin and the first check of the second decides them), and a
//     THREAD count can fall at most by the exits ahead of the lane in the
//     chunk, so an entry blocked at the start state is blocked in the serial
//     order too, by that rule;
//  2. lane 0 runs the reference walk (xg_event) over the other entries --
//     those the start state lets pass, prioritized entries, and the exits when
//     a THREAD rule reads thread counts -- in order;
//  3. the blocked entries' blocks and the remaining exits' completions only
//     add to the chunk's buckets (which no check of this chunk reads), so they
//     are summed per node in LDS and added once per node.
// Verdicts, node state and rule state equal the serial walk's.
enum : uint8_t { XWC_SERIAL = 1, XWC_BLOCK = 2, XWC_EXIT = 3, XWC_PASS = 4 };
constexpr uint32_t XW_KCAP = 128;                 // LDS node rows of a chunk (<= 64 origins + the ClusterNode)
struct XwRow {
    unsigned long long blk, succ, rt, exc, pass; long long thr, minrt;
    unsigned int nblk, ncmp, nexc, npass, key, pad;
};
__device__ __forceinline__ void xw_add(XwRow& r, int64_t blk, int nblk, int64_t succ, int64_t rt, int64_t minrt,
                                       int64_t exc, int nexc, int64_t thr, int ncmp, int64_t pass = 0, int npass = 0) {
    if (nblk) { atomicAdd(&r.blk, (unsigned long long)blk); atomicAdd(&r.nblk, 1u); }
    if (npass) {
        atomicAdd(&r.pass, (unsigned long long)pass); atomicAdd(&r.npass, 1u);
        atomicAdd((unsigned long long*)&r.thr, 1ull);
    }
    if (ncmp) {
        atomicAdd(&r.succ, (unsigned long long)succ); atomicAdd(&r.rt, (unsigned long long)rt);
        atomicMin(&r.minrt, (long long)minrt); atomicAdd((unsigned long long*)&r.thr, (unsigned long long)thr);
        atomicAdd(&r.ncmp, 1u);
    }
    if (nexc) { atomicAdd(&r.exc, (unsigned long long)exc); atomicAdd(&r.nexc, 1u); }
}
// a row's sums into a node (all events of the chunk are in the bucket of t0):
// one currentWindow lookup per window for all of the row's counters
template <int MAXS>
__device__ __forceinline__ void xw_apply(NodeWin<MAXS>& nd, const XwRow& r, int64_t t0) {
    const bool hp = r.npass != 0, hb = r.nblk != 0, hc = r.ncmp != 0, he = r.nexc != 0;
    if (!(hp || hb || hc || he)) return;
    const int64_t p = (int64_t)r.pass, b = (int64_t)r.blk, sc = (int64_t)r.succ, rt = (int64_t)r.rt, mr = r.minrt,
                  e = (int64_t)r.exc;
    auto f = [&](Bucket& x) {
        if (hp) x.pass = wadd(x.pass, p);
        if (hb) x.block = wadd(x.block, b);
        if (hc) { x.succ = wadd(x.succ, sc); x.rt = wadd(x.rt, rt); if (mr < x.min_rt) x.min_rt = mr; }
        if (he) x.exc = wadd(x.exc, e);
    };
    nd.sec_apply(t0, f);
    nd.min_apply(t0, f);
    if (hp || hc) nd.threads = wadd(nd.threads, r.thr);
}

// ---- the exact chunk solve (S <= 2, no prioritized entry in the chunk)
// The chunk's verdicts as the fixed point of the serial recurrence: each
// entry's checks read its nodes' pass counts / thread counts and each
// RateLimiter's latestPassedTime as left by the entries before it in the
// chunk; given a guess of every verdict (all pass to start), every lane
// re-evaluates its entry from prefix sums over the earlier lanes (pass counts
// per node, thread deltas per node with the exits' liveness from their
// entries' verdicts, a max-plus scan x -> max(x + cost, t) per RateLimiter
// rule over the entries that passed it).  Each round makes at least the
// earliest wrong lane right (its inputs come only from earlier lanes), so the
// iteration reaches the serial result within L + 1 rounds; under saturation
// two or three.  Node bases are read once per chunk: a pass count is its
// window sum at the chunk's time plus the chunk's earlier passes (all events
// of the chunk fall in the same current bucket, every older bucket stays
// valid through it), the WarmUp threshold and the RateLimiter cost are fixed
// for the second (the ClusterNode's syncToken is applied on a copy: its
// previous-second QPS is the same for every event).
struct XwRuleC { double thr, qps; int64_t lstart; DevRuleState rs; int32_t sync, pad; };
struct XwScratch {
    long long base[XW_KCAP], thr[XW_KCAP];
    uint32_t ko[XW_KCAP];
    int os[64];
    long long cm[64], td[64];
    XwRuleC rc[MAX_RULES];
};
constexpr long long XW_MPNEG = INT64_MIN / 4;                  // max-plus "minus infinity"
// the segment's origin nodes held in LDS across chunks (exact-solve chunks
// read and write them there; a chunk on the serial path, the end of the
// segment, or a full cache writes them back)
constexpr uint32_t XW_OC = XW_KCAP - 1;                        // (chunk row r = cache slot r - 1)
struct XwCache { unsigned int key[XW_OC]; uint32_t ko[XW_OC]; unsigned int n; };
__device__ __forceinline__ NodeWin<2>& xw_node(unsigned char* ocnw, uint32_t slot) {
    return reinterpret_cast<NodeWin<2>*>(ocnw)[slot];
}
__device__ void xw_cache_flush(const DevState& st, XwCache& oc, unsigned char* ocnw, uint32_t lane) {
    __syncthreads();
    for (uint32_t k = lane; k < XW_OC; k += 64) {
        if (oc.key[k] && oc.ko[k] != XNONE) nw_store(xw_node(ocnw, k), st, aux_rows(st, oc.ko[k]));
        oc.key[k] = 0;
    }
    if (lane == 0) oc.n = 0;
    __syncthreads();
}

// wavefront scans on DPP (row shifts inside each 16-lane row, then the row
// broadcasts of lanes 15 and 31): a handful of ALU cycles per step instead of
// an LDS-crossbar shuffle; 64-bit values move as two 32-bit halves, lanes
// without a source keep `idv` (the operation's identity)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ long long xw_dpp(long long v, long long idv) {
    const unsigned long long u = (unsigned long long)v, iu = (unsigned long long)idv;
    const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)iu, (int)(unsigned)u, CTRL, ROWMASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(iu >> 32), (int)(unsigned)(u >> 32), CTRL, ROWMASK, 0xf, false);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned long long)(unsigned)lo);
}
template <class F>
__device__ __forceinline__ long long xw_scan_op(long long x, long long idv, F f) {
    x = f(x, xw_dpp<0x111, 0xf>(x, idv));        // row_shr:1
    x = f(x, xw_dpp<0x112, 0xf>(x, idv));        // row_shr:2
    x = f(x, xw_dpp<0x114, 0xf>(x, idv));        // row_shr:4
    x = f(x, xw_dpp<0x118, 0xf>(x, idv));        // row_shr:8
    x = f(x, xw_dpp<0x142, 0xa>(x, idv));        // row_bcast:15 -> rows 1, 3
    x = f(x, xw_dpp<0x143, 0xc>(x, idv));        // row_bcast:31 -> rows 2, 3
    return x;
}
__device__ __forceinline__ long long xw_excl_scan(long long v, uint32_t) {
    return xw_scan_op(v, 0, [](long long x, long long y) { return x + y; }) - v;
}
// wavefront total / minimum (lane 63 of the inclusive scan)
__device__ __forceinline__ long long xw_wsum(long long v) {
    return __shfl(xw_scan_op(v, 0, [](long long x, long long y) { return x + y; }), 63);
}
__device__ __forceinline__ long long xw_wmin(long long v) {
    return __shfl(xw_scan_op(v, INT64_MAX, [](long long x, long long y) { return y < x ? y : x; }), 63);
}
// inclusive max-plus scan of f(x) = max(x + a, b) in lane order (an earlier
// lane's (pa, pb) composed under this lane's: (pa + a, max(pb + a, b)))
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void xw_mp_step(long long& a, long long& b) {
    const long long pa = xw_dpp<CTRL, ROWMASK>(a, 0), pb = xw_dpp<CTRL, ROWMASK>(b, XW_MPNEG);
    b = max(pb + a, b);
    a = pa + a;
}
__device__ __forceinline__ void xw_mp_scan(long long& a, long long& b, uint32_t) {
    xw_mp_step<0x111, 0xf>(a, b);
    xw_mp_step<0x112, 0xf>(a, b);
    xw_mp_step<0x114, 0xf>(a, b);
    xw_mp_step<0x118, 0xf>(a, b);
    xw_mp_step<0x142, 0xa>(a, b);
    xw_mp_step<0x143, 0xc>(a, b);
}

__device__ __forceinline__ void xw_solve_chunk(const DevState& st, NodeWin<2>& snap, XwRow* rows, XwScratch& xs,
                               XwCache& oc, unsigned char* ocnw,
                               uint32_t lane, uint32_t L, int64_t t0, int64_t t,
                               uint8_t fl, int32_t c, uint32_t origin, int eidx, bool live_pre, uint32_t l, uint32_t r0,
                               uint32_t r1, uint8_t* myc, uint8_t* mst, int* mrule, int64_t* mwait, int* my_row,
                               bool* x_live, unsigned long long* pfs = nullptr) {
#ifdef SF_XW_PROFILE
    unsigned long long pt_ = wall_clock64();
#define XS_PF(k) if (lane == 0 && pfs) { const unsigned long long x_ = wall_clock64(); pfs[k] += x_ - pt_; pt_ = x_; }
#else
#define XS_PF(k)
#endif
    const bool valid = lane < L;
    const bool is_exit = valid && (fl & SF_EV_EXIT);
    const bool is_sys = valid && !is_exit && (fl & EVF_SYSBLK);
    const bool is_solve = valid && !is_exit && !is_sys;
    const uint32_t nrules = r1 - r0;
    // the chunk's origin rows (row 0: the ClusterNode; row r: cache slot r - 1),
    // a node loaded into the cache at its first event of the segment; the
    // cache is written back only when this chunk's new origins do not fit
    {
        bool miss = false;
        if (valid && origin != SF_ORIGIN_NONE) {
            uint32_t h = (uint32_t)(mix64(origin) % XW_OC);
            miss = true;
            for (uint32_t q = 0; q < XW_OC; q++) {
                const unsigned int k = oc.key[h];
                if (k == origin + 1u) { miss = false; break; }
                if (k == 0u) break;
                h = h + 1 < XW_OC ? h + 1 : 0;
            }
        }
        if (oc.n + (uint32_t)__popcll(__ballot(miss)) > XW_OC) xw_cache_flush(st, oc, ocnw, lane);
    }
    int osr = -1;
    if (valid && origin != SF_ORIGIN_NONE) {
        uint32_t h = (uint32_t)(mix64(origin) % XW_OC);
        for (;;) {
            const unsigned int prev = atomicCAS(&oc.key[h], 0u, origin + 1u);
            if (prev == 0u) {                                  // new in the cache: load it
                atomicAdd(&oc.n, 1u);
                const uint32_t ko = aux_get(st, l, AX_ORIGIN, origin);
                oc.ko[h] = ko;
                if (ko != XNONE) nw_load(xw_node(ocnw, h), st, aux_rows(st, ko));
                break;
            }
            if (prev == origin + 1u) break;
            h = h + 1 < XW_OC ? h + 1 : 0;
        }
        osr = (int)h + 1;
    }
    XS_PF(0)
    xs.os[lane] = osr;
    __syncthreads();
    uint64_t sm = 0;                                           // earlier lanes of the same origin
    if (osr >= 0)
        for (int q = 0; q < 64; q++)
            if (xs.os[q] == osr) sm |= 1ull << q;
    sm &= (1ull << lane) - 1ull;
    XS_PF(1)
    // node bases (the first lane of each origin) and the rules' constants
    if (osr >= 0 && sm == 0) {
        const uint32_t ko = oc.ko[osr - 1];
        xs.ko[osr] = ko;
        long long b = 0, th = 0;
        if (ko != XNONE) {
            NodeWin<2> x = xw_node(ocnw, osr - 1);
            b = x.sec_sum_pass(t0);
            th = x.threads;
        }
        xs.base[osr] = b; xs.thr[osr] = th;
    }
    if (lane == 0) {
        NodeWin<2> x = snap;
        xs.base[0] = x.sec_sum_pass(t0);
        xs.thr[0] = x.threads;
        // (the previous second's QPS: read only at a second's first sync -- it is
        // a minute-bucket load from HBM)
        int64_t prevq = 0;
        bool have_prevq = false;
        for (uint32_t k = r0; k < r1; k++) {
            const DevRule& r = st.rules[k];
            XwRuleC& q = xs.rc[k - r0];
            q.rs = st.rstate[k];
            q.sync = 0;
            q.thr = r.count; q.qps = r.count;
            if (r.kind == CT_WARM_UP || r.kind == CT_WARM_UP_RATE_LIMITER) {
                if (r.limit_app == SF_APP_DEFAULT && q.rs.last_filled < t0 - t0 % 1000) {
                    if (!have_prevq) { prevq = j_d2l(x.previous_pass_qps(t0)); have_prevq = true; }
                    warm_sync(r, q.rs, t0, prevq);           // (the ClusterNode's previous second)
                    q.sync = 1;
                }
                const int64_t rest = q.rs.stored_tokens;
                if (rest >= r.warning_token) {
                    const int64_t above = rest - r.warning_token;
                    const double wq = j_next_up(1.0 / ((double)above * r.slope + 1.0 / r.count));
                    q.thr = wq; q.qps = wq;
                }
            }
            q.lstart = q.rs.latest_passed;
        }
    }
    __syncthreads();
    XS_PF(2)
    const double isec = st.interval / 1000.0;
    uint8_t sel[MAX_RULES];                                    // 0 none, 1 ClusterNode, 2 origin node
    long long cost[MAX_RULES];
    for (uint32_t kr = 0; kr < (uint32_t)MAX_RULES; kr++) {
        sel[kr] = 0; cost[kr] = -1;
        if (kr >= nrules) continue;
        const DevRule& r = st.rules[r0 + kr];
        if (is_solve && !r.always_pass) {
            const int s_ = xflow_select(st, r, r0, r1, origin, 0u);
            if (s_ == XS_CLUSTER) sel[kr] = 1;
            else if (s_ == XS_ORIGIN && osr >= 0 && xs.ko[osr] != XNONE) sel[kr] = 2;
        }
        if (r.kind == CT_RATE_LIMITER) {
            if (c > 0 && r.count > 0) cost[kr] = j_round(1.0 * c / r.count * 1000);
        } else if (r.kind == CT_WARM_UP_RATE_LIMITER) {
            cost[kr] = j_round(1.0 * c / xs.rc[kr].qps * 1000);
        }
    }
    // an exit's liveness: its entry passed (in this chunk: that lane's verdict,
    // eidx; before it: live_pre, from the walk's exit descriptor)
    XS_PF(3)
    int d = is_solve ? 1 : 0, ri = 0;
    uint32_t reach = 0, passk = 0;
    long long w = 0;
    for (int it = 0; it < 72; it++) {
        const int ed = __shfl(d, eidx >= 0 ? eidx : (int)lane);
        const bool live = is_exit && (eidx >= 0 ? ed != 0 : live_pre);
        const long long pc = (is_solve && d) ? (long long)c : 0;
        const long long td = ((is_solve && d) ? 1 : 0) - (live ? 1 : 0);
        const long long Pc = xw_excl_scan(pc, lane), Tc = xw_excl_scan(td, lane);
        xs.cm[lane] = pc; xs.td[lane] = td;
        __syncthreads();
        long long Po = 0, To = 0;
        for (uint64_t m = sm; m; m &= m - 1) {
            const int q = __ffsll((long long)m) - 1;
            Po += xs.cm[q]; To += xs.td[q];
        }
        __syncthreads();
        int nd = is_solve ? 1 : 0, nri = 0;
        uint32_t nreach = 0, npass = 0;
        long long nw = 0;
        for (uint32_t kr = 0; kr < nrules; kr++) {
            const DevRule& r = st.rules[r0 + kr];
            const bool rlk = r.kind == CT_RATE_LIMITER || r.kind == CT_WARM_UP_RATE_LIMITER;
            long long lat = 0;
            if (rlk) {                                         // latestPassedTime before this lane
                long long a = 0, b = XW_MPNEG;
                if (((passk >> kr) & 1u) && cost[kr] >= 0) { a = cost[kr]; b = t; }
                xw_mp_scan(a, b, lane);
                long long ea = __shfl_up(a, 1), eb = __shfl_up(b, 1);
                if (lane == 0) { ea = 0; eb = XW_MPNEG; }
                lat = max(xs.rc[kr].lstart + ea, eb);
            }
            if (!nd || !sel[kr]) continue;
            nreach |= 1u << kr;
            const bool on_c = sel[kr] == 1;
            const long long base = on_c ? xs.base[0] : xs.base[osr];
            const long long P = on_c ? Pc : Po;
            const long long T = on_c ? xs.thr[0] + Tc : xs.thr[osr] + To;
            bool ok = true;
            long long ww = 0;
            if (r.kind == CT_DEFAULT) {                        // DefaultController.canPass (prio excluded)
                const int32_t cur = r.grade == SF_GRADE_THREAD ? (int32_t)T : j_d2i((double)(base + P) / isec);
                ok = !((double)(int32_t)((uint32_t)cur + (uint32_t)c) > r.count);
            } else if (r.kind == CT_WARM_UP) {                 // WarmUpController.canPass
                const int64_t pq = j_d2l((double)(base + P) / isec);
                ok = (double)(pq + c) <= xs.rc[kr].thr;
            } else if (r.kind == CT_RATE_LIMITER && c <= 0) {
                ok = true;
            } else if (r.kind == CT_RATE_LIMITER && r.count <= 0) {
                ok = false;
            } else {                                           // RateLimiter / WarmUpRateLimiter
                const long long expected = cost[kr] + lat;
                if (expected > t) {
                    ww = expected - t;
                    ok = ww <= r.max_queue_ms;
                    if (!ok) ww = 0;
                }
            }
            if (!ok) { nd = 0; nri = (int)kr; }
            else { npass |= 1u << kr; nw += ww; }
        }
        const bool changed = nd != d || nreach != reach || npass != passk || nw != w || nri != ri;
        d = nd; reach = nreach; passk = npass; w = nw; ri = nri;
        if (lane == 0 && st.xw_stats) atomicAdd(&st.xw_stats[2], 1ull);
        if (!__ballot(changed)) break;
    }
    XS_PF(4)
    // the rules' state after the chunk (lane 0 writes)
    for (uint32_t kr = 0; kr < nrules; kr++) {
        const DevRule& r = st.rules[r0 + kr];
        const bool rlk = r.kind == CT_RATE_LIMITER || r.kind == CT_WARM_UP_RATE_LIMITER;
        const bool any_reach = __ballot((reach >> kr) & 1u) != 0ull;
        bool any_pass = false;
        long long fin = 0;
        if (rlk) {
            long long a = 0, b = XW_MPNEG;
            const bool el = ((passk >> kr) & 1u) && cost[kr] >= 0;
            if (el) { a = cost[kr]; b = t; }
            any_pass = __ballot(el) != 0ull;
            xw_mp_scan(a, b, lane);
            a = __shfl(a, 63); b = __shfl(b, 63);
            fin = max(xs.rc[kr].lstart + a, b);
        }
        if (lane == 0 && ((xs.rc[kr].sync && any_reach) || any_pass)) {
            DevRuleState rs = st.rstate[r0 + kr];
            if (xs.rc[kr].sync && any_reach) { rs.stored_tokens = xs.rc[kr].rs.stored_tokens; rs.last_filled = xs.rc[kr].rs.last_filled; }
            if (any_pass) rs.latest_passed = fin;
            st.rstate[r0 + kr] = rs;
        }
    }
    XS_PF(5)
    if (is_solve) {
        *myc = d ? XWC_PASS : XWC_BLOCK;
        *mst = d ? (uint8_t)(w > 0 ? SF_V_PASS_WAIT : SF_V_PASS) : (uint8_t)SF_V_BLOCK_FLOW;
        *mrule = d ? 0 : ri;
        *mwait = w;
    } else if (is_sys) {
        *myc = XWC_BLOCK; *mst = sysblk_status(fl); *mrule = sysblk_rule(fl); *mwait = 0;
    } else if (is_exit) {
        *myc = XWC_EXIT;
    }
    {   // the exits' final liveness, for the accounting
        const int ed = __shfl(d, eidx >= 0 ? eidx : (int)lane);
        *x_live = is_exit && (eidx >= 0 ? ed != 0 : live_pre);
    }
    *my_row = osr;
}

// One chunk's event fields, loaded a chunk ahead: the walk is a chain of
// dependent chunks, so HBM latency, not bandwidth, is its cost.  First level
// (sorted position j): time, flags, count, submission index, entry ref;
// second level (addresses from the first): the origin, and an exit's entry
// flags / time and -- when the entry was decided before the chunk that issues
// the loads (jd) -- its status; create time of an exit whose entry is older.
// k_gather_exit leaves a ref >= 0 only inside the exit's own segment.
struct XwEv {
    int64_t t, ref, rts, cts;
    int32_t c;
    uint32_t i, origin;
    uint8_t fl, rfl, rvs, pad;
};
__device__ __forceinline__ void xw_ld1(const SegIO& io, uint32_t j, uint32_t hi, XwEv& e) {
    if (j < hi) {
        e.t = io.ts[j]; e.fl = io.flags[j]; e.c = io.cnt[j]; e.i = io.perm[j];
        e.ref = io.eref ? io.eref[j] : -1;
    } else {
        e.t = INT64_MAX; e.fl = 0; e.c = 0; e.i = 0; e.ref = -1;
    }
}
__device__ __forceinline__ void xw_ld2(const SegIO& io, uint32_t j, uint32_t lo, uint32_t hi, uint32_t jd, XwEv& e) {
    e.origin = SF_ORIGIN_NONE; e.rfl = 0; e.rvs = 0; e.rts = 0; e.cts = 0;
    if (j >= hi) return;
    if (io.ev_origin) e.origin = io.ev_origin[e.i];
    if (e.fl & SF_EV_EXIT) {
        if (e.ref >= (int64_t)lo && e.ref < (int64_t)j) {
            e.rfl = io.flags[e.ref]; e.rts = io.ts[e.ref];
            if (e.ref < (int64_t)jd) e.rvs = io.v_status[e.ref];
        } else if (e.ref < 0 && io.cts) {
            e.cts = io.cts[j];
        }
    }
}
// the o_wait / o_rule half of emit_verdict with the submission index at hand
__device__ __forceinline__ void xw_emit(const SegIO& io, uint32_t i, int32_t wait, uint16_t rule) {
    if (!io.perm) return;
    if (io.o_wait && wait) io.o_wait[i] = wait;
    if (io.o_rule && rule) io.o_rule[i] = rule;
}

template <int MAXS>
__global__ void __launch_bounds__(64) k_decide_xw(DevState st, SegIO io, const uint32_t* seg_start,
                                                  const uint32_t* seg_res, const uint32_t* list,
                                                  const uint32_t* n_list) {
    __shared__ __align__(16) unsigned char snap_raw[sizeof(NodeWin<MAXS>)];
    __shared__ uint8_t cls[64];
    __shared__ uint8_t vch[64];                             // the previous chunk's final statuses
#ifdef SF_XW_PROFILE
    __shared__ unsigned long long pfs[8];
#else
    unsigned long long* pfs = nullptr;
#endif
    __shared__ XwRow rows[XW_KCAP];
    __shared__ XwScratch xs;
    __shared__ XwCache oc;
    __shared__ __align__(16) unsigned char ocnw[MAXS == 2 ? XW_OC * sizeof(NodeWin<2>) : 16];
    NodeWin<MAXS>& snap = *reinterpret_cast<NodeWin<MAXS>*>(snap_raw);
    const uint32_t lane = threadIdx.x;
    const ParamTable pt{st.ptab, st.pcap_mask, st.err, st.pins};
    const uint32_t nl = *n_list;
    for (uint32_t q = blockIdx.x; q < nl; q += gridDim.x) {
        const uint32_t s = list[q];
        const uint32_t lo = seg_start[s], hi = seg_start[s + 1], l = seg_res[s];
        const uint32_t r0 = st.rule_off[l], r1 = st.rule_off[l + 1];
        const bool thr_sens = (st.xw[l] & XWF_THREAD) != 0;
        // the ClusterNode lives in LDS (lane 0 updates it, every lane reads it):
        // no registers held across the chunk loop for it
        NodeWin<MAXS>& cn = snap;
        uint32_t cl = XNONE;
        if (lane == 0) { nw_load(cn, st, cluster_rows(st, l)); cl = l; }
        for (uint32_t k = lane; k < XW_OC; k += 64) oc.key[k] = 0;
        if (lane == 0) oc.n = 0;
        XwEv e;
        xw_ld1(io, lo + lane, hi, e);
        xw_ld2(io, lo + lane, lo, hi, lo, e);
        uint32_t jprev = lo;                               // start of the previous chunk (vch)
        __syncthreads();
#ifdef SF_XW_PROFILE
        unsigned long long pf_setup = 0, pf_solve = 0, pf_post = 0, pf_n = 0, pf_t = 0, pf_p[6] = {0, 0, 0, 0, 0, 0};
        if (lane < 8) pfs[lane] = 0;
#define XW_PF(k) { const unsigned long long x_ = wall_clock64(); pf_p[k] += x_ - pf_t; pf_t = x_; pf_post += 0; }
#else
#define XW_PF(k)
#endif
        for (uint32_t j0 = lo; j0 < hi;) {
#ifdef SF_XW_PROFILE
            pf_t = wall_clock64(); pf_n++;
#endif
            const int64_t t0 = __shfl(e.t, 0);
            const int64_t bs = t0 - t0 % st.wl, bm = t0 - t0 % 1000;
            const uint32_t j = j0 + lane;
            const bool valid = j < hi;
            const int64_t t = valid ? e.t : t0;
            const bool same = valid && t >= bs && t < bs + st.wl && t >= bm && t < bm + 1000;
            const unsigned long long nb = __ballot(!same);
            const uint32_t L = nb ? (uint32_t)(__ffsll((long long)nb) - 1) : 64u;   // (lane 0 is always in)
            const uint32_t jn = j0 + L;
            // the next chunk's first-level fields, in flight while this one is decided
            XwEv nx;
            xw_ld1(io, jn + lane, hi, nx);
            for (uint32_t k = lane; k < XW_KCAP; k += 64) {
                rows[k].blk = rows[k].succ = rows[k].rt = rows[k].exc = rows[k].pass = 0; rows[k].thr = 0;
                rows[k].minrt = INT64_MAX;
                rows[k].nblk = rows[k].ncmp = rows[k].nexc = rows[k].npass = 0; rows[k].key = 0;
            }
            // 1. classify
            uint8_t myc = 0, mst = 0;
            int mrule = 0;
            int64_t mwait = 0;
            const bool act = lane < L;
            const uint32_t origin = act ? e.origin : SF_ORIGIN_NONE;
            const int32_t c = act ? e.c : 0;
            const uint8_t fl = act ? e.fl : 0;
            // an exit's entry: in this chunk (eidx: that lane's verdict), or decided
            // before it (live_pre), or before this batch (ref < 0)
            int eidx = -1;
            bool live_pre = false;
            int64_t xcts = t;
            if (act && (fl & SF_EV_EXIT)) {
                const int64_t ref = e.ref;
                if (ref >= 0) {
                    if (ref < (int64_t)lo || ref >= (int64_t)j || (e.rfl & SF_EV_EXIT)) {
                        *st.err = SF_ERR_INVALID;                  // (an exit of itself: blocked)
                    } else {
                        xcts = e.rts;
                        if (ref >= (int64_t)j0) eidx = (int)(ref - j0);
                        else live_pre = !v_blocked(ref >= (int64_t)jprev ? vch[ref - jprev] : e.rvs);
                    }
                } else {
                    live_pre = ref != EREF_DEAD;
                    xcts = io.cts ? e.cts : t;
                }
            }
            // the exact chunk solve (below) unless a prioritized entry is in the chunk
            // (its occupy path) or an origin-node WarmUp rule has not synced this second
            bool jac = false;
            if constexpr (MAXS == 2) {
                jac = __ballot(act && !(fl & (SF_EV_EXIT | EVF_SYSBLK)) && (fl & SF_EV_PRIO)) == 0ull;
                for (uint32_t k = r0; k < r1 && jac; k++) {
                    const DevRule& r = st.rules[k];
                    if ((r.kind == CT_WARM_UP || r.kind == CT_WARM_UP_RATE_LIMITER) && r.limit_app != SF_APP_DEFAULT &&
                        st.rstate[k].last_filled < t0 - t0 % 1000)
                        jac = false;
                }
            }
            if constexpr (MAXS == 2) {
                if (!jac && oc.n) xw_cache_flush(st, oc, ocnw, lane);   // (the serial walk reads HBM)
            }
            if (lane == 0) {
                if (cl != l) { if (cl != XNONE) nw_store(cn, st, cluster_rows(st, cl)); nw_load(cn, st, cluster_rows(st, l)); cl = l; }
                cn.min_flush();                              // (a copy that moves to another minute slot reads HBM)
            }
            __syncthreads();
            int my_row = -1;
            bool x_live = false;
#ifdef SF_XW_PROFILE
            { const unsigned long long x = wall_clock64(); pf_setup += x - pf_t; pf_t = x; }
#endif
            if (jac) {
                if constexpr (MAXS == 2)
                    xw_solve_chunk(st, snap, rows, xs, oc, ocnw, lane, L, t0, t, fl, c, origin, eidx, live_pre, l,
                                   r0, r1, &myc, &mst, &mrule, &mwait, &my_row, &x_live, pfs);
            } else {
                if (act) {
                    if (fl & SF_EV_EXIT) myc = thr_sens ? XWC_SERIAL : XWC_EXIT;
                    else if (fl & EVF_SYSBLK) { myc = XWC_BLOCK; mst = sysblk_status(fl); mrule = sysblk_rule(fl); }
                    else myc = XWC_SERIAL;
                }
                const unsigned long long exits = __ballot(act && (fl & SF_EV_EXIT));
                const int64_t ex_before = (int64_t)__popcll(exits & ((1ull << lane) - 1ull));
                if (myc == XWC_SERIAL && !(fl & (SF_EV_EXIT | SF_EV_PRIO))) {
                    for (uint32_t k = r0; k < r1; k++) {
                        const DevRule& r = st.rules[k];
                        if (r.always_pass) continue;
                        const int sel = xflow_select(st, r, r0, r1, origin, 0u);
                        if (sel == XS_NONE) continue;
                        DevRuleState rs = st.rstate[k];
                        int64_t w = 0; bool pw = false; int ok = 1;
                        if (sel == XS_CLUSTER) {
                            NodeWin<MAXS> x = snap;                  // (minute bucket clean: never written back)
                            x.threads -= ex_before;
                            ok = can_pass<MAXS>(r, rs, x, t, c, false, st.occupy_timeout, &w, &pw);
                        } else if (sel == XS_ORIGIN) {
                            // a WarmUp rule shared by several origin nodes (`other`) syncs its
                            // tokens at the second's first check, with THAT event's origin's
                            // previous QPS: until the walk has synced this second, its entries
                            // stay in the serial part
                            const bool warm = r.kind == CT_WARM_UP || r.kind == CT_WARM_UP_RATE_LIMITER;
                            if (warm && rs.last_filled < t - t % 1000) break;
                            const uint32_t ko = aux_get(st, l, AX_ORIGIN, origin);
                            if (ko != XNONE) {
                                NodeWin<MAXS> x;
                                nw_load(x, st, aux_rows(st, ko));
                                x.threads -= ex_before;
                                ok = can_pass<MAXS>(r, rs, x, t, c, false, st.occupy_timeout, &w, &pw);
                            }
                        }
                        if (!ok) { myc = XWC_BLOCK; mst = SF_V_BLOCK_FLOW; mrule = (int)(k - r0); }
                        break;                                   // only the first selecting rule decides here
                    }
                }
            }
#ifdef SF_XW_PROFILE
            { const unsigned long long x = wall_clock64(); pf_solve += x - pf_t; pf_t = x; }
#endif
            // the next chunk's second-level fields (its entries decided before this
            // chunk are final; those in this chunk come from vch below)
            xw_ld2(io, jn + lane, lo, hi, j0, nx);
            if (act) cls[lane] = myc;
            if (myc == XWC_BLOCK || myc == XWC_PASS) io.v_status[j] = mst;   // (before the walk: its exits read it)
            __syncthreads();
            XW_PF(0)
            // 2. the serial walk over the undecided events (entered only when there
            // are some: the walk's calls save and restore the live registers)
            const unsigned long long nser = __popcll(__ballot(act && myc == XWC_SERIAL));
            if (nser) {
                if (lane == 0) {
                    NodeWin<MAXS> on, dn;                    // (origin / context node of the walk)
                    uint32_t oi = XNONE, di = XNONE;
                    for (uint32_t k = 0; k < L; k++)
                        if (cls[k] == XWC_SERIAL) xg_event<MAXS>(st, io, pt, lo, j0 + k, cn, on, dn, cl, oi, di);
                    if (oi != XNONE) nw_store(on, st, aux_rows(st, oi));
                    if (di != XNONE) nw_store(dn, st, aux_rows(st, di));
                }
                __syncthreads();
            }
            if (lane == 0 && st.xw_stats) {
                atomicAdd(&st.xw_stats[jac ? 0 : 1], 1ull);
                if (nser) atomicAdd(&st.xw_stats[3], nser);
            }
            XW_PF(1)
            // 3. the blocks and completions, summed per node
            int64_t blk = 0, succ = 0, rt = 0, exc = 0, thr = 0, minrt = INT64_MAX;
            int nblk = 0, ncmp = 0, nexc = 0;
            int64_t pss = 0;
            int npss = 0;
            uint8_t vfin = mst;                                  // this lane's final status (vch)
            if (myc == XWC_BLOCK) {
                xw_emit(io, e.i, (int32_t)mwait, (uint16_t)mrule);
                blk = c; nblk = 1;
            } else if (myc == XWC_PASS) {
                xw_emit(io, e.i, (int32_t)mwait, 0);
                pss = c; npss = 1;
            } else if (myc == XWC_EXIT) {                    // StatisticSlot.exit :134-165
                // (liveness from the solve; on the serial path an entry of this
                // chunk has its status in v_status by now)
                const bool live = jac ? x_live
                                      : (eidx >= 0 ? !v_blocked(io.v_status[j0 + eidx]) : live_pre);
                uint8_t v = SF_V_EXIT_IGNORED;
                if (live) {
                    v = SF_V_EXIT;
                    succ = c; rt = t - xcts; minrt = rt; thr = -1; ncmp = 1;
                    if (fl & SF_EV_ERROR) { exc = c; nexc = 1; }
                }
                io.v_status[j] = v;
                vfin = v;
            } else if (myc == XWC_SERIAL) {
                vfin = io.v_status[j];                       // (lane 0's walk wrote it)
            }
            // the ClusterNode's sums: wavefront reductions (every lane adds to it)
            XwRow crow;
            {
                long long v[6] = {blk, succ, rt, exc, thr, pss};
#pragma unroll
                for (int f = 0; f < 6; f++) v[f] = xw_wsum(v[f]);
                const long long mr = xw_wmin(minrt);
                crow.blk = (unsigned long long)v[0]; crow.succ = (unsigned long long)v[1];
                crow.rt = (unsigned long long)v[2]; crow.exc = (unsigned long long)v[3];
                crow.thr = v[4] + (long long)__popcll(__ballot(npss != 0)); crow.pass = (unsigned long long)v[5];
                crow.minrt = mr;
                crow.nblk = (unsigned)__popcll(__ballot(nblk != 0)); crow.ncmp = (unsigned)__popcll(__ballot(ncmp != 0));
                crow.nexc = (unsigned)__popcll(__ballot(nexc != 0)); crow.npass = (unsigned)__popcll(__ballot(npss != 0));
            }
            XW_PF(2)
            if (nblk || ncmp || npss) {
                if (jac) {
                    if (my_row > 0) xw_add(rows[my_row], blk, nblk, succ, rt, minrt, exc, nexc, thr, ncmp, pss, npss);
                } else if (origin != SF_ORIGIN_NONE) {
                    uint32_t h = 1 + (uint32_t)(mix64(origin) % (XW_KCAP - 1));
                    for (;;) {
                        const unsigned int prev = atomicCAS(&rows[h].key, 0u, origin + 1u);
                        if (prev == 0u || prev == origin + 1u) break;
                        h = h + 1 < XW_KCAP ? h + 1 : 1;
                    }
                    xw_add(rows[h], blk, nblk, succ, rt, minrt, exc, nexc, thr, ncmp, pss, npss);
                }
            }
            __syncthreads();
            XW_PF(3)
            if (lane == 0) xw_apply<MAXS>(cn, crow, t0);
            if constexpr (MAXS == 2) {
                if (jac) {                                       // into the cached origin nodes
                    for (uint32_t k = 1 + lane; k < XW_KCAP; k += 64)
                        if ((rows[k].nblk | rows[k].ncmp | rows[k].npass | rows[k].nexc) && oc.ko[k - 1] != XNONE)
                            xw_apply<2>(xw_node(ocnw, k - 1), rows[k], t0);
                }
            }
            for (uint32_t k = 1 + lane; k < XW_KCAP && !jac; k += 64) {
                if (!rows[k].key) continue;
                const uint32_t ko = aux_get(st, l, AX_ORIGIN, rows[k].key - 1u);
                if (ko == XNONE) continue;
                NodeWin<MAXS> x;
                const NodeRows nr = aux_rows(st, ko);
                nw_load(x, st, nr);
                xw_apply<MAXS>(x, rows[k], t0);
                nw_store(x, st, nr);
            }
            XW_PF(4)
            // the next chunk: its exits of entries in this chunk read vch
            if (act) vch[lane] = vfin;
            __syncthreads();
            jprev = j0;
            e = nx;
            XW_PF(5)
            j0 = jn;
        }
#ifdef SF_XW_PROFILE
        if (lane == 0 && hi - lo > 20000)
            printf("xw seg n=%u chunks=%llu setup=%llu solve=%llu (%llu %llu %llu %llu %llu %llu) post %llu %llu %llu %llu %llu %llu (x10ns)\n", hi - lo,
                   pf_n, pf_setup, pf_solve, pfs[0], pfs[1], pfs[2], pfs[3], pfs[4], pfs[5], pf_p[0], pf_p[1], pf_p[2], pf_p[3], pf_p[4], pf_p[5]);
#endif
        if constexpr (MAXS == 2) xw_cache_flush(st, oc, ocnw, lane);
        if (lane == 0 && cl != XNONE) nw_store(cn, st, cluster_rows(st, cl));
        __syncthreads();
    }
}

// One lane per short segment routed to the lean QPS walk (SM_LIGHTQ), from
// the back of the dense short list like k_decide_short.
template <int MAXS>
__global__ void __launch_bounds__(128) k_decide_short_qps(DevState st, SegIO io, const uint32_t* seg_start,
                                                          const uint32_t* seg_res, LightLists ll,
                                                          const uint32_t* n_short) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_short[1]) return;
    const uint32_t s = ll.list[ll.off[0] + ll.cap[0] - 1 - t];
    decide_qps_segment<MAXS>(st, io, seg_res[s], seg_start[s], seg_start[s + 1]);
}

static HeavyCtx heavy_ctx(const Work& w) {
    HeavyCtx hc;
    hc.seg_start = w.seg_start; hc.seg_res = w.seg_res; hc.seg_mode = w.seg_mode;
    hc.heavy_list = w.heavy_list; hc.n_heavy = w.counters + 1; hc.pcg = w.pcg; hc.seg_cap = w.seg_cap;
    hc.acc_hw = (Acc*)w.acc_hw; hc.acc_sec = (Acc*)w.acc_sec;
    hc.acc_hw_base = w.acc_hw_base; hc.acc_sec_base = w.acc_sec_base;
    hc.seg_hw0 = w.seg_hw0; hc.seg_sec0 = w.seg_sec0;
    hc.hticks = nullptr;
    hc.passbits = w.passbits;
    hc.exit_of = w.exit_of;
    hc.lxfar = w.lxfar;
    hc.thr_rec = w.thr_rec;
    hc.rid = w.keys_in; hc.run_start = w.head_scan; hc.run_pre = w.keys_out; hc.rrec = (uint2*)w.pv_in;
    hc.seg_rb = w.seg_rb; hc.seg_re = w.seg_re; hc.segflag = w.segflag;
    return hc;
}

// SM_PARAM: a ParamFlow-only resource whose rules are QPS-grade on one
// argument index (heavy_mode).  ParamFlowChecker's state is per (rule, value)
// (ParameterMetric token / time maps) and the node counters are only summed,
// so events of different values are independent: the wavefront takes 64
// events at a time, and the first lane of each distinct value in the 64 runs
// that value's events in order, rule by rule, with the (rule, value) state in
// registers (param_run_rule: one table find and one write per rule, however
// often the value recurs -- a Zipf head value recurs in most groups).  The
// finds of a rule all complete before any of its inserts (the wavefront runs
// them in lock-step; distinct values never share a key).  Verdict inputs go to
// the pass bits, v_wait (throttled passes) and v_rule (the blocking rule);
// k_heavy_fill and k_heavy_apply then do the StatisticSlot accounting as for
// the other window modes.
__device__ void heavy_param(const DevState& st, const SegIO& io, const HeavyCtx& hc, uint32_t res, uint32_t lo,
                            uint32_t hi) {
    __shared__ int64_t s_now[64], s_wait[64];
    __shared__ int32_t s_c[64];
    __shared__ uint8_t s_rule[64], s_ok[64];
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t p0 = st.prule_off[res], np = st.prule_off[res + 1] - p0;
    const int32_t pidx = st.prules[p0].param_idx;
    const uint8_t pm_init = (uint8_t)(st.pm_init[res] | (1u << pidx));   // initParamMetricsFor on the first entry
    ParamTable pt{st.ptab, st.pcap_mask, st.err, st.pins};
    for (uint32_t q = lo; q < hi; q += 64) {
        const uint32_t j = q + (uint32_t)lane;
        const bool valid = j < hi;
        const uint32_t jc = valid ? j : hi - 1;
        const int64_t now = io.ts[jc];
        const int32_t c = io.cnt[jc];
        const uint32_t na = io.arg_slots ? (io.nargs ? io.nargs[jc] : io.arg_slots) : 0;
        uint32_t tag = SF_TAG_NULL; uint64_t bits = 0;
        if ((int32_t)na > pidx) { tag = io.atag[(size_t)pidx * io.n + jc]; bits = io.abits[(size_t)pidx * io.n + jc]; }
        const bool sysb = valid && (io.flags[jc] & EVF_SYSBLK);   // blocked before ParamFlowSlot
        const bool key = valid && !sysb && tag != SF_TAG_NULL;  // a null value skips every rule (passCheck :53-60)
        s_now[lane] = now; s_c[lane] = c; s_wait[lane] = 0; s_rule[lane] = 0; s_ok[lane] = 0;
        // the lanes of each distinct value: `mine` on the value's first lane
        unsigned long long pend = __ballot(key), mine = 0;
        while (pend) {
            const int l = __ffsll((long long)pend) - 1;
            const uint32_t kt = (uint32_t)__builtin_amdgcn_readlane((int)tag, l);
            const uint64_t kb = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bits >> 32), l) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bits, l);
            const unsigned long long same = __ballot(key && tag == kt && bits == kb);
            if (lane == l) mine = same;
            pend &= ~same;
        }
        __syncthreads();
        if (mine) {
            uint64_t live = mine;
            for (uint32_t k = 0; k < np && live; k++) {
                const uint64_t before = live;
                live = param_run_rule(pt, res, (int)k, st.prules[p0 + k], st.items, tag, bits, live,
                                      [&](int o) { return s_now[o]; }, [&](int o) { return s_c[o]; },
                                      [&](int o, int64_t w) { s_wait[o] += w; });
                for (uint64_t m = before & ~live; m; m &= m - 1) s_rule[__builtin_ctzll(m)] = (uint8_t)k;
            }
            for (uint64_t m = live; m; m &= m - 1) s_ok[__builtin_ctzll(m)] = 1;
            // ParamFlowStatisticEntryCallback: the value's thread count, once for all its passes
            if (live && ((pm_init >> pidx) & 1)) pm_thread_add(pt, res, pidx, tag, bits, __popcll(live));
        }
        __syncthreads();
        const bool blocked = sysb || (key && !s_ok[lane]);
        const unsigned long long pm = __ballot(valid && !blocked);
        if (lane == 0 && pm) {
            const uint32_t sh = q & 63;
            atomicOr(hc.passbits + (q >> 6), pm << sh);
            if (sh) atomicOr(hc.passbits + (q >> 6) + 1, pm >> (64 - sh));
        }
        if (valid) { io.v_wait[j] = blocked ? 0 : (int32_t)s_wait[lane]; io.v_rule[j] = blocked && key ? s_rule[lane] : 0; }
    }
    if (lane == 0) st.pm_init[res] = pm_init;
}

// One wavefront per heavy QPS / WarmUp / no-rule / generic segment (64-thread
// workgroups: the team needs no barriers).  THREAD and RateLimiter segments
// run in k_heavy_stream (sf_stream.h).
template <int MAXS>
__global__ void __launch_bounds__(64) k_heavy_decide(DevState st, SegIO io, HeavyCtx hc) {
    // grid-stride over the list (medium ParamFlow segments can outnumber the
    // grid sized for segments above heavy_min); long segments are listed first
    uint32_t s;
    for (uint32_t b = blockIdx.x; heavy_at(hc, b, &s); b += gridDim.x) {
        const uint32_t lo = hc.seg_start[s], hi = hc.seg_start[s + 1], res = hc.seg_res[s];
        Team tm{(int)threadIdx.x};
        const uint64_t t_start = hc.hticks ? wall_clock64() : 0;
        switch (hc.seg_mode[s]) {
        case SM_QPS: heavy_qps<MAXS>(tm, st, io, hc, s, res, lo, hi, false); break;
        case SM_WARM: heavy_qps<MAXS>(tm, st, io, hc, s, res, lo, hi, true); break;
        case SM_NORULE: break;                      // every entry passes (k_heavy_fill)
        case SM_PARAM: heavy_param(st, io, hc, res, lo, hi); break;
        default:
            if (tm.leader()) decide_segment<MAXS>(st, io, res, lo, hi);
            break;
        }
        if (hc.hticks && tm.leader() && b < gridDim.x) hc.hticks[b] = wall_clock64() - t_start;
    }
}

struct PAcc {            // per-thread partial of one accumulator slot
    unsigned long long pass, block, succ, rt, exc, n_pass, n_exit, n_touch;
    long long min_rt;
    __device__ void clear() { pass = block = succ = rt = exc = n_pass = n_exit = n_touch = 0; min_rt = INT64_MAX; }
    __device__ void add(const EvContrib& e) {
        n_touch++;
        if (e.live_exit) {
            succ += (unsigned long long)e.c; rt += (unsigned long long)e.rt; n_exit++;
            if (e.err) exc += (unsigned long long)e.c;
            if (e.rt < min_rt) min_rt = e.rt;
        } else if (e.passed) { pass += (unsigned long long)e.c; n_pass++; }
        else block += (unsigned long long)e.c;
    }
    __device__ void merge(const PAcc& o) {
        pass += o.pass; block += o.block; succ += o.succ; rt += o.rt; exc += o.exc;
        n_pass += o.n_pass; n_exit += o.n_exit; n_touch += o.n_touch;
        if (o.min_rt < min_rt) min_rt = o.min_rt;
    }
    __device__ void flush(Acc* table, uint32_t key) const {
        if (!n_touch) return;
        Acc* a = table + key;
        atomicAdd(&a->pass, pass); atomicAdd(&a->block, block); atomicAdd(&a->succ, succ);
        atomicAdd(&a->rt, rt); atomicAdd(&a->exc, exc); atomicAdd(&a->n_pass, n_pass);
        atomicAdd(&a->n_exit, n_exit); atomicAdd(&a->n_touch, n_touch);
        if (min_rt != INT64_MAX) atomicMin(&a->min_rt, min_rt);
    }
};

__device__ unsigned long long wave_sum(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ long long wave_min(long long v) {
    for (int o = 32; o > 0; o >>= 1) { long long u = __shfl_xor(v, o); v = u < v ? u : v; }
    return v;
}
// flush at wave level: one set of atomics per wave when all active lanes share a key
__device__ void wave_flush(PAcc& p, uint32_t key, Acc* table) {
    const uint32_t NONE = 0xffffffffu;
    bool act = key != NONE && p.n_touch;
    unsigned long long m = __ballot(act);
    if (!m) return;
    int l0 = __ffsll((long long)m) - 1;
    uint32_t k0 = __shfl(key, l0);
    bool differ = __ballot(act && key != k0) != 0;
    if (differ) { if (act) p.flush(table, key); return; }
    if (!act) p.clear();
    PAcc r;
    r.pass = wave_sum(p.pass); r.block = wave_sum(p.block); r.succ = wave_sum(p.succ); r.rt = wave_sum(p.rt);
    r.exc = wave_sum(p.exc); r.n_pass = wave_sum(p.n_pass); r.n_exit = wave_sum(p.n_exit);
    r.n_touch = wave_sum(p.n_touch); r.min_rt = wave_min(p.min_rt);
    if ((int)(threadIdx.x & 63) == l0) r.flush(table, k0);
}

// workgroup flush: the waves' partials of one key are merged in LDS first,
// so a hot window row takes one set of atomics per workgroup
struct PAccSlot { PAcc p; uint32_t key; };
__device__ void block_flush(PAcc& p, uint32_t key, Acc* table, PAccSlot* lds) {
    const uint32_t NONE = 0xffffffffu;
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6), nw = (int)(blockDim.x >> 6);
    bool act = key != NONE && p.n_touch;
    const unsigned long long m = __ballot(act);
    uint32_t k0 = NONE;
    bool uni = false;
    if (m) {
        const int l0 = __ffsll((long long)m) - 1;
        k0 = __shfl(key, l0);
        uni = __ballot(act && key != k0) == 0;
    }
    if (m && !uni) { if (act) p.flush(table, key); }      // mixed keys: lane atomics
    PAcc r; r.clear();
    if (m && uni) {
        if (!act) p.clear();
        r.pass = wave_sum(p.pass); r.block = wave_sum(p.block); r.succ = wave_sum(p.succ); r.rt = wave_sum(p.rt);
        r.exc = wave_sum(p.exc); r.n_pass = wave_sum(p.n_pass); r.n_exit = wave_sum(p.n_exit);
        r.n_touch = wave_sum(p.n_touch); r.min_rt = wave_min(p.min_rt);
    }
    if (lane == 0) { lds[wv].p = r; lds[wv].key = (m && uni) ? k0 : NONE; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int a = 0; a < nw; a++) {
            if (lds[a].key == NONE) continue;
            PAcc acc = lds[a].p;
            for (int b = a + 1; b < nw; b++) {
                if (lds[b].key != lds[a].key) continue;
                const PAcc& o = lds[b].p;
                acc.pass += o.pass; acc.block += o.block; acc.succ += o.succ; acc.rt += o.rt; acc.exc += o.exc;
                acc.n_pass += o.n_pass; acc.n_exit += o.n_exit; acc.n_touch += o.n_touch;
                if (o.min_rt < acc.min_rt) acc.min_rt = o.min_rt;
                lds[b].key = NONE;
            }
            acc.flush(table, lds[a].key);
        }
    }
    __syncthreads();
}


// Tiles of FILL_TILE events over the heavy segments of each class (block c:
// class c): cls 0 = k_heavy_decide's list (QPS / WarmUp / no rule; generic
// segments wrote their verdicts themselves), cls 1 = k_heavy_stream's list
// (THREAD / RL).  k_heavy_fill then reads only the events of its class.
__global__ void __launch_bounds__(1024) k_fill_tiles(HeavyCtx hc, StreamCtx sc, uint2* tiles, uint32_t cap,
                                                     uint32_t* ntiles) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const int c = (int)blockIdx.x;
    uint2* out = tiles + (size_t)c * cap;
    const uint32_t nl = c == 0 ? hc.n_heavy[0] + hc.n_heavy[3] : sc.n_list[0] + sc.n_list[1];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nl; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        uint32_t s = 0, nt = 0;
        if (i < nl) {
            const bool ok = c == 0 ? heavy_at(hc, i, &s) : stream_at(sc, i, &s);
            if (ok && hc.seg_mode[s] >= SM_QPS)                 // aligned FILL_TILE blocks the segment overlaps
                nt = (hc.seg_start[s + 1] - 1) / FILL_TILE - hc.seg_start[s] / FILL_TILE + 1;
        }
        const uint32_t incl = (uint32_t)wave_scan_add((int)nt);
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        uint32_t before = carry;
        for (int k = 0; k < wv; k++) before += wsum[k];
        const uint32_t base = before + incl - nt;
        const uint32_t g0 = nt ? hc.seg_start[s] / FILL_TILE : 0;
        for (uint32_t k = 0; k < nt && base + k < cap; k++) out[base + k] = make_uint2(s, g0 + k);
        __syncthreads();
        if (threadIdx.x == 1023) carry = before + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) ntiles[c] = min(carry, cap);
}

// THREAD-grade stream segments, state-independent preparation (at the head of
// the decide phase, launch_thr_prep), grid-stride over the stream class's fill
// tiles.  A run is a maximal stretch of a segment's checked entries, or of its
// other events (sf_stream.h run mode).
//   k_thr_heads  run heads of each tile; the segment flag of an acquireCount
//                beyond THR_CBIG
__global__ void __launch_bounds__(256) k_thr_heads(const uint8_t* flags, const int32_t* cnt, HeavyCtx hc,
                                                   const uint2* tiles, const uint32_t* ntiles, uint32_t* tile_rc,
                                                   uint32_t* segflag) {
    __shared__ uint32_t heads;
    const uint32_t nt = ntiles[1];
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const uint2 tl = tiles[t];
        const uint32_t s = tl.x;
        if (hc.seg_mode[s] != SM_THREAD) { if (threadIdx.x == 0) tile_rc[t] = 0; continue; }
        if (threadIdx.x == 0) heads = 0;
        __syncthreads();
        const uint32_t lo = hc.seg_start[s], hi = hc.seg_start[s + 1];
        uint32_t nh = 0;
        bool big = false;
        for (uint32_t j = max(tl.y * FILL_TILE, lo) + threadIdx.x; j < min(tl.y * FILL_TILE + FILL_TILE, hi); j += 256) {
            const uint8_t f = flags[j];
            const bool ent = is_checked_entry(f);
            if (ent) big |= cnt[j] > THR_CBIG;
            nh += (j == lo || ent != is_checked_entry(flags[j - 1])) ? 1u : 0u;
        }
        if (__ballot(big) && (threadIdx.x & 63) == 0) atomicOr(&segflag[s], SEGF_BIGC);
        nh = (uint32_t)wave_sum(nh);
        if ((threadIdx.x & 63) == 0 && nh) atomicAdd(&heads, nh);
        __syncthreads();
        if (threadIdx.x == 0) tile_rc[t] = heads;
        __syncthreads();
    }
}

//   k_thr_rscan  exclusive scan of the tiles' run counts (global run ids:
//                the runs of a segment are a contiguous range, in order)
//   k_thr_rid    run id of every event, run starts, the segment's run range
//   k_thr_rec    the event records the stream kernel reads: run-mode segments
//                (thr_run_mode) entry records (run id of the exit,
//                acquireCount), exits live from before the batch counted per
//                run; the others one 8-B window-walk record per event
__global__ void __launch_bounds__(1024) k_thr_rscan(uint32_t* tile_rc, const uint32_t* ntiles) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const uint32_t nt = ntiles[1];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nt; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < nt ? tile_rc[i] : 0u;
        const uint32_t incl = (uint32_t)wave_scan_add((int)v);
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        uint32_t before = carry;
        for (int k = 0; k < wv; k++) before += wsum[k];
        if (i < nt) tile_rc[i] = before + incl - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry = before + incl;
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) k_thr_rid(const uint8_t* flags, HeavyCtx hc, const uint2* tiles,
                                                 const uint32_t* ntiles, const uint32_t* tile_rb) {
    __shared__ uint32_t wsum[4];
    constexpr uint32_t PER = FILL_TILE / 256;
    const uint32_t nt = ntiles[1];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const uint2 tl = tiles[t];
        const uint32_t s = tl.x;
        if (hc.seg_mode[s] != SM_THREAD) continue;
        const uint32_t lo = hc.seg_start[s], hi = hc.seg_start[s + 1];
        const uint32_t base = tl.y * FILL_TILE + PER * threadIdx.x;
        uint32_t hm = 0;                                   // heads among this thread's PER events
#pragma unroll
        for (uint32_t k = 0; k < PER; k++) {
            const uint32_t j = base + k;
            if (j >= lo && j < hi && (j == lo || is_checked_entry(flags[j]) != is_checked_entry(flags[j - 1])))
                hm |= 1u << k;
        }
        const uint32_t c = (uint32_t)__popc(hm);
        const uint32_t incl = (uint32_t)wave_scan_add((int)c);
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        uint32_t run = tile_rb[t] + incl - c;              // heads before this thread's events in the tile
        for (int k = 0; k < wv; k++) run += wsum[k];
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < PER; k++) {
            const uint32_t j = base + k;
            if (j < lo || j >= hi) continue;
            if ((hm >> k) & 1u) { run++; hc.run_start[run - 1] = j; hc.run_pre[run - 1] = 0u; }
            hc.rid[j] = run - 1;                           // (a tile's events before its first head: the last run before it)
            if (j == lo) hc.seg_rb[s] = run - 1;
            if (j == hi - 1) hc.seg_re[s] = run;
        }
    }
}

__global__ void __launch_bounds__(256) k_thr_rec(const uint8_t* flags, const int32_t* cnt, const int64_t* eref,
                                                 HeavyCtx hc, const uint2* tiles, const uint32_t* ntiles,
                                                 const uint32_t* segflag) {
    const uint32_t nt = ntiles[1];
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const uint2 tl = tiles[t];
        const uint32_t s = tl.x;
        if (hc.seg_mode[s] != SM_THREAD) continue;
        const uint32_t lo = hc.seg_start[s], hi = hc.seg_start[s + 1];
        const bool runs = thr_run_mode(hc, s, lo, hi, segflag[s]);
        for (uint32_t j = max(tl.y * FILL_TILE, lo) + threadIdx.x; j < min(tl.y * FILL_TILE + FILL_TILE, hi); j += 256) {
            const uint8_t f = flags[j];
            if (runs) {
                if (is_checked_entry(f)) {
                    const uint32_t x = hc.exit_of[j];
                    hc.rrec[j] = make_uint2(x < hi ? hc.rid[x] : XO_NONE, (uint32_t)cnt[j]);
                } else if ((f & SF_EV_EXIT) && (eref ? eref[j] : -1) == -1) {
                    atomicAdd(&hc.run_pre[hc.rid[j]], 1u);      // its entry passed before this batch: live
                }
                continue;
            }
            uint2 r;
            if (is_checked_entry(f)) { r.x = hc.exit_of[j]; r.y = (uint32_t)cnt[j]; }
            else if (!(f & SF_EV_EXIT)) { r.x = 0u; r.y = THR_REC_EXIT; }   // blocked before: a no-op (dead exit)
            else {
                const int64_t ref = eref ? eref[j] : -1;
                r.x = ref >= 0 ? j - (uint32_t)ref : 0u;
                r.y = THR_REC_EXIT | (ref == -1 ? THR_REC_LIVE : 0u);
            }
            ((uint2*)hc.thr_rec)[j] = r;
        }
    }
}

// Verdicts and per-window counter deltas of the heavy segments of one class.
// A tile is one segment's part of an aligned FILL_TILE-event block of the
// sorted batch; lane t owns the aligned group of 16 events at block + 16 t, so
// every array is read and written with 16-byte vector accesses (groups cut by
// a segment edge fall back to per-event accesses) and all of a lane's loads
// are in flight together.  Each event is one pass-bit lookup (its entry's bit
// for an exit).  Persistent grid, each workgroup a contiguous run of tiles; a
// thread's partial sums carry across the run while the window row repeats.
// Window rows of a run of tiles accumulated in LDS: ACC_K consecutive
// accumulator slots from `base`, 64-bit LDS atomics; flushed to the global
// rows (one set of atomics per touched slot) only when a tile's window range
// leaves the table or the workgroup's run ends, so the rows of a hot
// resource take one flush per window, not one per thread or tile.
constexpr int ACC_K = 32;
struct LdsAcc {
    unsigned long long v[8][ACC_K];                 // pass, block, succ, rt, exc, n_pass, n_exit, n_touch
    long long min_rt[ACC_K];
};
__device__ __forceinline__ void lds_acc_clear(LdsAcc& A) {
    for (int i = threadIdx.x; i < 8 * ACC_K; i += blockDim.x) A.v[i / ACC_K][i % ACC_K] = 0ull;
    for (int i = threadIdx.x; i < ACC_K; i += blockDim.x) A.min_rt[i] = INT64_MAX;
}
__device__ __forceinline__ void lds_acc_add(LdsAcc& A, uint32_t k, const PAcc& p) {
    if (!p.n_touch) return;
    if (p.pass) atomicAdd(&A.v[0][k], p.pass);
    if (p.block) atomicAdd(&A.v[1][k], p.block);
    if (p.succ) atomicAdd(&A.v[2][k], p.succ);
    if (p.rt) atomicAdd(&A.v[3][k], p.rt);
    if (p.exc) atomicAdd(&A.v[4][k], p.exc);
    if (p.n_pass) atomicAdd(&A.v[5][k], p.n_pass);
    if (p.n_exit) atomicAdd(&A.v[6][k], p.n_exit);
    atomicAdd(&A.v[7][k], p.n_touch);
    if (p.min_rt != INT64_MAX) atomicMin(&A.min_rt[k], p.min_rt);
}
// flush slots to table[base + k] (thread k), then clear; callers bracket with barriers
__device__ __forceinline__ void lds_acc_flush(LdsAcc& A, Acc* table, uint32_t base) {
    const int k = (int)threadIdx.x;
    if (k < ACC_K && A.v[7][k]) {
        PAcc p;
        p.pass = A.v[0][k]; p.block = A.v[1][k]; p.succ = A.v[2][k]; p.rt = A.v[3][k]; p.exc = A.v[4][k];
        p.n_pass = A.v[5][k]; p.n_exit = A.v[6][k]; p.n_touch = A.v[7][k]; p.min_rt = A.min_rt[k];
        p.flush(table, base + (uint32_t)k);
    }
}

constexpr int FG = (int)FILL_TILE / 256;         // events per lane
struct FillGrp { uint8_t f[FG]; int32_t c[FG]; int64_t t[FG]; };

// vector copy of an aligned group: 16-byte accesses (8-byte for an 8-byte group)
__device__ __forceinline__ void load16(void* dst, const void* src, int bytes) {
    if (bytes == 8) { *(uint2*)dst = *(const uint2*)src; return; }
    uint4* d = (uint4*)dst; const uint4* q = (const uint4*)src;
#pragma unroll
    for (int k = 0; k < bytes / 16; k++) d[k] = q[k];
}
__device__ __forceinline__ void store16(void* dst, const void* src, int bytes) {
    if (bytes == 8) { *(uint2*)dst = *(const uint2*)src; return; }
    uint4* d = (uint4*)dst; const uint4* q = (const uint4*)src;
#pragma unroll
    for (int k = 0; k < bytes / 16; k++) d[k] = q[k];
}

#ifndef SF_FILL_MINB
#define SF_FILL_MINB 1
#endif
__global__ void __launch_bounds__(256, SF_FILL_MINB) k_heavy_fill(DevState st, SegIO io, HeavyCtx hc, const uint2* tiles,
                                                    const uint32_t* ntiles, int cls) {
    __shared__ LdsAcc acc_h, acc_s;
    const uint32_t NONE = 0xffffffffu;
    const uint32_t nt = ntiles[cls];
    const uint32_t wl = (uint32_t)st.wl;
    const uint32_t tb = (uint32_t)((uint64_t)nt * blockIdx.x / gridDim.x);
    const uint32_t te = (uint32_t)((uint64_t)nt * (blockIdx.x + 1) / gridDim.x);
    lds_acc_clear(acc_h); lds_acc_clear(acc_s);
    uint32_t bh_k = NONE, bs_k = NONE;                // LDS table bases (workgroup-uniform)
    __syncthreads();
    for (uint32_t t = tb; t < te; t++) {
        const uint2 tl = tiles[t];
        const uint32_t s = tl.x;
        const uint32_t lo = hc.seg_start[s], hi = hc.seg_start[s + 1];
        const uint8_t mode = hc.seg_mode[s];
        const bool all = mode == SM_NORULE, rl = mode == SM_RL, prm = mode == SM_PARAM;
        const uint32_t hwb = hc.acc_hw_base[s], secb = hc.acc_sec_base[s];
        const int64_t hw0 = hc.seg_hw0[s], sec0 = hc.seg_sec0[s];
        const int64_t bh = hw0 * st.wl, bs = sec0 * 1000;
        const bool rel32 = io.ts[hi - 1] - bs < (int64_t)0xffffffffLL;   // window keys by 32-bit division
        auto key_of = [&](int64_t tj, uint32_t& kh_, uint32_t& ks_) {
            if (rel32) { kh_ = hwb + (uint32_t)(tj - bh) / wl; ks_ = secb + (uint32_t)(tj - bs) / 1000u; }
            else { kh_ = hwb + (uint32_t)(tj / st.wl - hw0); ks_ = secb + (uint32_t)(tj / 1000 - sec0); }
        };
        // the tile's window rows; a range that leaves the LDS tables flushes them first
        uint32_t th0, ts0, th1, ts1;
        key_of(io.ts[max(tl.y * FILL_TILE, lo)], th0, ts0);
        key_of(io.ts[min(tl.y * FILL_TILE + FILL_TILE, hi) - 1], th1, ts1);
        const bool wide = th1 - th0 >= (uint32_t)ACC_K || ts1 - ts0 >= (uint32_t)ACC_K;
        if (wide || bh_k == NONE || th0 < bh_k || th1 >= bh_k + ACC_K || ts0 < bs_k || ts1 >= bs_k + ACC_K) {
            __syncthreads();
            if (bh_k != NONE) { lds_acc_flush(acc_h, hc.acc_hw, bh_k); lds_acc_flush(acc_s, hc.acc_sec, bs_k); }
            __syncthreads();
            lds_acc_clear(acc_h); lds_acc_clear(acc_s);
            bh_k = wide ? NONE : th0; bs_k = wide ? NONE : ts0;
            __syncthreads();
        }
        const uint32_t base = tl.y * FILL_TILE + (uint32_t)FG * threadIdx.x;
        const uint32_t a = max(base, lo), b = min(base + (uint32_t)FG, hi);
        if (a >= b) continue;
        const bool full = a == base && b == base + (uint32_t)FG;
        FillGrp g;
        int32_t wt[FG];
        if (full) {
            load16(g.f, io.flags + base, FG); load16(g.c, io.cnt + base, FG * 4); load16(g.t, io.ts + base, FG * 8);
            if (rl || prm) load16(wt, io.v_wait + base, FG * 4);
        } else {
#pragma unroll
            for (int k = 0; k < FG; k++) {
                const uint32_t j = base + (uint32_t)k;
                const bool in = j >= a && j < b;
                g.f[k] = in ? io.flags[j] : (uint8_t)0;
                g.c[k] = in ? io.cnt[j] : 0;
                g.t[k] = in ? io.ts[j] : 0;
                wt[k] = (in && (rl || prm)) ? io.v_wait[j] : 0;
            }
        }
        const unsigned long long pw = hc.passbits[base >> 6];
        uint32_t sysm = 0;                                 // entries blocked before the controllers (EVF_SYSBLK)
#pragma unroll
        for (int k = 0; k < FG; k++)
            if ((g.f[k] & (SF_EV_EXIT | EVF_SYSBLK)) == EVF_SYSBLK) sysm |= 1u << k;
        const uint32_t bits = (all ? 0xffffu : (uint32_t)(pw >> (base & 63)) & ((1u << FG) - 1u)) & ~sysm;
        // exits: their entries' bits and times (gathers, all issued together)
        uint32_t exm = 0;
#pragma unroll
        for (int k = 0; k < FG; k++)
            if (base + (uint32_t)k >= a && base + (uint32_t)k < b && (g.f[k] & SF_EV_EXIT)) exm |= 1u << k;
        int64_t rf[FG], rts[FG]; uint32_t rlive = 0;
        if (exm) {
            if (io.eref) {
                if (full) load16(rf, io.eref + base, FG * 8);
                else {
#pragma unroll
                    for (int k = 0; k < FG; k++) rf[k] = ((exm >> k) & 1u) ? io.eref[base + k] : -1;
                }
            } else {
#pragma unroll
                for (int k = 0; k < FG; k++) rf[k] = -1;
            }
            unsigned long long rw[FG]; uint8_t rfl[FG];
#pragma unroll
            for (int k = 0; k < FG; k++) {
                const int64_t r = ((exm >> k) & 1u) ? rf[k] : -1;
                const uint32_t rc = r >= 0 && r < (int64_t)io.n ? (uint32_t)r : base;
                rw[k] = hc.passbits[rc >> 6];
                rts[k] = r >= 0 ? io.ts[rc] : (io.cts ? io.cts[base + k] : g.t[k]);
                rfl[k] = io.flags[rc];
            }
#pragma unroll
            for (int k = 0; k < FG; k++) {
                if (!((exm >> k) & 1u)) continue;
                const int64_t r = rf[k];
                const uint32_t j = base + (uint32_t)k;
                if (r >= 0 && (r < (int64_t)lo || r >= (int64_t)j || !is_entry(rfl[k]))) *st.err = SF_ERR_INVALID;
                const bool live = r == -1 || (r >= (int64_t)lo && r < (int64_t)j && !(rfl[k] & EVF_SYSBLK) &&
                                            (all || ((rw[k] >> ((uint32_t)r & 63)) & 1ull)));
                if (live) rlive |= 1u << k;
            }
        }
        // verdicts and the group's contribution
        uint8_t vs[FG]; int32_t vw[FG]; uint16_t vr[FG];
        PAcc gp; gp.clear();
#pragma unroll
        for (int k = 0; k < FG; k++) {
            const uint32_t j = base + (uint32_t)k;
            vr[k] = 0; vw[k] = 0; vs[k] = 0;
            if (j < a || j >= b) continue;
            EvContrib e{};
            e.c = g.c[k];
            if (!(g.f[k] & SF_EV_EXIT)) {
                e.passed = (bits >> k) & 1u;
                e.wait = ((rl || prm) && e.passed) ? wt[k] : 0;
                if ((sysm >> k) & 1u) { e.status = sysblk_status(g.f[k]); vr[k] = (uint16_t)sysblk_rule(g.f[k]); }
                else {
                    e.status = e.passed ? (e.wait > 0 ? SF_V_PASS_WAIT : SF_V_PASS) : (prm ? SF_V_BLOCK_PARAM : SF_V_BLOCK_FLOW);
                    if (prm && !e.passed) vr[k] = io.v_rule[j];
                }
                e.touch = true;
            } else {
                e.live_exit = (rlive >> k) & 1u;
                e.status = e.live_exit ? SF_V_EXIT : SF_V_EXIT_IGNORED;
                e.touch = e.live_exit;
                e.rt = g.t[k] - rts[k];
                e.err = (g.f[k] & SF_EV_ERROR) != 0;
            }
            vs[k] = e.status; vw[k] = e.wait;
            if (e.touch) gp.add(e);
        }
        // statuses in sorted order (launch_scatter moves them); the few nonzero
        // waits and rule indices straight to the caller's arrays
        if (full) store16(io.v_status + base, vs, FG);     // (aligned like the flags loaded above)
        else {
#pragma unroll
            for (int k = 0; k < FG; k++)
                if (base + (uint32_t)k >= a && base + (uint32_t)k < b) io.v_status[base + k] = vs[k];
        }
        bool sparse = false;
#pragma unroll
        for (int k = 0; k < FG; k++) sparse |= (io.o_wait && vw[k]) || (io.o_rule && vr[k]);
        if (sparse) {
#pragma unroll
            for (int k = 0; k < FG; k++) {
                const uint32_t j = base + (uint32_t)k;
                if (j < a || j >= b || !((io.o_wait && vw[k]) || (io.o_rule && vr[k]))) continue;
                const uint32_t pi = io.perm[j];
                if (io.o_wait && vw[k]) io.o_wait[pi] = vw[k];       // (cleared before the decide phase)
                if (io.o_rule && vr[k]) io.o_rule[pi] = vr[k];
            }
        }
#ifdef SF_EXP_NOACC
        continue;
#endif
        if (!gp.n_touch) continue;
        // window rows of the group's first and last event (time-sorted): usually one
        int64_t tfirst = 0, tlast = 0;                    // unrolled selects (no dynamic register indexing)
#pragma unroll
        for (int k = 0; k < FG; k++) {
            if (base + (uint32_t)k == a) tfirst = g.t[k];
            if (base + (uint32_t)k + 1 == b) tlast = g.t[k];
        }
        uint32_t h0, s0, h1, s1;
        key_of(tfirst, h0, s0);
        key_of(tlast, h1, s1);
        if (h0 == h1 && s0 == s1) {
            if (bh_k != NONE) { lds_acc_add(acc_h, h0 - bh_k, gp); lds_acc_add(acc_s, s0 - bs_k, gp); }
            else { gp.flush(hc.acc_hw, h0); gp.flush(hc.acc_sec, s0); }
        } else {
            PAcc ph, ps; ph.clear(); ps.clear();
            uint32_t kh = NONE, ks = NONE;
            auto out = [&](PAcc& p, uint32_t key, bool sec) {
                if (key == NONE) return;
                if (bh_k != NONE) lds_acc_add(sec ? acc_s : acc_h, key - (sec ? bs_k : bh_k), p);
                else p.flush(sec ? hc.acc_sec : hc.acc_hw, key);
            };
#pragma unroll
            for (int k = 0; k < FG; k++) {
                const uint32_t j = base + (uint32_t)k;
                if (j < a || j >= b) continue;
                EvContrib e{};
                e.c = g.c[k];
                if (!(g.f[k] & SF_EV_EXIT)) { e.passed = (bits >> k) & 1u; e.touch = true; }
                else {
                    e.live_exit = (rlive >> k) & 1u; e.touch = e.live_exit;
                    e.rt = g.t[k] - rts[k]; e.err = (g.f[k] & SF_EV_ERROR) != 0;
                }
                if (!e.touch) continue;
                uint32_t kh_, ks_;
                key_of(g.t[k], kh_, ks_);
                if (kh_ != kh) { out(ph, kh, false); ph.clear(); kh = kh_; }
                if (ks_ != ks) { out(ps, ks, true); ps.clear(); ks = ks_; }
                ph.add(e); ps.add(e);
            }
            out(ph, kh, false); out(ps, ks, true);
        }
    }
    __syncthreads();
    if (bh_k != NONE) { lds_acc_flush(acc_h, hc.acc_hw, bh_k); lds_acc_flush(acc_s, hc.acc_sec, bs_k); }
}

__global__ void k_heavy_apply(DevState st, HeavyCtx hc, StreamCtx sc, const uint32_t* seg_nhw,
                              const uint32_t* seg_nsec, int cls) {
    uint32_t s;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;; t += gridDim.x * blockDim.x) {
        if (cls == 0) { if (!heavy_at(hc, t, &s)) return; }
        else if (!stream_at(sc, t, &s)) return;
        if (hc.seg_mode[s] >= SM_QPS) heavy_apply(st, hc, s, hc.seg_res[s], seg_nhw[s], seg_nsec[s]);
    }
}

// occupancy and longest probe distance of the exact param table (diagnostics)
__global__ void k_param_stats(DevState st, unsigned long long* out) {
    unsigned long long used = 0, maxp = 0;
    const uint64_t cap = st.pcap_mask + 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
        const ParamSlot& s = st.ptab[i];
        if (s.hi == 0) continue;
        used++;
        const uint64_t home = ParamTable::hash(s.hi, s.lo) & st.pcap_mask;
        const unsigned long long d = (i - home) & st.pcap_mask;
        if (d > maxp) maxp = d;
    }
    for (int o = 32; o > 0; o >>= 1) {
        used += __shfl_xor(used, o);
        const unsigned long long m = __shfl_xor(maxp, o);
        maxp = m > maxp ? m : maxp;
    }
    if ((threadIdx.x & 63) == 0) { atomicAdd(&out[0], used); atomicMax(&out[1], maxp); }
}
hipError_t launch_param_stats(const DevState& st, unsigned long long* out, hipStream_t s) {
    hipMemsetAsync(out, 0, 16, s);
    hipLaunchKernelGGL(k_param_stats, dim3(2048), dim3(256), 0, s, st, out);
    return hipGetLastError();
}

// ParameterMetric.getThreadCount(index, value) (ParameterMetric.java:241-253) of one
// (local resource, param index, typed value): 0 when the value has no counter
__global__ void k_param_thread_read(DevState st, uint32_t l, int idx, uint32_t tag, uint64_t bits, long long* out) {
    if (threadIdx.x != 0) return;
    const ParamTable pt{st.ptab, st.pcap_mask, st.err, nullptr};
    *out = (long long)pm_thread_get(pt, l, idx, tag, bits);
}
hipError_t launch_param_thread_read(const DevState& st, uint32_t l, int idx, uint32_t tag, uint64_t bits,
                                    long long* out, hipStream_t s) {
    hipLaunchKernelGGL(k_param_thread_read, dim3(1), dim3(64), 0, s, st, l, idx, tag, bits, out);
    return hipGetLastError();
}

// sf_node_digests: one FNV-1a digest per resource row over its canonical
// sf_node_state words (absent buckets: SF_WS_ABSENT and zeros), in the word
// order of include/sentinel_flow.h.  A verification read, not a hot path: one
// thread per row walks the row's ~4 KB.
__device__ __forceinline__ uint64_t fnv_w(uint64_t h, int64_t w) { h ^= (uint64_t)w; return h * 0x100000001b3ull; }
__device__ __forceinline__ uint64_t fnv_bucket(uint64_t h, const Bucket& b) {
    if (b.ws == WS_NONE) {
        h = fnv_w(h, SF_WS_ABSENT);
        for (int k = 0; k < 7; k++) h = fnv_w(h, 0);
        return h;
    }
    h = fnv_w(h, b.ws); h = fnv_w(h, b.pass); h = fnv_w(h, b.block); h = fnv_w(h, b.exc);
    h = fnv_w(h, b.succ); h = fnv_w(h, b.rt); h = fnv_w(h, b.occ); return fnv_w(h, b.min_rt);
}
__global__ void k_node_digests(DevState st, uint32_t n, unsigned long long* out) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    const NodeRows r = cluster_rows(st, l);
    uint64_t h = 0xcbf29ce484222325ull;
    for (int i = 0; i < st.S; i++) {
        h = fnv_bucket(h, r.sec[i]);
        const Borrow b = r.bor[i];
        h = fnv_w(h, b.ws == WS_NONE ? SF_WS_ABSENT : b.ws);
        h = fnv_w(h, b.ws == WS_NONE ? 0 : b.pass);
    }
    for (int i = 0; i < MINUTE; i++) h = fnv_bucket(h, r.min[i]);
    out[l] = fnv_w(h, *r.thr);
}
hipError_t launch_node_digests(const DevState& st, uint32_t n, unsigned long long* out, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_node_digests, dim3((n + 255) / 256), dim3(256), 0, s, st, n, out);
    return hipGetLastError();
}

static inline unsigned blocks(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// Several buffer fills in one launch (each hipMemsetAsync is a launch of its
// own: the SystemRule planner's small sub-batches paid more for the launch gaps
// than for the bytes).  Range blockIdx.y: a byte head up to 16-B alignment,
// 16-B stores, a byte tail.
struct FillSet {
    static constexpr int MAX = 8;
    uint8_t* p[MAX]; size_t n[MAX]; uint32_t v[MAX];   // v: the byte repeated
    int k = 0;
    void add(void* ptr, size_t bytes, uint8_t byte) {
        if (!ptr || !bytes) return;
        p[k] = (uint8_t*)ptr; n[k] = bytes; v[k] = 0x01010101u * byte; k++;
    }
};
__global__ void k_fill(FillSet f) {
    const int r = blockIdx.y;
    uint8_t* p = f.p[r];
    const size_t n = f.n[r];
    const uint32_t v = f.v[r];
    size_t head = (16 - ((uintptr_t)p & 15)) & 15;
    if (head > n) head = n;
    const size_t body = (n - head) / 16, tail0 = head + body * 16;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    if (t < head) p[t] = (uint8_t)v;
    if (t < n - tail0) p[tail0 + t] = (uint8_t)v;
    uint4* q = (uint4*)(p + head);
    const uint4 w = make_uint4(v, v, v, v);
    for (size_t i = t; i < body; i += stride) q[i] = w;
}
static void launch_fill(const FillSet& f, hipStream_t s) {
    if (!f.k) return;
    size_t most = 0;
    for (int r = 0; r < f.k; r++) most = std::max(most, f.n[r] / 16 + 16);
    hipLaunchKernelGGL(k_fill, dim3((unsigned)std::min<size_t>(2048, (most + 255) / 256), (unsigned)f.k), dim3(256), 0, s, f);
}

using PcIter = rocprim::transform_iterator<rocprim::counting_iterator<uint32_t>, EntryCount, int64_t>;
using HeadIter = rocprim::transform_iterator<rocprim::counting_iterator<uint32_t>, HeadFlag, uint32_t>;
// rocprim has no tuned scan configs for gfx950 (its default is 256 threads x
// 16 / 8 items); tools/micro/scanbench.hip at 2^27 elements: u32 heads 0.516
// (default) -> 0.480 ms (256 x 21, warp scan), int64 counts 0.922 -> 0.822 ms
// (256 x 12, warp scan)
#ifndef SF_HEAD_SCAN_CFG
#define SF_HEAD_SCAN_CFG rocprim::scan_config<256, 21, rocprim::block_load_method::block_load_transpose, \
    rocprim::block_store_method::block_store_transpose, rocprim::block_scan_algorithm::using_warp_scan>
#endif
#ifndef SF_PC_SCAN_CFG
#define SF_PC_SCAN_CFG rocprim::scan_config<256, 12, rocprim::block_load_method::block_load_transpose, \
    rocprim::block_store_method::block_store_transpose, rocprim::block_scan_algorithm::using_warp_scan>
#endif
using HeadScanCfg = SF_HEAD_SCAN_CFG;
using PcScanCfg = SF_PC_SCAN_CFG;

hipError_t query_temp_bytes(uint32_t max_n, uint32_t key_bits, size_t* sort_bytes, size_t* scan_bytes,
                            size_t* pscan_bytes) {
    hipError_t e = rocprim::radix_sort_pairs(nullptr, *sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, max_n, 0u, key_bits);
    if (e != hipSuccess) return e;
    size_t packed_bytes = 0;
    e = rocprim::radix_sort_pairs(nullptr, packed_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (PackedEv*)nullptr, (PackedEv*)nullptr, max_n, 0u, key_bits);
    if (e != hipSuccess) return e;
    if (packed_bytes > *sort_bytes) *sort_bytes = packed_bytes;
    e = rocprim::radix_sort_pairs(nullptr, packed_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (PackedEvO*)nullptr, (PackedEvO*)nullptr, max_n, 0u, key_bits);
    if (e != hipSuccess) return e;
    if (packed_bytes > *sort_bytes) *sort_bytes = packed_bytes;
    if (rs_scratch_bytes() > *sort_bytes) *sort_bytes = rs_scratch_bytes();
    HeadIter hit(rocprim::counting_iterator<uint32_t>(0), HeadFlag{nullptr});
    e = rocprim::inclusive_scan<HeadScanCfg>(nullptr, *scan_bytes, hit, (uint32_t*)nullptr, (size_t)max_n,
                                rocprim::plus<uint32_t>());
    if (e != hipSuccess) return e;
    PcIter it(rocprim::counting_iterator<uint32_t>(0), EntryCount{nullptr, nullptr});
    return rocprim::inclusive_scan<PcScanCfg>(nullptr, *pscan_bytes, it, (int64_t*)nullptr, (size_t)max_n,
                                   rocprim::plus<int64_t>());
}

hipError_t rocprim_scan_bytes(uint32_t n, size_t* bytes) {
    return rocprim::exclusive_scan(nullptr, *bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n,
                                   rocprim::plus<uint32_t>());
}

__global__ void k_rdesc(DevState st, RDesc* out) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < st.R) out[r] = make_rdesc(st, r);
}
// after any change of rule_off / rules / prule_off / dg_rr_of
hipError_t launch_rdesc(const DevState& st, hipStream_t s) {
    hipLaunchKernelGGL(k_rdesc, dim3(blocks(st.R, 256)), dim3(256), 0, s, st, (RDesc*)st.rdesc);
    return hipGetLastError();
}

hipError_t launch_init_state(const DevState& st, hipStream_t s) {
    size_t n_sec = (size_t)st.R * st.S, n_min = (size_t)st.R * MINUTE;
    hipLaunchKernelGGL(k_init_state, dim3(2048), dim3(256), 0, s, st, n_sec, n_min);
    return hipGetLastError();
}

// Sort phase of a batch (state-independent): keys, radix sort, segments,
// sorted SoA, exit map, acquireCount prefix, classification and fill tiles.
// Runs on its own stream into one of the engine's two Work sets, so the next
// batch is sorted while the current one is decided.
// segment routing (k_classify) and the heavy fill tiles: the end of the sort
// phase when the origin index passes follow (they read the routes), else the
// head of the decide phase (the sort phase is the longer of the two)
static void launch_classify(const DevState& st, Work& w, const DevBatch& b, hipStream_t s, hipEvent_t* ev, bool timing) {
    const uint32_t n = b.n;
    FillSet f;
    f.add(w.counters, 16 * sizeof(uint32_t), 0);
    f.add(w.lcounts, 2 * LCLS * sizeof(uint32_t), 0);
    f.add(w.passbits, ((size_t)n / 64 + 2) * 8, 0);
    if (st.n_stream_rules) f.add(w.lxfar, ((size_t)n / 64 + 2) * 8, 0);
    launch_fill(f, s);
    const uint32_t max_seg = n < st.R ? n : st.R;
    if (timing) hipEventRecord(ev[10], s);
    hipLaunchKernelGGL(k_classify, dim3(blocks(max_seg, 1024)), dim3(1024), 0, s, st, w, w.s_ts);
    HeavyCtx hc = heavy_ctx(w);
    StreamCtx sc{w.stream_list, w.counters + 5, w.seg_cap, nullptr, w.counters + 7};
    hipLaunchKernelGGL(k_fill_tiles, dim3(2), dim3(1024), 0, s, hc, sc, w.fill_tiles, w.fill_tile_cap, w.fill_ntiles);
    if (timing) hipEventRecord(ev[2], s);
}

static bool sort_uses_rocprim() {
    static const bool v = [] { const char* x = getenv("SF_SORT_ROCPRIM"); return x && x[0] == '1'; }();
    return v;
}
// k_segs_red / _tscan / _out or, SF_SEGS_LB=0, the rocprim head scan + k_segs + the rocprim acquireCount scan (A/B)
static bool segs_one_pass() {
    static const bool v = [] { const char* x = getenv("SF_SEGS_LB"); return !(x && x[0] == '0'); }();
    return v && !sort_uses_rocprim();
}

hipError_t launch_sort(const DevState& st, Work& w, const DevBatch& b, uint32_t shard_count, uint32_t shard_index,
                       uint32_t key_bits, hipStream_t s, hipEvent_t* ev, bool timing, bool classify) {
    const uint32_t n = b.n;
    if (n == 0) return hipSuccess;
    const unsigned T = 256;
    if (timing) hipEventRecord(ev[0], s);
    hipError_t e;
    const bool org = b.origin != nullptr;                       // the origin rides in a 12-B payload
    // the hand-written chunked LSD sort (sf_rsort.h); SF_SORT_ROCPRIM=1: k_keys_packed + rocprim onesweep (A/B)
    const bool use_rocprim = sort_uses_rocprim();
    if (!use_rocprim) {
        // middle passes in (keys_in, pv_in) and (head_scan, pv_out); the last pass writes keys_out and the sorted SoA
        const RsBatchSrc src{b, shard_count, shard_index, st.R, st.err, st.last_ts, st.xmap};
        if (org) {
            const RsSinkFinal<PackedEvO> fin{b, w.keys_out, w.perm, w.s_ts, w.s_cnt, w.s_flags, w.s_origin,
                                             w.s_nargs, w.s_atag, w.s_abits};
            e = rs_sort(src, n, key_bits, w.keys_in, (PackedEvO*)w.pv_in, w.head_scan, (PackedEvO*)w.pv_out, fin,
                        w.sort_tmp, s);
        } else {
            const RsSinkFinal<PackedEv> fin{b, w.keys_out, w.perm, w.s_ts, w.s_cnt, w.s_flags, nullptr,
                                            w.s_nargs, w.s_atag, w.s_abits};
            e = rs_sort(src, n, key_bits, w.keys_in, w.pv_in, w.head_scan, w.pv_out, fin, w.sort_tmp, s);
        }
    } else if (org) {
        hipLaunchKernelGGL(k_keys_packed<true>, dim3(blocks(n, T)), dim3(T), 0, s, b, w.keys_in, (void*)w.pv_in,
                           shard_count, shard_index, st.R, st.err, st.last_ts, st.xmap);
        e = rocprim::radix_sort_pairs(w.sort_tmp, w.sort_tmp_bytes, w.keys_in, w.keys_out, (PackedEvO*)w.pv_in,
                                      (PackedEvO*)w.pv_out, n, 0u, key_bits, s);
    } else {
        hipLaunchKernelGGL(k_keys_packed<false>, dim3(blocks(n, T)), dim3(T), 0, s, b, w.keys_in, (void*)w.pv_in,
                           shard_count, shard_index, st.R, st.err, st.last_ts, st.xmap);
        e = rocprim::radix_sort_pairs(w.sort_tmp, w.sort_tmp_bytes, w.keys_in, w.keys_out, w.pv_in, w.pv_out, n, 0u,
                                      key_bits, s);
    }
    if (e != hipSuccess) return e;
    if (!segs_one_pass()) {
        HeadIter hit(rocprim::counting_iterator<uint32_t>(0), HeadFlag{w.keys_out});
        e = rocprim::inclusive_scan<HeadScanCfg>(w.scan_tmp, w.scan_tmp_bytes, hit, w.head_scan, (size_t)n,
                                    rocprim::plus<uint32_t>(), s);
        if (e != hipSuccess) return e;
    }
    hipMemsetAsync(w.segflag, 0, (size_t)(n < st.R ? n : st.R) * 4, s);
    if (timing) hipEventRecord(ev[1], s);
    if (!use_rocprim && !segs_one_pass()) {
        hipLaunchKernelGGL(k_segs, dim3(blocks(n, T)), dim3(T), 0, s, b, w.s_cnt, w.s_flags, w.s_atag, w.keys_out,
                           w.head_scan, w.seg_start, w.seg_res, w.n_seg, w.segflag, st.last_ts, st.err,
                           st.n_prule != 0, st.prio_seen);
    } else if (!use_rocprim) {
        // segment table, head scan and (window rules loaded) the acquireCount prefix: reduce, scan, rescan
        if (st.n_window_rules) launch_segs3<true>(st, w, b, s);
        else launch_segs3<false>(st, w, b, s);
    } else if (org)
        hipLaunchKernelGGL(k_unpack<true>, dim3(blocks(n, T)), dim3(T), 0, s, b, (const void*)w.pv_out, w.keys_out,
                           w.perm, w.s_ts, w.s_cnt, w.s_flags, w.s_nargs, w.s_atag, w.s_abits, w.head_scan,
                           w.seg_start, w.seg_res, w.n_seg, w.segflag, st.last_ts, st.err, st.n_prule != 0, w.s_origin,
                           st.prio_seen);
    else
        hipLaunchKernelGGL(k_unpack<false>, dim3(blocks(n, T)), dim3(T), 0, s, b, (const void*)w.pv_out, w.keys_out,
                           w.perm, w.s_ts, w.s_cnt, w.s_flags, w.s_nargs, w.s_atag, w.s_abits, w.head_scan,
                           w.seg_start, w.seg_res, w.n_seg, w.segflag, st.last_ts, st.err, st.n_prule != 0,
                           (uint32_t*)nullptr, st.prio_seen);
    if (classify) launch_classify(st, w, b, s, ev, timing);
    return hipGetLastError();
}

// ============================================================ verdict scatter
// Every deciding kernel leaves its statuses in sorted order (v_status); the
// caller's array is in submission order, a permutation away (perm).  One byte
// stored per event at a random address costs a partial-line write each (the
// lean QPS walk of config 2 spent half its time on them), so the statuses
// travel instead in bucketed passes whose every global store is part of a
// run: A buckets by submission index >> s1 (<= 256 buckets of 2^s1), B by
// index >> VS_REG inside an A bucket, C assembles each 2^VS_REG region in LDS
// and stores it with coalesced writes.  A record is (status << 24) | (the
// index bits below its bucket).  A permutation fills every bucket exactly, so
// bucket sizes are known and no histogram pass is needed: each workgroup
// counting-sorts its tile in LDS, claims a run per bucket with one global
// atomic, and writes the run.
#ifndef SF_VS_T
#define SF_VS_T 1024                 // 16 waves per workgroup: 256 x 32 ran the scatter 4.4 -> 2.3 ms slower
#define SF_VS_PER 8
#endif
constexpr uint32_t VS_T = SF_VS_T, VS_PER = SF_VS_PER, VS_TILE = VS_T * VS_PER;
// k_vs_bucket's LDS: hist / lbase / gbase (3 x 4 KiB), part, buf (4 B per record)
// and kb (2 B per record); a record's rank in its bucket is packed in 16 bits
static_assert(VS_TILE < 65536u, "k_vs_bucket packs a record's rank into 16 bits");
static_assert(3u * 1024u * 4u + VS_T * 4u + VS_TILE * 4u + VS_TILE * 2u <= 65536u,
              "k_vs_bucket LDS footprint over 64 KiB: retune SF_VS_T / SF_VS_PER");
constexpr uint32_t VS_DIRECT_MAX = 1u << 20;        // smaller batches: one direct scatter

// A (FIRST: sorted positions [blockIdx * VS_TILE, +VS_TILE) -> bucket idx >> s1)
// or B (records of A bucket blockIdx / tpb, tile blockIdx % tpb -> region idx >> VS_REG)
template <bool FIRST>
__global__ void __launch_bounds__(VS_T) k_vs_bucket(const uint32_t* perm, const uint8_t* v_status, const uint32_t* in,
                                                     uint32_t* out, uint32_t* cursor, uint32_t n, uint32_t s1,
                                                     uint32_t tpb, int32_t* err) {
    __shared__ uint32_t hist[1024], lbase[1024], gbase[1024], part[VS_T];
    __shared__ uint32_t buf[VS_TILE];
    __shared__ uint16_t kb[VS_TILE];
    const uint32_t tid = threadIdx.x;
    const uint32_t m1 = s1 >= 32 ? 0xffffffffu : (1u << s1) - 1u;
    uint32_t lo, hi, nk, bb = 0;
    if (FIRST) {
        lo = blockIdx.x * VS_TILE;
        hi = min(n, lo + VS_TILE);
        nk = (uint32_t)(((uint64_t)n + m1) >> s1);
    } else {
        bb = blockIdx.x / tpb;
        const uint64_t b0 = (uint64_t)bb << s1;
        const uint64_t bend = min((uint64_t)n, b0 + (1ull << s1));
        const uint64_t l = b0 + (uint64_t)(blockIdx.x % tpb) * VS_TILE;
        if (l >= bend) return;                           // (whole workgroup)
        lo = (uint32_t)l; hi = (uint32_t)min(bend, l + VS_TILE);
        nk = 1u << (s1 - VS_REG);
    }
    for (uint32_t k = tid; k < nk; k += VS_T) hist[k] = 0;
    __syncthreads();
    uint32_t rec[VS_PER], kr[VS_PER];                    // record, key << 16 | rank in the tile's bucket
#pragma unroll
    for (uint32_t r = 0; r < VS_PER; r++) {
        const uint32_t e = lo + r * VS_T + tid;
        kr[r] = 0xffffffffu;
        if (e < hi) {
            uint32_t key;
            if (FIRST) {
                const uint32_t i = perm[e];
                key = i >> s1; rec[r] = ((uint32_t)v_status[e] << 24) | (i & m1);
            } else {
                const uint32_t v = in[e];
                key = (v & m1) >> VS_REG; rec[r] = (v & 0xff000000u) | (v & ((1u << VS_REG) - 1u));
            }
            kr[r] = (key << 16) | atomicAdd(&hist[key], 1u);
        }
    }
    __syncthreads();
    // exclusive scan of the bucket counts (ceil(nk / VS_T) per thread), then one claim per bucket
    const uint32_t per = (nk + VS_T - 1) / VS_T;
    uint32_t sum = 0;
    for (uint32_t q = 0; q < per; q++) { const uint32_t k = tid * per + q; if (k < nk) sum += hist[k]; }
    // (wavefront scans, then the wavefronts' totals: one barrier)
    const uint32_t lane = tid & 63u, wv = tid >> 6;
    uint32_t incl = sum;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63u) part[wv] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (uint32_t q = 0; q < wv; q++) run += part[q];
    for (uint32_t q = 0; q < per; q++) {
        const uint32_t k = tid * per + q;
        if (k >= nk) break;
        const uint32_t h = hist[k];
        lbase[k] = run; run += h;
        if (h) {
            const uint32_t c = FIRST ? k : 256u + bb * nk + k;
            const uint32_t g = atomicAdd(&cursor[c], h);
            // bucket capacity: what the permutation puts there (anything more is a broken permutation)
            const uint64_t first = FIRST ? ((uint64_t)k << s1) : (((uint64_t)bb * nk + k) << VS_REG);
            const uint64_t cap = min((uint64_t)(FIRST ? (1ull << s1) : (1ull << VS_REG)), (uint64_t)n - min((uint64_t)n, first));
            if ((uint64_t)g + h > cap) *err = SF_ERR_INVALID;
            gbase[k] = (uint32_t)first + g - lbase[k];       // destination of the tile's k-th record, minus k
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < VS_PER; r++)
        if (kr[r] != 0xffffffffu) {
            const uint32_t key = kr[r] >> 16, p = lbase[key] + (kr[r] & 0xffffu);
            buf[p] = rec[r]; kb[p] = (uint16_t)key;
        }
    __syncthreads();
    for (uint32_t k = tid; k < hi - lo; k += VS_T) {
        const uint32_t dst = gbase[kb[k]] + k;              // (a broken permutation: flagged above, kept in bounds)
        if (dst < n) out[dst] = buf[k];
    }
}

// C: region blockIdx (2^VS_REG submission indices) assembled in LDS, stored coalesced
__global__ void __launch_bounds__(VS_T) k_vs_region(const uint32_t* in, uint8_t* o_status, uint32_t n) {
    __shared__ __align__(16) uint8_t reg[1u << VS_REG];
    const uint32_t base = blockIdx.x << VS_REG;
    const uint32_t cnt = min(1u << VS_REG, n - base);
    for (uint32_t k = threadIdx.x; k < cnt; k += VS_T) {
        const uint32_t v = in[base + k];
        reg[v & ((1u << VS_REG) - 1u)] = (uint8_t)(v >> 24);
    }
    __syncthreads();
    uint8_t* o = o_status + base;
    if (((uintptr_t)o & 15) == 0) {
        for (uint32_t k = threadIdx.x; k < cnt / 16; k += VS_T) ((uint4*)o)[k] = ((const uint4*)reg)[k];
        for (uint32_t k = (cnt & ~15u) + threadIdx.x; k < cnt; k += VS_T) o[k] = reg[k];
    } else {
        for (uint32_t k = threadIdx.x; k < cnt; k += VS_T) o[k] = reg[k];
    }
}

__global__ void k_vs_direct(const uint32_t* perm, const uint8_t* v_status, uint8_t* o_status, uint32_t n) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) o_status[perm[j]] = v_status[j];
}

// statuses of a decided batch: sorted order -> the caller's array (submission order)
static void launch_scatter(Work& w, uint32_t n, uint8_t* o_status, hipStream_t s) {
    if (n <= VS_DIRECT_MAX) {
        hipLaunchKernelGGL(k_vs_direct, dim3(blocks(n, 256)), dim3(256), 0, s, w.perm, w.v_status, o_status, n);
        return;
    }
    const uint32_t lg = 32u - (uint32_t)__builtin_clz(n - 1u);          // ceil(log2 n)
    const uint32_t s1 = std::max(VS_REG, lg - 8u);                      // <= 256 A buckets
    const uint32_t nb1 = (uint32_t)(((uint64_t)n + (1ull << s1) - 1) >> s1);
    const uint32_t nk = 1u << (s1 - VS_REG);
    hipMemsetAsync(w.vs_cursor, 0, (256 + (size_t)nb1 * nk) * 4, s);
    // staging: the sort's key buffers (dead once the batch is unpacked)
    hipLaunchKernelGGL(k_vs_bucket<true>, dim3((n + VS_TILE - 1) / VS_TILE), dim3(VS_T), 0, s, w.perm, w.v_status,
                       nullptr, w.keys_in, w.vs_cursor, n, s1, 0u, w.err);
    const uint32_t* regions = w.keys_in;
    if (s1 > VS_REG) {
        const uint32_t tpb = (1u << s1) / VS_TILE;
        hipLaunchKernelGGL(k_vs_bucket<false>, dim3(nb1 * tpb), dim3(VS_T), 0, s, nullptr, nullptr, w.keys_in,
                           w.keys_out, w.vs_cursor, n, s1, tpb, w.err);
        regions = w.keys_out;
    }
    hipLaunchKernelGGL(k_vs_region, dim3((n + (1u << VS_REG) - 1) >> VS_REG), dim3(VS_T), 0, s, regions, o_status, n);
}

// THREAD stream records and run tables (state-independent; at the head of the
// decide phase on stream A, before k_heavy_stream reads them: the sort phase of
// the next batch is the longer of the two pipelined phases)
static void launch_thr_prep(Work& w, const DevBatch& b, hipStream_t s) {
    const uint32_t n = b.n;
    HeavyCtx hc = heavy_ctx(w);
    // (grids sized to the most tiles a batch of n events can have: small
    // SystemRule sub-batches do not pay for full-chip launches)
    const uint32_t tile_ub = n / FILL_TILE + n / (w.heavy_min + 1) + 2;
    const uint2* tiles1 = w.fill_tiles + w.fill_tile_cap;
    const int64_t* seref = b.eref ? w.s_eref : nullptr;
    const dim3 tgrid(std::min<uint32_t>(1024u, tile_ub));
    hipLaunchKernelGGL(k_thr_heads, tgrid, dim3(256), 0, s, w.s_flags, w.s_cnt, hc, tiles1, w.fill_ntiles,
                       w.tile_rc, w.segflag);
    // THREAD run mode tables (sf_stream.h thr_runs_segment)
    hipLaunchKernelGGL(k_thr_rscan, dim3(1), dim3(1024), 0, s, w.tile_rc, w.fill_ntiles);
    hipLaunchKernelGGL(k_thr_rid, tgrid, dim3(256), 0, s, w.s_flags, hc, tiles1, w.fill_ntiles, w.tile_rc);
    hipLaunchKernelGGL(k_thr_rec, tgrid, dim3(256), 0, s, w.s_flags, w.s_cnt, seref, hc, tiles1, w.fill_ntiles,
                       w.segflag);
}

// the light lanes of a batch (k_classify's lists), longest class first; the
// lean QPS walks only where a QPS DefaultController rule is loaded
// (the lean QPS walks go on stream B after its heavy kernels, beside the
// generic walks on C: different segments, different resources)
template <int MAXS, bool PF>
static void launch_light(const DevState& st, const SegIO& io, const Work& w, const LightLists& ll, uint32_t max_seg,
                         hipStream_t s3, hipStream_t s2) {
    const unsigned TD = 128;
    hipLaunchKernelGGL((k_decide_light<MAXS, PF>), dim3(blocks(max_seg, TD)), dim3(TD), 0, s3, st, io, w.seg_start,
                       w.seg_res, ll);
    if (st.n_window_rules) {
        hipLaunchKernelGGL(k_decide_light_qps<MAXS>, dim3(blocks(max_seg, TD)), dim3(TD), 0, s2, st, io, w.seg_start,
                           w.seg_res, ll);
        hipLaunchKernelGGL(k_decide_short_qps<MAXS>, dim3(blocks(max_seg, TD)), dim3(TD), 0, s2, st, io, w.seg_start,
                           w.seg_res, ll, w.counters + 8);
    }
    hipLaunchKernelGGL((k_decide_short<MAXS, PF>), dim3(blocks(max_seg, TD)), dim3(TD), 0, s3, st, io, w.seg_start,
                       w.seg_res, ll, w.counters + 8);
}

// Decide phase (stateful, batch order): the serial chains (k_heavy_stream)
// start first, on A; QPS/WarmUp heavy segments on B, the light lanes on C;
// then the verdicts are scattered back to submission order.
hipError_t launch_decide(const DevState& st, Work& w, const DevBatch& b, const DevVerdicts& out,
                         hipStream_t s, hipStream_t s2, hipStream_t s3, hipStream_t s4, hipEvent_t* ev, bool timing,
                         const OxPlan* ox, bool classify, hipStream_t sv) {
    const uint32_t n = b.n;
    if (n == 0) return hipSuccess;
    if (classify) launch_classify(st, w, b, s, ev, timing);
    SegIO io;
    io.ts = w.s_ts; io.cnt = w.s_cnt; io.flags = w.s_flags;
    io.eref = b.eref ? w.s_eref : nullptr; io.cts = b.eref ? w.s_cts : nullptr;
    io.arg_slots = b.arg_slots; io.nargs = (b.arg_slots && b.nargs) ? w.s_nargs : nullptr;
    io.atag = w.s_atag; io.abits = w.s_abits; io.n = n;
    io.aoff = b.aoff; io.etag = b.etag; io.ebits = b.ebits;
    io.v_status = w.v_status; io.v_wait = w.v_wait; io.v_rule = w.v_rule;
    io.perm = w.perm; io.o_status = out.status; io.o_wait = out.wait; io.o_rule = out.rule;
    io.ev_res = b.res; io.ev_origin = b.origin; io.ev_ctx = b.ctx; io.shard_count = st.shard_count;
    HeavyCtx hc = heavy_ctx(w);
    if (timing) hc.hticks = w.hticks;
    const uint32_t max_seg = n < st.R ? n : st.R;
    const uint32_t max_heavy = n / (w.heavy_min + 1) + 1;
    StreamCtx sc{w.stream_list, w.counters + 5, w.seg_cap, timing ? w.sticks : nullptr, w.counters + 7};
    // each exit's entry (sorted position, exit_of) and create time: state-
    // independent, but here at the head of the decide phase rather than in the
    // sort phase, the longer of the two pipelined phases (k_classify does not
    // read them; every deciding kernel does)
    {
        FillSet f;
        if (b.eref || st.n_stream_rules) f.add(w.exit_of, (size_t)n * 4, 0xff);   // (read by k_gather_exit, k_thr_rec)
        // waits and rule indices are zero for almost every event: clear them with
        // coalesced stores, then the deciding kernels scatter only the nonzero ones
        f.add(out.wait, (size_t)n * sizeof(int32_t), 0);
        f.add(out.rule, (size_t)n * sizeof(uint16_t), 0);
        launch_fill(f, s);
    }
    if (b.eref)
        hipLaunchKernelGGL(k_gather_exit, dim3(blocks(n, 256)), dim3(256), 0, s, b, w.perm, w.s_flags,
                           w.head_scan, w.seg_start, w.s_eref, w.s_cts, w.exit_of, st.err);
    hipEventRecord(ev[5], s);                      // fork
    // (the THREAD / RateLimiter class exists only with such rules loaded)
    if (st.n_stream_rules) launch_thr_prep(w, b, s);
    hipEventRecord(ev[11], s);
    if (st.n_stream_rules)
        hipLaunchKernelGGL(k_heavy_stream, dim3(std::min(max_heavy, w.stream_grid)), dim3(HS_T), 0, s, st, io, hc, sc);
    hipEventRecord(ev[12], s);
    hipStreamWaitEvent(s2, ev[5], 0);
    hipStreamWaitEvent(s3, ev[5], 0);
    // long one-resource xflow segments: the wave walk, on its own stream from
    // the fork (its segments share no node or rule with any other kernel of the
    // phase; the longest of them is usually the phase's critical path)
    const bool xw_on = st.xmap && st.xw;
    auto launch_xw = [&](hipStream_t sx) {
        const unsigned g = (unsigned)std::min<size_t>((size_t)b.n / XW_MIN + 1, 2048);
        if (st.S <= 2)
            hipLaunchKernelGGL(k_decide_xw<2>, dim3(g), dim3(64), 0, sx, st, io, w.seg_start, w.seg_res,
                               w.xw_list, w.counters + 12);
        else
            hipLaunchKernelGGL(k_decide_xw<SF_MAX_SAMPLE_COUNT>, dim3(g), dim3(64), 0, sx, st, io, w.seg_start,
                               w.seg_res, w.xw_list, w.counters + 12);
        hipEventRecord(ev[15], sx);
    };
    if (xw_on) {
        hipStreamWaitEvent(s4, ev[5], 0);
        launch_xw(s4);
    }
    if (st.n_window_rules && !segs_one_pass()) {
        // acquireCount prefix of the entries (QPS / WarmUp window budgets, k_heavy_decide
        // only; the hand-written sort path writes it in k_segs_out): state-independent, but
        // here on stream B rather than in the sort phase, the longer of the two pipelined phases
        PcIter it(rocprim::counting_iterator<uint32_t>(0), EntryCount{w.s_cnt, w.s_flags});
        const hipError_t e = rocprim::inclusive_scan<PcScanCfg>(w.pscan_tmp, w.pscan_tmp_bytes, it, w.pcg,
                                                                (size_t)n, rocprim::plus<int64_t>(), s2);
        if (e != hipSuccess) return e;
    }
    if (st.S <= 2)
        hipLaunchKernelGGL(k_heavy_decide<2>, dim3(max_heavy), dim3(64), 0, s2, st, io, hc);
    else
        hipLaunchKernelGGL(k_heavy_decide<SF_MAX_SAMPLE_COUNT>, dim3(max_heavy), dim3(64), 0, s2, st, io, hc);
    if (timing) hipEventRecord(ev[7], s2);
    // verdicts + window deltas of each heavy class as soon as its decisions are done
    const uint32_t fgrid = std::min<uint32_t>(w.fill_grid, n / FILL_TILE + max_heavy + 1);   // tiles of this batch at most
    hipLaunchKernelGGL(k_heavy_fill, dim3(fgrid), dim3(256), 0, s2, st, io, hc, w.fill_tiles, w.fill_ntiles, 0);
    if (timing) hipEventRecord(ev[8], s2);
    hipLaunchKernelGGL(k_heavy_apply, dim3(blocks(max_heavy, 64)), dim3(64), 0, s2, st, hc, sc, w.seg_nhw, w.seg_nsec, 0);
    if (st.n_stream_rules) {
        hipLaunchKernelGGL(k_heavy_fill, dim3(fgrid), dim3(256), 0, s, st, io, hc,
                           w.fill_tiles + w.fill_tile_cap, w.fill_ntiles, 1);
        hipLaunchKernelGGL(k_heavy_apply, dim3(blocks(max_heavy, 64)), dim3(64), 0, s, st, hc, sc, w.seg_nhw,
                           w.seg_nsec, 1);
    }

    LightLists ll{w.light_list, w.lcounts, {}, {}};
    for (int c = 0; c < LCLS; c++) { ll.off[c] = w.loff[c]; ll.cap[c] = w.lcap[c]; }
    // (no ParamFlow / degrade rule loaded: the lanes without that code)
    const bool pf = st.n_prule != 0 || st.dg_rr_of != nullptr;
    if (st.S <= 2) {
        if (pf) launch_light<2, true>(st, io, w, ll, max_seg, s3, s2);
        else launch_light<2, false>(st, io, w, ll, max_seg, s3, s2);
    } else {
        if (pf) launch_light<SF_MAX_SAMPLE_COUNT, true>(st, io, w, ll, max_seg, s3, s2);
        else launch_light<SF_MAX_SAMPLE_COUNT, false>(st, io, w, ll, max_seg, s3, s2);
    }
    if (st.xmap) {
        if (st.S <= 2)
            hipLaunchKernelGGL(k_decide_x<2>, dim3(blocks(max_seg, 64)), dim3(64), 0, s3, st, io, w.seg_start,
                               w.seg_res, w.seg_mode, w.n_seg);
        else
            hipLaunchKernelGGL(k_decide_x<SF_MAX_SAMPLE_COUNT>, dim3(blocks(max_seg, 64)), dim3(64), 0, s3, st, io,
                               w.seg_start, w.seg_res, w.seg_mode, w.n_seg);
    }
    hipEventRecord(ev[9], s3);                     // light done (also the join of C)
    hipEventRecord(ev[16], s2);                    // the lean QPS walks done (after B's heavy kernels)
    hipEventRecord(ev[6], s2);                     // join B and C
    hipStreamWaitEvent(s, ev[6], 0);
    hipStreamWaitEvent(s, ev[9], 0);
    hipEventRecord(ev[13], s);                     // (the origin pass below does not wait for the wave walk)
    if (xw_on) hipStreamWaitEvent(s, ev[15], 0);
    if (timing) hipEventRecord(ev[3], s);
    // origin nodes no rule reads (sf_origin.hip): from the sorted verdicts
    // of the other segments, beside the wave walk and the verdict scatter
    if (ox) {
        hipStreamWaitEvent(s2, ev[13], 0);
        const hipError_t e = launch_ox_apply(st, w, b, ox->n_heavy, ox->n_pairs, ox->win, s2);
        if (e != hipSuccess) return e;
        hipEventRecord(ev[14], s2);
    }
    // the verdict scatter on sv when given (an asynchronous batch: beside the
    // next batch's decide phase, which reads no status of this one)
    hipStream_t vs = sv ? sv : s;
    if (vs != s) {
        hipEventRecord(ev[17], s);
        hipStreamWaitEvent(vs, ev[17], 0);
    }
    launch_scatter(w, n, out.status, vs);
    if (ox) {
        hipStreamWaitEvent(s, ev[14], 0);          // the next batch reads the origin nodes
        if (vs != s) hipStreamWaitEvent(vs, ev[14], 0);
    }
    if (timing) hipEventRecord(ev[4], vs);
    return hipGetLastError();
}

// ============================================================ compact batches
// sf_packed_batch -> the SoA DevBatch arrays (res, ts, count, flags, entry_ref,
// create_ts).  EXIT events and count-0 events take the next value of the
// sparse exit_ref / exit_cts / count_ext arrays: a per-tile count, one scan of
// the tile counts, then each tile's own scan (PK_T threads x PK_PER events).
constexpr uint32_t PK_T = 256, PK_PER = 16, PK_TILE = PK_T * PK_PER;
struct PkIn { const uint64_t* ev; const int64_t* xref; const int64_t* xcts; const int32_t* cext; int64_t base;
              uint32_t n, n_exit, n_cext;
              const uint32_t* ev4; const uint32_t* ms_end; uint32_t n_ms; };   // the narrow form: ev null
struct PkOut { uint32_t* res; int64_t* ts; int32_t* cnt; uint8_t* flags; int64_t* eref; int64_t* cts; };

__device__ __forceinline__ uint32_t pk_flags(uint64_t w) { return (uint32_t)(w >> SF_PK_FLAGS_SHIFT) & 0x1fu; }
__device__ __forceinline__ uint32_t pk_count(uint64_t w) { return (uint32_t)(w >> SF_PK_COUNT_SHIFT) & 0x7fu; }
// the narrow form's word as the 8-byte one without the time (res, acquireCount, flags)
__device__ __forceinline__ uint64_t pk_widen(uint32_t w) {
    return (uint64_t)(w & 0xffffffu) | ((uint64_t)((w >> SF_PK4_COUNT_SHIFT) & 7u) << SF_PK_COUNT_SHIFT) |
           ((uint64_t)(w >> SF_PK4_FLAGS_SHIFT) << SF_PK_FLAGS_SHIFT);
}
__device__ __forceinline__ uint64_t pk_word(const PkIn& in, uint32_t i) {
    return in.ev4 ? pk_widen(in.ev4[i]) : in.ev[i];
}
// first m in [lo, hi) with ms_end[m] > i (hi when none)
__device__ __forceinline__ uint32_t pk_ms_search(const uint32_t* ms_end, uint32_t lo, uint32_t hi, uint32_t i) {
    while (lo < hi) { const uint32_t m = lo + (hi - lo) / 2; if (ms_end[m] > i) hi = m; else lo = m + 1; }
    return lo;
}
constexpr uint32_t PK_ME = 1024;   // ms_end entries of a tile staged in LDS (longer spans search HBM)

__global__ void __launch_bounds__(PK_T) k_pk_count(PkIn in, uint2* tile_cnt) {
    __shared__ uint32_t sx, sc;
    if (threadIdx.x == 0) { sx = 0; sc = 0; }
    __syncthreads();
    uint32_t x = 0, c = 0;
    const uint32_t t0 = blockIdx.x * PK_TILE;
    for (uint32_t k = 0; k < PK_PER; k++) {
        const uint32_t i = t0 + k * PK_T + threadIdx.x;
        if (i >= in.n) break;
        const uint64_t w = pk_word(in, i);
        x += (pk_flags(w) & SF_EV_EXIT) ? 1u : 0u;
        c += pk_count(w) == 0 ? 1u : 0u;
    }
    x = (uint32_t)wave_sum(x); c = (uint32_t)wave_sum(c);
    if ((threadIdx.x & 63) == 0) { atomicAdd(&sx, x); atomicAdd(&sc, c); }
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = make_uint2(sx, sc);
}

// exclusive scan of the tile counts (one workgroup); err when a sparse array is short
__global__ void __launch_bounds__(1024) k_pk_scan(uint2* tile_cnt, uint32_t nt, PkIn in, int32_t* err) {
    __shared__ uint32_t wx[16], wc[16];
    __shared__ uint32_t cx, cc;
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    if (threadIdx.x == 0) { cx = 0; cc = 0; }
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nt; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        const uint2 v = i < nt ? tile_cnt[i] : make_uint2(0u, 0u);
        const uint32_t ix = (uint32_t)wave_scan_add((int)v.x), ic = (uint32_t)wave_scan_add((int)v.y);
        if (lane == 63) { wx[wv] = ix; wc[wv] = ic; }
        __syncthreads();
        uint32_t bx = cx, bc = cc;
        for (int k = 0; k < wv; k++) { bx += wx[k]; bc += wc[k]; }
        if (i < nt) tile_cnt[i] = make_uint2(bx + ix - v.x, bc + ic - v.y);
        __syncthreads();
        if (threadIdx.x == 1023) { cx = bx + ix; cc = bc + ic; }
        __syncthreads();
    }
    if (threadIdx.x == 0 && (cx > in.n_exit || cc > in.n_cext)) *err = SF_ERR_INVALID;
    // the narrow form's time table must cover every event
    if (threadIdx.x == 0 && in.ev4 && (in.n_ms == 0 || in.ms_end[in.n_ms - 1] != in.n)) *err = SF_ERR_INVALID;
}

// coalesced: round k of a tile holds events t0 + 256 k + thread, scanned in
// that (batch) order with a carry from round to round
// The narrow form's time: event i is at ts_base + the first m with
// ms_end[m] > i; the tile's first millisecond is searched once, the next
// PK_ME entries staged in LDS.
__global__ void __launch_bounds__(PK_T) k_pk_expand(PkIn in, const uint2* tile_base, PkOut out) {
    __shared__ uint32_t wx[PK_T / 64], wc[PK_T / 64];
    __shared__ uint32_t sme[PK_ME];
    __shared__ uint32_t s_m0;
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const uint2 tb = tile_base[blockIdx.x];
    uint32_t cx = tb.x, cc = tb.y;
    uint32_t m0 = 0;
    if (in.ev4) {
        if (threadIdx.x == 0) s_m0 = pk_ms_search(in.ms_end, 0, in.n_ms, blockIdx.x * PK_TILE);
        __syncthreads();
        m0 = s_m0;
        for (uint32_t j = threadIdx.x; j < PK_ME; j += PK_T) sme[j] = m0 + j < in.n_ms ? in.ms_end[m0 + j] : 0xffffffffu;
        __syncthreads();
    }
    for (uint32_t k = 0; k < PK_PER; k++) {
        const uint32_t i = blockIdx.x * PK_TILE + k * PK_T + threadIdx.x;
        const bool in_b = i < in.n;
        const uint64_t w = in_b ? pk_word(in, i) : 0ull;
        const uint32_t f = pk_flags(w), c8 = pk_count(w);
        const uint32_t x = (in_b && (f & SF_EV_EXIT)) ? 1u : 0u, c = (in_b && c8 == 0) ? 1u : 0u;
        const uint32_t ix = (uint32_t)wave_scan_add((int)x), ic = (uint32_t)wave_scan_add((int)c);
        if (lane == 63) { wx[wv] = ix; wc[wv] = ic; }
        __syncthreads();
        uint32_t bx = cx + ix - x, bc = cc + ic - c, tx = 0, tc = 0;
        for (int q = 0; q < PK_T / 64; q++) {
            if (q < wv) { bx += wx[q]; bc += wc[q]; }
            tx += wx[q]; tc += wc[q];
        }
        __syncthreads();
        cx += tx; cc += tc;
        if (!in_b) continue;
        out.res[i] = (uint32_t)w;
        if (in.ev4) {
            uint32_t m;
            if (sme[PK_ME - 1] > i) {
                uint32_t lo = 0, hi = PK_ME;
                while (lo < hi) { const uint32_t md = (lo + hi) / 2; if (sme[md] > i) hi = md; else lo = md + 1; }
                m = m0 + lo;
            } else {
                m = pk_ms_search(in.ms_end, m0 + PK_ME, in.n_ms, i);
            }
            out.ts[i] = in.base + (int64_t)m;
        } else {
            out.ts[i] = in.base + (int64_t)((w >> 32) & 0xfffffu);
        }
        out.flags[i] = (uint8_t)f;
        out.cnt[i] = c8 ? (int32_t)c8 : (bc < in.n_cext ? in.cext[bc] : 0);
        if (f & SF_EV_EXIT) {
            out.eref[i] = bx < in.n_exit ? in.xref[bx] : -1;
            if (out.cts) out.cts[i] = (in.xcts && bx < in.n_exit) ? in.xcts[bx] : 0;
        } else {
            out.eref[i] = -1;
            if (out.cts) out.cts[i] = 0;
        }
    }
}

// Sparse copy back of a packed batch's verdicts (sf_sparse_verdicts): the
// nonzero waits and rule indices as (index << 32 | value), any order.
// counts[0], counts[1]: lengths.  One workgroup per SV_TILE events and one
// atomic per workgroup and list: a counter bumped once per wavefront (2M
// atomics on one address per 2^27 events) serialised the kernel to 13-17 ms
// beside the next batch (profiles/r06_e2e_trace.txt).  Each thread keeps its
// SV_PT values in registers between the count and the write.
constexpr int SV_T = 256, SV_PT = 16;
constexpr uint32_t SV_TILE = SV_T * SV_PT;
__global__ void __launch_bounds__(SV_T) k_sparse_verdicts(const int32_t* wait, const uint16_t* rule, uint32_t n,
                                                          unsigned long long* wl, unsigned long long* rl,
                                                          uint32_t* counts) {
    __shared__ uint32_t wsum[2][SV_T / 64];
    __shared__ uint32_t base[2];
    const uint32_t t0 = blockIdx.x * SV_TILE;
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    int32_t w[SV_PT];
    uint16_t r[SV_PT];
    uint32_t cw = 0, cr = 0;
#pragma unroll
    for (int k = 0; k < SV_PT; k++) {
        const uint32_t i = t0 + (uint32_t)k * SV_T + threadIdx.x;
        w[k] = i < n ? wait[i] : 0;
        r[k] = i < n ? rule[i] : (uint16_t)0;
        cw += w[k] != 0;
        cr += r[k] != 0;
    }
    const uint32_t sw = (uint32_t)wave_scan_add((int)cw), sr = (uint32_t)wave_scan_add((int)cr);
    if (lane == 63) { wsum[0][wave] = sw; wsum[1][wave] = sr; }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint32_t tot = 0;
        for (int k = 0; k < SV_T / 64; k++) tot += wsum[threadIdx.x][k];
        base[threadIdx.x] = tot ? atomicAdd(&counts[threadIdx.x], tot) : 0u;
    }
    __syncthreads();
    uint32_t ow = base[0] + sw - cw, orr = base[1] + sr - cr;
    for (int k = 0; k < wave; k++) { ow += wsum[0][k]; orr += wsum[1][k]; }
#pragma unroll
    for (int k = 0; k < SV_PT; k++) {
        const unsigned long long i = t0 + (uint32_t)k * SV_T + threadIdx.x;
        if (w[k] != 0) wl[ow++] = (i << 32) | (uint32_t)w[k];
        if (r[k] != 0) rl[orr++] = (i << 32) | r[k];
    }
}
hipError_t launch_sparse_verdicts(const int32_t* wait, const uint16_t* rule, uint32_t n, unsigned long long* wl,
                                  unsigned long long* rl, uint32_t* counts, hipStream_t s) {
    hipMemsetAsync(counts, 0, 8, s);
    if (n) hipLaunchKernelGGL(k_sparse_verdicts, dim3((n + SV_TILE - 1) / SV_TILE), dim3(SV_T), 0, s, wait, rule, n,
                              wl, rl, counts);
    return hipGetLastError();
}

hipError_t launch_pk_expand(const uint64_t* ev, const uint32_t* ev4, const uint32_t* ms_end, uint32_t n_ms,
                            const int64_t* xref, const int64_t* xcts, const int32_t* cext,
                            int64_t base, uint32_t n, uint32_t n_exit, uint32_t n_cext, uint2* tile_cnt,
                            uint32_t* res, int64_t* ts, int32_t* cnt, uint8_t* flags, int64_t* eref, int64_t* cts,
                            int32_t* err, hipStream_t s) {
    if (!n) return hipSuccess;
    const PkIn in{ev, xref, xcts, cext, base, n, n_exit, n_cext, ev ? nullptr : ev4, ms_end, n_ms};
    const PkOut out{res, ts, cnt, flags, eref, cts};
    const uint32_t nt = (n + PK_TILE - 1) / PK_TILE;
    hipLaunchKernelGGL(k_pk_count, dim3(nt), dim3(PK_T), 0, s, in, tile_cnt);
    hipLaunchKernelGGL(k_pk_scan, dim3(1), dim3(1024), 0, s, tile_cnt, nt, in, err);
    hipLaunchKernelGGL(k_pk_expand, dim3(nt), dim3(PK_T), 0, s, in, (const uint2*)tile_cnt, out);
    return hipGetLastError();
}

}  // namespace sf
