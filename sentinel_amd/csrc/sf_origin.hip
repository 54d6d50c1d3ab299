// sf_origin.hip — origin nodes of the traffic that no rule reads (product code).
//
// ClusterBuilderSlot.entry gives every entry with a caller origin the origin
// node ClusterNode.getOrCreateOriginNode(origin) (ClusterBuilderSlot.java:107-110,
// ClusterNode.java:101-120), and StatisticSlot updates it beside the
// resource's node on every outcome (StatisticSlot.java:64-123 entry, :139-178
// exit): pass + thread, PriorityWaitException thread only, block, and on the
// exit of a passed entry rt + success (+ exception) and thread.  A flow rule
// reads an origin node only through its limitApp
// (FlowRuleChecker.selectNodeByRequesterAndStrategy :129-161); resources with
// such rules run on the xflow walk (sf_xflow.h), which updates their origin
// nodes in line.  For every other resource the origin nodes are written and
// never read while the batch is decided, so they are brought up to date after
// the verdicts, in bulk, on the ordinary pipeline's segments:
//
//   sort phase   k_ox_index   every (resource, origin) key of the batch -- and
//                             the CHAIN context keys of xflow segments -- in the
//                             pool's index table, a pool slot for each new one
//                             (the host then grows the pool to cover them before
//                             the decide phase: no batch fails on capacity), the
//                             slot of each event (s_oslot), and a dense id for
//                             each pair of a long segment
//   decide phase k_ox_light   segments of at most OX_LIGHT events: one thread
//                             per (resource, origin) pair replays the pair's
//                             events in time order on its node (NodeWin, the
//                             lane interpreter's window code)
//                k_ox_hacc    longer segments: per-window sums of every pair of
//                             the block (LDS), then global atomics
//                k_ox_happly  one thread per pair of a long segment: the latest
//                             window of each bucket slot merged with
//                             LeapArray.currentWindow's reset rule (a later
//                             window of the slot overwrites an earlier one), and
//                             the thread delta
#include <cstring>

#include "sf_heavy.h"
#include "sf_xflow.h"

namespace sf {

constexpr int OX_T = 256;
constexpr uint32_t OX_ITILE = 1024;            // events per k_ox_index workgroup
constexpr uint32_t OX_KCAP = 2048;             // its LDS key table (<= 2 keys per event)
constexpr uint64_t AX_CLAIM = 1ull << 63;      // index slot being claimed (pkey_hi never sets bit 63: R < 2^30)
constexpr uint32_t HX_CLAIM = 0xfffffffeu;     // heavy id being assigned

// LDS key of (local resource, kind, id): nonzero
__device__ __forceinline__ unsigned long long ox_pack(uint32_t l, uint32_t kind, uint32_t id) {
    return ((unsigned long long)(l + 1u) << 34) | ((unsigned long long)kind << 32) | id;
}
__device__ __forceinline__ uint32_t ox_l(unsigned long long k) { return (uint32_t)(k >> 34) - 1u; }
__device__ __forceinline__ uint32_t ox_kind(unsigned long long k) { return (uint32_t)(k >> 32) & 3u; }

// insert into a block's LDS key set; returns the position, *fresh when this call added it
__device__ __forceinline__ uint32_t ox_lds_insert(unsigned long long* keys, unsigned long long k, bool* fresh) {
    uint32_t h = (uint32_t)(mix64(k) & (OX_KCAP - 1));
    for (uint32_t p = 0; p < OX_KCAP; p++) {
        const unsigned long long prev = atomicCAS(&keys[h], 0ull, k);
        if (prev == 0ull) { *fresh = true; return h; }
        if (prev == k) { *fresh = false; return h; }
        h = (h + 1) & (OX_KCAP - 1);
    }
    *fresh = false;
    return XNONE;                                   // (unreachable: at most OX_KCAP keys)
}

struct OxIdx {
    const uint32_t* head_scan; const uint32_t* seg_start; const uint32_t* seg_res; const uint8_t* seg_mode;
    const uint32_t* segflag; const uint32_t* perm; const uint32_t* s_origin; uint32_t* s_oslot;
    uint32_t* hmap; uint32_t hmap_n; uint32_t* hslot; uint32_t hslot_n; uint32_t* cnt;
    uint32_t* bflags;          // [n / OX_TILE + 1] OXB_* work of each OX_TILE block for the decide-phase kernels
};
enum : uint32_t { OXB_LIGHT = 1u, OXB_HEAVY = 2u };

// One workgroup per OX_ITILE sorted events.  Keys are deduplicated in LDS;
// each distinct key is found in the index table or claimed (CAS of the key's
// high word with AX_CLAIM), and the claims of a round get consecutive pool
// slots from one atomic on ax_count, then are published.  A key another
// workgroup is claiming is retried in the next round (no thread waits on
// another workgroup across a barrier).  Once ax_count passes `lim` (the table's
// load limit) nothing more is claimed: OXC_OVERFLOW tells the host to grow the
// table and run the pass again (the pass is idempotent).
__global__ void __launch_bounds__(OX_T) k_ox_index(DevState st, DevBatch b, OxIdx ox, uint32_t lim) {
    __shared__ unsigned long long kk[OX_KCAP];
    __shared__ uint32_t kslot[OX_KCAP];        // pool slot, XNONE until resolved
    __shared__ uint32_t kclaim[OX_KCAP];       // index-table position claimed this round (XNONE: none)
    __shared__ uint32_t ul[OX_KCAP];           // LDS positions of the distinct keys
    __shared__ uint8_t kheavy[OX_KCAP];        // a pair of a long segment (dense heavy id wanted)
    __shared__ uint32_t nu, nclaim, base, retry, stop, bfl;
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < OX_KCAP; k += OX_T) { kk[k] = 0; kslot[k] = XNONE; kclaim[k] = XNONE; kheavy[k] = 0; }
    if (tid == 0) { nu = 0; bfl = 0; }
    __syncthreads();
    const uint32_t j0 = blockIdx.x * OX_ITILE, j1 = min(b.n, j0 + OX_ITILE);
    // 1. the keys of the tile's events
    for (uint32_t j = j0 + tid; j < j1; j += OX_T) {
        const uint32_t sid = ox.head_scan[j] - 1u;
        const uint32_t lo = ox.seg_start[sid], hi = ox.seg_start[sid + 1];
        const uint32_t o = ox.s_origin ? ox.s_origin[j] : SF_ORIGIN_NONE;
        bool fresh;
        if (ox.seg_mode[sid] == SM_XFLOW) {
            // the xflow walk's nodes: the origin node of every entry with an
            // origin, the context node while a CHAIN rule names the context
            // (decide_xgroup's want_on / want_dn)
            const uint32_t i = ox.perm[j];
            const uint32_t l = b.res[i] / st.shard_count;
            if (o != SF_ORIGIN_NONE) {
                const uint32_t p = ox_lds_insert(kk, ox_pack(l, AX_ORIGIN, o), &fresh);
                if (fresh) ul[atomicAdd(&nu, 1u)] = p;
            }
            const uint32_t ctx = b.ctx ? b.ctx[i] : 0u;
            bool want = false;
            for (uint32_t k = st.rule_off[l]; k < st.rule_off[l + 1]; k++)
                if (st.rules[k].strategy == SF_STRATEGY_CHAIN && st.rules[k].ref == ctx) want = true;
            if (want) {
                const uint32_t p = ox_lds_insert(kk, ox_pack(l, AX_CTX, ctx), &fresh);
                if (fresh) ul[atomicAdd(&nu, 1u)] = p;
            }
        } else if (o != SF_ORIGIN_NONE) {
            const uint32_t p = ox_lds_insert(kk, ox_pack(ox.seg_res[sid], AX_ORIGIN, o), &fresh);
            if (fresh) ul[atomicAdd(&nu, 1u)] = p;
            if (hi - lo > OX_LIGHT) { kheavy[p] = 1; atomicOr(&bfl, OXB_HEAVY); }
            else atomicOr(&bfl, OXB_LIGHT);           // (its segment starts in this OX_TILE block or the one before)
        }
    }
    __syncthreads();
    if (tid == 0 && bfl) {
        // a light segment is walked by the block it starts in
        const uint32_t blk = j0 / OX_TILE;
        atomicOr(&ox.bflags[blk], bfl);
        if ((bfl & OXB_LIGHT) && ox.seg_start[ox.head_scan[j0] - 1u] < blk * OX_TILE) atomicOr(&ox.bflags[blk - 1], OXB_LIGHT);
    }
    // 2. resolve the distinct keys against the index table, in rounds
    ParamTable t{st.xtab, st.xcap_mask, st.err};
    const uint64_t reach = t.mask < PT_MAX_PROBE ? t.mask : PT_MAX_PROBE;
    for (;;) {
        if (tid == 0) {
            nclaim = 0; retry = 0;
            stop = __hip_atomic_load(st.ax_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > lim;
        }
        __syncthreads();
        for (uint32_t u = tid; u < nu; u += OX_T) {
            const uint32_t p = ul[u];
            if (kslot[p] != XNONE) continue;
            const unsigned long long key = kk[p];
            const uint64_t khi = pkey_hi(ox_l(key), PK_AUX, ox_kind(key), 0), klo = (uint32_t)key;
            uint64_t i = ParamTable::hash(khi, klo) & t.mask;
            for (uint64_t probe = 0;; ) {
                ParamSlot& s = t.slots[i];
                const uint64_t h = __hip_atomic_load(&s.hi, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if (h == 0) {
                    if (stop) { atomicOr((uint32_t*)&ox.cnt[OXC_OVERFLOW], 1u); break; }
                    unsigned long long expected = 0;
                    if (__hip_atomic_compare_exchange_strong((unsigned long long*)&s.hi, &expected,
                                                             (unsigned long long)(khi | AX_CLAIM), __ATOMIC_ACQUIRE,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        kclaim[p] = (uint32_t)i;
                        atomicAdd(&nclaim, 1u);
                        break;
                    }
                    continue;                          // lost the race: this slot again
                }
                if (h & AX_CLAIM) { retry = 1; break; }   // being claimed by another workgroup
                if (h == khi && s.lo == klo) { kslot[p] = (uint32_t)s.a; break; }
                i = (i + 1) & t.mask;
                if (++probe > reach) { atomicOr((uint32_t*)&ox.cnt[OXC_OVERFLOW], 1u); break; }
            }
        }
        __syncthreads();
        if (tid == 0 && nclaim) base = atomicAdd(st.ax_count, nclaim);
        if (tid == 0) nclaim = 0;
        __syncthreads();
        for (uint32_t u = tid; u < nu; u += OX_T) {
            const uint32_t p = ul[u];
            if (kclaim[p] == XNONE) continue;
            ParamSlot& s = t.slots[kclaim[p]];
            const uint32_t a = base + atomicAdd(&nclaim, 1u);
            const unsigned long long key = kk[p];
            s.lo = (uint32_t)key; s.a = a; s.b = 0;
            __hip_atomic_store(&s.hi, pkey_hi(ox_l(key), PK_AUX, ox_kind(key), 0), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
            kslot[p] = a;
            kclaim[p] = XNONE;
        }
        __syncthreads();
        if (!retry) break;
        __syncthreads();
    }
    // 3. dense ids of the pairs of long segments (k_ox_hacc / k_ox_happly), same rounds
    for (;;) {
        if (tid == 0) { nclaim = 0; retry = 0; }
        __syncthreads();
        for (uint32_t u = tid; u < nu; u += OX_T) {
            const uint32_t p = ul[u];
            const uint32_t a = kslot[p];
            if (!kheavy[p] || a == XNONE) continue;
            if (a >= ox.hmap_n) { atomicOr((uint32_t*)&ox.cnt[OXC_OVERFLOW], 2u); kheavy[p] = 0; continue; }
            const uint32_t h = __hip_atomic_load(&ox.hmap[a], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (h == XNONE) {
                uint32_t expected = XNONE;
                if (__hip_atomic_compare_exchange_strong(&ox.hmap[a], &expected, HX_CLAIM, __ATOMIC_ACQUIRE,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    kclaim[p] = atomicAdd(&nclaim, 1u);
                    continue;
                }
                retry = 1;
            } else if (h == HX_CLAIM) {
                retry = 1;
            } else {
                kheavy[p] = 0;                         // has its id
            }
        }
        __syncthreads();
        if (tid == 0 && nclaim) base = atomicAdd(&ox.cnt[OXC_HEAVY], nclaim);
        __syncthreads();
        for (uint32_t u = tid; u < nu; u += OX_T) {
            const uint32_t p = ul[u];
            if (kclaim[p] == XNONE) continue;
            const uint32_t hid = base + kclaim[p];
            const uint32_t a = kslot[p];
            if (hid < ox.hslot_n) ox.hslot[hid] = a;
            else atomicOr((uint32_t*)&ox.cnt[OXC_OVERFLOW], 2u);
            __hip_atomic_store(&ox.hmap[a], hid < ox.hslot_n ? hid : XNONE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            kclaim[p] = XNONE;
            kheavy[p] = 0;
        }
        __syncthreads();
        if (!retry) break;
        __syncthreads();
    }
    // 4. the slot of every event (ordinary segments; the xflow walk finds its own)
    for (uint32_t j = j0 + tid; j < j1; j += OX_T) {
        const uint32_t sid = ox.head_scan[j] - 1u;
        const uint32_t o = ox.s_origin ? ox.s_origin[j] : SF_ORIGIN_NONE;
        uint32_t a = XNONE;
        if (o != SF_ORIGIN_NONE && ox.seg_mode[sid] != SM_XFLOW) {
            bool fresh;
            const uint32_t p = ox_lds_insert(kk, ox_pack(ox.seg_res[sid], AX_ORIGIN, o), &fresh);
            if (p != XNONE) a = kslot[p];
        }
        ox.s_oslot[j] = a;
    }
}

// ------------------------------------------------------------------ decide phase
struct OxRun {
    const uint32_t* seg_start; const uint32_t* seg_res; const uint8_t* seg_mode; const uint32_t* segflag;
    const uint32_t* n_seg;
    const int64_t* ts; const int32_t* cnt; const uint8_t* flags; const int64_t* eref; const int64_t* cts;
    const uint8_t* v_status; const uint32_t* s_oslot;
    const uint32_t* hmap; const uint32_t* hslot; OxAcc* acc; int64_t* thr;
    const uint32_t* bflags;
    uint32_t n; OxWin win;
};

// last segment whose start is <= j
__device__ __forceinline__ uint32_t ox_seg_of(const OxRun& r, uint32_t j) {
    uint32_t a = 0, e = *r.n_seg;                  // seg_start[a] <= j < seg_start[e]
    while (e - a > 1) { const uint32_t m = (a + e) >> 1; if (r.seg_start[m] <= j) a = m; else e = m; }
    return a;
}
__device__ __forceinline__ bool ox_origin_seg(const OxRun& r, uint32_t s) {
    return r.seg_mode[s] != SM_XFLOW && (r.segflag[s] & SEGF_ORIGIN);
}

// StatisticSlot's update of the origin node for sorted event j (verdict known)
template <int MAXS>
__device__ __forceinline__ void ox_apply_event(NodeWin<MAXS>& on, const OxRun& r, uint32_t j) {
    const uint8_t v = r.v_status[j], fl = r.flags[j];
    const int64_t t = r.ts[j];
    const int32_t c = r.cnt[j];
    if (fl & SF_EV_EXIT) {                                   // StatisticSlot.exit :139-165 (recordCompleteFor)
        if (v != SF_V_EXIT) return;                          // its entry was blocked: nothing is recorded
        const int64_t ref = r.eref ? r.eref[j] : -1;
        const int64_t cts = ref >= 0 ? r.ts[ref] : (r.cts ? r.cts[j] : t);
        on.add_rt_success(t, t - cts, c);
        on.threads--;
        if (fl & SF_EV_ERROR) on.add_exception(t, c);
    } else if (v_blocked(v)) {                               // :102-124 BlockException
        on.add_block(t, c);
    } else {
        on.threads++;                                        // pass, or PriorityWaitException (:84-101)
        if (v != SF_V_PRIORITY_WAIT) on.add_pass(t, c);
    }
}

// One workgroup per OX_TILE block: the segments of at most OX_LIGHT events that
// start in it.  Each (resource, origin) pair is owned by one thread (the first
// to put its pool slot into the block's LDS set), which walks the pair's
// segment in time order and applies the pair's events to the node.
constexpr uint32_t OX_LSPAN = OX_TILE + OX_LIGHT;
template <int MAXS>
__global__ void __launch_bounds__(OX_T) k_ox_light(DevState st, OxRun r) {
    __shared__ uint32_t lslot[OX_LSPAN];        // s_oslot of [A, A + OX_LSPAN)
    __shared__ uint32_t sstart[OX_TILE + 2];    // starts of the block's segments (+ the end of the last)
    __shared__ uint32_t owners[OX_LSPAN];       // owner event positions (relative to A)
    __shared__ uint32_t owseg[OX_LSPAN];        // their segment (index into sstart)
    __shared__ uint32_t set[2 * OX_LSPAN];      // LDS set of the pool slots (XNONE: empty)
    __shared__ uint32_t s0, ns, nown, A;
    constexpr uint32_t SETN = 2 * OX_LSPAN;
    const uint32_t tid = threadIdx.x;
    const uint32_t j0 = blockIdx.x * OX_TILE;
    if (j0 >= r.n || !(r.bflags[blockIdx.x] & OXB_LIGHT)) return;
    const uint32_t jend = min(r.n, j0 + OX_TILE);
    if (tid == 0) {
        uint32_t s = ox_seg_of(r, j0);
        if (r.seg_start[s] < j0) s++;                // the first segment starting in the block
        s0 = s; nown = 0;
        const uint32_t nseg = *r.n_seg;
        const uint32_t e = ox_seg_of(r, jend - 1) + 1; // one past the last segment starting in the block
        ns = e > s ? e - s : 0;
        A = s < nseg ? r.seg_start[s] : r.n;
    }
    for (uint32_t k = tid; k < SETN; k += OX_T) set[k] = XNONE;
    __syncthreads();
    if (ns == 0) return;
    for (uint32_t k = tid; k <= ns; k += OX_T) sstart[k] = r.seg_start[s0 + k];
    for (uint32_t q = tid; q < OX_LSPAN; q += OX_T) lslot[q] = A + q < r.n ? r.s_oslot[A + q] : XNONE;
    __syncthreads();
    // owners: per event of a light origin segment, the first insert of its slot
    const uint32_t span = min(OX_LSPAN, sstart[ns] - A);
    for (uint32_t q = tid; q < span; q += OX_T) {
        const uint32_t a = lslot[q];
        if (a == XNONE) continue;
        uint32_t lo_ = 0, hi_ = ns;                  // segment k of A + q: sstart[k] <= A + q < sstart[k + 1]
        while (hi_ - lo_ > 1) { const uint32_t m = (lo_ + hi_) >> 1; if (sstart[m] <= A + q) lo_ = m; else hi_ = m; }
        const uint32_t k = lo_;
        if (sstart[k + 1] - sstart[k] > OX_LIGHT || !ox_origin_seg(r, s0 + k)) continue;
        uint32_t h = (uint32_t)(mix64(a) % SETN);
        for (;;) {
            const uint32_t prev = atomicCAS(&set[h], XNONE, a);
            if (prev == XNONE) { const uint32_t w = atomicAdd(&nown, 1u); owners[w] = q; owseg[w] = k; break; }
            if (prev == a) break;
            h = h + 1 == SETN ? 0 : h + 1;
        }
    }
    __syncthreads();
    for (uint32_t w = tid; w < nown; w += OX_T) {
        const uint32_t q = owners[w], k = owseg[w];
        const uint32_t a = lslot[q];
        const uint32_t lo = sstart[k], hi = sstart[k + 1];
        const NodeRows rows = aux_rows(st, a);
        NodeWin<MAXS> on;
        nw_load(on, st, rows);
        for (uint32_t j = lo; j < hi; j++)                   // the pair's events in time order
            if (lslot[j - A] == a) ox_apply_event<MAXS>(on, r, j);
        nw_store(on, st, rows);
    }
}

// ---- long segments: per-window sums
__device__ __forceinline__ unsigned long long ox_minrt_key(int64_t rt) {
    return ~((unsigned long long)rt ^ 0x8000000000000000ull);            // larger key = smaller rt; 0 = none
}
__device__ __forceinline__ int64_t ox_minrt_of(unsigned long long k) {
    return (int64_t)(~k ^ 0x8000000000000000ull);
}

constexpr uint32_t OX_HCAP = 512;                 // LDS (pair, window) rows of a k_ox_hacc block
struct OxRow { unsigned long long key; unsigned long long v[7]; };   // key: hid << 32 | kind << 31 | window + 1

__device__ __forceinline__ void ox_add_row(unsigned long long* v, const unsigned long long* d) {
    for (int f = 0; f < 6; f++) if (d[f]) atomicAdd(&v[f], d[f]);
    if (d[6]) atomicMax(&v[6], d[6]);
}

// One workgroup per OX_TILE block with events of long origin segments: the
// block's (pair, window) sums in LDS, then one set of global atomics per row.
__global__ void __launch_bounds__(OX_T) k_ox_hacc(DevState st, OxRun r) {
    __shared__ OxRow rows[OX_HCAP];
    __shared__ uint32_t sst[OX_TILE + 1];        // starts of the segments overlapping the block, then their end
    __shared__ uint32_t sfirst, nseg_b;
    const uint32_t tid = threadIdx.x;
    const uint32_t j0 = blockIdx.x * OX_TILE;
    if (j0 >= r.n || !(r.bflags[blockIdx.x] & OXB_HEAVY)) return;
    const uint32_t j1 = min(r.n, j0 + OX_TILE);
    if (tid == 0) { sfirst = ox_seg_of(r, j0); nseg_b = ox_seg_of(r, j1 - 1) - sfirst + 1; }
    for (uint32_t k = tid; k < OX_HCAP; k += OX_T) {
        rows[k].key = 0;
        for (int f = 0; f < 7; f++) rows[k].v[f] = 0;
    }
    __syncthreads();
    for (uint32_t k = tid; k <= nseg_b; k += OX_T) sst[k] = r.seg_start[sfirst + k];
    __syncthreads();
    const uint32_t W = r.win.ws + r.win.wm;
    const int64_t b_s = r.win.w0s * st.wl, b_m = r.win.w0m * 1000;
    for (uint32_t j = j0 + tid; j < j1; j += OX_T) {
        uint32_t a_ = 0, e_ = nseg_b;                   // sst[a_] <= j < sst[a_ + 1]
        while (e_ - a_ > 1) { const uint32_t m = (a_ + e_) >> 1; if (sst[m] <= j) a_ = m; else e_ = m; }
        if (sst[a_ + 1] - sst[a_] <= OX_LIGHT || !ox_origin_seg(r, sfirst + a_)) continue;
        const uint32_t a = r.s_oslot[j];
        if (a == XNONE) continue;
        const uint32_t hid = r.hmap[a];
        if (hid == XNONE) continue;                       // (cannot happen: k_ox_index gave every such pair an id)
        const uint8_t v = r.v_status[j], fl = r.flags[j];
        const int64_t t = r.ts[j];
        const int32_t c = r.cnt[j];
        unsigned long long d[7] = {0, 0, 0, 0, 0, 0, 0};
        int64_t dthr = 0;
        bool touch = true;
        if (fl & SF_EV_EXIT) {
            if (v != SF_V_EXIT) continue;
            const int64_t ref = r.eref ? r.eref[j] : -1;
            const int64_t cts = ref >= 0 ? r.ts[ref] : (r.cts ? r.cts[j] : t);
            const int64_t rt = t - cts;
            d[2] = (unsigned long long)(int64_t)c; d[3] = (unsigned long long)rt;
            if (fl & SF_EV_ERROR) d[4] = (unsigned long long)(int64_t)c;
            d[6] = ox_minrt_key(rt);
            dthr = -1;
        } else if (v_blocked(v)) {
            d[1] = (unsigned long long)(int64_t)c;
        } else {
            dthr = 1;
            if (v == SF_V_PRIORITY_WAIT) touch = false;
            else d[0] = (unsigned long long)(int64_t)c;
        }
        d[5] = 1;
        const uint32_t wsec = (uint32_t)((t - b_s) / st.wl), wmin = (uint32_t)((t - b_m) / 1000);
        // rows: the second window, the minute window, the thread delta (row W)
        for (int kind = 0; kind < 3; kind++) {
            if (kind < 2 && !touch) continue;
            if (kind == 2 && !dthr) continue;
            const uint32_t w = kind == 0 ? wsec : (kind == 1 ? r.win.ws + wmin : W);
            unsigned long long dt[7] = {(unsigned long long)dthr, 0, 0, 0, 0, 0, 0};
            const unsigned long long* dd = kind == 2 ? dt : d;
            const unsigned long long key = ((unsigned long long)hid << 32) | (w + 1u);
            uint32_t h = (uint32_t)(mix64(key) & (OX_HCAP - 1));
            bool done = false;
            for (uint32_t p = 0; p < 16 && !done; p++) {
                const unsigned long long prev = atomicCAS(&rows[h].key, 0ull, key);
                if (prev == 0ull || prev == key) { ox_add_row(rows[h].v, dd); done = true; }
                else h = (h + 1) & (OX_HCAP - 1);
            }
            if (!done) {                                  // LDS rows full: straight to the global sums
                if (kind == 2) atomicAdd((unsigned long long*)&r.thr[hid], (unsigned long long)dthr);
                else ox_add_row(&r.acc[(size_t)hid * W + w].pass, dd);   // (OxAcc fields in v[] order)
            }
        }
    }
    __syncthreads();
    for (uint32_t k = tid; k < OX_HCAP; k += OX_T) {
        const unsigned long long key = rows[k].key;
        if (!key) continue;
        const uint32_t hid = (uint32_t)(key >> 32), w = (uint32_t)key - 1u;
        if (w == W) { if (rows[k].v[0]) atomicAdd((unsigned long long*)&r.thr[hid], rows[k].v[0]); }
        else ox_add_row(&r.acc[(size_t)hid * W + w].pass, rows[k].v);
    }
}

// merge one window's sums into a bucket (LeapArray.currentWindow: a newer
// window resets the bucket; OccupiableBucketLeapArray.newEmptyBucket /
// resetWindowTo seed a reset second-window bucket with the borrowed pass)
__device__ __forceinline__ void ox_merge(Bucket& bk, int64_t ws, const OxAcc& a, int64_t max_rt, const Borrow* br,
                                         int32_t wl) {
    if (bk.ws != ws) {
        if (ws < bk.ws) return;                          // throwaway window (time never goes back)
        Bucket nb = fresh_bucket(ws, max_rt);
        if (br && br->ws <= ws && ws < br->ws + wl) nb.pass = (int64_t)(int32_t)br->pass;
        bk = nb;
    }
    bk.pass = wadd(bk.pass, (int64_t)a.pass); bk.block = wadd(bk.block, (int64_t)a.block);
    bk.succ = wadd(bk.succ, (int64_t)a.succ); bk.rt = wadd(bk.rt, (int64_t)a.rt); bk.exc = wadd(bk.exc, (int64_t)a.exc);
    if (a.min_rt_key) { const int64_t m = ox_minrt_of(a.min_rt_key); if (m < bk.min_rt) bk.min_rt = m; }
}

__global__ void k_ox_happly(DevState st, OxRun r, const uint32_t* n_heavy) {
    const uint32_t hid = blockIdx.x * blockDim.x + threadIdx.x;
    if (hid >= *n_heavy) return;
    const uint32_t a = r.hslot[hid];
    const NodeRows rows = aux_rows(st, a);
    const uint32_t W = r.win.ws + r.win.wm;
    const OxAcc* acc = r.acc + (size_t)hid * W;
    unsigned long long done = 0;                        // second-window slots merged (S <= 16)
    for (int w = (int)r.win.ws - 1; w >= 0; w--) {
        const OxAcc x = acc[w];
        if (!x.n_touch) continue;
        const int64_t wa = r.win.w0s + w;
        const int idx = (int)(wa % st.S);
        if ((done >> idx) & 1ull) continue;              // a later window of the slot overwrote it
        done |= 1ull << idx;
        Bucket bk = rows.sec[idx];
        ox_merge(bk, wa * st.wl, x, st.max_rt, &rows.bor[idx], st.wl);
        rows.sec[idx] = bk;
    }
    done = 0;
    for (int w = (int)r.win.wm - 1; w >= 0; w--) {
        const OxAcc x = acc[r.win.ws + w];
        if (!x.n_touch) continue;
        const int64_t wa = r.win.w0m + w;
        const int idx = (int)(wa % MINUTE);
        if ((done >> idx) & 1ull) continue;
        done |= 1ull << idx;
        Bucket bk = rows.min[idx];
        ox_merge(bk, wa * 1000, x, st.max_rt, nullptr, st.wl);
        rows.min[idx] = bk;
    }
    *rows.thr = wadd(*rows.thr, r.thr[hid]);
}

// the heavy ids of this batch back to XNONE (the map is reused by the Work set's next batch)
__global__ void k_ox_reset(OxRun r, uint32_t* hmap, const uint32_t* n_heavy) {
    const uint32_t hid = blockIdx.x * blockDim.x + threadIdx.x;
    if (hid < *n_heavy) hmap[r.hslot[hid]] = XNONE;
}

// ------------------------------------------------------------------ launchers
static inline unsigned ox_blocks(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

hipError_t launch_ox_index(const DevState& st, Work& w, const DevBatch& b, uint32_t lim, hipStream_t s) {
    if (!b.n) return hipSuccess;
    OxIdx ox{w.head_scan, w.seg_start, w.seg_res, w.seg_mode, w.segflag, w.perm, b.origin ? w.s_origin : nullptr,
             w.s_oslot,
             w.ox_hmap, (uint32_t)std::min<size_t>(w.ox_hmap_n, 0xffffffffu), w.ox_hslot,
             (uint32_t)std::min<size_t>(w.ox_hslot_n, 0xffffffffu), w.ox_cnt, w.ox_bflags};
    hipMemsetAsync(w.ox_cnt, 0, 8 * sizeof(uint32_t), s);
    hipMemsetAsync(w.ox_bflags, 0, ((size_t)b.n / OX_TILE + 1) * sizeof(uint32_t), s);
    hipLaunchKernelGGL(k_ox_index, dim3(ox_blocks(b.n, OX_ITILE)), dim3(OX_T), 0, s, st, b, ox, lim);
    return hipGetLastError();
}

hipError_t launch_ox_apply(const DevState& st, Work& w, const DevBatch& b, uint32_t n_heavy, const OxWin& win,
                           hipStream_t s) {
    if (!b.n) return hipSuccess;
    OxRun r{};
    r.seg_start = w.seg_start; r.seg_res = w.seg_res; r.seg_mode = w.seg_mode; r.segflag = w.segflag;
    r.n_seg = w.n_seg;
    r.ts = w.s_ts; r.cnt = w.s_cnt; r.flags = w.s_flags;
    r.eref = b.eref ? w.s_eref : nullptr; r.cts = b.eref ? w.s_cts : nullptr;
    r.v_status = w.v_status; r.s_oslot = w.s_oslot;
    r.hmap = w.ox_hmap; r.hslot = w.ox_hslot; r.acc = (OxAcc*)w.ox_acc; r.thr = w.ox_thr; r.bflags = w.ox_bflags;
    r.n = b.n; r.win = win;
    const unsigned nblk = ox_blocks(b.n, OX_TILE);
    if (st.S <= 2) hipLaunchKernelGGL(k_ox_light<2>, dim3(nblk), dim3(OX_T), 0, s, st, r);
    else hipLaunchKernelGGL(k_ox_light<SF_MAX_SAMPLE_COUNT>, dim3(nblk), dim3(OX_T), 0, s, st, r);
    if (n_heavy) {
        const size_t W = (size_t)win.ws + win.wm;
        hipMemsetAsync(w.ox_acc, 0, (size_t)n_heavy * W * sizeof(OxAcc), s);
        hipMemsetAsync(w.ox_thr, 0, (size_t)n_heavy * sizeof(int64_t), s);
        hipLaunchKernelGGL(k_ox_hacc, dim3(nblk), dim3(OX_T), 0, s, st, r);
        hipLaunchKernelGGL(k_ox_happly, dim3(ox_blocks(n_heavy, 256)), dim3(256), 0, s, st, r, w.ox_cnt + OXC_HEAVY);
        hipLaunchKernelGGL(k_ox_reset, dim3(ox_blocks(n_heavy, 256)), dim3(256), 0, s, r, w.ox_hmap,
                           w.ox_cnt + OXC_HEAVY);
    }
    return hipGetLastError();
}

// the index table rebuilt in a larger one (between batches: nothing else runs)
__global__ void k_ox_rehash(const ParamSlot* old_tab, uint64_t old_n, ParamSlot* tab, uint64_t mask, int32_t* err) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= old_n) return;
    const ParamSlot s = old_tab[k];
    if (s.hi == 0) return;
    uint64_t i = ParamTable::hash(s.hi, s.lo) & mask;
    for (uint64_t p = 0; p <= mask; p++) {
        unsigned long long expected = 0;
        if (__hip_atomic_compare_exchange_strong((unsigned long long*)&tab[i].hi, &expected, (unsigned long long)s.hi,
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            tab[i].lo = s.lo; tab[i].a = s.a; tab[i].b = s.b;
            return;
        }
        i = (i + 1) & mask;
    }
    *err = SF_ERR_CAPACITY;
}
hipError_t launch_ox_rehash(const ParamSlot* old_tab, uint64_t old_n, ParamSlot* new_tab, uint64_t new_mask,
                            int32_t* err, hipStream_t s) {
    if (!old_n) return hipSuccess;
    hipLaunchKernelGGL(k_ox_rehash, dim3(ox_blocks(old_n, 256)), dim3(256), 0, s, old_tab, old_n, new_tab, new_mask, err);
    return hipGetLastError();
}

// sf_read_origin_node / sf_read_context_node: one key's pool slot (XNONE: not kept)
__global__ void k_aux_find(DevState st, uint64_t hi, uint64_t lo, uint32_t* out) {
    ParamTable t{st.xtab, st.xcap_mask, st.err};
    const ParamSlot* p = t.find(hi, lo);
    *out = p ? (uint32_t)p->a : XNONE;
}
hipError_t launch_aux_find(const DevState& st, uint64_t hi, uint64_t lo, uint32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_aux_find, dim3(1), dim3(1), 0, s, st, hi, lo, out);
    return hipGetLastError();
}

}  // namespace sf
