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
//   sort phase   k_ox_ilight  segments of at most OX_LIGHT events: the distinct
//                             (resource, origin) pairs of the segments starting in
//                             a block (LDS) and each pair's events in time order
//                             (block radix sort), listed for the next two kernels
//                k_ox_lfind   one thread per listed pair: its pool slot from the
//                             index table, or a new one
//                k_ox_index   longer segments and the xflow walk's segments: the
//                             distinct keys of a tile (and the CHAIN context keys
//                             of xflow segments) resolved per workgroup, a dense
//                             id per pair of a long segment, each event's slot
//                             (s_oslot)
//                             (the host then grows the pool to cover every new
//                             slot before the decide phase: no batch fails on
//                             capacity)
//   decide phase k_ox_lapply  one thread per listed pair replays the pair's events
//                             in time order on its node (NodeWin, the lane
//                             interpreter's window code)
//                k_ox_hacc    longer segments: per-window sums of every pair of
//                             the block (LDS), then global atomics
//                k_ox_happly  one thread per pair of a long segment: the latest
//                             window of each bucket slot merged with
//                             LeapArray.currentWindow's reset rule (a later
//                             window of the slot overwrites an earlier one), and
//                             the thread delta
#include <cstring>

#include <rocprim/block/block_radix_sort.hpp>

#include "sf_heavy.h"
#include "sf_xflow.h"

namespace sf {

constexpr int OX_T = 256;
constexpr uint32_t OX_ITILE = 2048;            // events per k_ox_index workgroup (one OX_TILE block)
constexpr uint32_t OX_LTILE = 1024;            // sorted positions whose segments one k_ox_ilight workgroup lists
constexpr uint32_t OX_KCAP = 2048;             // k_ox_ilight's LDS key table (<= 1536 keys)
constexpr uint32_t OX_IKCAP = 4096;            // k_ox_index's (<= 2 keys per event)
constexpr uint64_t AX_CLAIM = 1ull << 63;      // index slot being claimed (pkey_hi never sets bit 63: R < 2^30)
constexpr uint32_t KS_CLAIMED = 0x80000000u;   // kslot: index-table position claimed this round (pool slots < 2^31)
constexpr uint32_t HX_CLAIM = 0xfffffffeu;     // heavy id being assigned
enum : uint32_t { OXB_LIGHT = 1u, OXB_HEAVY = 2u };

// LDS key: (local resource, kind, id) for k_ox_index, (segment - first + 1, origin) for k_ox_ilight; nonzero
__device__ __forceinline__ unsigned long long ox_pack(uint32_t l, uint32_t kind, uint32_t id) {
    return ((unsigned long long)(l + 1u) << 34) | ((unsigned long long)kind << 32) | id;
}
__device__ __forceinline__ uint32_t ox_l(unsigned long long k) { return (uint32_t)(k >> 34) - 1u; }
__device__ __forceinline__ uint32_t ox_kind(unsigned long long k) { return (uint32_t)(k >> 32) & 3u; }

// insert into a block's LDS key set; returns the position, *fresh when this call added it
template <uint32_t CAP = OX_KCAP>
__device__ __forceinline__ uint32_t ox_lds_insert(unsigned long long* keys, unsigned long long k, bool* fresh) {
    uint32_t h = (uint32_t)(mix64(k) & (CAP - 1));
    for (uint32_t p = 0; p < CAP; p++) {
        const unsigned long long prev = atomicCAS(&keys[h], 0ull, k);
        if (prev == 0ull) { *fresh = true; return h; }
        if (prev == k) { *fresh = false; return h; }
        h = (h + 1) & (CAP - 1);
    }
    *fresh = false;
    return XNONE;                                   // (unreachable: at most CAP keys)
}
template <uint32_t CAP = OX_KCAP>
__device__ __forceinline__ uint32_t ox_lds_find(const unsigned long long* keys, unsigned long long k) {
    uint32_t h = (uint32_t)(mix64(k) & (CAP - 1));
    for (uint32_t p = 0; p < CAP; p++) {
        const unsigned long long cur = keys[h];
        if (cur == k) return h;
        if (cur == 0ull) return XNONE;
        h = (h + 1) & (CAP - 1);
    }
    return XNONE;
}

struct OxIdx {
    const uint32_t* head_scan; const uint32_t* seg_start; const uint32_t* seg_res; const uint8_t* seg_mode;
    const uint32_t* perm; const uint32_t* s_origin; uint32_t* s_oslot;
    uint32_t* hmap; uint32_t hmap_n; uint32_t* hslot; uint32_t hslot_n; uint32_t* cnt;
    uint32_t* bflags;          // [n / OX_TILE + 1] OXB_* work of each OX_TILE block for the decide phase
    uint2* bseg;               // [n / OX_TILE + 1] first and last segment overlapping each OX_TILE block
    uint4* pairs; uint32_t pairs_cap;   // k_ox_lapply's work: (pool slot, plist start, plist end)
    uint32_t* plist; uint32_t plist_cap; // each pair's events (sorted positions), in time order
};

// Resolve a workgroup's distinct LDS keys against the index table.  First a
// find of every key (a probe stops at the key or at an empty slot); the
// workgroup then reserves room for the keys it did not find with one atomic on
// OXC_RESERVED (the table's keys plus every reservation so far): past `lim`
// (the table's load limit) it claims nothing and sets OXC_OVERFLOW, and the
// host grows the table to the reserved total and runs the pass again (it is
// idempotent).  Otherwise the absent keys are claimed in rounds (CAS of the
// slot's high word to the key | AX_CLAIM); a round's claims get consecutive
// pool slots from one atomic on ax_count and are then published (lo, slot, the
// high word with release).  A key another workgroup is claiming is tried again
// next round -- no thread waits on another workgroup across a barrier, so a
// claimer always publishes.  key_of(p, &hi, &lo) gives LDS position p's key.
template <uint32_t CAP, class KeyOf>
__device__ void ox_resolve(const DevState& st, uint32_t* cnt, const unsigned long long* kk, uint32_t* kslot,
                           uint32_t lim, uint32_t* sh, KeyOf key_of) {
    ParamTable t{st.xtab, st.xcap_mask, st.err};
    const uint64_t reach = t.mask < PT_MAX_PROBE ? t.mask : PT_MAX_PROBE;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) sh[0] = 0;
    __syncthreads();
    // 1. find: the probes read the high words only, relaxed (no cache
    // invalidation per probe); one acquire fence per thread, then the low word
    // and slot of each candidate (a high word seen published by a release
    // store: the fence makes the publisher's earlier stores visible).  A
    // candidate of the same resource and another origin continues the probe
    // with acquire loads (rare).
    uint64_t cand[CAP / OX_T];
    bool any_cand = false;
#pragma unroll
    for (uint32_t k = 0; k < CAP / OX_T; k++) {
        const uint32_t p = k * OX_T + tid;
        cand[k] = ~0ull;
        if (!kk[p] || kslot[p] != XNONE) continue;
        uint64_t khi, klo;
        key_of(p, &khi, &klo);
        uint64_t i = ParamTable::hash(khi, klo) & t.mask;
        for (uint64_t probe = 0; probe <= reach; probe++) {
            const uint64_t h = __hip_atomic_load(&t.slots[i].hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (h == 0 || (h & AX_CLAIM)) break;               // absent (or being inserted: next rounds)
            if (h == khi) { cand[k] = i; any_cand = true; break; }
            i = (i + 1) & t.mask;
        }
    }
    if (any_cand) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
    for (uint32_t k = 0; k < CAP / OX_T; k++) {
        const uint32_t p = k * OX_T + tid;
        if (!kk[p] || kslot[p] != XNONE) continue;
        if (cand[k] != ~0ull) {
            uint64_t khi, klo;
            key_of(p, &khi, &klo);
            uint64_t i = cand[k];
            if (t.slots[i].lo == klo) {
                kslot[p] = (uint32_t)t.slots[i].a;
            } else {
                i = (i + 1) & t.mask;
                for (uint64_t probe = 0; probe <= reach; probe++) {
                    const ParamSlot& s = t.slots[i];
                    const uint64_t h = __hip_atomic_load(&s.hi, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    if (h == 0 || (h & AX_CLAIM)) break;
                    if (h == khi && s.lo == klo) { kslot[p] = (uint32_t)s.a; break; }
                    i = (i + 1) & t.mask;
                }
            }
        }
        if (kslot[p] == XNONE) atomicAdd(&sh[0], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        sh[2] = 0;
        if (sh[0]) {
            const uint32_t r = atomicAdd(&cnt[OXC_RESERVED], sh[0]);
            if ((uint64_t)r + sh[0] > lim) { sh[2] = 1; atomicOr(&cnt[OXC_OVERFLOW], 1u); }
        }
    }
    __syncthreads();
    if (!sh[0] || sh[2]) return;                                 // all found, or no room: the host grows the table
    for (;;) {                                                   // 2. claim the absent keys, in rounds
        if (tid == 0) { sh[0] = 0; sh[1] = 0; }
        __syncthreads();
        for (uint32_t p = tid; p < CAP; p += OX_T) {
            if (!kk[p] || kslot[p] != XNONE) continue;
            uint64_t khi, klo;
            key_of(p, &khi, &klo);
            uint64_t i = ParamTable::hash(khi, klo) & t.mask;
            for (uint64_t probe = 0;;) {
                ParamSlot& s = t.slots[i];
                const uint64_t h = __hip_atomic_load(&s.hi, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if (h == 0) {
                    unsigned long long expected = 0;
                    if (__hip_atomic_compare_exchange_strong((unsigned long long*)&s.hi, &expected,
                                                             (unsigned long long)(khi | AX_CLAIM), __ATOMIC_ACQUIRE,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        kslot[p] = KS_CLAIMED | (uint32_t)i;
                        atomicAdd(&sh[0], 1u);
                        break;
                    }
                    continue;                          // lost the race: this slot again
                }
                if (h & AX_CLAIM) { sh[1] = 1; break; }   // being claimed by another workgroup
                if (h == khi && s.lo == klo) { kslot[p] = (uint32_t)s.a; break; }
                i = (i + 1) & t.mask;
                if (++probe > reach) { atomicOr(&cnt[OXC_OVERFLOW], 1u); break; }
            }
        }
        __syncthreads();
        if (tid == 0) { if (sh[0]) sh[3] = atomicAdd(st.ax_count, sh[0]); sh[0] = 0; }
        __syncthreads();
        for (uint32_t p = tid; p < CAP; p += OX_T) {
            const uint32_t ks = kslot[p];
            if (ks == XNONE || !(ks & KS_CLAIMED)) continue;
            ParamSlot& s = t.slots[ks & ~KS_CLAIMED];
            const uint32_t a = sh[3] + atomicAdd(&sh[0], 1u);
            uint64_t khi, klo;
            key_of(p, &khi, &klo);
            s.lo = klo; s.a = a; s.b = 0;
            __hip_atomic_store(&s.hi, khi, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            kslot[p] = a;
        }
        __syncthreads();
        if (!sh[1]) break;
        __syncthreads();
    }
}

// k_ox_ilight: one workgroup per OX_LTILE sorted positions; the segments of at
// most OX_LIGHT events starting there (the ordinary pipeline's, not the xflow
// walk's).  A block radix sort of (pair rank, position) lists each distinct
// (resource, origin) pair's events in time order (plist), and each pair is
// recorded (resource, plist range, origin) for k_ox_lfind / k_ox_lapply.  No
// index-table access here: the lookups are k_ox_lfind's, one thread per pair.
constexpr uint32_t OX_LSPAN = OX_LTILE + OX_LIGHT;            // <= 1536 events of the block's light segments
constexpr uint32_t OX_SORT_ITEMS = 8;                          // block radix sort: 256 x 8 >= OX_LSPAN
static_assert(OX_T * OX_SORT_ITEMS >= OX_LSPAN && OX_LSPAN <= 2048, "k_ox_ilight: (rank, position) keys of 11 bits");
using OxBlockSort = rocprim::block_radix_sort<uint32_t, OX_T, OX_SORT_ITEMS>;
__global__ void __launch_bounds__(OX_T) k_ox_ilight(DevBatch b, OxIdx ox) {
    __shared__ unsigned long long kk[OX_KCAP];
    __shared__ uint16_t krank[OX_KCAP];
    __shared__ uint16_t rpos[OX_LSPAN];                        // pair rank -> LDS key position
    __shared__ uint32_t sorted[OX_T * OX_SORT_ITEMS];
    __shared__ typename OxBlockSort::storage_type sort_tmp;
    __shared__ uint32_t nu, nev, sA, A, span, pbase, lbase;
    const uint32_t tid = threadIdx.x;
    const uint32_t j0 = blockIdx.x * OX_LTILE, jend = min(b.n, j0 + OX_LTILE);
    for (uint32_t k = tid; k < OX_KCAP; k += OX_T) kk[k] = 0;
    if (tid == 0) {
        uint32_t s0 = ox.head_scan[j0] - 1u;
        if (ox.seg_start[s0] < j0) s0++;               // the first segment starting in the block
        const uint32_t s1 = ox.head_scan[jend - 1] - 1u + 1u;
        sA = s0; nu = 0; nev = 0;
        A = s0 < s1 ? ox.seg_start[s0] : 0u;
        span = s0 < s1 ? min(ox.seg_start[s1] - A, OX_LSPAN) : 0u;
    }
    __syncthreads();
    if (!span) return;
    // the pairs and each event's (pair, position) sort key
    uint32_t key8[OX_SORT_ITEMS];
    uint32_t kp[OX_SORT_ITEMS];
#pragma unroll
    for (uint32_t k = 0; k < OX_SORT_ITEMS; k++) { key8[k] = 0xffffffffu; kp[k] = XNONE; }
    bool any = false;
#pragma unroll
    for (uint32_t k = 0; k < OX_SORT_ITEMS; k++) {
        const uint32_t q = A + k * OX_T + tid;
        if (k * OX_T + tid >= span) continue;
        const uint32_t sid = ox.head_scan[q] - 1u;
        if (ox.seg_start[sid + 1] - ox.seg_start[sid] > OX_LIGHT || ox.seg_mode[sid] == SM_XFLOW) continue;
        const uint32_t o = ox.s_origin[q];
        if (o == SF_ORIGIN_NONE) continue;
        bool fresh;
        const uint32_t p = ox_lds_insert(kk, ((unsigned long long)(sid - sA + 1u) << 32) | o, &fresh);
        if (fresh) { const uint32_t r = atomicAdd(&nu, 1u); krank[p] = (uint16_t)r; rpos[r] = (uint16_t)p; }
        kp[k] = p;
        any = true;
    }
    if (__syncthreads_or(any) == 0) return;
    uint32_t mine = 0;
#pragma unroll
    for (uint32_t k = 0; k < OX_SORT_ITEMS; k++)
        if (kp[k] != XNONE) { key8[k] = ((uint32_t)krank[kp[k]] << 11) | (k * OX_T + tid); mine++; }
    if (mine) atomicAdd(&nev, mine);
    // each pair's events, in time order: sort by (rank, position)
    OxBlockSort().sort(key8, sort_tmp, 0, 22);
#pragma unroll
    for (uint32_t k = 0; k < OX_SORT_ITEMS; k++) sorted[tid * OX_SORT_ITEMS + k] = key8[k];
    if (tid == 0) { pbase = atomicAdd(&ox.cnt[OXC_PAIRS], nu); lbase = atomicAdd(&ox.cnt[OXC_PLIST], nev); }
    __syncthreads();
    for (uint32_t i = tid; i < nev; i += OX_T) {
        const uint32_t k = sorted[i], r = k >> 11, q = A + (k & 2047u);
        if (lbase + i < ox.plist_cap) ox.plist[lbase + i] = q;
        if (i == 0 || (sorted[i - 1] >> 11) != r) {           // the pair's first event: its record
            uint32_t e = i + 1;
            while (e < nev && (sorted[e] >> 11) == r) e++;
            const unsigned long long key = kk[rpos[r]];
            if (pbase + r < ox.pairs_cap && lbase + e <= ox.plist_cap)
                ox.pairs[pbase + r] = make_uint4(ox.seg_res[sA + (uint32_t)(key >> 32) - 1u], lbase + i, lbase + e,
                                                 (uint32_t)key);
            else atomicOr(&ox.cnt[OXC_OVERFLOW], 4u);
        }
    }
}

// k_ox_lfind: one thread per pair of k_ox_ilight's list (grid-stride): the
// pair's origin node in the index table, or a new pool slot for it.  The
// pairs are distinct keys (a resource's segment lies in one k_ox_ilight block,
// which lists each of its origins once), so no two threads insert the same
// key; a thread reserves room first (OXC_RESERVED against the load limit, as
// in ox_resolve), then claims an empty slot (high word | AX_CLAIM), takes a
// pool slot and publishes -- all in the same loop iteration, so a lane that
// meets a claimed slot of its own resource (another origin being inserted)
// only ever waits for a claimer that is not waiting itself.  Writes the pool
// slot over the record's resource (XNONE when unresolved: overflow, the host
// grows the table and the sort-phase passes run again).
// one pair's lookup / insert from its home slot (the general path)
__device__ uint32_t ox_lf_slow(const ParamTable& t, const DevState& st, uint32_t* cnt, uint32_t lim, uint64_t khi,
                               uint64_t klo) {
    const uint64_t reach = t.mask < PT_MAX_PROBE ? t.mask : PT_MAX_PROBE;
    uint64_t i = ParamTable::hash(khi, klo) & t.mask;
    uint32_t a = XNONE;
    bool reserved = false, done = false;
    for (uint64_t probe = 0; !done;) {
        ParamSlot& s = t.slots[i];
        const uint64_t h = __hip_atomic_load(&s.hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (h == 0) {
            if (!reserved) {
                if (atomicAdd(&cnt[OXC_RESERVED], 1u) >= lim) { atomicOr(&cnt[OXC_OVERFLOW], 1u); done = true; continue; }
                reserved = true;
            }
            unsigned long long expected = 0;
            if (__hip_atomic_compare_exchange_strong((unsigned long long*)&s.hi, &expected,
                                                     (unsigned long long)(khi | AX_CLAIM), __ATOMIC_ACQUIRE,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                a = atomicAdd(st.ax_count, 1u);
                s.lo = klo; s.a = a; s.b = 0;
                __hip_atomic_store(&s.hi, khi, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                done = true;
            }
            continue;                                   // lost the race: this slot again
        }
        if (h == (khi | AX_CLAIM)) continue;            // same resource, another origin being published
        if (h == khi) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");    // (the publisher's lo / a before its release of hi)
            if (s.lo == klo) { a = (uint32_t)s.a; done = true; continue; }
        }
        i = (i + 1) & t.mask;
        if (++probe > reach) { atomicOr(&cnt[OXC_OVERFLOW], 1u); done = true; }
    }
    return a;
}

// Each thread takes LF_B pairs at a time and probes them together (their
// loads in flight at once); a pair found within LF_STEPS slots of its home
// costs one acquire fence shared by the thread's pairs, the rest (absent
// keys, claims in progress, long chains) take ox_lf_slow.
constexpr int LF_B = 4, LF_STEPS = 6;
__global__ void __launch_bounds__(256) k_ox_lfind(DevState st, uint4* pairs, uint32_t* cnt, uint32_t lim) {
    ParamTable t{st.xtab, st.xcap_mask, st.err};
    const uint32_t np = min(cnt[OXC_PAIRS], 0xffffffffu);
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t q0 = blockIdx.x * blockDim.x + threadIdx.x; q0 < np; q0 += stride * LF_B) {
        uint64_t khi[LF_B], klo[LF_B], pos[LF_B];
        uint32_t a[LF_B];
        int state[LF_B];                                // 0 probing, 1 candidate at pos, 2 slow path, 3 unused
#pragma unroll
        for (int k = 0; k < LF_B; k++) {
            const uint32_t q = q0 + (uint32_t)k * stride;
            a[k] = XNONE;
            if (q >= np) { state[k] = 3; khi[k] = klo[k] = pos[k] = 0; continue; }
            const uint4 pr = pairs[q];
            khi[k] = pkey_hi(pr.x, PK_AUX, AX_ORIGIN, 0); klo[k] = pr.w;
            pos[k] = ParamTable::hash(khi[k], klo[k]) & t.mask;
            state[k] = 0;
        }
        for (int step = 0; step < LF_STEPS; step++) {
            uint64_t h[LF_B];
#pragma unroll
            for (int k = 0; k < LF_B; k++)
                h[k] = state[k] == 0 ? __hip_atomic_load(&t.slots[pos[k]].hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : 0ull;
            bool more = false;
#pragma unroll
            for (int k = 0; k < LF_B; k++) {
                if (state[k] != 0) continue;
                if (h[k] == khi[k]) state[k] = 1;
                else if (h[k] == 0 || (h[k] & AX_CLAIM)) state[k] = 2;
                else { pos[k] = (pos[k] + 1) & t.mask; more = true; }
            }
            if (!more) break;
        }
        bool cand = false;
#pragma unroll
        for (int k = 0; k < LF_B; k++) {
            if (state[k] == 0) state[k] = 2;            // (a long chain)
            cand |= state[k] == 1;
        }
        if (cand) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // (the publishers' lo / a before hi)
#pragma unroll
        for (int k = 0; k < LF_B; k++) {
            if (state[k] != 1) continue;
            const ParamSlot& s = t.slots[pos[k]];
            if (s.lo == klo[k]) a[k] = (uint32_t)s.a;
            else state[k] = 2;                          // same resource, another origin: on from its home
        }
#pragma unroll
        for (int k = 0; k < LF_B; k++) {
            if (state[k] == 2) a[k] = ox_lf_slow(t, st, cnt, lim, khi[k], klo[k]);
            if (state[k] != 3) pairs[q0 + (uint32_t)k * stride].x = a[k];
        }
    }
}

// k_ox_index: one workgroup per OX_ITILE sorted events of the long segments and
// of the xflow walk's segments (the light ones are k_ox_ilight's).  Long
// segments: the pairs' slots (s_oslot) and a dense id per pair for the
// window sums; xflow segments: every node key the walk will look up (the
// origin node of every entry with an origin, the context node while a CHAIN
// rule names the context: decide_xgroup's want_on / want_dn).
__global__ void __launch_bounds__(OX_T) k_ox_index(DevState st, DevBatch b, OxIdx ox, uint32_t lim) {
    __shared__ unsigned long long kk[OX_IKCAP];
    __shared__ uint32_t kslot[OX_IKCAP];
    __shared__ uint8_t kheavy[OX_IKCAP];
    __shared__ uint32_t sh[4], bfl;
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < OX_IKCAP; k += OX_T) { kk[k] = 0; kslot[k] = XNONE; kheavy[k] = 0; }
    if (tid == 0) bfl = 0;
    __syncthreads();
    const uint32_t j0 = blockIdx.x * OX_ITILE, j1 = min(b.n, j0 + OX_ITILE);
    if (tid == 0 && j0 % OX_TILE == 0) {                  // the decide phase's segment range of this OX_TILE block
        const uint32_t je = min(b.n, j0 + OX_TILE);
        ox.bseg[j0 / OX_TILE] = make_uint2(ox.head_scan[j0] - 1u, ox.head_scan[je - 1] - 1u);
    }
    bool any = false;
    constexpr uint32_t PER = OX_ITILE / OX_T;
    uint32_t kp[PER];                                     // LDS key position of each of this thread's long-segment events
    // the loads of all PER events first (in flight together), then the inserts
    uint32_t sidv[PER], lov[PER], hiv[PER], ov[PER], resv[PER];
    uint8_t modev[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        const uint32_t j = j0 + k * OX_T + tid;
        sidv[k] = j < j1 ? ox.head_scan[j] - 1u : XNONE;
        ov[k] = (j < j1 && ox.s_origin) ? ox.s_origin[j] : SF_ORIGIN_NONE;
    }
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        const uint32_t sid = sidv[k];
        if (sid == XNONE) { lov[k] = hiv[k] = resv[k] = 0; modev[k] = 0; continue; }
        lov[k] = ox.seg_start[sid]; hiv[k] = ox.seg_start[sid + 1];
        modev[k] = ox.seg_mode[sid]; resv[k] = ox.seg_res[sid];
    }
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        const uint32_t j = j0 + k * OX_T + tid;
        kp[k] = XNONE;
        if (j >= j1) continue;
        const uint32_t lo = lov[k], hi = hiv[k];
        const bool xf = modev[k] == SM_XFLOW;
        if (!xf && hi - lo <= OX_LIGHT) continue;          // (k_ox_ilight)
        const uint32_t o = ov[k];
        bool fresh;
        if (xf) {
            ox.s_oslot[j] = XNONE;
            const uint32_t i = ox.perm[j];
            const uint32_t l = b.res[i] / st.shard_count;
            if (o != SF_ORIGIN_NONE) { ox_lds_insert<OX_IKCAP>(kk, ox_pack(l, AX_ORIGIN, o), &fresh); any = true; }
            const uint32_t ctx = b.ctx ? b.ctx[i] : 0u;
            bool want = false;
            for (uint32_t r = st.rule_off[l]; r < st.rule_off[l + 1]; r++)
                if (st.rules[r].strategy == SF_STRATEGY_CHAIN && st.rules[r].ref == ctx) want = true;
            if (want) { ox_lds_insert<OX_IKCAP>(kk, ox_pack(l, AX_CTX, ctx), &fresh); any = true; }
        } else if (o != SF_ORIGIN_NONE) {
            const uint32_t p = ox_lds_insert<OX_IKCAP>(kk, ox_pack(resv[k], AX_ORIGIN, o), &fresh);
            if (fresh) kheavy[p] = 1;
            kp[k] = p;
            any = true;
        } else {
            ox.s_oslot[j] = XNONE;
        }
    }
    if (__syncthreads_or(any) == 0) return;
    ox_resolve<OX_IKCAP>(st, ox.cnt, kk, kslot, lim, sh, [&](uint32_t p, uint64_t* hi, uint64_t* lo) {
        const unsigned long long k = kk[p];
        *hi = pkey_hi(ox_l(k), PK_AUX, ox_kind(k), 0);
        *lo = (uint32_t)k;
    });
    // dense ids of the pairs of long segments (k_ox_hacc / k_ox_happly): the
    // first workgroup to swing a slot's hmap entry from XNONE claims it and
    // gives it an id; nothing in this kernel reads hmap, so no one waits
    if (tid == 0) sh[0] = 0;
    __syncthreads();
    for (uint32_t p = tid; p < OX_IKCAP; p += OX_T) {
        const uint32_t a = kslot[p];
        if (!kheavy[p]) continue;
        kheavy[p] = 0;
        if (a == XNONE || (a & KS_CLAIMED)) continue;
        if (a >= ox.hmap_n) { atomicOr(&ox.cnt[OXC_OVERFLOW], 2u); continue; }
        bfl = OXB_HEAVY;
        if (__hip_atomic_load(&ox.hmap[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != XNONE) continue;
        uint32_t expected = XNONE;
        if (__hip_atomic_compare_exchange_strong(&ox.hmap[a], &expected, HX_CLAIM, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            kheavy[p] = 2;
            atomicAdd(&sh[0], 1u);
        }
    }
    __syncthreads();
    if (tid == 0) { if (sh[0]) sh[3] = atomicAdd(&ox.cnt[OXC_HEAVY], sh[0]); sh[0] = 0; }
    __syncthreads();
    for (uint32_t p = tid; p < OX_IKCAP; p += OX_T) {
        if (kheavy[p] != 2) continue;
        const uint32_t hid = sh[3] + atomicAdd(&sh[0], 1u);
        const uint32_t a = kslot[p];
        if (hid < ox.hslot_n) ox.hslot[hid] = a;
        else atomicOr(&ox.cnt[OXC_OVERFLOW], 2u);
        ox.hmap[a] = hid < ox.hslot_n ? hid : XNONE;
    }
    if (tid == 0 && bfl) atomicOr(&ox.bflags[j0 / OX_TILE], bfl);
    // the slot of every event of the long segments
#pragma unroll
    for (uint32_t k = 0; k < OX_ITILE / OX_T; k++)
        if (kp[k] != XNONE) {
            const uint32_t a = kslot[kp[k]];
            ox.s_oslot[j0 + k * OX_T + tid] = (a & KS_CLAIMED) ? XNONE : a;
        }
}

// ------------------------------------------------------------------ decide phase
struct OxRun {
    const uint32_t* seg_start; const uint8_t* seg_mode;
    const int64_t* ts; const int32_t* cnt; const uint8_t* flags; const int64_t* eref; const int64_t* cts;
    const uint8_t* v_status; const uint32_t* s_oslot;
    const uint32_t* hmap; const uint32_t* hslot; OxAcc* acc; int64_t* thr;
    const uint32_t* bflags; const uint2* bseg; const uint4* pairs; const uint32_t* plist;
    uint32_t n; OxWin win;
};

// The origin node of one pair while its events are replayed in time order:
// only the second-window and minute buckets the events touch are held (one of
// each; a move to another slot stores the held one back), the thread count as
// a delta.  Same window rules as NodeWin (sf_decide.h: sec_current with the
// borrow seed of OccupiableBucketLeapArray.resetWindowTo, min_current, the
// throwaway window of LeapArray.java:220-223) for the four adds StatisticSlot
// makes on an origin node -- none reads the borrow array or another bucket,
// so nothing else of the node is loaded.
struct OxNode {
    NodeRows rows;
    Bucket sb; int32_t si = -1; int32_t sdirty = 0; int64_t s_ws = INT64_MIN;
    Bucket mb; int32_t mi = -1; int32_t mdirty = 0; int64_t m_ws = INT64_MIN;
    int64_t dthr = 0;
    int32_t S, wl; int64_t max_rt;
    __device__ void flush_sec() { if (sdirty) { rows.sec[si] = sb; sdirty = 0; } }
    __device__ void flush_min() { if (mdirty) { rows.min[mi] = mb; mdirty = 0; } }
    __device__ bool sec(int64_t t) {
        if (!(t >= s_ws && t < s_ws + (int64_t)wl)) {
            const int64_t q = t / wl;
            s_ws = t - (t - q * wl);
            const int32_t idx = (int32_t)(q % S);
            if (idx != si) { flush_sec(); sb = rows.sec[idx]; si = idx; }
        }
        if (sb.ws == s_ws) return true;
        if (s_ws < sb.ws) return false;                           // throwaway window
        const Borrow br = rows.bor[si];
        const int64_t bp = (br.ws <= s_ws && s_ws < br.ws + wl) ? br.pass : -1;
        sb = fresh_bucket(s_ws, max_rt);
        if (bp >= 0) sb.pass = (int64_t)(int32_t)bp;
        sdirty = 1;
        return true;
    }
    __device__ bool min(int64_t t) {
        if (!(t >= m_ws && t < m_ws + 1000)) {
            const int32_t idx = (int32_t)((t / 1000) % MINUTE);
            m_ws = t - t % 1000;
            if (idx != mi) { flush_min(); mb = rows.min[idx]; mi = idx; }
        }
        if (mb.ws == m_ws) return true;
        if (m_ws < mb.ws) return false;
        mb = fresh_bucket(m_ws, max_rt);
        mdirty = 1;
        return true;
    }
    template <class F> __device__ void add(int64_t t, F f) {
        if (sec(t)) { f(sb); sdirty = 1; }
        if (min(t)) { f(mb); mdirty = 1; }
    }
    __device__ void store() { flush_sec(); flush_min(); if (dthr) *rows.thr = wadd(*rows.thr, dthr); }
};

// StatisticSlot's update of the origin node for sorted event j (verdict known)
__device__ __forceinline__ void ox_apply_event(OxNode& on, const OxRun& r, uint32_t j) {
    const uint8_t v = r.v_status[j], fl = r.flags[j];
    const int64_t t = r.ts[j];
    const int32_t c = r.cnt[j];
    if (fl & SF_EV_EXIT) {                                   // StatisticSlot.exit :139-165 (recordCompleteFor)
        if (v != SF_V_EXIT) return;                          // its entry was blocked: nothing is recorded
        const int64_t ref = r.eref ? r.eref[j] : -1;
        const int64_t cts = ref >= 0 ? r.ts[ref] : (r.cts ? r.cts[j] : t);
        const int64_t rt = t - cts;
        on.add(t, [&](Bucket& b) {                           // StatisticNode.addRtAndSuccess, MetricBucket.addRT
            b.succ = wadd(b.succ, c); b.rt = wadd(b.rt, rt); if (rt < b.min_rt) b.min_rt = rt;
        });
        on.dthr--;
        if (fl & SF_EV_ERROR) on.add(t, [&](Bucket& b) { b.exc = wadd(b.exc, c); });
    } else if (v_blocked(v)) {                               // :102-124 BlockException
        on.add(t, [&](Bucket& b) { b.block = wadd(b.block, c); });
    } else {
        on.dthr++;                                           // pass, or PriorityWaitException (:84-101)
        if (v != SF_V_PRIORITY_WAIT) on.add(t, [&](Bucket& b) { b.pass = wadd(b.pass, c); });
    }
}

// One thread per (resource, origin) pair of a short segment (k_ox_ilight's
// list, k_ox_lfind's slot): the pair's events applied in time order.  No LDS
// and few registers: many wavefronts keep the bucket loads of many pairs in
// flight.
__global__ void __launch_bounds__(256) k_ox_lapply(DevState st, OxRun r, uint32_t npairs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npairs) return;
    const uint4 pr = r.pairs[t];
    if (pr.x == XNONE) return;
    OxNode on;
    on.rows = aux_rows(st, pr.x);
    on.S = st.S; on.wl = st.wl; on.max_rt = st.max_rt;
    for (uint32_t k = pr.y; k < pr.z; k++) ox_apply_event(on, r, r.plist[k]);
    on.store();
}

// ---- long segments: per-window sums
__device__ __forceinline__ unsigned long long ox_minrt_key(int64_t rt) {
    return ~((unsigned long long)rt ^ 0x8000000000000000ull);            // larger key = smaller rt; 0 = none
}
__device__ __forceinline__ int64_t ox_minrt_of(unsigned long long k) {
    return (int64_t)(~k ^ 0x8000000000000000ull);
}

constexpr uint32_t OX_HCAP = 512;                 // LDS (pair, window) rows of a k_ox_hacc block
struct OxRow { unsigned long long key; unsigned long long v[7]; };   // key: pool slot << 32 | window + 1

__device__ __forceinline__ void ox_add_row(unsigned long long* v, const unsigned long long* d) {
    for (int f = 0; f < 6; f++) if (d[f]) atomicAdd(&v[f], d[f]);
    if (d[6]) atomicMax(&v[6], d[6]);
}

// One workgroup per OX_TILE block with events of long origin segments: the
// block's (pair, window) sums in LDS, keyed by pool slot; at the flush each
// row's pair id (hmap) and one set of global atomics.  Rows: the second
// window, the minute window, the thread delta (row W).
__global__ void __launch_bounds__(OX_T) k_ox_hacc(DevState st, OxRun r) {
    __shared__ OxRow rows[OX_HCAP];
    __shared__ uint32_t sst[OX_TILE + 1];        // starts of the segments overlapping the block, then their end
    const uint32_t tid = threadIdx.x;
    const uint32_t j0 = blockIdx.x * OX_TILE;
    if (j0 >= r.n || !(r.bflags[blockIdx.x] & OXB_HEAVY)) return;
    const uint32_t j1 = min(r.n, j0 + OX_TILE);
    const uint2 bs = r.bseg[blockIdx.x];
    const uint32_t nsb = bs.y - bs.x + 1;
    for (uint32_t k = tid; k < OX_HCAP; k += OX_T) {
        rows[k].key = 0;
        for (int f = 0; f < 7; f++) rows[k].v[f] = 0;
    }
    for (uint32_t k = tid; k <= nsb; k += OX_T) sst[k] = r.seg_start[bs.x + k];
    __syncthreads();
    const uint32_t W = r.win.ws + r.win.wm;
    const int64_t b_s = r.win.w0s * st.wl, b_m = r.win.w0m * 1000;
    const uint32_t wl = (uint32_t)st.wl;
    for (uint32_t j = j0 + tid; j < j1; j += OX_T) {
        uint32_t a_ = 0, e_ = nsb;                      // sst[a_] <= j < sst[a_ + 1]
        while (e_ - a_ > 1) { const uint32_t m = (a_ + e_) >> 1; if (sst[m] <= j) a_ = m; else e_ = m; }
        if (sst[a_ + 1] - sst[a_] <= OX_LIGHT || r.seg_mode[bs.x + a_] == SM_XFLOW) continue;
        const uint32_t a = r.s_oslot[j];
        if (a == XNONE) continue;
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
        // (the batch spans less than 2^32 ms: 32-bit window arithmetic)
        const uint32_t wsec = (uint32_t)(t - b_s) / wl, wmin = (uint32_t)(t - b_m) / 1000u;
        for (int kind = 0; kind < 3; kind++) {
            if (kind < 2 && !touch) continue;
            if (kind == 2 && !dthr) continue;
            const uint32_t w = kind == 0 ? wsec : (kind == 1 ? r.win.ws + wmin : W);
            unsigned long long dt[7] = {(unsigned long long)dthr, 0, 0, 0, 0, 0, 0};
            const unsigned long long* dd = kind == 2 ? dt : d;
            const unsigned long long key = ((unsigned long long)a << 32) | (w + 1u);
            uint32_t h = (uint32_t)(mix64(key) & (OX_HCAP - 1));
            bool done = false;
            for (uint32_t p = 0; p < 16 && !done; p++) {
                const unsigned long long prev = atomicCAS(&rows[h].key, 0ull, key);
                if (prev == 0ull || prev == key) { ox_add_row(rows[h].v, dd); done = true; }
                else h = (h + 1) & (OX_HCAP - 1);
            }
            if (!done) {                                  // LDS rows full: straight to the global sums
                const uint32_t hid = r.hmap[a];
                if (kind == 2) atomicAdd((unsigned long long*)&r.thr[hid], (unsigned long long)dthr);
                else ox_add_row(&r.acc[(size_t)hid * W + w].pass, dd);   // (OxAcc fields in v[] order)
            }
        }
    }
    __syncthreads();
    for (uint32_t k = tid; k < OX_HCAP; k += OX_T) {
        const unsigned long long key = rows[k].key;
        if (!key) continue;
        const uint32_t hid = r.hmap[(uint32_t)(key >> 32)], w = (uint32_t)key - 1u;
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
    OxIdx ox{w.head_scan, w.seg_start, w.seg_res, w.seg_mode, w.perm, b.origin ? w.s_origin : nullptr, w.s_oslot,
             w.ox_hmap, (uint32_t)std::min<size_t>(w.ox_hmap_n, 0xffffffffu), w.ox_hslot,
             (uint32_t)std::min<size_t>(w.ox_hslot_n, 0xffffffffu), w.ox_cnt, w.ox_bflags, w.ox_bseg, w.ox_pairs,
             w.ox_pairs_cap, w.ox_plist, w.ox_pairs_cap};
    hipMemsetAsync(w.ox_cnt, 0, 8 * sizeof(uint32_t), s);
    // (reservations start from the table's key count: every pool slot is one key)
    hipMemcpyAsync(w.ox_cnt + OXC_RESERVED, st.ax_count, sizeof(uint32_t), hipMemcpyDeviceToDevice, s);
    hipMemsetAsync(w.ox_bflags, 0, ((size_t)b.n / OX_TILE + 1) * sizeof(uint32_t), s);
    if (b.origin) {
        hipLaunchKernelGGL(k_ox_ilight, dim3(ox_blocks(b.n, OX_LTILE)), dim3(OX_T), 0, s, b, ox);
        const unsigned g = (unsigned)std::min<size_t>(ox_blocks(b.n, 256), 8192);
        hipLaunchKernelGGL(k_ox_lfind, dim3(g), dim3(256), 0, s, st, w.ox_pairs, w.ox_cnt, lim);
    }
    hipLaunchKernelGGL(k_ox_index, dim3(ox_blocks(b.n, OX_ITILE)), dim3(OX_T), 0, s, st, b, ox, lim);
    return hipGetLastError();
}

hipError_t launch_ox_apply(const DevState& st, Work& w, const DevBatch& b, uint32_t n_heavy, uint32_t n_pairs,
                           const OxWin& win, hipStream_t s) {
    if (!b.n) return hipSuccess;
    OxRun r{};
    r.seg_start = w.seg_start; r.seg_mode = w.seg_mode;
    r.ts = w.s_ts; r.cnt = w.s_cnt; r.flags = w.s_flags;
    r.eref = b.eref ? w.s_eref : nullptr; r.cts = b.eref ? w.s_cts : nullptr;
    r.v_status = w.v_status; r.s_oslot = w.s_oslot;
    r.hmap = w.ox_hmap; r.hslot = w.ox_hslot; r.acc = (OxAcc*)w.ox_acc; r.thr = w.ox_thr;
    r.bflags = w.ox_bflags; r.bseg = w.ox_bseg; r.pairs = w.ox_pairs; r.plist = w.ox_plist;
    r.n = b.n; r.win = win;
    if (n_pairs) {
        hipLaunchKernelGGL(k_ox_lapply, dim3(ox_blocks(n_pairs, 256)), dim3(256), 0, s, st, r, n_pairs);
    }
    if (n_heavy) {
        const size_t W = (size_t)win.ws + win.wm;
        hipMemsetAsync(w.ox_acc, 0, (size_t)n_heavy * W * sizeof(OxAcc), s);
        hipMemsetAsync(w.ox_thr, 0, (size_t)n_heavy * sizeof(int64_t), s);
        hipLaunchKernelGGL(k_ox_hacc, dim3(ox_blocks(b.n, OX_TILE)), dim3(OX_T), 0, s, st, r);
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
    // a key is never placed farther than PT_MAX_PROBE from its home slot (the
    // probes of find / insert stop there): past it the host grows the table again
    const uint64_t reach = mask < PT_MAX_PROBE ? mask : PT_MAX_PROBE;
    for (uint64_t p = 0; p <= reach; p++) {
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
