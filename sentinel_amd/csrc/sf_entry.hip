// sf_entry.hip — ENTRY_NODE aggregate and the per-second metric snapshot
// (product code).
//
// ENTRY_NODE (Constants.java:66) is the ClusterNode that StatisticSlot
// updates for every EntryType.IN event (StatisticSlot.java:64-123 entry,
// :139-165 exit).  Its windows only ever see adds, so after a time-ordered
// batch each bucket slot holds the latest window with IN activity in its
// residue class, with that window's sums: one pass finds the latest window per
// slot (atomicMax), one reduces the contributions of exactly those windows
// (LDS first, then global atomics; all integer, order-independent), one merges
// them into the state with LeapArray.currentWindow's reset rule.
//
// The snapshot is StatisticNode.metrics() (StatisticNode.java:120-151) over
// every resource with a node, as MetricTimerListener.run calls it
// (MetricTimerListener.java:40-69): currentWindow(now) of the minute window,
// then every valid bucket with timestamp in (lastFetchTime, now - now % 1000)
// and some non-zero counter, in bucket-slot order; lastFetchTime advances.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "sf_sysx.h"

namespace sf {

constexpr int EN_T = 256, EN_PER = 16;          // a workgroup reduces 4096 consecutive events
constexpr int EN_K = 8;                           // LDS rows per workgroup (windows after its first)

struct EnEvent { bool touch, pass, block; int thr; int64_t c, t, rt; bool err; };

// StatisticSlot's ENTRY_NODE updates of one event (original order; verdict known)
__device__ __forceinline__ EnEvent en_event(const DevBatch& b, const uint8_t* vs, uint32_t i) {
    EnEvent e{};
    const uint8_t f = b.flags[i];
    if (!(f & SF_EV_IN)) return e;
    const uint8_t v = vs[i];
    e.c = b.cnt[i];
    e.t = b.ts[i];
    if (!(f & SF_EV_EXIT)) {
        e.pass = v == SF_V_PASS || v == SF_V_PASS_WAIT;
        e.block = v_blocked(v);
        e.touch = e.pass || e.block;                                 // PriorityWait: thread only
        e.thr = (e.pass || v == SF_V_PRIORITY_WAIT) ? 1 : 0;
    } else if (v == SF_V_EXIT) {
        const int64_t ref = b.eref ? b.eref[i] : -1;              // batch index (view-local: ref - base)
        const int64_t cts = ref >= 0 ? b.ts[ref - b.base] : (b.cts ? b.cts[i] : e.t);
        e.touch = true; e.rt = e.t - cts; e.err = (f & SF_EV_ERROR) != 0; e.thr = -1;
    }
    return e;
}

struct EnPart {                 // one lane's sums for one window
    long long key;              // window row, -1 none
    unsigned long long v[6]; long long minrt;
    __device__ void clear(long long k) { key = k; for (int i = 0; i < 6; i++) v[i] = 0; minrt = INT64_MAX; }
    __device__ void add(const EnEvent& e) {
        const unsigned long long c = (unsigned long long)e.c;
        v[5]++;
        if (e.pass) v[0] += c;
        else if (e.block) v[1] += c;
        else {
            v[2] += c; v[3] += (unsigned long long)e.rt;
            if (e.err) v[4] += c;
            if (e.rt < minrt) minrt = e.rt;
        }
    }
};

__device__ __forceinline__ void en_global(unsigned long long (*tbl)[6], long long* mr, unsigned int* overflow,
                                          const EnPart& p) {
    if (p.key < 0 || !p.v[5]) return;
    if (p.key >= (long long)EN_TBL) { atomicOr(overflow, 1u); return; }
    for (int i = 0; i < 6; i++) if (p.v[i]) atomicAdd(&tbl[p.key][i], p.v[i]);
    if (p.minrt != INT64_MAX) atomicMin(&mr[p.key], p.minrt);
}

// lane partial -> workgroup LDS rows (wave-combined when the whole wave shares the row)
__device__ void en_flush(EnPart& p, long long row0, unsigned long long (*lt)[6], long long* lmr,
                         unsigned long long (*gt)[6], long long* gmr, unsigned int* overflow) {
    const bool act = p.key >= 0 && p.v[5];
    const unsigned long long m = __ballot(act);
    if (!m) return;
    const int lane = (int)(threadIdx.x & 63);
    const int l0 = __ffsll((long long)m) - 1;
    const long long k0 = __shfl(p.key, l0);
    if (__ballot(act && p.key != k0) == 0) {
        EnPart r;
        r.key = k0;
        for (int i = 0; i < 6; i++) {
            unsigned long long x = act ? p.v[i] : 0;
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
            r.v[i] = x;
        }
        long long mn = act ? p.minrt : INT64_MAX;
        for (int o = 32; o > 0; o >>= 1) { const long long y = __shfl_xor(mn, o); mn = y < mn ? y : mn; }
        r.minrt = mn;
        if (lane != l0) return;
        p = r;
    } else if (!act) {
        return;
    }
    const long long lr = p.key - row0;
    if (lr >= 0 && lr < EN_K) {
        for (int i = 0; i < 6; i++) if (p.v[i]) atomicAdd(&lt[lr][i], p.v[i]);
        if (p.minrt != INT64_MAX) atomicMin(&lmr[lr], p.minrt);
    } else {
        en_global(gt, gmr, overflow, p);
    }
}

__global__ void __launch_bounds__(EN_T) k_entry_acc(DevState st, DevBatch b, const uint8_t* vs, EntryAcc* acc) {
    __shared__ unsigned long long ls[EN_K][6], lm[EN_K][6];
    __shared__ long long lrs[EN_K], lrm[EN_K], lthr;
    for (int i = threadIdx.x; i < EN_K * 6; i += EN_T) { ls[i / 6][i % 6] = 0; lm[i / 6][i % 6] = 0; }
    for (int i = threadIdx.x; i < EN_K; i += EN_T) { lrs[i] = INT64_MAX; lrm[i] = INT64_MAX; }
    if (threadIdx.x == 0) lthr = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * (EN_T * EN_PER);
    const int64_t W0s = b.ts[0] / st.wl, W0m = b.ts[0] / 1000;
    const uint32_t first = min(base, b.n - 1);
    const long long r0s = b.ts[first] / st.wl - W0s, r0m = b.ts[first] / 1000 - W0m;
    EnPart ps, pm;
    ps.clear(-1); pm.clear(-1);
    long long thr = 0;
    // coalesced; a workgroup's 4096 consecutive events span few windows (time order),
    // so a lane's window key rarely changes.  Window indices by 32-bit division of the
    // offset from the batch's first window when the batch spans < 2^32 ms.
    const int64_t base_s = W0s * st.wl, base_m = W0m * 1000;
    const bool span32 = b.ts[b.n - 1] - base_m < (int64_t)0xffffffffLL;
    for (int k = 0; k < EN_PER; k++) {
        const uint32_t i = base + (uint32_t)(k * EN_T) + threadIdx.x;
        if (i >= b.n) break;
        const EnEvent e = en_event(b, vs, i);
        thr += e.thr;
        if (!e.touch) continue;
        long long ks, km;
        if (span32) {
            ks = (long long)((uint32_t)(e.t - base_s) / (uint32_t)st.wl);
            km = (long long)((uint32_t)(e.t - base_m) / 1000u);
        } else {
            ks = e.t / st.wl - W0s; km = e.t / 1000 - W0m;
        }
        if (ks != ps.key) { en_global(acc->sec, acc->minrt_sec, &acc->overflow, ps); ps.clear(ks); }
        if (km != pm.key) { en_global(acc->min, acc->minrt_min, &acc->overflow, pm); pm.clear(km); }
        ps.add(e); pm.add(e);
    }
    en_flush(ps, r0s, ls, lrs, acc->sec, acc->minrt_sec, &acc->overflow);
    en_flush(pm, r0m, lm, lrm, acc->min, acc->minrt_min, &acc->overflow);
    for (int o = 32; o > 0; o >>= 1) thr += __shfl_xor(thr, o);
    if ((threadIdx.x & 63) == 0 && thr) atomicAdd((unsigned long long*)&lthr, (unsigned long long)thr);
    __syncthreads();
    for (int i = threadIdx.x; i < EN_K * 6; i += EN_T) {
        const int r = i / 6, f = i % 6;
        if (ls[r][f] && r0s + r < (long long)EN_TBL) atomicAdd(&acc->sec[r0s + r][f], ls[r][f]);
        if (lm[r][f] && r0m + r < (long long)EN_TBL) atomicAdd(&acc->min[r0m + r][f], lm[r][f]);
        if ((ls[r][f] && r0s + r >= (long long)EN_TBL) || (lm[r][f] && r0m + r >= (long long)EN_TBL))
            atomicOr(&acc->overflow, 1u);
    }
    for (int r = threadIdx.x; r < EN_K; r += EN_T) {
        if (lrs[r] != INT64_MAX && r0s + r < (long long)EN_TBL) atomicMin(&acc->minrt_sec[r0s + r], lrs[r]);
        if (lrm[r] != INT64_MAX && r0m + r < (long long)EN_TBL) atomicMin(&acc->minrt_min[r0m + r], lrm[r]);
    }
    if (threadIdx.x == 0 && lthr) atomicAdd((unsigned long long*)&acc->threads, (unsigned long long)lthr);
}

// merge one reduced window into a state bucket (LeapArray.currentWindow reset rule;
// ENTRY_NODE never borrows, so a reset bucket starts empty)
__device__ void en_merge(Bucket& bk, int64_t ws, const unsigned long long* sums, long long minrt, int64_t max_rt) {
    if (bk.ws != ws) {
        if (ws < bk.ws) return;                 // older than the slot: a throwaway window (lost adds)
        bk = fresh_bucket(ws, max_rt);
    }
    bk.pass = wadd(bk.pass, (int64_t)sums[0]); bk.block = wadd(bk.block, (int64_t)sums[1]);
    bk.succ = wadd(bk.succ, (int64_t)sums[2]); bk.rt = wadd(bk.rt, (int64_t)sums[3]); bk.exc = wadd(bk.exc, (int64_t)sums[4]);
    if (minrt < bk.min_rt) bk.min_rt = minrt;
}




__global__ void k_entry_apply_if(DevState st, DevBatch b, EntryNode* en, EntryAcc* acc, const uint8_t* vs) {
    if (acc->overflow) {
        if (threadIdx.x == 0) {
            // rare: a batch over more than EN_TBL windows; exact replay in time order
            for (uint32_t i = 0; i < b.n; i++) {
                const EnEvent e = en_event(b, vs, i);
                en->threads = wadd(en->threads, (int64_t)e.thr);
                if (!e.touch) continue;
                unsigned long long sums[5] = {0, 0, 0, 0, 0};
                long long mr = INT64_MAX;
                if (e.pass) sums[0] = (unsigned long long)e.c;
                else if (e.block) sums[1] = (unsigned long long)e.c;
                else { sums[2] = (unsigned long long)e.c; sums[3] = (unsigned long long)e.rt;
                       if (e.err) sums[4] = (unsigned long long)e.c; mr = e.rt; }
                const int64_t ws = e.t / st.wl, wm = e.t / 1000;
                en_merge(en->second[(int)(ws % st.S)], ws * st.wl, sums, mr, st.max_rt);
                en_merge(en->minute[(int)(wm % MINUTE)], wm * 1000, sums, mr, st.max_rt);
            }
        }
        return;
    }
    __shared__ int last_s[SF_MAX_SAMPLE_COUNT], last_m[MINUTE];
    const int i = threadIdx.x;
    const int64_t W0s = b.ts[0] / st.wl, W0m = b.ts[0] / 1000;
    if (i < SF_MAX_SAMPLE_COUNT) last_s[i] = -1;
    if (i < MINUTE) last_m[i] = -1;
    __syncthreads();
    // latest touched window row of each slot's residue class
    for (int r = i; r < (int)EN_TBL; r += blockDim.x) {
        if (acc->sec[r][5]) atomicMax(&last_s[(int)((W0s + r) % st.S)], r);
        if (acc->min[r][5]) atomicMax(&last_m[(int)((W0m + r) % MINUTE)], r);
    }
    __syncthreads();
    if (i < st.S && last_s[i] >= 0) {
        const int r = last_s[i];
        en_merge(en->second[i], (W0s + r) * st.wl, acc->sec[r], acc->minrt_sec[r], st.max_rt);
    }
    if (i < MINUTE && last_m[i] >= 0) {
        const int r = last_m[i];
        en_merge(en->minute[i], (W0m + r) * 1000, acc->min[r], acc->minrt_min[r], st.max_rt);
    }
    if (i == 0) en->threads = wadd(en->threads, (int64_t)acc->threads);
}

__global__ void k_entry_minrt_init(EntryAcc* acc) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < EN_TBL) { acc->minrt_sec[r] = INT64_MAX; acc->minrt_min[r] = INT64_MAX; }
}

__global__ void k_entry_init(EntryNode* en, int64_t max_rt) {
    const int i = threadIdx.x;
    if (i < SF_MAX_SAMPLE_COUNT) en->second[i] = fresh_bucket(WS_NONE, max_rt);
    if (i < MINUTE) en->minute[i] = fresh_bucket(WS_NONE, max_rt);
    if (i == 0) { en->threads = 0; en->last_fetch = -1; }
}

hipError_t launch_entry_init(EntryNode* en, int64_t max_rt, hipStream_t s) {
    hipLaunchKernelGGL(k_entry_init, dim3(1), dim3(64), 0, s, en, max_rt);
    return hipGetLastError();
}

hipError_t launch_entry_node(const DevState& st, const DevBatch& b, const uint8_t* vstatus, EntryNode* en,
                             EntryAcc* acc, hipStream_t s) {
    if (!b.n) return hipSuccess;
    hipMemsetAsync(acc, 0, sizeof(EntryAcc), s);
    hipLaunchKernelGGL(k_entry_minrt_init, dim3((EN_TBL + 255) / 256), dim3(256), 0, s, acc);
    const unsigned nb = (unsigned)((b.n + EN_T * EN_PER - 1) / (EN_T * EN_PER));
    hipLaunchKernelGGL(k_entry_acc, dim3(nb), dim3(EN_T), 0, s, st, b, vstatus, acc);
    hipLaunchKernelGGL(k_entry_apply_if, dim3(1), dim3(256), 0, s, st, b, en, acc, vstatus);
    return hipGetLastError();
}

// ------------------------------------------------------------------ sharded SystemRule exchange (sf_sysx.h)
// a decided view of one plan window: its ENTRY_NODE sums (row 0 of the
// reduction: every event is in the window of the view's first event) as the
// delta words of this rank's next message
__global__ void k_sx_pack(const EntryAcc* acc, int64_t* msg, int64_t key) {
    if (threadIdx.x != 0) return;
    msg[SXD_KEY] = key;
    for (int f = 0; f < 6; f++) { msg[SXD_SEC + f] = (int64_t)acc->sec[0][f]; msg[SXD_MIN + f] = (int64_t)acc->min[0][f]; }
    msg[SXD_MRS] = acc->minrt_sec[0]; msg[SXD_MRM] = acc->minrt_min[0];
    msg[SXD_THR] = acc->threads;
    if (acc->overflow) msg[SXD_KEY] = INT64_MIN;          // (cannot happen: one window)
}
hipError_t launch_entry_delta(const DevState& st, const DevBatch& v, const uint8_t* vstatus, EntryAcc* acc,
                              int64_t* msg, int64_t key, hipStream_t s) {
    if (!v.n) return sx_nodelta(msg, s);
    hipMemsetAsync(acc, 0, sizeof(EntryAcc), s);
    hipLaunchKernelGGL(k_entry_minrt_init, dim3((EN_TBL + 255) / 256), dim3(256), 0, s, acc);
    const unsigned nb = (unsigned)((v.n + EN_T * EN_PER - 1) / (EN_T * EN_PER));
    hipLaunchKernelGGL(k_entry_acc, dim3(nb), dim3(EN_T), 0, s, st, v, vstatus, acc);
    hipLaunchKernelGGL(k_sx_pack, dim3(1), dim3(64), 0, s, acc, msg, key);
    return hipGetLastError();
}

// ------------------------------------------------------------------ node-wide merge (RCCL)
// pack: window start per slot (absent: INT64_MIN) for an all-reduce MAX
__global__ void k_en_pack_ws(const EntryNode* en, int S, int64_t* ws) {
    const int i = threadIdx.x;
    if (i < S) ws[i] = en->second[i].ws == WS_NONE ? INT64_MIN : en->second[i].ws;
    if (i < MINUTE) ws[S + i] = en->minute[i].ws == WS_NONE ? INT64_MIN : en->minute[i].ws;
}
// after the MAX: counters of slots that hold the node-wide latest window (others 0),
// minRt (others INT64_MAX), thread count last
__global__ void k_en_pack_vals(const EntryNode* en, int S, const int64_t* gws, int64_t* vals, int64_t* minrt) {
    const int i = threadIdx.x;
    const int nb = S + MINUTE;
    if (i < nb) {
        const Bucket& b = i < S ? en->second[i] : en->minute[i - S];
        const bool keep = b.ws != WS_NONE && b.ws == gws[i];
        const int64_t v[6] = {b.pass, b.block, b.exc, b.succ, b.rt, b.occ};
        for (int k = 0; k < 6; k++) vals[i * 6 + k] = keep ? v[k] : 0;
        minrt[i] = keep ? b.min_rt : INT64_MAX;
    }
    if (i == 0) vals[nb * 6] = en->threads;
}
hipError_t launch_en_pack_ws(const EntryNode* en, int S, int64_t* ws, hipStream_t s) {
    hipLaunchKernelGGL(k_en_pack_ws, dim3(1), dim3(64), 0, s, en, S, ws);
    return hipGetLastError();
}
hipError_t launch_en_pack_vals(const EntryNode* en, int S, const int64_t* gws, int64_t* vals, int64_t* minrt,
                               hipStream_t s) {
    hipLaunchKernelGGL(k_en_pack_vals, dim3(1), dim3(128), 0, s, en, S, gws, vals, minrt);
    return hipGetLastError();
}

// ------------------------------------------------------------------ snapshot
// one thread per resource; pass 0 counts rows, pass 1 (after an exclusive scan) writes them
__device__ __forceinline__ bool snap_row(const Bucket& b, int64_t now, int64_t last, int64_t cur_sec, sf_metric_row* r) {
    if (b.ws == WS_NONE || wsub(now, b.ws) > 60000) return false;          // list(): valid buckets only
    const int64_t rt = b.succ != 0 ? jdiv(b.rt, b.succ) : b.rt;           // ArrayMetric.fromBucket :199-214
    if (!(b.ws > last && b.ws < cur_sec)) return false;                    // isNodeInTime
    if (!(b.pass > 0 || b.block > 0 || b.succ > 0 || b.exc > 0 || rt > 0 || b.occ > 0)) return false;   // isValidMetricNode
    if (r) {
        r->concurrency = 0; r->timestamp = b.ws;
        r->pass_qps = b.pass; r->block_qps = b.block; r->success_qps = b.succ; r->exception_qps = b.exc;
        r->rt = rt; r->occupied_pass_qps = b.occ;
    }
    return true;
}

template <bool WRITE>
__global__ void k_snapshot(DevState st, int64_t now, uint32_t shard_count, uint32_t shard_index, uint32_t* counts,
                           const uint32_t* offsets, sf_metric_row* out, uint32_t cap) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= st.R) return;
    Bucket* row = st.minute + (size_t)l * MINUTE;
    // a node exists once the resource saw an event: some minute bucket was created
    bool exists = false;
    for (int i = 0; i < MINUTE && !exists; i++) exists = row[i].ws != WS_NONE;
    if (!exists) { if (!WRITE) counts[l] = 0; return; }
    const int64_t cur_sec = now - now % 1000;
    const int64_t last = st.last_fetch[l];
    if (!WRITE) {
        // rollingCounterInMinute.details(): currentWindow(now) first (creates / resets a bucket)
        const int idx = (int)((now / 1000) % MINUTE);
        if (row[idx].ws == WS_NONE || cur_sec > row[idx].ws) row[idx] = fresh_bucket(cur_sec, st.max_rt);
        uint32_t k = 0;
        for (int i = 0; i < MINUTE; i++) k += snap_row(row[i], now, last, cur_sec, nullptr);
        counts[l] = k;
        return;
    }
    uint32_t o = offsets[l];
    int64_t new_last = last;
    for (int i = 0; i < MINUTE; i++) {
        sf_metric_row r;
        if (!snap_row(row[i], now, last, cur_sec, &r)) continue;
        r.resource = l * shard_count + shard_index;
        if (o < cap) out[o] = r;
        o++;
        if (r.timestamp > new_last) new_last = r.timestamp;
    }
    st.last_fetch[l] = new_last;
}

__global__ void k_snapshot_total(const uint32_t* counts, const uint32_t* offsets, uint32_t R, uint32_t* total) {
    *total = R ? offsets[R - 1] + counts[R - 1] : 0;
}

hipError_t launch_snapshot(const DevState& st, int64_t now, uint32_t shard_count, uint32_t shard_index,
                           uint32_t* counts, uint32_t* offsets, sf_metric_row* out, uint32_t cap, uint32_t* total,
                           void* scan_tmp, size_t scan_bytes, hipStream_t s) {
    const unsigned T = 256, nb = (unsigned)((st.R + T - 1) / T);
    hipLaunchKernelGGL(k_snapshot<false>, dim3(nb), dim3(T), 0, s, st, now, shard_count, shard_index, counts,
                       (const uint32_t*)nullptr, out, cap);
    hipError_t e = rocprim::exclusive_scan(scan_tmp, scan_bytes, counts, offsets, 0u, (size_t)st.R,
                                           rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_snapshot_total, dim3(1), dim3(1), 0, s, counts, offsets, st.R, total);
    hipLaunchKernelGGL(k_snapshot<true>, dim3(nb), dim3(T), 0, s, st, now, shard_count, shard_index, counts, offsets,
                       out, cap);
    return hipGetLastError();
}

}  // namespace sf
