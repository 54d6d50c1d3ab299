// sf_rsort.h — the sort phase's stable radix sort by resource (product code).
//
// Events are sorted by shard-local resource id, stably, so each resource's
// segment keeps the submission (= mocked clock) order LeapArray needs.  An LSD
// radix sort of RS_DB-bit digits, every pass chunked so that no workgroup
// ever waits for another (no decoupled look-back, no spin):
//
//   count  one workgroup per chunk (a contiguous range of the pass input):
//          the chunk's digit histogram -> h[chunk][bin]
//   scan   per bin: exclusive prefix over the chunks (in place), bin totals
//   pass   one workgroup per chunk walks its tiles (W waves x K rows of 64
//          events) in order: each wave ranks its rows by the digit (lanes of
//          one digit found with one ballot per digit bit; a per-wave running
//          count per bin in LDS), the waves' counts are scanned per bin, the
//          tile is placed in LDS in (bin, rank) order and written out by
//          consecutive threads -- every store instruction writes runs of
//          consecutive addresses, one per bin.  An event goes to
//          start[bin] + h[chunk][bin] + (earlier tiles of the chunk) + rank.
//   Ranks follow (tile, wave, row, lane) = input order: the sort is stable.
//
// Pass 0 reads the caller's batch itself (key = shard-local resource id, or
// its xflow group key; the 8-B / 12-B payload of k_keys_packed; the checks of
// the resource's shard and of the clock order), so no key array is written
// before the first pass.  A chunk's tile stream is written by one workgroup on
// one CU, so the partial lines at a bin run's ends are completed by the same
// workgroup's next tile while still in its XCD's L2.
#pragma once
#include "sf_internal.h"

namespace sf {

#ifndef SF_RS_DB
#define SF_RS_DB 8
#endif
#ifndef SF_RS_W
#define SF_RS_W 8
#endif
constexpr int RS_DB = SF_RS_DB, RS_NB = 1 << RS_DB, RS_W = SF_RS_W;
constexpr int RS_T = RS_W * 64;
constexpr uint32_t RS_MAX_CHUNKS = 1024;

// the event's payload (sf_internal.h PackedEv): index, time offset from the
// batch's first event, flags (the planner's forced SystemBlockException and
// AuthoritySlot blocks folded in), acquireCount when it fits in 8 bits
__device__ __forceinline__ uint32_t rs_meta(const DevBatch& b, uint32_t i, int64_t ts, int64_t ts0) {
    const int64_t d = ts - ts0;
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
    return dts | (fl << 16) | (c8 << 24);
}

__device__ __forceinline__ void rs_put_origin(uint32_t*, uint32_t, const PackedEv&) {}
// member-wise copies (a 12-B aggregate copy is lowered to a memcpy that keeps the arrays in scratch)
__device__ __forceinline__ void rs_cp(PackedEv& d, const PackedEv& s) { d.idx = s.idx; d.meta = s.meta; }
__device__ __forceinline__ void rs_cp(PackedEvO& d, const PackedEvO& s) { d.idx = s.idx; d.meta = s.meta; d.origin = s.origin; }
__device__ __forceinline__ void rs_put_origin(uint32_t* o, uint32_t j, const PackedEvO& v) { o[j] = v.origin; }

// pass-0 source: the caller's batch
struct RsBatchSrc {
    DevBatch b;
    uint32_t shard_count, shard_index, R;
    int32_t* err;
    const int64_t* last_ts;
    const uint32_t* xmap;
    static constexpr bool kContig = false;    // random keys: the count reads coalesced, one atomic per event
    __device__ __forceinline__ uint32_t key(uint32_t i, bool check) const {
        const uint32_t r = b.res[i];
        uint32_t l = r;
        bool bad;
        if (shard_count == 1) bad = l >= R;     // (uniform branch: no integer division on one GPU)
        else { l = r / shard_count; bad = r % shard_count != shard_index || l >= R; }
        if (bad) { if (check) *err = SF_ERR_INVALID; l = 0; }
        if (xmap) {                                               // an xflow group is one segment (sf_xflow.h)
            const uint32_t g = xmap[l];
            if (g != XNONE) l = g;
        }
        return l;
    }
    __device__ __forceinline__ void set_origin(PackedEvO& v, uint32_t i) const { v.origin = b.origin[i]; }
    __device__ __forceinline__ void set_origin(PackedEv&, uint32_t) const {}
    template <class V>
    __device__ __forceinline__ void load(uint32_t i, uint32_t& k, V& v) const {
        k = key(i, true);
        const int64_t t = b.ts[i];
        // the mocked clock never goes back: within the batch and across batches
        // (LeapArray would hand such an event a throwaway window)
        if (t < (i ? b.ts[i - 1] : *last_ts)) *err = SF_ERR_INVALID;
        v.idx = i;
        v.meta = rs_meta(b, i, t, b.ts[0]);
        set_origin(v, i);
    }
};
// later passes: the previous pass's output
template <class V>
struct RsArraySrc {
    static constexpr bool kContig = true;     // sorted by the lower digits: runs of equal digits
    const uint32_t* k; const V* v;
    __device__ __forceinline__ uint32_t key(uint32_t i, bool) const { return k[i]; }
    __device__ __forceinline__ void load(uint32_t i, uint32_t& kk, V& vv) const { kk = k[i]; rs_cp(vv, v[i]); }
};

__device__ __forceinline__ uint64_t rs_match(uint32_t d, uint64_t act) {
    uint64_t m = act;
#pragma unroll
    for (int b = 0; b < RS_DB; b++) {
        const uint64_t x = __ballot((d >> b) & 1u);
        m &= ((d >> b) & 1u) ? x : ~x;
    }
    return m;
}

// exclusive scan of RS_NB values held RS_NB / RS_T per thread (or one) through `part`
template <class GET, class PUT>
__device__ __forceinline__ void rs_block_scan(uint32_t* part, GET get, PUT put) {
    constexpr int BPT = RS_NB / RS_T > 0 ? RS_NB / RS_T : 1;
    const int tid = threadIdx.x;
    uint32_t loc[BPT], s = 0;
#pragma unroll
    for (int j = 0; j < BPT; j++) { const int b = tid * BPT + j; loc[j] = b < RS_NB ? get(b) : 0u; s += loc[j]; }
    // wave-inclusive scan of s, then the waves' totals
    const int lane = tid & 63, w = tid >> 6;
    uint32_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) part[w] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (int k = 0; k < w; k++) wbase += part[k];
    uint32_t acc = wbase + x - s;
#pragma unroll
    for (int j = 0; j < BPT; j++) {
        const int b = tid * BPT + j;
        if (b < RS_NB) put(b, acc);
        acc += loc[j];
    }
    __syncthreads();
}

// Each thread counts RS_CE consecutive events and adds a run of equal digits
// with one LDS atomic: the inputs of the later passes are sorted by the lower
// digits, so a wave's lanes would otherwise all hit one counter.
constexpr int RS_CE = 16;
template <class SRC>
__global__ void __launch_bounds__(256) k_rs_count(SRC src, uint32_t n, uint32_t chunk, uint32_t shift, uint32_t mask,
                                                  uint32_t* h) {
    __shared__ uint32_t hist[RS_NB];
    for (int b = threadIdx.x; b < RS_NB; b += 256) hist[b] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    if constexpr (!SRC::kContig) {
        constexpr int U = 8;                                      // 8 coalesced loads in flight per thread
        uint64_t i = lo + threadIdx.x;
        for (; i + (U - 1) * 256 < hi; i += U * 256) {
            uint32_t d[U];
#pragma unroll
            for (int u = 0; u < U; u++) d[u] = (src.key((uint32_t)(i + u * 256), false) >> shift) & mask;
#pragma unroll
            for (int u = 0; u < U; u++) atomicAdd(&hist[d[u]], 1u);
        }
        for (; i < hi; i += 256) atomicAdd(&hist[(src.key((uint32_t)i, false) >> shift) & mask], 1u);
    } else {
        // RS_CE consecutive keys per thread (four 16-B loads; chunks are whole tiles, so
        // every full group is 16-B aligned); a run of equal digits is one atomic
        for (uint64_t i0 = lo + (uint64_t)threadIdx.x * RS_CE; i0 < hi; i0 += 256u * RS_CE) {
            uint32_t d[RS_CE];
            if (i0 + RS_CE <= hi) {
                const uint4* q = (const uint4*)(src.k + i0);
#pragma unroll
                for (int u = 0; u < RS_CE / 4; u++) {
                    const uint4 x = q[u];
                    d[4 * u] = (x.x >> shift) & mask; d[4 * u + 1] = (x.y >> shift) & mask;
                    d[4 * u + 2] = (x.z >> shift) & mask; d[4 * u + 3] = (x.w >> shift) & mask;
                }
            } else {
#pragma unroll
                for (int u = 0; u < RS_CE; u++) d[u] = i0 + u < hi ? (src.k[i0 + u] >> shift) & mask : ~0u;
            }
            uint32_t cur = d[0], run = 1;
#pragma unroll
            for (int u = 1; u < RS_CE; u++) {
                if (d[u] == cur) { run++; continue; }
                if (cur != ~0u) atomicAdd(&hist[cur], run);
                cur = d[u]; run = 1;
            }
            if (cur != ~0u) atomicAdd(&hist[cur], run);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < RS_NB; b += 256) h[(size_t)blockIdx.x * RS_NB + b] = hist[b];
}

// per bin (one workgroup each): exclusive prefix over the chunks (in place),
// the bin's total -- one chunk per thread, a workgroup scan (the chunks of one
// bin are RS_NB words apart: a handful of lines per workgroup, all in flight)
__global__ void __launch_bounds__(RS_MAX_CHUNKS) k_rs_scan(uint32_t* h, uint32_t nchunks, uint32_t* tot) {
    __shared__ uint32_t wsum[RS_MAX_CHUNKS / 64];
    const uint32_t b = blockIdx.x, c = threadIdx.x, lane = c & 63, wv = c >> 6;
    const uint32_t x = c < nchunks ? h[(size_t)c * RS_NB + b] : 0u;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t k = 0; k < wv; k++) base += wsum[k];
    if (c < nchunks) h[(size_t)c * RS_NB + b] = base + inc - x;
    if (c == blockDim.x - 1) tot[b] = base + inc;
}

// rows per wave of a tile: 8 (tile 4096, 48 / 64 KiB of LDS staging for 8-B /
// 12-B payloads: two workgroups per CU; 12 rows with the next tile's loads in
// flight spill registers)
template <class V> struct RsGeom {
    static constexpr int K = 8;
    static constexpr int TILE = RS_W * K * 64;
};

// where a pass puts an event: the key and payload arrays of the next pass
template <class V>
struct RsSinkKV {
    uint32_t* k; V* v;
    __device__ __forceinline__ void put(uint32_t dst, uint32_t key, const V& val) const { k[dst] = key; rs_cp(v[dst], val); }
};
// the last pass: the sorted SoA the decide phase reads (k_unpack's per-event
// part): key, submission index, time, acquireCount, flags, origin, and the
// ParamFlow arguments gathered from the batch
template <class V>
struct RsSinkFinal {
    DevBatch b;
    uint32_t* keys; uint32_t* perm; int64_t* s_ts; int32_t* s_cnt; uint8_t* s_flags;
    uint32_t* s_origin; uint8_t* s_nargs; uint8_t* s_atag; uint64_t* s_abits;
    __device__ __forceinline__ void put(uint32_t j, uint32_t key, const V& val) const {
        keys[j] = key;
        const uint32_t i = val.idx;
        const uint32_t dts = val.meta & 0xffffu, c8 = val.meta >> 24;
        perm[j] = i;
        s_ts[j] = dts != PV_DTS_FAR ? b.ts[0] + (int64_t)dts : b.ts[i];
        s_cnt[j] = c8 ? (int32_t)c8 : b.cnt[i];
        s_flags[j] = (uint8_t)(val.meta >> 16);
        rs_put_origin(s_origin, j, val);
        if (b.arg_slots) {
            if (b.nargs) s_nargs[j] = b.nargs[i];
            for (uint32_t a = 0; a < b.arg_slots; a++) {
                const uint8_t tg = b.atag[(size_t)a * b.arg_stride + i];
                s_atag[(size_t)a * b.n + j] = tg;
                // a collection argument carries its index into the batch's element CSR
                s_abits[(size_t)a * b.n + j] = tg == SF_TAG_COLLECTION ? (uint64_t)a * b.arg_stride + (uint64_t)b.base + i
                                                                      : b.abits[(size_t)a * b.arg_stride + i];
            }
        }
    }
};

// (at most 128 VGPRs: two workgroups of eight waves per CU, as the LDS allows)
template <class SRC, class SINK, class V>
__global__ void __launch_bounds__(RS_T, 4) k_rs_pass(SRC src, SINK sink, uint32_t n, uint32_t chunk, uint32_t shift,
                                                  uint32_t mask, const uint32_t* h, const uint32_t* tot) {
    constexpr int K = RsGeom<V>::K, TILE = RsGeom<V>::TILE;
    __shared__ uint16_t wc[RS_W][RS_NB];     // per-wave running counts, then the waves' exclusive prefixes
    __shared__ uint16_t ttot[RS_NB], tstart[RS_NB];
    __shared__ uint32_t run[RS_NB];          // next global position of each bin for this chunk
    __shared__ uint32_t part[RS_W];
    __shared__ uint32_t skey[TILE];
    __shared__ V sval[TILE];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t* hc = h + (size_t)blockIdx.x * RS_NB;
    rs_block_scan(part, [&](int b) { return tot[b]; }, [&](int b, uint32_t x) { run[b] = x + hc[b]; });
    for (int b = tid; b < RS_NB; b += RS_T) {
#pragma unroll
        for (int x = 0; x < RS_W; x++) wc[x][b] = 0;
    }
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const uint64_t lt = (1ull << lane) - 1ull;
    // the next tile's loads are issued before this tile is ranked and written
    // (a barrier waits for LDS traffic only, so they stay in flight)
    uint32_t nkey[K];
    V nval[K];
    auto fetch = [&](uint64_t t) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t + (uint64_t)(w * K + k) * 64 + lane;
            if (i < hi) src.load((uint32_t)i, nkey[k], nval[k]);
            else nkey[k] = 0;
        }
    };
    fetch(lo);
    for (uint64_t t0 = lo; t0 < hi; t0 += TILE) {
        const uint32_t nt = (uint32_t)(hi - t0 < (uint64_t)TILE ? hi - t0 : (uint64_t)TILE);
        uint32_t key[K];
        V val[K];
        uint16_t rk[K];
#pragma unroll
        for (int k = 0; k < K; k++) { key[k] = nkey[k]; rs_cp(val[k], nval[k]); }
        if (t0 + TILE < hi) fetch(t0 + TILE);
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t0 + (uint64_t)(w * K + k) * 64 + lane;
            const bool ok = i < hi;
            const uint64_t act = __ballot(ok);
            rk[k] = 0;
            if (!act) continue;
            const uint32_t d = (key[k] >> shift) & mask;
            const uint64_t m = rs_match(d, act);
            const uint32_t before = ok ? wc[w][d] : 0u;
            const uint32_t r = (uint32_t)__popcll(m & lt);
            rk[k] = (uint16_t)(before + r);
            if (ok && r == 0) wc[w][d] = (uint16_t)(before + __popcll(m));
        }
        __syncthreads();
        for (int b = tid; b < RS_NB; b += RS_T) {
            uint32_t acc = 0;
#pragma unroll
            for (int x = 0; x < RS_W; x++) { const uint32_t c = wc[x][b]; wc[x][b] = (uint16_t)acc; acc += c; }
            ttot[b] = (uint16_t)acc;
        }
        __syncthreads();
        rs_block_scan(part, [&](int b) { return (uint32_t)ttot[b]; }, [&](int b, uint32_t x) { tstart[b] = (uint16_t)x; });
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t i = t0 + (uint64_t)(w * K + k) * 64 + lane;
            if (i < hi) {
                const uint32_t d = (key[k] >> shift) & mask;
                const uint32_t p = (uint32_t)tstart[d] + wc[w][d] + rk[k];
                skey[p] = key[k];
                rs_cp(sval[p], val[k]);
            }
        }
        __syncthreads();
        for (uint32_t p = tid; p < nt; p += RS_T) {
            const uint32_t kk = skey[p];
            const uint32_t d = (kk >> shift) & mask;
            sink.put(run[d] + (p - tstart[d]), kk, sval[p]);
        }
        __syncthreads();
        for (int b = tid; b < RS_NB; b += RS_T) {
            run[b] += ttot[b];
#pragma unroll
            for (int x = 0; x < RS_W; x++) wc[x][b] = 0;
        }
        __syncthreads();
    }
}

// scratch in bytes: h[RS_MAX_CHUNKS][RS_NB] + tot[RS_NB]
inline size_t rs_scratch_bytes() { return ((size_t)RS_MAX_CHUNKS + 1) * RS_NB * 4; }

// chunk geometry of a pass over n events: C chunks of `chunk` (a whole number of tiles)
template <class V>
inline void rs_chunks(uint32_t n, uint32_t* C, uint32_t* chunk) {
    constexpr uint32_t TILE = RsGeom<V>::TILE;
    uint32_t c = (n + TILE - 1) / TILE;
    if (c > RS_MAX_CHUNKS) c = RS_MAX_CHUNKS;
    uint32_t ch = (n + c - 1) / c;
    ch = (ch + TILE - 1) / TILE * TILE;
    *chunk = ch;
    *C = (n + ch - 1) / ch;
}

template <class SRC, class SINK, class V>
inline void rs_launch_pass(const SRC& src, const SINK& sink, uint32_t n, uint32_t shift, uint32_t mask, void* scratch,
                           hipStream_t s) {
    uint32_t C, chunk;
    rs_chunks<V>(n, &C, &chunk);
    uint32_t* h = (uint32_t*)scratch;
    uint32_t* tot = h + (size_t)RS_MAX_CHUNKS * RS_NB;
    hipLaunchKernelGGL(k_rs_count<SRC>, dim3(C), dim3(256), 0, s, src, n, chunk, shift, mask, h);
    hipLaunchKernelGGL(k_rs_scan, dim3(RS_NB), dim3(RS_MAX_CHUNKS), 0, s, h, C, tot);
    hipLaunchKernelGGL((k_rs_pass<SRC, SINK, V>), dim3(C), dim3(RS_T), 0, s, src, sink, n, chunk, shift, mask,
                       (const uint32_t*)h, (const uint32_t*)tot);
}

// The whole sort of a batch: the last pass writes the sorted SoA (`fin`);
// keys_a / pv_a and keys_b / pv_b are the buffers of the middle passes (pass p
// writes a for even p, b for odd p; the last pass reads the one before, so
// `fin` must not alias the pair it reads).
template <class V>
hipError_t rs_sort(const RsBatchSrc& src, uint32_t n, uint32_t key_bits, uint32_t* keys_a, V* pv_a, uint32_t* keys_b,
                   V* pv_b, const RsSinkFinal<V>& fin, void* scratch, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t kb = key_bits ? key_bits : 1;
    const uint32_t P = (kb + RS_DB - 1) / RS_DB;
    const uint32_t D = (kb + P - 1) / P;                  // digit bits per pass (<= RS_DB)
    const uint32_t mask = (1u << D) - 1u;
    const RsSinkKV<V> sa{keys_a, pv_a}, sb{keys_b, pv_b};
    for (uint32_t p = 0; p < P; p++) {
        const uint32_t shift = p * D;
        const bool last = p + 1 == P;
        const RsSinkKV<V>& mid = (p & 1) ? sb : sa;
        if (p == 0) {
            if (last) rs_launch_pass<RsBatchSrc, RsSinkFinal<V>, V>(src, fin, n, shift, mask, scratch, s);
            else rs_launch_pass<RsBatchSrc, RsSinkKV<V>, V>(src, mid, n, shift, mask, scratch, s);
        } else {
            const RsSinkKV<V>& prev = (p & 1) ? sa : sb;
            const RsArraySrc<V> as{prev.k, prev.v};
            if (last) rs_launch_pass<RsArraySrc<V>, RsSinkFinal<V>, V>(as, fin, n, shift, mask, scratch, s);
            else rs_launch_pass<RsArraySrc<V>, RsSinkKV<V>, V>(as, mid, n, shift, mask, scratch, s);
        }
    }
    return hipGetLastError();
}

}  // namespace sf
