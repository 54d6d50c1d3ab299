// sf_metric.hip — metrics.log on the GPU: one MetricTimerListener.run over a
// shard's ClusterNodes (and ENTRY_NODE), formatted as MetricWriter appends it.
//
// Reference: MetricTimerListener.run (CORE/node/metric/MetricTimerListener.java:40-69)
// calls StatisticNode.metrics() (CORE/node/StatisticNode.java:120-151) on every
// ClusterNode and on Constants.ENTRY_NODE, groups the rows by second in a
// TreeMap and hands each second to MetricWriter.write (MetricWriter.java:120-170),
// which appends MetricNode.toFatString (MetricNode.java:213-229) per row.
//
// Pipeline (HBM-bound byte work, no MFMA):
//   k_mlog_count  one wavefront per node: lane i holds minute bucket i (the
//                 node's 60 x 64 B row read once, coalesced), rolls the current
//                 bucket (ArrayMetric.details -> currentWindow), ballots the rows
//                 metrics() keeps -> 64-bit mask + count
//   exclusive scan of the counts
//   k_mlog_rows   one wavefront per node with rows: each valid lane writes its
//                 row at offset + rank-in-mask, a 6-bit second key, advances
//                 lastFetchTime (wave max)
//   radix sort (key = second, 6 bits, stable): TreeMap order, nodes in id order
//   k_fmt<false>  line length per row; exclusive scan (u64) -> line offsets
//   k_fmt<true>   each lane writes its line
// Algorithmic bytes: 3840 B per node (the 60-bucket minute row metrics() walks)
// + 64 B per row + the log bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "sf_decide.h"
#include "sf_internal.h"

namespace sf {

// StatisticNode.metrics filters of one bucket (isNodeInTime :144-146,
// isValidMetricNode :148-151) on ArrayMetric.fromBucket's values (:199-214)
__device__ __forceinline__ bool mlog_keep(const Bucket& b, int64_t now, int64_t last, int64_t cur_sec) {
    if (b.ws == WS_NONE || wsub(now, b.ws) > 60000) return false;        // LeapArray.list(): deprecated dropped
    const int64_t rt = b.succ != 0 ? jdiv(b.rt, b.succ) : b.rt;
    if (!(b.ws > last && b.ws < cur_sec)) return false;
    return b.pass > 0 || b.block > 0 || b.succ > 0 || b.exc > 0 || rt > 0 || b.occ > 0;
}

struct MlogNodes {
    DevState st;
    EntryNode* en;
    uint32_t nodes;          // st.R (+1 with ENTRY_NODE as node st.R)
    uint32_t shard_count, shard_index;
    __device__ Bucket* row(uint32_t l) const { return l < st.R ? st.minute + (size_t)l * MINUTE : en->minute; }
    __device__ int64_t* last(uint32_t l) const { return l < st.R ? st.last_fetch + l : &en->last_fetch; }
    __device__ uint32_t id(uint32_t l) const { return l < st.R ? l * shard_count + shard_index : SF_RES_ENTRY_NODE; }
};

__device__ __forceinline__ uint32_t wave_id() { return (blockIdx.x * blockDim.x + threadIdx.x) >> 6; }
__device__ __forceinline__ uint32_t n_waves() { return (gridDim.x * blockDim.x) >> 6; }

__global__ void __launch_bounds__(256) k_mlog_count(MlogNodes m, int64_t now, unsigned long long* mask,
                                                    uint32_t* counts) {
    const int lane = (int)(threadIdx.x & 63);
    const int64_t cur_sec = now - now % 1000;
    const int idx = (int)((now / 1000) % MINUTE);
    for (uint32_t l = wave_id(); l < m.nodes; l += n_waves()) {
        Bucket* row = m.row(l);
        Bucket b;
        b.ws = WS_NONE;
        if (lane < MINUTE) b = row[lane];
        // a ClusterNode exists once its resource saw an event (some minute bucket
        // was created); ENTRY_NODE always exists (Constants.java:66)
        if (l < m.st.R && __ballot(b.ws != WS_NONE) == 0ull) {
            if (lane == 0) { counts[l] = 0; mask[l] = 0; }
            continue;
        }
        if (lane == idx && (b.ws == WS_NONE || cur_sec > b.ws)) {      // currentWindow(now): create / reset
            b = fresh_bucket(cur_sec, m.st.max_rt);
            row[lane] = b;
        }
        const int64_t last = *m.last(l);
        const unsigned long long k = __ballot(lane < MINUTE && mlog_keep(b, now, last, cur_sec));
        if (lane == 0) { counts[l] = (uint32_t)__popcll(k); mask[l] = k; }
    }
}

__global__ void __launch_bounds__(256) k_mlog_rows(MlogNodes m, int64_t now, const unsigned long long* mask,
                                                   const uint32_t* offsets, sf_metric_row* rows, uint8_t* keys,
                                                   uint32_t* order) {
    const int lane = (int)(threadIdx.x & 63);
    const int64_t cur_sec = now - now % 1000;
    for (uint32_t l = wave_id(); l < m.nodes; l += n_waves()) {
        const unsigned long long k = mask[l];
        if (!k) continue;
        int64_t ws = INT64_MIN;
        if ((k >> lane) & 1ull) {
            const Bucket b = m.row(l)[lane];
            const uint32_t o = offsets[l] + (uint32_t)__popcll(k & ((1ull << lane) - 1ull));
            sf_metric_row r;
            r.resource = m.id(l); r.concurrency = 0; r.timestamp = b.ws;
            r.pass_qps = b.pass; r.block_qps = b.block; r.success_qps = b.succ; r.exception_qps = b.exc;
            r.rt = b.succ != 0 ? jdiv(b.rt, b.succ) : b.rt; r.occupied_pass_qps = b.occ;
            rows[o] = r;
            keys[o] = (uint8_t)(63 - (cur_sec - b.ws) / 1000);          // ascending second (1..60 s back)
            order[o] = o;
            ws = b.ws;
        }
        for (int d = 32; d; d >>= 1) { const int64_t x = __shfl_xor(ws, d); ws = x > ws ? x : ws; }
        if (lane == 0 && ws > *m.last(l)) *m.last(l) = ws;              // newLastFetchTime
    }
}

__global__ void k_mlog_total(const uint32_t* counts, const uint32_t* offsets, uint32_t n, uint32_t* total) {
    *total = n ? offsets[n - 1] + counts[n - 1] : 0;
}

// ---------------------------------------------------------------- formatting
struct NameTab {
    const char* bytes; const uint64_t* off; const int32_t* types; uint32_t n;
};
__device__ const char ENTRY_NAME[] = "__total_inbound_traffic__";   // Constants.TOTAL_IN_RESOURCE_NAME :45
constexpr int ENTRY_NAME_LEN = 25;

__device__ __forceinline__ int dec_len_u(uint64_t v) {
    int n = 1;
    while (v >= 10) { v /= 10; n++; }
    return n;
}
__device__ __forceinline__ int dec_len(int64_t v) {            // Long.toString
    return v < 0 ? 1 + dec_len_u(0ull - (uint64_t)v) : dec_len_u((uint64_t)v);
}
__device__ __forceinline__ char* put_dec(char* p, int64_t v) {
    uint64_t u = (uint64_t)v;
    if (v < 0) { *p++ = '-'; u = 0ull - u; }
    const int n = dec_len_u(u);
    for (int i = n - 1; i >= 0; i--) { p[i] = (char)('0' + u % 10); u /= 10; }
    return p + n;
}
__device__ __forceinline__ char* put_pad(char* p, int64_t v, int w) {    // zero-padded, v >= 0
    const int n = dec_len_u((uint64_t)v);
    for (int i = n; i < w; i++) *p++ = '0';
    return put_dec(p, v);
}

struct Civil { int64_t y, m, d, hh, mm, ss; };
// SimpleDateFormat("yyyy-MM-dd HH:mm:ss") in a fixed zone: proleptic
// Gregorian civil date of the day count
__device__ Civil civil(int64_t t) {
    int64_t days = t / 86400000, msd = t % 86400000;
    if (msd < 0) { msd += 86400000; days--; }
    const int64_t z = days + 719468, era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097, yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100), mp = (5 * doy + 2) / 153;
    Civil c;
    c.d = doy - (153 * mp + 2) / 5 + 1;
    c.m = mp < 10 ? mp + 3 : mp - 9;
    c.y = yoe + era * 400 + (c.m <= 2);
    c.hh = msd / 3600000; c.mm = msd / 60000 % 60; c.ss = msd / 1000 % 60;
    return c;
}
__device__ __forceinline__ int pad_len(int64_t v, int w) { const int n = dec_len_u((uint64_t)v); return n < w ? w : n; }

// name of a row: [p, p + len), its ResourceTypeConstants, and, without a
// loaded name, the decimal id
struct RowName { const char* p; uint32_t len; int32_t cls; bool dec; };
__device__ __forceinline__ RowName row_name(const NameTab& nt, uint32_t res) {
    RowName r{nullptr, 0, 0, false};
    if (res == SF_RES_ENTRY_NODE) { r.p = ENTRY_NAME; r.len = ENTRY_NAME_LEN; return r; }
    if (res < nt.n) {
        r.p = nt.bytes + nt.off[res]; r.len = (uint32_t)(nt.off[res + 1] - nt.off[res]);
        if (nt.types) r.cls = nt.types[res];
        return r;
    }
    r.dec = true; r.len = (uint32_t)dec_len_u(res);
    return r;
}

// MetricNode.toFatString :213-229; WRITE: the line at out + line_off[p]
template <bool WRITE>
__global__ void __launch_bounds__(256) k_fmt(const sf_metric_row* rows, const uint32_t* order, uint32_t n,
                                             NameTab nt, int64_t tz, uint64_t* line_len, const uint64_t* line_off,
                                             char* out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const sf_metric_row r = rows[order ? order[p] : p];
    const Civil c = civil(r.timestamp + tz);
    const RowName nm = row_name(nt, r.resource);
    if (!WRITE) {
        uint64_t len = dec_len(r.timestamp) + 1 + pad_len(c.y, 4) + 15 + 1 + nm.len + 1;
        len += dec_len(r.pass_qps) + dec_len(r.block_qps) + dec_len(r.success_qps) + dec_len(r.exception_qps) +
               dec_len(r.rt) + dec_len(r.occupied_pass_qps) + dec_len(r.concurrency) + dec_len(nm.cls) + 7 + 1;
        line_len[p] = len;
        return;
    }
    char* q = out + line_off[p];
    q = put_dec(q, r.timestamp); *q++ = '|';
    q = put_pad(q, c.y, 4); *q++ = '-'; q = put_pad(q, c.m, 2); *q++ = '-'; q = put_pad(q, c.d, 2); *q++ = ' ';
    q = put_pad(q, c.hh, 2); *q++ = ':'; q = put_pad(q, c.mm, 2); *q++ = ':'; q = put_pad(q, c.ss, 2); *q++ = '|';
    if (nm.dec) q = put_dec(q, (int64_t)r.resource);
    else
        for (uint32_t i = 0; i < nm.len; i++) { const char ch = nm.p[i]; *q++ = ch == '|' ? '_' : ch; }   // replaceAll("\\|", "_")
    *q++ = '|';
    q = put_dec(q, r.pass_qps); *q++ = '|';
    q = put_dec(q, r.block_qps); *q++ = '|';
    q = put_dec(q, r.success_qps); *q++ = '|';
    q = put_dec(q, r.exception_qps); *q++ = '|';
    q = put_dec(q, r.rt); *q++ = '|';
    q = put_dec(q, r.occupied_pass_qps); *q++ = '|';
    q = put_dec(q, r.concurrency); *q++ = '|';
    q = put_dec(q, nm.cls); *q = '\n';
}

__global__ void k_fmt_total(const uint64_t* len, const uint64_t* off, uint32_t n, uint64_t* total) {
    *total = n ? off[n - 1] + len[n - 1] : 0;
}

static inline unsigned grid_for(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

hipError_t mlog_temp_bytes(uint32_t nodes, uint32_t rows, size_t* bytes) {
    size_t a = 0, b = 0, c = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)nodes,
                                           rocprim::plus<uint32_t>());
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(nullptr, b, (uint8_t*)nullptr, (uint8_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, rows, 0u, 6u);
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan(nullptr, c, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, (size_t)rows,
                                rocprim::plus<uint64_t>());
    if (e != hipSuccess) return e;
    *bytes = std::max(a, std::max(b, c));
    return hipSuccess;
}

// pass 1 + scan: counts, masks and row offsets of every node; *total rows
hipError_t launch_mlog_count(const DevState& st, EntryNode* en, bool with_entry, uint32_t shard_count,
                             uint32_t shard_index, int64_t now, unsigned long long* mask, uint32_t* counts,
                             uint32_t* offsets, uint32_t* total, void* tmp, size_t tmp_bytes, unsigned grid,
                             hipEvent_t after_count, hipStream_t s) {
    MlogNodes m{st, en, st.R + (with_entry ? 1u : 0u), shard_count, shard_index};
    hipLaunchKernelGGL(k_mlog_count, dim3(grid), dim3(256), 0, s, m, now, mask, counts);
    if (after_count) hipEventRecord(after_count, s);
    hipError_t e = rocprim::exclusive_scan(tmp, tmp_bytes, counts, offsets, 0u, (size_t)m.nodes,
                                           rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mlog_total, dim3(1), dim3(1), 0, s, counts, offsets, m.nodes, total);
    return hipGetLastError();
}

// pass 2 + second sort: rows in TreeMap order (order_out indexes rows)
hipError_t launch_mlog_rows(const DevState& st, EntryNode* en, bool with_entry, uint32_t shard_count,
                            uint32_t shard_index, int64_t now, const unsigned long long* mask, const uint32_t* offsets,
                            uint32_t n_rows, sf_metric_row* rows, uint8_t* keys, uint8_t* keys_out, uint32_t* order,
                            uint32_t* order_out, void* tmp, size_t tmp_bytes, unsigned grid, hipStream_t s) {
    MlogNodes m{st, en, st.R + (with_entry ? 1u : 0u), shard_count, shard_index};
    hipLaunchKernelGGL(k_mlog_rows, dim3(grid), dim3(256), 0, s, m, now, mask, offsets, rows, keys, order);
    if (!n_rows) return hipGetLastError();
    return rocprim::radix_sort_pairs(tmp, tmp_bytes, keys, keys_out, order, order_out, n_rows, 0u, 6u, s);
}

// line lengths + offsets (*total bytes), then the lines into out (cap checked by the host first)
hipError_t launch_fmt_len(const sf_metric_row* rows, const uint32_t* order, uint32_t n, const char* names,
                          const uint64_t* name_off, const int32_t* types, uint32_t n_names, int64_t tz,
                          uint64_t* line_len, uint64_t* line_off, uint64_t* total, void* tmp, size_t tmp_bytes,
                          hipStream_t s) {
    NameTab nt{names, name_off, types, n_names};
    if (n) {
        hipLaunchKernelGGL(k_fmt<false>, dim3(grid_for(n, 256)), dim3(256), 0, s, rows, order, n, nt, tz, line_len,
                           (const uint64_t*)nullptr, (char*)nullptr);
        hipError_t e = rocprim::exclusive_scan(tmp, tmp_bytes, line_len, line_off, (uint64_t)0, (size_t)n,
                                               rocprim::plus<uint64_t>(), s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_fmt_total, dim3(1), dim3(1), 0, s, line_len, line_off, n, total);
    return hipGetLastError();
}
hipError_t launch_fmt_write(const sf_metric_row* rows, const uint32_t* order, uint32_t n, const char* names,
                            const uint64_t* name_off, const int32_t* types, uint32_t n_names, int64_t tz,
                            const uint64_t* line_off, char* out, hipStream_t s) {
    NameTab nt{names, name_off, types, n_names};
    if (n)
        hipLaunchKernelGGL(k_fmt<true>, dim3(grid_for(n, 256)), dim3(256), 0, s, rows, order, n, nt, tz,
                           (uint64_t*)nullptr, line_off, out);
    return hipGetLastError();
}

}  // namespace sf
