// sf_kernels.hip — gfx950 kernels of one sf_submit (product code).
//
// Pipeline (one HIP stream, no host round trip inside):
//   k_keys      validate + map resource ids to shard-local keys, iota values
//   radix sort  stable (key, index) sort by resource: per-resource time order
//               is the input order (LeapArray semantics need it)
//   k_heads + exclusive scan + k_segments   segment table of touched resources
//   k_gather    events into sorted order (SoA), inverse permutation for EXIT refs
//   k_decide    one lane per resource segment: the exact interpreter (sf_decide.h)
//   k_scatter   verdicts back to submission order
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "sf_decide.h"

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

__global__ void k_keys(DevBatch b, uint32_t* keys, uint32_t* vals, uint32_t shard_count,
                       uint32_t shard_index, uint32_t R, int32_t* err) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    uint32_t r = b.res[i];
    uint32_t l = r / shard_count;
    if (r % shard_count != shard_index || l >= R) { *err = SF_ERR_INVALID; l = 0; }
    keys[i] = l;
    vals[i] = i;
}

__global__ void k_heads(const uint32_t* keys, uint32_t n, uint32_t* head) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    head[j] = (j == 0 || keys[j] != keys[j - 1]) ? 1u : 0u;
}

__global__ void k_segments(const uint32_t* keys, const uint32_t* head, const uint32_t* pos, uint32_t n,
                           uint32_t* seg_start, uint32_t* seg_res, uint32_t* n_seg) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    if (head[j]) { seg_start[pos[j]] = j; seg_res[pos[j]] = keys[j]; }
    if (j == n - 1) { uint32_t ns = pos[j] + head[j]; *n_seg = ns; seg_start[ns] = n; }
}

__global__ void k_gather(DevBatch b, const uint32_t* perm, int64_t* s_ts, int32_t* s_cnt, uint8_t* s_flags,
                         uint32_t* inv, uint8_t* s_nargs, uint8_t* s_atag, uint64_t* s_abits) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= b.n) return;
    uint32_t i = perm[j];
    s_ts[j] = b.ts[i];
    s_cnt[j] = b.cnt[i];
    s_flags[j] = b.flags[i];
    if (inv) inv[i] = j;
    if (b.arg_slots) {
        if (b.nargs) s_nargs[j] = b.nargs[i];
        for (uint32_t a = 0; a < b.arg_slots; a++) {
            s_atag[(size_t)a * b.n + j] = b.atag[(size_t)a * b.n + i];
            s_abits[(size_t)a * b.n + j] = b.abits[(size_t)a * b.n + i];
        }
    }
}

__global__ void k_gather_exit(DevBatch b, const uint32_t* perm, const uint32_t* inv, int64_t* s_eref,
                              int64_t* s_cts, int32_t* err) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= b.n) return;
    uint32_t i = perm[j];
    int64_t r = b.eref[i];
    if (r >= (int64_t)b.n) { *err = SF_ERR_INVALID; r = -1; }
    s_eref[j] = (r >= 0) ? (int64_t)inv[r] : -1;
    s_cts[j] = b.cts ? b.cts[i] : 0;
}

template <int MAXS>
__global__ void __launch_bounds__(128) k_decide(DevState st, SegIO io, const uint32_t* seg_start,
                                                const uint32_t* seg_res, const uint32_t* n_seg) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= *n_seg) return;
    decide_segment<MAXS>(st, io, seg_res[s], seg_start[s], seg_start[s + 1]);
}

__global__ void k_scatter(const uint32_t* perm, uint32_t n, const uint8_t* vs, const int32_t* vw,
                          const uint16_t* vr, DevVerdicts out) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint32_t i = perm[j];
    out.status[i] = vs[j];
    if (out.wait) out.wait[i] = vw[j];
    if (out.rule) out.rule[i] = vr[j];
}

static inline unsigned blocks(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

hipError_t query_temp_bytes(uint32_t max_n, uint32_t key_bits, size_t* sort_bytes, size_t* scan_bytes) {
    hipError_t e = rocprim::radix_sort_pairs(nullptr, *sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, max_n, 0u, key_bits);
    if (e != hipSuccess) return e;
    return rocprim::exclusive_scan(nullptr, *scan_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u,
                                   (size_t)max_n, rocprim::plus<uint32_t>());
}

hipError_t launch_init_state(const DevState& st, hipStream_t s) {
    size_t n_sec = (size_t)st.R * st.S, n_min = (size_t)st.R * MINUTE;
    hipLaunchKernelGGL(k_init_state, dim3(2048), dim3(256), 0, s, st, n_sec, n_min);
    return hipGetLastError();
}

hipError_t launch_pipeline(const DevState& st, Work& w, const DevBatch& b, const DevVerdicts& out,
                           uint32_t shard_count, uint32_t shard_index, uint32_t key_bits,
                           hipStream_t s, hipEvent_t* ev) {
    const uint32_t n = b.n;
    if (n == 0) return hipSuccess;
    const unsigned T = 256;
    if (ev) hipEventRecord(ev[0], s);
    hipLaunchKernelGGL(k_keys, dim3(blocks(n, T)), dim3(T), 0, s, b, w.keys_in, w.vals_in, shard_count,
                       shard_index, st.R, st.err);
    hipError_t e = rocprim::radix_sort_pairs(w.sort_tmp, w.sort_tmp_bytes, w.keys_in, w.keys_out, w.vals_in,
                                             w.perm, n, 0u, key_bits, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_heads, dim3(blocks(n, T)), dim3(T), 0, s, w.keys_out, n, w.head);
    e = rocprim::exclusive_scan(w.scan_tmp, w.scan_tmp_bytes, w.head, w.head_scan, 0u, (size_t)n,
                                rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_segments, dim3(blocks(n, T)), dim3(T), 0, s, w.keys_out, w.head, w.head_scan, n,
                       w.seg_start, w.seg_res, w.n_seg);
    if (ev) hipEventRecord(ev[1], s);
    hipLaunchKernelGGL(k_gather, dim3(blocks(n, T)), dim3(T), 0, s, b, w.perm, w.s_ts, w.s_cnt, w.s_flags,
                       b.eref ? w.inv : nullptr, w.s_nargs, w.s_atag, w.s_abits);
    if (b.eref)
        hipLaunchKernelGGL(k_gather_exit, dim3(blocks(n, T)), dim3(T), 0, s, b, w.perm, w.inv, w.s_eref,
                           w.s_cts, st.err);
    if (ev) hipEventRecord(ev[2], s);
    SegIO io;
    io.ts = w.s_ts; io.cnt = w.s_cnt; io.flags = w.s_flags;
    io.eref = b.eref ? w.s_eref : nullptr; io.cts = b.eref ? w.s_cts : nullptr;
    io.arg_slots = b.arg_slots; io.nargs = (b.arg_slots && b.nargs) ? w.s_nargs : nullptr;
    io.atag = w.s_atag; io.abits = w.s_abits; io.n = n;
    io.v_status = w.v_status; io.v_wait = w.v_wait; io.v_rule = w.v_rule;
    uint32_t max_seg = n < st.R ? n : st.R;
    const unsigned TD = 128;
    if (st.S <= 2)
        hipLaunchKernelGGL(k_decide<2>, dim3(blocks(max_seg, TD)), dim3(TD), 0, s, st, io, w.seg_start,
                           w.seg_res, w.n_seg);
    else
        hipLaunchKernelGGL(k_decide<SF_MAX_SAMPLE_COUNT>, dim3(blocks(max_seg, TD)), dim3(TD), 0, s, st, io,
                           w.seg_start, w.seg_res, w.n_seg);
    if (ev) hipEventRecord(ev[3], s);
    hipLaunchKernelGGL(k_scatter, dim3(blocks(n, T)), dim3(T), 0, s, w.perm, n, w.v_status, w.v_wait,
                       w.v_rule, out);
    if (ev) hipEventRecord(ev[4], s);
    return hipGetLastError();
}

}  // namespace sf
