// sf_engine.cpp — host runtime behind the C-ABI (include/sentinel_flow.h).
//
// Owns one GPU's shard of resource state in HBM, the rule tables, the batch
// working buffers and one HIP stream.  sf_submit is serialised by a mutex
// (the Java shim batches from many threads into one flusher).
// There is no CPU fallback: without a usable gfx950 device sf_create fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "sf_decide.h"
#include "sf_xflow.h"
#include "sf_sysx.h"
#include "sf_token.h"
#include "sf_wire.h"
#include "sf_degrade.h"
#include <rccl/rccl.h>
#include <functional>
#include <unordered_map>

using namespace sf;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            return fail(_e == hipErrorOutOfMemory ? SF_ERR_NOMEM : SF_ERR_DEVICE,       \
                        std::string(#expr ": ") + hipGetErrorString(_e));               \
    } while (0)

// a device copy of host event arrays, remembered by their addresses (stage_in_events)
struct StageBuf {
    void* p = nullptr; size_t bytes = 0; const void* key[5] = {}; uint32_t n = 0;
    int64_t fp[3] = {};                                     // ts[0], ts[n-1], flags[0] of the staged arrays
    const uint8_t* st_src = nullptr; uint32_t st_n = 0;    // verdicts [0, st_n) of st_src already staged
};

struct sf_engine {
    sf_config cfg{};
    hipStream_t stream = nullptr, stream2 = nullptr, stream3 = nullptr, stream4 = nullptr;   // 4: the wave walk
    hipStream_t sstream = nullptr;  // sort phase of the next batch (overlaps the decide phase on `stream`)
    // ENTRY_NODE's update of an asynchronous batch (after its verdicts, beside
    // the next batch's decide phase: decisions read ENTRY_NODE only with
    // SystemRules, whose batches are synchronous); ev_en: the last one enqueued,
    // en_async: `stream` is not yet ordered after it (en_fence)
    hipStream_t enstream = nullptr;
    bool en_own = false;            // enstream is a stream of its own (else one of the decide streams)
    int side_mode = 3;
    hipEvent_t ev_en = nullptr;
    bool en_async = false;
    bool serial = false;            // diagnostics (SF_SERIAL_STREAMS=1): every kernel on one stream
    uint32_t R = 0, key_bits = 1;
    DevState st{};
    Work w[2]{};                    // two Work sets: batch k sorts into w[k % 2] while k-1 is decided
    bool w_ready[2] = {false, false};
    int cur = 0, last = 0;          // Work set of the next / last submitted batch
    unsigned pending = 0;           // Work sets with an asynchronous batch not yet checked by sf_sync
    bool used[2] = {false, false};
    hipEvent_t ev_sorted[2]{}, ev_done[2]{};
    hipEvent_t ev_end[2]{};                          // ev_done and the batch's ENTRY_NODE update (reads the batch)
    hipEvent_t ev_core[2]{};                         // the verdicts of the slot's batch are written
    SysRule sys{};                  // SystemRuleManager statics; sys.check: batches go through the planner
    SysPlanDev* sys_plan = nullptr; SysExitQ* sys_pa = nullptr; SysEntQ* sys_pb = nullptr;
    uint8_t* sys_ibuf = nullptr;                  // the planner's inert flags (sys_plan)
    uint8_t* sys_mask = nullptr;    // [max_batch] planner verdicts (sf_system.h)
    // rules
    std::vector<uint32_t> flow_pos;        // loaded valid rule index -> CSR position
    uint32_t n_flow = 0, n_prule = 0;
    // the exact ParamFlow table's fill (param_reserve): inserts counted on the
    // device (st.pins), as of the last drain; upper bound of the inserts of
    // batches enqueued since; the most keys one event can insert
    uint64_t p_used = 0, p_pending = 0, p_kmax = 0, p_grows = 0;
    // staging for host-memory batches
    void* stage_in = nullptr; size_t stage_in_bytes = 0;
    void* stage_out = nullptr; size_t stage_out_bytes = 0;
    StageBuf plan_sb, en_sb;                       // sf_system_plan / sf_entry_node_add inputs
    hipEvent_t evs[2][SF_NUM_EVENTS]{};   // per Work set: fork/join and timing events of its batch
    bool timed[2] = {false, false};       // that batch ran with timing on and is not yet in stats
    bool timing = false;
    sf_stats stats{};
    std::vector<void*> user_allocs;
    std::vector<void*> host_allocs;      // sf_host_alloc (pinned host memory)
    std::mutex mu;
    // cluster token server (sf_token.hip)
    TokState ts{};
    TokWork tw{};
    uint32_t tw_cap = 0;
    std::vector<sf_namespace> host_ns;
    std::vector<sf_cluster_flow_rule> host_cflow;
    std::vector<sf_cluster_param_rule> host_cparam;
    std::vector<sf_hot_item> host_citems;
    std::vector<int64_t> cflow_ids;           // flow rule index -> flowId
    void* tok_stage = nullptr; size_t tok_stage_bytes = 0;
    int64_t* d_sum = nullptr;
    void* wire_arena = nullptr; size_t wire_bytes = 0;   // sf_serve_frames scratch (grow-only)
    // ENTRY_NODE and the metric snapshot (sf_entry.hip)
    EntryNode* en = nullptr;
    EntryAcc* en_acc = nullptr;
    // sf_set_report_entry_node: the ENTRY_NODE sf_metric_log writes (node-wide merge), host copy
    bool report_set = false;
    EntryNode report{};
    EntryNode* en_report = nullptr;    // device staging of `report` for the metric kernels
    uint32_t* snap_counts = nullptr; uint32_t* snap_offsets = nullptr; uint32_t* snap_total = nullptr;
    sf_metric_row* snap_rows = nullptr; uint32_t snap_cap = 0;
    void* snap_scan = nullptr; size_t snap_scan_bytes = 0;
    // metrics.log (sf_metric.hip)
    char* nm_bytes = nullptr; uint64_t* nm_off = nullptr; int32_t* nm_types = nullptr; uint32_t n_names = 0;
    unsigned long long* ml_mask = nullptr; uint32_t* ml_counts = nullptr; uint32_t* ml_offsets = nullptr;
    uint32_t* ml_total = nullptr;
    sf_metric_row* ml_rows = nullptr; uint8_t* ml_keys = nullptr; uint32_t* ml_order = nullptr; uint32_t ml_row_cap = 0;
    uint64_t* ml_len = nullptr; uint64_t* ml_off = nullptr; uint64_t* ml_bytes = nullptr;
    char* ml_out = nullptr; uint64_t ml_out_cap = 0;
    void* ml_tmp = nullptr; size_t ml_tmp_bytes = 0;
    hipEvent_t ml_ev[3]{};
    // node-wide aggregate over the ranks of a node (RCCL over xGMI)
    ncclComm_t comm = nullptr;
    // sharded SystemRules, the per-window exchange (sf_sysx.h, sf_submit_node)
    int64_t* sx_msg = nullptr;            // this rank's message [SX_WORDS] (+ the setup words)
    int64_t* sx_recv = nullptr; size_t sx_recv_words = 0;
    int64_t* sx_seq = nullptr;            // [max_batch] device copy of host sequence numbers
    uint8_t* sx_ibuf = nullptr;           // [max_batch] inert flags of the round
    std::vector<int64_t> sx_hsend, sx_hrecv;   // host side of a callback all-gather
    int64_t* agg = nullptr;               // [ws (S+60) | gws (S+60) | vals ((S+60)*6+1) | minrt (S+60)]
    // DegradeSlot circuit breakers (sf_degrade.hip)
    DegradeDev dg{};
    DegradeWork dgw{};
    std::vector<uint32_t> dg_pos;         // breaker index (load order) -> CSR position
    std::vector<sf_degrade_rule> dg_rules;   // the valid rules of the loaded breakers (load order)
    void* dg_stage = nullptr; size_t dg_stage_bytes = 0;
    // xflow walk (sf_xflow.h): group keys and the origin / context node pool
    uint32_t* xmap_buf = nullptr;
    uint8_t* xw_buf = nullptr;
    // the pool's chunks (host mirror of the device directory st.ax_chunks) and
    // the index table's growth (sf_origin.hip); counts for sf_stats
    std::vector<AuxChunk> ax_host;
    AuxChunk* ax_dir = nullptr;
    uint64_t aux_grows = 0;
    // compact batches (sf_submit_packed): per Work set, the device copy of the
    // packed input, its SoA expansion and the verdicts copied back; copy
    // streams so that H2D(k+1), decide(k) and D2H(k-1) overlap
    struct PkStage {
        char* buf = nullptr; size_t bytes = 0;
        hipEvent_t h2d = nullptr, d2h = nullptr;
        hipEvent_t consumed = nullptr;     // the packed inputs expanded (the next H2D into them may start)
        bool d2h_pending = false, consumed_pending = false;
        const uint8_t* out_status = nullptr;   // host verdicts of the async batch in flight (sf_sync_packed)
        int32_t* err_host = nullptr;           // its error flag, copied back with its verdicts (pinned)
        // sf_sparse_verdicts of that batch: the caller's struct, the list lengths
        // (pinned, copied back with the status bytes), the device lists
        bool sparse = false;
        sf_sparse_verdicts sp{};
        uint32_t* sp_counts = nullptr;
        const unsigned long long* sp_wl = nullptr; const unsigned long long* sp_rl = nullptr;
    } pk[2];
    hipStream_t h2d = nullptr, d2h = nullptr;
    int32_t* rh_err = nullptr;            // rehash_table's overflow flag
};

static void free_tok_work(TokWork& w) {
    void* ptrs[] = {w.nskey_in, w.nskey_out, w.idx_in, w.idx_out, w.key_in, w.key_out, w.rule_of, w.pending,
                    w.head, w.head_scan, w.seg_start, w.n_seg, w.sort8_tmp, w.sort64_tmp, w.scan_tmp};
    for (void* p : ptrs) if (p) hipFree(p);
    w = TokWork{};
}

extern "C" {

int sf_abi_version(void) { return SF_ABI_VERSION; }
const char* sf_last_error(void) { return g_err.c_str(); }

void sf_config_default(sf_config* c) {
    std::memset(c, 0, sizeof *c);
    c->sample_count = 2; c->interval_ms = 1000; c->occupy_timeout_ms = 500; c->cold_factor = 3;
    c->statistic_max_rt = 5000; c->max_resources = 1024; c->max_batch = 1u << 20;
    c->param_capacity = 1u << 16; c->shard_count = 1; c->shard_index = 0; c->device = 0;
    c->cluster_sample_count = 10; c->cluster_interval_ms = 1000; c->exceed_count = 1.0;
    c->max_occupy_ratio = 1.0; c->max_flow_ids = 1024; c->aux_capacity = 65536;
}

static int dalloc(void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return fail(SF_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return SF_OK;
}
#define DALLOC(ptr, bytes)                                               \
    do {                                                                 \
        int _rc = dalloc((void**)&(ptr), (bytes));                       \
        if (_rc) { sf_destroy(e); return _rc; }                          \
    } while (0)

static void free_work(Work& w) {
    void* ptrs[] = {w.pv_in, w.pv_out, w.wide, w.err, w.keys_in, w.keys_out, w.perm, w.head, w.head_scan,
                    w.seg_start, w.seg_res, w.n_seg, w.s_ts, w.s_cnt, w.s_flags, w.s_eref,
                    w.s_cts, w.s_nargs, w.s_atag, w.s_abits, w.v_status, w.v_wait,
                    w.v_rule, w.sort_tmp, w.scan_tmp,
                    w.segflag, w.seg_mode, w.light_list, w.lcounts, w.heavy_list, w.counters, w.pcg, w.segs_lb,
                    w.pscan_tmp, w.fill_tiles, w.fill_ntiles, w.acc_hw,
                    w.acc_sec, w.acc_hw_base, w.acc_sec_base, w.seg_hw0, w.seg_sec0,
                    w.seg_nhw, w.seg_nsec, w.hticks, w.passbits, w.stream_list, w.sticks,
                    w.exit_of, w.lxfar, w.thr_rec, w.vs_cursor, w.tile_rc, w.seg_rb, w.seg_re,
                    w.s_origin, w.s_oslot, w.ox_cnt, w.ox_bflags, w.ox_hmap, w.ox_hslot, w.ox_thr, w.ox_acc,
                    w.ox_bseg, w.ox_pairs, w.ox_plist};
    for (void* p : ptrs) if (p) hipFree(p);
    w = Work{};
}

void sf_destroy(sf_engine* e) {
    if (!e) return;
    if (e->sstream) hipStreamSynchronize(e->sstream);
    if (e->stream) hipStreamSynchronize(e->stream);
    for (Work& w : e->w) free_work(w);
    void* ptrs[] = {e->st.second, e->st.borrow, e->st.minute, e->st.threads, (void*)e->st.rule_off,
                    (void*)e->st.rules, e->st.rstate, (void*)e->st.prule_off, e->st.prules, (void*)e->st.items,
                    e->st.pm_init, e->st.ptab, e->st.err, e->stage_in, e->stage_out, e->plan_sb.p, e->en_sb.p, e->st.pins,
                    e->st.xw_stats, (void*)e->st.rdesc, e->st.prio_seen};
    for (void* p : ptrs) if (p) hipFree(p);
    for (void* p : e->user_allocs) hipFree(p);
    for (void* p : e->host_allocs) hipHostFree(p);
    if (e->en_report) hipFree(e->en_report);
    void* tptrs[] = {(void*)e->ts.rules, e->ts.fstate, (void*)e->ts.idtab, (void*)e->ts.ns, e->ts.lim, e->ts.cptab,
                     (void*)e->ts.items, e->ts.rmulti, e->tok_stage, e->wire_arena, e->d_sum, e->en, e->en_acc, e->snap_counts, e->snap_offsets,
                     e->snap_total, e->snap_rows, e->snap_scan, e->st.last_fetch, e->st.last_ts, e->nm_bytes, e->nm_off,
                     e->nm_types, e->ml_mask, e->ml_counts, e->ml_offsets, e->ml_total, e->ml_rows, e->ml_keys,
                     e->ml_order, e->ml_len, e->ml_off, e->ml_bytes, e->ml_out, e->ml_tmp};
    for (void* p : tptrs) if (p) hipFree(p);
    if (e->agg) hipFree(e->agg);
    void* sptrs[] = {e->sys_plan, e->sys_pa, e->sys_pb, e->sys_mask, e->sys_ibuf, e->sx_msg, e->sx_recv,
                     e->sx_seq, e->sx_ibuf};
    for (void* p : sptrs) if (p) hipFree(p);
    void* dptrs[] = {(void*)e->dg.rr_of, (void*)e->dg.off, (void*)e->dg.rules, e->dg.state, e->dgw.keys_in,
                     e->dgw.keys_out, e->dgw.idx_in, e->dgw.idx_out, e->dgw.beg, e->dgw.end, e->dgw.sort_tmp,
                     e->dgw.err, e->rh_err, e->dg_stage, e->dgw.heavy, e->dgw.n_heavy, e->dgw.sev, e->dgw.inv};
    for (void* p : dptrs) if (p) hipFree(p);
    void* xptrs[] = {e->xmap_buf, e->xw_buf, e->st.xtab, e->ax_dir, e->st.ax_count};
    for (void* p : xptrs) if (p) hipFree(p);
    for (const AuxChunk& c : e->ax_host) hipFree(c.sec);          // (one allocation per chunk)
    for (auto& p : e->pk) {
        if (p.buf) hipFree(p.buf);
        if (p.h2d) hipEventDestroy(p.h2d);
        if (p.d2h) hipEventDestroy(p.d2h);
        if (p.consumed) hipEventDestroy(p.consumed);
        if (p.err_host) hipHostFree(p.err_host);
        if (p.sp_counts) hipHostFree(p.sp_counts);
    }
    if (e->h2d) { hipStreamSynchronize(e->h2d); hipStreamDestroy(e->h2d); }
    if (e->d2h) { hipStreamSynchronize(e->d2h); hipStreamDestroy(e->d2h); }
    if (e->comm) ncclCommDestroy(e->comm);
    free_tok_work(e->tw);
    for (auto& a : e->evs) for (auto& x : a) if (x) hipEventDestroy(x);
    for (auto& x : e->ml_ev) if (x) hipEventDestroy(x);
    for (int k = 0; k < 2; k++) {
        if (e->ev_sorted[k]) hipEventDestroy(e->ev_sorted[k]);
        if (e->ev_done[k]) hipEventDestroy(e->ev_done[k]);
        if (e->ev_end[k]) hipEventDestroy(e->ev_end[k]);
        if (e->ev_core[k]) hipEventDestroy(e->ev_core[k]);
    }
    if (e->stream) hipStreamDestroy(e->stream);
    if (e->stream2) hipStreamDestroy(e->stream2);
    if (e->stream3) hipStreamDestroy(e->stream3);
    if (e->stream4) hipStreamDestroy(e->stream4);
    if (e->sstream) hipStreamDestroy(e->sstream);
    if (e->enstream && e->en_own) hipStreamDestroy(e->enstream);
    if (e->ev_en) hipEventDestroy(e->ev_en);
    delete e;
}

#define WALLOC(ptr, bytes)                                               \
    do {                                                                 \
        int _rc = dalloc((void**)&(ptr), (bytes));                       \
        if (_rc) { free_work(w); return _rc; }                           \
    } while (0)

// One Work set: every sorted-order buffer of one batch (sf_internal.h).
static int alloc_work(sf_engine* e, Work& w) {
    const sf_config& c = e->cfg;
    const size_t N = c.max_batch, R = e->R;
    WALLOC(w.keys_in, N * 4); WALLOC(w.keys_out, N * 4); WALLOC(w.perm, N * 4);
    // (12-B payloads when the batch has origins)
    WALLOC(w.pv_in, N * sizeof(PackedEvO)); WALLOC(w.pv_out, N * sizeof(PackedEvO));
    WALLOC(w.wide, 4); WALLOC(w.err, 4);
    WALLOC(w.head_scan, N * 4);
    WALLOC(w.seg_start, (N + 1) * 4); WALLOC(w.seg_res, N * 4); WALLOC(w.n_seg, 4);
    WALLOC(w.s_ts, N * 8); WALLOC(w.s_cnt, N * 4); WALLOC(w.s_flags, N);
    WALLOC(w.s_eref, N * 8); WALLOC(w.s_cts, N * 8);
    WALLOC(w.s_nargs, N); WALLOC(w.s_atag, N * SF_MAX_ARGS); WALLOC(w.s_abits, N * SF_MAX_ARGS * 8);
    WALLOC(w.v_status, N); WALLOC(w.v_wait, N * 4); WALLOC(w.v_rule, N * 2);
    {
        hipError_t he = query_temp_bytes((uint32_t)N, e->key_bits, &w.sort_tmp_bytes, &w.scan_tmp_bytes,
                                         &w.pscan_tmp_bytes);
        if (he != hipSuccess) { free_work(w); return fail(SF_ERR_DEVICE, "rocprim temp size query"); }
    }
    WALLOC(w.sort_tmp, w.sort_tmp_bytes);
    WALLOC(w.scan_tmp, w.scan_tmp_bytes);
    WALLOC(w.pscan_tmp, w.pscan_tmp_bytes);
    // heavy / light split
    w.heavy_min = c.heavy_min_events ? c.heavy_min_events : 512;
    {
        int dev = 0, ncu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
        w.stream_grid = 2u * (uint32_t)(ncu > 0 ? ncu : 256);
        w.fill_grid = 8u * (uint32_t)(ncu > 0 ? ncu : 256);
    }
    const size_t SC = std::min<size_t>(N, R) + 1;
    w.seg_cap = (uint32_t)SC;
    WALLOC(w.segflag, SC * 4); WALLOC(w.seg_mode, SC); WALLOC(w.lcounts, 2 * LCLS * 4);
    {   // light_list regions per length class: class c holds segments of >= lo_len(c) events
        size_t off = 0;
        for (int k = 0; k < LCLS; k++) {
            const size_t lo_len = k == 0 ? 1 : (k == 1 ? 2 : ((size_t)1 << (k - 1)) + 1);
            const size_t cap = lo_len > w.heavy_min ? 0 : std::min<size_t>(SC, N / lo_len + 1);
            w.loff[k] = (uint32_t)off;
            w.lcap[k] = (uint32_t)cap;
            off += cap;
        }
        WALLOC(w.light_list, off * 4);
    }
    WALLOC(w.heavy_list, SC * 4);
    WALLOC(w.counters, 16 * 4); WALLOC(w.pcg, N * 8); WALLOC(w.segs_lb, segs_lb_bytes((uint32_t)N));
    // <= len/TILE + 2 tiles per heavy segment; a ParamFlow-only segment of more
    // than 32 events is heavy too (SM_PARAM, k_classify), whatever heavy_min
    w.fill_tile_cap = (uint32_t)(N / FILL_TILE + 2 * (N / (std::min<uint32_t>(w.heavy_min, 32u) + 1)) + 2);
    WALLOC(w.fill_tiles, (size_t)2 * w.fill_tile_cap * sizeof(uint2)); WALLOC(w.fill_ntiles, 2 * 4);
    w.acc_cap = (uint32_t)std::min<size_t>(std::max<size_t>(N / w.heavy_min * 64, 1 << 16), 1u << 24);
    WALLOC(w.acc_hw, (size_t)w.acc_cap * ACC_BYTES); WALLOC(w.acc_sec, (size_t)w.acc_cap * ACC_BYTES);
    WALLOC(w.acc_hw_base, SC * 4); WALLOC(w.acc_sec_base, SC * 4); WALLOC(w.seg_hw0, SC * 8);
    WALLOC(w.seg_sec0, SC * 8); WALLOC(w.seg_nhw, SC * 4); WALLOC(w.seg_nsec, SC * 4);
    WALLOC(w.hticks, (N / (w.heavy_min + 1) + 2) * 8);
    WALLOC(w.sticks, (N / (w.heavy_min + 1) + 2) * 8);
    WALLOC(w.stream_list, SC * 4);
    WALLOC(w.xw_list, (N / XW_MIN + 1) * 4);
    WALLOC(w.passbits, (N / 64 + 2) * 8);
    WALLOC(w.exit_of, N * 4);
    WALLOC(w.lxfar, (N / 64 + 2) * 8);
    WALLOC(w.thr_rec, N * 8);
    WALLOC(w.tile_rc, (size_t)w.fill_tile_cap * 4); WALLOC(w.seg_rb, SC * 4); WALLOC(w.seg_re, SC * 4);
    WALLOC(w.vs_cursor, VS_CURSORS(N) * 4);
    WALLOC(w.s_origin, N * 4); WALLOC(w.s_oslot, N * 4); WALLOC(w.ox_cnt, 8 * 4);
    WALLOC(w.ox_bflags, (N / OX_TILE + 1) * 4); WALLOC(w.ox_bseg, (N / OX_TILE + 1) * 8);
    return SF_OK;
}

int sf_create(const sf_config* cfg, sf_engine** out) {
    if (!cfg || !out) return fail(SF_ERR_INVALID, "null argument");
    *out = nullptr;
    const sf_config& c = *cfg;
    if (c.sample_count <= 0 || c.sample_count > SF_MAX_SAMPLE_COUNT || c.interval_ms <= 0 ||
        c.interval_ms % c.sample_count != 0)
        return fail(SF_ERR_INVALID, "sample_count/interval_ms invalid (LeapArray.java:70-87)");
    if (c.max_resources == 0 || c.max_batch == 0) return fail(SF_ERR_INVALID, "max_resources/max_batch must be > 0");
    if (c.shard_count == 0 || c.shard_index >= c.shard_count) return fail(SF_ERR_INVALID, "bad shard");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(SF_ERR_DEVICE, "no HIP device visible: the engine has no CPU fallback");
    if (c.device < 0 || c.device >= ndev) return fail(SF_ERR_DEVICE, "device ordinal out of range");
    HIP_TRY(hipSetDevice(c.device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, c.device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SF_ERR_DEVICE, std::string("engine is built for gfx950, device is ") + prop.gcnArchName);

    sf_engine* e = new sf_engine();
    e->cfg = c;
    e->R = c.max_resources;
    while ((1ull << e->key_bits) < e->R) e->key_bits++;
    {   // stream priorities of the decide phase (SF_STREAM_PRIO, diagnostics):
        // 0 = the light lanes' stream C first, 1 = stream A (THREAD / RL chains) first
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        const char* pv = getenv("SF_STREAM_PRIO");
        const bool a_first = pv && pv[0] == '1';
        HIP_TRY(hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, a_first ? greatest : least));
        HIP_TRY(hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithPriority(&e->stream3, hipStreamNonBlocking, a_first ? least : greatest));
        // the sort stream (batch k+1's sort phase runs beside batch k's decide phase)
        const char* ps = getenv("SF_SORT_PRIO");
        if (ps && ps[0] == '1') HIP_TRY(hipStreamCreateWithPriority(&e->sstream, hipStreamNonBlocking, greatest));
        else if (ps && ps[0] == '0') HIP_TRY(hipStreamCreateWithPriority(&e->sstream, hipStreamNonBlocking, least));
        else HIP_TRY(hipStreamCreateWithFlags(&e->sstream, hipStreamNonBlocking));
    }
    if (const char* v = getenv("SF_SERIAL_STREAMS")) e->serial = v[0] == '1';
    {   // the side stream of asynchronous batches: stream C, whose light lanes end
        // first (diagnostics SF_SIDE: 0 none -- on `stream` as before round 6 --,
        // 1 a stream of its own, 2 stream B, 3 stream C).  Same-box means of the
        // driver's step (tools/gpu_var.sh, 3-4 runs each): 13.32 / 13.65 / 13.24 /
        // 13.15 ms; a stream of its own is slower even with GPU_MAX_HW_QUEUES=8.
        const char* v = getenv("SF_SIDE");
        e->side_mode = v ? v[0] - '0' : 3;
        if (e->side_mode == 1) {
            HIP_TRY(hipStreamCreateWithFlags(&e->enstream, hipStreamNonBlocking));
            e->en_own = true;
        } else if (e->side_mode == 2) e->enstream = e->stream2;
        else if (e->side_mode == 3) e->enstream = e->stream3;
        else e->side_mode = 0;
    }
    HIP_TRY(hipEventCreateWithFlags(&e->ev_en, hipEventDisableTiming));
    for (auto& a : e->evs) for (auto& x : a) HIP_TRY(hipEventCreate(&x));
    for (int k = 0; k < 2; k++) {
        HIP_TRY(hipEventCreateWithFlags(&e->ev_sorted[k], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&e->ev_done[k], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&e->ev_end[k], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&e->ev_core[k], hipEventDisableTiming));
    }

    DevState& st = e->st;
    st.S = c.sample_count; st.wl = c.interval_ms / c.sample_count; st.interval = c.interval_ms;
    st.occupy_timeout = c.occupy_timeout_ms; st.max_rt = c.statistic_max_rt; st.R = e->R;
    st.shard_count = c.shard_count;
    const size_t R = e->R, S = c.sample_count;
    DALLOC(st.second, R * S * sizeof(Bucket));
    DALLOC(st.borrow, R * S * sizeof(Borrow));
    DALLOC(st.minute, R * MINUTE * sizeof(Bucket));
    DALLOC(st.threads, R * sizeof(int64_t));
    DALLOC(st.rule_off, (R + 1) * sizeof(uint32_t));
    DALLOC(st.prule_off, (R + 1) * sizeof(uint32_t));
    DALLOC(st.pm_init, R);
    DALLOC(st.rdesc, R * sizeof(RDesc));
    DALLOC(st.prio_seen, sizeof(int32_t));
    DALLOC(st.err, sizeof(int32_t));
    uint64_t pcap = 16;
    while (pcap < (uint64_t)c.param_capacity) pcap <<= 1;
    DALLOC(st.ptab, pcap * sizeof(ParamSlot));
    st.pcap_mask = pcap - 1;
    HIP_TRY(hipMemsetAsync((void*)st.rule_off, 0, (R + 1) * sizeof(uint32_t), e->stream));
    HIP_TRY(hipMemsetAsync((void*)st.prule_off, 0, (R + 1) * sizeof(uint32_t), e->stream));
    HIP_TRY(hipMemsetAsync(st.pm_init, 0, R, e->stream));
    HIP_TRY(hipMemsetAsync((void*)st.rdesc, 0, R * sizeof(RDesc), e->stream));   // (= no rules)
    HIP_TRY(hipMemsetAsync(st.prio_seen, 0, sizeof(int32_t), e->stream));
    HIP_TRY(hipMemsetAsync(st.ptab, 0, pcap * sizeof(ParamSlot), e->stream));
    DALLOC(st.pins, 256 * 16 * sizeof(unsigned int));
    DALLOC(st.xw_stats, 4 * sizeof(unsigned long long));
    if (hipMemset(e->st.xw_stats, 0, 4 * sizeof(unsigned long long)) != hipSuccess) { sf_destroy(e); return fail(SF_ERR_DEVICE, "memset"); }
    HIP_TRY(hipMemsetAsync(st.pins, 0, 256 * 16 * sizeof(unsigned int), e->stream));
    HIP_TRY(hipMemsetAsync(st.err, 0, sizeof(int32_t), e->stream));
    HIP_TRY(launch_init_state(st, e->stream));
    e->ts.err = st.err;
    e->ts.exceed_count = c.exceed_count;
    e->ts.shard_count = c.shard_count; e->ts.shard_index = c.shard_index;
    e->ts.max_occupy_ratio = c.max_occupy_ratio;
    DALLOC(e->d_sum, sizeof(int64_t));
    DALLOC(st.last_fetch, R * sizeof(int64_t));
    DALLOC(st.last_ts, sizeof(int64_t));
    {
        const int64_t t_min = INT64_MIN;
        HIP_TRY(hipMemcpyAsync(st.last_ts, &t_min, 8, hipMemcpyHostToDevice, e->stream));
    }
    HIP_TRY(hipMemsetAsync(st.last_fetch, 0xff, R * sizeof(int64_t), e->stream));   // lastFetchTime = -1
    DALLOC(e->en, sizeof(EntryNode));
    DALLOC(e->en_acc, sizeof(EntryAcc));
    HIP_TRY(launch_entry_init(e->en, st.max_rt, e->stream));

    {
        const int rc = alloc_work(e, e->w[0]);
        if (rc) { sf_destroy(e); return rc; }
        e->w_ready[0] = true;
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
    *out = e;
    return SF_OK;
}

static int local_of(const sf_engine* e, uint32_t res, uint32_t* l) {
    if (res % e->cfg.shard_count != e->cfg.shard_index) return 0;
    *l = res / e->cfg.shard_count;
    return *l < e->R;
}

// Per-kernel device times of the batch last run in Work set `slot` (its
// events), added to the stats once, after that batch has completed.
static void acc_timing(sf_engine* e, int slot) {
    if (!e->timed[slot]) return;
    e->timed[slot] = false;
    hipEvent_t* ev = e->evs[slot];
    float a = 0, b2 = 0, c = 0, d = 0;
    hipEventElapsedTime(&a, ev[0], ev[1]);
    hipEventElapsedTime(&b2, ev[1], ev[2]);
    hipEventElapsedTime(&c, ev[2], ev[3]);
    hipEventElapsedTime(&d, ev[3], ev[4]);
    float cl = 0, li = 0, hd = 0, hf = 0, hs = 0;
    hipEventElapsedTime(&cl, ev[10], ev[2]);
    hipEventElapsedTime(&li, ev[5], ev[9]);
    if (e->st.n_window_rules) {                    // the lean walks end on stream B
        float lq = 0;
        hipEventElapsedTime(&lq, ev[5], ev[16]);
        li = std::max(li, lq);
    }
    hipEventElapsedTime(&hd, ev[5], ev[7]);
    hipEventElapsedTime(&hf, ev[7], ev[8]);
    hipEventElapsedTime(&hs, ev[11], ev[12]);
    e->stats.classify_ms += cl; e->stats.light_ms += li;
    e->stats.heavy_decide_ms += hd; e->stats.heavy_fill_ms += hf; e->stats.stream_ms += hs;
    e->stats.sort_ms += a + b2;
    e->stats.decide_ms += c;
    e->stats.scatter_ms += d;
    e->stats.total_ms += a + b2 + c + d;
}

static int sparse_complete(sf_engine::PkStage& pk);
// Drain asynchronously submitted batches: wait for both streams, then report
// the first error flag raised by any of them.  An async packed batch whose
// verdicts the caller has not collected keeps its error for its own
// sf_sync_packed, unless `all` (sf_sync: every batch collected here).
// order `stream` after the last asynchronous ENTRY_NODE update (every host
// call that reads or writes ENTRY_NODE on `stream` does this first)
static int en_fence(sf_engine* e) {
    if (!e->en_async) return SF_OK;
    HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_en, 0));
    e->en_async = false;
    return SF_OK;
}

static int drain(sf_engine* e, bool all = false) {
    if (e->en_async) { HIP_TRY(hipStreamSynchronize(e->enstream)); e->en_async = false; }
    if (!e->pending) return SF_OK;
    HIP_TRY(hipStreamSynchronize(e->sstream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->d2h) HIP_TRY(hipStreamSynchronize(e->d2h));
    for (auto& p : e->pk) p.d2h_pending = false;
    int first = 0;
    unsigned keep = 0;
    for (int k = 0; k < 2; k++) {
        if (!(e->pending & (1u << k))) continue;
        // an async packed batch whose verdicts the caller has not collected: its
        // error came back with them and is reported by its own sf_sync_packed
        if (e->pk[k].out_status && !all) { keep |= 1u << k; continue; }
        if (e->pk[k].out_status) {
            e->pk[k].out_status = nullptr;
            if (e->pk[k].sparse) { const int rc = sparse_complete(e->pk[k]); if (rc) return rc; }
        }
        int32_t err = 0;
        HIP_TRY(hipMemcpy(&err, e->w[k].err, 4, hipMemcpyDeviceToHost));
        if (err && !first) first = err;
    }
    e->pending = keep;
    for (int k = 0; k < 2; k++) acc_timing(e, k);
    {
        uint32_t nseg = 0;
        HIP_TRY(hipMemcpy(&nseg, e->w[e->last].n_seg, 4, hipMemcpyDeviceToHost));
        e->stats.n_segments = nseg;
    }
    if (first) return fail(first, first == SF_ERR_CAPACITY ? "capacity exceeded (param table, or the origin / context node pool: aux_capacity)"
                                                           : "invalid batch (resource outside shard or bad entry_ref)");
    return SF_OK;
}

// The origin / context node pool and its index table (sf_xflow.h,
// sf_origin.hip), allocated with the first batch with origins or the first
// rule that reads such nodes; the nodes live as long as the engine
// (ClusterNode.originCountMap / NodeSelectorSlot maps are never pruned).  The
// pool grows by chunks of AX_CHUNK nodes (no node moves) and the index table
// by rehashing into a larger one, both between batches, so that a batch never
// fails on their capacity.
static int pool_grow(sf_engine* e, uint64_t need) {
    DevState& st = e->st;
    const size_t S = st.S;
    if ((uint64_t)st.ax_cap >= need) return SF_OK;
    while ((uint64_t)st.ax_cap < need) {
        if (e->ax_host.size() >= AX_MAX_CHUNKS) return fail(SF_ERR_CAPACITY, "origin / context node pool at its limit");
        const size_t sec_b = (size_t)AX_CHUNK * S * sizeof(Bucket), bor_b = (size_t)AX_CHUNK * S * sizeof(Borrow);
        const size_t min_b = (size_t)AX_CHUNK * MINUTE * sizeof(Bucket), thr_b = (size_t)AX_CHUNK * sizeof(int64_t);
        char* m = nullptr;
        HIP_TRY(hipMalloc((void**)&m, sec_b + bor_b + min_b + thr_b));
        AuxChunk c{(Bucket*)m, (Borrow*)(m + sec_b), (Bucket*)(m + sec_b + bor_b), (int64_t*)(m + sec_b + bor_b + min_b)};
        DevState pool = st;                    // fresh nodes: the resource-row initialiser on the chunk
        pool.second = c.sec; pool.borrow = c.bor; pool.minute = c.min; pool.threads = c.thr; pool.R = AX_CHUNK;
        const hipError_t le = launch_init_state(pool, e->stream);
        if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("aux init: ") + hipGetErrorString(le));
        HIP_TRY(hipMemcpyAsync(e->ax_dir + e->ax_host.size(), &c, sizeof c, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        e->ax_host.push_back(c);
        st.ax_cap += AX_CHUNK;
    }
    return SF_OK;
}

// Rebuild an open-addressed table (origin index or ParamFlow table) into a new
// one of at least `ncap` slots; a key that would land farther than
// PT_MAX_PROBE from its home slot makes k_ox_rehash raise its flag, and the
// rebuild is retried at twice the size (nothing in flight).
static int rehash_table(sf_engine* e, const ParamSlot* old, uint64_t old_n, uint64_t ncap,
                        ParamSlot** out, uint64_t* out_cap, const char* what) {
    if (!e->rh_err) HIP_TRY(hipMalloc((void**)&e->rh_err, sizeof(int32_t)));
    for (;;) {
        ParamSlot* nt = nullptr;
        HIP_TRY(hipMalloc((void**)&nt, ncap * sizeof(ParamSlot)));
        HIP_TRY(hipMemsetAsync(nt, 0, ncap * sizeof(ParamSlot), e->stream));
        HIP_TRY(hipMemsetAsync(e->rh_err, 0, sizeof(int32_t), e->stream));
        const hipError_t le = launch_ox_rehash(old, old_n, nt, ncap - 1, e->rh_err, e->stream);
        if (le != hipSuccess) { hipFree(nt); return fail(SF_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(le)); }
        int32_t flag = 0;
        HIP_TRY(hipMemcpyAsync(&flag, e->rh_err, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (!flag) { *out = nt; *out_cap = ncap; return SF_OK; }
        HIP_TRY(hipFree(nt));
        ncap *= 2;
    }
}

static int ensure_aux(sf_engine* e) {
    DevState& st = e->st;
    if (st.xtab) return SF_OK;
    const uint32_t cap = e->cfg.aux_capacity ? e->cfg.aux_capacity : 65536;
    uint64_t tcap = 16;
    while (tcap < 2ull * cap) tcap <<= 1;
    HIP_TRY(hipMalloc((void**)&e->ax_dir, AX_MAX_CHUNKS * sizeof(AuxChunk)));
    HIP_TRY(hipMalloc((void**)&st.ax_count, sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&st.xtab, tcap * sizeof(ParamSlot)));
    HIP_TRY(hipMemsetAsync(st.ax_count, 0, sizeof(uint32_t), e->stream));
    HIP_TRY(hipMemsetAsync(st.xtab, 0, tcap * sizeof(ParamSlot), e->stream));
    st.xcap_mask = tcap - 1;
    st.ax_chunks = e->ax_dir;
    st.ax_cap = 0;
    return pool_grow(e, cap);
}

// the index table rebuilt with room for `need` keys at half load (nothing in flight)
static int index_grow(sf_engine* e, uint64_t need) {
    DevState& st = e->st;
    uint64_t tcap = (st.xcap_mask + 1) * 4;
    while (tcap < 2 * need) tcap <<= 1;
    ParamSlot* nt = nullptr;
    HIP_TRY(hipDeviceSynchronize());
    { const int rc = rehash_table(e, st.xtab, st.xcap_mask + 1, tcap, &nt, &tcap, "index rehash"); if (rc) return rc; }
    HIP_TRY(hipFree(st.xtab));
    st.xtab = nt;
    st.xcap_mask = tcap - 1;
    e->aux_grows++;
    return SF_OK;
}

// per-Work-set maps of the origin pass sized for the index table (every pool
// slot is below its capacity), the slot -> heavy id map reset to XNONE
static int ox_maps(sf_engine* e, Work& w, bool reset, hipStream_t ss) {
    const size_t need = (size_t)e->st.xcap_mask + 1;
    if (w.ox_hmap_n < need) {
        if (w.ox_hmap) hipFree(w.ox_hmap);
        if (w.ox_hslot) hipFree(w.ox_hslot);
        if (w.ox_thr) hipFree(w.ox_thr);
        w.ox_hmap = nullptr; w.ox_hslot = nullptr; w.ox_thr = nullptr; w.ox_hmap_n = w.ox_hslot_n = 0;
        HIP_TRY(hipMalloc((void**)&w.ox_hmap, need * 4));
        HIP_TRY(hipMalloc((void**)&w.ox_hslot, need * 4));
        HIP_TRY(hipMalloc((void**)&w.ox_thr, need * 8));
        w.ox_hmap_n = w.ox_hslot_n = need;
        reset = true;
    }
    if (reset) HIP_TRY(hipMemsetAsync(w.ox_hmap, 0xff, w.ox_hmap_n * 4, ss));
    return SF_OK;
}

// After the sort phase of a batch with origins (or with rules that read origin
// / context nodes): the index pass inserts every key the batch needs (growing
// the table and running again when it fills), then the pool grows to cover
// the new slots -- all before the decide phase, so nothing is ever dropped.
// The host waits for the sort stream here (the previous batch's decide phase
// keeps running).  Fills `plan` for the origin-node pass of the decide phase.
static int ox_prologue(sf_engine* e, Work& w, const DevBatch& b, hipStream_t ss) {
    { const int rc = ensure_aux(e); if (rc) return rc; }
    // a batch that stopped between its index pass and its origin apply (an
    // early error return) left its heavy ids in ox_hmap: reset them
    { const int rc = ox_maps(e, w, w.ox_dirty, ss); if (rc) return rc; }
    if (b.origin && !w.ox_pairs) {                 // (at most one pair per event)
        HIP_TRY(hipMalloc((void**)&w.ox_pairs, (size_t)e->cfg.max_batch * sizeof(uint4)));
        HIP_TRY(hipMalloc((void**)&w.ox_plist, (size_t)e->cfg.max_batch * sizeof(uint32_t)));
        w.ox_pairs_cap = e->cfg.max_batch;
    }
    return SF_OK;
}
static int ox_launch_index(sf_engine* e, Work& w, const DevBatch& b, hipStream_t ss) {
    DevState stl = e->st;
    stl.err = w.err;
    const uint64_t xcap = e->st.xcap_mask + 1;
    const uint32_t lim = (uint32_t)std::min<uint64_t>(xcap * 7 / 10, 0xffffff00u);
    DevBatch bi = b;
    if (!w.s_origin || !b.origin) bi.origin = nullptr;
    w.ox_dirty = true;
    const hipError_t le = launch_ox_index(stl, w, bi, lim, ss);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("origin index: ") + hipGetErrorString(le));
    return SF_OK;
}
// after the index passes (counts read): the pool covers every slot, the index
// stays at most half full, the plan of the origin-node pass
static int ox_plan(sf_engine* e, Work& w, const uint32_t* cnt, uint32_t ax, const int64_t* t01, OxPlan* plan) {
    { const int rc = pool_grow(e, ax); if (rc) return rc; }
    // keep the index at most half full for the next batches
    if ((uint64_t)ax * 2 > e->st.xcap_mask + 1) {
        HIP_TRY(hipDeviceSynchronize());
        // (the Work set's hmap entries of this batch are slot-indexed: still valid after a rehash)
        const size_t old_n = w.ox_hmap_n;
        { const int rc = index_grow(e, (uint64_t)ax * 2); if (rc) return rc; }
        if (w.ox_hmap_n < (size_t)e->st.xcap_mask + 1) {
            // regrow the maps keeping this batch's heavy ids
            uint32_t* nh = nullptr; uint32_t* ns = nullptr; int64_t* nt = nullptr;
            const size_t need = (size_t)e->st.xcap_mask + 1;
            HIP_TRY(hipMalloc((void**)&nh, need * 4));
            HIP_TRY(hipMalloc((void**)&ns, need * 4));
            HIP_TRY(hipMalloc((void**)&nt, need * 8));
            HIP_TRY(hipMemsetAsync(nh, 0xff, need * 4, e->stream));
            HIP_TRY(hipMemcpyAsync(nh, w.ox_hmap, old_n * 4, hipMemcpyDeviceToDevice, e->stream));
            HIP_TRY(hipMemcpyAsync(ns, w.ox_hslot, old_n * 4, hipMemcpyDeviceToDevice, e->stream));
            HIP_TRY(hipStreamSynchronize(e->stream));
            hipFree(w.ox_hmap); hipFree(w.ox_hslot); hipFree(w.ox_thr);
            w.ox_hmap = nh; w.ox_hslot = ns; w.ox_thr = nt; w.ox_hmap_n = w.ox_hslot_n = need;
        }
    }
    plan->n_heavy = cnt[OXC_HEAVY];
    plan->n_pairs = cnt[OXC_PAIRS];
    const int64_t wl = e->st.wl;
    plan->win.w0s = t01[0] / wl; plan->win.w0m = t01[0] / 1000;
    plan->win.ws = (uint32_t)(t01[1] / wl - plan->win.w0s + 1);
    plan->win.wm = (uint32_t)(t01[1] / 1000 - plan->win.w0m + 1);
    const size_t acc_n = (size_t)plan->n_heavy * ((size_t)plan->win.ws + plan->win.wm);
    if (w.ox_acc_n < acc_n) {
        if (w.ox_acc) hipFree(w.ox_acc);
        w.ox_acc = nullptr; w.ox_acc_n = 0;
        const size_t n2 = acc_n + acc_n / 4;
        HIP_TRY(hipMalloc(&w.ox_acc, n2 * sizeof(OxAcc)));
        w.ox_acc_n = n2;
    }
    return SF_OK;
}
static int prepare_origins(sf_engine* e, Work& w, const DevBatch& b, hipStream_t ss, OxPlan* plan) {
    { const int rc = ox_prologue(e, w, b, ss); if (rc) return rc; }
    uint32_t cnt[8] = {0};
    uint32_t ax = 0;
    for (int round = 0;; round++) {
        { const int rc = ox_launch_index(e, w, b, ss); if (rc) return rc; }
        HIP_TRY(hipMemcpyAsync(cnt, w.ox_cnt, sizeof cnt, hipMemcpyDeviceToHost, ss));
        HIP_TRY(hipMemcpyAsync(&ax, e->st.ax_count, 4, hipMemcpyDeviceToHost, ss));
        HIP_TRY(hipStreamSynchronize(ss));
        if (!cnt[OXC_OVERFLOW]) break;
        if (round > 12) return fail(SF_ERR_CAPACITY, "origin / context node index cannot grow");
        // no room for the keys: everything drains, the table grows to the keys
        // reserved (every absent key counted, by each workgroup that missed it),
        // the pass runs again
        HIP_TRY(hipDeviceSynchronize());
        { const int rc = index_grow(e, std::max<uint64_t>((uint64_t)cnt[OXC_RESERVED], ax) * 3 / 2); if (rc) return rc; }
        { const int rc = ox_maps(e, w, true, ss); if (rc) return rc; }
    }
    int64_t t01[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&t01[0], b.ts, 8, hipMemcpyDeviceToHost, ss));
    HIP_TRY(hipMemcpyAsync(&t01[1], b.ts + (b.n - 1), 8, hipMemcpyDeviceToHost, ss));
    HIP_TRY(hipStreamSynchronize(ss));
    return ox_plan(e, w, cnt, ax, t01, plan);
}


int sf_load_flow_rules(sf_engine* e, const sf_flow_rule* rules, uint32_t n) {
    if (!e || (n && !rules)) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = drain(e); if (rc) return rc; }   // pending batches were sorted under the old rules
    std::vector<uint32_t> counts(e->R + 1, 0);
    std::vector<const sf_flow_rule*> valid;
    std::vector<uint32_t> valid_local, valid_ref;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t l;
        if (!local_of(e, rules[i].resource, &l)) return fail(SF_ERR_INVALID, "rule resource outside this shard");
        if (!valid_flow_rule(rules[i])) continue;
        uint32_t ref = XNONE;
        if (rules[i].strategy == SF_STRATEGY_RELATE && rules[i].ref_resource != SF_REF_NONE) {
            // RELATE reads refResource's ClusterNode: it must be decided by the same
            // engine (co-locate the pair); an id beyond this shard's
            // resources never gets a node (the rule passes)
            if (rules[i].ref_resource % e->cfg.shard_count != e->cfg.shard_index)
                return fail(SF_ERR_UNSUPPORTED, "RELATE refResource on another shard: co-locate it with the resource");
            const uint32_t rl = rules[i].ref_resource / e->cfg.shard_count;
            if (rl < e->R) ref = rl;
        }
        if (rules[i].control_behavior != SF_BEHAVIOR_DEFAULT && rules[i].grade == SF_GRADE_QPS &&
            e->cfg.cold_factor <= 1 &&
            (rules[i].control_behavior == SF_BEHAVIOR_WARM_UP || rules[i].control_behavior == SF_BEHAVIOR_WARM_UP_RATE_LIMITER))
            return fail(SF_ERR_INVALID, "Cold factor should be larger than 1 (WarmUpController.java:114-116)");
        if (++counts[l] > SF_MAX_RULES_PER_RESOURCE)
            return fail(SF_ERR_UNSUPPORTED, "more than SF_MAX_RULES_PER_RESOURCE rules on one resource");
        valid.push_back(&rules[i]);
        valid_local.push_back(l);
        valid_ref.push_back(ref);
    }
    std::vector<uint32_t> off(e->R + 1, 0);
    for (uint32_t r = 0; r < e->R; r++) off[r + 1] = off[r] + counts[r];
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    std::vector<DevRule> dr(valid.size());
    std::vector<DevRuleState> ds(valid.size());
    e->flow_pos.assign(valid.size(), 0);
    for (size_t k = 0; k < valid.size(); k++) {
        const sf_flow_rule& r = *valid[k];
        uint32_t pos = fill[valid_local[k]]++;
        e->flow_pos[k] = pos;
        DevRule d = make_dev_rule(r, e->cfg.cold_factor, (int32_t)k, valid_ref[k]);
        dr[pos] = d;
        ds[pos] = fresh_rule_state();
    }
    std::vector<uint32_t> xmap;
    const bool xflow = build_xmap(dr.data(), off.data(), e->R, xmap);
    if (xflow) {
        const int rc = ensure_aux(e);
        if (rc) return rc;
        if (!e->xmap_buf) HIP_TRY(hipMalloc((void**)&e->xmap_buf, (size_t)e->R * sizeof(uint32_t)));
        HIP_TRY(hipMemcpyAsync(e->xmap_buf, xmap.data(), (size_t)e->R * sizeof(uint32_t), hipMemcpyHostToDevice,
                               e->stream));
        std::vector<uint8_t> xw;
        build_xw(dr.data(), off.data(), e->R, xmap, xw);
        if (!e->xw_buf) HIP_TRY(hipMalloc((void**)&e->xw_buf, (size_t)e->R));
        HIP_TRY(hipMemcpyAsync(e->xw_buf, xw.data(), (size_t)e->R, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    e->n_flow = (uint32_t)valid.size();
    {   // which segment classes the rules allow (launches of absent classes are skipped)
        uint32_t ns = 0, nw = 0;
        for (const DevRule& r : dr) {
            if (r.kind == CT_RATE_LIMITER || (r.kind == CT_DEFAULT && r.grade == SF_GRADE_THREAD)) ns++;
            if ((r.kind == CT_DEFAULT && r.grade == SF_GRADE_QPS) || r.kind == CT_WARM_UP) nw++;
        }
        e->st.n_stream_rules = ns; e->st.n_window_rules = nw;
    }
    if (e->st.rules) { hipFree((void*)e->st.rules); e->st.rules = nullptr; }
    if (e->st.rstate) { hipFree(e->st.rstate); e->st.rstate = nullptr; }
    HIP_TRY(hipMalloc((void**)&e->st.rules, std::max<size_t>(1, dr.size()) * sizeof(DevRule)));
    HIP_TRY(hipMalloc((void**)&e->st.rstate, std::max<size_t>(1, ds.size()) * sizeof(DevRuleState)));
    if (!dr.empty()) {
        HIP_TRY(hipMemcpyAsync((void*)e->st.rules, dr.data(), dr.size() * sizeof(DevRule), hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipMemcpyAsync(e->st.rstate, ds.data(), ds.size() * sizeof(DevRuleState), hipMemcpyHostToDevice, e->stream));
    }
    HIP_TRY(hipMemcpyAsync((void*)e->st.rule_off, off.data(), off.size() * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(launch_rdesc(e->st, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->st.xmap = xflow ? e->xmap_buf : nullptr;
    e->st.xw = xflow ? e->xw_buf : nullptr;
    // the wave walk's stream, created at the first table that routes to it and
    // after the pipeline's four (a stream created earlier changes which hardware
    // queue each of those gets: config 3 lost 2.3 ms/step to a shared queue)
    if (e->st.xw && !e->stream4) HIP_TRY(hipStreamCreateWithFlags(&e->stream4, hipStreamNonBlocking));
    return SF_OK;
}

int sf_load_param_rules(sf_engine* e, const sf_param_rule* rules, uint32_t n, const sf_hot_item* items,
                        uint32_t n_items) {
    if (!e || (n && !rules) || (n_items && !items)) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = drain(e); if (rc) return rc; }   // pending batches were sorted under the old rules
    std::vector<uint32_t> counts(e->R + 1, 0), loc(n);
    for (uint32_t i = 0; i < n; i++) {
        if (!local_of(e, rules[i].resource, &loc[i])) return fail(SF_ERR_INVALID, "rule resource outside this shard");
        if ((uint64_t)rules[i].item_offset + rules[i].item_count > n_items) return fail(SF_ERR_INVALID, "hot item range");
        if (++counts[loc[i]] > SF_MAX_RULES_PER_RESOURCE)
            return fail(SF_ERR_UNSUPPORTED, "more than SF_MAX_RULES_PER_RESOURCE param rules on one resource");
    }
    std::vector<uint32_t> off(e->R + 1, 0);
    for (uint32_t r = 0; r < e->R; r++) off[r + 1] = off[r] + counts[r];
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    std::vector<DevParamRule> dp(n);
    for (uint32_t i = 0; i < n; i++) {
        const sf_param_rule& r = rules[i];
        DevParamRule d = make_dev_param_rule(r, (int32_t)i);
        dp[fill[loc[i]]++] = d;
    }
    std::vector<DevHotItem> di(n_items);
    for (uint32_t i = 0; i < n_items; i++) { di[i].bits = items[i].bits; di[i].count = items[i].count; di[i].tag = items[i].tag; }
    e->n_prule = n;
    e->st.n_prule = n;
    if (e->st.prules) { hipFree(e->st.prules); e->st.prules = nullptr; }
    if (e->st.items) { hipFree((void*)e->st.items); e->st.items = nullptr; }
    HIP_TRY(hipMalloc((void**)&e->st.prules, std::max<size_t>(1, dp.size()) * sizeof(DevParamRule)));
    HIP_TRY(hipMalloc((void**)&e->st.items, std::max<size_t>(1, di.size()) * sizeof(DevHotItem)));
    if (n) HIP_TRY(hipMemcpyAsync(e->st.prules, dp.data(), dp.size() * sizeof(DevParamRule), hipMemcpyHostToDevice, e->stream));
    if (n_items) HIP_TRY(hipMemcpyAsync((void*)e->st.items, di.data(), di.size() * sizeof(DevHotItem), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync((void*)e->st.prule_off, off.data(), off.size() * 4, hipMemcpyHostToDevice, e->stream));
    // a rule reload drops all ParameterMetric state (new ParameterMetric per resource)
    HIP_TRY(hipMemsetAsync(e->st.pm_init, 0, e->R, e->stream));
    HIP_TRY(hipMemsetAsync(e->st.ptab, 0, (e->st.pcap_mask + 1) * sizeof(ParamSlot), e->stream));
    HIP_TRY(hipMemsetAsync(e->st.pins, 0, 256 * 16 * sizeof(unsigned int), e->stream));
    e->p_used = e->p_pending = 0;
    // keys one event (or one collection element) can insert: a rule key per rule
    // (ParameterMetric token / time maps) and a thread-count key per rule's index
    uint32_t kmax = 0;
    for (uint32_t r = 0; r < e->R; r++) kmax = std::max(kmax, counts[r]);
    e->p_kmax = 2ull * kmax;
    HIP_TRY(launch_rdesc(e->st, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return SF_OK;
}

// SystemRuleManager.loadSystemConf (SystemRuleManager.java:267-289) through
// SystemPropertyListener.configUpdate (:173-196): the minimum of every set
// threshold; checkSystemStatus follows the last rule, as in the reference.
int sf_load_system_rules(sf_engine* e, const sf_system_rule* rules, uint32_t n) {
    if (!e || (n && !rules)) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = drain(e); if (rc) return rc; }
    SysRule r{};
    r.qps = r.highest_load = r.highest_cpu = 1.7976931348623157e308;
    r.max_rt = r.max_thread = INT64_MAX;
    r.cur_load = e->sys.cur_load; r.cur_cpu = e->sys.cur_cpu;
    for (uint32_t i = 0; i < n; i++) {
        const sf_system_rule& x = rules[i];
        int check = 0;
        if (x.highest_system_load >= 0) { r.highest_load = std::fmin(r.highest_load, x.highest_system_load); r.load_set = 1; check = 1; }
        if (x.highest_cpu_usage >= 0 && x.highest_cpu_usage <= 1) {
            r.highest_cpu = std::fmin(r.highest_cpu, x.highest_cpu_usage); r.cpu_set = 1; check = 1;
        }
        if (x.avg_rt >= 0) { if (x.avg_rt < r.max_rt) r.max_rt = x.avg_rt; check = 1; }
        if (x.max_thread >= 0) { if (x.max_thread < r.max_thread) r.max_thread = x.max_thread; check = 1; }
        if (x.qps >= 0) { r.qps = std::fmin(r.qps, x.qps); check = 1; }
        r.check = check;
    }
    e->sys = r;
    return SF_OK;
}
// SystemStatusListener readings (system load average, cpu usage): fixed inputs of a replay
int sf_set_system_status(sf_engine* e, double avg_load, double cpu_usage) {
    if (!e) return fail(SF_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    e->sys.cur_load = avg_load; e->sys.cur_cpu = cpu_usage;
    return SF_OK;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// The exact ParamFlow table never fills during a batch: before a batch with
// ParamFlow rules, the keys it can insert at most ((events + collection
// elements) x the most keys per event) must fit in the table's free half,
// counting the inserts of the batches still in flight the same way.  When
// they may not, everything drains, the device's insert counters give the
// exact fill, and the table is rebuilt larger if it is still too small
// (ParameterMetric's maps have no capacity in the reference apart from the
// LRU, ParameterMetric.java:99-118, whose eviction the exact table replaces).
static int param_reserve(sf_engine* e, uint64_t bound) {
    if (!e->n_prule || !bound) return SF_OK;
    const uint64_t cap = e->st.pcap_mask + 1;
    if ((e->p_used + e->p_pending + bound) * 2 <= cap) { e->p_pending += bound; return SF_OK; }
    auto read_used = [&](uint64_t* used) -> int {
        std::vector<unsigned int> c(256 * 16);
        HIP_TRY(hipMemcpy(c.data(), e->st.pins, c.size() * sizeof(unsigned int), hipMemcpyDeviceToHost));
        uint64_t u = 0;
        for (int k = 0; k < 256; k++) u += c[k * 16];
        *used = u;
        return SF_OK;
    };
    // The batches counted in p_pending may have finished already: when every
    // enqueued decide phase is done (a non-blocking event query), the device
    // counters give the exact fill without a drain, and the pending worst-case
    // bounds are released (they only ever grew before).
    bool idle = true;
    for (int k = 0; k < 2 && idle; k++)
        if (e->used[k] && hipEventQuery(e->ev_done[k]) != hipSuccess) idle = false;
    if (idle) {
        uint64_t used = 0;
        { const int rc = read_used(&used); if (rc) return rc; }
        e->p_used = used;
        e->p_pending = 0;
        if ((used + bound) * 2 <= cap) { e->p_pending = bound; return SF_OK; }
    }
    { const int rc = drain(e); if (rc) return rc; }
    HIP_TRY(hipStreamSynchronize(e->stream));
    uint64_t used = 0;
    { const int rc = read_used(&used); if (rc) return rc; }
    e->p_used = used;
    e->p_pending = 0;
    if ((used + bound) * 2 > cap) {
        uint64_t ncap = cap * 2;
        while ((used + bound) * 2 > ncap) ncap <<= 1;
        ParamSlot* nt = nullptr;
        HIP_TRY(hipDeviceSynchronize());
        { const int rc = rehash_table(e, e->st.ptab, cap, ncap, &nt, &ncap, "param rehash"); if (rc) return rc; }
        HIP_TRY(hipFree(e->st.ptab));
        e->st.ptab = nt;
        e->st.pcap_mask = ncap - 1;
        e->p_grows++;
    }
    e->p_pending = bound;
    return SF_OK;
}

// the caller's batch and verdict arrays as device pointers: host arrays are
// copied to the engine's staging buffers on stream ss (verdicts come back
// from stage_out after the decision)
static int stage_batch(sf_engine* e, const sf_event_batch* in, const sf_verdicts* out, hipStream_t ss,
                       DevBatch& b, DevVerdicts& dv) {
    const uint32_t n = in->n;
    if (in->mem == SF_MEM_HOST) {
        size_t need = 0;
        size_t o_res = need; need += align_up((size_t)n * 4);
        size_t o_ts = need; need += align_up((size_t)n * 8);
        size_t o_cnt = need; need += align_up((size_t)n * 4);
        size_t o_fl = need; need += align_up((size_t)n);
        size_t o_er = need; need += in->entry_ref ? align_up((size_t)n * 8) : 0;
        size_t o_ct = need; need += (in->entry_ref && in->create_ts) ? align_up((size_t)n * 8) : 0;
        size_t o_na = need; need += in->n_args ? align_up((size_t)n) : 0;
        size_t o_at = need; need += align_up((size_t)n * in->arg_slots);
        size_t o_ab = need; need += align_up((size_t)n * in->arg_slots * 8);
        const bool coll = in->arg_elem_off != nullptr;
        size_t o_eo = need; need += coll ? align_up(((size_t)n * in->arg_slots + 1) * 4) : 0;
        size_t o_et = need; need += coll ? align_up((size_t)in->n_elems) : 0;
        size_t o_eb = need; need += coll ? align_up((size_t)in->n_elems * 8) : 0;
        size_t o_og = need; need += in->origin ? align_up((size_t)n * 4) : 0;
        size_t o_cx = need; need += in->context ? align_up((size_t)n * 4) : 0;
        if (need > e->stage_in_bytes) {
            if (e->stage_in) hipFree(e->stage_in);
            e->stage_in = nullptr;
            HIP_TRY(hipMalloc(&e->stage_in, need));
            e->stage_in_bytes = need;
        }
        char* base = (char*)e->stage_in;
        auto up = [&](size_t off, const void* src, size_t bytes) -> const void* {
            if (!src || !bytes) return nullptr;
            hipMemcpyAsync(base + off, src, bytes, hipMemcpyHostToDevice, ss);
            return base + off;
        };
        b.res = (const uint32_t*)up(o_res, in->res_id, (size_t)n * 4);
        b.ts = (const int64_t*)up(o_ts, in->ts_ms, (size_t)n * 8);
        b.cnt = (const int32_t*)up(o_cnt, in->count, (size_t)n * 4);
        b.flags = (const uint8_t*)up(o_fl, in->flags, n);
        b.eref = (const int64_t*)up(o_er, in->entry_ref, in->entry_ref ? (size_t)n * 8 : 0);
        b.cts = (const int64_t*)up(o_ct, in->entry_ref ? in->create_ts : nullptr, (size_t)n * 8);
        b.nargs = (const uint8_t*)up(o_na, in->n_args, n);
        b.atag = (const uint8_t*)up(o_at, in->arg_tag, (size_t)n * in->arg_slots);
        b.abits = (const uint64_t*)up(o_ab, in->arg_bits, (size_t)n * in->arg_slots * 8);
        if (coll) {
            b.aoff = (const uint32_t*)up(o_eo, in->arg_elem_off, ((size_t)n * in->arg_slots + 1) * 4);
            b.etag = (const uint8_t*)up(o_et, in->elem_tag, in->n_elems);
            b.ebits = (const uint64_t*)up(o_eb, in->elem_bits, (size_t)in->n_elems * 8);
        }
        b.origin = (const uint32_t*)up(o_og, in->origin, (size_t)n * 4);
        b.ctx = (const uint32_t*)up(o_cx, in->context, (size_t)n * 4);
    } else {
        b.res = in->res_id; b.ts = in->ts_ms; b.cnt = in->count; b.flags = in->flags;
        b.eref = in->entry_ref; b.cts = in->entry_ref ? in->create_ts : nullptr;
        b.nargs = in->n_args; b.atag = in->arg_tag; b.abits = in->arg_bits;
        b.aoff = in->arg_elem_off; b.etag = in->elem_tag; b.ebits = in->elem_bits;
        b.origin = in->origin; b.ctx = in->context;
    }
    if (out->mem == SF_MEM_HOST) {
        size_t need = align_up((size_t)n) + align_up((size_t)n * 4) + align_up((size_t)n * 2);
        if (need > e->stage_out_bytes) {
            if (e->stage_out) hipFree(e->stage_out);
            e->stage_out = nullptr;
            HIP_TRY(hipMalloc(&e->stage_out, need));
            e->stage_out_bytes = need;
        }
        char* base = (char*)e->stage_out;
        dv.status = (uint8_t*)base;
        dv.wait = out->wait_ms ? (int32_t*)(base + align_up(n)) : nullptr;
        dv.rule = out->rule_idx ? (uint16_t*)(base + align_up(n) + align_up((size_t)n * 4)) : nullptr;
    } else {
        dv.status = out->status; dv.wait = out->wait_ms; dv.rule = out->rule_idx;
    }
    return SF_OK;
}

// Sort and decide the view [p, q) of a staged batch (a SystemRule sub-batch):
// its IN entries' system verdicts are in e->sys_mask, the verdicts of the
// events before it in dv; stream e->stream (the caller fenced the batch's
// staging).  v / dvv: the view, for the caller's ENTRY_NODE step.
static int decide_view(sf_engine* e, Work& w, int slot, DevState& stl, const DevBatch& b, const DevVerdicts& dv,
                       uint32_t p, uint32_t q, bool with_ox, DevBatch& v, DevVerdicts& dvv) {
    hipStream_t s = e->stream;
    v = b;
    v.n = q - p; v.base = p;
    v.res = b.res + p; v.ts = b.ts + p; v.cnt = b.cnt + p; v.flags = b.flags + p;
    v.eref = b.eref ? b.eref + p : nullptr; v.cts = b.cts ? b.cts + p : nullptr;
    v.nargs = b.nargs ? b.nargs + p : nullptr;
    v.atag = b.atag ? b.atag + p : nullptr; v.abits = b.abits ? b.abits + p : nullptr;
    v.origin = b.origin ? b.origin + p : nullptr; v.ctx = b.ctx ? b.ctx + p : nullptr;
    v.sys = e->sys_mask + p; v.vprev = dv.status + p;
    dvv = DevVerdicts{dv.status + p, dv.wait ? dv.wait + p : nullptr, dv.rule ? dv.rule + p : nullptr};
    hipError_t le = launch_sort(stl, w, v, e->cfg.shard_count, e->cfg.shard_index, e->key_bits, s, e->evs[slot], false);
    OxPlan plan{};
    if (le == hipSuccess && with_ox) {
        const int rc = prepare_origins(e, w, v, s, &plan);
        if (rc) return rc;
        stl.xtab = e->st.xtab; stl.xcap_mask = e->st.xcap_mask; stl.ax_cap = e->st.ax_cap;
    }
    if (le == hipSuccess)
        le = launch_decide(stl, w, v, dvv, s, e->serial ? s : e->stream2, e->serial ? s : e->stream3,
                           e->serial ? s : e->stream4, e->evs[slot], false, with_ox ? &plan : nullptr);
    if (le == hipSuccess && with_ox) w.ox_dirty = false;     // k_ox_reset enqueued
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("launch: ") + hipGetErrorString(le));
    return SF_OK;
}

// pre: launched on the sort stream after the batch's error flag is cleared and
// before its sort (sf_submit_packed's expansion of the packed words)
using PreSort = std::function<hipError_t(hipStream_t, int32_t*)>;
static int submit_core(sf_engine* e, const sf_event_batch* in, sf_verdicts* out, bool async,
                       const uint8_t* forced = nullptr, const PreSort* pre = nullptr) {
    if (!e || !in || !out || !out->status) return fail(SF_ERR_INVALID, "null argument");
    if (in->n == 0) return SF_OK;
    if (!in->res_id || !in->ts_ms || !in->count || !in->flags) return fail(SF_ERR_INVALID, "missing event array");
    if (in->n > e->cfg.max_batch) return fail(SF_ERR_CAPACITY, "batch larger than max_batch");
    if (in->arg_slots > SF_MAX_ARGS || (in->arg_slots && (!in->arg_tag || !in->arg_bits)))
        return fail(SF_ERR_INVALID, "bad arg arrays");
    if (in->arg_elem_off && in->n_elems && (!in->elem_tag || !in->elem_bits))
        return fail(SF_ERR_INVALID, "collection arguments without element arrays");
    // SystemRules read the node-wide ENTRY_NODE: a sharded engine decides them
    // only through the round protocol (sf_system_plan / sf_submit_forced)
    if (e->sys.check && e->cfg.shard_count > 1 && !forced)
        return fail(SF_ERR_UNSUPPORTED, "SystemRules on a sharded engine: use sf_system_plan + sf_submit_forced "
                                        "+ sf_entry_node_add (the node-wide round protocol)");
    const uint32_t n = in->n;
    DevBatch b{};
    b.n = n; b.arg_slots = in->arg_slots;
    hipStream_t s = e->stream, ss = e->serial ? e->stream : e->sstream;
    if ((in->origin || e->st.xmap) && !e->st.xtab) {
        // the first batch with origins: the origin-node pool (every entry with an
        // origin has one, ClusterBuilderSlot.java:107-110)
        { const int rc = drain(e); if (rc) return rc; }
        const int rc = ensure_aux(e);
        if (rc) return rc;
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    // the origin-node pass (sf_origin.hip) runs for batches with origins and
    // whenever rules read origin / context nodes (the xflow walk's node keys)
    const bool with_ox = in->origin || e->st.xmap;
    // asynchronous only for HBM-resident batches and verdicts, without SystemRules
    async = async && in->mem != SF_MEM_HOST && out->mem != SF_MEM_HOST && !e->sys.check && !forced;
    if (!async) { const int rc = drain(e); if (rc) return rc; }
    {   // room in the ParamFlow table for every key this batch can insert
        const uint64_t elems = in->arg_elem_off ? in->n_elems : 0;
        const int rc = param_reserve(e, ((uint64_t)n + elems) * e->p_kmax);
        if (rc) return rc;
    }
    if (async && !e->w_ready[1]) {                 // second Work set on first asynchronous use
        HIP_TRY(hipStreamSynchronize(s));
        const int rc = alloc_work(e, e->w[1]);
        if (rc) return rc;
        e->w_ready[1] = true;
    }
    const int slot = e->cur;
    Work& w = e->w[slot];
    if (e->used[slot]) {
        // the batch that last used this Work set (two submits ago) must be done:
        // its events and buffers are reused (sort(k) still overlaps decide(k-1))
        HIP_TRY(hipEventSynchronize(e->ev_done[slot]));
        acc_timing(e, slot);
    }
    DevVerdicts dv{};
    { const int rc = stage_batch(e, in, out, ss, b, dv); if (rc) return rc; }
    b.arg_stride = n;
    if (forced) {
        // the forced SystemRule verdicts of this (sub-)batch, planned node-wide
        if (!e->sys_mask) HIP_TRY(hipMalloc((void**)&e->sys_mask, e->cfg.max_batch));
        HIP_TRY(hipMemcpyAsync(e->sys_mask, forced, n, hipMemcpyHostToDevice, e->serial ? e->stream : e->sstream));
        b.sys = e->sys_mask;
    }
    if (e->sys.check && !forced) {
        // SystemRules couple every IN entry to the global ENTRY_NODE: the batch
        // is decided as a sequence of safe sub-batches (sf_system.h), each
        // planned on the exact ENTRY_NODE, then sorted / decided / reduced by
        // the ordinary pipeline.  One host round trip per sub-batch (its end q).
        if (!e->sys_plan) {
            HIP_TRY(hipMalloc((void**)&e->sys_plan, sizeof(SysPlanDev)));
            HIP_TRY(hipMalloc((void**)&e->sys_pa, SYS_PLAN_BLOCKS * sizeof(SysExitQ)));
            HIP_TRY(hipMalloc((void**)&e->sys_pb, SYS_PLAN_BLOCKS * sizeof(SysEntQ)));
            HIP_TRY(hipMalloc((void**)&e->sys_mask, e->cfg.max_batch));
        }
        if (!e->sys_ibuf && e->st.n_prule) HIP_TRY(hipMalloc((void**)&e->sys_ibuf, SYS_PLAN_CAP));
        HIP_TRY(hipMemsetAsync(w.err, 0, sizeof(int32_t), ss));
        if (pre) {
            const hipError_t pe = (*pre)(ss, w.err);
            if (pe != hipSuccess) return fail(SF_ERR_DEVICE, std::string("pre-sort: ") + hipGetErrorString(pe));
        }
        HIP_TRY(hipEventRecord(e->ev_sorted[slot], ss));
        HIP_TRY(hipStreamWaitEvent(s, e->ev_sorted[slot], 0));
        { const int rc = en_fence(e); if (rc) return rc; }
        DevState stl = e->st;
        stl.err = w.err;
        uint32_t p = 0, rounds = 0;
        while (p < n) {
            hipError_t le = sys_plan(stl, b, dv.status, e->sys_mask, e->sys, e->en, p, e->sys_plan, e->sys_pa,
                                     e->sys_pb, s, e->sys_ibuf);
            if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("system plan: ") + hipGetErrorString(le));
            uint32_t qi[2] = {0, 0};                        // q, inert entries planned
            static_assert(offsetof(SysPlanDev, n_inert) == offsetof(SysPlanDev, q) + 4, "q, n_inert adjacent");
            HIP_TRY(hipMemcpyAsync(qi, &e->sys_plan->q, 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            const uint32_t q = qi[0];
            if (q <= p || q > n) return fail(SF_ERR_DEVICE, "system planner made no progress");
            DevBatch v;
            DevVerdicts dvv;
            { const int rc = decide_view(e, w, slot, stl, b, dv, p, q, with_ox, v, dvv); if (rc) return rc; }
            // the system verdicts of the inert entries (ENTRY_NODE is still at p)
            if (le == hipSuccess && qi[1])
                le = sys_plan_fix(stl, b, dv, e->sys_mask, e->sys, p, q, e->sys_plan, e->sys_pa, e->sys_pb, s);
            if (le == hipSuccess) le = launch_entry_node(stl, v, dvv.status, e->en, e->en_acc, s);
            if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("launch: ") + hipGetErrorString(le));
            p = q;
            rounds++;
        }
        HIP_TRY(hipEventRecord(e->ev_core[slot], s));
        HIP_TRY(hipEventRecord(e->ev_done[slot], s));
    HIP_TRY(hipEventRecord(e->ev_end[slot], s));
        e->used[slot] = true;
        e->last = slot;
        e->stats.n_events = n;
        e->stats.n_launches++;
        e->stats.sys_rounds += rounds;
        if (out->mem == SF_MEM_HOST) {
            HIP_TRY(hipMemcpyAsync(out->status, dv.status, n, hipMemcpyDeviceToHost, s));
            if (dv.wait) HIP_TRY(hipMemcpyAsync(out->wait_ms, dv.wait, (size_t)n * 4, hipMemcpyDeviceToHost, s));
            if (dv.rule) HIP_TRY(hipMemcpyAsync(out->rule_idx, dv.rule, (size_t)n * 2, hipMemcpyDeviceToHost, s));
        }
        int32_t err = 0;
        HIP_TRY(hipMemcpyAsync(&err, w.err, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (err) return fail(err, err == SF_ERR_CAPACITY ? "capacity exceeded (param table, or the origin / context node pool: aux_capacity)"
                                                         : "invalid batch (resource outside shard or bad entry_ref)");
        return SF_OK;
    }
    // sort phase on the sort stream, into this batch's Work set (after the
    // decide phase of the batch that used it last)
    if (e->used[slot]) HIP_TRY(hipStreamWaitEvent(ss, e->ev_done[slot], 0));
    HIP_TRY(hipMemsetAsync(w.err, 0, sizeof(int32_t), ss));
    if (pre) {
        const hipError_t pe = (*pre)(ss, w.err);
        if (pe != hipSuccess) return fail(SF_ERR_DEVICE, std::string("pre-sort: ") + hipGetErrorString(pe));
    }
    DevState stl = e->st;
    stl.err = w.err;
    hipError_t le = launch_sort(stl, w, b, e->cfg.shard_count, e->cfg.shard_index, e->key_bits, ss, e->evs[slot], e->timing);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("launch: ") + hipGetErrorString(le));
    OxPlan plan{};
    if (with_ox) {
        const int rc = prepare_origins(e, w, b, ss, &plan);
        if (rc) return rc;
        stl.xtab = e->st.xtab; stl.xcap_mask = e->st.xcap_mask; stl.ax_cap = e->st.ax_cap;
    }
    HIP_TRY(hipEventRecord(e->ev_sorted[slot], ss));
    // decide phase in batch order on the main streams
    HIP_TRY(hipStreamWaitEvent(s, e->ev_sorted[slot], 0));
    // an asynchronous batch's verdict scatter and ENTRY_NODE update run on the
    // ENTRY_NODE stream, beside the next batch's decide phase
    const bool side = !forced && async && !e->serial && e->side_mode != 0;
    le = launch_decide(stl, w, b, dv, s, e->serial ? s : e->stream2, e->serial ? s : e->stream3,
                       e->serial ? s : e->stream4, e->evs[slot], e->timing,
                       with_ox ? &plan : nullptr, false, side ? e->enstream : nullptr);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("launch: ") + hipGetErrorString(le));
    if (with_ox) w.ox_dirty = false;                                  // k_ox_reset enqueued
    // ENTRY_NODE: every IN event's StatisticSlot updates (after the verdicts, stream
    // order); under the round protocol the node-wide stream updates it (sf_entry_node_add)
    if (side) {
        // asynchronous: on the side stream after the scatter.  The Work set is
        // free after the scatter (ev_done: the sort of the batch after next waits
        // for it), the batch k_entry_acc reads after the update (ev_end)
        HIP_TRY(hipEventRecord(e->ev_core[slot], e->enstream));
        HIP_TRY(hipEventRecord(e->ev_done[slot], e->enstream));
        le = launch_entry_node(stl, b, dv.status, e->en, e->en_acc, e->enstream);
        if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("entry node: ") + hipGetErrorString(le));
        HIP_TRY(hipEventRecord(e->ev_end[slot], e->enstream));
        HIP_TRY(hipEventRecord(e->ev_en, e->enstream));
        e->en_async = true;
    } else {
        if (!forced) {
            { const int rc = en_fence(e); if (rc) return rc; }
            le = launch_entry_node(stl, b, dv.status, e->en, e->en_acc, s);
            if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("entry node: ") + hipGetErrorString(le));
        }
        HIP_TRY(hipEventRecord(e->ev_core[slot], s));
        HIP_TRY(hipEventRecord(e->ev_done[slot], s));
    HIP_TRY(hipEventRecord(e->ev_end[slot], s));
    }
    e->used[slot] = true;
    e->timed[slot] = e->timing;
    e->last = slot;
    e->stats.n_events = n;
    e->stats.n_launches++;
    if (async) {
        e->pending |= 1u << slot;
        e->cur ^= 1;
        return SF_OK;
    }
    if (out->mem == SF_MEM_HOST) {
        HIP_TRY(hipMemcpyAsync(out->status, dv.status, n, hipMemcpyDeviceToHost, s));
        if (dv.wait) HIP_TRY(hipMemcpyAsync(out->wait_ms, dv.wait, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        if (dv.rule) HIP_TRY(hipMemcpyAsync(out->rule_idx, dv.rule, (size_t)n * 2, hipMemcpyDeviceToHost, s));
    }
    int32_t err = 0;
    uint32_t nseg = 0;
    HIP_TRY(hipMemcpyAsync(&err, w.err, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&nseg, w.n_seg, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    e->stats.n_segments = nseg;
    acc_timing(e, slot);
    if (err) return fail(err, err == SF_ERR_CAPACITY ? "capacity exceeded (param table, or the origin / context node pool: aux_capacity)"
                                                     : "invalid batch (resource outside shard or bad entry_ref)");
    return SF_OK;
}

int sf_submit(sf_engine* e, const sf_event_batch* in, sf_verdicts* out) {
    if (!e) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    return submit_core(e, in, out, false);
}

int sf_submit_async(sf_engine* e, const sf_event_batch* in, sf_verdicts* out) {
    if (!e) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    return submit_core(e, in, out, true);
}

// ---------------------------------------------------------------- compact batches
// sf_packed_batch: the packed words (and the sparse exit / count arrays) go to
// the Work set's device stage on the H2D stream, are expanded to the SoA batch
// on the sort stream, decided by submit_core (asynchronously when asked), and
// the verdicts come back on the D2H stream once the batch is decided.
// the rest of a sparse batch's lists (beyond the prefetch) and their lengths, once its copies are done
static int sparse_complete(sf_engine::PkStage& pk) {
    const uint32_t nw = pk.sp_counts[0], nr = pk.sp_counts[1], pre = pk.sp.prefetch;
    if (nw > pre) HIP_TRY(hipMemcpy(pk.sp.waits + pre, pk.sp_wl + pre, (size_t)(nw - pre) * 8, hipMemcpyDeviceToHost));
    if (nr > pre) HIP_TRY(hipMemcpy(pk.sp.rules + pre, pk.sp_rl + pre, (size_t)(nr - pre) * 8, hipMemcpyDeviceToHost));
    pk.sp.counts[0] = nw; pk.sp.counts[1] = nr;
    pk.sparse = false;
    return SF_OK;
}

static int submit_packed(sf_engine* e, const sf_packed_batch* in, sf_verdicts* out, bool async,
                         const sf_sparse_verdicts* sp = nullptr) {
    if (!e || !in || !out || !out->status) return fail(SF_ERR_INVALID, "null argument");
    if (sp && (!sp->waits || !sp->rules || !sp->counts)) return fail(SF_ERR_INVALID, "null sparse list");
    if (in->n == 0) return SF_OK;
    const bool narrow = !in->ev && in->ev4;
    if ((!in->ev && !narrow) || (in->n_exit && !in->exit_ref) || (in->n_count_ext && !in->count_ext) ||
        (narrow && (!in->ms_end || in->n_ms == 0)))
        return fail(SF_ERR_INVALID, "missing packed arrays");
    if (narrow && in->n_ms > SF_PK4_MAX_MS) return fail(SF_ERR_INVALID, "narrow packed batch spans more than 2^20 ms");
    if (in->n > e->cfg.max_batch) return fail(SF_ERR_CAPACITY, "batch larger than max_batch");
    std::lock_guard<std::mutex> lk(e->mu);
    const uint32_t n = in->n;
    const bool host_in = in->mem == SF_MEM_HOST, host_out = sp || out->mem == SF_MEM_HOST;
    if (!e->h2d) {
        HIP_TRY(hipStreamCreateWithFlags(&e->h2d, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&e->d2h, hipStreamNonBlocking));
        for (auto& p : e->pk) {
            HIP_TRY(hipEventCreateWithFlags(&p.h2d, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&p.d2h, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&p.consumed, hipEventDisableTiming));
            HIP_TRY(hipHostMalloc((void**)&p.err_host, 4, hipHostMallocDefault));
            *p.err_host = 0;
            HIP_TRY(hipHostMalloc((void**)&p.sp_counts, 8, hipHostMallocDefault));
        }
    }
    // (submit_core decides asynchronously only without SystemRules; the slot it takes is e->cur)
    const bool core_async = async && !e->sys.check;
    if (!core_async) { const int rc = drain(e); if (rc) return rc; }
    const int slot = e->cur;
    auto& pk = e->pk[slot];
    // The slot's staging buffer: its packed inputs are free once the batch
    // before in this slot has expanded them (early in its sort phase), its
    // expanded arrays once that batch is decided (submit_core waits for it
    // before the expansion), its staged verdicts once their D2H copy is done.
    // All are waited for on the device, so the H2D of batch k+1 follows the
    // H2D of batch k back to back and overlaps the decision of k and the D2H
    // of k-1; the host blocks only to reallocate.
    const size_t N = e->cfg.max_batch;
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += align_up(bytes); return o; };
    const size_t o_ev = take(N * 8), o_xr = take(N * 8), o_xc = take(N * 8), o_ce = take(N * 4), o_og = take(N * 4);
    const size_t o_res = take(N * 4), o_ts = take(N * 8), o_cnt = take(N * 4), o_fl = take(N), o_er = take(N * 8);
    const size_t o_ct = take(N * 8), o_tc = take((N / 4096 + 2) * 8);
    const size_t o_st = take(N), o_wt = take(N * 4), o_ru = take(N * 2);
    const size_t o_wl = sp ? take(N * 8) : 0, o_rl = sp ? take(N * 8) : 0, o_sc = sp ? take(16) : 0;
    const size_t o_ms = narrow ? take((size_t)SF_PK4_MAX_MS * 4) : 0;   // (the narrow words use o_ev's room)
    if (pk.bytes < off) {
        if (e->used[slot]) HIP_TRY(hipEventSynchronize(e->ev_end[slot]));
        if (pk.consumed_pending) { HIP_TRY(hipEventSynchronize(pk.consumed)); pk.consumed_pending = false; }
        if (pk.d2h_pending) { HIP_TRY(hipEventSynchronize(pk.d2h)); pk.d2h_pending = false; }
        if (pk.buf) hipFree(pk.buf);
        pk.buf = nullptr; pk.bytes = 0;
        HIP_TRY(hipMalloc((void**)&pk.buf, off));
        pk.bytes = off;
    }
    char* B = pk.buf;
    hipStream_t ss = e->serial ? e->stream : e->sstream;
    const uint64_t* ev = in->ev; const int64_t* xr = in->exit_ref; const int64_t* xc = in->exit_cts;
    const uint32_t* ev4 = narrow ? in->ev4 : nullptr; const uint32_t* mse = narrow ? in->ms_end : nullptr;
    const uint32_t n_ms = narrow ? in->n_ms : 0;
    const int32_t* ce = in->count_ext; const uint32_t* og = in->origin;
    if (host_in) {
        hipStream_t h = e->serial ? e->stream : e->h2d;
        if (pk.consumed_pending) HIP_TRY(hipStreamWaitEvent(h, pk.consumed, 0));
        if (narrow) {
            HIP_TRY(hipMemcpyAsync(B + o_ev, in->ev4, (size_t)n * 4, hipMemcpyHostToDevice, h));
            HIP_TRY(hipMemcpyAsync(B + o_ms, in->ms_end, (size_t)n_ms * 4, hipMemcpyHostToDevice, h));
            ev4 = (const uint32_t*)(B + o_ev);
            mse = (const uint32_t*)(B + o_ms);
        } else {
            HIP_TRY(hipMemcpyAsync(B + o_ev, in->ev, (size_t)n * 8, hipMemcpyHostToDevice, h));
            ev = (const uint64_t*)(B + o_ev);
        }
        if (in->n_exit) {
            HIP_TRY(hipMemcpyAsync(B + o_xr, in->exit_ref, (size_t)in->n_exit * 8, hipMemcpyHostToDevice, h));
            xr = (const int64_t*)(B + o_xr);
            if (in->exit_cts) {
                HIP_TRY(hipMemcpyAsync(B + o_xc, in->exit_cts, (size_t)in->n_exit * 8, hipMemcpyHostToDevice, h));
                xc = (const int64_t*)(B + o_xc);
            }
        }
        if (in->n_count_ext) {
            HIP_TRY(hipMemcpyAsync(B + o_ce, in->count_ext, (size_t)in->n_count_ext * 4, hipMemcpyHostToDevice, h));
            ce = (const int32_t*)(B + o_ce);
        }
        if (in->origin) {
            HIP_TRY(hipMemcpyAsync(B + o_og, in->origin, (size_t)n * 4, hipMemcpyHostToDevice, h));
            og = (const uint32_t*)(B + o_og);
        }
        HIP_TRY(hipEventRecord(pk.h2d, h));
        HIP_TRY(hipStreamWaitEvent(ss, pk.h2d, 0));
    }
    const bool exits = in->n_exit != 0;
    const int64_t base = in->ts_base;
    const uint32_t n_exit = in->n_exit, n_cext = in->n_count_ext;
    const hipEvent_t consumed = pk.consumed;
    const PreSort expand = [=](hipStream_t st_, int32_t* err) {
        const hipError_t le = launch_pk_expand(ev, ev4, mse, n_ms, xr, xc, ce, base, n, n_exit, n_cext, (uint2*)(B + o_tc),
                                               (uint32_t*)(B + o_res), (int64_t*)(B + o_ts), (int32_t*)(B + o_cnt),
                                               (uint8_t*)(B + o_fl), (int64_t*)(B + o_er),
                                               exits ? (int64_t*)(B + o_ct) : nullptr, err, st_);
        if (le != hipSuccess) return le;
        return hipEventRecord(consumed, st_);
    };
    if (pk.d2h_pending) { HIP_TRY(hipStreamWaitEvent(ss, pk.d2h, 0)); pk.d2h_pending = false; }
    sf_event_batch eb{};
    eb.n = n; eb.mem = SF_MEM_DEVICE;
    eb.res_id = (const uint32_t*)(B + o_res); eb.ts_ms = (const int64_t*)(B + o_ts);
    eb.count = (const int32_t*)(B + o_cnt); eb.flags = (const uint8_t*)(B + o_fl);
    eb.entry_ref = exits ? (const int64_t*)(B + o_er) : nullptr;
    eb.create_ts = exits ? (const int64_t*)(B + o_ct) : nullptr;
    eb.origin = og;
    sf_verdicts dv{};
    dv.mem = SF_MEM_DEVICE;
    dv.status = host_out ? (uint8_t*)(B + o_st) : out->status;
    dv.wait_ms = (sp || out->wait_ms) ? (host_out ? (int32_t*)(B + o_wt) : out->wait_ms) : nullptr;
    dv.rule_idx = (sp || out->rule_idx) ? (host_out ? (uint16_t*)(B + o_ru) : out->rule_idx) : nullptr;
    // (the expansion rewrites the arrays the ENTRY_NODE update of this slot's
    // previous batch reads)
    if (e->used[slot]) HIP_TRY(hipStreamWaitEvent(ss, e->ev_end[slot], 0));
    const int rc = submit_core(e, &eb, &dv, core_async, nullptr, &expand);
    if (rc) return rc;
    pk.consumed_pending = true;
    if (host_out) {
        hipStream_t d = e->serial ? e->stream : e->d2h;
        HIP_TRY(hipStreamWaitEvent(d, e->ev_core[slot], 0));
        HIP_TRY(hipMemcpyAsync(out->status, dv.status, n, hipMemcpyDeviceToHost, d));
        pk.sparse = sp != nullptr;
        if (sp) {
            // 1 byte per event plus the exceptions: the nonzero waits / rule indices
            // compacted on the device, their first `prefetch` back with the statuses
            unsigned long long* wl = (unsigned long long*)(B + o_wl);
            unsigned long long* rl = (unsigned long long*)(B + o_rl);
            uint32_t* sc = (uint32_t*)(B + o_sc);
            HIP_TRY(launch_sparse_verdicts(dv.wait_ms, dv.rule_idx, n, wl, rl, sc, d));
            HIP_TRY(hipMemcpyAsync(pk.sp_counts, sc, 8, hipMemcpyDeviceToHost, d));
            const size_t pre = std::min<size_t>(sp->prefetch, n) * 8;
            if (pre) {
                HIP_TRY(hipMemcpyAsync(sp->waits, wl, pre, hipMemcpyDeviceToHost, d));
                HIP_TRY(hipMemcpyAsync(sp->rules, rl, pre, hipMemcpyDeviceToHost, d));
            }
            pk.sp = *sp; pk.sp_wl = wl; pk.sp_rl = rl;
        } else {
            if (out->wait_ms) HIP_TRY(hipMemcpyAsync(out->wait_ms, dv.wait_ms, (size_t)n * 4, hipMemcpyDeviceToHost, d));
            if (out->rule_idx) HIP_TRY(hipMemcpyAsync(out->rule_idx, dv.rule_idx, (size_t)n * 2, hipMemcpyDeviceToHost, d));
        }
        if (core_async) HIP_TRY(hipMemcpyAsync(pk.err_host, e->w[slot].err, 4, hipMemcpyDeviceToHost, d));
        HIP_TRY(hipEventRecord(pk.d2h, d));
        pk.d2h_pending = true;
        pk.out_status = core_async ? out->status : nullptr;
        if (!core_async) {
            HIP_TRY(hipEventSynchronize(pk.d2h));
            pk.d2h_pending = false;
            if (sp) { const int rc = sparse_complete(pk); if (rc) return rc; }
        }
    }
    return SF_OK;
}

int sf_submit_packed(sf_engine* e, const sf_packed_batch* in, sf_verdicts* out) {
    return submit_packed(e, in, out, false);
}
int sf_submit_packed_async(sf_engine* e, const sf_packed_batch* in, sf_verdicts* out) {
    return submit_packed(e, in, out, true);
}

// Wait for ONE asynchronous packed batch: the one whose host verdicts go to
// out->status (its D2H copy, which follows its decision on the device); the
// batch submitted after it stays in flight.  Its error flag came back with the
// verdicts.  A batch already collected (by sf_sync, a rule reload's drain, or
// an earlier call) has nothing left to wait for: SF_OK.
static int sync_packed(sf_engine* e, const uint8_t* status) {
    for (int k = 0; k < 2; k++) {
        auto& pk = e->pk[k];
        if (!status || pk.out_status != status) continue;
        // (a drain may have waited for its copies already; its error stays this batch's)
        if (pk.d2h_pending) HIP_TRY(hipEventSynchronize(pk.d2h));
        pk.d2h_pending = false;
        pk.out_status = nullptr;
        e->pending &= ~(1u << k);          // checked here, not again by sf_sync
        if (pk.sparse) { const int rc = sparse_complete(pk); if (rc) return rc; }
        const int32_t err = *pk.err_host;
        if (err) return fail(err, err == SF_ERR_CAPACITY ? "capacity exceeded (param table, or the origin / context node pool: aux_capacity)"
                                                         : "invalid batch (resource outside shard or bad entry_ref)");
        return SF_OK;
    }
    return SF_OK;
}

int sf_sync_packed(sf_engine* e, const sf_verdicts* out) {
    if (!e || !out || !out->status) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    return sync_packed(e, out->status);
}

int sf_submit_packed_sparse_async(sf_engine* e, const sf_packed_batch* in, sf_sparse_verdicts* out) {
    if (!e || !in || !out || !out->status) return fail(SF_ERR_INVALID, "null argument");
    sf_verdicts v{};
    v.mem = SF_MEM_HOST; v.status = out->status;
    return submit_packed(e, in, &v, true, out);
}

int sf_sync_packed_sparse(sf_engine* e, const sf_sparse_verdicts* out) {
    if (!e || !out || !out->status) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    return sync_packed(e, out->status);
}

// ---------------------------------------------------------------- node-wide SystemRule rounds
// (sentinel_flow.h: sf_system_plan / sf_submit_forced / sf_entry_node_add)
int sf_submit_forced(sf_engine* e, const sf_event_batch* in, sf_verdicts* out, const uint8_t* sys_mask) {
    if (!e || !in || !out || !sys_mask) return fail(SF_ERR_INVALID, "null argument");
    if (in->mem != SF_MEM_HOST) return fail(SF_ERR_INVALID, "sf_submit_forced takes host arrays");
    std::lock_guard<std::mutex> lk(e->mu);
    return submit_core(e, in, out, false, sys_mask);
}

// stage host IN-event arrays (ts, count, flags, entry_ref, create_ts) + optional
// verdicts at a device scratch (StageBuf); DevBatch over them.  keep: the
// scratch already holds these event arrays (a later round of the same merged
// stream): only the verdicts are copied.
static int stage_in_events(sf_engine* e, StageBuf& sb, const sf_event_batch* in, const uint8_t* status,
                           uint32_t n_status, DevBatch& b, uint8_t** dstatus, bool keep = false) {
    const uint32_t n = in->n;
    size_t need = 0;
    const size_t o_ts = need; need += align_up((size_t)n * 8);
    const size_t o_cnt = need; need += align_up((size_t)n * 4);
    const size_t o_fl = need; need += align_up((size_t)n);
    const size_t o_er = need; need += align_up((size_t)n * 8);
    const size_t o_ct = need; need += align_up((size_t)n * 8);
    const size_t o_st = need; need += align_up((size_t)n + 1);
    const void* key[5] = {in->ts_ms, in->count, in->flags, in->entry_ref, in->create_ts};
    // the same host arrays as the round before: a cheap fingerprint of their
    // contents must match too (the contract is that the caller only appends
    // verdicts between rounds; an edited event array is restaged, not trusted)
    const int64_t fp[3] = {n ? in->ts_ms[0] : 0, n ? in->ts_ms[n - 1] : 0, n ? (int64_t)in->flags[0] : 0};
    keep = keep && sb.p && sb.n == n && std::equal(key, key + 5, sb.key) && std::equal(fp, fp + 3, sb.fp) &&
           need <= sb.bytes;
    if (need > sb.bytes) {
        if (sb.p) hipFree(sb.p);
        sb.p = nullptr; sb.bytes = 0; sb.n = 0;
        HIP_TRY(hipMalloc(&sb.p, need));
        sb.bytes = need;
    }
    char* base = (char*)sb.p;
    hipStream_t s = e->stream;
    if (!keep) {
        HIP_TRY(hipMemcpyAsync(base + o_ts, in->ts_ms, (size_t)n * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(base + o_cnt, in->count, (size_t)n * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(base + o_fl, in->flags, n, hipMemcpyHostToDevice, s));
        if (in->entry_ref) HIP_TRY(hipMemcpyAsync(base + o_er, in->entry_ref, (size_t)n * 8, hipMemcpyHostToDevice, s));
        if (in->create_ts) HIP_TRY(hipMemcpyAsync(base + o_ct, in->create_ts, (size_t)n * 8, hipMemcpyHostToDevice, s));
        std::copy(key, key + 5, sb.key);
        std::copy(fp, fp + 3, sb.fp);
        sb.n = n;
    }
    if (status && n_status) {
        // a continued stream: the verdicts staged for the round before are
        // final (the caller only appends), only the new ones are copied
        const uint32_t from = (keep && sb.st_src == status && sb.st_n <= n_status) ? sb.st_n : 0;
        if (n_status > from)
            HIP_TRY(hipMemcpyAsync(base + o_st + from, status + from, n_status - from, hipMemcpyHostToDevice, s));
        sb.st_src = status; sb.st_n = n_status;
    } else {
        sb.st_src = nullptr; sb.st_n = 0;
    }
    b = DevBatch{};
    b.n = n;
    b.ts = (const int64_t*)(base + o_ts); b.cnt = (const int32_t*)(base + o_cnt); b.flags = (const uint8_t*)(base + o_fl);
    b.eref = in->entry_ref ? (const int64_t*)(base + o_er) : nullptr;
    b.cts = in->create_ts ? (const int64_t*)(base + o_ct) : nullptr;
    *dstatus = (uint8_t*)(base + o_st);
    return SF_OK;
}

// ---------------------------------------------------------------- sharded SystemRules: the per-window exchange
// (sf_sysx.h; sentinel_flow.h sf_submit_node).  All ranks run the same number
// of all-gathers in the same order: every decision that shapes the loop is
// made from exchanged data (plan windows, the plan's levels and q).  RCCL:
// device buffers into d_recv; a callback: host buffers, the result in sx_hrecv.
static int sx_exchange(sf_engine* e, sf_allgather_fn fn, void* ctx, const int64_t* d_send, int64_t* d_recv,
                       size_t words) {
    const size_t bytes = words * 8, N = e->cfg.shard_count;
    hipStream_t s = e->stream;
    if (!fn) {
        const ncclResult_t r = ncclAllGather(d_send, d_recv, bytes, ncclInt8, e->comm, s);
        if (r != ncclSuccess) return fail(SF_ERR_DEVICE, std::string("ncclAllGather: ") + ncclGetErrorString(r));
        return SF_OK;
    }
    e->sx_hsend.resize(words);
    e->sx_hrecv.resize(words * N);
    HIP_TRY(hipMemcpyAsync(e->sx_hsend.data(), d_send, bytes, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (fn(ctx, e->sx_hsend.data(), e->sx_hrecv.data(), bytes) != 0) return fail(SF_ERR_DEVICE, "all-gather callback failed");
    return SF_OK;                               // (every rank's message in sx_hrecv; the plan step reads it there)
}

static int sx_recv_reserve(sf_engine* e, size_t words) {
    if (e->sx_recv_words >= words) return SF_OK;
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->sx_recv) hipFree(e->sx_recv);
    e->sx_recv = nullptr; e->sx_recv_words = 0;
    HIP_TRY(hipMalloc((void**)&e->sx_recv, words * 8));
    e->sx_recv_words = words;
    return SF_OK;
}

int sf_submit_node(sf_engine* e, const sf_event_batch* in, const int64_t* seq, sf_verdicts* out,
                   sf_allgather_fn allgather, void* ctx) {
    if (!e || !in || !out) return fail(SF_ERR_INVALID, "null argument");
    if (in->n && (!seq || !out->status || !in->res_id || !in->ts_ms || !in->count || !in->flags))
        return fail(SF_ERR_INVALID, "missing event array");
    if (in->n > e->cfg.max_batch) return fail(SF_ERR_CAPACITY, "batch larger than max_batch");
    if (in->arg_slots > SF_MAX_ARGS || (in->arg_slots && (!in->arg_tag || !in->arg_bits)))
        return fail(SF_ERR_INVALID, "bad arg arrays");
    if (in->arg_elem_off && in->n_elems && (!in->elem_tag || !in->elem_bits))
        return fail(SF_ERR_INVALID, "collection arguments without element arrays");
    std::lock_guard<std::mutex> lk(e->mu);
    if (!e->sys.check) return in->n ? submit_core(e, in, out, false) : SF_OK;   // nothing node-wide to decide
    if (!sx_rule_ok(e->sys))
        return fail(SF_ERR_UNSUPPORTED, "SystemRule with thread / RT / BBR checks: the event all-gather protocol "
                                        "(sf_system_plan + sf_submit_forced + sf_entry_node_add)");
    if (!allgather && !e->comm) return fail(SF_ERR_INVALID, "no exchange: sf_comm_init or an all-gather callback");
    { const int rc = drain(e); if (rc) return rc; }
    const uint32_t n = in->n, N = e->cfg.shard_count;
    hipStream_t s = e->stream;
    if (!e->sx_msg) {
        HIP_TRY(hipMalloc((void**)&e->sx_msg, SX_WORDS * 8));
        HIP_TRY(hipMalloc((void**)&e->sx_ibuf, e->cfg.max_batch));
    }
    if (!e->sys_mask) HIP_TRY(hipMalloc((void**)&e->sys_mask, e->cfg.max_batch));
    { const int rc = sx_recv_reserve(e, (size_t)N * SX_WORDS); if (rc) return rc; }
    const bool with_ox = in->origin || e->st.xmap;
    if (with_ox && !e->st.xtab) { const int rc = ensure_aux(e); if (rc) return rc; HIP_TRY(hipStreamSynchronize(s)); }
    {
        const uint64_t elems = in->arg_elem_off ? in->n_elems : 0;
        const int rc = param_reserve(e, ((uint64_t)n + elems) * e->p_kmax);
        if (rc) return rc;
    }
    const int slot = e->cur;
    Work& w = e->w[slot];
    if (e->used[slot]) { HIP_TRY(hipEventSynchronize(e->ev_done[slot])); acc_timing(e, slot); }
    DevBatch b{};
    b.n = n; b.arg_slots = in->arg_slots;
    DevVerdicts dv{};
    { const int rc = stage_batch(e, in, out, s, b, dv); if (rc) return rc; }
    b.arg_stride = n;
    const int64_t* dseq = seq;
    if (in->mem == SF_MEM_HOST && n) {
        if (!e->sx_seq) HIP_TRY(hipMalloc((void**)&e->sx_seq, (size_t)e->cfg.max_batch * 8));
        HIP_TRY(hipMemcpyAsync(e->sx_seq, seq, (size_t)n * 8, hipMemcpyHostToDevice, s));
        dseq = e->sx_seq;
    }
    HIP_TRY(hipMemsetAsync(w.err, 0, sizeof(int32_t), s));
    DevState stl = e->st;
    stl.err = w.err;
    SxArgs a{};
    a.b = b; a.seq = dseq; a.msg = e->sx_msg;
    a.r = e->sys; a.S = stl.S; a.wl = stl.wl; a.interval = stl.interval; a.max_rt = stl.max_rt;
    a.interval_sec = stl.interval / 1000.0; a.st = stl;
    a.ibuf = e->st.n_prule ? e->sx_ibuf : nullptr;
    a.g = std::__gcd((int64_t)stl.wl, (int64_t)1000);
    // every rank's message on the host: the plan step runs there (one sync per level)
    auto gather = [&](const int64_t* d_send, size_t words, std::vector<int64_t>& h) -> int {
        const int rc = sx_exchange(e, allgather, ctx, d_send, e->sx_recv, words);
        if (rc) return rc;
        if (allgather) { h.assign(e->sx_hrecv.begin(), e->sx_hrecv.begin() + words * N); return SF_OK; }
        h.resize(words * N);
        HIP_TRY(hipMemcpyAsync(h.data(), e->sx_recv, words * N * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        return SF_OK;
    };
    // ---- per batch: the node's plan windows (cells of g ms) and where each starts
    int64_t C0 = INT64_MAX, C1 = INT64_MIN, seq_end = INT64_MIN;
    bool neg = false;
    std::vector<int64_t> h;
    {
        HIP_TRY(sx_header(a, e->sx_msg, s));
        { const int rc = gather(e->sx_msg, 5, h); if (rc) return rc; }
        for (uint32_t k = 0; k < N; k++) {
            const int64_t* x = &h[(size_t)k * 5];
            if (!x[4]) continue;
            C0 = std::min(C0, x[0]); C1 = std::max(C1, x[1]); seq_end = std::max(seq_end, x[2]);
            neg |= x[3] != 0;
        }
    }
    if (neg) return fail(SF_ERR_UNSUPPORTED, "an IN entry with acquireCount < 0: the event all-gather protocol");
    std::vector<int64_t> wseq;                  // start sequence number of each non-empty plan window
    std::vector<int64_t> wkey;                  // its index (cell - C0)
    if (seq_end != INT64_MIN) {
        const uint64_t nw = (uint64_t)(C1 - C0) + 1;
        if (nw > (1u << 22)) return fail(SF_ERR_CAPACITY, "batch spans too many plan windows");
        { const int rc = sx_recv_reserve(e, (size_t)N * nw); if (rc) return rc; }
        int64_t* wbuf = nullptr;
        HIP_TRY(hipMalloc((void**)&wbuf, nw * 8));
        a.c0 = C0;
        const hipError_t le = sx_winfirst(a, wbuf, (uint32_t)nw, s);
        const int rc = le == hipSuccess ? gather(wbuf, nw, h)
                                        : fail(SF_ERR_DEVICE, std::string("plan windows: ") + hipGetErrorString(le));
        hipFree(wbuf);
        if (rc) return rc;
        for (uint64_t k = 0; k < nw; k++) {
            int64_t m = INT64_MAX;
            for (uint32_t r = 0; r < N; r++) m = std::min(m, h[(size_t)r * nw + k]);
            if (m != INT64_MAX) { wseq.push_back(m); wkey.push_back((int64_t)k); }
        }
    }
    a.c0 = C0;
    // ENTRY_NODE, identical on every rank, advanced on the host by the node's deltas (no
    // kernel reads it while the batch is decided: the system verdicts are forced)
    EntryNode enh;
    HIP_TRY(hipMemcpyAsync(&enh, e->en, sizeof enh, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    uint32_t* d_lq = (uint32_t*)e->sx_recv;     // (sx_locate's result: the recv buffer is free then)
    // ---- rounds
    HIP_TRY(sx_nodelta(e->sx_msg, s));
    int64_t sp = wseq.empty() ? INT64_MAX : wseq[0];
    uint32_t lp = 0, rounds = 0;
    size_t j = 0;
    uint64_t levels = 0;
    for (;;) {
        const bool fin = wseq.empty() || sp >= seq_end;
        while (!fin && j + 1 < wseq.size() && wseq[j + 1] <= sp) j++;
        const int64_t lo = fin ? 0 : sp, hi = fin ? 0 : (j + 1 < wseq.size() ? wseq[j + 1] : seq_end);
        const int64_t wstart = fin ? 0 : (C0 + wkey[j]) * a.g;
        SxPlan hp;
        sx_begin(&hp, lo, hi);
        for (int level = 0;; level++) {
            const hipError_t le = sx_stats(a, hp, lp, level == 0, s);
            if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("exchange stats: ") + hipGetErrorString(le));
            { const int rc = gather(e->sx_msg, SX_WORDS, h); if (rc) return rc; }
            levels++;
            if (level == 0) {
                // the node's ENTRY_NODE contribution of the last sub-batch (its plan window is the key)
                int64_t key = -1;
                for (uint32_t k = 0; k < N; k++) key = std::max(key, h[(size_t)k * SX_WORDS + SXD_KEY]);
                if (key >= 0) {
                    const int64_t W = (C0 + key) * a.g;
                    sx_apply_delta(h.data(), (int)N, &enh, W - W % a.wl, a.S, a.wl, W - W % 1000, a.max_rt);
                }
                hp.P = sys_base(enh.second, a.S, a.wl, a.interval, a.max_rt, enh.threads, wstart).P;
            }
            sx_reduce(h.data(), (int)N, &hp, a.r, a.interval_sec);
            if (hp.done) break;
            if (level > 64) return fail(SF_ERR_DEVICE, "exchange plan did not converge");
        }
        if (fin) break;
        if (hp.q <= sp || hp.q > hi) return fail(SF_ERR_DEVICE, "exchange plan made no progress");
        uint32_t lq;
        if (in->mem == SF_MEM_HOST) {
            lq = (uint32_t)(std::lower_bound(seq + lp, seq + n, hp.q) - seq);
        } else {
            HIP_TRY(sx_locate(a, lp, hp.q, d_lq, s));
            HIP_TRY(hipMemcpyAsync(&lq, d_lq, 4, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
        }
        if (lq < lp || lq > n) return fail(SF_ERR_DEVICE, "exchange plan: bad local range");
        if (lq > lp) {
            hipError_t le = sx_mask(a, e->sys_mask, lp, lq, hp.P, s);
            if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("exchange mask: ") + hipGetErrorString(le));
            DevBatch v;
            DevVerdicts dvv;
            { const int rc = decide_view(e, w, slot, stl, b, dv, lp, lq, with_ox, v, dvv); if (rc) return rc; }
            le = launch_entry_delta(stl, v, dvv.status, e->en_acc, e->sx_msg, wkey[j], s);
            if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("exchange delta: ") + hipGetErrorString(le));
        } else {
            HIP_TRY(sx_nodelta(e->sx_msg, s));
        }
        lp = lq;
        sp = hp.q;
        rounds++;
    }
    HIP_TRY(hipMemcpyAsync(e->en, &enh, sizeof enh, hipMemcpyHostToDevice, s));
    if (lp != n) return fail(SF_ERR_DEVICE, "exchange rounds left events undecided");
    HIP_TRY(hipEventRecord(e->ev_core[slot], s));
    HIP_TRY(hipEventRecord(e->ev_done[slot], s));
    HIP_TRY(hipEventRecord(e->ev_end[slot], s));
    e->used[slot] = true;
    e->last = slot;
    e->stats.n_events = n;
    e->stats.n_launches++;
    e->stats.sys_rounds += rounds;
    e->stats.sys_exchanges += levels;
    if (out->mem == SF_MEM_HOST && n) {
        HIP_TRY(hipMemcpyAsync(out->status, dv.status, n, hipMemcpyDeviceToHost, s));
        if (dv.wait) HIP_TRY(hipMemcpyAsync(out->wait_ms, dv.wait, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        if (dv.rule) HIP_TRY(hipMemcpyAsync(out->rule_idx, dv.rule, (size_t)n * 2, hipMemcpyDeviceToHost, s));
    }
    int32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, w.err, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (err) return fail(err, err == SF_ERR_CAPACITY ? "capacity exceeded (param table, or the origin / context node pool: aux_capacity)"
                                                     : "invalid batch (resource outside shard or bad entry_ref)");
    return SF_OK;
}

int sf_system_plan(sf_engine* e, const sf_event_batch* in, const uint8_t* status, uint32_t p, uint32_t* q,
                   uint8_t* sys_mask) {
    if (!e || !in || !q || !sys_mask || (p && !status)) return fail(SF_ERR_INVALID, "null argument");
    if (in->mem != SF_MEM_HOST || !in->ts_ms || !in->count || !in->flags)
        return fail(SF_ERR_INVALID, "sf_system_plan takes the node's IN events in host arrays");
    if (in->n > e->cfg.max_batch) return fail(SF_ERR_CAPACITY, "batch larger than max_batch");
    if (p >= in->n) return fail(SF_ERR_INVALID, "plan position past the batch");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = drain(e); if (rc) return rc; }
    const uint32_t n = in->n;
    if (!e->sys.check) {                                   // no SystemRule: nothing is forced
        std::memset(sys_mask + p, SYS_NONE, n - p);
        *q = n;
        return SF_OK;
    }
    if (!e->sys_plan) {
        HIP_TRY(hipMalloc((void**)&e->sys_plan, sizeof(SysPlanDev)));
        HIP_TRY(hipMalloc((void**)&e->sys_pa, SYS_PLAN_BLOCKS * sizeof(SysExitQ)));
        HIP_TRY(hipMalloc((void**)&e->sys_pb, SYS_PLAN_BLOCKS * sizeof(SysEntQ)));
        HIP_TRY(hipMalloc((void**)&e->sys_mask, e->cfg.max_batch));
    }
    DevBatch b;
    uint8_t* dstatus = nullptr;
    // a later round of the same merged stream (p > 0, same arrays): the events
    // staged for the round before are reused, only the verdicts are copied
    { const int rc = stage_in_events(e, e->plan_sb, in, status, p, b, &dstatus, p > 0); if (rc) return rc; }
    hipStream_t s = e->stream;
    DevState stl = e->st;
    hipError_t le = sys_plan(stl, b, dstatus, e->sys_mask, e->sys, e->en, p, e->sys_plan, e->sys_pa, e->sys_pb, s);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("system plan: ") + hipGetErrorString(le));
    uint32_t qq = 0;
    HIP_TRY(hipMemcpyAsync(&qq, &e->sys_plan->q, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (qq <= p || qq > n) return fail(SF_ERR_DEVICE, "system planner made no progress");
    HIP_TRY(hipMemcpy(sys_mask + p, e->sys_mask + p, qq - p, hipMemcpyDeviceToHost));
    *q = qq;
    return SF_OK;
}

int sf_entry_node_add(sf_engine* e, const sf_event_batch* in, const uint8_t* status) {
    if (!e || !in || !status) return fail(SF_ERR_INVALID, "null argument");
    if (in->mem != SF_MEM_HOST || !in->ts_ms || !in->count || !in->flags)
        return fail(SF_ERR_INVALID, "sf_entry_node_add takes host arrays");
    if (in->n > e->cfg.max_batch) return fail(SF_ERR_CAPACITY, "batch larger than max_batch");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = drain(e); if (rc) return rc; }
    if (!in->n) return SF_OK;
    DevBatch b;
    uint8_t* dstatus = nullptr;
    { const int rc = stage_in_events(e, e->en_sb, in, status, in->n, b, &dstatus); if (rc) return rc; }
    hipError_t le = launch_entry_node(e->st, b, dstatus, e->en, e->en_acc, e->stream);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("entry node: ") + hipGetErrorString(le));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return SF_OK;
}

static Bucket from_abi_bucket(const sf_bucket& o, int64_t max_rt) {
    Bucket d{};
    if (o.window_start == SF_WS_ABSENT) { d = Bucket{WS_NONE, 0, 0, 0, 0, 0, 0, max_rt}; return d; }
    d.ws = o.window_start; d.pass = o.pass; d.block = o.block; d.exc = o.exception; d.succ = o.success; d.rt = o.rt;
    d.occ = o.occupied_pass; d.min_rt = o.min_rt;
    return d;
}
static void to_abi_bucket(const Bucket& d, sf_bucket* o) {
    o->window_start = d.ws == WS_NONE ? SF_WS_ABSENT : d.ws;
    o->pass = d.pass; o->block = d.block; o->exception = d.exc; o->success = d.succ; o->rt = d.rt;
    o->occupied_pass = d.occ; o->min_rt = d.min_rt;
    if (d.ws == WS_NONE) { o->pass = o->block = o->exception = o->success = o->rt = o->occupied_pass = o->min_rt = 0; }
}

// one node's rows (a resource row or an origin / context pool slot) -> sf_node_state
static int read_rows(sf_engine* e, const Bucket* gsec, const Borrow* gbor, const Bucket* gmin, const int64_t* gthr,
                     sf_node_state* out) {
    const int S = e->cfg.sample_count;
    std::vector<Bucket> sec(S), mins(MINUTE);
    std::vector<Borrow> bor(S);
    int64_t th = 0;
    HIP_TRY(hipMemcpyAsync(sec.data(), gsec, S * sizeof(Bucket), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(bor.data(), gbor, S * sizeof(Borrow), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(mins.data(), gmin, MINUTE * sizeof(Bucket), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(&th, gthr, 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    std::memset(out, 0, sizeof *out);
    for (int i = 0; i < SF_MAX_SAMPLE_COUNT; i++) { out->second[i].window_start = SF_WS_ABSENT; out->borrow_ws[i] = SF_WS_ABSENT; }
    for (int i = 0; i < S; i++) {
        to_abi_bucket(sec[i], &out->second[i]);
        out->borrow_ws[i] = bor[i].ws == WS_NONE ? SF_WS_ABSENT : bor[i].ws;
        out->borrow_pass[i] = bor[i].ws == WS_NONE ? 0 : bor[i].pass;
    }
    for (int i = 0; i < MINUTE; i++) to_abi_bucket(mins[i], &out->minute[i]);
    out->cur_thread_num = th;
    return SF_OK;
}

int sf_read_node(sf_engine* e, uint32_t resource, sf_node_state* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    uint32_t l;
    if (!local_of(e, resource, &l)) return fail(SF_ERR_INVALID, "resource outside this shard");
    std::lock_guard<std::mutex> lk(e->mu);
    const NodeRows r = cluster_rows(e->st, l);
    return read_rows(e, r.sec, r.bor, r.min, r.thr, out);
}

// origin / context node of local resource l (sf_xflow.h aux_get): its pool
// slot found on the device, its rows read through the host's chunk directory
static int read_aux(sf_engine* e, uint32_t resource, uint32_t kind, uint32_t id, sf_node_state* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    uint32_t l;
    if (!local_of(e, resource, &l)) return fail(SF_ERR_INVALID, "resource outside this shard");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = drain(e); if (rc) return rc; }
    if (!e->st.xtab) return fail(SF_ERR_INVALID, "no origin / context node is kept");
    uint32_t* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, 4));
    uint32_t k = XNONE;
    hipError_t le = launch_aux_find(e->st, pkey_hi(l, PK_AUX, kind, 0), id, d, e->stream);
    if (le == hipSuccess) le = hipMemcpyAsync(&k, d, 4, hipMemcpyDeviceToHost, e->stream);
    if (le == hipSuccess) le = hipStreamSynchronize(e->stream);
    hipFree(d);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("aux find: ") + hipGetErrorString(le));
    if (k == XNONE || k >= e->st.ax_cap) return fail(SF_ERR_INVALID, "that origin / context node is not kept");
    DevState hs = e->st;
    hs.ax_chunks = e->ax_host.data();            // host mirror of the chunk directory
    const NodeRows r = aux_rows(hs, k);
    return read_rows(e, r.sec, r.bor, r.min, r.thr, out);
}
int sf_read_origin_node(sf_engine* e, uint32_t resource, uint32_t origin, sf_node_state* out) {
    return read_aux(e, resource, AX_ORIGIN, origin, out);
}
int sf_read_context_node(sf_engine* e, uint32_t context, uint32_t resource, sf_node_state* out) {
    return read_aux(e, resource, AX_CTX, context, out);
}

int sf_read_entry_node(sf_engine* e, sf_node_state* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = en_fence(e); if (rc) return rc; }
    EntryNode en;
    HIP_TRY(hipMemcpyAsync(&en, e->en, sizeof en, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    std::memset(out, 0, sizeof *out);
    for (int i = 0; i < SF_MAX_SAMPLE_COUNT; i++) { out->second[i].window_start = SF_WS_ABSENT; out->borrow_ws[i] = SF_WS_ABSENT; }
    for (int i = 0; i < e->cfg.sample_count; i++) to_abi_bucket(en.second[i], &out->second[i]);
    for (int i = 0; i < MINUTE; i++) to_abi_bucket(en.minute[i], &out->minute[i]);
    out->cur_thread_num = en.threads;
    return SF_OK;
}

int sf_read_rule_state(sf_engine* e, uint32_t idx, sf_rule_state* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    if (idx >= e->n_flow) return fail(SF_ERR_INVALID, "rule index");
    std::lock_guard<std::mutex> lk(e->mu);
    DevRuleState s{};
    HIP_TRY(hipMemcpy(&s, e->st.rstate + e->flow_pos[idx], sizeof s, hipMemcpyDeviceToHost));
    out->stored_tokens = s.stored_tokens; out->last_filled_time = s.last_filled; out->latest_passed_time = s.latest_passed;
    return SF_OK;
}

int sf_node_digests(sf_engine* e, uint64_t* out, uint32_t n_rows) {
    if (!e || (n_rows && !out)) return fail(SF_ERR_INVALID, "null argument");
    if (n_rows > e->R) return fail(SF_ERR_INVALID, "n_rows above max_resources");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = drain(e); if (rc) return rc; }
    if (!n_rows) return SF_OK;
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, (size_t)n_rows * 8));
    hipError_t he = launch_node_digests(e->st, n_rows, d, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(out, d, (size_t)n_rows * 8, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    hipFree(d);
    if (he != hipSuccess) return fail(SF_ERR_DEVICE, std::string("node digests: ") + hipGetErrorString(he));
    return SF_OK;
}

int sf_read_rule_states(sf_engine* e, uint32_t first, uint32_t n, sf_rule_state* out) {
    if (!e || (n && !out)) return fail(SF_ERR_INVALID, "null argument");
    if ((uint64_t)first + n > e->n_flow) return fail(SF_ERR_INVALID, "rule index");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = drain(e); if (rc) return rc; }
    if (!n) return SF_OK;
    std::vector<DevRuleState> all(e->n_flow);      // CSR order: the positions of a range are not contiguous
    HIP_TRY(hipMemcpyAsync(all.data(), e->st.rstate, all.size() * sizeof(DevRuleState), hipMemcpyDeviceToHost,
                           e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (uint32_t i = 0; i < n; i++) {
        const DevRuleState& s = all[e->flow_pos[first + i]];
        out[i].stored_tokens = s.stored_tokens; out[i].last_filled_time = s.last_filled;
        out[i].latest_passed_time = s.latest_passed;
    }
    return SF_OK;
}

int sf_snapshot(sf_engine* e, int64_t now_ms, sf_metric_row* out, uint32_t cap, uint32_t* n_out) {
    if (!e || !n_out || (cap && !out)) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = en_fence(e); if (rc) return rc; }
    *n_out = 0;
    hipStream_t s = e->stream;
    if (!e->snap_counts) {
        HIP_TRY(hipMalloc((void**)&e->snap_counts, (size_t)e->R * 4));
        HIP_TRY(hipMalloc((void**)&e->snap_offsets, (size_t)e->R * 4));
        HIP_TRY(hipMalloc((void**)&e->snap_total, 4));
        HIP_TRY(rocprim_scan_bytes(e->R, &e->snap_scan_bytes));
        HIP_TRY(hipMalloc(&e->snap_scan, std::max<size_t>(e->snap_scan_bytes, 16)));
    }
    if (cap > e->snap_cap) {
        if (e->snap_rows) hipFree(e->snap_rows);
        e->snap_rows = nullptr;
        HIP_TRY(hipMalloc((void**)&e->snap_rows, (size_t)cap * sizeof(sf_metric_row)));
        e->snap_cap = cap;
    }
    HIP_TRY(launch_snapshot(e->st, now_ms, e->cfg.shard_count, e->cfg.shard_index, e->snap_counts, e->snap_offsets,
                            e->snap_rows, cap, e->snap_total, e->snap_scan, e->snap_scan_bytes, s));
    uint32_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, e->snap_total, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint32_t k = std::min(total, cap);
    if (k) HIP_TRY(hipMemcpy(out, e->snap_rows, (size_t)k * sizeof(sf_metric_row), hipMemcpyDeviceToHost));
    *n_out = total;
    return total <= cap ? SF_OK : fail(SF_ERR_CAPACITY, "snapshot rows exceed cap");
}
// ---------------------------------------------------------------- metrics.log
int sf_load_resource_names(sf_engine* e, const char* bytes, const uint64_t* offsets, const int32_t* types,
                           uint32_t n) {
    if (!e || (n && (!offsets || (!bytes && offsets[n])))) return fail(SF_ERR_INVALID, "null argument");
    for (uint32_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i]) return fail(SF_ERR_INVALID, "name offsets must be non-decreasing");
    std::lock_guard<std::mutex> lk(e->mu);
    void* old[] = {e->nm_bytes, e->nm_off, e->nm_types};
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (void* p : old) if (p) hipFree(p);
    e->nm_bytes = nullptr; e->nm_off = nullptr; e->nm_types = nullptr; e->n_names = 0;
    const uint64_t nb = n ? offsets[n] - offsets[0] : 0;
    HIP_TRY(hipMalloc((void**)&e->nm_bytes, std::max<uint64_t>(nb, 16)));
    HIP_TRY(hipMalloc((void**)&e->nm_off, ((size_t)n + 1) * 8));
    if (nb) HIP_TRY(hipMemcpy(e->nm_bytes, bytes + offsets[0], nb, hipMemcpyHostToDevice));
    std::vector<uint64_t> off(offsets, offsets + n + 1);
    for (auto& o : off) o -= offsets[0];
    HIP_TRY(hipMemcpy(e->nm_off, off.data(), off.size() * 8, hipMemcpyHostToDevice));
    if (types) {
        HIP_TRY(hipMalloc((void**)&e->nm_types, std::max<size_t>((size_t)n * 4, 16)));
        if (n) HIP_TRY(hipMemcpy(e->nm_types, types, (size_t)n * 4, hipMemcpyHostToDevice));
    }
    e->n_names = n;
    return SF_OK;
}

static int ml_reserve(sf_engine* e, uint32_t rows) {
    const uint32_t nodes = e->R + 1;
    if (!e->ml_mask) {
        HIP_TRY(hipMalloc((void**)&e->ml_mask, (size_t)nodes * 8));
        HIP_TRY(hipMalloc((void**)&e->ml_counts, (size_t)nodes * 4));
        HIP_TRY(hipMalloc((void**)&e->ml_offsets, (size_t)nodes * 4));
        HIP_TRY(hipMalloc((void**)&e->ml_total, 4));
        HIP_TRY(hipMalloc((void**)&e->ml_bytes, 8));
        for (auto& x : e->ml_ev) HIP_TRY(hipEventCreate(&x));
    }
    if (rows > e->ml_row_cap || !e->ml_rows) {
        const uint32_t cap = std::max<uint32_t>(rows, 1024);
        void* old[] = {e->ml_rows, e->ml_keys, e->ml_order, e->ml_len, e->ml_off};
        for (void* p : old) if (p) hipFree(p);
        e->ml_rows = nullptr; e->ml_keys = nullptr; e->ml_order = nullptr; e->ml_len = nullptr; e->ml_off = nullptr;
        e->ml_row_cap = 0;
        HIP_TRY(hipMalloc((void**)&e->ml_rows, (size_t)cap * sizeof(sf_metric_row)));
        HIP_TRY(hipMalloc((void**)&e->ml_keys, (size_t)cap * 2));
        HIP_TRY(hipMalloc((void**)&e->ml_order, (size_t)cap * 8));
        HIP_TRY(hipMalloc((void**)&e->ml_len, (size_t)cap * 8));
        HIP_TRY(hipMalloc((void**)&e->ml_off, (size_t)cap * 8));
        e->ml_row_cap = cap;
    }
    size_t tb = 0;
    HIP_TRY(mlog_temp_bytes(nodes, e->ml_row_cap, &tb));
    if (tb > e->ml_tmp_bytes) {
        if (e->ml_tmp) hipFree(e->ml_tmp);
        e->ml_tmp = nullptr; e->ml_tmp_bytes = 0;
        HIP_TRY(hipMalloc(&e->ml_tmp, tb));
        e->ml_tmp_bytes = tb;
    }
    return SF_OK;
}

// line lengths -> offsets -> lines, copied to the caller's host buffer
static int ml_format(sf_engine* e, const uint32_t* order, uint32_t n, int64_t tz, char* out, uint64_t cap,
                     uint64_t* len_out) {
    hipStream_t s = e->stream;
    HIP_TRY(launch_fmt_len(e->ml_rows, order, n, e->nm_bytes, e->nm_off, e->nm_types, e->n_names, tz, e->ml_len,
                           e->ml_off, e->ml_bytes, e->ml_tmp, e->ml_tmp_bytes, s));
    uint64_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, e->ml_bytes, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *len_out = total;
    if (total > cap) return fail(SF_ERR_CAPACITY, "metric log bytes exceed cap");
    if (total > e->ml_out_cap) {
        if (e->ml_out) hipFree(e->ml_out);
        e->ml_out = nullptr; e->ml_out_cap = 0;
        HIP_TRY(hipMalloc((void**)&e->ml_out, total));
        e->ml_out_cap = total;
    }
    HIP_TRY(launch_fmt_write(e->ml_rows, order, n, e->nm_bytes, e->nm_off, e->nm_types, e->n_names, tz, e->ml_off,
                             e->ml_out, s));
    HIP_TRY(hipEventRecord(e->ml_ev[2], s));
    if (total) HIP_TRY(hipMemcpyAsync(out, e->ml_out, total, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SF_OK;
}

int sf_metric_log(sf_engine* e, int64_t now_ms, int64_t tz_offset_ms, int include_entry_node, char* out,
                  uint64_t cap, uint64_t* len_out, uint32_t* n_lines) {
    if (!e || !len_out || (cap && !out)) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = en_fence(e); if (rc) return rc; }
    *len_out = 0;
    if (n_lines) *n_lines = 0;
    int rc = ml_reserve(e, 0);
    if (rc) return rc;
    hipStream_t s = e->stream;
    const bool with_en = include_entry_node != 0;
    const uint32_t nodes = e->R + (with_en ? 1u : 0u);
    // the ENTRY_NODE line: this engine's node, or the one set by sf_set_report_entry_node
    // (its windows; lastFetchTime stays this engine's, MetricTimerListener.java:40-69)
    EntryNode* en = e->en;
    if (with_en && e->report_set) {
        if (!e->en_report) HIP_TRY(hipMalloc((void**)&e->en_report, sizeof(EntryNode)));
        HIP_TRY(hipMemcpyAsync(e->en_report, &e->report, sizeof(EntryNode), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(&e->en_report->last_fetch, &e->en->last_fetch, 8, hipMemcpyDeviceToDevice, s));
        en = e->en_report;
    }
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const unsigned grid = (unsigned)std::min<uint64_t>(((uint64_t)nodes + 3) / 4, (uint64_t)cus * 16);
    HIP_TRY(hipEventRecord(e->ml_ev[0], s));
    HIP_TRY(launch_mlog_count(e->st, en, with_en, e->cfg.shard_count, e->cfg.shard_index, now_ms, e->ml_mask,
                              e->ml_counts, e->ml_offsets, e->ml_total, e->ml_tmp, e->ml_tmp_bytes, grid, e->ml_ev[1], s));
    uint32_t rows = 0;
    HIP_TRY(hipMemcpyAsync(&rows, e->ml_total, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    rc = ml_reserve(e, rows);
    if (rc) return rc;
    uint32_t* ord = e->ml_order;
    HIP_TRY(launch_mlog_rows(e->st, en, with_en, e->cfg.shard_count, e->cfg.shard_index, now_ms, e->ml_mask,
                             e->ml_offsets, rows, e->ml_rows, e->ml_keys, e->ml_keys + e->ml_row_cap, ord,
                             ord + e->ml_row_cap, e->ml_tmp, e->ml_tmp_bytes, grid, s));
    if (n_lines) *n_lines = rows;
    if (en != e->en) HIP_TRY(hipMemcpyAsync(&e->en->last_fetch, &en->last_fetch, 8, hipMemcpyDeviceToDevice, s));
    rc = ml_format(e, ord + e->ml_row_cap, rows, tz_offset_ms, out, cap, len_out);
    if (rc) return rc;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e->ml_ev[0], e->ml_ev[1]) == hipSuccess) e->stats.metric_scan_ms = ms;
    if (hipEventElapsedTime(&ms, e->ml_ev[0], e->ml_ev[2]) == hipSuccess) e->stats.metric_log_ms = ms;
    return SF_OK;
}

int sf_format_metric_rows(sf_engine* e, const sf_metric_row* rows, uint32_t n, int64_t tz_offset_ms, char* out,
                          uint64_t cap, uint64_t* len_out) {
    if (!e || !len_out || (n && !rows) || (cap && !out)) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    *len_out = 0;
    int rc = ml_reserve(e, n);
    if (rc) return rc;
    if (n) HIP_TRY(hipMemcpyAsync(e->ml_rows, rows, (size_t)n * sizeof(sf_metric_row), hipMemcpyHostToDevice,
                                  e->stream));
    return ml_format(e, nullptr, n, tz_offset_ms, out, cap, len_out);
}
// ---------------------------------------------------------------- cluster token server
// Owner shard of a cluster rule's requests (sentinel_flow.h, sf_token_shard):
// a namespace with a GlobalRequestLimiter is one sequential gate, so all its
// rules live on namespace_id % N; any other rule on flow_id % N.
static uint32_t tok_rule_owner(int64_t flow_id, uint32_t ns_id, const std::vector<sf_namespace>& ns, uint32_t N) {
    for (const sf_namespace& x : ns)
        if (x.namespace_id == ns_id) {
            if (x.max_allowed_qps >= 0) return ns_id % N;
            break;
        }
    return flow_id <= 0 ? 0u : (uint32_t)((uint64_t)flow_id % N);
}

// Rebuild the device rule table, flowId index and namespace table from the
// host copies (ClusterFlowRuleManager / ClusterParamFlowRuleManager /
// ClusterServerConfigManager state).  Metric state is reset when
// `reset_state` (a rule reload creates new ClusterMetric objects:
// ClusterFlowRuleManager.java:361-362, ClusterParamFlowRuleManager.java:354-355).
static int tok_rebuild(sf_engine* e, bool reset_state) {
    TokState& ts = e->ts;
    const uint32_t nf = (uint32_t)e->host_cflow.size(), np = (uint32_t)e->host_cparam.size();
    std::unordered_map<uint32_t, int32_t> ns_index;
    for (size_t i = 0; i < e->host_ns.size(); i++) ns_index.emplace(e->host_ns[i].namespace_id, (int32_t)i);
    std::vector<ClRule> rules(nf + np);
    auto fill = [&](ClRule& r, int64_t id, double count, int32_t tt, uint32_t ns, int32_t S, int32_t I) {
        r.count = count; r.flow_id = id; r.threshold_type = tt;
        auto it = ns_index.find(ns);
        r.ns = it == ns_index.end() ? -1 : it->second;
        r.S = S; r.wl = I / S; r.interval = I;
    };
    const uint32_t N = e->cfg.shard_count;
    for (uint32_t i = 0; i < nf; i++) {
        const sf_cluster_flow_rule& f = e->host_cflow[i];
        fill(rules[i], f.flow_id, f.count, f.threshold_type, f.namespace_id, f.sample_count, f.window_interval_ms);
        rules[i].is_param = 0; rules[i].item_off = rules[i].item_cnt = 0;
        rules[i].owner = tok_rule_owner(f.flow_id, f.namespace_id, e->host_ns, N);
    }
    for (uint32_t i = 0; i < np; i++) {
        const sf_cluster_param_rule& f = e->host_cparam[i];
        ClRule& r = rules[nf + i];
        fill(r, f.flow_id, f.count, f.threshold_type, f.namespace_id, f.sample_count, f.window_interval_ms);
        r.is_param = 1; r.item_off = f.item_offset; r.item_cnt = f.item_count;
        r.owner = tok_rule_owner(f.flow_id, f.namespace_id, e->host_ns, N);
    }
    // flowId -> rule index, open addressing; the first rule of an id wins (like the oracle's lookup)
    uint64_t cap = 16;
    while (cap < 2ull * (nf + np) + 2) cap <<= 1;
    std::vector<IdSlot> tab(cap, IdSlot{0, -1, -1});
    auto put = [&](int64_t id, int32_t idx, bool param) {
        uint64_t x = (uint64_t)id * 0x9e3779b97f4a7c15ULL;
        uint64_t i = mix64(x) & (cap - 1);
        while (tab[i].id != 0 && tab[i].id != id) i = (i + 1) & (cap - 1);
        tab[i].id = id;
        int32_t& slot = param ? tab[i].param : tab[i].flow;
        if (slot < 0) slot = idx;
    };
    for (uint32_t i = 0; i < nf; i++) if (rules[i].flow_id > 0) put(rules[i].flow_id, (int32_t)i, false);
    for (uint32_t i = 0; i < np; i++) if (rules[nf + i].flow_id > 0) put(rules[nf + i].flow_id, (int32_t)(nf + i), true);
    std::vector<ClNs> ns(e->host_ns.size());
    for (size_t i = 0; i < ns.size(); i++) {
        ns[i].connected = e->host_ns[i].connected_count;
        ns[i].has_limiter = e->host_ns[i].max_allowed_qps >= 0;   // GlobalRequestLimiter.initIfAbsent
        ns[i].max_qps = e->host_ns[i].max_allowed_qps;
    }
    std::vector<DevHotItem> items(e->host_citems.size());
    for (size_t i = 0; i < items.size(); i++) {
        items[i].bits = e->host_citems[i].bits; items[i].count = e->host_citems[i].count; items[i].tag = e->host_citems[i].tag;
    }
    hipStream_t s = e->stream;
    auto upload = [&](void** dst, const void* src, size_t bytes) -> int {
        if (*dst) { hipFree(*dst); *dst = nullptr; }
        HIP_TRY(hipMalloc(dst, std::max<size_t>(bytes, 16)));
        if (bytes) HIP_TRY(hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, s));
        return SF_OK;
    };
    int rc;
    if ((rc = upload((void**)&ts.rules, rules.data(), rules.size() * sizeof(ClRule)))) return rc;
    if ((rc = upload((void**)&ts.idtab, tab.data(), tab.size() * sizeof(IdSlot)))) return rc;
    if ((rc = upload((void**)&ts.ns, ns.data(), ns.size() * sizeof(ClNs)))) return rc;
    if ((rc = upload((void**)&ts.items, items.data(), items.size() * sizeof(DevHotItem)))) return rc;
    if (ts.rmulti) { hipFree(ts.rmulti); ts.rmulti = nullptr; }
    HIP_TRY(hipMalloc((void**)&ts.rmulti, std::max<size_t>(rules.size(), 16)));   // per-call multi-value flags
    ts.id_mask = cap - 1;
    ts.n_flow = nf; ts.n_rules = nf + np; ts.n_ns = (uint32_t)ns.size();
    if (reset_state) {
        if (ts.fstate) { hipFree(ts.fstate); ts.fstate = nullptr; }
        HIP_TRY(hipMalloc((void**)&ts.fstate, std::max<size_t>(nf, 1) * sizeof(ClFlowState)));
        HIP_TRY(tok_init_flow_state(ts.fstate, nf, s));
        if (!ts.cptab) {
            uint64_t pc = 1024;
            while (pc < std::max<uint64_t>(e->cfg.param_capacity, 1024)) pc <<= 1;
            HIP_TRY(hipMalloc((void**)&ts.cptab, pc * sizeof(CpSlot)));
            ts.cp_mask = pc - 1;
        }
        HIP_TRY(hipMemsetAsync(ts.cptab, 0, (ts.cp_mask + 1) * sizeof(CpSlot), s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return SF_OK;
}

int sf_load_namespaces(sf_engine* e, const sf_namespace* ns, uint32_t n) {
    if (!e || (n && !ns)) return fail(SF_ERR_INVALID, "null argument");
    if (n > 255) return fail(SF_ERR_UNSUPPORTED, "at most 255 namespaces");
    std::lock_guard<std::mutex> lk(e->mu);
    e->host_ns.assign(ns, ns + n);
    // GlobalRequestLimiter state of the loaded namespaces starts empty
    LimState z;
    for (int k = 0; k < LIM_S; k++) { z.ws[k] = WS_NONE; z.v[k] = 0; }
    std::vector<LimState> lim(std::max<uint32_t>(n, 1), z);
    if (e->ts.lim) { hipFree(e->ts.lim); e->ts.lim = nullptr; }
    HIP_TRY(hipMalloc((void**)&e->ts.lim, lim.size() * sizeof(LimState)));
    HIP_TRY(hipMemcpyAsync(e->ts.lim, lim.data(), lim.size() * sizeof(LimState), hipMemcpyHostToDevice, e->stream));
    return tok_rebuild(e, false);
}

int sf_load_cluster_rules(sf_engine* e, const sf_cluster_flow_rule* flow, uint32_t n_flow,
                          const sf_cluster_param_rule* param, uint32_t n_param, const sf_hot_item* items,
                          uint32_t n_items) {
    if (!e || (n_flow && !flow) || (n_param && !param) || (n_items && !items)) return fail(SF_ERR_INVALID, "null argument");
    auto check = [&](int32_t S, int32_t I) {
        return S > 0 && S <= CL_MAXS && I > 0 && I % S == 0;   // LeapArray.java:70-87
    };
    for (uint32_t i = 0; i < n_flow; i++)
        if (!check(flow[i].sample_count, flow[i].window_interval_ms))
            return fail(SF_ERR_UNSUPPORTED, "cluster flow rule: sample_count must be 1..16 and divide window_interval_ms");
    for (uint32_t i = 0; i < n_param; i++) {
        if (!check(param[i].sample_count, param[i].window_interval_ms))
            return fail(SF_ERR_UNSUPPORTED, "cluster param rule: sample_count must be 1..16 and divide window_interval_ms");
        if ((uint64_t)param[i].item_offset + param[i].item_count > n_items) return fail(SF_ERR_INVALID, "hot item range");
    }
    std::lock_guard<std::mutex> lk(e->mu);
    e->host_cflow.assign(flow, flow + n_flow);
    e->host_cparam.assign(param, param + n_param);
    e->host_citems.assign(items, items + n_items);
    return tok_rebuild(e, true);
}

static int tok_work_ensure(sf_engine* e, uint32_t n) {
    if (n <= e->tw_cap) return SF_OK;
    free_tok_work(e->tw);
    TokWork& w = e->tw;
    const size_t N = std::max<uint32_t>(n, e->cfg.max_batch);
    auto A = [&](void** p, size_t bytes) -> int { HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 16))); return SF_OK; };
    int rc = 0;
    rc |= A((void**)&w.nskey_in, N); rc |= A((void**)&w.nskey_out, N);
    rc |= A((void**)&w.idx_in, N * 4); rc |= A((void**)&w.idx_out, N * 4);
    rc |= A((void**)&w.key_in, N * 8); rc |= A((void**)&w.key_out, N * 8);
    rc |= A((void**)&w.rule_of, N * 4); rc |= A((void**)&w.pending, N);
    rc |= A((void**)&w.head, std::max<size_t>(N, 512) * 4); rc |= A((void**)&w.head_scan, N * 4);
    rc |= A((void**)&w.seg_start, (N + 1) * 4); rc |= A((void**)&w.n_seg, 4);
    if (rc) return SF_ERR_NOMEM;
    HIP_TRY(tok_query_temp((uint32_t)N, &w.sort8_bytes, &w.sort64_bytes, &w.scan_bytes));
    rc |= A(&w.sort8_tmp, w.sort8_bytes); rc |= A(&w.sort64_tmp, w.sort64_bytes); rc |= A(&w.scan_tmp, w.scan_bytes);
    if (rc) return SF_ERR_NOMEM;
    e->tw_cap = (uint32_t)N;
    return SF_OK;
}

// token state present (rules built, namespace limiter allocated); caller holds e->mu
static int tok_ready(sf_engine* e) {
    if (!e->ts.rules) { int r2 = tok_rebuild(e, true); if (r2) return r2; }
    if (!e->ts.lim) {
        LimState z; for (int k = 0; k < LIM_S; k++) { z.ws[k] = WS_NONE; z.v[k] = 0; }
        HIP_TRY(hipMalloc((void**)&e->ts.lim, sizeof(LimState)));
        HIP_TRY(hipMemcpy(e->ts.lim, &z, sizeof z, hipMemcpyHostToDevice));
    }
    return SF_OK;
}

int sf_request_tokens(sf_engine* e, const sf_token_batch* in, sf_token_results* out) {
    if (!e || !in || !out || !out->status) return fail(SF_ERR_INVALID, "null argument");
    if (in->n == 0) return SF_OK;
    if (!in->flow_id || !in->count || !in->flags || !in->ts_ms) return fail(SF_ERR_INVALID, "missing request array");
    if ((in->param_tag == nullptr) != (in->param_bits == nullptr)) return fail(SF_ERR_INVALID, "param_tag/param_bits");
    std::lock_guard<std::mutex> lk(e->mu);
    const uint32_t n = in->n;
    int rc = tok_work_ensure(e, n);
    if (rc) return fail(rc, "token work buffers");
    { int r2 = tok_ready(e); if (r2) return r2; }
    hipStream_t s = e->stream;
    TokBatch b{};
    b.n = n;
    const bool has_param = in->param_tag != nullptr;
    // Collection params: the value arrays hold param_off[n] elements
    uint32_t n_vals = n;
    if (in->param_off) {
        if (in->mem == SF_MEM_HOST) n_vals = in->param_off[n];
        else HIP_TRY(hipMemcpy(&n_vals, in->param_off + n, 4, hipMemcpyDeviceToHost));
    }
    // staging: inputs then outputs, 256-B aligned
    size_t off_fid = 0, off_cnt = align_up(off_fid + (size_t)n * 8), off_fl = align_up(off_cnt + (size_t)n * 4),
           off_ts = align_up(off_fl + n), off_tag = align_up(off_ts + (size_t)n * 8),
           off_bits = align_up(off_tag + (has_param ? n_vals : 0)),
           off_po = align_up(off_bits + (has_param ? (size_t)n_vals * 8 : 0)),
           off_st = align_up(off_po + (in->param_off ? ((size_t)n + 1) * 4 : 0)),
           off_rem = align_up(off_st + n), off_wt = align_up(off_rem + (size_t)n * 4), need = align_up(off_wt + (size_t)n * 4);
    if (need > e->tok_stage_bytes) {
        if (e->tok_stage) hipFree(e->tok_stage);
        e->tok_stage = nullptr;
        HIP_TRY(hipMalloc(&e->tok_stage, need));
        e->tok_stage_bytes = need;
    }
    char* base = (char*)e->tok_stage;
    if (in->mem == SF_MEM_HOST) {
        HIP_TRY(hipMemcpyAsync(base + off_fid, in->flow_id, (size_t)n * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(base + off_cnt, in->count, (size_t)n * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(base + off_fl, in->flags, n, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(base + off_ts, in->ts_ms, (size_t)n * 8, hipMemcpyHostToDevice, s));
        if (has_param && n_vals) {
            HIP_TRY(hipMemcpyAsync(base + off_tag, in->param_tag, n_vals, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(base + off_bits, in->param_bits, (size_t)n_vals * 8, hipMemcpyHostToDevice, s));
        }
        if (in->param_off)
            HIP_TRY(hipMemcpyAsync(base + off_po, in->param_off, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, s));
        b.flow_id = (const int64_t*)(base + off_fid); b.count = (const int32_t*)(base + off_cnt);
        b.flags = (const uint8_t*)(base + off_fl); b.ts = (const int64_t*)(base + off_ts);
        b.ptag = has_param ? (const uint8_t*)(base + off_tag) : nullptr;
        b.pbits = has_param ? (const uint64_t*)(base + off_bits) : nullptr;
        b.poff = in->param_off ? (const uint32_t*)(base + off_po) : nullptr;
    } else {
        b.flow_id = in->flow_id; b.count = in->count; b.flags = in->flags; b.ts = in->ts_ms;
        b.ptag = in->param_tag; b.pbits = in->param_bits; b.poff = in->param_off;
    }
    TokOut o{};
    const bool host_out = out->mem == SF_MEM_HOST;
    if (host_out) {
        o.status = (int8_t*)(base + off_st); o.remaining = (int32_t*)(base + off_rem); o.wait = (int32_t*)(base + off_wt);
    } else {
        if (!out->remaining || !out->wait_ms) return fail(SF_ERR_INVALID, "device results need remaining and wait_ms");
        o.status = out->status; o.remaining = out->remaining; o.wait = out->wait_ms;
    }
    HIP_TRY(hipMemsetAsync(e->st.err, 0, sizeof(int32_t), s));
    hipError_t le = tok_launch(e->ts, e->tw, b, o, s);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("token launch: ") + hipGetErrorString(le));
    if (host_out) {
        HIP_TRY(hipMemcpyAsync(out->status, o.status, n, hipMemcpyDeviceToHost, s));
        if (out->remaining) HIP_TRY(hipMemcpyAsync(out->remaining, o.remaining, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        if (out->wait_ms) HIP_TRY(hipMemcpyAsync(out->wait_ms, o.wait, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    }
    int32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, e->st.err, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (err) return fail(err, err == SF_ERR_CAPACITY ? "cluster param table capacity exceeded"
                                                     : "invalid token batch (a request owned by another shard?)");
    return SF_OK;
}

int sf_token_shard(const sf_cluster_flow_rule* flow, uint32_t n_flow, const sf_cluster_param_rule* param,
                   uint32_t n_param, const sf_namespace* ns, uint32_t n_ns, uint32_t shard_count,
                   const int64_t* flow_id, const uint8_t* flags, uint32_t n, uint32_t* out_shard) {
    if ((n_flow && !flow) || (n_param && !param) || (n_ns && !ns) || (n && (!flow_id || !flags || !out_shard)) ||
        shard_count == 0)
        return fail(SF_ERR_INVALID, "sf_token_shard arguments");
    const std::vector<sf_namespace> nsv(ns, ns + n_ns);
    std::unordered_map<int64_t, uint32_t> fo, po;                  // first rule of an id (tok_rebuild's lookup)
    for (uint32_t i = 0; i < n_flow; i++)
        if (flow[i].flow_id > 0) fo.emplace(flow[i].flow_id, tok_rule_owner(flow[i].flow_id, flow[i].namespace_id, nsv, shard_count));
    for (uint32_t i = 0; i < n_param; i++)
        if (param[i].flow_id > 0) po.emplace(param[i].flow_id, tok_rule_owner(param[i].flow_id, param[i].namespace_id, nsv, shard_count));
    for (uint32_t i = 0; i < n; i++) {
        const int64_t id = flow_id[i];
        if (id <= 0) { out_shard[i] = 0; continue; }
        const auto& m = (flags[i] & SF_TOK_PARAM) ? po : fo;
        const auto it = m.find(id);
        out_shard[i] = it != m.end() ? it->second : (uint32_t)((uint64_t)id % shard_count);
    }
    return SF_OK;
}

uint64_t sf_string_key(const uint8_t* bytes, uint32_t len) {   // FNV-1a 64 (the wire path's String key)
    uint64_t h = 0xcbf29ce484222325ULL;
    for (uint32_t i = 0; i < len; i++) { h ^= bytes[i]; h *= 0x100000001b3ULL; }
    return h;
}

int sf_serve_frames(sf_engine* e, const sf_wire_batch* in, sf_wire_out* out) {
    if (!e || !in || !out || !in->stream_off || !out->resp_off || !out->consumed || !out->stop)
        return fail(SF_ERR_INVALID, "null argument");
    if (in->n_streams == 0) return fail(SF_ERR_INVALID, "n_streams must be > 0");
    if (e->cfg.shard_count > 1)
        return fail(SF_ERR_UNSUPPORTED, "sf_serve_frames on a sharded token server: route decoded requests with sf_token_shard");
    const uint32_t S = in->n_streams;
    std::vector<uint64_t> soff(S + 1);
    if (in->mem == SF_MEM_HOST) std::memcpy(soff.data(), in->stream_off, (S + 1) * sizeof(uint64_t));
    else HIP_TRY(hipMemcpy(soff.data(), in->stream_off, (S + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    for (uint32_t s = 0; s < S; s++)
        if (soff[s + 1] < soff[s]) return fail(SF_ERR_INVALID, "stream_off must be non-decreasing");
    if (soff[S] >= (1ull << 31)) return fail(SF_ERR_CAPACITY, "wire batch must be < 2^31 bytes");
    if (soff[S] && !in->bytes) return fail(SF_ERR_INVALID, "null bytes");
    std::lock_guard<std::mutex> lk(e->mu);
    out->n_frames = out->n_requests = out->n_responses = 0;
    const uint32_t n = (uint32_t)soff[S];
    if (soff[0] == n) {                          // nothing to read: every stream handled, no response
        for (uint32_t s = 0; s < S; s++) { out->consumed[s] = 0; out->stop[s] = SF_WIRE_DONE; }
        for (uint32_t s = 0; s <= S; s++) out->resp_off[s] = 0;
        return SF_OK;
    }
    { int r2 = tok_ready(e); if (r2) return r2; }
    hipStream_t st = e->stream;
    WireBufs w{};
    w.n = n; w.S = S;
    w.n_tiles = (n + WIRE_TILE - 1) / WIRE_TILE;
    const uint32_t F = n / 2 + 1;                 // frames are >= 2 bytes
    size_t tmp = 0;
    { hipError_t qe = wire_query_temp(w.n_tiles, S, F, &tmp);
      if (qe != hipSuccess) return fail(SF_ERR_DEVICE, std::string("wire temp: ") + hipGetErrorString(qe)); }
    // one grow-only arena, 256-B aligned pieces
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + std::max<size_t>(bytes, 16)); return o; };
    const bool host_in = in->mem == SF_MEM_HOST;
    const size_t o_bytes = host_in ? take(n + 16) : 0, o_soff = host_in ? take((S + 1) * 8) : 0;
    const size_t o_exit = take((size_t)n * 4), o_tent = take((size_t)w.n_tiles * 4),
                 o_bm = take((size_t)w.n_tiles * (WIRE_TILE / 32) * 4), o_tc = take(((size_t)w.n_tiles + 1) * 4),
                 o_tb = take(((size_t)w.n_tiles + 1) * 4), o_cons = take((size_t)S * 4), o_stop = take((size_t)S * 4),
                 o_rsc = take(((size_t)S + 1) * 4), o_fr = take((size_t)F * 4), o_wf = take((size_t)F * sizeof(WFrame)),
                 o_fl = take((size_t)F * 8), o_pos = take((size_t)F * 8), o_cnt = take(16),
                 o_qf = take((size_t)F * 8), o_qc = take((size_t)F * 4), o_qfl = take(F), o_qts = take((size_t)F * 8),
                 o_qtg = take(n), o_qb = take((size_t)n * 8), o_rs = take(F), o_rr = take((size_t)F * 4),
                 o_nv = take((size_t)F * 4), o_qnv = take(((size_t)F + 1) * 4), o_qpo = take(((size_t)F + 1) * 4),
                 o_rw = take((size_t)F * 4), o_resp = take((size_t)F * 16), o_sb = take(S),
                 o_crel = take((size_t)S * 8), o_tmp = take(tmp);
    if (off > e->wire_bytes) {
        if (e->wire_arena) hipFree(e->wire_arena);
        e->wire_arena = nullptr; e->wire_bytes = 0;
        HIP_TRY(hipMalloc(&e->wire_arena, off));
        e->wire_bytes = off;
    }
    char* A = (char*)e->wire_arena;
    if (host_in) {
        HIP_TRY(hipMemcpyAsync(A + o_bytes, in->bytes, n, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(A + o_soff, soff.data(), (S + 1) * 8, hipMemcpyHostToDevice, st));
        w.bytes = (const uint8_t*)(A + o_bytes); w.soff = (const uint64_t*)(A + o_soff);
    } else {
        w.bytes = in->bytes; w.soff = in->stream_off;
    }
    w.exitv = (uint32_t*)(A + o_exit); w.tentry = (uint32_t*)(A + o_tent); w.bitmap = (uint32_t*)(A + o_bm);
    w.tcount = (uint32_t*)(A + o_tc); w.tbase = (uint32_t*)(A + o_tb); w.consumed = (uint32_t*)(A + o_cons);
    w.stopoff = (uint32_t*)(A + o_stop); w.resp_cnt = nullptr; w.resp_scan = (uint32_t*)(A + o_rsc);
    w.frames = (uint32_t*)(A + o_fr); w.wf = (WFrame*)(A + o_wf); w.fl = (uint64_t*)(A + o_fl);
    w.pos = (uint64_t*)(A + o_pos); w.counters = (uint32_t*)(A + o_cnt);
    w.q_fid = (int64_t*)(A + o_qf); w.q_cnt = (int32_t*)(A + o_qc); w.q_flags = (uint8_t*)(A + o_qfl);
    w.q_ts = (int64_t*)(A + o_qts); w.q_tag = (uint8_t*)(A + o_qtg); w.q_bits = (uint64_t*)(A + o_qb);
    w.nval = (uint32_t*)(A + o_nv); w.q_nval = (uint32_t*)(A + o_qnv); w.q_poff = (uint32_t*)(A + o_qpo);
    w.r_status = (int8_t*)(A + o_rs); w.r_rem = (int32_t*)(A + o_rr); w.r_wait = (int32_t*)(A + o_rw);
    w.resp = (uint8_t*)(A + o_resp); w.stop = (uint8_t*)(A + o_sb); w.consumed_rel = (uint64_t*)(A + o_crel);
    w.tmp = A + o_tmp; w.tmp_bytes = tmp;

    if (e->timing) {
        for (auto& x : e->ml_ev) if (!x) HIP_TRY(hipEventCreate(&x));
        HIP_TRY(hipEventRecord(e->ml_ev[0], st));
    }
    hipError_t le = wire_frame(w, st);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("wire framing: ") + hipGetErrorString(le));
    uint32_t nf = 0;
    HIP_TRY(hipMemcpyAsync(&nf, w.tbase + w.n_tiles, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    uint64_t tot[2] = {0, 0};
    if (nf) {
        le = wire_decode(w, nf, in->now_ms, st);
        if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("wire decode: ") + hipGetErrorString(le));
        HIP_TRY(hipMemcpyAsync(&tot[0], w.pos + nf - 1, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&tot[1], w.fl + nf - 1, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    const uint64_t both = tot[0] + tot[1];
    const uint32_t n_req = (uint32_t)(both >> 32), n_resp = (uint32_t)both;
    HIP_TRY(hipMemsetAsync(e->st.err, 0, sizeof(int32_t), st));
    if (n_req) {
        int rc = tok_work_ensure(e, n_req);
        if (rc) return fail(rc, "token work buffers");
        le = wire_compact(w, nf, n_req, in->now_ms, st);
        if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("wire compact: ") + hipGetErrorString(le));
        TokBatch b{};
        b.n = n_req; b.flow_id = w.q_fid; b.count = w.q_cnt; b.flags = w.q_flags; b.ts = w.q_ts;
        b.ptag = w.q_tag; b.pbits = w.q_bits; b.poff = w.q_poff;
        TokOut o{w.r_status, w.r_rem, w.r_wait};
        le = tok_launch(e->ts, e->tw, b, o, st);
        if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("token launch: ") + hipGetErrorString(le));
    }
    le = wire_encode(w, nf, st);
    if (le != hipSuccess) return fail(SF_ERR_DEVICE, std::string("wire encode: ") + hipGetErrorString(le));
    if (e->timing) HIP_TRY(hipEventRecord(e->ml_ev[1], st));
    const bool fits = (uint64_t)n_resp * SF_WIRE_RESP_BYTES <= out->cap;
    if (fits && n_resp) {
        if (!out->resp) return fail(SF_ERR_INVALID, "null resp");
        HIP_TRY(hipMemcpyAsync(out->resp, w.resp, (size_t)n_resp * SF_WIRE_RESP_BYTES, hipMemcpyDeviceToHost, st));
    }
    std::vector<uint32_t> roff(S + 1);
    uint32_t handled = 0;
    int32_t err = 0;
    HIP_TRY(hipMemcpyAsync(roff.data(), w.resp_scan, (S + 1) * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out->consumed, w.consumed_rel, (size_t)S * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(out->stop, w.stop, S, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&handled, w.counters, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&err, e->st.err, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (e->timing) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, e->ml_ev[0], e->ml_ev[1]));
        e->stats.wire_ms = ms;
    }
    for (uint32_t s = 0; s <= S; s++) out->resp_off[s] = (uint64_t)roff[s] * SF_WIRE_RESP_BYTES;
    out->n_frames = handled; out->n_requests = n_req; out->n_responses = n_resp;
    if (err) return fail(err, err == SF_ERR_CAPACITY ? "cluster param table capacity exceeded" : "invalid token batch");
    if (!fits) return fail(SF_ERR_CAPACITY, "response buffer too small (n_responses * 16 bytes needed)");
    return SF_OK;
}

int sf_cluster_sum(sf_engine* e, int64_t flow_id, int event, int64_t now_ms, int64_t* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    if (event < 0 || event >= CE_COUNT) return fail(SF_ERR_INVALID, "event");
    std::lock_guard<std::mutex> lk(e->mu);
    *out = 0;
    for (size_t i = 0; i < e->host_cflow.size(); i++) {
        if (e->host_cflow[i].flow_id != flow_id) continue;
        HIP_TRY(tok_cluster_sum(e->ts, (uint32_t)i, event, now_ms, e->d_sum, e->stream));
        HIP_TRY(hipMemcpyAsync(out, e->d_sum, 8, hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        return SF_OK;
    }
    return SF_OK;
}

// ---------------------------------------------------------------- node-wide aggregate (RCCL)
int sf_comm_unique_id(uint8_t* out, size_t len) {
    if (!out || len < NCCL_UNIQUE_ID_BYTES) return fail(SF_ERR_INVALID, "unique id buffer");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(SF_ERR_DEVICE, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return SF_OK;
}

int sf_comm_init(sf_engine* e, int nranks, int rank, const uint8_t* id, size_t len) {
    if (!e || !id || len < NCCL_UNIQUE_ID_BYTES || nranks <= 0 || rank < 0 || rank >= nranks)
        return fail(SF_ERR_INVALID, "sf_comm_init arguments");
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->comm) { ncclCommDestroy(e->comm); e->comm = nullptr; }
    HIP_TRY(hipSetDevice(e->cfg.device));
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&e->comm, nranks, uid, rank);
    if (r != ncclSuccess) { e->comm = nullptr; return fail(SF_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)); }
    if (!e->agg) HIP_TRY(hipMalloc((void**)&e->agg, 4096 * sizeof(int64_t)));
    return SF_OK;
}

int sf_set_report_entry_node(sf_engine* e, const sf_node_state* node) {
    if (!e) return fail(SF_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = en_fence(e); if (rc) return rc; }
    if (!node) { e->report_set = false; return SF_OK; }
    EntryNode& r = e->report;
    r = EntryNode{};
    const int64_t mrt = e->cfg.statistic_max_rt;
    for (int i = 0; i < SF_MAX_SAMPLE_COUNT; i++)
        r.second[i] = i < e->cfg.sample_count ? from_abi_bucket(node->second[i], mrt) : Bucket{WS_NONE, 0, 0, 0, 0, 0, 0, mrt};
    for (int i = 0; i < MINUTE; i++) r.minute[i] = from_abi_bucket(node->minute[i], mrt);
    r.threads = node->cur_thread_num;
    e->report_set = true;
    return SF_OK;
}

int sf_entry_node_allreduce(sf_engine* e, sf_node_state* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    { const int rc = en_fence(e); if (rc) return rc; }
    if (!e->comm) return fail(SF_ERR_INVALID, "sf_comm_init first");
    const int S = e->cfg.sample_count, nb = S + MINUTE;
    hipStream_t s = e->stream;
    int64_t *ws = e->agg, *gws = ws + nb, *vals = gws + nb, *minrt = vals + nb * 6 + 1;
    HIP_TRY(launch_en_pack_ws(e->en, S, ws, s));
    auto nc = [&](ncclResult_t r, const char* what) -> int {
        return r == ncclSuccess ? SF_OK : fail(SF_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
    };
    int rc;
    if ((rc = nc(ncclAllReduce(ws, gws, nb, ncclInt64, ncclMax, e->comm, s), "allreduce max"))) return rc;
    HIP_TRY(launch_en_pack_vals(e->en, S, gws, vals, minrt, s));
    if ((rc = nc(ncclAllReduce(vals, vals, (size_t)nb * 6 + 1, ncclInt64, ncclSum, e->comm, s), "allreduce sum"))) return rc;
    if ((rc = nc(ncclAllReduce(minrt, minrt, nb, ncclInt64, ncclMin, e->comm, s), "allreduce min"))) return rc;
    std::vector<int64_t> h_ws(nb), h_vals((size_t)nb * 6 + 1), h_min(nb);
    HIP_TRY(hipMemcpyAsync(h_ws.data(), gws, nb * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(h_vals.data(), vals, h_vals.size() * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(h_min.data(), minrt, nb * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::memset(out, 0, sizeof *out);
    for (int i = 0; i < SF_MAX_SAMPLE_COUNT; i++) { out->second[i].window_start = SF_WS_ABSENT; out->borrow_ws[i] = SF_WS_ABSENT; }
    for (int i = 0; i < MINUTE; i++) out->minute[i].window_start = SF_WS_ABSENT;
    for (int i = 0; i < nb; i++) {
        sf_bucket& b = i < S ? out->second[i] : out->minute[i - S];
        if (h_ws[i] == INT64_MIN) continue;
        b.window_start = h_ws[i];
        const int64_t* v = &h_vals[(size_t)i * 6];
        b.pass = v[0]; b.block = v[1]; b.exception = v[2]; b.success = v[3]; b.rt = v[4]; b.occupied_pass = v[5];
        b.min_rt = h_min[i] == INT64_MAX ? e->cfg.statistic_max_rt : h_min[i];
    }
    out->cur_thread_num = h_vals[(size_t)nb * 6];
    return SF_OK;
}

int sf_device_alloc(sf_engine* e, size_t bytes, void** ptr) {
    if (!e || !ptr) return fail(SF_ERR_INVALID, "null argument");
    HIP_TRY(hipMalloc(ptr, bytes ? bytes : 16));
    std::lock_guard<std::mutex> lk(e->mu);
    e->user_allocs.push_back(*ptr);
    return SF_OK;
}
int sf_device_free(sf_engine* e, void* ptr) {
    if (!e) return fail(SF_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    auto it = std::find(e->user_allocs.begin(), e->user_allocs.end(), ptr);
    if (it == e->user_allocs.end()) return fail(SF_ERR_INVALID, "pointer not from sf_device_alloc");
    e->user_allocs.erase(it);
    HIP_TRY(hipFree(ptr));
    return SF_OK;
}
int sf_host_alloc(sf_engine* e, size_t bytes, void** ptr) {
    if (!e || !ptr) return fail(SF_ERR_INVALID, "null argument");
    HIP_TRY(hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocDefault));
    std::lock_guard<std::mutex> lk(e->mu);
    e->host_allocs.push_back(*ptr);
    return SF_OK;
}
int sf_host_free(sf_engine* e, void* ptr) {
    if (!e) return fail(SF_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    auto it = std::find(e->host_allocs.begin(), e->host_allocs.end(), ptr);
    if (it == e->host_allocs.end()) return fail(SF_ERR_INVALID, "pointer not from sf_host_alloc");
    e->host_allocs.erase(it);
    HIP_TRY(hipHostFree(ptr));
    return SF_OK;
}
int sf_memcpy(sf_engine* e, void* dst, const void* src, size_t bytes, int kind) {
    if (!e) return fail(SF_ERR_INVALID, "null engine");
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, k, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return SF_OK;
}
int sf_sync(sf_engine* e) {
    if (!e) return fail(SF_ERR_INVALID, "null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipStreamSynchronize(e->sstream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return drain(e, true);
}
int sf_get_stats(sf_engine* e, sf_stats* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    *out = e->stats;
    if (e->st.ax_count) {
        uint32_t ax = 0;
        HIP_TRY(hipMemcpy(&ax, e->st.ax_count, 4, hipMemcpyDeviceToHost));
        out->aux_nodes = ax;
    }
    out->aux_capacity = e->st.ax_cap;
    out->aux_index_grows = e->aux_grows;
    out->param_table_grows = e->p_grows;
    if (e->st.xw_stats) {
        unsigned long long x[4];
        HIP_TRY(hipMemcpy(x, e->st.xw_stats, sizeof x, hipMemcpyDeviceToHost));
        out->xw_chunks_exact = x[0]; out->xw_chunks_serial = x[1]; out->xw_rounds = x[2]; out->xw_serial_events = x[3];
    }
    return SF_OK;
}
int sf_set_timing(sf_engine* e, int enabled) {
    if (!e) return fail(SF_ERR_INVALID, "null engine");
    e->timing = enabled != 0;
    std::memset(&e->stats, 0, sizeof e->stats);
    return SF_OK;
}

int sf_read_param_thread(sf_engine* e, uint32_t resource, int param_idx, uint8_t tag, uint64_t bits, int64_t* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    uint32_t l = 0;
    if (!local_of(e, resource, &l)) return fail(SF_ERR_INVALID, "resource outside this shard");
    std::lock_guard<std::mutex> g(e->mu);
    { const int rc = drain(e); if (rc) return rc; }
    long long* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, 8));
    long long h = 0;
    hipError_t he = launch_param_thread_read(e->st, l, param_idx, tag, bits, d, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    hipFree(d);
    if (he != hipSuccess) return fail(SF_ERR_DEVICE, std::string("param thread read: ") + hipGetErrorString(he));
    *out = h;
    return SF_OK;
}

int sf_param_table_stats(sf_engine* e, uint64_t* used, uint64_t* capacity, uint32_t* max_probe) {
    if (!e || !used || !capacity || !max_probe) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    { const int rc = drain(e); if (rc) return rc; }
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, 16));
    unsigned long long h[2] = {0, 0};
    hipError_t he = launch_param_stats(e->st, d, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    hipFree(d);
    if (he != hipSuccess) return fail(SF_ERR_DEVICE, std::string("param stats: ") + hipGetErrorString(he));
    *used = h[0]; *capacity = e->st.pcap_mask + 1; *max_probe = (uint32_t)h[1];
    return SF_OK;
}

int sf_heavy_profile_read(sf_engine* e, sf_heavy_profile* out, uint32_t cap, uint32_t* n_out) {
    if (!e || !n_out || (cap && !out)) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    uint32_t cnt[7] = {0, 0, 0, 0, 0, 0, 0}, nseg = 0;
    { const int rc = drain(e); if (rc) return rc; }
    const Work& lw = e->w[e->last];
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream2));
    HIP_TRY(hipStreamSynchronize(e->stream3));
    if (e->stream4) HIP_TRY(hipStreamSynchronize(e->stream4));
    HIP_TRY(hipMemcpy(cnt, lw.counters, sizeof cnt, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&nseg, lw.n_seg, 4, hipMemcpyDeviceToHost));
    const uint32_t n1 = cnt[1] + cnt[4], n2 = cnt[5] + cnt[6];
    const uint32_t nh = std::min(n1 + n2, cap);
    std::vector<uint32_t> full(lw.seg_cap), full2(lw.seg_cap), list(nh), start(nseg + 1), res(nseg);
    std::vector<uint8_t> mode(nseg);
    std::vector<uint64_t> ticks(n1 + 1), ticks2(n2 + 1), tk(nh);
    if (nh) {
        HIP_TRY(hipMemcpy(full.data(), lw.heavy_list, (size_t)lw.seg_cap * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(full2.data(), lw.stream_list, (size_t)lw.seg_cap * 4, hipMemcpyDeviceToHost));
        // per-block clocks exist for the first grid-size entries only (grid-stride beyond)
        const size_t hcap = (size_t)e->cfg.max_batch / (lw.heavy_min + 1) + 2;
        HIP_TRY(hipMemcpy(ticks.data(), lw.hticks, std::min<size_t>(n1, hcap) * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(ticks2.data(), lw.sticks, n2 * 8, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < nh; i++) {
            if (i < n1) {
                list[i] = i < cnt[1] ? full[i] : full[lw.seg_cap - 1 - (i - cnt[1])];
                tk[i] = ticks[i];
            } else {
                const uint32_t k = i - n1;
                list[i] = k < cnt[5] ? full2[k] : full2[lw.seg_cap - 1 - (k - cnt[5])];
                tk[i] = ticks2[k];
            }
        }
        HIP_TRY(hipMemcpy(start.data(), lw.seg_start, (nseg + 1) * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(res.data(), lw.seg_res, nseg * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(mode.data(), lw.seg_mode, nseg, hipMemcpyDeviceToHost));
    }
    uint64_t t0 = ~0ull;
    for (uint32_t i = n1; i < nh; i++) t0 = std::min(t0, tk[i] >> 24);
    for (uint32_t i = 0; i < nh; i++) {
        const uint32_t sg = list[i];
        out[i].resource = res[sg]; out[i].events = start[sg + 1] - start[sg];
        out[i].mode = mode[sg]; out[i].start = 0; out[i].ticks = e->timing ? tk[i] : 0;
        if (i >= n1 && e->timing) {          // stream segments: (start & 2^40-1) << 24 | duration
            out[i].ticks = tk[i] & 0xffffffull;
            out[i].start = (uint32_t)((tk[i] >> 24) - t0);
        }
    }
    *n_out = nh;
    return SF_OK;
}


// ---------------------------------------------------------------- DegradeSlot circuit breakers
// DegradeRule.equals (DegradeRule.java:153-164, AbstractRule.equals :76-93):
// resource, limitApp (always "default" here) and the six fields, doubles by
// Double.compare (bit pattern; every NaN equal).
static bool dg_same_double(double a, double b) {
    if (a != a && b != b) return true;
    int64_t x, y;
    std::memcpy(&x, &a, 8); std::memcpy(&y, &b, 8);
    return x == y;
}
static bool dg_rule_equal(const sf_degrade_rule& a, const sf_degrade_rule& b) {
    return a.resource == b.resource && a.grade == b.grade && dg_same_double(a.count, b.count) &&
           a.time_window_s == b.time_window_s && a.min_request_amount == b.min_request_amount &&
           dg_same_double(a.slow_ratio_threshold, b.slow_ratio_threshold) && a.stat_interval_ms == b.stat_interval_ms;
}

int sf_load_degrade_rules(sf_engine* e, const sf_degrade_rule* rules, uint32_t n, uint32_t* n_loaded) {
    if (!e || (n && !rules)) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    const int rc = drain(e);
    if (rc) return rc;
    // buildCircuitBreakers (DegradeRuleManager.java:236-265): valid rules, list order per resource.
    // Everything is built in locals first; the engine's tables are swapped only
    // after every check and allocation succeeded (a failed load keeps the old rules).
    std::vector<uint32_t> loc, valid;
    for (uint32_t i = 0; i < n; i++) {
        if (!dg_valid(rules[i])) continue;
        uint32_t l;
        if (!local_of(e, rules[i].resource, &l)) return fail(SF_ERR_INVALID, "degrade rule resource outside this shard");
        valid.push_back(i);
        loc.push_back(l);
    }
    const uint32_t nv = (uint32_t)valid.size();
    std::vector<uint32_t> order(nv);
    for (uint32_t i = 0; i < nv; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return loc[a] < loc[b]; });
    std::vector<uint32_t> rr_of(e->R, 0), off;
    std::vector<DevBreakerRule> dr(nv);
    std::vector<sf_breaker_state> st(nv);
    std::vector<uint32_t> pos(nv, 0);
    uint32_t n_rres = 0;
    for (uint32_t p = 0; p < nv; p++) {
        const uint32_t v = order[p];
        if (p == 0 || loc[order[p - 1]] != loc[v]) {
            off.push_back(p);
            n_rres++;
        }
        if (p - off.back() >= SF_MAX_BREAKERS_PER_RESOURCE)
            return fail(SF_ERR_UNSUPPORTED, "more than SF_MAX_BREAKERS_PER_RESOURCE degrade rules on one resource");
        const sf_degrade_rule& r = rules[valid[v]];
        dr[p] = make_dev_breaker_rule(r);
        st[p] = sf_breaker_state{SF_CB_CLOSED, 0, 0, DG_WS_NONE, 0, 0};
        pos[v] = p;
    }
    off.push_back(nv);
    for (auto& x : rr_of) x = n_rres;
    for (uint32_t k = 0; k < n_rres; k++) rr_of[loc[order[off[k]]]] = k;
    // getExistingSameCbOrNew (DegradeRuleManager.java:151-163): a rule equal to
    // one of the resource's current breakers keeps that breaker and its state.
    // The reference hands the SAME breaker object to two equal new rules of one
    // resource; that aliasing is refused rather than approximated.
    if (nv && !e->dg_rules.empty()) {
        std::vector<sf_breaker_state> old(e->dg_rules.size());
        for (size_t k = 0; k < old.size(); k++)
            HIP_TRY(hipMemcpy(&old[k], e->dg.state + e->dg_pos[k], sizeof(sf_breaker_state), hipMemcpyDeviceToHost));
        std::vector<uint8_t> taken(old.size(), 0);
        for (uint32_t v = 0; v < nv; v++) {
            const sf_degrade_rule& r = rules[valid[v]];
            for (size_t k = 0; k < old.size(); k++) {
                if (!dg_rule_equal(r, e->dg_rules[k])) continue;
                if (taken[k])
                    return fail(SF_ERR_UNSUPPORTED, "two equal degrade rules would share one existing breaker");
                taken[k] = 1;
                st[pos[v]] = old[k];
                break;
            }
        }
    }
    uint32_t *d_rr = nullptr, *d_off = nullptr;
    DevBreakerRule* d_rules = nullptr;
    sf_breaker_state* d_st = nullptr;
    auto release = [&]() {
        void* p[] = {d_rr, d_off, d_rules, d_st};
        for (void* x : p) if (x) hipFree(x);
    };
    if (dalloc((void**)&d_rr, (size_t)e->R * 4) || dalloc((void**)&d_off, off.size() * 4) ||
        dalloc((void**)&d_rules, (size_t)nv * sizeof(DevBreakerRule)) ||
        dalloc((void**)&d_st, (size_t)nv * sizeof(sf_breaker_state))) {
        release();
        return SF_ERR_NOMEM;
    }
    hipError_t he = hipMemcpy(d_rr, rr_of.data(), (size_t)e->R * 4, hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemcpy(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice);
    if (he == hipSuccess && nv) he = hipMemcpy(d_rules, dr.data(), (size_t)nv * sizeof(DevBreakerRule), hipMemcpyHostToDevice);
    if (he == hipSuccess && nv) he = hipMemcpy(d_st, st.data(), (size_t)nv * sizeof(sf_breaker_state), hipMemcpyHostToDevice);
    if (he != hipSuccess) { release(); return fail(SF_ERR_DEVICE, std::string("degrade rule upload: ") + hipGetErrorString(he)); }
    void* dptrs[] = {(void*)e->dg.rr_of, (void*)e->dg.off, (void*)e->dg.rules, e->dg.state};
    for (void* p : dptrs) if (p) hipFree(p);
    e->dg = DegradeDev{};
    e->dg.rr_of = d_rr; e->dg.off = d_off; e->dg.rules = d_rules; e->dg.state = d_st;
    e->dg.n_rres = n_rres;
    // DegradeSlot inside sf_submit's chain (sf_decide.h decide_segment)
    e->st.dg_rr_of = n_rres ? d_rr : nullptr;
    e->st.dg_off = d_off; e->st.dg_rules = d_rules; e->st.dg_state = d_st; e->st.dg_n = n_rres;
    e->dg_pos = pos;
    e->dg_rules.clear();
    for (uint32_t v = 0; v < nv; v++) e->dg_rules.push_back(rules[valid[v]]);
    uint32_t kb = 1;
    while ((1ull << kb) <= n_rres) kb++;                        // keys 0..n_rres (n_rres = no breaker)
    e->dg.key_bits = kb;
    e->dgw.sort_tmp_bytes = 0;                                  // re-sized for the new key width
    if (e->dgw.sort_tmp) { hipFree(e->dgw.sort_tmp); e->dgw.sort_tmp = nullptr; }
    {   // the routing summary reads dg_rr_of
        hipError_t re = launch_rdesc(e->st, e->stream);
        if (re == hipSuccess) re = hipStreamSynchronize(e->stream);
        if (re != hipSuccess) return fail(SF_ERR_DEVICE, std::string("rdesc: ") + hipGetErrorString(re));
    }
    if (n_loaded) *n_loaded = nv;
    return SF_OK;
}

static int dg_ensure(sf_engine* e, uint32_t n) {
    DegradeWork& w = e->dgw;
    if (n > w.cap) {
        void* ptrs[] = {w.keys_in, w.keys_out, w.idx_in, w.idx_out, w.sev, w.inv};
        for (void* p : ptrs) if (p) hipFree(p);
        w.keys_in = w.keys_out = w.idx_in = w.idx_out = nullptr;
        w.sev = nullptr;
        w.inv = nullptr;
        if (dalloc((void**)&w.keys_in, (size_t)n * 4) || dalloc((void**)&w.keys_out, (size_t)n * 4) ||
            dalloc((void**)&w.idx_in, (size_t)n * 4) || dalloc((void**)&w.idx_out, (size_t)n * 4) ||
            dalloc((void**)&w.sev, (size_t)n * sizeof(DgEv)) || dalloc((void**)&w.inv, (size_t)n * 4))
            return SF_ERR_NOMEM;
        w.cap = n;
        if (w.sort_tmp) { hipFree(w.sort_tmp); w.sort_tmp = nullptr; }
        w.sort_tmp_bytes = 0;
    }
    if (!w.sort_tmp) {
        size_t bytes = 0;
        HIP_TRY(dg_sort_bytes(w.cap, e->dg.key_bits, &bytes));
        if (dalloc(&w.sort_tmp, bytes)) return SF_ERR_NOMEM;
        w.sort_tmp_bytes = bytes;
    }
    if (e->dg.n_rres > w.beg_cap || !w.beg) {
        if (w.beg) hipFree(w.beg);
        if (w.end) hipFree(w.end);
        if (w.heavy) hipFree(w.heavy);
        w.beg = w.end = w.heavy = nullptr;
        const uint32_t c = std::max<uint32_t>(e->dg.n_rres, 1);
        if (dalloc((void**)&w.beg, (size_t)c * 4) || dalloc((void**)&w.end, (size_t)c * 4) ||
            dalloc((void**)&w.heavy, (size_t)c * 4))
            return SF_ERR_NOMEM;
        w.beg_cap = c;
    }
    if (!w.err && dalloc((void**)&w.err, 4)) return SF_ERR_NOMEM;
    if (!w.n_heavy && dalloc((void**)&w.n_heavy, 4)) return SF_ERR_NOMEM;
    return SF_OK;
}

int sf_degrade_submit(sf_engine* e, const sf_event_batch* in, sf_verdicts* out) {
    if (!e || !in || !out || !out->status) return fail(SF_ERR_INVALID, "null argument");
    if (in->n == 0) return SF_OK;
    if (!in->res_id || !in->ts_ms || !in->flags) return fail(SF_ERR_INVALID, "missing event array");
    if (in->n > e->cfg.max_batch) return fail(SF_ERR_CAPACITY, "batch larger than max_batch");
    std::lock_guard<std::mutex> lk(e->mu);
    int rc = drain(e);
    if (rc) return rc;
    const uint32_t n = in->n;
    rc = dg_ensure(e, n);
    if (rc) return rc;
    hipStream_t s = e->stream;
    DegradeBatch b{};
    b.n = n; b.shard_count = e->cfg.shard_count; b.shard_index = e->cfg.shard_index; b.R = e->R;
    b.last_ts = e->st.last_ts;
    uint8_t* status = out->status;
    uint16_t* rule = out->rule_idx;
    int32_t* wait = out->wait_ms;
    const bool host_in = in->mem == SF_MEM_HOST, host_out = out->mem == SF_MEM_HOST;
    if (host_in || host_out) {
        size_t need = 0;
        const size_t o_res = need; need += host_in ? align_up((size_t)n * 4) : 0;
        const size_t o_ts = need; need += host_in ? align_up((size_t)n * 8) : 0;
        const size_t o_fl = need; need += host_in ? align_up((size_t)n) : 0;
        const size_t o_er = need; need += host_in && in->entry_ref ? align_up((size_t)n * 8) : 0;
        const size_t o_ct = need; need += host_in && in->create_ts ? align_up((size_t)n * 8) : 0;
        const size_t o_st = need; need += host_out ? align_up((size_t)n) : 0;
        const size_t o_ru = need; need += host_out && rule ? align_up((size_t)n * 2) : 0;
        const size_t o_wa = need; need += host_out && wait ? align_up((size_t)n * 4) : 0;
        if (need > e->dg_stage_bytes) {
            if (e->dg_stage) hipFree(e->dg_stage);
            e->dg_stage = nullptr;
            if (dalloc(&e->dg_stage, need)) return SF_ERR_NOMEM;
            e->dg_stage_bytes = need;
        }
        char* base = (char*)e->dg_stage;
        auto up = [&](size_t off, const void* src, size_t bytes) -> const void* {
            if (!src) return nullptr;
            hipMemcpyAsync(base + off, src, bytes, hipMemcpyHostToDevice, s);
            return base + off;
        };
        if (host_in) {
            b.res = (const uint32_t*)up(o_res, in->res_id, (size_t)n * 4);
            b.ts = (const int64_t*)up(o_ts, in->ts_ms, (size_t)n * 8);
            b.flags = (const uint8_t*)up(o_fl, in->flags, n);
            b.eref = (const int64_t*)up(o_er, in->entry_ref, (size_t)n * 8);
            b.cts = (const int64_t*)up(o_ct, in->create_ts, (size_t)n * 8);
        }
        if (host_out) {
            status = (uint8_t*)(base + o_st);
            rule = rule ? (uint16_t*)(base + o_ru) : nullptr;
            wait = wait ? (int32_t*)(base + o_wa) : nullptr;
        }
    }
    if (!host_in) {
        b.res = in->res_id; b.ts = in->ts_ms; b.flags = in->flags; b.eref = in->entry_ref; b.cts = in->create_ts;
    }
    HIP_TRY(hipMemsetAsync(e->dgw.err, 0, 4, s));
    HIP_TRY(dg_launch(e->dg, e->dgw, b, status, rule, wait, s));
    int err = 0;
    HIP_TRY(hipMemcpyAsync(&err, e->dgw.err, 4, hipMemcpyDeviceToHost, s));
    if (host_out) {
        HIP_TRY(hipMemcpyAsync(out->status, status, n, hipMemcpyDeviceToHost, s));
        if (rule) HIP_TRY(hipMemcpyAsync(out->rule_idx, rule, (size_t)n * 2, hipMemcpyDeviceToHost, s));
        if (wait) HIP_TRY(hipMemcpyAsync(out->wait_ms, wait, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (err & 1) return fail(SF_ERR_INVALID, "event resource outside this shard");
    if (err & 2) return fail(SF_ERR_INVALID, "EXIT without a valid entry_ref or create_ts");
    if (err & 4) return fail(SF_ERR_INVALID, "event times must be non-decreasing (within and across batches)");
    return SF_OK;
}

int sf_read_breaker(sf_engine* e, uint32_t k, sf_breaker_state* out) {
    if (!e || !out) return fail(SF_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    if (k >= e->dg_pos.size()) return fail(SF_ERR_INVALID, "breaker index");
    HIP_TRY(hipMemcpy(out, e->dg.state + e->dg_pos[k], sizeof *out, hipMemcpyDeviceToHost));
    if (out->window_start == DG_WS_NONE) out->window_start = SF_WS_ABSENT;
    return SF_OK;
}

}  // extern "C"
