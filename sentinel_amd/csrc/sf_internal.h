// sf_internal.h — device state layout and kernel launch interface of the
// MI355X flow-check engine (product code; never includes oracle/).
//
// HBM layout (per engine = one GPU = one resource shard), SURVEY.md §8(d):
//   second  [R][S]  Bucket (64 B)  OccupiableBucketLeapArray main buckets
//   borrow  [R][S]  Borrow (16 B)  FutureBucketLeapArray (only PASS is ever used)
//   minute  [R][60] Bucket (64 B)  BucketLeapArray(60, 60000)
//   threads [R]     int64          StatisticNode.curThreadNum
//   rules   CSR     DevRule + DevRuleState (controller state)
//   param   open-addressed exact table of 32-B slots (ParameterMetric maps)
// A bucket slot that Java would hold as null has ws == WS_NONE.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sentinel_flow.h"
#include "sf_degrade.h"

namespace sf {

constexpr int64_t WS_NONE = -(1LL << 62);   // "null" WindowWrap slot; far below any time
constexpr int MINUTE = SF_MINUTE_BUCKETS;   // 60 x 1000 ms (StatisticNode.java:105)
constexpr int MAX_RULES = SF_MAX_RULES_PER_RESOURCE;

struct Bucket {          // WindowWrap<MetricBucket>: windowStart + MetricBucket (MetricBucket.java:28-142)
    int64_t ws, pass, block, exc, succ, rt, occ, min_rt;
};
struct Borrow {          // WindowWrap<MetricBucket> of FutureBucketLeapArray: only PASS is written
    int64_t ws, pass;
};

// Controller kinds (FlowRuleUtil.generateRater, FlowRuleUtil.java:132-152)
enum : int32_t { CT_DEFAULT = 0, CT_WARM_UP = 1, CT_RATE_LIMITER = 2, CT_WARM_UP_RATE_LIMITER = 3 };

struct DevRule {         // 48 B, constants precomputed at load (WarmUpController.construct :113-139)
    uint8_t kind, grade;
    uint8_t strategy;              // SF_STRATEGY_* (>= 3: another value, selects no node)
    uint8_t always_pass;           // cluster rule without fallback (no token service in the process)
    int32_t max_queue_ms;
    double count;
    double slope;
    int32_t warning_token, max_token;
    int32_t cold_factor, host_index;
    // node selection (FlowRuleChecker.selectNodeByRequesterAndStrategy :129-161);
    // rules other than limitApp "default" + DIRECT run on the xflow walk (sf_xflow.h)
    uint32_t limit_app;            // SF_APP_DEFAULT / SF_APP_OTHER / origin id
    uint32_t ref;                  // RELATE: local resource id (XNONE: never a node); CHAIN: context id
};
static_assert(sizeof(DevRule) == 48, "DevRule layout");
constexpr uint32_t XNONE = 0xFFFFFFFFu;
struct DevRuleState {    // AtomicLong fields of the controllers
    int64_t stored_tokens, last_filled, latest_passed, pad;
};

// Per-resource summary of the rule tables, rebuilt on the device after every
// flow / param / degrade rule load (k_rdesc): the routing and the light lanes
// read this one 16-B record instead of rule_off, prule_off, dg_rr_of and the
// first DevRule (four lines of four arrays per segment)
struct RDesc {
    double count0;                 // the first flow rule's count
    uint32_t r0;                   // rule_off[res]
    uint8_t nrules;                // rule_off[res + 1] - r0 (<= SF_MAX_RULES_PER_RESOURCE)
    uint8_t flags;                 // RD_*
    uint16_t pad;
};
static_assert(sizeof(RDesc) == 16, "RDesc layout");
enum : uint8_t {
    RD_LEAN = 1,                   // one QPS DefaultController rule and nothing else in the chain
    RD_PRULE = 2,                  // ParamFlow rules on the resource
    RD_BRK = 4,                    // circuit breakers on the resource
    RD_STATE0 = 8,                 // the first rule's controller keeps state (not a DefaultController)
};

struct DevParamRule {    // ParamFlowRule (ParamFlowRule.java:45-83)
    int32_t grade, param_idx, behavior, max_queue_ms;
    double count;
    int64_t duration_sec;
    int32_t burst, item_off, item_cnt, host_index;
};
struct DevHotItem { uint64_t bits; int32_t count; uint32_t tag; };

struct ParamSlot {       // exact hash slot: key (hi, lo) -> (a, b)
    uint64_t hi, lo;     // hi == 0: empty
    int64_t a, b;
};
constexpr uint64_t PK_RULE = 1, PK_THREAD = 2;

// Everything a decision kernel needs, passed by value.
struct DevState {
    int32_t S, wl, interval, occupy_timeout;
    int64_t max_rt;
    uint32_t R;
    uint32_t shard_count;          // resource sharding (local id = res / shard_count)
    Bucket* second;
    Borrow* borrow;
    Bucket* minute;
    int64_t* threads;
    const uint32_t* rule_off;      // [R+1]
    const DevRule* rules;
    uint32_t n_stream_rules;       // THREAD-grade / RateLimiter rules (0: no k_heavy_stream segment can exist)
    uint32_t n_window_rules;       // QPS / WarmUp rules (0: no k_heavy_decide window segment, no acquireCount scan)
    DevRuleState* rstate;
    const uint32_t* prule_off;     // [R+1]
    uint32_t n_prule;              // ParamFlow rules loaded (0: no segment needs the ParamFlow routing flags)
    DevParamRule* prules;          // param_idx is mutated (ParamFlowSlot.applyRealParamIdx)
    const DevHotItem* items;
    uint8_t* pm_init;              // [R] bitmask: thread maps created per paramIdx (<8)
    ParamSlot* ptab;
    uint64_t pcap_mask;
    unsigned int* pins;            // [256 * 16] inserts into ptab (ParamTable::ins), null: not counted
    unsigned long long* xw_stats;  // [4] wave walk: exact-solve chunks, serial-path chunks, solve rounds, serial events
    int32_t* err;                  // device error word (capacity, invalid input)
    int64_t* last_fetch;           // [R] StatisticNode.lastFetchTime (metric snapshot)
    int64_t* last_ts;              // engine clock: last event time of the previous batch (time never goes back)
    const RDesc* rdesc;            // [R] (k_rdesc)
    // nonzero once any prioritized entry was submitted (k_segs): only those
    // write borrow buckets (tryOccupyNext), so until then every borrow bucket is
    // the initial empty one and the light lanes need not read it
    int32_t* prio_seen;
    // DegradeSlot (after FlowSlot): breakers of local resource l are
    // [dg_off[k], dg_off[k+1]) with k = dg_rr_of[l] < dg_n; dg_rr_of null = none
    const uint32_t* dg_rr_of;
    const uint32_t* dg_off;
    const DevBreakerRule* dg_rules;
    sf_breaker_state* dg_state;
    uint32_t dg_n;
    // xflow walk (sf_xflow.h): resources whose rules read an origin node, a
    // context (DefaultNode) node or another resource's ClusterNode (RELATE),
    // grouped by RELATE references.  xmap[l] = the group's key (its smallest
    // member), XNONE for every other resource; null: no such rule loaded.
    const uint32_t* xmap;
    // xw[l] (XWF_* bits): l's segments may take the wave walk (k_decide_xw): a
    // group of one resource whose rules all check DIRECT; XWF_THREAD: a THREAD
    // grade rule among them (exits stay in the serial part)
    const uint8_t* xw;
    // origin / context nodes: index table (key (kind, resource, id) -> pool
    // slot) and the node pool in the layout of the resource rows, in chunks of
    // AX_CHUNK nodes (node k: chunk k >> AX_SHIFT), so the pool grows between
    // batches without moving a node
    ParamSlot* xtab; uint64_t xcap_mask;
    const struct AuxChunk* ax_chunks;
    uint32_t* ax_count; uint32_t ax_cap;
};
// one chunk of the origin / context node pool
struct AuxChunk { Bucket* sec; Borrow* bor; Bucket* min; int64_t* thr; };
constexpr uint32_t AX_SHIFT = 16, AX_CHUNK = 1u << AX_SHIFT, AX_MAX_CHUNKS = 8192;

// Constants.ENTRY_NODE (Constants.java:66): the ClusterNode of all inbound
// traffic, updated by StatisticSlot for EntryType.IN (StatisticSlot.java:64-178)
// SystemRuleManager statics (SystemRuleManager.java:68-101), as loadSystemConf
// leaves them (:267-289), and the SystemStatusListener readings.
struct SysRule {
    int32_t check, load_set, cpu_set;
    double qps, highest_load, highest_cpu, cur_load, cur_cpu;
    int64_t max_rt, max_thread;
};

struct EntryNode {
    Bucket second[SF_MAX_SAMPLE_COUNT];
    Bucket minute[SF_MINUTE_BUCKETS];
    int64_t threads;
    int64_t last_fetch;                    // StatisticNode.lastFetchTime (metrics.log)
};
// per-submit reduction of the IN events into the ENTRY_NODE windows: one row
// per window of the batch (relative to the window of its first event)
constexpr uint32_t EN_TBL = 4096;
struct EntryAcc {
    unsigned long long sec[EN_TBL][6];     // pass, block, succ, rt, exc, touched
    unsigned long long min[EN_TBL][6];
    long long minrt_sec[EN_TBL], minrt_min[EN_TBL];
    long long threads;
    unsigned int overflow;                 // a window beyond EN_TBL rows: slow exact path
    unsigned int pad;
};

// 16-B radix-sort payload of one event (batch time span < 2^32 ms)
// Sort payload, 8 B: submission index, and meta = time offset from the batch's
// first event (16 bits, PV_DTS_FAR: read the batch's ts) | flags (8 bits) << 16
// | acquireCount (8 bits, 1..255; 0: read the batch's count) << 24.
struct alignas(8) PackedEv { uint32_t idx, meta; };
// the payload of a batch with origins: the origin id rides along (k_unpack
// writes it in sorted order for the origin-node pass, sf_origin.hip)
struct PackedEvO { uint32_t idx, meta, origin; };
constexpr uint32_t PV_DTS_FAR = 0xffffu;

// light segments are listed by length class (len 1, 2, 3-4, 5-8, ...) so the
// lanes of a wavefront interpret segments of similar length
constexpr int LCLS = 16;
// Light segments of at most SHORT_MAX events are decided in sorted (resource
// id) order by k_decide_short, so a wavefront's lanes touch neighbouring rows
// of every state array and neighbouring events; longer light segments go to
// the length-class lists of k_decide_light.
#ifndef SF_SHORT_MAX
#define SF_SHORT_MAX 8
#endif
constexpr uint32_t SHORT_MAX = SF_SHORT_MAX;
__host__ __device__ inline int light_class(uint32_t len) {
    if (len <= 1) return 0;
    const int c = 32 - __builtin_clz(len - 1);
    return c < LCLS - 1 ? c : LCLS - 1;
}
#ifndef SF_FILL_TILE
#define SF_FILL_TILE 2048
#endif
constexpr uint32_t FILL_TILE = SF_FILL_TILE;             // events per k_heavy_fill tile (256 threads x 8)

// Sorted-order working buffers of one batch.
struct Work {
    uint32_t n;
    uint32_t* keys_in;   uint32_t* keys_out;     // local resource id
    uint32_t* perm;                              // sorted position -> submission index
    PackedEv* pv_in; PackedEv* pv_out;           // sort payload
    uint32_t* wide;                              // batch times exceed 32-bit offsets (k_unpack reads the batch)
    int32_t* err;                                // batch error flag (this Work set's batch)
    bool ox_dirty;                               // index pass ran, origin apply (k_ox_reset) not enqueued
    uint32_t* head;      uint32_t* head_scan;    // segment flags and positions
    uint32_t* seg_start; uint32_t* seg_res; uint32_t* n_seg;
    int64_t* s_ts; int32_t* s_cnt; uint8_t* s_flags;
    int64_t* s_eref; int64_t* s_cts;
    uint8_t* s_nargs; uint8_t* s_atag; uint64_t* s_abits;  // [slot][n]
    uint8_t* v_status; int32_t* v_wait; uint16_t* v_rule;
    void* sort_tmp; size_t sort_tmp_bytes;
    void* scan_tmp; size_t scan_tmp_bytes;
    // heavy / light split (sf_heavy.h)
    uint32_t seg_cap;                                   // min(max_batch, R)
    uint32_t* segflag; uint8_t* seg_mode;
    uint32_t* light_list; uint32_t* heavy_list; uint32_t* counters;
    uint32_t* lcounts;                                  // [2][LCLS] light segments per length class: generic, lean QPS
    uint32_t loff[LCLS];                                // light_list region of each class: generic from the
    uint32_t lcap[LCLS];                                //   front, lean QPS (SM_LIGHTQ) from the back                                // light_list region of each length class   // [0] n_light [1] n_heavy front [2] hw slots [3] sec slots [4] n_heavy back
                                                                      // [5] n_stream front [6] n_stream back
    int64_t* pcg; void* pscan_tmp; size_t pscan_tmp_bytes;
    void* segs_lb;                                      // k_segs_red / k_segs_out tile totals (segs_lb_bytes)
    uint2* fill_tiles; uint32_t fill_tile_cap;         // [2][cap] (segment, tile) of each class for k_heavy_fill
    uint32_t* fill_ntiles;                              // [2] tiles per class
    uint32_t fill_grid;                                 // persistent k_heavy_fill workgroups (8 per CU)
    void* acc_hw; void* acc_sec; uint32_t acc_cap;
    uint32_t* acc_hw_base; uint32_t* acc_sec_base; int64_t* seg_hw0; int64_t* seg_sec0;
    uint32_t* seg_nhw; uint32_t* seg_nsec;
    uint32_t heavy_min;                                 // segments longer than this go heavy
    uint32_t stream_grid;                               // persistent k_heavy_stream workgroups (2 per CU)
    uint64_t* hticks;                                   // [max heavy] k_heavy_decide clock per segment (timing)
    uint32_t* stream_list;                              // THREAD / RL heavy segments (k_heavy_stream)
    uint32_t* xw_list;                                  // [N / XW_MIN + 1] xflow segments of the wave walk (counters[12])
    uint64_t* sticks;                                   // [max heavy] k_heavy_stream clock per segment (timing)
    unsigned long long* passbits;                       // [n/64+2] pass bit per sorted entry (heavy segments)
    uint32_t* exit_of;                                  // [n] sorted index of each entry's exit, ~0 if none
    unsigned long long* lxfar;                          // [n/64+2] far live exits (SM_THREAD)
    uint2* thr_rec;                                     // [n] THREAD-segment window-walk records (k_thr_rec, sf_stream.h)
    uint32_t* tile_rc;                                  // [fill_tile_cap] runs starting in each stream tile -> run id base
    uint32_t* seg_rb; uint32_t* seg_re;                 // [seg_cap] run id range of each SM_THREAD segment
    // (THREAD run mode also borrows buffers dead after the sort: rid = keys_in,
    //  run_start = head_scan, run_pre = keys_out, entry records = pv_in; sf_kernels.hip heavy_ctx)
    uint32_t* vs_cursor;                                // [VS_CURSORS(N)] fill counts of the verdict scatter's buckets
// origin nodes (sf_origin.hip), batches with origins only
    uint32_t* s_origin;                                 // [N] origin id in sorted order
    uint32_t* s_oslot;                                  // [N] pool slot of the event's origin node (XNONE: none)
    uint32_t* ox_cnt;                                   // [8] OXC_* counters of the index pass
    uint32_t* ox_bflags;                                // [N / OX_TILE + 1] origin work of each OX_TILE block
    uint2* ox_bseg;                                     // [N / OX_TILE + 1] first / last segment overlapping each block
    uint4* ox_pairs; uint32_t ox_pairs_cap;             // (pool slot, plist start, end) of each short segment's pair
    uint32_t* ox_plist;                                 // [ox_pairs_cap] the pairs' events (sorted positions) in time order
    uint32_t* ox_hmap; size_t ox_hmap_n;                // [ox_hmap_n] pool slot -> heavy pair id (XNONE between batches)
    uint32_t* ox_hslot; size_t ox_hslot_n;              // [ox_hslot_n] heavy pair id -> pool slot
    int64_t* ox_thr;                                    // [ox_hslot_n] thread delta per heavy pair
    void* ox_acc; size_t ox_acc_n;                      // [H][Ws + Wm] OxAcc window sums of the heavy pairs
};
// origin-node pass (sf_origin.hip): a block is OX_TILE sorted positions; a
// segment of at most OX_LIGHT events is walked whole by the block it starts in
constexpr uint32_t OX_TILE = 2048, OX_LIGHT = 512;
enum : int { OXC_HEAVY = 0, OXC_PAIRS = 1, OXC_PLIST = 2, OXC_OVERFLOW = 3, OXC_RESERVED = 4 };
struct OxAcc {             // one heavy pair's sums in one window; min_rt encoded for a max (0: none)
    unsigned long long pass, block, succ, rt, exc, n_touch, min_rt_key;
};
// verdict scatter (sorted order -> submission order, launch_scatter): regions of
// 2^VS_REG verdicts are assembled in LDS; its first pass has at most 256 buckets
#ifndef SF_VS_REG
#define SF_VS_REG 14
#endif
constexpr uint32_t VS_REG = SF_VS_REG;
inline size_t VS_CURSORS(size_t N) { return 256 + (N >> VS_REG) + 1024 + 16; }

// Device view of a caller batch (pointers already on device).
// A sub-batch (SystemRule planner, sf_system.h) is a view of events
// [base, base + n) of the caller's batch: every pointer is offset by base,
// entry_ref values stay batch indices (an entry before the view is at a
// negative local index), args keep the batch's slot stride.
struct DevBatch {
    uint32_t n;
    const uint32_t* res; const int64_t* ts; const int32_t* cnt; const uint8_t* flags;
    const int64_t* eref; const int64_t* cts;
    uint32_t arg_slots; const uint8_t* nargs; const uint8_t* atag; const uint64_t* abits;
    uint32_t arg_stride;           // slot stride of atag / abits (the whole batch's n)
    const uint32_t* aoff; const uint8_t* etag; const uint64_t* ebits;   // collection elements (batch-wide CSR)
    const uint32_t* origin; const uint32_t* ctx;   // context of each event (or null)
    int64_t base;                  // index of the view's first event in the batch (0: whole batch)
    const uint8_t* sys;            // planner verdicts of IN entries (SYS_NONE: none), or null
    const uint8_t* vprev;          // verdicts of the batch (decided before the view), or null
};
struct DevVerdicts { uint8_t* status; int32_t* wait; uint16_t* rule; };

// internal event flags (sorted-order s_flags; never set by the caller): a
// SystemBlockException forced by the SystemRule planner, reason in bits 4-6
constexpr uint8_t EVF_SYSBLK = 0x80u;
constexpr uint8_t EVF_SYSREASON_SHIFT = 4;
constexpr uint8_t SYS_NONE = 0xFFu;      // planner mask: no forced block
// planner mask: the system verdict is not known yet, but should the entry pass
// SystemSlot its first ParamFlow rule certainly blocks it (sf_system.h,
// "inert entries"): decided as not forced, its reason settled after the sub-batch
constexpr uint8_t SYS_INERT = 0xFEu;
// EVF_SYSBLK reason of an SF_EV_BLOCKED entry: blocked by a slot StatisticSlot
// wraps but the engine does not run (AuthoritySlot), verdict SF_V_BLOCK_OTHER.
// Like a SystemBlockException it is only a block count to every other slot.
constexpr uint8_t SYSR_OTHER = 7;
// sorted entry_ref of an exit whose entry was decided in an earlier sub-batch:
// -1 it passed (the exit is live, like an entry of an earlier batch), -2 blocked
constexpr int64_t EREF_DEAD = -2;

// ---- launchers (sf_kernels.hip) ----
hipError_t query_temp_bytes(uint32_t max_n, uint32_t key_bits, size_t* sort_bytes, size_t* scan_bytes,
                            size_t* pscan_bytes);
hipError_t launch_init_state(const DevState& st, hipStream_t s);
hipError_t launch_rdesc(const DevState& st, hipStream_t s);   // RDesc of every resource from the rule tables
hipError_t launch_entry_node(const DevState& st, const DevBatch& b, const uint8_t* vstatus, EntryNode* en,
                             EntryAcc* acc, hipStream_t s);
hipError_t launch_entry_init(EntryNode* en, int64_t max_rt, hipStream_t s);
hipError_t rocprim_scan_bytes(uint32_t n, size_t* bytes);
hipError_t launch_en_pack_ws(const EntryNode* en, int S, int64_t* ws, hipStream_t s);
hipError_t launch_en_pack_vals(const EntryNode* en, int S, const int64_t* gws, int64_t* vals, int64_t* minrt,
                               hipStream_t s);
hipError_t launch_snapshot(const DevState& st, int64_t now, uint32_t shard_count, uint32_t shard_index,
                           uint32_t* counts, uint32_t* offsets, sf_metric_row* out, uint32_t cap, uint32_t* total,
                           void* scan_tmp, size_t scan_bytes, hipStream_t s);
// metrics.log (sf_metric.hip)
hipError_t mlog_temp_bytes(uint32_t nodes, uint32_t rows, size_t* bytes);
hipError_t launch_mlog_count(const DevState& st, EntryNode* en, bool with_entry, uint32_t shard_count,
                             uint32_t shard_index, int64_t now, unsigned long long* mask, uint32_t* counts,
                             uint32_t* offsets, uint32_t* total, void* tmp, size_t tmp_bytes, unsigned grid,
                             hipEvent_t after_count, hipStream_t s);
hipError_t launch_mlog_rows(const DevState& st, EntryNode* en, bool with_entry, uint32_t shard_count,
                            uint32_t shard_index, int64_t now, const unsigned long long* mask, const uint32_t* offsets,
                            uint32_t n_rows, sf_metric_row* rows, uint8_t* keys, uint8_t* keys_out, uint32_t* order,
                            uint32_t* order_out, void* tmp, size_t tmp_bytes, unsigned grid, hipStream_t s);
hipError_t launch_fmt_len(const sf_metric_row* rows, const uint32_t* order, uint32_t n, const char* names,
                          const uint64_t* name_off, const int32_t* types, uint32_t n_names, int64_t tz,
                          uint64_t* line_len, uint64_t* line_off, uint64_t* total, void* tmp, size_t tmp_bytes,
                          hipStream_t s);
hipError_t launch_fmt_write(const sf_metric_row* rows, const uint32_t* order, uint32_t n, const char* names,
                            const uint64_t* name_off, const int32_t* types, uint32_t n_names, int64_t tz,
                            const uint64_t* line_off, char* out, hipStream_t s);
hipError_t launch_param_stats(const DevState& st, unsigned long long* out, hipStream_t s);   // out[0] used, out[1] max probe
size_t segs_lb_bytes(uint32_t max_n);
hipError_t launch_node_digests(const DevState& st, uint32_t n, unsigned long long* out, hipStream_t s);
hipError_t launch_param_thread_read(const DevState& st, uint32_t l, int idx, uint32_t tag, uint64_t bits,
                                    long long* out, hipStream_t s);
// classify = true: k_classify / k_fill_tiles end the sort phase (the origin
// index passes read the routes); false: launch_decide runs them first
hipError_t launch_sort(const DevState& st, Work& w, const DevBatch& b, uint32_t shard_count, uint32_t shard_index,
                       uint32_t key_bits, hipStream_t s, hipEvent_t* ev, bool timing, bool classify = true);
struct OxWin { int64_t w0s, w0m; uint32_t ws, wm; };    // the batch's first second / minute window and counts
struct OxPlan { uint32_t n_heavy, n_pairs; OxWin win; };   // the batch's origin-node pass (sf_origin.hip)
hipError_t launch_decide(const DevState& st, Work& w, const DevBatch& b, const DevVerdicts& out,
                         hipStream_t s, hipStream_t s2, hipStream_t s3, hipStream_t s4, hipEvent_t* ev, bool timing,
                         const OxPlan* ox = nullptr, bool classify = false, hipStream_t sv = nullptr);
// sf_packed_batch -> SoA (sf_kernels.hip); tile_cnt: [n / 4096 + 1] uint2.  ev4 / ms_end /
// n_ms: the narrow form (ev null)
hipError_t launch_pk_expand(const uint64_t* ev, const uint32_t* ev4, const uint32_t* ms_end, uint32_t n_ms,
                            const int64_t* xref, const int64_t* xcts, const int32_t* cext,
                            int64_t base, uint32_t n, uint32_t n_exit, uint32_t n_cext, uint2* tile_cnt,
                            uint32_t* res, int64_t* ts, int32_t* cnt, uint8_t* flags, int64_t* eref, int64_t* cts,
                            int32_t* err, hipStream_t s);
// sf_sparse_verdicts: the nonzero waits / rule indices of n verdicts as (index << 32 | value) lists
hipError_t launch_sparse_verdicts(const int32_t* wait, const uint16_t* rule, uint32_t n, unsigned long long* wl,
                                  unsigned long long* rl, uint32_t* counts, hipStream_t s);
// origin nodes (sf_origin.hip)
hipError_t launch_ox_index(const DevState& st, Work& w, const DevBatch& b, uint32_t lim, hipStream_t s);
hipError_t launch_ox_apply(const DevState& st, Work& w, const DevBatch& b, uint32_t n_heavy, uint32_t n_pairs,
                           const OxWin& win, hipStream_t s);
hipError_t launch_ox_rehash(const ParamSlot* old_tab, uint64_t old_n, ParamSlot* new_tab, uint64_t new_mask,
                            int32_t* err, hipStream_t s);
hipError_t launch_aux_find(const DevState& st, uint64_t hi, uint64_t lo, uint32_t* out, hipStream_t s);
constexpr size_t ACC_BYTES = 72;                         // sizeof(Acc)
// pipeline events: 0 start, 1 segments, 2 classified, 3 joined, 4 scattered,
// 5 fork, 6 join (stream B), 7 heavy decided, 8 heavy filled, 9 light decided, 10 before classify,
// 11 stream start (stream C), 12 stream done (stream C), 13 stream fill + apply done (stream C),
// 14 origin-node pass done (stream B)
constexpr int SF_NUM_EVENTS = 18;

}  // namespace sf
