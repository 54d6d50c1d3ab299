package com.alibaba.csp.sentinel.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.StructLayout;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.nio.file.Path;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * Panama FFM (JDK 22+) bindings of include/sentinel_flow.h, the C ABI of
 * libsentinel_flow.so.  Struct layouts mirror the header field by field; their
 * sizes are pinned against gcc's sizeof by tests/test_abi.py.
 */
final class SentinelFlowNative {
    static final Linker L = Linker.nativeLinker();
    static final SymbolLookup LIB = SymbolLookup.libraryLookup(
            Path.of(System.getProperty("sentinel.gpu.lib", "libsentinel_flow.so")), Arena.global());

    private static MethodHandle fn(String name, FunctionDescriptor d) {
        return L.downcallHandle(LIB.find(name).orElseThrow(() -> new UnsatisfiedLinkError(name)), d);
    }

    // int sf_create(const sf_config*, sf_engine**); void sf_destroy(sf_engine*)
    static final MethodHandle CONFIG_DEFAULT = fn("sf_config_default", FunctionDescriptor.ofVoid(ADDRESS));
    static final MethodHandle CREATE = fn("sf_create", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    static final MethodHandle DESTROY = fn("sf_destroy", FunctionDescriptor.ofVoid(ADDRESS));
    static final MethodHandle LAST_ERROR = fn("sf_last_error", FunctionDescriptor.of(ADDRESS));
    // rules (FlowRuleManager / ParamFlowRuleManager / SystemRuleManager loadRules)
    static final MethodHandle LOAD_FLOW = fn("sf_load_flow_rules",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT));
    static final MethodHandle LOAD_PARAM = fn("sf_load_param_rules",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT));
    static final MethodHandle LOAD_SYSTEM = fn("sf_load_system_rules",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT));
    static final MethodHandle SET_SYSTEM_STATUS = fn("sf_set_system_status",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_DOUBLE, JAVA_DOUBLE));
    static final MethodHandle LOAD_DEGRADE = fn("sf_load_degrade_rules",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS));
    // decisions
    static final MethodHandle SUBMIT = fn("sf_submit", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS));
    static final MethodHandle SUBMIT_PACKED = fn("sf_submit_packed",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS));
    // double-buffered packed batches: enqueue k+1, then wait for k alone
    static final MethodHandle SUBMIT_PACKED_ASYNC = fn("sf_submit_packed_async",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS));
    static final MethodHandle SYNC_PACKED = fn("sf_sync_packed", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    static final MethodHandle SUBMIT_PACKED_SPARSE_ASYNC = fn("sf_submit_packed_sparse_async",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS));
    static final MethodHandle SYNC_PACKED_SPARSE = fn("sf_sync_packed_sparse",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    // page-locked host memory (the batch arrays: the H2D copy runs at PCIe speed)
    static final MethodHandle HOST_ALLOC = fn("sf_host_alloc",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle DEGRADE_SUBMIT = fn("sf_degrade_submit",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS));
    // cluster token server
    static final MethodHandle LOAD_NAMESPACES = fn("sf_load_namespaces",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT));
    static final MethodHandle LOAD_CLUSTER = fn("sf_load_cluster_rules",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT));
    static final MethodHandle REQUEST_TOKENS = fn("sf_request_tokens",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS));

    /** sf_config (sentinel_flow.h): 19 fields, natural alignment: 88 bytes. */
    static final StructLayout CONFIG = MemoryLayout.structLayout(
            JAVA_INT.withName("sample_count"), JAVA_INT.withName("interval_ms"),
            JAVA_INT.withName("occupy_timeout_ms"), JAVA_INT.withName("cold_factor"),
            JAVA_LONG.withName("statistic_max_rt"),
            JAVA_INT.withName("max_resources"), JAVA_INT.withName("max_batch"),
            JAVA_INT.withName("param_capacity"), JAVA_INT.withName("shard_count"),
            JAVA_INT.withName("shard_index"), JAVA_INT.withName("device"),
            JAVA_INT.withName("cluster_sample_count"), JAVA_INT.withName("cluster_interval_ms"),
            JAVA_DOUBLE.withName("exceed_count"), JAVA_DOUBLE.withName("max_occupy_ratio"),
            JAVA_INT.withName("max_flow_ids"), JAVA_INT.withName("heavy_min_events"),
            JAVA_INT.withName("aux_capacity"), JAVA_INT.withName("pad"));

    /** sf_flow_rule: 48 bytes.  limit_app: 0 "default", 1 "other", else an interned origin id;
     *  ref_resource: RELATE a resource id, CHAIN a context-name id (0xFFFFFFFF blank). */
    static final StructLayout FLOW_RULE = MemoryLayout.structLayout(
            JAVA_INT.withName("resource"), JAVA_INT.withName("grade"), JAVA_DOUBLE.withName("count"),
            JAVA_INT.withName("strategy"), JAVA_INT.withName("control_behavior"),
            JAVA_INT.withName("warm_up_period_sec"), JAVA_INT.withName("max_queueing_time_ms"),
            JAVA_INT.withName("cluster_mode"), JAVA_INT.withName("ref_resource"),
            JAVA_INT.withName("limit_app"), JAVA_INT.withName("cluster_fallback"));

    /** sf_hot_item: {u8 tag, pad[3], i32 count, u64 bits}: 16 bytes. */
    static final StructLayout HOT_ITEM = MemoryLayout.structLayout(
            java.lang.foreign.ValueLayout.JAVA_BYTE.withName("tag"), MemoryLayout.paddingLayout(3),
            JAVA_INT.withName("count"), JAVA_LONG.withName("bits"));

    /** sf_param_rule: 48 bytes. */
    static final StructLayout PARAM_RULE = MemoryLayout.structLayout(
            JAVA_INT.withName("resource"), JAVA_INT.withName("grade"), JAVA_INT.withName("param_idx"),
            JAVA_INT.withName("control_behavior"), JAVA_DOUBLE.withName("count"),
            JAVA_INT.withName("max_queueing_time_ms"), JAVA_INT.withName("burst_count"),
            JAVA_LONG.withName("duration_in_sec"), JAVA_INT.withName("item_offset"),
            JAVA_INT.withName("item_count"));

    /** sf_degrade_rule: 40 bytes. */
    static final StructLayout DEGRADE_RULE = MemoryLayout.structLayout(
            JAVA_INT.withName("resource"), JAVA_INT.withName("grade"), JAVA_DOUBLE.withName("count"),
            JAVA_INT.withName("time_window_s"), JAVA_INT.withName("min_request_amount"),
            JAVA_DOUBLE.withName("slow_ratio_threshold"), JAVA_INT.withName("stat_interval_ms"),
            JAVA_INT.withName("pad"));

    /** sf_system_rule: 40 bytes (negative = unset). */
    static final StructLayout SYSTEM_RULE = MemoryLayout.structLayout(
            JAVA_DOUBLE.withName("highest_system_load"), JAVA_DOUBLE.withName("highest_cpu_usage"),
            JAVA_DOUBLE.withName("qps"), JAVA_LONG.withName("avg_rt"), JAVA_LONG.withName("max_thread"));

    /** sf_event_batch: SoA pointers, host memory (mem = SF_MEM_HOST). */
    static final StructLayout EVENT_BATCH = MemoryLayout.structLayout(
            JAVA_INT.withName("n"), JAVA_INT.withName("mem"),
            ADDRESS.withName("res_id"), ADDRESS.withName("ts_ms"), ADDRESS.withName("count"),
            ADDRESS.withName("flags"), ADDRESS.withName("entry_ref"), ADDRESS.withName("create_ts"),
            JAVA_INT.withName("arg_slots"), MemoryLayout.paddingLayout(4),
            ADDRESS.withName("n_args"), ADDRESS.withName("arg_tag"), ADDRESS.withName("arg_bits"),
            ADDRESS.withName("arg_elem_off"), ADDRESS.withName("elem_tag"), ADDRESS.withName("elem_bits"),
            JAVA_INT.withName("n_elems"), MemoryLayout.paddingLayout(4),
            ADDRESS.withName("origin"), ADDRESS.withName("context"));

    /** sf_packed_batch: 8 bytes per event (res | ts - ts_base << 32 | count << 52 | flags << 59); the
     *  narrow form (ev NULL): ev4 words res | count << 24 | flags << 27 and the table ms_end[n_ms]. */
    static final StructLayout PACKED_BATCH = MemoryLayout.structLayout(
            JAVA_INT.withName("n"), JAVA_INT.withName("mem"), JAVA_LONG.withName("ts_base"),
            ADDRESS.withName("ev"), ADDRESS.withName("exit_ref"), ADDRESS.withName("exit_cts"),
            ADDRESS.withName("count_ext"), ADDRESS.withName("origin"),
            JAVA_INT.withName("n_exit"), JAVA_INT.withName("n_count_ext"),
            ADDRESS.withName("ev4"), ADDRESS.withName("ms_end"), JAVA_INT.withName("n_ms"),
            JAVA_INT.withName("pad0"));
    static final int PK_COUNT_SHIFT = 52, PK_FLAGS_SHIFT = 59;
    static final int PK4_COUNT_SHIFT = 24, PK4_FLAGS_SHIFT = 27, PK4_MAX_MS = 1048576;

    /** sf_verdicts. */
    static final StructLayout VERDICTS = MemoryLayout.structLayout(
            JAVA_INT.withName("mem"), MemoryLayout.paddingLayout(4),
            ADDRESS.withName("status"), ADDRESS.withName("wait_ms"), ADDRESS.withName("rule_idx"));

    /** sf_sparse_verdicts: 1 status byte per event plus (index << 32 | value) lists of the
     *  nonzero waits and rule indices (the copy back of a packed batch). */
    static final StructLayout SPARSE_VERDICTS = MemoryLayout.structLayout(
            ADDRESS.withName("status"), ADDRESS.withName("waits"), ADDRESS.withName("rules"),
            ADDRESS.withName("counts"), JAVA_INT.withName("prefetch"), JAVA_INT.withName("pad"));

    /** sf_token_batch. */
    static final StructLayout TOKEN_BATCH = MemoryLayout.structLayout(
            JAVA_INT.withName("n"), JAVA_INT.withName("mem"),
            ADDRESS.withName("flow_id"), ADDRESS.withName("count"), ADDRESS.withName("flags"),
            ADDRESS.withName("ts_ms"), ADDRESS.withName("param_tag"), ADDRESS.withName("param_bits"),
            ADDRESS.withName("param_off"));

    /** sf_token_results. */
    static final StructLayout TOKEN_RESULTS = MemoryLayout.structLayout(
            JAVA_INT.withName("mem"), MemoryLayout.paddingLayout(4),
            ADDRESS.withName("status"), ADDRESS.withName("remaining"), ADDRESS.withName("wait_ms"));

    // SF_EV_* / SF_V_* / SF_TOK_* / SF_TAG_* (sentinel_flow.h)
    static final byte EV_EXIT = 0x01, EV_IN = 0x02, EV_PRIO = 0x04, EV_ERROR = 0x08, EV_BLOCKED = 0x10;
    static final int V_PASS = 0, V_PASS_WAIT = 1, V_PRIORITY_WAIT = 2, V_BLOCK_FLOW = 3, V_BLOCK_PARAM = 4,
            V_BLOCK_SYSTEM = 5, V_EXIT = 6, V_EXIT_IGNORED = 7, V_BLOCK_DEGRADE = 8, V_BLOCK_OTHER = 9;
    static final byte TOK_PRIORITIZED = 0x01, TOK_PARAM = 0x02;
    static final byte TAG_NULL = 0, TAG_INT = 1, TAG_LONG = 2, TAG_STRING = 3, TAG_DOUBLE = 4, TAG_BOOL = 5,
            TAG_OTHER = 6, TAG_BYTE = 7, TAG_SHORT = 8, TAG_FLOAT = 9, TAG_COLLECTION = 0x40;

    /** Byte offset of a named field (the C struct's offsetof; tests/test_java_shim.py). */
    static long off(StructLayout layout, String field) {
        return layout.byteOffset(MemoryLayout.PathElement.groupElement(field));
    }

    static void check(int rc) {
        if (rc != 0) {
            String msg;
            try {
                MemorySegment p = (MemorySegment) LAST_ERROR.invokeExact();
                msg = p.reinterpret(4096).getString(0);
            } catch (Throwable t) {
                msg = "?";
            }
            throw new IllegalStateException("sentinel_flow error " + rc + ": " + msg);
        }
    }

    private SentinelFlowNative() {}
}
