package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.slots.block.RuleConstant;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowItem;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRuleManager;
import com.alibaba.csp.sentinel.slots.system.SystemRule;
import com.alibaba.csp.sentinel.slots.system.SystemRuleManager;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.atomic.AtomicLong;

import static com.alibaba.csp.sentinel.gpu.SentinelFlowNative.*;
import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * One engine per JVM (one GPU): resource-name interning, rule reloads and the
 * native handle.  The rule lists are read from the reference managers, so
 * their order is the managers' own (FlowRuleUtil.buildFlowRuleMap: HashSet,
 * then the stable FlowRuleComparator sort; ParamFlowRuleUtil: HashSet), which
 * is the order sf_load_*_rules expects.  Hosts without the Java managers get
 * the same order from sf_flow_rule_order / sf_param_rule_order.
 */
public final class GpuEngine {
    private static volatile GpuEngine INSTANCE;

    public static GpuEngine get() {
        GpuEngine e = INSTANCE;
        if (e == null) {
            synchronized (GpuEngine.class) {
                if (INSTANCE == null) INSTANCE = new GpuEngine(Integer.getInteger("sentinel.gpu.maxResources", 1 << 20),
                        Integer.getInteger("sentinel.gpu.maxBatch", 1 << 20));
                e = INSTANCE;
            }
        }
        return e;
    }

    final MemorySegment handle;
    private final Arena arena = Arena.ofShared();
    private final ConcurrentHashMap<String, Integer> resourceIds = new ConcurrentHashMap<>();
    private final int maxResources;
    /** Bumped by {@link #reloadRules()}; the batcher reloads before its next submit. */
    final AtomicLong ruleVersion = new AtomicLong();
    /** Per resource: the rule lists the engine's rule indices refer to (exception payloads). */
    volatile Map<Integer, List<FlowRule>> flowRulesByResource = new HashMap<>();
    volatile Map<Integer, List<ParamFlowRule>> paramRulesByResource = new HashMap<>();
    final EventBatcher batcher;

    private GpuEngine(int maxResources, int maxBatch) {
        this.maxResources = maxResources;
        MemorySegment cfg = arena.allocate(CONFIG);
        try {
            CONFIG_DEFAULT.invokeExact(cfg);
            cfg.set(JAVA_INT, CONFIG.byteOffset(MemoryLayout_path("max_resources")), maxResources);
            cfg.set(JAVA_INT, CONFIG.byteOffset(MemoryLayout_path("max_batch")), maxBatch);
            MemorySegment out = arena.allocate(ADDRESS);
            check((int) CREATE.invokeExact(cfg, out));
            handle = out.get(ADDRESS, 0);
        } catch (RuntimeException ex) {
            throw ex;
        } catch (Throwable t) {
            throw new IllegalStateException(t);
        }
        batcher = new EventBatcher(this, maxBatch);
        reloadRules();
    }

    private static java.lang.foreign.MemoryLayout.PathElement MemoryLayout_path(String name) {
        return java.lang.foreign.MemoryLayout.PathElement.groupElement(name);
    }

    /** Dense id of a resource name (ResourceWrapper identity is the name, ResourceWrapper.java:81-95). */
    int resourceId(String name) {
        Integer id = resourceIds.get(name);
        if (id != null) return id;
        synchronized (resourceIds) {
            return resourceIds.computeIfAbsent(name, k -> {
                int v = resourceIds.size();
                if (v >= maxResources) throw new IllegalStateException("more than " + maxResources + " resources");
                return v;
            });
        }
    }

    private final ConcurrentHashMap<String, Integer> originIds = new ConcurrentHashMap<>();
    private final ConcurrentHashMap<String, Integer> contextIds = new ConcurrentHashMap<>();

    /** Origin / limitApp id: "default" 0, "other" 1, names from 2; "" (no origin) -1 (SF_ORIGIN_NONE). */
    int originId(String origin) {
        if (origin == null || origin.isEmpty()) return -1;
        if (RuleConstant.LIMIT_APP_DEFAULT.equals(origin)) return 0;
        if (RuleConstant.LIMIT_APP_OTHER.equals(origin)) return 1;
        Integer id = originIds.get(origin);
        if (id != null) return id;
        synchronized (originIds) {
            return originIds.computeIfAbsent(origin, k -> originIds.size() + 2);
        }
    }

    /** Context-name id (CHAIN refResource / Context.getName()). */
    int contextId(String name) {
        Integer id = contextIds.get(name);
        if (id != null) return id;
        synchronized (contextIds) {
            return contextIds.computeIfAbsent(name, k -> contextIds.size());
        }
    }

    /** Called after FlowRuleManager / ParamFlowRuleManager / SystemRuleManager.loadRules. */
    public void reloadRules() {
        ruleVersion.incrementAndGet();
    }

    /** Runs on the flusher thread (the engine is single-threaded). */
    void loadRulesNow() throws Throwable {
        try (Arena a = Arena.ofConfined()) {
            // flow rules: one sf_flow_rule per rule, in the manager's per-resource order
            List<FlowRule> flow = FlowRuleManager.getRules();
            Map<Integer, List<FlowRule>> byRes = new HashMap<>();
            MemorySegment fr = a.allocate(FLOW_RULE, Math.max(1, flow.size()));
            int i = 0;
            for (FlowRule r : flow) {
                int res = resourceId(r.getResource());
                byRes.computeIfAbsent(res, k -> new ArrayList<>()).add(r);
                MemorySegment s = fr.asSlice((long) i++ * FLOW_RULE.byteSize(), FLOW_RULE.byteSize());
                s.set(JAVA_INT, 0, res);
                s.set(JAVA_INT, 4, r.getGrade());
                s.set(JAVA_DOUBLE, 8, r.getCount());
                s.set(JAVA_INT, 16, r.getStrategy());
                s.set(JAVA_INT, 20, r.getControlBehavior());
                s.set(JAVA_INT, 24, r.getWarmUpPeriodSec());
                s.set(JAVA_INT, 28, r.getMaxQueueingTimeMs());
                s.set(JAVA_INT, 32, r.isClusterMode() ? 1 : 0);
                String ref = r.getRefResource();
                int refId = ref == null || ref.isEmpty() ? -1            // SF_REF_NONE
                        : r.getStrategy() == RuleConstant.STRATEGY_CHAIN ? contextId(ref) : resourceId(ref);
                s.set(JAVA_INT, 36, refId);
                String app = r.getLimitApp();                            // blank -> "default" (FlowRuleUtil.java:99-101)
                s.set(JAVA_INT, 40, app == null || app.trim().isEmpty() ? 0 : originId(app));
                s.set(JAVA_INT, 44, r.getClusterConfig() == null || r.getClusterConfig().isFallbackToLocalWhenFail() ? 1 : 0);
            }
            check((int) LOAD_FLOW.invokeExact(handle, fr, flow.size()));
            flowRulesByResource = byRes;

            // param rules + hot items
            List<ParamFlowRule> param = ParamFlowRuleManager.getRules();
            Map<Integer, List<ParamFlowRule>> pByRes = new HashMap<>();
            int nItems = 0;
            for (ParamFlowRule r : param) nItems += r.getParamFlowItemList() == null ? 0 : r.getParamFlowItemList().size();
            MemorySegment pr = a.allocate(PARAM_RULE, Math.max(1, param.size()));
            MemorySegment items = a.allocate(HOT_ITEM, Math.max(1, nItems));
            int k = 0, it = 0;
            for (ParamFlowRule r : param) {
                int res = resourceId(r.getResource());
                pByRes.computeIfAbsent(res, x -> new ArrayList<>()).add(r);
                MemorySegment s = pr.asSlice((long) k++ * PARAM_RULE.byteSize(), PARAM_RULE.byteSize());
                s.set(JAVA_INT, 0, res);
                s.set(JAVA_INT, 4, r.getGrade());
                s.set(JAVA_INT, 8, r.getParamIdx() == null ? 0 : r.getParamIdx());
                s.set(JAVA_INT, 12, r.getControlBehavior());
                s.set(JAVA_DOUBLE, 16, r.getCount());
                s.set(JAVA_INT, 24, r.getMaxQueueingTimeMs());
                s.set(JAVA_INT, 28, r.getBurstCount());
                s.set(JAVA_LONG, 32, r.getDurationInSec());
                s.set(JAVA_INT, 40, it);
                int cnt = 0;
                if (r.getParamFlowItemList() != null) {
                    for (ParamFlowItem item : r.getParamFlowItemList()) {
                        Object v = HotItems.parse(item);          // ParamFlowRuleUtil.parseValue (:188-240)
                        if (v == null) continue;
                        MemorySegment h = items.asSlice((long) it++ * HOT_ITEM.byteSize(), HOT_ITEM.byteSize());
                        h.set(JAVA_BYTE, 0, ParamPacker.tag(v));
                        h.set(JAVA_INT, 4, item.getCount());
                        h.set(JAVA_LONG, 8, ParamPacker.bits(v));
                        cnt++;
                    }
                }
                s.set(JAVA_INT, 44, cnt);
            }
            check((int) LOAD_PARAM.invokeExact(handle, pr, param.size(), items, it));
            paramRulesByResource = pByRes;

            // system rules (SystemRuleManager.loadSystemConf keeps the minimum of each threshold)
            List<SystemRule> sys = SystemRuleManager.getRules();
            MemorySegment sr = a.allocate(SYSTEM_RULE, Math.max(1, sys.size()));
            int j = 0;
            for (SystemRule r : sys) {
                MemorySegment s = sr.asSlice((long) j++ * SYSTEM_RULE.byteSize(), SYSTEM_RULE.byteSize());
                s.set(JAVA_DOUBLE, 0, r.getHighestSystemLoad());
                s.set(JAVA_DOUBLE, 8, r.getHighestCpuUsage());
                s.set(JAVA_DOUBLE, 16, r.getQps());
                s.set(JAVA_LONG, 24, r.getAvgRt());
                s.set(JAVA_LONG, 32, r.getMaxThread());
            }
            check((int) LOAD_SYSTEM.invokeExact(handle, sr, sys.size()));
        }
    }

    /** SystemStatusListener's load and cpu, pushed before each batch (SystemRuleManager.java:300-330). */
    void pushSystemStatus() throws Throwable {
        check((int) SET_SYSTEM_STATUS.invokeExact(handle, SystemRuleManager.getCurrentSystemAvgLoad(),
                SystemRuleManager.getCurrentCpuUsage()));
    }
}
