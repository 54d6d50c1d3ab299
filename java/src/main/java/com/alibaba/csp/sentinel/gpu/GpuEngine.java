package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.property.PropertyListener;
import com.alibaba.csp.sentinel.property.SentinelProperty;
import com.alibaba.csp.sentinel.slots.block.RuleConstant;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRule;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowItem;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRuleManager;
import com.alibaba.csp.sentinel.slots.system.SystemRule;
import com.alibaba.csp.sentinel.slots.system.SystemRuleManager;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.lang.invoke.MethodHandles;
import java.lang.invoke.VarHandle;
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
    /** Per resource: its circuit breakers' rules in the engine's breaker order (DegradeException payload). */
    volatile Map<Integer, List<DegradeRule>> degradeRulesByResource = new HashMap<>();
    final EventBatcher batcher;

    private GpuEngine(int maxResources, int maxBatch) {
        this.maxResources = maxResources;
        MemorySegment cfg = arena.allocate(CONFIG);
        try {
            CONFIG_DEFAULT.invokeExact(cfg);
            cfg.set(JAVA_INT, off(CONFIG, "max_resources"), maxResources);
            cfg.set(JAVA_INT, off(CONFIG, "max_batch"), maxBatch);
            MemorySegment out = arena.allocate(ADDRESS);
            check((int) CREATE.invokeExact(cfg, out));
            handle = out.get(ADDRESS, 0);
        } catch (RuntimeException ex) {
            throw ex;
        } catch (Throwable t) {
            throw new IllegalStateException(t);
        }
        batcher = new EventBatcher(this, maxBatch);
        installRuleListeners();
        reloadRules();
    }

    /**
     * Every FlowRuleManager / ParamFlowRuleManager / SystemRuleManager /
     * DegradeRuleManager.loadRules reaches the engine without a manual
     * {@link #reloadRules()}.  The engine never calls a manager's
     * register2Property: that would hand the manager a property whose value is
     * null, and DynamicSentinelProperty.addListener runs configLoad(null) at once
     * (DynamicSentinelProperty.java:37-40), which replaces the manager's rules by
     * an empty map (FlowRuleUtil.java:85-88) and detaches whatever data-source
     * property the application registered before (FlowRuleManager.java:92-100,
     * NacosDataSourceDemo.java:67).  Instead our listener is added to the
     * property each manager holds right now (its private static currentProperty;
     * loadRules is currentProperty.updateValue, FlowRuleManager.java:120-122), and
     * {@link #followRuleProperties()} re-attaches it whenever the application
     * later swaps a manager's property (register2Property of a data source), so
     * both orders -- loadRules / a data source before or after the first
     * SphU.entry -- keep the manager's live rules and reach the engine.
     */
    private void installRuleListeners() {
        followRuleProperties();
    }

    /** The four managers' property slots, read reflectively (private static currentProperty). */
    private static final VarHandle[] PROPERTY_SLOTS = {
            propertySlot(FlowRuleManager.class), propertySlot(ParamFlowRuleManager.class),
            propertySlot(SystemRuleManager.class), propertySlot(DegradeRuleManager.class)};
    private final Object[] followed = new Object[PROPERTY_SLOTS.length];
    private final PropertyListener<Object> listener = ruleListener();

    private static VarHandle propertySlot(Class<?> manager) {
        try {
            return MethodHandles.privateLookupIn(manager, MethodHandles.lookup())
                    .findStaticVarHandle(manager, "currentProperty", SentinelProperty.class);
        } catch (ReflectiveOperationException ex) {
            throw new IllegalStateException("rule manager without currentProperty: " + manager.getName(), ex);
        }
    }

    /**
     * Adds our listener to every manager's current property it is not on yet
     * (addListener's configLoad only bumps the rule version).  Called at start and
     * by the flusher before each batch, so a property swapped in by a data source
     * is followed from the next batch on; the old property keeps our listener,
     * which is harmless (the manager no longer listens to it).
     */
    @SuppressWarnings("unchecked")
    synchronized void followRuleProperties() {
        for (int i = 0; i < PROPERTY_SLOTS.length; i++) {
            Object p = PROPERTY_SLOTS[i].getVolatile();
            if (p != null && p != followed[i]) {
                followed[i] = p;
                ((SentinelProperty<Object>) p).addListener(listener);
            }
        }
    }

    /** A property listener that bumps the rule version (add it to a data-source property). */
    public <T> PropertyListener<T> ruleListener() {
        return new PropertyListener<T>() {
            @Override public void configUpdate(T value) { reloadRules(); }
            @Override public void configLoad(T value) { reloadRules(); }
        };
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

    /** Bumps the rule version; called by the managers' property listeners (installRuleListeners). */
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
                s.set(JAVA_INT, off(FLOW_RULE, "resource"), res);
                s.set(JAVA_INT, off(FLOW_RULE, "grade"), r.getGrade());
                s.set(JAVA_DOUBLE, off(FLOW_RULE, "count"), r.getCount());
                s.set(JAVA_INT, off(FLOW_RULE, "strategy"), r.getStrategy());
                s.set(JAVA_INT, off(FLOW_RULE, "control_behavior"), r.getControlBehavior());
                s.set(JAVA_INT, off(FLOW_RULE, "warm_up_period_sec"), r.getWarmUpPeriodSec());
                s.set(JAVA_INT, off(FLOW_RULE, "max_queueing_time_ms"), r.getMaxQueueingTimeMs());
                s.set(JAVA_INT, off(FLOW_RULE, "cluster_mode"), r.isClusterMode() ? 1 : 0);
                String ref = r.getRefResource();
                int refId = ref == null || ref.isEmpty() ? -1            // SF_REF_NONE
                        : r.getStrategy() == RuleConstant.STRATEGY_CHAIN ? contextId(ref) : resourceId(ref);
                s.set(JAVA_INT, off(FLOW_RULE, "ref_resource"), refId);
                String app = r.getLimitApp();                            // blank -> "default" (FlowRuleUtil.java:99-101)
                s.set(JAVA_INT, off(FLOW_RULE, "limit_app"), app == null || app.trim().isEmpty() ? 0 : originId(app));
                s.set(JAVA_INT, off(FLOW_RULE, "cluster_fallback"), r.getClusterConfig() == null || r.getClusterConfig().isFallbackToLocalWhenFail() ? 1 : 0);
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
                s.set(JAVA_INT, off(PARAM_RULE, "resource"), res);
                s.set(JAVA_INT, off(PARAM_RULE, "grade"), r.getGrade());
                s.set(JAVA_INT, off(PARAM_RULE, "param_idx"), r.getParamIdx() == null ? 0 : r.getParamIdx());
                s.set(JAVA_INT, off(PARAM_RULE, "control_behavior"), r.getControlBehavior());
                s.set(JAVA_DOUBLE, off(PARAM_RULE, "count"), r.getCount());
                s.set(JAVA_INT, off(PARAM_RULE, "max_queueing_time_ms"), r.getMaxQueueingTimeMs());
                s.set(JAVA_INT, off(PARAM_RULE, "burst_count"), r.getBurstCount());
                s.set(JAVA_LONG, off(PARAM_RULE, "duration_in_sec"), r.getDurationInSec());
                s.set(JAVA_INT, off(PARAM_RULE, "item_offset"), it);
                int cnt = 0;
                if (r.getParamFlowItemList() != null) {
                    for (ParamFlowItem item : r.getParamFlowItemList()) {
                        Object v = HotItems.parse(item);          // ParamFlowRuleUtil.parseValue (:188-240)
                        if (v == null) continue;
                        MemorySegment h = items.asSlice((long) it++ * HOT_ITEM.byteSize(), HOT_ITEM.byteSize());
                        h.set(JAVA_BYTE, off(HOT_ITEM, "tag"), ParamPacker.tag(v));
                        h.set(JAVA_INT, off(HOT_ITEM, "count"), item.getCount());
                        h.set(JAVA_LONG, off(HOT_ITEM, "bits"), ParamPacker.bits(v));
                        cnt++;
                    }
                }
                s.set(JAVA_INT, off(PARAM_RULE, "item_count"), cnt);
            }
            check((int) LOAD_PARAM.invokeExact(handle, pr, param.size(), items, it));
            paramRulesByResource = pByRes;

            // system rules (SystemRuleManager.loadSystemConf keeps the minimum of each threshold)
            List<SystemRule> sys = SystemRuleManager.getRules();
            MemorySegment sr = a.allocate(SYSTEM_RULE, Math.max(1, sys.size()));
            int j = 0;
            for (SystemRule r : sys) {
                MemorySegment s = sr.asSlice((long) j++ * SYSTEM_RULE.byteSize(), SYSTEM_RULE.byteSize());
                s.set(JAVA_DOUBLE, off(SYSTEM_RULE, "highest_system_load"), r.getHighestSystemLoad());
                s.set(JAVA_DOUBLE, off(SYSTEM_RULE, "highest_cpu_usage"), r.getHighestCpuUsage());
                s.set(JAVA_DOUBLE, off(SYSTEM_RULE, "qps"), r.getQps());
                s.set(JAVA_LONG, off(SYSTEM_RULE, "avg_rt"), r.getAvgRt());
                s.set(JAVA_LONG, off(SYSTEM_RULE, "max_thread"), r.getMaxThread());
            }
            check((int) LOAD_SYSTEM.invokeExact(handle, sr, sys.size()));

            // circuit breakers: DegradeSlot is the last slot of the engine's chain.  The valid
            // rules (DegradeRuleManager.isValidRule :183-204) in list order; sf_load_degrade_rules
            // keeps the breaker of every unchanged rule (getExistingSameCbOrNew :151-163) and
            // rule_idx of a DegradeException is the position in the resource's list
            List<DegradeRule> dg = new ArrayList<>();
            for (DegradeRule r : DegradeRuleManager.getRules()) if (DegradeRuleManager.isValidRule(r)) dg.add(r);
            Map<Integer, List<DegradeRule>> dByRes = new HashMap<>();
            MemorySegment dr = a.allocate(DEGRADE_RULE, Math.max(1, dg.size()));
            int d = 0;
            for (DegradeRule r : dg) {
                int res = resourceId(r.getResource());
                dByRes.computeIfAbsent(res, x -> new ArrayList<>()).add(r);
                MemorySegment s = dr.asSlice((long) d++ * DEGRADE_RULE.byteSize(), DEGRADE_RULE.byteSize());
                s.set(JAVA_INT, off(DEGRADE_RULE, "resource"), res);
                s.set(JAVA_INT, off(DEGRADE_RULE, "grade"), r.getGrade());
                s.set(JAVA_DOUBLE, off(DEGRADE_RULE, "count"), r.getCount());
                s.set(JAVA_INT, off(DEGRADE_RULE, "time_window_s"), r.getTimeWindow());
                s.set(JAVA_INT, off(DEGRADE_RULE, "min_request_amount"), r.getMinRequestAmount());
                s.set(JAVA_DOUBLE, off(DEGRADE_RULE, "slow_ratio_threshold"), r.getSlowRatioThreshold());
                s.set(JAVA_INT, off(DEGRADE_RULE, "stat_interval_ms"), r.getStatIntervalMs());
                s.set(JAVA_INT, off(DEGRADE_RULE, "pad"), 0);
            }
            check((int) LOAD_DEGRADE.invokeExact(handle, dr, dg.size(), MemorySegment.NULL));
            degradeRulesByResource = dByRes;
        }
    }

    /** SystemStatusListener's load and cpu, pushed before each batch (SystemRuleManager.java:300-330). */
    void pushSystemStatus() throws Throwable {
        check((int) SET_SYSTEM_STATUS.invokeExact(handle, SystemRuleManager.getCurrentSystemAvgLoad(),
                SystemRuleManager.getCurrentCpuUsage()));
    }
}
