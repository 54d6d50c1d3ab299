package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.EntryType;
import com.alibaba.csp.sentinel.context.Context;
import com.alibaba.csp.sentinel.node.DefaultNode;
import com.alibaba.csp.sentinel.slotchain.AbstractLinkedProcessorSlot;
import com.alibaba.csp.sentinel.slotchain.ResourceWrapper;
import com.alibaba.csp.sentinel.slots.block.BlockException;
import com.alibaba.csp.sentinel.slots.block.authority.AuthorityException;
import com.alibaba.csp.sentinel.slots.block.authority.AuthoritySlot;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeException;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRule;
import com.alibaba.csp.sentinel.slots.block.flow.FlowException;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowException;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.system.SystemBlockException;
import com.alibaba.csp.sentinel.util.TimeUtil;

import java.util.List;

import static com.alibaba.csp.sentinel.gpu.SentinelFlowNative.*;

/**
 * The default chain's StatisticSlot (-7000) and every slot it wraps --
 * AuthoritySlot (-6000), SystemSlot (-5000), ParamFlowSlot (-3000), FlowSlot
 * (-2000), DegradeSlot (-1000) (Constants.java:77-84) -- in one slot whose
 * checks and statistics run on the GPU.  Each entry and exit is one event of
 * the engine's next batch (EventBatcher); the engine does StatisticSlot's
 * accounting of every outcome (StatisticSlot.java:55-131), so this slot only
 * turns the verdict back into the reference's behaviour:
 * <ul>
 * <li>AuthoritySlot reads no statistics and runs here, on the caller's thread,
 * before the event is submitted: an AuthorityException is submitted as an
 * SF_EV_BLOCKED entry (the engine counts block += count on the node and, for
 * an IN entry, on ENTRY_NODE, and runs no other check), then thrown;</li>
 * <li>SystemBlockException, ParamFlowException, FlowException and
 * DegradeException (the engine's circuit breakers, loaded from
 * DegradeRuleManager) are thrown with the blocking rule, after setting the
 * entry's blockError as StatisticSlot does (:102-105);</li>
 * <li>PASS_WAIT: RateLimiterController slept, then passed (:80-95);
 * PRIORITY_WAIT: DefaultController slept and threw PriorityWaitException,
 * which StatisticSlot catches (:86-101) -- the entry returns normally and the
 * slots after FlowSlot (DegradeSlot, any later slot) do not run.</li>
 * </ul>
 * The exit of a passed entry is one EXIT event (RT, success, thread count,
 * breaker completion); a blocked entry's exit submits nothing (:139).
 * The statistics live in the engine (sf_read_node / sf_snapshot serve the
 * dashboard and MetricWriter); the DefaultNode passed along is untouched.
 */
public class GpuFlowSlot extends AbstractLinkedProcessorSlot<DefaultNode> {
    private static final String[] SYSTEM_LIMIT = {"qps", "thread", "rt", "load", "cpu"};
    private final GpuEngine engine;
    /** The reference AuthoritySlot, ending the chain it is called through (no next slot). */
    private final AuthoritySlot authority = new AuthoritySlot();

    public GpuFlowSlot(GpuEngine engine) {
        this.engine = engine;
        authority.setNext(new AbstractLinkedProcessorSlot<DefaultNode>() {
            @Override
            public void entry(Context c, ResourceWrapper r, DefaultNode n, int k, boolean p, Object... a) {}

            @Override
            public void exit(Context c, ResourceWrapper r, int k, Object... a) {}
        });
    }

    private EventBatcher.Ticket ticket(Context context, ResourceWrapper resourceWrapper, int count, boolean prioritized,
                                       Object[] args) {
        EventBatcher.Ticket t = new EventBatcher.Ticket();
        t.resource = engine.resourceId(resourceWrapper.getName());
        t.origin = engine.originId(context.getOrigin());    // limitApp / origin node (FlowRuleChecker.java:129-161)
        t.context = engine.contextId(context.getName());    // CHAIN rules' DefaultNode
        t.count = count;
        t.flags = (byte) ((resourceWrapper.getEntryType() == EntryType.IN ? EV_IN : 0) | (prioritized ? EV_PRIO : 0));
        t.ts = TimeUtil.currentTimeMillis();
        t.args = args;
        return t;
    }

    @Override
    public void entry(Context context, ResourceWrapper resourceWrapper, DefaultNode node, int count,
                      boolean prioritized, Object... args) throws Throwable {
        EventBatcher.Ticket t = ticket(context, resourceWrapper, count, prioritized, args);
        try {
            authority.entry(context, resourceWrapper, node, count, prioritized, args);   // AuthoritySlot.java:38-44
        } catch (AuthorityException ex) {
            t.flags |= EV_BLOCKED;                           // counted as a block by the engine's StatisticSlot
            engine.batcher.submit(t);
            throw block(context, ex);
        }
        engine.batcher.submit(t);
        switch (t.status) {
            case V_PASS:
                break;
            case V_PASS_WAIT:                                  // RateLimiterController: sleep, then pass
                if (t.waitMs > 0) Thread.sleep(t.waitMs);
                break;
            case V_PRIORITY_WAIT:                              // DefaultController occupy: sleep, then
                Thread.sleep(t.waitMs);                        // PriorityWaitException, caught by StatisticSlot
                remember(context, t);
                return;                                        // (no later slot runs)
            case V_BLOCK_FLOW: {
                List<FlowRule> rules = engine.flowRulesByResource.get(t.resource);
                FlowRule rule = rules != null && t.ruleIdx < rules.size() ? rules.get(t.ruleIdx) : null;
                throw block(context, new FlowException(rule == null ? "default" : rule.getLimitApp(), rule));
            }
            case V_BLOCK_PARAM: {
                List<ParamFlowRule> rules = engine.paramRulesByResource.get(t.resource);
                ParamFlowRule rule = rules != null && t.ruleIdx < rules.size() ? rules.get(t.ruleIdx) : null;
                Object value = rule != null && args != null && rule.getParamIdx() != null ?
                        args[rule.getParamIdx() < 0 ? args.length + rule.getParamIdx() : rule.getParamIdx()] : null;
                throw block(context, new ParamFlowException(resourceWrapper.getName(),
                        String.valueOf(ParamPacker.key(value)), rule));
            }
            case V_BLOCK_SYSTEM:
                throw block(context, new SystemBlockException(resourceWrapper.getName(), SYSTEM_LIMIT[t.ruleIdx]));
            case V_BLOCK_DEGRADE: {                            // DegradeSlot.performChecking (DegradeSlot.java:50-61)
                List<DegradeRule> rules = engine.degradeRulesByResource.get(t.resource);
                DegradeRule rule = rules != null && t.ruleIdx < rules.size() ? rules.get(t.ruleIdx) : null;
                throw block(context, new DegradeException(rule == null ? "default" : rule.getLimitApp(), rule));
            }
            default:
                throw new IllegalStateException("unexpected verdict " + t.status);
        }
        remember(context, t);
        fireEntry(context, resourceWrapper, node, count, prioritized, args);
    }

    private static BlockException block(Context context, BlockException e) {
        context.getCurEntry().setBlockError(e);               // StatisticSlot.java:102-105
        return e;
    }

    /** The ticket of each passed entry until its exit (entry_ref / create_ts of the EXIT event). */
    private static final java.util.concurrent.ConcurrentHashMap<com.alibaba.csp.sentinel.Entry, EventBatcher.Ticket>
            ENTRY_TICKETS = new java.util.concurrent.ConcurrentHashMap<>();

    private static void remember(Context context, EventBatcher.Ticket t) {
        ENTRY_TICKETS.put(context.getCurEntry(), t);
    }

    @Override
    public void exit(Context context, ResourceWrapper resourceWrapper, int count, Object... args) {
        EventBatcher.Ticket entry = ENTRY_TICKETS.remove(context.getCurEntry());
        if (context.getCurEntry().getBlockError() == null && entry != null) {
            EventBatcher.Ticket t = new EventBatcher.Ticket();
            t.resource = entry.resource;
            t.origin = entry.origin; t.context = entry.context;
            t.count = count;
            t.flags = (byte) (EV_EXIT | (entry.flags & EV_IN)
                    | (context.getCurEntry().getError() != null ? EV_ERROR : 0));
            t.ts = TimeUtil.currentTimeMillis();
            t.entry = entry;
            t.createTs = context.getCurEntry().getCreateTimestamp();
            t.args = args;
            engine.batcher.submit(t);                         // SF_V_EXIT: StatisticSlot.exit + DegradeSlot.exit
        }
        fireExit(context, resourceWrapper, count, args);
    }
}
