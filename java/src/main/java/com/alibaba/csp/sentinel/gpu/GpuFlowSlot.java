package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.EntryType;
import com.alibaba.csp.sentinel.context.Context;
import com.alibaba.csp.sentinel.node.DefaultNode;
import com.alibaba.csp.sentinel.slotchain.AbstractLinkedProcessorSlot;
import com.alibaba.csp.sentinel.slotchain.ResourceWrapper;
import com.alibaba.csp.sentinel.slots.block.BlockException;
import com.alibaba.csp.sentinel.slots.block.flow.FlowException;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowException;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.system.SystemBlockException;
import com.alibaba.csp.sentinel.util.TimeUtil;

import java.util.List;

import static com.alibaba.csp.sentinel.gpu.SentinelFlowNative.*;

/**
 * StatisticSlot + SystemSlot + ParamFlowSlot + FlowSlot in one slot, decided
 * on the GPU: each entry and exit becomes one event of the engine's next
 * batch (EventBatcher), and the verdict is turned back into the reference's
 * behaviour (StatisticSlot.java:64-130, DefaultController.java:60-72,
 * RateLimiterController.java:80-95, SystemRuleManager.java:291-348,
 * ParamFlowSlot.java:58-88).  The statistics the reference keeps in
 * StatisticNode live in the engine (sf_read_node / sf_snapshot serve the
 * dashboard and MetricWriter); the DefaultNode passed along is untouched.
 */
public class GpuFlowSlot extends AbstractLinkedProcessorSlot<DefaultNode> {
    private static final String[] SYSTEM_LIMIT = {"qps", "thread", "rt", "load", "cpu"};
    private static final String TICKET_KEY = "sentinel.gpu.ticket";
    private final GpuEngine engine;

    public GpuFlowSlot(GpuEngine engine) {
        this.engine = engine;
    }

    @Override
    public void entry(Context context, ResourceWrapper resourceWrapper, DefaultNode node, int count,
                      boolean prioritized, Object... args) throws Throwable {
        EventBatcher.Ticket t = new EventBatcher.Ticket();
        t.resource = engine.resourceId(resourceWrapper.getName());
        t.origin = engine.originId(context.getOrigin());    // limitApp / origin node (FlowRuleChecker.java:129-161)
        t.context = engine.contextId(context.getName());    // CHAIN rules' DefaultNode
        t.count = count;
        t.flags = (byte) ((resourceWrapper.getEntryType() == EntryType.IN ? EV_IN : 0) | (prioritized ? EV_PRIO : 0));
        t.ts = TimeUtil.currentTimeMillis();
        t.args = args;
        engine.batcher.submit(t);
        switch (t.status) {
            case V_PASS:
                break;
            case V_PASS_WAIT:                                  // RateLimiterController: sleep, then pass
                if (t.waitMs > 0) Thread.sleep(t.waitMs);
                break;
            case V_PRIORITY_WAIT:                              // DefaultController occupy: sleep, pass borrowed
                Thread.sleep(t.waitMs);                        // (the engine counted it as PriorityWaitException)
                break;
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
                throw block(context, new ParamFlowException(resourceWrapper.getName(), String.valueOf(value), rule));
            }
            case V_BLOCK_SYSTEM:
                throw block(context, new SystemBlockException(resourceWrapper.getName(), SYSTEM_LIMIT[t.ruleIdx]));
            default:
                throw new IllegalStateException("unexpected verdict " + t.status);
        }
        remember(context, t);
        // the slots after FlowSlot (AuthoritySlot has run before, DegradeSlot after)
        fireEntry(context, resourceWrapper, node, count, prioritized, args);
    }

    private static BlockException block(Context context, BlockException e) {
        context.getCurEntry().setBlockError(e);               // StatisticSlot.java:99-101
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
            engine.batcher.submit(t);                         // SF_V_EXIT: recorded (RT, success, thread count)
        }
        fireExit(context, resourceWrapper, count, args);
    }
}
