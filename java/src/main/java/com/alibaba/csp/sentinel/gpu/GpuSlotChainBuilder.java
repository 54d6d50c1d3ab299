package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.slotchain.DefaultProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.SlotChainBuilder;
import com.alibaba.csp.sentinel.slots.block.authority.AuthoritySlot;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeSlot;
import com.alibaba.csp.sentinel.slots.clusterbuilder.ClusterBuilderSlot;
import com.alibaba.csp.sentinel.slots.logger.LogSlot;
import com.alibaba.csp.sentinel.slots.nodeselector.NodeSelectorSlot;
import com.alibaba.csp.sentinel.spi.Spi;

/**
 * SlotChainProvider.newSlotChain() takes the first SlotChainBuilder that is
 * not the default (SlotChainProvider.java:39-56, SpiLoader.java:228-238).
 * This one keeps the reference's slots around the GPU slot; the statistic,
 * system, param-flow and flow checks are one GpuFlowSlot.  AuthoritySlot runs
 * before it (its origin check reads no statistics); DegradeSlot after it, as
 * in the reference order (Constants.ORDER_*).  For the GPU circuit breakers
 * replace DegradeSlot with a slot over sf_degrade_submit (INTEGRATION.md §2).
 */
@Spi(order = -100)
public final class GpuSlotChainBuilder implements SlotChainBuilder {
    @Override
    public ProcessorSlotChain build() {
        ProcessorSlotChain chain = new DefaultProcessorSlotChain();
        chain.addLast(new NodeSelectorSlot());
        chain.addLast(new ClusterBuilderSlot());
        chain.addLast(new LogSlot());
        chain.addLast(new AuthoritySlot());
        chain.addLast(new GpuFlowSlot(GpuEngine.get()));
        chain.addLast(new DegradeSlot());
        return chain;
    }
}
