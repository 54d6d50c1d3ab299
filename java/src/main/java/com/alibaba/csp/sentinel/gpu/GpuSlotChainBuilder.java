package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.slotchain.DefaultProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.SlotChainBuilder;
import com.alibaba.csp.sentinel.slots.clusterbuilder.ClusterBuilderSlot;
import com.alibaba.csp.sentinel.slots.logger.LogSlot;
import com.alibaba.csp.sentinel.slots.nodeselector.NodeSelectorSlot;
import com.alibaba.csp.sentinel.spi.Spi;

/**
 * SlotChainProvider.newSlotChain() takes the first SlotChainBuilder that is
 * not the default (SlotChainProvider.java:39-56, SpiLoader.java:228-238).
 * The reference's slots before StatisticSlot stay (NodeSelectorSlot -10000,
 * ClusterBuilderSlot -9000, LogSlot -8000); StatisticSlot and everything it
 * wraps -- AuthoritySlot, SystemSlot, ParamFlowSlot, FlowSlot, DegradeSlot
 * (Constants.java:77-84) -- is one GpuFlowSlot: the engine accounts for every
 * outcome of those slots as StatisticSlot does (StatisticSlot.java:55-131),
 * including the circuit breakers (DegradeRuleManager's rules, loaded into the
 * engine) and AuthorityExceptions (AuthoritySlot runs inside GpuFlowSlot).
 */
@Spi(order = -100)
public final class GpuSlotChainBuilder implements SlotChainBuilder {
    @Override
    public ProcessorSlotChain build() {
        ProcessorSlotChain chain = new DefaultProcessorSlotChain();
        chain.addLast(new NodeSelectorSlot());
        chain.addLast(new ClusterBuilderSlot());
        chain.addLast(new LogSlot());
        chain.addLast(new GpuFlowSlot(GpuEngine.get()));
        return chain;
    }
}
