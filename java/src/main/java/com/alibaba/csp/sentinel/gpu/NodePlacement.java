package com.alibaba.csp.sentinel.gpu;

import java.util.Arrays;

/**
 * Resource placement over the GPUs of a node (one engine per GPU, each created
 * with shard_count = N and shard_index = its rank): the routing a multi-GPU
 * host puts in front of {@link EventBatcher}s, the Java twin of
 * sentinel_amd/placement.py.  An engine owns the resources whose engine id
 * e satisfies e % N == rank.  By default a resource's engine id is its dense
 * id ({@link GpuEngine#resourceId}); {@link #balanced} moves the top-K
 * resources by the previous batch's counts, longest first, each to the rank
 * with the least load so far (the other resources counted at their default
 * rank), and gives each moved resource a fresh engine id
 * {@code rPad + N * j + rank} past every default id.  Resources are
 * independent on the decision path (one ClusterNode each,
 * ClusterBuilderSlot.java:83-114), so the verdicts do not depend on the map.
 * Events and rules are renamed with {@link #engineId}; route an event to
 * {@link #owner}.
 */
public final class NodePlacement {
    private final int n;
    private final int[] engineId;
    private final int rows;

    private NodePlacement(int n, int[] engineId, int rows) {
        this.n = n;
        this.engineId = engineId;
        this.rows = rows;
    }

    /** Every resource at its default rank (id % n). */
    public static NodePlacement identity(int resources, int n) {
        int[] e = new int[resources];
        Arrays.setAll(e, i -> i);
        return new NodePlacement(n, e, (resources + n - 1) / n);
    }

    /** counts[r]: events of resource r in the previous batch. */
    public static NodePlacement balanced(long[] counts, int n, int k) {
        int r = counts.length;
        if (n <= 1) return identity(r, Math.max(n, 1));
        k = Math.min(k, r);
        Integer[] order = new Integer[r];
        Arrays.setAll(order, i -> i);
        Arrays.sort(order, (a, b) -> Long.compare(counts[b], counts[a]));       // stable: ties by id
        boolean[] top = new boolean[r];
        for (int i = 0; i < k; i++) top[order[i]] = true;
        long[] load = new long[n];
        for (int i = 0; i < r; i++) if (!top[i]) load[i % n] += counts[i];
        int rPad = ((r + n - 1) / n) * n;
        int[] slot = new int[n];
        int[] e = new int[r];
        Arrays.setAll(e, i -> i);
        for (int i = 0; i < k; i++) {
            int res = order[i], best = 0;
            for (int q = 1; q < n; q++) if (load[q] < load[best]) best = q;
            load[best] += counts[res];
            e[res] = rPad + n * slot[best] + best;
            slot[best]++;
        }
        int extra = 0;
        for (int q = 0; q < n; q++) extra = Math.max(extra, slot[q]);
        return new NodePlacement(n, e, rPad / n + extra);
    }

    /** The id the engines know the resource by (events, rules, names). */
    public int engineId(int resource) { return engineId[resource]; }

    /** The rank whose engine decides the resource. */
    public int owner(int resource) { return engineId[resource] % n; }

    /** max_resources of every rank's engine. */
    public int engineRows() { return rows; }
}
