package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.cluster.TokenResult;
import com.alibaba.csp.sentinel.util.TimeUtil;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.List;
import java.util.concurrent.ArrayBlockingQueue;
import java.util.concurrent.BlockingQueue;
import java.util.concurrent.TimeUnit;
import java.util.concurrent.locks.LockSupport;

import static com.alibaba.csp.sentinel.gpu.SentinelFlowNative.*;
import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * Token requests of all server threads, decided in arrival order one batch
 * per sf_request_tokens call (sf_token_batch: flowId, acquireCount, flags,
 * server clock, and for requestParamToken the values' CSR).  The server's
 * rules and namespaces are loaded by the embedding server through
 * sf_load_cluster_rules / sf_load_namespaces when ClusterFlowRuleManager /
 * ClusterParamFlowRuleManager change.
 */
final class TokenBatcher implements Runnable {
    private static volatile TokenBatcher INSTANCE;

    static TokenBatcher get() {
        if (INSTANCE == null) {
            synchronized (TokenBatcher.class) {
                if (INSTANCE == null) INSTANCE = new TokenBatcher(GpuEngine.get(), 1 << 16, 1 << 18);
            }
        }
        return INSTANCE;
    }

    private static final class Req {
        final Thread caller = Thread.currentThread();
        long flowId; int count; boolean prio; Object[] params; long ts;
        volatile boolean done; int status, remaining, waitMs;
    }

    private final GpuEngine engine;
    private final BlockingQueue<Req> queue;
    private final int maxBatch, maxValues;
    private final Arena arena = Arena.ofShared();
    private final MemorySegment flow, cnt, flags, ts, ptag, pbits, poff, status, remaining, waitMs, batch, results;
    private long lastTs = Long.MIN_VALUE;

    private TokenBatcher(GpuEngine engine, int maxBatch, int maxValues) {
        this.engine = engine; this.maxBatch = maxBatch; this.maxValues = maxValues;
        queue = new ArrayBlockingQueue<>(4 * maxBatch);
        flow = arena.allocate(8L * maxBatch); cnt = arena.allocate(4L * maxBatch); flags = arena.allocate(maxBatch);
        ts = arena.allocate(8L * maxBatch); ptag = arena.allocate(maxValues); pbits = arena.allocate(8L * maxValues);
        poff = arena.allocate(4L * (maxBatch + 1));
        status = arena.allocate(maxBatch); remaining = arena.allocate(4L * maxBatch); waitMs = arena.allocate(4L * maxBatch);
        batch = arena.allocate(TOKEN_BATCH); results = arena.allocate(TOKEN_RESULTS);
        Thread t = new Thread(this, "sentinel-gpu-token-flusher");
        t.setDaemon(true);
        t.start();
    }

    TokenResult request(long flowId, int count, boolean prio, Object[] params) {
        Req r = new Req();
        r.flowId = flowId; r.count = count; r.prio = prio; r.params = params; r.ts = TimeUtil.currentTimeMillis();
        try {
            queue.put(r);
        } catch (InterruptedException ex) {
            Thread.currentThread().interrupt();
            return new TokenResult(com.alibaba.csp.sentinel.cluster.TokenResultStatus.FAIL);
        }
        while (!r.done) LockSupport.park(this);
        return new TokenResult(r.status).setRemaining(r.remaining).setWaitInMs(r.waitMs);
    }

    @Override
    public void run() {
        List<Req> b = new ArrayList<>(maxBatch);
        while (true) {
            try {
                Req first = queue.poll(1, TimeUnit.SECONDS);
                if (first == null) continue;
                b.clear();
                b.add(first);
                queue.drainTo(b, maxBatch - 1);
                flush(b);
            } catch (Throwable t) {
                for (Req r : b) { r.status = -1; r.done = true; LockSupport.unpark(r.caller); }   // FAIL
            }
        }
    }

    private void flush(List<Req> b) throws Throwable {
        int n = b.size(), nv = 0;
        boolean anyParam = false;
        poff.set(JAVA_INT, 0, 0);
        for (int i = 0; i < n; i++) {
            Req r = b.get(i);
            lastTs = Math.max(lastTs, r.ts);
            flow.setAtIndex(JAVA_LONG, i, r.flowId);
            cnt.setAtIndex(JAVA_INT, i, r.count);
            flags.setAtIndex(JAVA_BYTE, i, (byte) ((r.prio ? TOK_PRIORITIZED : 0) | (r.params != null ? TOK_PARAM : 0)));
            ts.setAtIndex(JAVA_LONG, i, lastTs);
            if (r.params != null) {
                anyParam = true;
                for (Object v : r.params) {
                    if (nv == maxValues) throw new IllegalStateException("too many parameter values in one batch");
                    ptag.setAtIndex(JAVA_BYTE, nv, ParamPacker.tag(v));
                    pbits.setAtIndex(JAVA_LONG, nv, ParamPacker.bits(v));      // a String: sf_string_key
                    nv++;
                }
            }
            poff.setAtIndex(JAVA_INT, i + 1, nv);
        }
        batch.set(JAVA_INT, off(TOKEN_BATCH, "n"), n);
        batch.set(JAVA_INT, off(TOKEN_BATCH, "mem"), 0);
        batch.set(ADDRESS, off(TOKEN_BATCH, "flow_id"), flow);
        batch.set(ADDRESS, off(TOKEN_BATCH, "count"), cnt);
        batch.set(ADDRESS, off(TOKEN_BATCH, "flags"), flags);
        batch.set(ADDRESS, off(TOKEN_BATCH, "ts_ms"), ts);
        batch.set(ADDRESS, off(TOKEN_BATCH, "param_tag"), anyParam ? ptag : MemorySegment.NULL);
        batch.set(ADDRESS, off(TOKEN_BATCH, "param_bits"), anyParam ? pbits : MemorySegment.NULL);
        batch.set(ADDRESS, off(TOKEN_BATCH, "param_off"), anyParam ? poff : MemorySegment.NULL);
        results.set(JAVA_INT, off(TOKEN_RESULTS, "mem"), 0);
        results.set(ADDRESS, off(TOKEN_RESULTS, "status"), status);
        results.set(ADDRESS, off(TOKEN_RESULTS, "remaining"), remaining);
        results.set(ADDRESS, off(TOKEN_RESULTS, "wait_ms"), waitMs);
        check((int) REQUEST_TOKENS.invokeExact(engine.handle, batch, results));
        for (int i = 0; i < n; i++) {
            Req r = b.get(i);
            r.status = status.getAtIndex(JAVA_BYTE, i);
            r.remaining = remaining.getAtIndex(JAVA_INT, i);
            r.waitMs = waitMs.getAtIndex(JAVA_INT, i);
            r.done = true;
            LockSupport.unpark(r.caller);
        }
    }
}
