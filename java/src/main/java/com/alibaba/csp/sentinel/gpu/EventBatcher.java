package com.alibaba.csp.sentinel.gpu;

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
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

/**
 * Callers enqueue one {@link Ticket} per entry / exit; a single flusher thread
 * drains the queue into off-heap arrays, calls the engine once per batch
 * (events in enqueue order = the mocked clock order), writes each verdict
 * into its ticket and unparks the caller.  Timestamps are
 * TimeUtil.currentTimeMillis() taken at enqueue and made non-decreasing in
 * queue order, as the engine requires.  The arrays are page-locked host
 * memory from sf_host_alloc (the engine's H2D copy runs at PCIe speed, no
 * staging copy); a batch without ParamFlow arguments or context names, whose
 * clock spans less than 2^20 ms, goes as sf_packed_batch (8 bytes per event,
 * sf_submit_packed), every other one as the sf_event_batch SoA (sf_submit).
 */
final class EventBatcher implements Runnable {
    static final class Ticket {
        final Thread caller = Thread.currentThread();
        int resource, count;
        int origin = -1, context;        // interned Context origin (-1: "") and context name
        byte flags;
        long ts, entryRef = -1, createTs;
        Object[] args;
        Ticket entry;                    // EXIT: the ENTRY's ticket (its batch index, if in the same batch)
        long batchSeq = -1; int batchIndex = -1;
        volatile int status = -1;
        int waitMs, ruleIdx;
    }

    private final GpuEngine engine;
    private final BlockingQueue<Ticket> queue;
    private final int maxBatch;
    private final Arena arena = Arena.ofShared();
    private final MemorySegment res, ts, cnt, flags, eref, cts, nArgs, argTag, argBits, elemOff, elemTag, elemBits;
    private final MemorySegment origin, context;
    private final MemorySegment status, waitMs, ruleIdx, batch, verdicts;
    private final MemorySegment pev, pxref, pxcts, pcext, packed;   // sf_packed_batch arrays
    private long seq, lastTs = Long.MIN_VALUE, loadedRuleVersion = -1;
    static final int ARG_SLOTS = Integer.getInteger("sentinel.gpu.argSlots", 2);
    static final int MAX_ELEMS = Integer.getInteger("sentinel.gpu.maxElems", 1 << 20);

    EventBatcher(GpuEngine engine, int maxBatch) {
        this.engine = engine;
        this.maxBatch = maxBatch;
        this.queue = new ArrayBlockingQueue<>(maxBatch * 4);
        res = pinned(4L * maxBatch); ts = pinned(8L * maxBatch); cnt = pinned(4L * maxBatch);
        flags = pinned(maxBatch); eref = pinned(8L * maxBatch); cts = pinned(8L * maxBatch);
        nArgs = pinned(maxBatch); argTag = pinned((long) ARG_SLOTS * maxBatch);
        argBits = pinned(8L * ARG_SLOTS * maxBatch);
        elemOff = pinned(4L * ((long) ARG_SLOTS * maxBatch + 1));
        elemTag = pinned(MAX_ELEMS); elemBits = pinned(8L * MAX_ELEMS);
        origin = pinned(4L * maxBatch); context = pinned(4L * maxBatch);
        status = pinned(maxBatch); waitMs = pinned(4L * maxBatch); ruleIdx = pinned(2L * maxBatch);
        pev = pinned(8L * maxBatch); pxref = pinned(8L * maxBatch); pxcts = pinned(8L * maxBatch);
        pcext = pinned(4L * maxBatch);
        batch = arena.allocate(EVENT_BATCH); verdicts = arena.allocate(VERDICTS); packed = arena.allocate(PACKED_BATCH);
        Thread t = new Thread(this, "sentinel-gpu-flusher");
        t.setDaemon(true);
        t.start();
    }

    /** Page-locked host memory owned by the engine (released by sf_destroy). */
    private MemorySegment pinned(long bytes) {
        MemorySegment out = arena.allocate(ADDRESS);
        try {
            check((int) HOST_ALLOC.invokeExact(engine.handle, Math.max(bytes, 8L), out));
        } catch (Throwable t) {
            throw new IllegalStateException(t);
        }
        return out.get(ADDRESS, 0).reinterpret(Math.max(bytes, 8L));
    }

    /** Enqueue and wait for the verdict (the caller parks; the flusher unparks it). */
    Ticket submit(Ticket t) {
        try {
            queue.put(t);
        } catch (InterruptedException ex) {
            Thread.currentThread().interrupt();
            throw new IllegalStateException(ex);
        }
        while (t.status < 0) LockSupport.park(this);
        return t;
    }

    @Override
    public void run() {
        List<Ticket> drained = new ArrayList<>(maxBatch);
        while (true) {
            try {
                Ticket first = queue.poll(1, TimeUnit.SECONDS);
                if (first == null) continue;
                drained.clear();
                drained.add(first);
                queue.drainTo(drained, maxBatch - 1);
                flush(drained);
            } catch (Throwable t) {
                // an engine error fails the batch open (the reference never blocks on
                // an internal error, CtSph.java:155-158): every caller passes
                for (Ticket k : drained) { k.waitMs = 0; k.ruleIdx = 0; k.status = V_PASS; LockSupport.unpark(k.caller); }
            }
        }
    }

    private void flush(List<Ticket> b) throws Throwable {
        if (engine.ruleVersion.get() != loadedRuleVersion) {
            loadedRuleVersion = engine.ruleVersion.get();
            engine.loadRulesNow();
        }
        engine.pushSystemStatus();
        final long bs = ++seq;
        int n = b.size(), ne = 0;
        if (flushPacked(b, bs)) return;
        boolean anyExit = false;
        elemOff.set(JAVA_INT, 0, 0);
        for (int i = 0; i < n; i++) {
            Ticket t = b.get(i);
            t.batchSeq = bs; t.batchIndex = i;
            lastTs = Math.max(lastTs, t.ts);               // non-decreasing clock in submission order
            res.setAtIndex(JAVA_INT, i, t.resource);
            ts.setAtIndex(JAVA_LONG, i, lastTs);
            cnt.setAtIndex(JAVA_INT, i, t.count);
            flags.setAtIndex(JAVA_BYTE, i, t.flags);
            origin.setAtIndex(JAVA_INT, i, t.origin);
            context.setAtIndex(JAVA_INT, i, t.context);
            if ((t.flags & EV_EXIT) != 0) {
                anyExit = true;
                boolean same = t.entry != null && t.entry.batchSeq == bs;
                eref.setAtIndex(JAVA_LONG, i, same ? t.entry.batchIndex : -1L);
                cts.setAtIndex(JAVA_LONG, i, t.createTs);
            } else {
                eref.setAtIndex(JAVA_LONG, i, -1L);
                cts.setAtIndex(JAVA_LONG, i, 0L);
            }
            int na = t.args == null ? 0 : Math.min(t.args.length, ARG_SLOTS);
            nArgs.setAtIndex(JAVA_BYTE, i, (byte) na);
            for (int s = 0; s < ARG_SLOTS; s++) {
                long k = (long) s * n + i;
                Object v = s < na ? ParamPacker.key(t.args[s]) : null;
                byte tag = ParamPacker.tag(v);
                argTag.setAtIndex(JAVA_BYTE, k, tag);
                argBits.setAtIndex(JAVA_LONG, k, tag == TAG_COLLECTION ? 0L : ParamPacker.bits(v));
            }
        }
        // collection / array arguments: element CSR over (slot, event), slot-major
        for (int s = 0; s < ARG_SLOTS; s++) {
            for (int i = 0; i < n; i++) {
                long k = (long) s * n + i;
                Ticket t = b.get(i);
                Object v = t.args != null && s < t.args.length ? ParamPacker.key(t.args[s]) : null;
                if (v != null && ParamPacker.tag(v) == TAG_COLLECTION) {
                    for (Object el : ParamPacker.elements(v)) {
                        elemTag.setAtIndex(JAVA_BYTE, ne, ParamPacker.tag(el));
                        elemBits.setAtIndex(JAVA_LONG, ne, ParamPacker.bits(el));
                        ne++;
                    }
                }
                elemOff.setAtIndex(JAVA_INT, k + 1, ne);
            }
        }
        batch.set(JAVA_INT, off(EVENT_BATCH, "n"), n);
        batch.set(JAVA_INT, off(EVENT_BATCH, "mem"), SF_MEM_HOST_);
        batch.set(ADDRESS, off(EVENT_BATCH, "res_id"), res);
        batch.set(ADDRESS, off(EVENT_BATCH, "ts_ms"), ts);
        batch.set(ADDRESS, off(EVENT_BATCH, "count"), cnt);
        batch.set(ADDRESS, off(EVENT_BATCH, "flags"), flags);
        batch.set(ADDRESS, off(EVENT_BATCH, "entry_ref"), anyExit ? eref : MemorySegment.NULL);
        batch.set(ADDRESS, off(EVENT_BATCH, "create_ts"), anyExit ? cts : MemorySegment.NULL);
        batch.set(JAVA_INT, off(EVENT_BATCH, "arg_slots"), ARG_SLOTS);
        batch.set(ADDRESS, off(EVENT_BATCH, "n_args"), nArgs);
        batch.set(ADDRESS, off(EVENT_BATCH, "arg_tag"), argTag);
        batch.set(ADDRESS, off(EVENT_BATCH, "arg_bits"), argBits);
        batch.set(ADDRESS, off(EVENT_BATCH, "arg_elem_off"), ne > 0 ? elemOff : MemorySegment.NULL);
        batch.set(ADDRESS, off(EVENT_BATCH, "elem_tag"), elemTag);
        batch.set(ADDRESS, off(EVENT_BATCH, "elem_bits"), elemBits);
        batch.set(JAVA_INT, off(EVENT_BATCH, "n_elems"), ne);
        batch.set(ADDRESS, off(EVENT_BATCH, "origin"), origin);
        batch.set(ADDRESS, off(EVENT_BATCH, "context"), context);
        verdicts.set(JAVA_INT, off(VERDICTS, "mem"), SF_MEM_HOST_);
        verdicts.set(ADDRESS, off(VERDICTS, "status"), status);
        verdicts.set(ADDRESS, off(VERDICTS, "wait_ms"), waitMs);
        verdicts.set(ADDRESS, off(VERDICTS, "rule_idx"), ruleIdx);
        check((int) SUBMIT.invokeExact(engine.handle, batch, verdicts));
        for (int i = 0; i < n; i++) {
            Ticket t = b.get(i);
            t.waitMs = waitMs.getAtIndex(JAVA_INT, i);
            t.ruleIdx = Short.toUnsignedInt(ruleIdx.getAtIndex(JAVA_SHORT, i));
            t.status = status.getAtIndex(JAVA_BYTE, i);
            LockSupport.unpark(t.caller);
        }
    }

    /**
     * The batch as sf_packed_batch when it fits (no arguments, no context
     * names, clock span < 2^20 ms); false: the caller builds the SoA batch.
     */
    private boolean flushPacked(List<Ticket> b, long bs) throws Throwable {
        final int n = b.size();
        long t0 = Long.MIN_VALUE, last = lastTs;
        for (Ticket t : b) {
            if ((t.args != null && t.args.length > 0) || t.context != 0) return false;
            last = Math.max(last, t.ts);
            if (t0 == Long.MIN_VALUE) t0 = last;
        }
        if (last - t0 >= (1L << 20)) return false;
        int nx = 0, nc = 0;
        for (int i = 0; i < n; i++) {
            Ticket t = b.get(i);
            t.batchSeq = bs; t.batchIndex = i;
            lastTs = Math.max(lastTs, t.ts);
            long c = t.count;
            if (c < 1 || c > 127) { pcext.setAtIndex(JAVA_INT, nc++, t.count); c = 0; }
            long f = t.flags & 0x1f;
            pev.setAtIndex(JAVA_LONG, i, (t.resource & 0xffffffffL) | ((lastTs - t0) << 32)
                    | (c << PK_COUNT_SHIFT) | (f << PK_FLAGS_SHIFT));
            origin.setAtIndex(JAVA_INT, i, t.origin);
            if ((t.flags & EV_EXIT) != 0) {
                boolean same = t.entry != null && t.entry.batchSeq == bs;
                pxref.setAtIndex(JAVA_LONG, nx, same ? t.entry.batchIndex : -1L);
                pxcts.setAtIndex(JAVA_LONG, nx, t.createTs);
                nx++;
            }
        }
        packed.set(JAVA_INT, off(PACKED_BATCH, "n"), n);
        packed.set(JAVA_INT, off(PACKED_BATCH, "mem"), SF_MEM_HOST_);
        packed.set(JAVA_LONG, off(PACKED_BATCH, "ts_base"), t0);
        packed.set(ADDRESS, off(PACKED_BATCH, "ev"), pev);
        packed.set(ADDRESS, off(PACKED_BATCH, "exit_ref"), nx > 0 ? pxref : MemorySegment.NULL);
        packed.set(ADDRESS, off(PACKED_BATCH, "exit_cts"), nx > 0 ? pxcts : MemorySegment.NULL);
        packed.set(ADDRESS, off(PACKED_BATCH, "count_ext"), nc > 0 ? pcext : MemorySegment.NULL);
        packed.set(ADDRESS, off(PACKED_BATCH, "origin"), origin);
        packed.set(JAVA_INT, off(PACKED_BATCH, "n_exit"), nx);
        packed.set(JAVA_INT, off(PACKED_BATCH, "n_count_ext"), nc);
        verdicts.set(JAVA_INT, off(VERDICTS, "mem"), SF_MEM_HOST_);
        verdicts.set(ADDRESS, off(VERDICTS, "status"), status);
        verdicts.set(ADDRESS, off(VERDICTS, "wait_ms"), waitMs);
        verdicts.set(ADDRESS, off(VERDICTS, "rule_idx"), ruleIdx);
        check((int) SUBMIT_PACKED.invokeExact(engine.handle, packed, verdicts));
        for (int i = 0; i < n; i++) {
            Ticket t = b.get(i);
            t.waitMs = waitMs.getAtIndex(JAVA_INT, i);
            t.ruleIdx = Short.toUnsignedInt(ruleIdx.getAtIndex(JAVA_SHORT, i));
            t.status = status.getAtIndex(JAVA_BYTE, i);
            LockSupport.unpark(t.caller);
        }
        return true;
    }

    private static final int SF_MEM_HOST_ = 0;
}
