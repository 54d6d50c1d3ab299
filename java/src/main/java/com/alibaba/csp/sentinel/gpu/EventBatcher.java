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
 * clock spans less than 2^20 ms, goes as sf_packed_batch -- in the narrow form
 * (4 bytes per event plus a table of the batch's milliseconds) when every
 * resource id is below 2^24, else 8 bytes per event --, every other one as
 * the sf_event_batch SoA (sf_submit).
 *
 * Latency / throughput contract.  Packed batches are double-buffered: the
 * flusher enqueues batch k+1 with sf_submit_packed_sparse_async into the
 * buffer set batch k is not using, then waits for batch k alone
 * (sf_sync_packed_sparse) and hands out its verdicts (copied back as a status
 * byte per event plus the nonzero waits / rule indices), so the H2D copy of k+1 overlaps the decision of k
 * and the copy back of k-1.  A caller still waits only for its own batch: its
 * verdict is delivered as soon as its batch is back, and a batch is never held
 * for a later one -- when the queue is empty the flusher collects the batch in
 * flight at once.  An EXIT can never refer to an entry of the batch in flight
 * (its caller had that entry's verdict first), so exits need no ordering work.
 * A SoA batch, a rule reload, and an engine with SystemRules (whose packed
 * batches the engine decides synchronously) collect the batch in flight first.
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

    /** One buffer set of the packed path: the batch arrays, its verdicts and its tickets. */
    private final class PackedBuf {
        final MemorySegment pev = pinned(8L * maxBatch), pxref = pinned(8L * maxBatch), pxcts = pinned(8L * maxBatch);
        // the narrow form: 4-byte words and ms_end, the events up to each millisecond of the batch
        final MemorySegment pev4 = pinned(4L * maxBatch), pms = pinned(4L * PK4_MAX_MS);
        final MemorySegment pcext = pinned(4L * maxBatch), porigin = pinned(4L * maxBatch);
        // verdicts copied back sparse: a status byte per event, the nonzero waits / rule
        // indices as (index << 32 | value) lists, maxBatch / 64 of each with the batch
        final MemorySegment pstatus = pinned(maxBatch), pwaits = pinned(8L * maxBatch), prules = pinned(8L * maxBatch);
        final MemorySegment pcounts = pinned(8);
        final MemorySegment packed = arena.allocate(PACKED_BATCH), pverdicts = arena.allocate(SPARSE_VERDICTS);
        final List<Ticket> tickets = new ArrayList<>();
    }
    private final PackedBuf[] pbufs;
    private int pcur;
    private PackedBuf inFlight;                  // enqueued, verdicts not yet handed out
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
        batch = arena.allocate(EVENT_BATCH); verdicts = arena.allocate(VERDICTS);
        pbufs = new PackedBuf[] {new PackedBuf(), new PackedBuf()};
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
                // with a batch in flight, an empty queue collects it at once (no caller waits on a later batch)
                Ticket first = inFlight != null ? queue.poll() : queue.poll(1, TimeUnit.SECONDS);
                if (first == null) {
                    collect();
                    continue;
                }
                drained = new ArrayList<>(maxBatch);
                drained.add(first);
                queue.drainTo(drained, maxBatch - 1);
                flush(drained);
            } catch (Throwable t) {
                failOpen(drained);
            }
        }
    }

    /** An engine error fails the batch open (the reference never blocks on an internal error, CtSph.java:155-158). */
    private static void failOpen(List<Ticket> b) {
        for (Ticket k : b) {
            if (k.status >= 0) continue;
            k.waitMs = 0; k.ruleIdx = 0; k.status = V_PASS; LockSupport.unpark(k.caller);
        }
    }

    /** Waits for the batch in flight alone (sf_sync_packed) and hands out its verdicts. */
    private void collect() {
        PackedBuf f = inFlight;
        if (f == null) return;
        inFlight = null;
        try {
            check((int) SYNC_PACKED_SPARSE.invokeExact(engine.handle, f.pverdicts));
            deliverSparse(f.tickets, f.pstatus, f.pwaits, f.prules, f.pcounts);
        } catch (Throwable t) {
            failOpen(f.tickets);
        }
    }

    private static void deliver(List<Ticket> b, MemorySegment st, MemorySegment wt, MemorySegment ru) {
        for (int i = 0; i < b.size(); i++) {
            Ticket t = b.get(i);
            t.waitMs = wt.getAtIndex(JAVA_INT, i);
            t.ruleIdx = Short.toUnsignedInt(ru.getAtIndex(JAVA_SHORT, i));
            t.status = st.getAtIndex(JAVA_BYTE, i);
            LockSupport.unpark(t.caller);
        }
    }

    /** Statuses, then the listed waits / rule indices (every other one is 0). */
    private static void deliverSparse(List<Ticket> b, MemorySegment st, MemorySegment waits, MemorySegment rules,
                                      MemorySegment counts) {
        for (Ticket t : b) { t.waitMs = 0; t.ruleIdx = 0; }
        final int nw = counts.getAtIndex(JAVA_INT, 0), nr = counts.getAtIndex(JAVA_INT, 1);
        for (int k = 0; k < nw; k++) {
            long x = waits.getAtIndex(JAVA_LONG, k);
            b.get((int) (x >>> 32)).waitMs = (int) x;
        }
        for (int k = 0; k < nr; k++) {
            long x = rules.getAtIndex(JAVA_LONG, k);
            b.get((int) (x >>> 32)).ruleIdx = (int) (x & 0xffff);
        }
        for (int i = 0; i < b.size(); i++) {
            Ticket t = b.get(i);
            t.status = st.getAtIndex(JAVA_BYTE, i);
            LockSupport.unpark(t.caller);
        }
    }

    private void flush(List<Ticket> b) throws Throwable {
        engine.followRuleProperties();                       // a data source's property swapped in since
        if (engine.ruleVersion.get() != loadedRuleVersion) {
            collect();                                       // decided under the rules it was sorted with
            loadedRuleVersion = engine.ruleVersion.get();
            engine.loadRulesNow();
        }
        engine.pushSystemStatus();
        final long bs = ++seq;
        int n = b.size(), ne = 0;
        if (flushPacked(b, bs)) return;
        collect();                                           // the SoA path is synchronous
        boolean anyExit = false, anyOrigin = false;
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
            anyOrigin |= t.origin != -1;
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
        batch.set(ADDRESS, off(EVENT_BATCH, "origin"), anyOrigin ? origin : MemorySegment.NULL);
        batch.set(ADDRESS, off(EVENT_BATCH, "context"), context);
        verdicts.set(JAVA_INT, off(VERDICTS, "mem"), SF_MEM_HOST_);
        verdicts.set(ADDRESS, off(VERDICTS, "status"), status);
        verdicts.set(ADDRESS, off(VERDICTS, "wait_ms"), waitMs);
        verdicts.set(ADDRESS, off(VERDICTS, "rule_idx"), ruleIdx);
        check((int) SUBMIT.invokeExact(engine.handle, batch, verdicts));
        deliver(b, status, waitMs, ruleIdx);
    }

    /**
     * The batch as sf_packed_batch when it fits (no arguments, no context
     * names, clock span < 2^20 ms): enqueued into the free buffer set, then the
     * batch before it collected; false: the caller builds the SoA batch.
     */
    private boolean flushPacked(List<Ticket> b, long bs) throws Throwable {
        final int n = b.size();
        long t0 = Long.MIN_VALUE, last = lastTs;
        boolean narrow = true;
        for (Ticket t : b) {
            if ((t.args != null && t.args.length > 0) || t.context != 0) return false;
            last = Math.max(last, t.ts);
            if (t0 == Long.MIN_VALUE) t0 = last;
            narrow &= (t.resource & 0xffffffffL) < (1L << 24);
        }
        if (last - t0 >= (1L << 20)) return false;
        final PackedBuf p = pbufs[pcur];             // not the in-flight set: sets alternate
        int nx = 0, nc = 0, ms = 0;
        boolean anyOrigin = false;
        for (int i = 0; i < n; i++) {
            Ticket t = b.get(i);
            t.batchSeq = bs; t.batchIndex = i;
            lastTs = Math.max(lastTs, t.ts);
            final int d = (int) (lastTs - t0);
            long c = t.count;
            long f = t.flags & 0x1f;
            if (narrow) {
                if (c < 1 || c > 7) { p.pcext.setAtIndex(JAVA_INT, nc++, t.count); c = 0; }
                // ms_end[m] = events with delta <= m: the milliseconds before this event's end at i
                for (; ms < d; ms++) p.pms.setAtIndex(JAVA_INT, ms, i);
                p.pev4.setAtIndex(JAVA_INT, i, (int) ((t.resource & 0xffffffL) | (c << PK4_COUNT_SHIFT)
                        | (f << PK4_FLAGS_SHIFT)));
            } else {
                if (c < 1 || c > 127) { p.pcext.setAtIndex(JAVA_INT, nc++, t.count); c = 0; }
                p.pev.setAtIndex(JAVA_LONG, i, (t.resource & 0xffffffffL) | ((long) d << 32)
                        | (c << PK_COUNT_SHIFT) | (f << PK_FLAGS_SHIFT));
            }
            p.porigin.setAtIndex(JAVA_INT, i, t.origin);
            anyOrigin |= t.origin != -1;
            if ((t.flags & EV_EXIT) != 0) {
                boolean same = t.entry != null && t.entry.batchSeq == bs;
                p.pxref.setAtIndex(JAVA_LONG, nx, same ? t.entry.batchIndex : -1L);
                p.pxcts.setAtIndex(JAVA_LONG, nx, t.createTs);
                nx++;
            }
        }
        MemorySegment pk = p.packed;
        pk.set(JAVA_INT, off(PACKED_BATCH, "n"), n);
        pk.set(JAVA_INT, off(PACKED_BATCH, "mem"), SF_MEM_HOST_);
        pk.set(JAVA_LONG, off(PACKED_BATCH, "ts_base"), t0);
        if (narrow) p.pms.setAtIndex(JAVA_INT, ms, n);             // the last millisecond ends the batch
        pk.set(ADDRESS, off(PACKED_BATCH, "ev"), narrow ? MemorySegment.NULL : p.pev);
        pk.set(ADDRESS, off(PACKED_BATCH, "ev4"), narrow ? p.pev4 : MemorySegment.NULL);
        pk.set(ADDRESS, off(PACKED_BATCH, "ms_end"), narrow ? p.pms : MemorySegment.NULL);
        pk.set(JAVA_INT, off(PACKED_BATCH, "n_ms"), narrow ? ms + 1 : 0);
        pk.set(ADDRESS, off(PACKED_BATCH, "exit_ref"), nx > 0 ? p.pxref : MemorySegment.NULL);
        pk.set(ADDRESS, off(PACKED_BATCH, "exit_cts"), nx > 0 ? p.pxcts : MemorySegment.NULL);
        pk.set(ADDRESS, off(PACKED_BATCH, "count_ext"), nc > 0 ? p.pcext : MemorySegment.NULL);
        // no origin at all: NULL, so the engine runs no origin-node pass for the batch
        pk.set(ADDRESS, off(PACKED_BATCH, "origin"), anyOrigin ? p.porigin : MemorySegment.NULL);
        pk.set(JAVA_INT, off(PACKED_BATCH, "n_exit"), nx);
        pk.set(JAVA_INT, off(PACKED_BATCH, "n_count_ext"), nc);
        MemorySegment v = p.pverdicts;
        v.set(ADDRESS, off(SPARSE_VERDICTS, "status"), p.pstatus);
        v.set(ADDRESS, off(SPARSE_VERDICTS, "waits"), p.pwaits);
        v.set(ADDRESS, off(SPARSE_VERDICTS, "rules"), p.prules);
        v.set(ADDRESS, off(SPARSE_VERDICTS, "counts"), p.pcounts);
        v.set(JAVA_INT, off(SPARSE_VERDICTS, "prefetch"), Math.max(64, maxBatch / 64));
        p.tickets.clear();
        p.tickets.addAll(b);
        try {
            check((int) SUBMIT_PACKED_SPARSE_ASYNC.invokeExact(engine.handle, pk, v));
        } catch (Throwable t) {
            collect();
            throw t;
        }
        collect();                                   // batch k-1 back while batch k runs
        inFlight = p;
        pcur ^= 1;
        return true;
    }

    private static final int SF_MEM_HOST_ = 0;
}
