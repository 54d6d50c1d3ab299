package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowArgument;

import java.lang.reflect.Array;
import java.util.Collection;
import java.util.LinkedHashMap;
import java.util.Map;
import java.util.concurrent.atomic.AtomicLong;

import static com.alibaba.csp.sentinel.gpu.SentinelFlowNative.*;

/**
 * Java parameter value -> (tag, 64-bit bits), the engine's value identity
 * (sentinel_flow.h SF_TAG_*).  Java equals() becomes bit equality: boxed
 * primitives by value, a String by sf_string_key (FNV-1a 64 of its UTF-8
 * bytes, the same key as the token-server wire path: no table that grows with
 * the traffic; two different strings collide with probability about 2^-64,
 * DESIGN.md §6b), any other object by an id from a bounded LRU table keyed by
 * the object (equals / hashCode), ids from one counter and never reused.  An
 * object evicted from that table gets a fresh id when it comes back, so its
 * hot-parameter counters restart, as the reference's LRU of
 * ParameterMetric.java:99-118 forgets an evicted value.  A ParamFlowArgument
 * is replaced by its paramFlowKey() first (ParamFlowChecker.java:64-68,
 * ParamFlowSlot.java:95-98).  A Collection or an array argument is packed
 * element by element (TAG_COLLECTION; ParamFlowChecker.passLocalCheck :84-112).
 */
final class ParamPacker {
    private static final int OTHERS_CAP = Integer.getInteger("sentinel.gpu.paramObjectIds", 1 << 20);
    private static final AtomicLong NEXT_ID = new AtomicLong();
    private static final Map<Object, Long> OTHERS = new LinkedHashMap<Object, Long>(1024, 0.75f, true) {
        @Override
        protected boolean removeEldestEntry(Map.Entry<Object, Long> eldest) {
            return size() > OTHERS_CAP;
        }
    };

    /** The value the checker keys on (ParamFlowChecker.java:64-68). */
    static Object key(Object v) {
        return v instanceof ParamFlowArgument ? ((ParamFlowArgument) v).paramFlowKey() : v;
    }

    static byte tag(Object v) {
        if (v == null) return TAG_NULL;
        if (v instanceof Integer) return TAG_INT;
        if (v instanceof Long) return TAG_LONG;
        if (v instanceof String) return TAG_STRING;
        if (v instanceof Double) return TAG_DOUBLE;
        if (v instanceof Boolean) return TAG_BOOL;
        if (v instanceof Byte) return TAG_BYTE;
        if (v instanceof Short) return TAG_SHORT;
        if (v instanceof Float) return TAG_FLOAT;
        if (v instanceof Collection || v.getClass().isArray()) return TAG_COLLECTION;
        return TAG_OTHER;
    }

    static long bits(Object v) {
        switch (tag(v)) {
            case TAG_NULL: return 0L;
            case TAG_INT: return (Integer) v;
            case TAG_LONG: return (Long) v;
            case TAG_STRING: return stringKey((String) v);
            case TAG_DOUBLE: return Double.doubleToLongBits((Double) v);
            case TAG_BOOL: return ((Boolean) v) ? 1L : 0L;
            case TAG_BYTE: return (Byte) v;
            case TAG_SHORT: return (Short) v;
            case TAG_FLOAT: return Float.floatToIntBits((Float) v);
            default:
                synchronized (OTHERS) {
                    return OTHERS.computeIfAbsent(v, k -> NEXT_ID.incrementAndGet());
                }
        }
    }

    /** Elements of a Collection or array argument, in iteration order. */
    static Object[] elements(Object v) {
        if (v instanceof Collection) return ((Collection<?>) v).toArray();
        int n = Array.getLength(v);
        Object[] out = new Object[n];
        for (int i = 0; i < n; i++) out[i] = Array.get(v, i);
        return out;
    }

    /** The String key of sf_string_key (FNV-1a 64 of the UTF-8 bytes): in-process and cluster token server. */
    static long stringKey(String s) {
        long h = 0xcbf29ce484222325L;
        for (byte b : s.getBytes(java.nio.charset.StandardCharsets.UTF_8)) {
            h ^= (b & 0xff);
            h *= 0x100000001b3L;
        }
        return h;
    }

    private ParamPacker() {}
}
