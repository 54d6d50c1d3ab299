package com.alibaba.csp.sentinel.gpu;

import java.lang.reflect.Array;
import java.util.Collection;
import java.util.concurrent.ConcurrentHashMap;

import static com.alibaba.csp.sentinel.gpu.SentinelFlowNative.*;

/**
 * Java parameter value -> (tag, 64-bit bits), the engine's value identity
 * (sentinel_flow.h SF_TAG_*).  Java equals() becomes bit equality: boxed
 * primitives by value, Strings interned to a dense id (ParamFlowChecker's
 * HashMap lookups, ParamFlowChecker.java:126-155), any other object by its
 * identity-stable id.  A Collection or an array argument is packed element by
 * element (TAG_COLLECTION; ParamFlowChecker.passLocalCheck :84-112).
 */
final class ParamPacker {
    private static final ConcurrentHashMap<String, Long> STRINGS = new ConcurrentHashMap<>();
    private static final ConcurrentHashMap<Object, Long> OTHERS = new ConcurrentHashMap<>();

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
            case TAG_STRING: return STRINGS.computeIfAbsent((String) v, k -> (long) STRINGS.size() + 1);
            case TAG_DOUBLE: return Double.doubleToLongBits((Double) v);
            case TAG_BOOL: return ((Boolean) v) ? 1L : 0L;
            case TAG_BYTE: return (Byte) v;
            case TAG_SHORT: return (Short) v;
            case TAG_FLOAT: return Float.floatToIntBits((Float) v);
            default: return OTHERS.computeIfAbsent(v, k -> (long) OTHERS.size() + 1);
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

    /** Cluster token server: the String key of sf_string_key (FNV-1a 64 of the UTF-8 bytes). */
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
