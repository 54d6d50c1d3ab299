package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowItem;

/**
 * ParamFlowItem -> typed value, as ParamFlowRuleUtil.parseHotItems /
 * parseItemValue (ParamFlowRuleUtil.java:188-240): a blank class type and an
 * unknown one keep the String; a parse failure, a null value or a null or
 * negative count drops the item (null here).
 */
final class HotItems {
    static Object parse(ParamFlowItem item) {
        String v = item.getObject(), type = item.getClassType();
        if (v == null || item.getCount() == null || item.getCount() < 0) return null;
        try {
            if (type == null || type.trim().isEmpty()) return v;
            switch (type) {
                case "int": case "java.lang.Integer": return Integer.parseInt(v);
                case "boolean": case "java.lang.Boolean": return Boolean.parseBoolean(v);
                case "long": case "java.lang.Long": return Long.parseLong(v);
                case "double": case "java.lang.Double": return Double.parseDouble(v);
                case "float": case "java.lang.Float": return Float.parseFloat(v);
                case "byte": case "java.lang.Byte": return Byte.parseByte(v);
                case "short": case "java.lang.Short": return Short.parseShort(v);
                case "char": return v.isEmpty() ? null : v.charAt(0);
                default: return v;
            }
        } catch (RuntimeException ex) {
            return null;
        }
    }

    private HotItems() {}
}
