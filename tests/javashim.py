"""Static reader of the Java SPI shim (java/, no JDK here): the Panama FFM
struct layouts of SentinelFlowNative.java with their field offsets (explicit
padding, as FFM requires), the constants, the downcall symbol names, and the
field-name offsets the other sources write through."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JDIR = os.path.join(ROOT, "java", "src", "main", "java", "com", "alibaba", "csp", "sentinel", "gpu")
SIZES = {"JAVA_INT": 4, "JAVA_LONG": 8, "JAVA_DOUBLE": 8, "ADDRESS": 8, "JAVA_BYTE": 1, "JAVA_SHORT": 2}
C_STRUCT = {"CONFIG": "sf_config", "FLOW_RULE": "sf_flow_rule", "HOT_ITEM": "sf_hot_item",
            "PARAM_RULE": "sf_param_rule", "SYSTEM_RULE": "sf_system_rule", "DEGRADE_RULE": "sf_degrade_rule",
            "EVENT_BATCH": "sf_event_batch", "VERDICTS": "sf_verdicts", "TOKEN_BATCH": "sf_token_batch",
            "TOKEN_RESULTS": "sf_token_results", "PACKED_BATCH": "sf_packed_batch",
            "SPARSE_VERDICTS": "sf_sparse_verdicts"}


def source(name):
    return open(os.path.join(JDIR, name)).read()


def layouts():
    """{LAYOUT: (size, [(field, offset, size)])} from SentinelFlowNative.java."""
    src = source("SentinelFlowNative.java")
    out = {}
    for m in re.finditer(r"static final StructLayout (\w+) = MemoryLayout\.structLayout\((.*?)\);", src, re.S):
        name, body = m.group(1), m.group(2)
        off, fields = 0, []
        for item in re.finditer(r"(?:java\.lang\.foreign\.ValueLayout\.)?(\w+)\.withName\(\"(\w+)\"\)|"
                                r"MemoryLayout\.paddingLayout\((\d+)\)", body):
            if item.group(3):
                off += int(item.group(3))
                continue
            t, f = item.group(1), item.group(2)
            sz = SIZES[t]
            assert off % sz == 0, f"{name}.{f}: FFM refuses a misaligned field (offset {off})"
            fields.append((f, off, sz))
            off += sz
        out[name] = (off, fields)
    return out


def constants():
    src = source("SentinelFlowNative.java")
    out = {}
    for decl in re.findall(r"static final (?:byte|int) ([^;]+);", src):
        for k, v in re.findall(r"(\w+)\s*=\s*(0x[0-9a-fA-F]+|-?\d+)", decl):
            out[k] = int(v, 0)
    return out


def downcalls():
    return re.findall(r"fn\(\"(sf_\w+)\"", source("SentinelFlowNative.java"))


def field_refs():
    """(file, LAYOUT, field, JAVA_TYPE) of every write through off(LAYOUT, "field")."""
    refs = []
    for fn in sorted(os.listdir(JDIR)):
        if not fn.endswith(".java"):
            continue
        for t, lay, f in re.findall(r"\.set\((\w+),\s*off\((\w+),\s*\"(\w+)\"\)", source(fn)):
            refs.append((fn, lay, f, t))
    return refs


def numeric_struct_writes():
    """Writes into a struct at a literal offset (none should remain)."""
    bad = []
    for fn in sorted(os.listdir(JDIR)):
        if fn.endswith(".java"):
            bad += [(fn, m) for m in re.findall(r"\b(?:s|h|batch|verdicts|results|cfg)\.set\(\w+,\s*\d+,", source(fn))]
    return bad
