"""The Java SPI shim (java/) against the C ABI, statically: there is no JDK in
this image, so the sources are read, not compiled.  Every Panama FFM struct
layout equals the C struct (field offsets by gcc's offsetof, total size by
sizeof: arrays of structs are strided by the layout size), every write goes
through a named field of the right width, every flag / verdict / tag constant
equals the header's, every downcall names an exported function, the chain
matches the reference's StatisticSlot accounting (StatisticSlot.java:55-131:
no reference DegradeSlot after the GPU slot, AuthoritySlot run inside it,
PriorityWait without fireEntry), and INTEGRATION.md quotes the sources
verbatim."""
import os
import re
import subprocess

import pytest

from tests import javashim as j
from tests.test_abi import HEADER, declared_functions

ROOT = j.ROOT


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    """{struct: (sizeof, {field: (offsetof, sizeof)})} for the structs the shim mirrors."""
    lay = j.layouts()
    lines = []
    for jl, cs in j.C_STRUCT.items():
        lines.append('printf("%s - %%zu 0\\n", sizeof(%s));' % (cs, cs))
        for f, _, _ in lay[jl][1]:
            lines.append('printf("%s %s %%zu %%zu\\n", offsetof(%s, %s), sizeof(((%s*)0)->%s));'
                         % (cs, f, cs, f, cs, f))
    d = tmp_path_factory.mktemp("jshim")
    prog = d / "off.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\nint main(void){\n%s\nreturn 0;}\n'
                    % (HEADER, "\n".join(lines)))
    exe = d / "off"
    subprocess.check_call(["gcc", "-o", str(exe), str(prog)])
    out = {}
    for l in subprocess.check_output([str(exe)]).decode().split("\n"):
        if not l.strip():
            continue
        s, f, a, b = l.split()
        ent = out.setdefault(s, [0, {}])
        if f == "-":
            ent[0] = int(a)
        else:
            ent[1][f] = (int(a), int(b))
    return out


def test_every_layout_matches_the_c_struct(c_layout):
    for jl, (size, fields) in j.layouts().items():
        cs = j.C_STRUCT[jl]
        csize, cf = c_layout[cs]
        assert size == csize, f"{jl}: FFM layout {size} B, sizeof({cs}) {csize} B"
        for f, off, sz in fields:
            assert cf[f] == (off, sz), f"{jl}.{f}: Java ({off}, {sz}) vs C {cf[f]}"


def test_layouts_cover_the_whole_struct(c_layout):
    """No C field is missing from a layout (its bytes would be left as padding)."""
    src = open(HEADER).read()
    for jl, cs in j.C_STRUCT.items():
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cs, cs), src, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        names = re.findall(r"(\w+)(?:\[\w+\])?\s*;", body)
        have = {f for f, _, _ in j.layouts()[jl][1]}
        missing = [n for n in names if n not in have and not n.startswith("pad")]
        assert not missing, f"{jl}: {missing}"


def test_writes_use_named_fields_of_the_right_width(c_layout):
    lay = j.layouts()
    refs = j.field_refs()
    assert len(refs) > 60
    for fn, l, f, t in refs:
        fields = {a: c for a, b, c in lay[l][1]}
        assert f in fields, f"{fn}: {l} has no field {f}"
        assert j.SIZES[t] == fields[f], f"{fn}: {l}.{f} written as {t}"
    assert j.numeric_struct_writes() == []


def test_constants_equal_the_header():
    src = open(HEADER).read()
    hdr = {k: int(v.rstrip("u"), 0) for k, v in re.findall(r"#define (SF_\w+)\s+(-?0x[0-9a-fA-F]+u?|-?\d+)", src)}
    for k, v in j.constants().items():
        assert hdr["SF_" + k] == v, f"{k}: Java {v} vs header {hdr['SF_' + k]}"
    assert {"EV_BLOCKED", "V_BLOCK_DEGRADE", "V_BLOCK_OTHER"} <= set(j.constants())


def test_downcalls_name_declared_functions():
    fns = set(declared_functions())
    for f in j.downcalls():
        assert f in fns, f


def test_chain_is_statistic_slot_accounting():
    """StatisticSlot wraps AuthoritySlot .. DegradeSlot (Constants.java:77-84):
    all of them are inside GpuFlowSlot / the engine."""
    builder = j.source("GpuSlotChainBuilder.java")
    chain = re.findall(r"chain\.addLast\(new (\w+)\(", builder)
    assert chain == ["NodeSelectorSlot", "ClusterBuilderSlot", "LogSlot", "GpuFlowSlot"]
    for fn in os.listdir(j.JDIR):
        assert "new DegradeSlot(" not in j.source(fn), fn
    slot = j.source("GpuFlowSlot.java")
    assert "authority.entry(" in slot and "EV_BLOCKED" in slot and "catch (AuthorityException" in slot
    assert "case V_BLOCK_DEGRADE" in slot and "new DegradeException(" in slot
    pw = slot[slot.index("case V_PRIORITY_WAIT"):]
    pw = pw[:pw.index("case V_BLOCK_FLOW")]
    assert "return;" in pw and "fireEntry" not in pw
    eng = j.source("GpuEngine.java")
    assert "DegradeRuleManager.getRules()" in eng and "LOAD_DEGRADE.invokeExact" in eng
    pk = j.source("ParamPacker.java")
    assert "paramFlowKey()" in pk and "STRINGS" not in pk
    assert "ParamPacker.key(" in j.source("EventBatcher.java")


def test_integration_md_quotes_the_sources():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```java\n// java/\.\.\./(\w+\.java)\n(.*?)```", doc, re.S)
    assert len(blocks) >= 2
    for fn, body in blocks:
        src = j.source(fn)
        for line in body.split("\n"):
            if line.strip():
                assert line.strip() in src, f"INTEGRATION.md line not in {fn}: {line.strip()}"


def test_rule_listeners_keep_the_managers_rules():
    """GpuEngine must not hand a manager an empty property: register2Property
    moves the manager's listener onto it and DynamicSentinelProperty.addListener
    runs configLoad(null) at once (DynamicSentinelProperty.java:37-40), which
    wipes every rule loaded before the first SphU.entry (FlowRuleUtil.java:85-88)
    and detaches an earlier data source.  The shim attaches its listener to each
    manager's current property instead, and follows later swaps per batch."""
    for fn in os.listdir(j.JDIR):
        src = j.source(fn)
        for m in re.finditer(r"register2Property\(([^)]*)\)", src):
            assert False, f"{fn}: register2Property({m.group(1)}) would replace the manager's live rules"
        assert "new DynamicSentinelProperty<>()" not in src, fn
    eng = j.source("GpuEngine.java")
    for mgr in ("FlowRuleManager", "ParamFlowRuleManager", "SystemRuleManager", "DegradeRuleManager"):
        assert f"propertySlot({mgr}.class)" in eng, mgr
    assert '"currentProperty"' in eng and ".addListener(listener)" in eng
    assert "engine.followRuleProperties();" in j.source("EventBatcher.java")
    readme = open(os.path.join(ROOT, "java", "README.md")).read()
    assert "register2Property" in readme and "before or after" in readme


def test_batcher_double_buffers_packed_batches():
    """EventBatcher enqueues batch k+1 (sf_submit_packed_sparse_async) before
    it waits for batch k alone (sf_sync_packed_sparse); two buffer sets
    alternate; the verdicts come back sparse (a status byte per event plus the
    (index << 32 | value) lists of nonzero waits / rule indices, every other
    one 0), as include/sentinel_flow.h sf_sparse_verdicts lays them out."""
    src = j.source("EventBatcher.java")
    fp = src[src.index("private boolean flushPacked"):]
    assert fp.index("SUBMIT_PACKED_SPARSE_ASYNC.invokeExact") < fp.index("collect();                                   // batch k-1")
    assert "SYNC_PACKED_SPARSE.invokeExact(engine.handle, f.pverdicts)" in src
    assert "pbufs[pcur]" in fp and "pcur ^= 1" in fp
    assert "SUBMIT_PACKED.invokeExact" not in src          # no synchronous packed path left
    ds = src[src.index("private static void deliverSparse"):]
    ds = ds[:ds.index("private void flush(")]
    assert "t.waitMs = 0; t.ruleIdx = 0;" in ds and "(int) (x >>> 32)" in ds and "(int) (x & 0xffff)" in ds
    assert ds.index("t.waitMs = 0") < ds.index("getAtIndex(JAVA_LONG, k)") < ds.index("LockSupport.unpark")
    hdr = open(HEADER).read()
    assert "index << 32 | (uint32_t)wait_ms" in hdr and "index << 32 | rule_idx" in hdr
    readme = open(os.path.join(ROOT, "java", "README.md")).read()
    assert "sf_sync_packed" in readme and "latency" in readme.lower()


def test_node_placement_twin():
    """java NodePlacement and sentinel_amd/placement.py give moved resources
    the same engine ids (R_pad + N * j + rank, LPT to the least-loaded rank,
    ties to the lowest rank, stable top-K by count): the Java source carries
    the same expressions, and the Python placement on a Zipf count vector
    balances the ranks (checked statically: no JDK here)."""
    import numpy as np
    from sentinel_amd.placement import Placement
    src = open(os.path.join(ROOT, "java/src/main/java/com/alibaba/csp/sentinel/gpu/NodePlacement.java")).read()
    assert "e[res] = rPad + n * slot[best] + best;" in src
    assert "if (load[q] < load[best]) best = q;" in src
    assert "Long.compare(counts[b], counts[a])" in src
    counts = (1e6 / np.arange(1, 20001) ** 1.1).astype(np.int64)
    p = Placement.balanced(counts, 8, 16384)
    loads = p.loads(counts)
    head = counts[0] * 8 / counts.sum()              # the busiest resource alone, in mean-rank units
    default = Placement(20000, 8).loads(counts)
    assert loads.max() / loads.mean() < 1.05 * max(1.0, head) < default.max() / default.mean()
    assert p.moved.size == 16384
    assert np.all(p.owner(np.arange(20000)) == p.engine_id(np.arange(20000)) % 8)
    assert np.unique(p.engine_id(np.arange(20000))).size == 20000


def test_batcher_narrow_form_twin():
    """EventBatcher's narrow packing (no JDK: checked statically plus a Python
    twin of its loop): 4-byte words res | count << 24 | flags << 27 and
    ms_end[m] = the events with delta <= m, built in one pass over the
    time-ordered batch, equal abi.PackedBatch(narrow=True)'s."""
    import numpy as np
    from sentinel_amd import abi, trace
    src = j.source("EventBatcher.java")
    fp = src[src.index("private boolean flushPacked"):]
    assert "narrow &= (t.resource & 0xffffffffL) < (1L << 24);" in fp
    assert "for (; ms < d; ms++) p.pms.setAtIndex(JAVA_INT, ms, i);" in fp
    assert "if (narrow) p.pms.setAtIndex(JAVA_INT, ms, n);" in fp
    assert '"n_ms"), narrow ? ms + 1 : 0);' in fp and "(c < 1 || c > 7)" in fp
    hb = trace.mixed_zipf(300, 20_000, duration_ms=5000, seed=3)
    d = (hb.ts_ms - hb.ts_ms[0]).astype(np.int64)
    ms_end, ms = [], 0
    for i, di in enumerate(d):                 # the Java loop
        while ms < di:
            ms_end.append(i)
            ms += 1
    ms_end.append(hb.n)
    pb = abi.PackedBatch(hb, narrow=True)
    assert pb.n_ms == ms + 1 and np.array_equal(np.array(ms_end, np.uint32), pb.ms_end)
