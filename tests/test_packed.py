"""Compact batches (sf_submit_packed, include/sentinel_flow.h): the 8-byte
event words and sparse EXIT / acquireCount arrays a host stages for the PCIe
trip.  CPU: the packing is lossless (numpy unpack of abi.PackedBatch).  GPU:
packed batches -- synchronous, and asynchronous with H2D / decide / D2H
overlapped over page-locked buffers -- give the verdicts and node state of the
same batches submitted as SoA, against the oracle."""
import numpy as np
import pytest

from sentinel_amd import abi, trace


def _unpack(pb: abi.PackedBatch):
    w = pb.ev
    res = (w & np.uint64(0xffffffff)).astype(np.uint32)
    ts = pb.ts_base + ((w >> np.uint64(32)) & np.uint64(0xfffff)).astype(np.int64)
    c = ((w >> np.uint64(abi.PK_COUNT_SHIFT)) & np.uint64(0x7f)).astype(np.int32)
    fl = ((w >> np.uint64(abi.PK_FLAGS_SHIFT)) & np.uint64(0x1f)).astype(np.uint8)
    if pb.n_count_ext:
        c[c == 0] = pb.count_ext
    return res, ts, c, fl


def _unpack4(pb: abi.PackedBatch):
    w = pb.ev4
    res = (w & np.uint32(0xffffff)).astype(np.uint32)
    ms = np.searchsorted(pb.ms_end, np.arange(pb.n), side="right")     # first m with ms_end[m] > i
    ts = pb.ts_base + ms.astype(np.int64)
    c = ((w >> np.uint32(abi.PK4_COUNT_SHIFT)) & np.uint32(7)).astype(np.int32)
    fl = (w >> np.uint32(abi.PK4_FLAGS_SHIFT)).astype(np.uint8)
    if pb.n_count_ext:
        c[c == 0] = pb.count_ext
    return res, ts, c, fl


def _batch(seed=3, R=500, n=40_000):
    hb = trace.mixed_zipf(R, n, duration_ms=3000, seed=seed)
    rng = np.random.default_rng(seed)
    cnt = hb.count.copy()
    ent = np.nonzero((hb.flags & abi.EV_EXIT) == 0)[0]
    cnt[ent[rng.random(ent.size) < 0.01]] = 300                  # outside 1..127: count_ext
    return abi.HostBatch(hb.res_id, hb.ts_ms, cnt, hb.flags, entry_ref=hb.entry_ref), R


def test_packing_roundtrip():
    hb, _ = _batch()
    pb = abi.PackedBatch(hb)
    res, ts, c, fl = _unpack(pb)
    assert np.array_equal(res, hb.res_id) and np.array_equal(ts, hb.ts_ms)
    assert np.array_equal(c, hb.count) and np.array_equal(fl, hb.flags)
    ex = np.nonzero(hb.flags & abi.EV_EXIT)[0]
    assert np.array_equal(pb.exit_ref, hb.entry_ref[ex])
    assert pb.nbytes() < 0.45 * (hb.n * 25)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sync", "async", "double"])
def test_gpu_packed_equals_oracle(mode):
    """mode double: the Java flusher's double buffering -- batch k+1 enqueued,
    then sf_sync_packed waits for batch k alone, whose verdicts are checked
    while k+1 is still in flight."""
    from oracle.oracle import OracleEngine
    from sentinel_amd import engine
    from tests import parity
    hb, R = _batch(seed=5, R=800, n=120_000)
    hb = trace.with_origins(hb, n_origins=8, seed=6)
    rules = trace.mixed_rules(R, seed=5)
    cuts = [0, 40_000, 80_000, hb.n]
    parts = [hb.subset(cuts[k], cuts[k + 1]) for k in range(3)]
    cfg = abi.default_config(max_resources=R, max_batch=max(p.n for p in parts))
    eng, ora = engine.FlowEngine(cfg), OracleEngine(cfg)
    pin = engine.PinnedArrays(eng)
    try:
        for x in (eng, ora):
            x.load_flow_rules(rules)
        pbs = [abi.PackedBatch(p, alloc=pin.array) for p in parts]
        outs = [pin.verdicts(p.n) for p in parts]
        if mode == "async":
            for pb, o in zip(pbs, outs):
                eng.submit_packed_async(pb, o)
            eng.sync()
        elif mode == "double":
            eng.submit_packed_async(pbs[0], outs[0])
            for k in range(len(parts)):
                if k + 1 < len(parts):
                    eng.submit_packed_async(pbs[k + 1], outs[k + 1])
                eng.sync_packed(outs[k])
                parity.compare_verdicts(outs[k], ora.submit(parts[k]), f"batch {k}")
            eng.sync_packed(outs[-1])              # already collected: a no-op
            eng.sync()
        else:
            for pb, o in zip(pbs, outs):
                eng.submit_packed(pb, o)
        for k, (p, o) in enumerate(zip(parts, outs)):
            if mode != "double":
                parity.compare_verdicts(o, ora.submit(p), f"batch {k}")
        per_res = np.bincount(hb.res_id, minlength=R)
        parity.compare_nodes(eng, ora, np.argsort(-per_res)[:40])
        parity.compare_entry_node(eng, ora)
    finally:
        pin.free()
        eng.close()
        ora.close()


def test_narrow_packing_roundtrip():
    """The 4-byte form: resource (24 bits), acquireCount 1..7 (else
    count_ext), flags, and the time as the per-millisecond table ms_end."""
    hb, _ = _batch()
    pb = abi.PackedBatch(hb, narrow=True)
    assert pb.ev is None and pb.ev4.dtype == np.uint32 and pb.ms_end[-1] == hb.n
    res, ts, c, fl = _unpack4(pb)
    assert np.array_equal(res, hb.res_id) and np.array_equal(ts, hb.ts_ms)
    assert np.array_equal(c, hb.count) and np.array_equal(fl, hb.flags)
    assert pb.nbytes() < 0.6 * abi.PackedBatch(hb).nbytes()
    assert abi.PackedBatch(hb, narrow="auto").narrow
    big = abi.HostBatch(hb.res_id + np.uint32(1 << 24), hb.ts_ms, hb.count, hb.flags, entry_ref=hb.entry_ref)
    assert not abi.PackedBatch(big, narrow="auto").narrow
    with pytest.raises(ValueError):
        abi.PackedBatch(big, narrow=True)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["dense", "sparse_time"])
def test_gpu_narrow_packed_equals_oracle(kind):
    """The narrow form decided async (double-buffered) equals the oracle:
    dense traffic (a tile's milliseconds staged in LDS) and traffic so
    sparse in time that one 4096-event tile spans more than 1024 ms (the
    table searched in HBM)."""
    from oracle.oracle import OracleEngine
    from sentinel_amd import engine
    from tests import parity
    if kind == "dense":
        hb, R = _batch(seed=11, R=700, n=100_000)
    else:
        R = 300
        hb = trace.mixed_zipf(R, 12_000, duration_ms=60_000, seed=12)
    rules = trace.mixed_rules(R, seed=11)
    cuts = np.linspace(0, hb.n, 4).astype(int)
    parts = [hb.subset(int(cuts[k]), int(cuts[k + 1])) for k in range(3)]
    cfg = abi.default_config(max_resources=R, max_batch=max(p.n for p in parts))
    eng, ora = engine.FlowEngine(cfg), OracleEngine(cfg)
    pin = engine.PinnedArrays(eng)
    try:
        for x in (eng, ora):
            x.load_flow_rules(rules)
        pbs = [abi.PackedBatch(p, alloc=pin.array, narrow=True) for p in parts]
        if kind == "sparse_time":
            assert pbs[0].n_ms > 4096
        outs = [pin.verdicts(p.n) for p in parts]
        eng.submit_packed_async(pbs[0], outs[0])
        for k in range(len(parts)):
            if k + 1 < len(parts):
                eng.submit_packed_async(pbs[k + 1], outs[k + 1])
            eng.sync_packed(outs[k])
            parity.compare_verdicts(outs[k], ora.submit(parts[k]), f"batch {k}")
        eng.sync()
        per_res = np.bincount(hb.res_id, minlength=R)
        parity.compare_nodes(eng, ora, np.argsort(-per_res)[:40])
        parity.compare_all_nodes(eng, ora, R)
        parity.compare_entry_node(eng, ora)
    finally:
        pin.free()
        eng.close()
        ora.close()


@pytest.mark.gpu
def test_gpu_narrow_packed_bad_time_table():
    """A time table that does not end at n is refused at sync (SF_ERR_INVALID)."""
    from sentinel_amd import engine
    hb, R = _batch(seed=13, R=200, n=10_000)
    eng = engine.FlowEngine(abi.default_config(max_resources=R, max_batch=hb.n))
    pin = engine.PinnedArrays(eng)
    try:
        eng.load_flow_rules(trace.mixed_rules(R, seed=13))
        pb = abi.PackedBatch(hb, alloc=pin.array, narrow=True)
        pb.ms_end[-1] = hb.n - 1
        o = pin.verdicts(hb.n)
        with pytest.raises(engine.EngineError):
            eng.submit_packed(pb, o)
    finally:
        pin.free()
        eng.close()


def test_packing_refuses_a_long_span():
    """The ts delta has 20 bits: a longer batch is refused (ValueError, also under python -O)."""
    hb, _ = _batch(n=1000)
    ts = hb.ts_ms.copy()
    ts[-1] = ts[0] + (1 << 20)
    with pytest.raises(ValueError):
        abi.PackedBatch(abi.HostBatch(hb.res_id, ts, hb.count, hb.flags, entry_ref=hb.entry_ref))


@pytest.mark.gpu
@pytest.mark.parametrize("prefetch", [0, 64, 1 << 20])
def test_gpu_packed_sparse_verdicts(prefetch):
    """sf_submit_packed_sparse_async: 1 status byte per event back with the
    batch plus the nonzero waits / rule indices (the first `prefetch` of each
    list with it, the rest at sf_sync_packed_sparse or sf_sync): the dense
    verdicts of the same batches, double-buffered as the Java flusher does."""
    from oracle.oracle import OracleEngine
    from sentinel_amd import engine
    from tests import parity
    hb, R = _batch(seed=7, R=600, n=90_000)
    # a second, tighter QPS rule on every third resource: its blocks carry rule index 1
    rules = list(trace.mixed_rules(R, seed=7)) + [
        abi.sf_flow_rule(resource=r, grade=abi.GRADE_QPS, count=4.0, strategy=0, control_behavior=0,
                         warm_up_period_sec=10, max_queueing_time_ms=500) for r in range(0, R, 3)]
    cuts = [0, 30_000, 60_000, hb.n]
    parts = [hb.subset(cuts[k], cuts[k + 1]) for k in range(3)]
    cfg = abi.default_config(max_resources=R, max_batch=max(p.n for p in parts))
    eng, ora = engine.FlowEngine(cfg), OracleEngine(cfg)
    pin = engine.PinnedArrays(eng)
    try:
        for x in (eng, ora):
            x.load_flow_rules(rules)
        pbs = [abi.PackedBatch(p, alloc=pin.array) for p in parts]
        outs = [pin.sparse_verdicts(p.n, prefetch) for p in parts]
        eng.submit_packed_sparse_async(pbs[0], outs[0])
        waits = rules_n = 0
        for k in range(len(parts)):
            if k + 1 < len(parts):
                eng.submit_packed_sparse_async(pbs[k + 1], outs[k + 1])
            if k < len(parts) - 1:
                eng.sync_packed_sparse(outs[k])
            else:
                eng.sync()                                  # sf_sync completes the lists too
            want = ora.submit(parts[k])
            parity.compare_verdicts(outs[k].dense(), want, f"batch {k}")
            waits += int(outs[k].counts[0]); rules_n += int(outs[k].counts[1])
            assert outs[k].counts[0] == (want.wait_ms != 0).sum() and outs[k].counts[1] == (want.rule_idx != 0).sum()
        assert waits > 64 and rules_n > 64
    finally:
        pin.free()
        eng.close()
        ora.close()


@pytest.mark.gpu
def test_gpu_packed_error_stays_with_its_batch():
    """An async packed batch that raises an error (an exit whose entry ref is
    past the batch) keeps it: a synchronous submit in between drains the
    engine and succeeds, and the failing batch's own sf_sync_packed reports it."""
    from sentinel_amd import engine
    hb, R = _batch(seed=9, R=300, n=20_000)
    cfg = abi.default_config(max_resources=R, max_batch=hb.n)
    eng = engine.FlowEngine(cfg)
    pin = engine.PinnedArrays(eng)
    try:
        eng.load_flow_rules(trace.mixed_rules(R, seed=9))
        bad = abi.PackedBatch(hb, alloc=pin.array)
        bad.exit_ref[0] = hb.n + 5                          # no such entry in the batch
        ob = pin.verdicts(hb.n)
        eng.submit_packed_async(bad, ob)
        good = hb.subset(0, 1000)
        good = abi.HostBatch(good.res_id, good.ts_ms + 4000, good.count, good.flags, entry_ref=good.entry_ref,
                             create_ts=good.create_ts)
        eng.submit(good)                                    # drains; not the other batch's error
        with pytest.raises(engine.EngineError):
            eng.sync_packed(ob)
    finally:
        pin.free()
        eng.close()
