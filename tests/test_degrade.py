"""DegradeSlot circuit breakers: the oracle pinned by the
reference's own known-answer tests, then the HIP path (sf_degrade_submit)
against the oracle, bit for bit (verdicts, blocking breaker index, every
breaker's state and counters).

Known-answer scenarios restated from
sentinel-core/src/test/java/com/alibaba/csp/sentinel/slots/block/degrade/circuitbreaker/
- ResponseTimeCircuitBreakerTest.testMaxSlowRatioThreshold (:32-57)
- ExceptionCircuitBreakerTest.testRecordErrorOrSuccess (:47-83)
driven by AbstractTimeBasedTest's mocked clock (test/AbstractTimeBasedTest.java:40-98):
entryAndSleepFor = entry, sleep(ms), exit; entryWithErrorIfPresent = entry,
Tracer error, sleep(5..10 ms; 7 here), exit; a blocked entry neither sleeps nor exits.
"""
import numpy as np
import pytest

from oracle import degrade as od
from sentinel_amd import abi, trace

RES = 0


class Script:
    """Replays a reference test script against the oracle one event at a time
    (time advances only through sleeps of passed entries), recording the event
    trace and each call's return value."""

    def __init__(self, rules):
        self.o = od.DegradeOracle()
        self.o.load_rules(rules)
        self.t = 0
        self.res, self.ts, self.flags, self.eref = [], [], [], []
        self.returns = []

    def _event(self, flags, ref=-1, create=0):
        st, _ = self.o.submit([RES], [self.t], [flags], [-1], [create])
        self.res.append(RES)
        self.ts.append(self.t)
        self.flags.append(flags)
        self.eref.append(ref)
        return int(st[0])

    def sleep(self, ms):
        self.t += ms

    def _call(self, ms, error):
        t0, idx = self.t, len(self.ts)
        if self._event(0) == od.V_BLOCK_DEGRADE:
            self.returns.append(False)
            return False
        self.sleep(ms)
        self._event(od.EV_EXIT | (od.EV_ERROR if error else 0), ref=idx, create=t0)
        self.returns.append(True)
        return True

    def entry_and_sleep_for(self, ms):
        return self._call(ms, False)

    def entry_with_error(self, error=True):
        return self._call(7, error)

    def batch(self):
        n = len(self.ts)
        return abi.HostBatch(np.array(self.res), np.array(self.ts), np.ones(n, np.int32),
                             np.array(self.flags), entry_ref=np.array(self.eref))


def rt_script():
    rule = abi.degrade_rule(RES, abi.DEGRADE_GRADE_RT, 10, 5, min_request_amount=3, slow_ratio_threshold=1,
                            stat_interval_ms=5000)
    s = Script([rule])
    expect = []
    for _ in range(3):
        expect.append((s.entry_and_sleep_for(20), True))
    expect.append((s.entry_and_sleep_for(20), False))   # 3/3 slow -> open
    s.sleep(1000)
    expect.append((s.entry_and_sleep_for(20), False))
    s.sleep(4000)
    expect.append((s.entry_and_sleep_for(20), True))    # retry timeout -> half-open probe
    return [rule], s, expect


def exception_script():
    rule = abi.degrade_rule(RES, abi.DEGRADE_GRADE_EXCEPTION_RATIO, 0.2, 10, min_request_amount=1,
                            stat_interval_ms=20_000)
    retry = 10_000
    s = Script([rule])
    e = []
    e.append((s.entry_and_sleep_for(10), True))
    e.append((s.entry_with_error(), True))              # -> open
    e.append((s.entry_with_error(), False))
    e.append((s.entry_and_sleep_for(100), False))
    s.sleep(retry // 2)
    e.append((s.entry_and_sleep_for(100), False))
    s.sleep(retry // 2)
    e.append((s.entry_with_error(), True))              # -> half -> open
    e.append((s.entry_and_sleep_for(100), False))
    e.append((s.entry_and_sleep_for(100), False))
    s.sleep(retry)
    e.append((s.entry_and_sleep_for(100), True))        # -> half -> closed
    for _ in range(6):
        e.append((s.entry_and_sleep_for(100), True))
    e.append((s.entry_with_error(), True))
    e.append((s.entry_and_sleep_for(100), True))
    return [rule], s, e


SCRIPTS = {"rt_max_slow_ratio": rt_script, "exception_record_error_or_success": exception_script}


# ---------------------------------------------------------------- oracle (CPU)
@pytest.mark.parametrize("name", list(SCRIPTS))
def test_oracle_reference_scripts(name):
    _, _, expect = SCRIPTS[name]()
    got = [g for g, _ in expect]
    want = [w for _, w in expect]
    assert got == want


def test_oracle_state_machine_details():
    # half-open probe blocked by a later breaker falls back to OPEN with the old retry time
    # (AbstractCircuitBreaker.java:113-129), so the next entry probes again
    r0 = abi.degrade_rule(RES, abi.DEGRADE_GRADE_EXCEPTION_COUNT, 0, 1, min_request_amount=1)
    r1 = abi.degrade_rule(RES, abi.DEGRADE_GRADE_EXCEPTION_COUNT, 0, 3, min_request_amount=1)
    o = od.DegradeOracle()
    assert o.load_rules([r0, r1]) == 2
    st, _ = o.submit([RES, RES], [0, 5], [0, od.EV_EXIT | od.EV_ERROR], [-1, 0], None)
    assert list(st) == [od.V_PASS, od.V_EXIT]
    assert o.state(0)["state"] == od.OPEN and o.state(0)["next_retry_ms"] == 1005
    assert o.state(1)["state"] == od.OPEN and o.state(1)["next_retry_ms"] == 3005
    st, ri = o.submit([RES, RES], [1005, 1006], [0, 0])
    assert list(st) == [od.V_BLOCK_DEGRADE] * 2 and list(ri) == [1, 1]
    assert o.state(0)["state"] == od.OPEN and o.state(0)["next_retry_ms"] == 1005
    # both retry times reached: the probe passes both, a clean exit closes both and resets the bucket
    st, _ = o.submit([RES, RES], [3005, 3010], [0, od.EV_EXIT], [-1, 0])
    assert list(st) == [od.V_PASS, od.V_EXIT]
    for k in (0, 1):
        s = o.state(k)
        assert s["state"] == od.CLOSED and s["hit_count"] == 0 and s["total_count"] == 0
    # exit of a blocked entry records nothing (DegradeSlot.java:72-77)
    o = od.DegradeOracle()
    o.load_rules([r0])
    o.submit([RES, RES], [0, 1], [0, od.EV_EXIT | od.EV_ERROR], [-1, 0])
    st, _ = o.submit([RES, RES], [2, 3], [0, od.EV_EXIT | od.EV_ERROR], [-1, 0])
    assert list(st) == [od.V_BLOCK_DEGRADE, od.V_EXIT_IGNORED]
    assert o.state(0)["total_count"] == 1


def test_oracle_rule_validity():
    # DegradeRuleManager.isValidRule (:183-204)
    ok = abi.degrade_rule(1, abi.DEGRADE_GRADE_RT, 10, 1)
    assert od.is_valid_rule(ok)
    for bad in (dict(count=-1.0), dict(time_window_s=0), dict(min_request_amount=0), dict(stat_interval_ms=0),
                dict(slow_ratio_threshold=1.01), dict(slow_ratio_threshold=-0.1), dict(grade=3)):
        assert not od.is_valid_rule({**ok, **bad}), bad
    assert not od.is_valid_rule(abi.degrade_rule(1, abi.DEGRADE_GRADE_EXCEPTION_RATIO, 1.5, 1))
    assert od.is_valid_rule(abi.degrade_rule(1, abi.DEGRADE_GRADE_EXCEPTION_COUNT, 1.5, 1))
    assert od.java_round(10.5) == 11 and od.java_round(-10.5) == -10 and od.java_round(2.4999) == 2


def test_java_round_edges():
    """Math.round(double) is the exact floor(x + 1/2), saturated (JDK 7+):
    floor(x + 0.5) in double arithmetic gets 0.49999999999999994 wrong."""
    assert od.java_round(0.49999999999999994) == 0
    assert od.java_round(-0.5) == 0 and od.java_round(-0.5000000000000001) == -1
    assert od.java_round(4503599627370497.0) == 4503599627370497        # 2^52 + 1: no +0.5 rounding up
    assert od.java_round(1e19) == (1 << 63) - 1 and od.java_round(-1e19) == -(1 << 63)
    assert od.java_round(float("nan")) == 0 and od.java_round(float("inf")) == (1 << 63) - 1
    # an RT breaker with count 0.49999999999999994 treats rt = 1 as slow (maxAllowedRt 0)
    r = abi.degrade_rule(RES, abi.DEGRADE_GRADE_RT, 0.49999999999999994, 1, min_request_amount=1)
    assert od.Breaker(r).max_rt == 0


def reload_script():
    """A rule reload that keeps an unchanged rule keeps its breaker, OPEN state
    and retry time included (DegradeRuleManager.getExistingSameCbOrNew
    :151-163); a changed rule starts CLOSED."""
    r0 = abi.degrade_rule(RES, abi.DEGRADE_GRADE_EXCEPTION_COUNT, 0, 5, min_request_amount=1)
    r1 = abi.degrade_rule(RES + 1, abi.DEGRADE_GRADE_EXCEPTION_COUNT, 0, 5, min_request_amount=1)
    b1 = abi.HostBatch(np.array([RES, RES, RES + 1, RES + 1]), np.array([0, 3, 4, 6]), np.ones(4, np.int32),
                       np.array([0, od.EV_EXIT | od.EV_ERROR, 0, od.EV_EXIT | od.EV_ERROR], np.uint8),
                       entry_ref=np.array([-1, 0, -1, 2]))
    r1b = dict(r1, min_request_amount=2)                  # changed: a new breaker
    b2 = abi.HostBatch(np.array([RES, RES + 1]), np.array([100, 101]), np.ones(2, np.int32),
                       np.array([0, 0], np.uint8), entry_ref=np.array([-1, -1]))
    return [r0, r1], b1, [r1b, r0], b2


def test_oracle_reload_keeps_unchanged_breaker():
    rules1, b1, rules2, b2 = reload_script()
    o = od.DegradeOracle()
    o.load_rules(rules1)
    o.submit(b1.res_id, b1.ts_ms, b1.flags, b1.entry_ref)
    assert o.state(0)["state"] == od.OPEN and o.state(1)["state"] == od.OPEN
    o.load_rules(rules2)
    assert o.state(1)["state"] == od.OPEN and o.state(1)["next_retry_ms"] == 5003    # r0, now second
    assert o.state(0)["state"] == od.CLOSED                                          # r1 changed
    st, _ = o.submit(b2.res_id, b2.ts_ms, b2.flags, b2.entry_ref)
    assert list(st) == [od.V_BLOCK_DEGRADE, od.V_PASS]
    with pytest.raises(ValueError):
        o.load_rules([rules2[1], dict(rules2[1])])          # equal rules would share one breaker


def test_workload_generator_shape():
    b = trace.degrade_workload(100, 2000, duration_ms=500, seed=1)
    assert np.all(np.diff(b.ts_ms) >= 0)
    ex = np.nonzero(b.flags & abi.EV_EXIT)[0]
    assert np.all(b.entry_ref[ex] >= 0) and np.all(b.entry_ref[ex] < ex)
    assert np.all(b.res_id[b.entry_ref[ex]] == b.res_id[ex])
    assert np.all((b.flags[b.entry_ref[ex]] & abi.EV_EXIT) == 0)


def oracle_run(rules, batches):
    o = od.DegradeOracle()
    n = o.load_rules(rules)
    outs = [o.submit(b.res_id, b.ts_ms, b.flags, b.entry_ref, b.create_ts) for b in batches]
    return outs, [o.state(k) for k in range(n)]


# ---------------------------------------------------------------- HIP path (GPU)
def _engine(R, max_batch):
    from sentinel_amd import engine
    return engine.FlowEngine(abi.default_config(max_resources=R, max_batch=max_batch))


def check_gpu(rules, batches, R, tag):
    e = _engine(R, max(b.n for b in batches))
    try:
        n = e.load_degrade_rules(rules)
        outs, states = oracle_run(rules, batches)
        assert n == len(states)
        for bi, (b, (st, ri)) in enumerate(zip(batches, outs)):
            v = e.degrade_submit(b)
            bad = np.nonzero(v.status != st)[0]
            assert bad.size == 0, f"{tag} batch {bi}: {bad.size} verdicts differ, first at {bad[:5]}"
            blk = st == od.V_BLOCK_DEGRADE
            assert np.array_equal(v.rule_idx[blk], ri[blk]), f"{tag} batch {bi}: breaker index"
            assert np.all(v.wait_ms == 0)
        for k, want in enumerate(states):
            assert e.read_breaker(k) == want, f"{tag} breaker {k}"
        return outs
    finally:
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SCRIPTS))
def test_gpu_reference_scripts(name):
    rules, s, expect = SCRIPTS[name]()
    outs = check_gpu(rules, [s.batch()], 4, name)
    st = outs[0][0]
    entries = st[(s.batch().flags & abi.EV_EXIT) == 0]
    assert list(entries != od.V_BLOCK_DEGRADE) == [w for _, w in expect]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_mixed_breakers(seed):
    R = 3000
    rules = trace.degrade_rules(R, seed=seed)
    full = trace.degrade_workload(R, 60_000, duration_ms=8000, seed=seed, err_p=0.2)
    cut = [0, full.n // 3, full.n // 2, full.n]                # cross-batch exits via create_ts
    batches = [full.subset(cut[i], cut[i + 1]) for i in range(3)]
    outs = check_gpu(rules, batches, R, f"seed {seed}")
    allst = np.concatenate([o[0] for o in outs])
    assert (allst == od.V_BLOCK_DEGRADE).sum() > 100              # breakers did open
    assert (allst == od.V_EXIT_IGNORED).sum() > 0


@pytest.mark.gpu
def test_gpu_no_rules_and_sharding():
    from sentinel_amd import engine
    b = trace.degrade_workload(64, 5000, duration_ms=1000, seed=9)
    e = _engine(64, b.n)
    try:
        assert e.load_degrade_rules([]) == 0
        v = e.degrade_submit(b)
        want = np.where(b.flags & abi.EV_EXIT, od.V_EXIT, od.V_PASS)
        assert np.array_equal(v.status, want)
    finally:
        e.close()
    cfg = abi.default_config(max_resources=64, max_batch=b.n)
    cfg.shard_count, cfg.shard_index = 2, 1
    e = engine.FlowEngine(cfg)
    try:
        with pytest.raises(engine.EngineError):
            e.degrade_submit(b)                                   # events of the other shard
        sh = b.shard(2, 1)
        rules = [r for r in trace.degrade_rules(64, seed=4, invalid=0) if r["resource"] % 2 == 1]
        o = od.DegradeOracle()
        o.load_rules(rules)
        st, _ = o.submit(sh.res_id, sh.ts_ms, sh.flags, sh.entry_ref, sh.create_ts)
        e.load_degrade_rules(rules)
        assert np.array_equal(e.degrade_submit(sh).status, st)
    finally:
        e.close()


@pytest.mark.gpu
def test_gpu_reload_keeps_unchanged_breaker():
    from sentinel_amd import engine
    rules1, b1, rules2, b2 = reload_script()
    o = od.DegradeOracle()
    o.load_rules(rules1)
    e = _engine(4, 16)
    try:
        e.load_degrade_rules(rules1)
        st, _ = o.submit(b1.res_id, b1.ts_ms, b1.flags, b1.entry_ref)
        assert np.array_equal(e.degrade_submit(b1).status, st)
        o.load_rules(rules2)
        e.load_degrade_rules(rules2)
        for k in range(2):
            assert e.read_breaker(k) == o.state(k), k
        st, _ = o.submit(b2.res_id, b2.ts_ms, b2.flags, b2.entry_ref)
        assert np.array_equal(e.degrade_submit(b2).status, st)
        with pytest.raises(engine.EngineError):
            e.load_degrade_rules([rules2[1], dict(rules2[1])])
        for k in range(2):                                  # the failed load changed nothing
            assert e.read_breaker(k) == o.state(k), k
    finally:
        e.close()


@pytest.mark.gpu
def test_gpu_bad_exit_refs_and_clock():
    """An EXIT whose entry_ref names another resource's event, an exit, or a
    later event is refused (SF_ERR_INVALID), as is a clock that goes back
    (within a batch or against the previous batch)."""
    from sentinel_amd import engine
    rules = [abi.degrade_rule(r, abi.DEGRADE_GRADE_EXCEPTION_COUNT, 0, 5, min_request_amount=1) for r in range(2)]
    ok = abi.HostBatch(np.array([0, 1, 0, 1]), np.array([10, 11, 12, 13]), np.ones(4, np.int32),
                       np.array([0, 0, od.EV_EXIT, od.EV_EXIT], np.uint8), entry_ref=np.array([-1, -1, 0, 1]))
    bads = [np.array([-1, -1, 1, 1]), np.array([-1, -1, 3, 1]), np.array([-1, -1, 0, 2])]
    for eref in bads:
        e = _engine(4, 16)
        try:
            e.load_degrade_rules(rules)
            with pytest.raises(engine.EngineError):
                e.degrade_submit(abi.HostBatch(ok.res_id, ok.ts_ms, ok.count, ok.flags, entry_ref=eref))
        finally:
            e.close()
    e = _engine(4, 16)
    try:
        e.load_degrade_rules(rules)
        e.degrade_submit(ok)
        with pytest.raises(engine.EngineError):                       # earlier than the last batch
            e.degrade_submit(abi.HostBatch(ok.res_id, ok.ts_ms - 5, ok.count, ok.flags, entry_ref=ok.entry_ref))
        with pytest.raises(engine.EngineError):                       # backwards inside the batch
            e.degrade_submit(abi.HostBatch(ok.res_id, ok.ts_ms[::-1] + 100, ok.count, np.zeros(4, np.uint8)))
    finally:
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 5])
def test_gpu_long_segments(seed):
    """Few resources, thousands of events each: the wave walk (segments > 64
    events, <= 4 breakers), its chunk boundaries and tail chunks; resource 0
    carries 5 breakers and stays on the lane walk."""
    R = 16
    rules = trace.degrade_rules(R, seed=seed, frac=1.0, invalid=2)
    extra = [abi.degrade_rule(0, g, c, 1, min_request_amount=2, stat_interval_ms=500)
             for g, c in [(0, 15.0), (1, 0.4), (2, 3.0), (0, 25.0), (1, 0.2)]]
    rules = extra + [r for r in rules if r["resource"] != 0]
    full = trace.degrade_workload(R, 40_000, duration_ms=6000, seed=seed, err_p=0.2, s=0.8)
    cut = [0, 20_001, full.n]
    outs = check_gpu(rules, [full.subset(cut[i], cut[i + 1]) for i in range(2)], R, f"long {seed}")
    allst = np.concatenate([o[0] for o in outs])
    assert (allst == od.V_BLOCK_DEGRADE).sum() > 100 and (allst == od.V_EXIT_IGNORED).sum() > 0
