"""ParameterMetric's bounded maps (SURVEY.md §7 hard part 6).

The reference keeps every ParamFlow counter in a ConcurrentLinkedHashMap LRU
(ConcurrentLinkedHashMapWrapper.java:35-44) of capacity
min(4000 * durationInSec, 200000) per rule and 4000 per thread-count map
(ParameterMetric.java:37-39, 99-121); the engine keeps an exact table.  The
oracle restates both (oracle/sentinel_oracle.c, CacheMap section): exact by
default, the LRU with OracleEngine.set_param_lru / ParameterMetric(lru=True).

No reference test exceeds a map's capacity, so the LRU restatement follows
the library's published algorithm (CLHM 1.4.2, single-threaded: a strict LRU
over reads and inserts) and is pinned by the reference's own ParamFlow KATs
(which it must still pass) plus the hand-checked eviction cases below.

When exact and LRU agree: an evicted key's next access is a first sight
(tokens = maxCount - acquireCount, time = now).  If the key had been idle
longer than durationInSec, the exact map's refill (passTime > duration: toAdd
>= tokenCount, so newQps = maxCount - acquireCount, lastAddTokenTime = now,
ParamFlowChecker.java:173-195) leaves the same state, and a throttle rule
passes and records now either way (cost <= duration).  The verdicts differ
only when a key is evicted within durationInSec of its last access, i.e. when
a rule sees at least `capacity` distinct other keys in under durationInSec.
"""
import numpy as np
import pytest

from sentinel_amd import abi, trace
from tests.test_oracle_kat import S, STARTS, _prule

CAP = 4000   # BASE_PARAM_MAX_CAPACITY * durationInSec (1), THREAD_COUNT_MAX_CAPACITY


@pytest.mark.parametrize("t0", STARTS)
def test_lru_mode_passes_the_reference_kats(so, t0):
    """ParamFlowDefaultCheckerTest (:78-174): single-key sequences never evict."""
    pm = so.ParameterMetric(lru=True)
    rule = _prule(count=5)
    pm.initialize(0, rule)
    so.set_time(t0)
    assert [pm.pass_single(0, rule, S("valueA")) for _ in range(6)] == [True] * 5 + [False]
    so.set_time(t0 + 3000)
    assert [pm.pass_single(0, rule, S("valueA")) for _ in range(6)] == [True] * 5 + [False]
    pm = so.ParameterMetric(lru=True)
    rule = _prule(count=5, burst_count=3)
    pm.initialize(0, rule)
    t = t0
    for dt, n_true in [(0, 8), (1002, 5), (1002, 5), (2000, 8), (1002, 5)]:
        t += dt
        so.set_time(t)
        assert [pm.pass_single(0, rule, S("valueA")) for _ in range(n_true + 1)] == [True] * n_true + [False]
    assert pm.evictions() == 0


def _keys(n, base=1000):
    return [(abi.TAG_LONG, base + i) for i in range(n)]


def test_lru_evicts_the_least_recently_used_key(so):
    """Capacity 4000 at durationInSec 1: the 4001st distinct key evicts the
    least recently used one from both the time and the token map; a re-seen
    evicted key is a first sight (passes with fresh tokens) where the exact
    map blocks it."""
    rule = _prule(count=1)
    for lru in (False, True):
        pm = so.ParameterMetric(lru=lru)
        pm.initialize(0, rule)
        so.set_time(STARTS[0])
        a = (abi.TAG_LONG, 7)
        assert pm.pass_single(0, rule, a)            # tokens 1 -> 0
        for k in _keys(CAP):                         # 4000 more distinct keys
            assert pm.pass_single(0, rule, k)
        so.set_time(STARTS[0] + 1)
        assert pm.pass_single(0, rule, a) is lru     # exact: no token left; LRU: evicted -> first sight
        assert pm.evictions() == (2 * 2 if lru else 0)   # a, then the oldest of the 4000 (both maps)


def test_lru_reads_refresh_recency(so):
    """A read (putIfAbsent of a present key / get) moves the key to the back:
    the eviction takes the least recently *accessed* key, not the oldest insert."""
    rule = _prule(count=1)
    pm = so.ParameterMetric(lru=True)
    pm.initialize(0, rule)
    so.set_time(STARTS[1])
    a = (abi.TAG_LONG, 7)
    ks = _keys(CAP)
    assert pm.pass_single(0, rule, a)
    for k in ks[:CAP - 1]:                            # the map is full: a + 3999 keys
        pm.pass_single(0, rule, k)
    assert not pm.pass_single(0, rule, a)             # a read: a becomes the most recent
    assert pm.pass_single(0, rule, ks[CAP - 1])       # evicts ks[0], not a
    assert not pm.pass_single(0, rule, a)             # a still held, no token
    assert pm.pass_single(0, rule, ks[0])             # ks[0] was evicted: first sight again
    assert pm.evictions() == 2 * 2


def test_eviction_after_idle_duration_equals_exact(so):
    """A key evicted after more than durationInSec idle is decided as the
    exact map decides it (refill to maxCount - acquireCount)."""
    rule = _prule(count=3)
    got = {}
    for lru in (False, True):
        pm = so.ParameterMetric(lru=lru)
        pm.initialize(0, rule)
        t = STARTS[2]
        so.set_time(t)
        a = (abi.TAG_LONG, 7)
        seq = [pm.pass_single(0, rule, a) for _ in range(4)]
        so.set_time(t + 1200)
        for k in _keys(CAP + 10):
            pm.pass_single(0, rule, k)
        so.set_time(t + 1201)
        seq += [pm.pass_single(0, rule, a) for _ in range(4)]
        got[lru] = seq
    assert got[False] == got[True] == [True] * 3 + [False] + [True] * 3 + [False]


def test_throttle_rule_lru(so):
    """passThrottleLocalCheck's time map is bounded the same way."""
    rule = _prule(count=2, control_behavior=abi.BEHAVIOR_RATE_LIMITER, max_queueing_time_ms=0)
    for lru in (False, True):
        pm = so.ParameterMetric(lru=lru)
        pm.initialize(0, rule)
        so.set_time(STARTS[3])
        a = (abi.TAG_LONG, 7)
        assert pm.pass_single(0, rule, a)             # cost 500 ms
        for k in _keys(CAP):
            pm.pass_single(0, rule, k)
        so.set_time(STARTS[3] + 10)
        assert pm.pass_single(0, rule, a) is lru      # exact: 490 ms early, no queue; LRU: first sight


def test_thread_count_map_lru(so):
    """threadCountMap: THREAD_COUNT_MAX_CAPACITY 4000 (ParameterMetric.java:37)."""
    rule = _prule(grade=abi.GRADE_THREAD, count=1)
    for lru in (False, True):
        pm = so.ParameterMetric(lru=lru)
        pm.initialize(0, rule)
        a = (abi.TAG_LONG, 7)
        pm.add_thread(0, a)
        for k in _keys(CAP):
            pm.add_thread(0, k)
        assert pm.thread_count(0, a) == (0 if lru else 1)


def _cycling_batch(n_keys=5000, per_ms=10, cycles=3):
    """One resource, a rule of count 1: n_keys distinct keys in a fixed cycle,
    each re-seen n_keys / per_ms ms later (500 ms < durationInSec)."""
    n = n_keys * cycles
    ts = trace.T0 + np.arange(n, dtype=np.int64) // per_ms
    keys = (np.arange(n) % n_keys + 1).astype(np.uint64)
    b = abi.HostBatch(np.zeros(n, np.uint32), ts, np.ones(n, np.int32), np.full(n, abi.EV_IN, np.uint8),
                      arg_tag=np.full((1, n), abi.TAG_LONG, np.uint8), arg_bits=keys.reshape(1, -1))
    return [_prule(count=1)], b


def test_engine_lru_diverges_when_keys_cycle_within_the_duration(so):
    """5000 keys cycling every 500 ms through a 4000-entry map: every repeat is
    evicted before it comes back, so the reference passes it (first sight)
    while the exact map blocks it -- the divergence the exact table declares."""
    rules, b = _cycling_batch()
    cfg = abi.default_config(max_resources=1, max_batch=b.n)
    out = {}
    for lru in (False, True):
        o = so.OracleEngine(cfg)
        if lru:
            o.set_param_lru(True)
        o.load_param_rules(rules)
        out[lru] = o.submit(b).status
        ev, spins = o.param_lru_stats()
        assert spins == 0
        if lru:
            assert ev > 0
        o.close()
    first = np.arange(b.n) < 5000
    assert (out[False][first] == abi.V_PASS).all() and (out[True] == abi.V_PASS).all()
    # second cycle: 500 ms after the first sight, within the duration -> blocked by the exact map;
    # third cycle: passTime == 1000 is not > 1000 -> still blocked
    assert (out[False][~first] == abi.V_BLOCK_PARAM).all()


def config4_like(R=24, n=400_000, keys=100_000_000, qps_frac=0.6, seed=4):
    """The bench's config-4 shape at a test size: ~16.7k events per resource
    (as config 4), so ~6.9k distinct keys per rule -- over the 4000 capacity."""
    rules, b = trace.param_zipf(R, n, keys, duration_ms=4000, seed=seed)
    sysr = [abi.sf_system_rule(highest_system_load=-1, highest_cpu_usage=-1, qps=qps_frac * b.n / 4.0,
                               avg_rt=-1, max_thread=-1)]
    return rules, sysr, b


def _oracle(so, cfg, rules, sysr, b, lru):
    o = so.OracleEngine(cfg)
    if lru:
        o.set_param_lru(True)
    o.load_system_rules(sysr)
    o.load_param_rules(rules)
    v = o.submit(b)
    stats = o.param_lru_stats()
    o.close()
    return v, stats


def test_config4_shape_lru_equals_exact(so):
    """Over capacity (thousands of evictions) yet no verdict differs: the
    evicted keys had been idle longer than durationInSec (module docstring)."""
    rules, sysr, b = config4_like()
    pairs = np.unique(b.res_id.astype(np.uint64) << np.uint64(40) ^ (b.arg_bits[0] & np.uint64((1 << 40) - 1)))
    per_rule = np.bincount((pairs >> np.uint64(40)).astype(np.int64))
    assert per_rule.min() > CAP
    cfg = abi.default_config(max_resources=24, max_batch=b.n)
    exact, _ = _oracle(so, cfg, rules, sysr, b, False)
    lru, (ev, spins) = _oracle(so, cfg, rules, sysr, b, True)
    assert ev > 10_000 and spins == 0
    assert np.array_equal(exact.status, lru.status)
    assert np.array_equal(exact.wait_ms, lru.wait_ms) and np.array_equal(exact.rule_idx, lru.rule_idx)


@pytest.mark.gpu
def test_gpu_config4_shape_over_capacity_matches_the_lru_reference():
    """The engine's exact table against the LRU restatement of the reference on
    the config-4 shape with more distinct keys per rule than the reference's
    map holds: every verdict, wait and rule index equal."""
    from oracle import oracle as so
    from sentinel_amd import engine
    rules, sysr, b = config4_like()
    cfg = abi.default_config(max_resources=24, max_batch=b.n)
    lru, (ev, _) = _oracle(so, cfg, rules, sysr, b, True)
    assert ev > 10_000
    e = engine.FlowEngine(cfg)
    try:
        e.load_system_rules(sysr)
        e.load_param_rules(rules)
        got = e.submit(b)
    finally:
        e.close()
    assert (got.status == abi.V_BLOCK_PARAM).sum() > 1000 and (got.status == abi.V_BLOCK_SYSTEM).sum() > 1000
    assert np.array_equal(got.status, lru.status)
    assert np.array_equal(got.wait_ms, lru.wait_ms) and np.array_equal(got.rule_idx, lru.rule_idx)


@pytest.mark.gpu
def test_gpu_param_thread_counts_on_the_wave_path():
    """ParameterMetric's thread counts after a Zipf batch whose ParamFlow
    segments run on the wavefront path (heavy_param, one table update per
    distinct value of a 64-event group): every counted value of every
    resource equals the oracle's (ParamFlowStatisticEntryCallback adds one
    per passing entry, ParameterMetric.addThreadCount :184-239)."""
    from oracle import oracle as so
    from sentinel_amd import engine, trace
    R = 24
    rules, b = trace.param_zipf(R, 200_000, 5000, duration_ms=2000, seed=7)
    cfg = abi.default_config(max_resources=R, max_batch=b.n, param_capacity=1 << 20)
    e = engine.FlowEngine(cfg)
    o = so.OracleEngine(cfg)
    try:
        e.load_param_rules(rules)
        o.load_param_rules(rules)
        got = e.submit(b)
        want = o.submit(b)
        assert np.array_equal(got.status, want.status)
        checked = big = 0
        for r in range(R):
            sel = b.res_id == r
            vals, cnt = np.unique(b.arg_bits[0][sel], return_counts=True)
            for v in vals[np.argsort(-cnt)][:40]:
                w = o.param_thread(r, 0, (abi.TAG_LONG, int(v)))
                assert e.param_thread(r, 0, (abi.TAG_LONG, int(v))) == w, (r, int(v))
                checked += 1
                big += w > 1
        assert checked > 500 and big > 50
    finally:
        e.close()
