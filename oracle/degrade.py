"""TEST INFRASTRUCTURE ONLY — CPU restatement of Sentinel's DegradeSlot circuit
breakers, the checker for ``sf_degrade_submit``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it.

Replayed single-threaded with a mocked TimeUtil clock (every call within one
event returns that event's timestamp), exactly like the reference's
``AbstractTimeBasedTest``.  Pinned by the reference's own known-answer
scenarios (``tests/test_degrade.py`` restates ResponseTimeCircuitBreakerTest
and ExceptionCircuitBreakerTest step by step).

Reference (sentinel-core/src/main/java/com/alibaba/csp/sentinel/slots/block/degrade/):
- DegradeRuleManager.isValidRule            DegradeRuleManager.java:183-204
- DegradeRuleManager.buildCircuitBreakers   DegradeRuleManager.java:236-265 (rule list order)
- DegradeSlot.performChecking / exit        DegradeSlot.java:50-94
- AbstractCircuitBreaker.tryPass & state    circuitbreaker/AbstractCircuitBreaker.java:67-173
- ResponseTimeCircuitBreaker                circuitbreaker/ResponseTimeCircuitBreaker.java:52-130
- ExceptionCircuitBreaker                   circuitbreaker/ExceptionCircuitBreaker.java:47-119
- LeapArray(sampleCount=1).currentWindow    slots/statistic/base/LeapArray.java:128-225
"""
import math

import numpy as np

GRADE_RT, GRADE_EXC_RATIO, GRADE_EXC_COUNT = 0, 1, 2
CLOSED, OPEN, HALF_OPEN = 0, 1, 2

EV_EXIT, EV_ERROR, EV_BLOCKED = 0x01, 0x08, 0x10
V_PASS, V_EXIT, V_EXIT_IGNORED, V_BLOCK_DEGRADE, V_BLOCK_OTHER = 0, 6, 7, 8, 9


def java_round(x: float) -> int:
    """Math.round(double) (Java 7+): the exact floor(x + 1/2) -- no rounding
    error in the addition (0.49999999999999994 rounds to 0) -- saturated to
    the long range, NaN to 0."""
    x = float(x)
    if math.isnan(x):
        return 0
    if x >= 9223372036854775807.0:
        return (1 << 63) - 1
    if x <= -9223372036854775808.0:
        return -(1 << 63)
    f = math.floor(x)
    return int(f) + (1 if x - f >= 0.5 else 0)     # x - floor(x) is exact for a double


def is_valid_rule(r) -> bool:
    """DegradeRuleManager.isValidRule (:183-204); r = dict of sf_degrade_rule fields."""
    if not (r["count"] >= 0 and r["time_window_s"] > 0):
        return False
    if r["min_request_amount"] <= 0 or r["stat_interval_ms"] <= 0:
        return False
    g = r["grade"]
    if g == GRADE_RT:
        return 0 <= r["slow_ratio_threshold"] <= 1
    if g == GRADE_EXC_RATIO:
        return r["count"] <= 1
    return g == GRADE_EXC_COUNT


class Breaker:
    """One CircuitBreaker with its LeapArray(1, statIntervalMs) counter."""

    def __init__(self, r):
        self.rule = {k: r[k] for k in ("resource", "grade", "count", "time_window_s", "min_request_amount",
                                       "slow_ratio_threshold", "stat_interval_ms")}
        self.grade = r["grade"]
        self.max_rt = java_round(r["count"])             # ResponseTimeCircuitBreaker :52
        self.threshold = float(r["slow_ratio_threshold"] if self.grade == GRADE_RT else r["count"])
        self.min_req = int(r["min_request_amount"])
        self.recovery = int(r["time_window_s"]) * 1000   # AbstractCircuitBreaker :54
        self.interval = int(r["stat_interval_ms"])
        self.state = CLOSED
        self.next_retry = 0
        self.ws = None                                   # the single bucket (null until first use)
        self.hit = 0
        self.total = 0

    def same_rule(self, r) -> bool:
        """DegradeRule.equals: the six fields by Double.compare, same resource."""
        def deq(a, b):
            a, b = float(a), float(b)
            return (a != a and b != b) or np.float64(a).tobytes() == np.float64(b).tobytes()
        o = self.rule
        return (int(o["resource"]) == int(r["resource"]) and int(o["grade"]) == int(r["grade"])
                and deq(o["count"], r["count"]) and int(o["time_window_s"]) == int(r["time_window_s"])
                and int(o["min_request_amount"]) == int(r["min_request_amount"])
                and deq(o["slow_ratio_threshold"], r["slow_ratio_threshold"])
                and int(o["stat_interval_ms"]) == int(r["stat_interval_ms"]))

    def _current(self, t):
        """LeapArray.currentWindow(t) with one bucket: create / keep / reset (:128-225)."""
        ws = t - t % self.interval
        if self.ws is None or ws > self.ws:
            self.ws, self.hit, self.total = ws, 0, 0
        # ws < self.ws cannot happen: timestamps are non-decreasing

    def try_pass(self, t):
        """AbstractCircuitBreaker.tryPass (:67-82). Returns (passed, moved_to_half_open)."""
        if self.state == CLOSED:
            return True, False
        if self.state == OPEN and t >= self.next_retry:  # retryTimeoutArrived && fromOpenToHalfOpen
            self.state = HALF_OPEN
            return True, True
        return False, False

    def _to_open(self, t):
        self.state = OPEN
        self.next_retry = t + self.recovery              # updateNextRetryTimestamp (:93-95)

    def on_complete(self, t, rt, error):
        """onRequestComplete + handleStateChangeWhenThresholdExceeded."""
        self._current(t)
        hit = (rt > self.max_rt) if self.grade == GRADE_RT else bool(error)
        if hit:
            self.hit += 1
        self.total += 1
        if self.state == OPEN:
            return
        if self.state == HALF_OPEN:
            if hit:
                self._to_open(t)                         # fromHalfOpenToOpen
            else:
                self.state = CLOSED                      # fromHalfOpenToClose -> resetStat
                self._current(t)
                self.hit = self.total = 0
            return
        # values(t): the single bucket is current, so always valid
        if self.total < self.min_req:
            return
        if self.grade == GRADE_RT:
            ratio = self.hit * 1.0 / self.total
            if ratio > self.threshold or (ratio == self.threshold and self.threshold == 1.0):
                self._to_open(t)
        else:
            cur = self.hit * 1.0 / self.total if self.grade == GRADE_EXC_RATIO else float(self.hit)
            if cur > self.threshold:
                self._to_open(t)


class DegradeOracle:
    def __init__(self):
        self.breakers = []        # load order of valid rules
        self.by_res = {}          # resource -> [breaker indices] in rule order
        self.created = {}         # entries passed in earlier batches are looked up by create_ts

    def load_rules(self, rules):
        """buildCircuitBreakers (:236-265) with getExistingSameCbOrNew (:151-163):
        a valid rule equal (DegradeRule.equals :153-164) to one of the
        resource's current breakers keeps that breaker, state included."""
        old = {}
        for res, ks in self.by_res.items():
            old[res] = [self.breakers[k] for k in ks]
        self.breakers, self.by_res = [], {}
        for r in rules:
            if not is_valid_rule(r):
                continue
            res = int(r["resource"])
            cb = next((b for b in old.get(res, ()) if b.same_rule(r)), None)
            if cb is not None and any(b is cb for b in self.breakers):
                raise ValueError("two equal rules share one breaker (the engine refuses this reload)")
            self.by_res.setdefault(res, []).append(len(self.breakers))
            self.breakers.append(cb if cb is not None else Breaker(r))
        return len(self.breakers)

    def submit(self, res, ts, flags, entry_ref=None, create_ts=None):
        """Returns (status u8[n], rule_idx u16[n]) for a time-ordered batch."""
        n = len(res)
        status = np.zeros(n, np.uint8)
        rule_idx = np.zeros(n, np.uint16)
        for i in range(n):
            r, t, f = int(res[i]), int(ts[i]), int(flags[i])
            cbs = self.by_res.get(r, ())
            if not f & EV_EXIT:
                if f & EV_BLOCKED:                          # blocked by an earlier slot: DegradeSlot never runs
                    status[i] = V_BLOCK_OTHER
                    continue
                moved = []
                blocked = -1
                for k, b in enumerate(cbs):                 # DegradeSlot.performChecking (:50-61)
                    ok, mv = self.breakers[b].try_pass(t)
                    if mv:
                        moved.append(b)
                    if not ok:
                        blocked = k
                        break
                if blocked >= 0:
                    for b in moved:                         # whenTerminate hook (:113-129)
                        if self.breakers[b].state == HALF_OPEN:
                            self.breakers[b].state = OPEN
                    status[i], rule_idx[i] = V_BLOCK_DEGRADE, blocked
                else:
                    status[i] = V_PASS
                continue
            ref = -1 if entry_ref is None else int(entry_ref[i])
            if ref == -2:                                   # entry blocked in an earlier batch
                status[i] = V_EXIT_IGNORED
                continue
            if ref >= 0:
                if status[ref] in (V_BLOCK_DEGRADE, V_BLOCK_OTHER):   # DegradeSlot.exit (:72-77): blockError set
                    status[i] = V_EXIT_IGNORED
                    continue
                created = int(ts[ref])
            else:
                created = int(create_ts[i])
            rt = t - created
            for b in cbs:                                    # DegradeSlot.exit (:85-91)
                self.breakers[b].on_complete(t, rt, f & EV_ERROR)
            status[i] = V_EXIT
        return status, rule_idx

    def state(self, k):
        b = self.breakers[k]
        return dict(state=b.state, next_retry_ms=b.next_retry,
                    window_start=(b.ws if b.ws is not None else None), hit_count=b.hit, total_count=b.total)
