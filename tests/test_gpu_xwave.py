"""The wave walk of long xflow segments (sf_kernels.hip k_decide_xw) against
the C oracle.

A resource whose rules all check DIRECT (its ClusterNode, or an origin node
through an origin-specific or `other` limitApp; FlowRuleChecker.java:129-161)
and that has no ParamFlow rule and no circuit breaker is its own xflow group;
its segments of at least XW_MIN (256) events are decided by one wavefront in
chunks of one bucket: entries blocked by the first selecting rule at the
chunk's start state are settled in parallel, the rest walk serially, blocks
and completions are summed per node.  These tests cover every controller on
either node (QPS reject, WarmUp, RateLimiter, WarmUp + RateLimiter, THREAD),
prioritized entries, SF_EV_BLOCKED entries, exits in and across batches, and
compare every verdict, wait and rule index, the ClusterNodes, every origin
node of the busiest resources and ENTRY_NODE with the oracle."""
import numpy as np
import pytest

from sentinel_amd import abi, trace
from tests.test_gpu_origin import _run, _sample_pairs

pytestmark = pytest.mark.gpu


def _origin_rules(R, per_res, seed):
    """The config-3 rule of every resource, plus on the 40 busiest ones a rule
    that reads an origin node: `other` or origin-specific, each controller."""
    rules = list(trace.mixed_rules(R, seed=seed))
    busy = np.argsort(-per_res)[:40]
    kinds = [(abi.GRADE_QPS, abi.BEHAVIOR_DEFAULT), (abi.GRADE_QPS, abi.BEHAVIOR_WARM_UP),
             (abi.GRADE_QPS, abi.BEHAVIOR_RATE_LIMITER), (abi.GRADE_QPS, abi.BEHAVIOR_WARM_UP_RATE_LIMITER),
             (abi.GRADE_THREAD, abi.BEHAVIOR_DEFAULT)]
    for k, r in enumerate(busy):
        g, b = kinds[k % len(kinds)]
        app = abi.APP_OTHER if k % 3 else 2 + (k % 4)           # `other`, or origin 2..5 by name
        rules.append(abi.sf_flow_rule(resource=int(r), grade=g, count=float(3 + (k * 7) % 40), strategy=0,
                                      control_behavior=b, warm_up_period_sec=2, max_queueing_time_ms=200,
                                      limit_app=app))
    return rules, busy


def _flags(hb, seed, prio=0.02, blocked=0.03):
    rng = np.random.default_rng(seed)
    fl = hb.flags.copy()
    ent = (fl & abi.EV_EXIT) == 0
    fl[ent & (rng.random(hb.n) < prio)] |= abi.EV_PRIO
    bl = ent & (rng.random(hb.n) < blocked)
    fl[bl] |= abi.EV_BLOCKED
    # (an exit of a pre-blocked entry keeps its entry_ref: the engine sees the block)
    return abi.HostBatch(hb.res_id, hb.ts_ms, hb.count, fl, entry_ref=hb.entry_ref, create_ts=hb.create_ts,
                         origin=hb.origin)


@pytest.mark.parametrize("seed", [51, 52])
def test_gpu_xwave_controllers(seed):
    R = 3000
    hb = trace.with_origins(trace.mixed_zipf(R, 900_000, duration_ms=5000, seed=seed), n_origins=24, seed=seed + 1)
    hb = _flags(hb, seed + 2)
    per_res = np.bincount(hb.res_id, minlength=R)
    rules, busy = _origin_rules(R, per_res, seed)
    assert (per_res[busy] >= 3 * 256).all()                   # every rule-bearing resource: wave-walk segments
    cuts = [0, 300_011, 600_007, hb.n]
    batches = [hb.subset(cuts[i], cuts[i + 1]) for i in range(3)]
    cfg = abi.default_config(max_resources=R, max_batch=max(b.n for b in batches))
    pairs = _sample_pairs(hb, k_busy=40, k_rand=200, seed=seed)
    _run(rules, batches, cfg, pairs, np.concatenate([busy, np.argsort(-per_res)[40:60]]))


def test_gpu_xwave_async_and_short():
    """HBM-resident pipelined batches; short segments of the same resources
    (k_decide_x's lanes) beside long ones, and heavy_min 512."""
    R = 20_000
    hb = trace.with_origins(trace.mixed_zipf(R, 600_000, duration_ms=3000, seed=55), n_origins=32, seed=56)
    per_res = np.bincount(hb.res_id, minlength=R)
    rules, busy = _origin_rules(R, per_res, 55)
    xres = np.argsort(-per_res)[200:260]                      # mid-size: 256-event segments come and go
    for r in xres:
        rules.append(abi.sf_flow_rule(resource=int(r), grade=abi.GRADE_QPS, count=4.0, strategy=0,
                                      control_behavior=0, limit_app=abi.APP_OTHER))
    batches = [hb.subset(0, 300_000), hb.subset(300_000, hb.n)]
    cfg = abi.default_config(max_resources=R, max_batch=300_000, heavy_min_events=512)
    pairs = _sample_pairs(hb, k_busy=40, k_rand=300, seed=57)
    _run(rules, batches, cfg, pairs, np.concatenate([busy, xres]), async_dev=True)
