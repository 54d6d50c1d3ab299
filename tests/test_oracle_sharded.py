"""The resource-sharded multi-core oracle replay (oracle/sharded.py, the
bench's multi-core CPU baseline) equals one replay of the whole batch."""
import pytest

from oracle import oracle as so
from oracle import sharded
from sentinel_amd import abi, trace


@pytest.mark.parametrize("T", [1, 3, 8])
def test_sharded_replay_equals_single(T):
    R = 3000
    rules = trace.mixed_rules(R, seed=5)
    hb = trace.mixed_zipf(R, 60_000, duration_ms=2000, seed=5)
    o = so.OracleEngine(abi.default_config(max_resources=R, max_batch=hb.n))
    o.load_flow_rules(rules)
    want = o.submit(hb)
    o.close()
    got, dt = sharded.replay(rules, hb, R, T)
    assert (got.status == want.status).all()
    assert (got.wait_ms == want.wait_ms).all()
    assert (got.rule_idx == want.rule_idx).all()
    assert dt > 0


def test_sharded_whole_state_equals_one_engine():
    """bench.py's steady-state check compares every node and rule state through
    ShardedOracle.node_digests / rule_states: the shards' rows, put back in
    resource order, equal one oracle's."""
    import numpy as np
    from oracle import oracle as so, sharded
    from sentinel_amd import abi, trace
    R = 3000
    rules = trace.mixed_rules(R, seed=3)
    hb = trace.mixed_zipf(R, 50_000, duration_ms=4000, seed=3)
    sh = sharded.ShardedOracle(rules, R, 4, hb.n)
    sh.submit(hb)
    one = so.OracleEngine(abi.default_config(max_resources=R, max_batch=hb.n))
    one.load_flow_rules(rules)
    one.submit(hb)
    assert np.array_equal(sh.node_digests(R), one.node_digests(R))
    assert np.array_equal(sh.rule_states(R), one.rule_states(0, R))
    one.close(); sh.close()
