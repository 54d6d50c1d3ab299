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
