"""GPU parity of the batched cluster token server (sf_request_tokens) against
the oracle's DefaultTokenService replay: TokenResult status, remaining and
waitInMs per request, and every ClusterMetric counter afterwards, bit for bit.
Run with -m gpu on an MI355X."""
import numpy as np
import pytest

from sentinel_amd import abi, trace

pytestmark = pytest.mark.gpu

EVENTS = range(7)   # ClusterFlowEvent ordinals


@pytest.fixture(scope="module")
def eng_mod():
    from sentinel_amd import engine
    engine.lib()
    return engine


def compare_tokens(got, want, what=""):
    bad = np.nonzero((got.status != want.status) | (got.remaining != want.remaining) | (got.wait_ms != want.wait_ms))[0]
    if bad.size:
        i = bad[0]
        raise AssertionError(f"{what}: {bad.size} token results differ; first at {i}: engine=({got.status[i]},"
                             f"{got.remaining[i]},{got.wait_ms[i]}) oracle=({want.status[i]},{want.remaining[i]},"
                             f"{want.wait_ms[i]})")


def run_tokens(eng_mod, so, n_req, split=1, seed=5, max_qps=-1.0, check_sums=True, **kw):
    ns, flow, param, items, b = trace.token_workload(n_req, seed=seed, max_qps=max_qps, **kw)
    cfg = abi.default_config(max_resources=4, max_batch=b.n, param_capacity=1 << 16)
    e = eng_mod.FlowEngine(cfg)
    o = so.OracleEngine(cfg)
    for x in (e, o):
        x.load_namespaces(ns)
        x.load_cluster_rules(flow, param, items)
    cuts = np.linspace(0, b.n, split + 1).astype(int)
    for k, (lo, hi) in enumerate(zip(cuts[:-1], cuts[1:])):
        sub = abi.HostTokenBatch(b.flow_id[lo:hi], b.count[lo:hi], b.flags[lo:hi], b.ts_ms[lo:hi],
                                 param_tag=b.param_tag[lo:hi], param_bits=b.param_bits[lo:hi])
        compare_tokens(e.request_tokens(sub), o.request_tokens(sub), f"batch {k}")
    if check_sums:
        now = int(b.ts_ms[-1])
        for f in flow:
            for ev in EVENTS:
                a, w = e.cluster_sum(f.flow_id, ev, now), o.cluster_sum(f.flow_id, ev, now)
                assert a == w, f"flowId {f.flow_id} event {ev}: engine {a} oracle {w}"
    return e, o


@pytest.mark.parametrize("split", [1, 4])
def test_token_server_parity(eng_mod, so, split):
    run_tokens(eng_mod, so, 60_000, split=split)


@pytest.mark.parametrize("max_qps", [0.0, 500.0, 3000.0])
def test_token_server_namespace_limiter(eng_mod, so, max_qps):
    """GlobalRequestLimiter at and around the offered rate (TOO_MANY_REQUEST)."""
    run_tokens(eng_mod, so, 40_000, split=3, seed=7, max_qps=max_qps)


def test_token_server_heavy_values(eng_mod, so):
    """Few values, many requests each (long per-value chains) and all prioritized."""
    run_tokens(eng_mod, so, 50_000, split=2, seed=11, n_values=5, n_flow=5, n_param=3, prio_frac=1.0)


def test_token_server_bad_requests(eng_mod, so):
    run_tokens(eng_mod, so, 5_000, seed=13, bad_frac=0.5)


@pytest.mark.parametrize("seed", [21, 22])
def test_token_server_collection_params(eng_mod, so, seed):
    """requestParamToken with Collection params (1-4 values, some null; a few
    empty -> BAD_REQUEST): rules with multi-value requests are decided per rule
    in time order (every value must have room before any is added), the rest
    per value; results and every flow rule's ClusterMetric equal the oracle's."""
    ns, flow, param, items, b = trace.token_workload(30_000, seed=seed, n_values=60)
    rng = np.random.default_rng(seed)
    vals = []
    for i in range(b.n):
        if not (b.flags[i] & abi.TOK_PARAM):
            vals.append([])
            continue
        k = int(rng.choice([0, 1, 1, 1, 2, 3, 4])) if rng.random() < 0.6 else 1
        vals.append([(abi.TAG_NULL, 0) if rng.random() < 0.03 else (abi.TAG_LONG, int(rng.integers(0, 60)))
                     for _ in range(k)])
    off = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint32)
    tags = np.array([t for v in vals for t, _ in v], np.uint8)
    bits = np.array([x for v in vals for _, x in v], np.uint64)
    cfg = abi.default_config(max_resources=4, max_batch=b.n, param_capacity=1 << 16)
    e, o = eng_mod.FlowEngine(cfg), so.OracleEngine(cfg)
    for x in (e, o):
        x.load_namespaces(ns)
        x.load_cluster_rules(flow, param, items)
    for lo, hi in ((0, b.n // 2), (b.n // 2, b.n)):
        po = off[lo:hi + 1] - off[lo]
        sub = abi.HostTokenBatch(b.flow_id[lo:hi], b.count[lo:hi], b.flags[lo:hi], b.ts_ms[lo:hi],
                                 param_tag=tags[off[lo]:off[hi]], param_bits=bits[off[lo]:off[hi]], param_off=po)
        got, want = e.request_tokens(sub), o.request_tokens(sub)
        compare_tokens(got, want, f"[{lo}, {hi})")
    assert (want.remaining == -1).sum() > 0


@pytest.mark.parametrize("shard", [0, 1])
def test_token_server_sharded(eng_mod, so, shard):
    """A token server sharded over two GPUs (sf_token_shard): this shard's
    engine decides the requests it owns exactly as one token server deciding
    every request; a request of the other shard is refused."""
    ns, flow, param, items, b = trace.token_workload(30_000, seed=34, max_qps=1500.0, n_flow=60, n_param=20)
    owner = eng_mod.token_shard(flow, param, ns, 2, b)
    sel = np.nonzero(owner == shard)[0]
    cfg = abi.default_config(max_resources=4, max_batch=b.n, param_capacity=1 << 16, shard_count=2, shard_index=shard)
    e = eng_mod.FlowEngine(cfg)
    e.load_namespaces(ns)
    e.load_cluster_rules(flow, param, items)
    ref = so.OracleEngine(abi.default_config(max_resources=4, max_batch=b.n, param_capacity=1 << 16))
    ref.load_namespaces(ns)
    ref.load_cluster_rules(flow, param, items)
    want = ref.request_tokens(b)
    got = e.request_tokens(b.take(sel))
    sub = abi.HostTokenResults(sel.size)
    sub.status, sub.remaining, sub.wait_ms = want.status[sel], want.remaining[sel], want.wait_ms[sel]
    compare_tokens(got, sub, f"shard {shard}")
    other = np.nonzero(owner != shard)[0][:5]
    with pytest.raises(eng_mod.EngineError):
        e.request_tokens(b.take(other))
