"""GPU parity of the token-server wire path (sf_serve_frames) against the
oracle's restatement of the reference server pipeline (so_serve_frames):
response bytes, per-connection response ranges, consumed prefixes and stop
reasons byte for byte, then every ClusterMetric counter.  Run with -m gpu."""
import numpy as np
import pytest

from oracle import oracle as so
from sentinel_amd import abi, trace, wire

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng_mod():
    from sentinel_amd import engine
    engine.lib()
    return engine


def pair(eng_mod, ns, flow, param, items):
    cfg = abi.default_config(max_resources=4, max_batch=1 << 16, param_capacity=1 << 18)
    e, o = eng_mod.FlowEngine(cfg), so.OracleEngine(cfg)
    for x in (e, o):
        x.load_namespaces(ns)
        x.load_cluster_rules(flow, param, items)
    return e, o


def compare(got, want, what):
    assert (got.n_frames, got.n_requests, got.n_responses) == (want.n_frames, want.n_requests, want.n_responses), what
    assert np.array_equal(got.stop, want.stop), what
    assert np.array_equal(got.consumed, want.consumed), what
    assert np.array_equal(got.resp_off, want.resp_off), what
    if not np.array_equal(got.resp, want.resp):
        g, w = wire.decode_responses(got.resp), wire.decode_responses(want.resp)
        i = int(np.nonzero(g != w)[0][0])
        raise AssertionError(f"{what}: response {i} differs: engine {g[i]} oracle {w[i]}")


def compare_metrics(e, o, flow, now):
    for r in flow[:: max(1, len(flow) // 50)]:
        for ev in range(7):
            assert e.cluster_sum(r.flow_id, ev, now) == o.cluster_sum(r.flow_id, ev, now)


def test_wire_parity_500_connections(eng_mod):
    ns, flow, param, items, streams = trace.wire_workload(60000, n_streams=500, seed=31)
    e, o = pair(eng_mod, ns, flow, param, items)
    now = trace.T0 + 700
    compare(e.serve_frames(streams, now), o.serve_frames(streams, now), "500 connections")
    compare_metrics(e, o, flow, now)


def test_wire_parity_edge_frames_and_carry_over(eng_mod):
    """Edge frames, and each connection's bytes cut at arbitrary points over 3 calls
    (incomplete frames carried into the next call, as the host's socket buffers would)."""
    ns, flow, param, items, streams = trace.wire_workload(40000, n_streams=300, edge=True, seed=32)
    e, o = pair(eng_mod, ns, flow, param, items)
    rng = np.random.default_rng(5)
    cuts = [np.sort(rng.integers(0, len(s) + 1, 2)) for s in streams]
    parts = [[s[: c[0]], s[c[0]: c[1]], s[c[1]:]] for s, c in zip(streams, cuts)]
    carry = [b""] * len(streams)
    stopped = [False] * len(streams)
    for k in range(3):
        ins = [b"" if stopped[s] else carry[s] + parts[s][k] for s in range(len(streams))]
        now = trace.T0 + 400 * k
        got, want = e.serve_frames(ins, now), o.serve_frames(ins, now)
        compare(got, want, f"call {k}")
        for s in range(len(streams)):
            carry[s] = ins[s][int(want.consumed[s]):]
            stopped[s] = stopped[s] or want.stop[s] == abi.WIRE_HOST
    compare_metrics(e, o, flow, trace.T0 + 800)


def test_wire_parity_one_long_connection(eng_mod):
    """One connection over many framing tiles (the tile-exit chain), with too-long frames
    that jump across tiles."""
    ns, flow, param, items, streams = trace.wire_workload(120000, n_streams=1, edge=True, seed=33)
    assert len(streams[0]) > 40 * 16384
    e, o = pair(eng_mod, ns, flow, param, items)
    now = trace.T0 + 999
    compare(e.serve_frames(streams, now), o.serve_frames(streams, now), "one connection")
    compare_metrics(e, o, flow, now)


def test_wire_parity_many_tiny_and_empty_connections(eng_mod):
    """Many connections per framing tile, some empty."""
    ns, flow, param, items, streams = trace.wire_workload(30000, n_streams=20000, edge=True, seed=34)
    streams = [s if i % 7 else b"" for i, s in enumerate(streams)]
    e, o = pair(eng_mod, ns, flow, param, items)
    now = trace.T0 + 50
    compare(e.serve_frames(streams, now), o.serve_frames(streams, now), "tiny connections")
    compare(e.serve_frames([b""] * 3, now), o.serve_frames([b""] * 3, now), "empty")


def test_multi_value_param_frames(eng_mod):
    """PARAM_FLOW frames with several parameters are one Collection each
    (decided on the GPU, not handed to the host): byte-exact with the oracle."""
    ns, flow, param, items, b = trace.token_workload(8000, seed=17, n_values=50)
    rng = np.random.default_rng(4)
    streams = [bytearray() for _ in range(20)]
    for i in range(b.n):
        s = int(rng.integers(0, 20))
        if b.flags[i] & abi.TOK_PARAM:
            k = int(rng.integers(1, 5))
            vs = [("long", int(x)) if rng.random() < 0.7 else ("str", "v%d" % int(x)) for x in rng.integers(0, 50, k)]
            streams[s] += wire.param_frame(i, int(b.flow_id[i]), int(b.count[i]), vs)
        else:
            streams[s] += wire.flow_frame(i, int(b.flow_id[i]), int(b.count[i]), bool(b.flags[i] & abi.TOK_PRIORITIZED))
    streams = [bytes(x) for x in streams]
    e, o = pair(eng_mod, ns, flow, param, items)
    for k in range(2):
        now = trace.T0 + 300 * k
        compare(e.serve_frames(streams, now), o.serve_frames(streams, now), f"call {k}")
