"""Whole-engine state comparison (include/sentinel_flow.h sf_node_digests /
sf_read_rule_states; oracle so_node_digests / so_read_rule_states): the
oracle's per-row digest is FNV-1a 64 over the canonical sf_node_state words in
the header's order (restated here in Python from so_read_node), the bulk rule
states equal the per-rule reads; on the GPU the engine's digests equal the
oracle's for every row after a multi-batch config-3 run (workloads.run checks
the same on every GPU workload)."""
import numpy as np
import pytest

from sentinel_amd import abi
from tests import workloads

MASK = (1 << 64) - 1


def py_digest(st, S):
    h = 0xcbf29ce484222325
    def w(x):
        nonlocal h
        h ^= x & MASK
        h = (h * 0x100000001b3) & MASK
    d = abi.node_state_to_dict(st, S)
    for i in range(S):
        for x in d["second"][i]:
            w(x)
        w(d["borrow"][i][0]); w(d["borrow"][i][1])
    for b in d["minute"]:
        for x in b:
            w(x)
    w(d["threads"])
    return h


def _oracle_run(so, w):
    ora = so.OracleEngine(w["cfg"])
    ora.load_flow_rules(list(w["flow"]))
    for b in w["batches"]:
        ora.submit(b)
    return ora


def test_oracle_digest_is_the_header_fnv(so):
    w = workloads.config3(R=2000, n=40_000, seed=5, split=2)
    ora = _oracle_run(so, w)
    R = w["cfg"].max_resources
    dig = ora.node_digests(R)
    S = w["cfg"].sample_count
    rows = list(w["nodes"][:40]) + [R - 1]
    for r in rows:
        assert int(dig[r]) == py_digest(ora.read_node(int(r)), S), r
    assert np.unique(dig).size > 100                     # touched rows differ
    ora.close()


def test_oracle_bulk_rule_states(so):
    w = workloads.config3(R=500, n=20_000, seed=6, split=1)
    ora = _oracle_run(so, w)
    n = w["n_flow"]
    bulk = ora.rule_states(0, n)
    for k in range(0, n, 7):
        s = ora.read_rule_state(k)
        assert tuple(bulk[k]) == (s.stored_tokens, s.last_filled_time, s.latest_passed_time)
    ora.close()


@pytest.mark.gpu
def test_gpu_digests_every_row(so):
    from sentinel_amd import engine
    w = workloads.config3(R=30_000, n=400_000, seed=21, split=4)
    eng, ora, _ = workloads.run(engine.FlowEngine, so.OracleEngine, w)
    R = w["cfg"].max_resources
    a, b = eng.node_digests(R), ora.node_digests(R)
    assert np.array_equal(a, b)
    assert np.unique(a).size > 1000
    # one changed row changes its digest only
    S = w["cfg"].sample_count
    r = int(w["nodes"][0])
    assert int(a[r]) == py_digest(eng.read_node(r), S)
    eng.close(); ora.close()
