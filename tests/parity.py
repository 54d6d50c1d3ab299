"""Shared parity helpers: run one workload through an engine and the oracle and
compare verdicts, waits, rule indices, per-resource node state and controller
state bit for bit."""
import numpy as np

from sentinel_amd import abi


def compare_verdicts(a: abi.HostVerdicts, b: abi.HostVerdicts, what=""):
    bad = np.nonzero((a.status != b.status) | (a.wait_ms != b.wait_ms) | (a.rule_idx != b.rule_idx))[0]
    if bad.size:
        i = bad[0]
        raise AssertionError(f"{what}: {bad.size} verdicts differ; first at {i}: "
                             f"engine=({a.status[i]},{a.wait_ms[i]},{a.rule_idx[i]}) "
                             f"oracle=({b.status[i]},{b.wait_ms[i]},{b.rule_idx[i]})")


def compare_nodes(eng, ora, resources, sample_count=2, what=""):
    for r in resources:
        x = abi.node_state_to_dict(eng.read_node(int(r)), sample_count)
        y = abi.node_state_to_dict(ora.read_node(int(r)), sample_count)
        if x != y:
            for k in x:
                if x[k] != y[k]:
                    raise AssertionError(f"{what}: node {r} field {k} differs:\n engine={x[k]}\n oracle={y[k]}")


def compare_rule_states(eng, ora, n_rules, what=""):
    for k in range(n_rules):
        a, b = eng.read_rule_state(k), ora.read_rule_state(k)
        ta = (a.stored_tokens, a.last_filled_time, a.latest_passed_time)
        tb = (b.stored_tokens, b.last_filled_time, b.latest_passed_time)
        assert ta == tb, f"{what}: rule {k} state engine={ta} oracle={tb}"


def compare_all_nodes(eng, ora, n_rows, sample_count=2, what=""):
    """Every row at once: the engine's per-row digests (sf_node_digests, on the
    device) against the oracle's (so_node_digests); a differing row is then
    compared field by field."""
    a, b = eng.node_digests(n_rows), ora.node_digests(n_rows)
    bad = np.nonzero(a != b)[0]
    if bad.size:
        compare_nodes(eng, ora, bad[:4], sample_count, what)
        raise AssertionError(f"{what}: {bad.size} node digests differ (first rows {bad[:8].tolist()})")


def compare_all_rule_states(eng, ora, n_rules, what=""):
    a, b = eng.rule_states(0, n_rules), ora.rule_states(0, n_rules)
    bad = np.nonzero((a != b).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} rule states differ; first {bad[0]}: engine={a[bad[0]]} oracle={b[bad[0]]}"


def run_both(make_engine, make_oracle, cfg, flow_rules=(), param_rules=(), items=(), batches=(), system=(),
             status=None):
    eng, ora = make_engine(cfg), make_oracle(cfg)
    if status is not None:
        eng.set_system_status(*status)
        ora.set_system_status(*status)
    if system:
        eng.load_system_rules(list(system))
        ora.load_system_rules(list(system))
    if flow_rules:
        eng.load_flow_rules(list(flow_rules))
        ora.load_flow_rules(list(flow_rules))
    if param_rules:
        eng.load_param_rules(list(param_rules), list(items))
        ora.load_param_rules(list(param_rules), list(items))
    outs = []
    for b in batches:
        outs.append((eng.submit(b), ora.submit(b)))
    return eng, ora, outs


def compare_entry_node(eng, ora, sample_count=2, what=""):
    x = abi.node_state_to_dict(eng.read_entry_node(), sample_count)
    y = abi.node_state_to_dict(ora.read_entry_node(), sample_count)
    for k in x:
        if x[k] != y[k]:
            raise AssertionError(f"{what}: ENTRY_NODE field {k} differs:\n engine={x[k]}\n oracle={y[k]}")


def metric_rows(rows):
    return sorted((r.resource, r.timestamp, r.pass_qps, r.block_qps, r.success_qps, r.exception_qps, r.rt,
                   r.occupied_pass_qps) for r in rows)


def compare_aux_nodes(eng, ora, origin_nodes=(), context_nodes=(), sample_count=2, what=""):
    """Origin nodes (res, origin) and context DefaultNodes (context, res) kept for the rules."""
    for r, o in origin_nodes:
        x = abi.node_state_to_dict(eng.read_origin_node(r, o), sample_count)
        y = abi.node_state_to_dict(ora.read_origin_node(r, o), sample_count)
        assert x == y, f"{what}: origin node ({r}, {o}) differs:\n engine={x}\n oracle={y}"
    for c, r in context_nodes:
        x = abi.node_state_to_dict(eng.read_context_node(c, r), sample_count)
        y = abi.node_state_to_dict(ora.read_context_node(c, r), sample_count)
        assert x == y, f"{what}: context node ({c}, {r}) differs:\n engine={x}\n oracle={y}"
