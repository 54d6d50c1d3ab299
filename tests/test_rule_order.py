"""Rule-list order of the reference's managers.

FlowRuleUtil.buildFlowRuleMap (FlowRuleUtil.java:83-130) keeps a resource's
rules in HashSet iteration order, then sorts them stably with
FlowRuleComparator; ParamFlowRuleUtil.buildParamRuleMap
(ParamFlowRuleUtil.java:138-186) keeps the HashSet order.  The product helper
(sf_flow_rule_order / sf_param_rule_order, sentinel_amd/csrc/sf_rules.cpp)
is checked against oracle/rule_order.py, which is pinned by the reference's
FlowRuleComparatorTest and by well-known answers of java.lang.String.hashCode
and java.util.HashSet (JDK 8) iteration order.  Host only: no GPU.
"""
import random

import pytest

from oracle import rule_order as ro
from sentinel_amd import abi, engine

DEFAULT, OTHER = "default", "other"


def _key(resource, limit_app=DEFAULT, extra=None, cluster_hash=0, origins=None):
    """sf_rule_key from Java strings (origins: name -> id > 1)."""
    if limit_app in ("", None, DEFAULT):
        app_id, app_hash = 0, ro.java_string_hash(DEFAULT)
    elif limit_app == OTHER:
        app_id, app_hash = 1, ro.java_string_hash(OTHER)
    else:
        app_id = origins.setdefault(limit_app, 2 + len(origins)) if origins is not None else 2
        app_hash = ro.java_string_hash(limit_app)
    extra_hash = ro.java_string_hash(extra) if isinstance(extra, str) else (extra or 0)
    return (ro.java_string_hash(resource), app_id, app_hash, extra_hash, cluster_hash)


def _abi_key(k):
    return abi.sf_rule_key(*k)


def _flow(resource=0, count=10.0, grade=1, behavior=0, strategy=0, cluster=0, warm=10, queue=500, ref=0):
    return abi.sf_flow_rule(resource=resource, grade=grade, count=count, strategy=strategy,
                            control_behavior=behavior, warm_up_period_sec=warm, max_queueing_time_ms=queue,
                            cluster_mode=cluster, ref_resource=ref)


# ------------------------------------------------------------ oracle pins
def test_java_string_hash_known_answers():
    assert ro.java_string_hash("") == 0
    assert ro.java_string_hash("abc") == 96354
    assert ro.java_string_hash("hello") == 99162322
    assert ro.java_string_hash("Aa") == ro.java_string_hash("BB") == 2112
    assert ro.java_string_hash("polygenelubricants") == -2147483648      # the classic Integer.MIN_VALUE hash


def test_double_bits_known_answers():
    assert ro.double_bits(1.0) == 0x3FF0000000000000
    assert ro.double_bits(-0.0) == -0x8000000000000000
    assert ro.double_bits(float("nan")) == 0x7FF8000000000000
    # Double.hashCode(10.0) == 1076101120
    t = ro.double_bits(10.0)
    assert ro.i32(t ^ (t >> 32)) == 1076101120


def test_hashset_order_known_answers():
    # Integer keys hash to themselves: small ones iterate ascending
    assert ro.hashset_order([5, 3, 9, 1]) == [3, 1, 0, 2]
    # same bucket keeps insertion order: 33 and 17 share bucket 1 of 16
    assert ro.hashset_order([100, 5, 33, 17]) == [2, 3, 0, 1]
    # a 13th element passes 0.75 x 16 and doubles the table: 16 leaves bucket 0
    keys = [16] + list(range(12))
    assert [keys[i] for i in ro.hashset_order(keys)] == list(range(12)) + [16]
    # 12 elements stay in 16 buckets: 16 shares bucket 0 with 0 and came first
    keys = [16] + list(range(11))
    assert [keys[i] for i in ro.hashset_order(keys)] == [16, 0] + list(range(1, 11))
    # a 9th entry in one bin of a table under 64 doubles it (treeifyBin -> resize)
    keys = [16 * k for k in range(9)]
    assert [keys[i] for i in ro.hashset_order(keys)] == [0, 32, 64, 96, 128, 16, 48, 80, 112]
    keys = [16 * k for k in range(8)]
    assert [keys[i] for i in ro.hashset_order(keys)] == keys
    # high bits are folded in: 0x10000 lands in bucket 1, after 0 and before 2
    assert ro.hashset_order([2, 0x10000, 0]) == [2, 1, 0]
    with pytest.raises(NotImplementedError):
        ro.hashset_order([64 * k for k in range(9)])               # would treeify at 64 buckets


def test_flow_rule_comparator_reference_case():
    """FlowRuleComparatorTest.testFlowRuleComparator: B, C, D, A, E."""
    origins = {}
    rules = [_flow(count=10), _flow(), _flow(), _flow(), _flow(count=20)]
    apps = [DEFAULT, "originA", "originB", OTHER, DEFAULT]
    keys = [_key("abc", a, origins=origins) for a in apps]
    order = ro._stable_sort(list(range(5)), lambda a, b: ro.flow_comparator(rules[a], keys[a], rules[b], keys[b]))
    assert order == [1, 2, 3, 0, 4]


# ------------------------------------------------------------ product vs oracle
def _orders(rules, keys):
    got = engine.flow_rule_order(rules, [_abi_key(k) for k in keys]).tolist()
    assert got == ro.flow_rule_order(rules, keys)
    return got


def test_product_reference_comparator_rules():
    """The same five rules through HashSet + sort: origins first, then
    "default" ones; the product and the oracle agree on the whole order."""
    origins = {}
    rules = [_flow(count=10), _flow(), _flow(), _flow(), _flow(count=20)]
    keys = [_key("abc", a, origins=origins) for a in [DEFAULT, "originA", "originB", OTHER, DEFAULT]]
    got = _orders(rules, keys)
    assert sorted(got[:3]) == [1, 2, 3] and sorted(got[3:]) == [0, 4]


def test_product_drops_equal_and_invalid_rules():
    rules = [_flow(count=5), _flow(count=5), _flow(count=-1), _flow(behavior=2, queue=0), _flow(count=5, grade=0),
             _flow(grade=7), _flow(count=float("nan"))]
    keys = [_key("r")] * len(rules)
    got = _orders(rules, keys)
    assert sorted(got) == [0, 4]                     # 1 equals 0; 2, 3, 5, 6 invalid
    # equal except limitApp: both kept
    rules = [_flow(count=5), _flow(count=5)]
    got = _orders(rules, [_key("r"), _key("r", "app")])
    assert got == [1, 0]


def test_product_cluster_rules_last():
    rules = [_flow(cluster=1, count=1), _flow(count=2), _flow(cluster=1, count=3), _flow(count=4)]
    keys = [_key("r", cluster_hash=77 if r.cluster_mode else 0) for r in rules]
    got = _orders(rules, keys)
    assert sorted(got[:2]) == [1, 3] and sorted(got[2:]) == [0, 2]


def test_product_resources_in_first_appearance_order():
    rules = [_flow(resource=2, count=1), _flow(resource=1, count=1), _flow(resource=2, count=2)]
    keys = [_key("b"), _key("a"), _key("b")]
    got = _orders(rules, keys)
    assert got[2] == 1 and sorted(got[:2]) == [0, 2]


def test_product_empty():
    assert engine.flow_rule_order([], []).tolist() == []
    assert engine.param_rule_order([], []).tolist() == []


@pytest.mark.parametrize("seed", range(12))
def test_product_random_flow_rules(seed):
    rng = random.Random(seed)
    origins = {}
    names = ["res-%d" % k for k in range(rng.randint(1, 4))]
    rules, keys = [], []
    for _ in range(rng.randint(1, 40)):
        ri = rng.randrange(len(names))
        app = rng.choice([DEFAULT, OTHER, "appA", "appB", "", "appC"])
        beh = rng.choice([0, 0, 1, 2, 3])
        r = _flow(resource=ri, count=float(rng.choice([1, 2, 5, 10, -1])), grade=rng.choice([1, 1, 0]),
                  behavior=beh, cluster=1 if rng.random() < 0.2 else 0, warm=rng.choice([0, 10]),
                  queue=rng.choice([0, 500]))
        rules.append(r)
        keys.append(_key(names[ri], app, origins=origins, cluster_hash=9 if r.cluster_mode else 0))
    _orders(rules, keys)


def _param(resource=0, count=5.0, idx=0, grade=1, behavior=0, burst=0, dur=1, queue=0, off=0, nitems=0):
    return abi.sf_param_rule(resource=resource, grade=grade, param_idx=idx, control_behavior=behavior, count=count,
                             max_queueing_time_ms=queue, burst_count=burst, duration_in_sec=dur,
                             item_offset=off, item_count=nitems)


@pytest.mark.parametrize("seed", range(12))
def test_product_random_param_rules(seed):
    rng = random.Random(100 + seed)
    items = [abi.sf_hot_item(tag=abi.TAG_INT if hasattr(abi, "TAG_INT") else 1, count=rng.randint(0, 9),
                             bits=rng.randint(0, 3)) for _ in range(6)]
    rules, keys = [], []
    for _ in range(rng.randint(1, 40)):
        ri = rng.randrange(3)
        off = rng.randrange(4)
        n_it = rng.choice([0, 0, 1, 2])
        r = _param(resource=ri, count=float(rng.choice([0, 1, 5, -1])), idx=rng.choice([0, 1, -1]),
                   grade=rng.choice([1, 1, 0]), behavior=rng.choice([0, 2]), burst=rng.choice([0, 3, -1]),
                   dur=rng.choice([1, 2, 0]), queue=rng.choice([0, 100]), off=off, nitems=n_it)
        rules.append(r)
        # paramFlowItemList.hashCode() is the caller's; any value is fine as long as equal lists agree
        ih = hash(tuple((items[off + t].bits, items[off + t].count) for t in range(n_it))) & 0x7FFFFFFF
        keys.append(_key("p%d" % ri, rng.choice([DEFAULT, "x"]), extra=ih))
    got = engine.param_rule_order(rules, [_abi_key(k) for k in keys], items).tolist()
    assert got == ro.param_rule_order(rules, keys, items)


def test_param_rule_order_is_hashset_order_unsorted():
    # limitApp is not sorted for param rules: only the HashSet order counts
    rules = [_param(count=float(c)) for c in (1, 2, 3, 4, 5)]
    keys = [_key("r", a) for a in (DEFAULT, "a", DEFAULT, OTHER, "b")]
    got = engine.param_rule_order(rules, [_abi_key(k) for k in keys]).tolist()
    want = ro.hashset_order([ro.param_rule_hash(r, k) for r, k in zip(rules, keys)])
    assert got == want


def test_product_refuses_treeified_bin():
    # >8 rules of one resource in one bin of a 64-slot table: not modelled
    base = _key("r")
    rules, keys = [], []
    # find 9 rule counts whose hashes share a bucket of 64 slots
    buckets = {}
    c = 0
    while True:
        r = _flow(count=float(c))
        h = ro.flow_rule_hash(r, base) & 0xFFFFFFFF
        b = (h ^ (h >> 16)) & 63
        buckets.setdefault(b, []).append(r)
        if len(buckets[b]) == 9:
            rules = buckets[b]
            break
        c += 1
    keys = [base] * 9
    with pytest.raises(RuntimeError):
        engine.flow_rule_order(rules, [_abi_key(k) for k in keys])
    with pytest.raises(NotImplementedError):
        ro.flow_rule_order(rules, keys)
