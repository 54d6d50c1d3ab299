"""Token-server wire path on the CPU: the client codec helpers against the
reference codec tests (known answers), and the oracle's frame pipeline
(oracle.so_serve_frames) against its own token service on the same requests.
The GPU path (sf_serve_frames) is compared with this oracle in
tests/test_gpu_wire.py."""
import struct

import numpy as np
import pytest

from oracle import oracle as so
from sentinel_amd import abi, trace, wire


def test_param_transport_size_kat():
    # ParamFlowRequestDataWriterTest.testCalculateParamTransportSize (CC_T/codec/data/...:16-28)
    assert wire.param_transport_size(object()) == 0
    assert wire.param_transport_size(("int", 1)) == 4 + 1
    assert wire.param_transport_size(("byte", 1)) == 1 + 1
    assert wire.param_transport_size(("bool", False)) == 1 + 1
    assert wire.param_transport_size(("long", 2)) == 8 + 1
    assert wire.param_transport_size(("double", 4.0)) == 8 + 1
    assert wire.param_transport_size(("str", "Sentinel")) == 1 + 4 + len(b"Sentinel")


def test_resolve_valid_params_kat():
    # ParamFlowRequestDataWriterTest.testResolveValidParams (:31-55), maxSize 15
    ps = [("int", 1), ("int", 64), ("int", 3)]
    assert wire.resolve_valid_params(ps, 15) == ps
    assert ("int", 5) not in wire.resolve_valid_params(ps + [("int", 5)], 15)
    assert wire.resolve_valid_params([object()], 15) == []


def test_flow_response_layout_kat():
    # FlowResponseDataDecoderTest (CC_T/codec/data/FlowResponseDataDecoderTest.java:26-35): remaining 12, wait 13
    buf = struct.pack(">HibbIi", 14, 7, 1, 0, 12, 13)
    a = wire.decode_responses(buf)
    assert (a["xid"][0], a["type"][0], a["status"][0], a["remaining"][0], a["wait"][0]) == (7, 1, 0, 12, 13)


def test_string_key_matches_oracle():
    for s in [b"", b"a", b"Sentinel", "热点".encode()]:
        assert so.lib().so_string_key(s, len(s)) == wire.string_key(s)


def _oracle(ns, flow, param, items, max_batch=1 << 16):
    o = so.OracleEngine(abi.default_config(max_resources=4, max_batch=max_batch, param_capacity=1 << 16))
    o.load_namespaces(ns)
    o.load_cluster_rules(flow, param, items)
    return o


def test_wire_equals_token_service():
    """Frames decoded by the oracle == the same requests given to so_request_tokens."""
    n = 3000
    ns, flow, param, items, b = trace.token_workload(n, seed=21, bad_frac=0.0)
    now = trace.T0 + 1500
    tag = np.where(b.param_tag == abi.TAG_NULL, abi.TAG_LONG, b.param_tag).astype(np.uint8)
    frames = []
    for i in range(n):
        if b.flags[i] & abi.TOK_PARAM:
            v = int(b.param_bits[i]); v = v - (1 << 64) if v >= 1 << 63 else v
            frames.append(wire.param_frame(i, int(b.flow_id[i]), int(b.count[i]), [("long", v)]))
        else:
            frames.append(wire.flow_frame(i, int(b.flow_id[i]), int(b.count[i]), bool(b.flags[i] & abi.TOK_PRIORITIZED)))
    r = _oracle(ns, flow, param, items).serve_frames([b"".join(frames)], now)
    want = _oracle(ns, flow, param, items).request_tokens(abi.HostTokenBatch(
        b.flow_id, b.count, b.flags, np.full(n, now, np.int64), param_tag=tag, param_bits=b.param_bits))
    a = wire.decode_responses(r.resp)
    assert r.n_requests == n and r.n_responses == n and r.stop[0] == abi.WIRE_DONE
    assert (a["xid"] == np.arange(n)).all()
    assert (a["status"] == want.status).all()
    assert (a["remaining"] == want.remaining).all()
    is_param = (b.flags & abi.TOK_PARAM) != 0
    assert (a["wait"] == np.where(is_param, 0, want.wait_ms)).all()   # ParamFlowRequestProcessor: waitInMs 0


def test_wire_frame_edge_cases():
    """Reference decoder outcomes frame by frame (DefaultRequestEntityDecoder, the data decoders,
    the processors' null-data NPE, LengthFieldBasedFrameDecoder's 1024-byte cap)."""
    ns, flow, param, items, _ = trace.token_workload(10, seed=3)
    o = _oracle(ns, flow, param, items)
    now = trace.T0
    p = flow[0].flow_id
    pp = param[0].flow_id
    cases = [
        (wire.frame(b""), 0, abi.WIRE_DONE),                                        # nothing readable
        (wire.frame(struct.pack(">ib", 5, 1)), 0, abi.WIRE_DONE),                   # FLOW, no data: NPE, no response
        (wire.frame(struct.pack(">ib", 5, 9)), 0, abi.WIRE_DONE),                   # no decoder, nothing left
        (wire.frame(struct.pack(">ibqi", 5, 1, p, 1)), 1, abi.WIRE_DONE),           # no priority byte
        (struct.pack(">H", 1023) + bytes(1023), 0, abi.WIRE_DONE),                  # 1025 > 1024: skipped
        (wire.frame(struct.pack(">ibqii", 5, 2, pp, 1, 0)), 0, abi.WIRE_DONE),      # amount 0: null data
        (wire.frame(struct.pack(">ibqii", 5, 2, pp, 1, 1) + bytes([42])), 1, abi.WIRE_DONE),  # unknown tag: empty -> BAD
        (wire.frame(struct.pack(">ib", 5, 0) + b"\0\0\0\1x"), 0, abi.WIRE_HOST),    # PING
        (wire.param_frame(5, pp, 1, [("long", 1), ("int", 2)]), 1, abi.WIRE_DONE),  # two values: one Collection
        (wire.frame(struct.pack(">ibqi", 5, 1, p, 1) + b"\0\0"), 0, abi.WIRE_HOST), # bytes left over
        (wire.frame(b"\0\0\0"), 0, abi.WIRE_HOST),                                  # < 5 bytes
        (wire.flow_frame(5, p, 1)[:7], 0, abi.WIRE_PARTIAL),                        # incomplete
    ]
    for fr, n_resp, stop in cases:
        r = o.serve_frames([fr], now)
        assert (r.n_responses, int(r.stop[0])) == (n_resp, stop), fr
        assert int(r.consumed[0]) == (0 if stop != abi.WIRE_DONE else len(fr))
    r = o.serve_frames([wire.frame(struct.pack(">ibqii", 5, 2, pp, 1, 1) + bytes([42]))], now)
    assert wire.decode_responses(r.resp)["status"][0] == abi.TOKEN_BAD_REQUEST


def test_cluster_param_collection_semantics():
    """ClusterParamFlowChecker.acquireClusterToken (:42-87) over a Collection:
    every value must have room or nothing is added; remaining is -1 for more
    than one value; a null value counts 0 and is never added; an empty
    collection is BAD_REQUEST (DefaultTokenService.java:53-56)."""
    ns = [abi.sf_namespace(namespace_id=1, connected_count=1, max_allowed_qps=-1.0)]
    param = [abi.sf_cluster_param_rule(flow_id=7, count=2.0, threshold_type=abi.THRESHOLD_GLOBAL, namespace_id=1,
                                       sample_count=10, window_interval_ms=1000, item_offset=0, item_count=0)]
    o = _oracle(ns, [], param, [])
    L = abi.TAG_LONG
    reqs = [[(L, 1), (L, 2)], [(L, 1)], [(L, 1), (L, 3)], [(L, 3)], [(L, 3)], [(abi.TAG_NULL, 0), (L, 4)], []]
    off = np.concatenate([[0], np.cumsum([len(r) for r in reqs])]).astype(np.uint32)
    tags = np.array([t for r in reqs for t, _ in r], np.uint8)
    bits = np.array([b for r in reqs for _, b in r], np.uint64)
    n = len(reqs)
    b = abi.HostTokenBatch(np.full(n, 7), np.ones(n), np.full(n, abi.TOK_PARAM), np.full(n, trace.T0),
                           param_tag=tags, param_bits=bits, param_off=off)
    r = o.request_tokens(b)
    OK, BL, BAD = abi.TOKEN_OK, abi.TOKEN_BLOCKED, abi.TOKEN_BAD_REQUEST
    assert list(r.status) == [OK, OK, BL, OK, OK, OK, BAD]
    assert list(r.remaining) == [-1, 0, 0, 1, 0, -1, 0]    # [1,3] blocked at 1: 3 not added (room 1 after)


def test_wire_multi_value_frames_match_token_service():
    """PARAM_FLOW frames with several parameters (one Collection) give the
    decisions of requestParamToken with those values, in frame order."""
    ns, flow, param, items, b = trace.token_workload(3000, seed=13)
    rng = np.random.default_rng(5)
    now = trace.T0 + 100
    frames, vals = [], []
    for i in range(b.n):
        if b.flags[i] & abi.TOK_PARAM:
            k = int(rng.integers(1, 4))
            v = [int(x) for x in rng.integers(0, 40, k)]
            vals.append(v)
            frames.append(wire.param_frame(i, int(b.flow_id[i]), int(b.count[i]), [("long", x) for x in v]))
        else:
            vals.append([])
            frames.append(wire.flow_frame(i, int(b.flow_id[i]), int(b.count[i]), bool(b.flags[i] & abi.TOK_PRIORITIZED)))
    r = _oracle(ns, flow, param, items).serve_frames([b"".join(frames)], now)
    off = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint32)
    allv = np.array([x for v in vals for x in v], np.uint64)
    want = _oracle(ns, flow, param, items).request_tokens(abi.HostTokenBatch(
        b.flow_id, b.count, b.flags, np.full(b.n, now, np.int64), param_tag=np.full(allv.size, abi.TAG_LONG, np.uint8),
        param_bits=allv, param_off=off))
    a = wire.decode_responses(r.resp)
    assert r.stop[0] == abi.WIRE_DONE and r.n_responses == b.n
    assert (a["status"] == want.status).all() and (a["remaining"] == want.remaining).all()
    multi = np.array([len(v) > 1 for v in vals])
    assert multi.sum() > 100 and (a["remaining"][multi & (a["status"] == abi.TOKEN_OK)] == -1).all()


def test_wire_streams_stop_independently():
    ns, flow, param, items, streams = trace.wire_workload(4000, n_streams=40, edge=True, seed=8)
    r = _oracle(ns, flow, param, items).serve_frames(streams, trace.T0 + 10)
    for s, x in enumerate(streams):
        c = int(r.consumed[s])
        assert c <= len(x)
        assert (c == len(x)) == (r.stop[s] == abi.WIRE_DONE)
    assert r.resp_off[-1] == r.n_responses * 16
