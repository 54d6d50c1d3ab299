"""Token-server wire format (C1 frames): the client-side request writer and the
response reader, for hosts that feed ``sf_serve_frames`` and for its tests.

Mirrors the reference client codec byte for byte (CC = sentinel-cluster/
sentinel-cluster-client-default/src/main/java/com/alibaba/csp/sentinel/cluster/client):
  DefaultRequestEntityWriter.java:34-52   xid:int32, type:int8, data
  FlowRequestDataWriter.java:31-36        flowId:int64, count:int32, priority:bool
  ParamFlowRequestDataWriter.java:45-150  flowId, count, n:int32, n x (tag:int8, value);
                                          resolveValidParams drops non-primitive values and
                                          stops at maxParamByteSize (1024)
  PingRequestDataWriter.java:30-37        length:int32, bytes
  NettyTransportClient.java:103-105       LengthFieldPrepender(2) (2-byte big-endian length)
and the server's response layout (DefaultResponseEntityWriter.java:48-52,
FlowResponseDataWriter.java:30-33): xid, type, status:int8, remaining:int32,
waitInMs:int32.  Parameters are (java type, value) pairs: "int", "long",
"byte", "short", "float", "double", "bool", "str".
"""
import struct

import numpy as np

MSG_TYPE_PING, MSG_TYPE_FLOW, MSG_TYPE_PARAM_FLOW = 0, 1, 2          # ClusterConstants.java:24-28
PARAM_TYPE = {"int": 0, "long": 1, "byte": 2, "double": 3, "float": 4, "short": 5, "bool": 6, "str": 7}
DEFAULT_PARAM_MAX_SIZE = 1024                                        # ParamFlowRequestDataWriter.java:148


def string_key(s) -> int:
    """sf_string_key: FNV-1a 64 of the String's bytes (the engine's key for a wire String)."""
    b = s.encode() if isinstance(s, str) else bytes(s)
    h = 0xcbf29ce484222325
    for c in b:
        h = ((h ^ c) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def param_transport_size(p) -> int:
    """ParamFlowRequestDataWriter.calculateParamTransportSize (:111-146)."""
    if p is None or not isinstance(p, tuple) or p[0] not in PARAM_TYPE:
        return 0
    kind, v = p
    if kind == "str":
        return 1 + 4 + len(v.encode() if isinstance(v, str) else v)
    return {"int": 5, "bool": 2, "long": 9, "double": 9, "float": 5, "byte": 2, "short": 3}[kind]


def resolve_valid_params(params, max_size=DEFAULT_PARAM_MAX_SIZE):
    """ParamFlowRequestDataWriter.resolveValidParams (:60-80)."""
    out, size = [], 0
    for p in params:
        s = param_transport_size(p)
        if s <= 0:
            continue
        if size + s > max_size:
            break
        size += s
        out.append(p)
    return out


def encode_param(p) -> bytes:
    kind, v = p
    t = bytes([PARAM_TYPE[kind]])
    if kind == "int":
        return t + struct.pack(">i", v)
    if kind == "long":
        return t + struct.pack(">q", v)
    if kind == "byte":
        return t + struct.pack(">b", v)
    if kind == "short":
        return t + struct.pack(">h", v)
    if kind == "float":
        return t + struct.pack(">f", v)
    if kind == "double":
        return t + struct.pack(">d", v)
    if kind == "bool":
        return t + bytes([1 if v else 0])
    b = v.encode() if isinstance(v, str) else bytes(v)
    return t + struct.pack(">i", len(b)) + b


def frame(body: bytes) -> bytes:
    """LengthFieldPrepender(2)."""
    return struct.pack(">H", len(body)) + body


def flow_frame(xid, flow_id, count, prioritized=False) -> bytes:
    return frame(struct.pack(">ibqi?", xid, MSG_TYPE_FLOW, flow_id, count, prioritized))


def param_frame(xid, flow_id, count, params, max_size=DEFAULT_PARAM_MAX_SIZE) -> bytes:
    ps = resolve_valid_params(params, max_size)
    return frame(struct.pack(">ibqii", xid, MSG_TYPE_PARAM_FLOW, flow_id, count, len(ps))
                 + b"".join(encode_param(p) for p in ps))


def ping_frame(xid, namespace: str) -> bytes:
    b = namespace.encode()
    return frame(struct.pack(">ibi", xid, MSG_TYPE_PING, len(b)) + b)


def param_key(p):
    """(SF_TAG_*, bits) the engine keys a wire parameter by (Java equals)."""
    from . import abi
    kind, v = p
    if kind == "int":
        return abi.TAG_INT, v & 0xFFFFFFFFFFFFFFFF
    if kind == "long":
        return abi.TAG_LONG, v & 0xFFFFFFFFFFFFFFFF
    if kind == "byte":
        return abi.TAG_BYTE, v & 0xFFFFFFFFFFFFFFFF
    if kind == "short":
        return abi.TAG_SHORT, v & 0xFFFFFFFFFFFFFFFF
    if kind == "bool":
        return abi.TAG_BOOL, int(bool(v))
    if kind == "double":
        b = struct.unpack(">Q", struct.pack(">d", v))[0]
        return abi.TAG_DOUBLE, 0x7ff8000000000000 if v != v else b
    if kind == "float":
        b = struct.unpack(">I", struct.pack(">f", v))[0]
        return abi.TAG_FLOAT, 0x7fc00000 if v != v else b
    return abi.TAG_STRING, string_key(v)


RESP_DTYPE = np.dtype([("len", ">u2"), ("xid", ">i4"), ("type", "i1"), ("status", "i1"), ("remaining", ">i4"),
                       ("wait", ">i4")])


def decode_responses(buf: bytes) -> np.ndarray:
    """Response frames (16 B each) as a structured array."""
    a = np.frombuffer(bytes(buf), dtype=RESP_DTYPE)
    assert (a["len"] == 14).all()
    return a
