"""TEST-ONLY: ctypes wrapper of the host build of the engine's interpreter
(sentinel_amd/csrc/sf_decide.h compiled for the CPU).  Lets the CPU suite check
the kernel logic against the oracle; never used by the product."""
import ctypes as C
import os
import subprocess

from sentinel_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libsf_hostsim.so")
_lib = None
P = C.c_void_p


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", _HERE])
        L = C.CDLL(_LIB)
        L.hs_create.restype = P
        L.hs_create.argtypes = [C.POINTER(abi.sf_config)]
        L.hs_destroy.argtypes = [P]
        L.hs_load_flow_rules.argtypes = [P, C.POINTER(abi.sf_flow_rule), C.c_uint32]
        L.hs_load_param_rules.argtypes = [P, C.POINTER(abi.sf_param_rule), C.c_uint32,
                                          C.POINTER(abi.sf_hot_item), C.c_uint32]
        L.hs_submit.argtypes = [P, C.POINTER(abi.sf_event_batch), C.POINTER(abi.sf_verdicts)]
        L.hs_read_node.argtypes = [P, C.c_uint32, C.POINTER(abi.sf_node_state)]
        L.hs_read_rule_state.argtypes = [P, C.c_uint32, C.POINTER(abi.sf_rule_state)]
        L.hs_read_origin_node.argtypes = [P, C.c_uint32, C.c_uint32, C.POINTER(abi.sf_node_state)]
        L.hs_read_context_node.argtypes = [P, C.c_uint32, C.c_uint32, C.POINTER(abi.sf_node_state)]
        L.hs_load_degrade_rules.argtypes = [P, C.POINTER(abi.sf_degrade_rule), C.c_uint32, C.POINTER(C.c_uint32)]
        L.hs_read_breaker.argtypes = [P, C.c_uint32, C.POINTER(abi.sf_breaker_state)]
        L.hs_sx_reduce.argtypes = [P, C.c_int, P, C.c_double, C.c_double]
        _lib = L
    return _lib


class HostSimEngine:
    def __init__(self, cfg):
        self.cfg = cfg
        self.h = lib().hs_create(C.byref(cfg))

    def close(self):
        if self.h:
            lib().hs_destroy(self.h)
            self.h = None

    __del__ = close

    def load_flow_rules(self, rules):
        ptr, n = abi.flow_rules_ptr(rules)
        assert lib().hs_load_flow_rules(self.h, ptr, n) == 0

    def load_param_rules(self, rules, items=()):
        assert lib().hs_load_param_rules(self.h, abi.rules_array(abi.sf_param_rule, rules), len(rules),
                                         abi.rules_array(abi.sf_hot_item, list(items)), len(items)) == 0

    def load_degrade_rules(self, rules) -> int:
        arr = (abi.sf_degrade_rule * max(1, len(rules)))()
        for i, r in enumerate(rules):
            for k, v in r.items():
                setattr(arr[i], k, v)
        n = C.c_uint32(0)
        assert lib().hs_load_degrade_rules(self.h, arr, len(rules), C.byref(n)) == 0
        return int(n.value)

    def read_breaker(self, k):
        st = abi.sf_breaker_state()
        assert lib().hs_read_breaker(self.h, k, C.byref(st)) == 0
        return st

    def submit(self, batch):
        out = abi.HostVerdicts(batch.n)
        b, v = batch.c_struct(), out.c_struct()
        rc = lib().hs_submit(self.h, C.byref(b), C.byref(v))
        assert rc == 0, rc
        return out

    def read_node(self, res):
        st = abi.sf_node_state()
        assert lib().hs_read_node(self.h, res, C.byref(st)) == 0
        return st

    def read_rule_state(self, idx):
        s = abi.sf_rule_state()
        assert lib().hs_read_rule_state(self.h, idx, C.byref(s)) == 0
        return s

    def read_origin_node(self, res, origin):
        st = abi.sf_node_state()
        if lib().hs_read_origin_node(self.h, res, origin, C.byref(st)):
            raise KeyError((res, origin))
        return st

    def read_context_node(self, context, res):
        st = abi.sf_node_state()
        if lib().hs_read_context_node(self.h, context, res, C.byref(st)):
            raise KeyError((context, res))
        return st
