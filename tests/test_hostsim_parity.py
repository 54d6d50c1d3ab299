"""CPU check of the engine's decision interpreter (sf_decide.h, host build)
against the oracle on every seeded parity workload.  The GPU parity suite
(test_gpu_parity.py) runs the same workloads through libsentinel_flow.so."""
import numpy as np
import pytest

from sentinel_amd import abi
from tests import workloads


@pytest.fixture(scope="module")
def hs():
    from tests.hostsim import hostsim
    hostsim.lib()
    return hostsim


@pytest.mark.parametrize("name", list(workloads.ALL))
def test_workload(hs, so, name):
    w = workloads.ALL[name]()
    _, _, outs = workloads.run(hs.HostSimEngine, so.OracleEngine, w)
    if name == "config1":
        b = w["batches"][0]
        st = outs[0][1].status
        ent = (b.flags & abi.EV_EXIT) == 0
        pt = b.ts_ms[ent][st[ent] == abi.V_PASS]
        hw = pt // 500
        c = np.bincount(hw - hw.min())
        assert (c[:-1] + c[1:]).max() <= 20     # FlowQpsDemo: <= 20 passes per 1 s window
    if name == "prioritized":
        assert (outs[0][1].status == abi.V_PRIORITY_WAIT).sum() > 0


def test_config3_two_seeds(hs, so):
    workloads.run(hs.HostSimEngine, so.OracleEngine, workloads.config3(seed=11, split=3))
