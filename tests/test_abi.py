"""The C-ABI drop-in: the built library loads (no GPU needed), exports every
function include/sentinel_flow.h declares, and every struct the Python mirror
uses has the C layout.  No compute calls are made here."""
import ctypes as C
import os
import re
import subprocess

import pytest

from sentinel_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sentinel_flow.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**(sf_[a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ("sf_create", "sf_destroy", "sf_load_flow_rules", "sf_load_param_rules", "sf_load_system_rules",
                 "sf_submit", "sf_request_tokens", "sf_snapshot", "sf_last_error"):
        assert must in fns


def test_library_exports_every_declared_symbol():
    from sentinel_amd import engine
    L = engine.lib()
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert not missing, missing
    assert L.sf_abi_version() == abi.SF_ABI_VERSION


def test_struct_layouts_match_c(tmp_path):
    names = list(abi.STRUCT_SIZES)
    prog = tmp_path / "sizes.c"
    prog.write_text('#include <stdio.h>\n#include "%s"\nint main(void){\n%s\nreturn 0;}\n' % (
        HEADER, "\n".join('printf("%s %%zu\\n", sizeof(%s));' % (n, n) for n in names)))
    exe = tmp_path / "sizes"
    subprocess.check_call(["gcc", "-o", str(exe), str(prog)])
    out = subprocess.check_output([str(exe)]).decode().split("\n")
    got = {l.split()[0]: int(l.split()[1]) for l in out if l.strip()}
    assert got == abi.STRUCT_SIZES


def test_config_default_matches_reference_defaults():
    from sentinel_amd import engine
    c = abi.sf_config()
    engine.lib().sf_config_default(C.byref(c))
    d = abi.default_config()
    for f, _ in abi.sf_config._fields_:
        if f in ("max_resources", "max_batch", "param_capacity", "max_flow_ids"):
            continue
        assert getattr(c, f) == getattr(d, f), f


def test_create_without_gpu_fails_loudly():
    """No CPU fallback: without a gfx950 device sf_create returns an error."""
    from sentinel_amd import engine
    try:
        import torch  # noqa: F401  (only to ask whether a GPU is present)
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(engine.EngineError):
        engine.FlowEngine(abi.default_config())
