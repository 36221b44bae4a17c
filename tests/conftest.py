import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


def gold(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def gpath(name):
    return os.path.join(GOLDEN, name)


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from crimp_amd import _native
    _native.load()
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def device_builds(tmp_path_factory):
    """The A/B device builds the CPU checks of the exact search kernel inspect, compiled concurrently once per session:
    {name: path} -- 'default' / 'noclob_noopen' / 'noopen' listings (.s) and the 'noopen_co' code object."""
    import importlib.util
    import subprocess
    spec = importlib.util.spec_from_file_location("agpr_check", os.path.join(ROOT, "tools", "agpr_check.py"))
    A = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(A)
    d = tmp_path_factory.mktemp("device_builds")
    jobs = {"default": ((), True), "noclob_noopen": (("-DCRIMP_EX_AGPR_CLOBBERS=0", "-DCRIMP_EX_OPEN=0"), True),
            "noopen": (("-DCRIMP_EX_OPEN=0",), True), "noopen_co": (("-DCRIMP_EX_OPEN=0",), False)}
    procs, out = {}, {}
    for name, (defs, asm) in jobs.items():
        out[name] = str(d / (name + (".s" if asm else ".co")))
        procs[name] = subprocess.Popen(A.compile_cmd(out[name], defs, asm), cwd=A.SRC, stdout=subprocess.DEVNULL,
                                       stderr=subprocess.PIPE)
    for name, p in procs.items():
        _, err = p.communicate()
        assert p.returncode == 0, (name, err[-2000:])
    return out
