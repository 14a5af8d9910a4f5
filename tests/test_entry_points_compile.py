"""The driver's entry points compile (CPU): bench.py and __graft_entry__.py are run only on the GPU box at round end,
so a syntax error in either would first show there."""
import os
import py_compile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["bench.py", "__graft_entry__.py", "oracle/cpu_baseline.py",
                                  "tests/shadow_modes_worker.py", "tests/dp_worker.py"])
def test_entry_point_compiles(name, tmp_path):
    """bench.py's CPU leg (oracle/cpu_baseline.py) is imported only after the timed region on the GPU box"""
    path = os.path.join(REPO, name)
    assert os.path.exists(path), f"{name} missing"
    py_compile.compile(path, cfile=str(tmp_path / (os.path.basename(name) + "c")), doraise=True)
