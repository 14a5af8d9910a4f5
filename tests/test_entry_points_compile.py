"""The driver's entry points compile (CPU): bench.py and __graft_entry__.py are run only on the GPU box at round end,
so a syntax error in either would first show there."""
import os
import py_compile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["bench.py", "__graft_entry__.py", "cpu_baseline.py"])
def test_entry_point_compiles(name, tmp_path):
    path = os.path.join(REPO, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not in this tree")
    py_compile.compile(path, cfile=str(tmp_path / (name + "c")), doraise=True)
