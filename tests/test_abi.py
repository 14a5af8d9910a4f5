"""CPU-only checks of the drop-in boundary: the C-ABI library loads without a GPU and exports
every entry point the public headers declare; the Python binding covers them all."""
import ctypes
import os
import subprocess

import pytest

from tnet_amd import _lib


def test_library_built():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() / make -C nnet-asr_amd"


def test_exports_every_header_symbol():
    L = _lib.lib()
    missing = [n for n in _lib.header_symbols() if not hasattr(L, n)]
    assert not missing, f"declared in include/*.h but not exported: {missing}"


def test_binding_covers_headers():
    declared = set(_lib.header_symbols())
    bound = set(_lib._SIGS)
    assert declared == bound, (sorted(declared - bound), sorted(bound - declared))


def test_no_torch_or_oracle_dependency():
    """The product library links only the HIP runtime and RCCL (no torch, no oracle)."""
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "libtorch" not in out and "oracle" not in out
    assert "libamdhip64" in out and "librccl" in out


@pytest.mark.parametrize("order", ["lib_then_torch", "torch_then_lib"])
def test_one_hip_runtime_and_clean_exit(order):
    """One HIP runtime and one RCCL per process whatever the import order (tnet_amd maps torch's
    before the library), and the process exits cleanly (a second RCCL mapped before libtorch_hip
    ended in 'double free or corruption' at exit)."""
    import sys
    steps = ["import tnet_amd; tnet_amd._lib.lib()", "import torch, torch.distributed"]
    if order == "torch_then_lib":
        steps.reverse()
    code = ("import sys; sys.path.insert(0, %r); " % os.path.dirname(os.path.dirname(_lib.__file__)) +
            "; ".join(steps) + "; from tnet_amd import _lib; rt = _lib.hip_runtimes_mapped(); "
            "rc = sorted({l.split()[-1] for l in open('/proc/self/maps') if 'librccl' in l}); "
            "print(len(rt), len(rc))")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.split() == ["1", "1"], p.stdout


def test_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/llvm/bin/llvm-readelf", "-n", _lib.LIB_PATH], capture_output=True, text=True)
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_status_strings_without_gpu():
    L = _lib.lib()
    assert b"gfx950" in L.tnet_version()
    assert L.tnet_status_str(-1) == b"invalid argument"


def test_utterance_shape_checks_before_the_abi():
    """The binding rejects mis-shaped utterances before their pointers reach the C ABI, which copies
    feats.shape[0] rows and as many labels (a short labels array would be read past its end)."""
    import numpy as np

    from tnet_amd import _utterance
    f, l = _utterance(np.zeros((5, 3)), np.arange(5))
    assert f.dtype == np.float32 and l.dtype == np.int32 and f.flags.c_contiguous
    with pytest.raises(ValueError):
        _utterance(np.zeros((5, 3)), np.arange(4))
    with pytest.raises(ValueError):
        _utterance(np.zeros(15), np.arange(15))
    with pytest.raises(ValueError):
        _utterance(np.zeros((5, 3)), np.zeros((5, 1)))
    f, l = _utterance(np.zeros((2, 3)), None)
    assert l is None


def _fake(base, k):
    """a 16-B aligned device-address stand-in (never dereferenced: the refusals come before any launch)"""
    return ctypes.c_void_p(base + k * (1 << 28))


def test_gather_ride_refuses_dependent_operands():
    """tnet_affine_update_bias_gather / tnet_rbm_update_stats_gather run a gather beside an update in ONE
    launch; any operand the gather writes that the update reads or writes, or that the update writes and the
    gather reads, is a race the separate calls do not have: TNET_ERR_ARG before anything is launched
    (ADVICE r3).  CPU only: fake 16-B aligned addresses, refused before the first HIP call."""
    from tnet_amd._lib import MatrixDim
    L = _lib.lib()
    base = 1 << 44
    rows, n_in, n_out = 256, 64, 128
    X, E, W, C, P, b, cb = (_fake(base, k) for k in range(7))
    y, x, lo, li, cf = (_fake(base, k) for k in range(7, 12))
    dX, dE, dW = MatrixDim(rows, n_in, n_in), MatrixDim(rows, n_out, n_out), MatrixDim(n_in, n_out, n_out)
    dy, dx = MatrixDim(64, 40, 40), MatrixDim(1000, 40, 40)
    nil = [None, MatrixDim(0, 0, 0), None, MatrixDim(0, 0, 0), None, MatrixDim(0, 0, 0), None, 0, 0.0, 0.0, 0.0,
           None, 0, None, None]

    def upd(y_, x_, lo_, li_, cf_):
        return L.tnet_affine_update_bias_gather(X, dX, E, dE, W, dW, C, n_out, -0.1, 0.5, 0.0, P, n_out, b, cb, *nil,
                                                y_, x_, lo_, li_, cf_, dy, dx, None)
    assert upd(y, x, lo, li, cf) != -1  # independent: not refused for overlap
    for bad in (X, E, W, C, P, b, cb):  # the gather's rows written into an update operand
        assert upd(bad, x, lo, li, cf) == -1
    for bad in (E, P, b, x, cf):        # the gather's class ids written into an update operand / its own source
        assert upd(y, x, bad, li, cf) == -1
    for bad in (W, C, b, cb):           # the gather reads what the update writes
        assert upd(y, bad, lo, li, cf) == -1
        assert upd(y, x, lo, bad, cf) == -1
        assert upd(y, x, lo, li, bad) == -1

    G, gb = W, b  # the data-parallel form: the gradient and the bias gradient are what the GEMM writes

    def grad(y_, x_, lo_, li_, cf_):
        return L.tnet_affine_grad_bias_gather(X, dX, E, dE, G, dW, P, n_out, gb, None, MatrixDim(0, 0, 0), None,
                                              MatrixDim(0, 0, 0), None, MatrixDim(0, 0, 0), None, 0, None,
                                              y_, x_, lo_, li_, cf_, dy, dx, None)
    assert grad(y, x, lo, li, cf) != -1
    for bad in (X, E, G, P, gb):
        assert grad(bad, x, lo, li, cf) == -1
        assert grad(y, x, bad, li, cf) == -1
    for bad in (G, gb):
        assert grad(y, bad, lo, li, cf) == -1
        assert grad(y, x, lo, bad, cf) == -1
        assert grad(y, x, lo, li, bad) == -1

    V, H, vb, cvb, hb, chb, ms = (_fake(base, k) for k in range(12, 19))
    B, nv, nh = 64, 40, 256
    dV, dH, dWr = MatrixDim(2 * B, nv, nv), MatrixDim(2 * B, nh, nh), MatrixDim(nv, nh, nh)

    def rbm(y_, x_, lo_, li_, cf_):
        return L.tnet_rbm_update_stats_gather(V, dV, H, dH, W, dWr, C, nh, 0.1, 0.5, 0.0, B, vb, cvb, hb, chb, ms,
                                              y_, x_, lo_, li_, cf_, dy, dx, None)
    assert rbm(y, x, lo, li, cf) != -1
    for bad in (V, H, W, C, vb, cvb, hb, chb, ms):
        assert rbm(bad, x, lo, li, cf) == -1
        assert rbm(y, x, bad, li, cf) == -1
    for bad in (W, C, vb, hb, ms):
        assert rbm(y, bad, lo, li, cf) == -1
        assert rbm(y, x, lo, li, bad) == -1
