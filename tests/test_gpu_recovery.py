"""A training step that throws must not corrupt the steps after it (trainer.cpp Step):
the next bunch's gather is handed to the step's last launch (CuNetwork::SetTailGather) and the cache has
already moved past that bunch, so a step that fails before that launch must still deliver the bunch
into the other buffer, and must not leave the network holding the gather.

The fault is injected with tnet_debug_fail_train_bunch (the n-th next TrainBunch throws before it
enqueues anything).  Reference: the oracle restatement stepping the same bunches with the failed one
left out (cuBiasedLinearity.cc:46-64 semantics, GRADDIVFRM=T, momentum 0).

Tolerances: per-step weights rtol 2e-4, atol 1e-6 (as tests/test_gpu_train.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as orc  # noqa: E402
from tnet_amd import DeviceArray, Network, Objective, TnetError, Trainer, formats  # noqa: E402
from tnet_amd._lib import check, lib  # noqa: E402


@pytest.mark.parametrize("dims,B", [([598, 1024, 135], 256), ([440, 512, 512, 300], 128)])
def test_failed_step_keeps_the_bunch_stream(dims, B):
    nb = 8
    rng = np.random.default_rng(11)
    X = rng.standard_normal((nb * B, dims[0])).astype(np.float32)
    L = rng.integers(0, dims[-1], nb * B).astype(np.int32)
    layers = formats.gen_mlp_init(dims, seed=5)
    lr = 0.5
    net = Network.from_layers(layers)
    net.set_learn_rate(lr)
    net.set_grad_div_frm(True)
    obj = Objective()
    tr = Trainer(net, obj, bunchsize=B, cachesize=nb * B, seed=1, randomize=False)
    taken = lib().tnet_trainer_prefill(tr.h, X.ctypes.data, X.shape[0], X.shape[1], X.shape[1], L.ctypes.data)
    assert taken == nb * B
    ref = orc.MLP.from_layers(layers)

    def ref_step(j):
        ref.step(X[j * B:(j + 1) * B], L[j * B:(j + 1) * B], lr)

    tr.replay(2)  # bunches 0, 1 (bunch 2 gathered by bunch 1's last launch)
    ref_step(0)
    ref_step(1)
    check(lib().tnet_debug_fail_train_bunch(1))
    with pytest.raises(TnetError, match="injected fault"):
        tr.replay(1)  # bunch 2 fails before any launch; bunch 3 must still reach the other buffer
    # a direct network call right after the failure must not carry a stale gather descriptor
    Xe = rng.standard_normal((B, dims[0])).astype(np.float32)
    Le = rng.integers(0, dims[-1], B).astype(np.int32)
    net.train_bunch(obj, DeviceArray.from_numpy(Xe), DeviceArray.vector(Le))
    ref.step(Xe, Le, lr)
    tr.replay(5)  # bunches 3..7
    for j in range(3, nb):
        ref_step(j)
    for k, (W, b) in enumerate(net.linear_params()):
        np.testing.assert_allclose(W, ref.W[k], rtol=2e-4, atol=1e-6)
        np.testing.assert_allclose(b, ref.b[k], rtol=2e-4, atol=1e-6)
    assert tr.steps == nb - 1
    check(lib().tnet_debug_fail_train_bunch(0))
