"""Subprocess worker of tests/test_gpu_shadow.py::test_shadow_across_training_modes (TNET_BWD_SHADOW is read once per
process): trains one small sigmoid MLP through a sequence of training modes that all write W -- the fused step (which
keeps the hidden layers' transposed shadows), the generic component path on a ONE-row bunch (CuBiasedLinearity::
UpdateFrom's rank-1 kernel, which writes W only), the data-parallel step on a one-rank RCCL communicator (the flat
SGD apply, W only), then the fused step again -- and writes every parameter to an .npz.  A shadow left marked valid
after a writer that did not update it would feed the next fused backward the pre-update weights."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nnet-asr_amd"))
from tnet_amd import Comm, DeviceArray, Network, Objective, formats, synchronize  # noqa: E402


def main(out, with_dp):
    with_dp = with_dp == "1"
    dims = [64, 128, 128, 128, 16]
    net = Network.from_layers(formats.gen_mlp_init(dims, seed=3))
    net.set_learn_rate(2.0)  # large: a stale-weight backward moves the result far outside the fp32 reorder band
    obj = Objective()
    rng = np.random.default_rng(5)

    def bunch(rows):
        X = rng.standard_normal((rows, dims[0])).astype(np.float32)
        L = rng.integers(0, dims[-1], rows).astype(np.int32)
        return DeviceArray.from_numpy(X), DeviceArray.vector(L)

    def fused(rows=96):
        X, L = bunch(rows)
        net.train_bunch(obj, X, L)

    def generic_one_row():
        X, L = bunch(1)
        Y = net.propagate(X)
        y = Y.numpy()
        e = y.copy()
        e[0, int(L.numpy()[0])] -= 1.0  # dE/dz of softmax + cross-entropy
        net.backpropagate(DeviceArray.from_numpy(e))

    fused()
    fused()
    generic_one_row()
    fused()
    fused(1)  # a one-row fused step too
    fused()
    if with_dp:
        comm = Comm(0, 1, Comm.unique_id())
        net.set_comm(comm)
        fused()
        fused()
        net.set_comm(None)
        fused()
        fused()
        synchronize()
        del comm
    synchronize()
    np.savez(out, **{f"p{i}_{k}": a for i, (W, b) in enumerate(net.linear_params()) for k, a in (("W", W), ("b", b))})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
