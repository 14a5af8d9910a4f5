"""tnet_amd -- MI355X-native TNet frame-batched SGD path (Python host binding).

The compute path is C++ + hand-written gfx950 HIP kernels in lib/libtnet_amd.so; this package
is a thin host-side mirror of the reference C++ interface (CuNetwork, CuObjectiveFunction, the
TNetCu loop) over its C ABI, used by the tests and bench.py.  Device memory is owned by
DeviceArray (hipMalloc through the library), never by a CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional, Sequence

import numpy as np

from . import formats  # noqa: F401  (host formats; no device code)
from ._lib import HOST_ALLREDUCE_FN, LIB_PATH, MatrixDim, TnetError, check, check_ptr, header_symbols, lib

__all__ = ["DeviceArray", "Network", "Objective", "Trainer", "RbmTrainer", "RnnTrainer", "Comm", "TnetError", "synchronize",
           "FeatureReader", "htk_read", "mask_match", "mlf_lookup",
           "pad_stride",
           "device_count", "version", "LIB_PATH", "header_symbols", "formats"]


def pad_stride(cols: int) -> int:
    return ((cols + 63) // 64) * 64 if cols else 0


def device_count() -> int:
    n = C.c_int(0)
    lib().tnet_device_count(C.byref(n))
    return n.value


def version() -> str:
    return lib().tnet_version().decode()


def synchronize() -> None:
    check(lib().tnet_synchronize(), "synchronize")


def _utterance(feats, labels=None, who: str = "utterance"):
    """Host-side shape check of one utterance before its pointers reach the C ABI: the library
    copies feats.shape[0] rows and as many labels, so a short labels array would be read past."""
    feats = np.ascontiguousarray(feats, np.float32)
    if feats.ndim != 2:
        raise ValueError(f"{who}: feats must be 2-D [frames x dim], got shape {feats.shape}")
    if labels is None:
        return feats, None
    labels = np.ascontiguousarray(labels, np.int32)
    if labels.ndim != 1 or labels.shape[0] != feats.shape[0]:
        raise ValueError(f"{who}: labels must be 1-D with one class id per frame "
                         f"({feats.shape[0]} frames), got shape {labels.shape}")
    return feats, labels


class DeviceArray:
    """Row-major device matrix (rows x cols) with a padded stride (multiple of 64 elements)."""

    def __init__(self, rows: int, cols: int = 1, dtype=np.float32, stride: Optional[int] = None, zero=True):
        self.rows, self.cols = int(rows), int(cols)
        self.dtype = np.dtype(dtype)
        self.stride = int(stride) if stride is not None else pad_stride(self.cols)
        self.nbytes = max(self.rows * self.stride * self.dtype.itemsize, 16)
        p = C.c_void_p()
        check(lib().tnet_malloc(C.byref(p), self.nbytes), "tnet_malloc")
        self.ptr = p.value
        if zero:
            check(lib().tnet_memset(self.ptr, 0, self.nbytes), "tnet_memset")

    @classmethod
    def from_numpy(cls, a: np.ndarray, stride: Optional[int] = None) -> "DeviceArray":
        a = np.asarray(a)
        if a.ndim == 1:
            a = a.reshape(1, -1) if a.dtype != np.int32 else a.reshape(-1, 1)
        d = cls(a.shape[0], a.shape[1], a.dtype, stride=stride if stride is not None else pad_stride(a.shape[1]))
        d.upload(a)
        return d

    @classmethod
    def vector(cls, v: np.ndarray) -> "DeviceArray":
        v = np.ascontiguousarray(v)
        d = cls(v.shape[0], 1, v.dtype, stride=1)
        d.upload(v.reshape(-1, 1))
        return d

    def upload(self, a: np.ndarray) -> None:
        a = np.asarray(a, dtype=self.dtype).reshape(self.rows, self.cols)
        host = np.zeros((self.rows, self.stride), self.dtype)
        host[:, : self.cols] = a
        check(lib().tnet_memcpy_h2d(self.ptr, host.ctypes.data, host.nbytes), "h2d")

    def numpy(self) -> np.ndarray:
        host = np.empty((self.rows, self.stride), self.dtype)
        check(lib().tnet_memcpy_d2h(host.ctypes.data, self.ptr, host.nbytes), "d2h")
        return host[:, : self.cols].copy()

    @property
    def dim(self) -> MatrixDim:
        return MatrixDim(self.rows, self.cols, self.stride)

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                lib().tnet_synchronize()
                lib().tnet_free(self.ptr)
                self.ptr = None
        except Exception:
            pass


class Network:
    """CuNetwork (src/CuTNetLib/cuNetwork.h:22-194) handle."""

    def __init__(self, path: Optional[str] = None, text: Optional[str] = None):
        if path is not None:
            self.h = check_ptr(lib().tnet_net_read(path.encode()), "tnet_net_read")
        elif text is not None:
            self.h = check_ptr(lib().tnet_net_read_text(text.encode()), "tnet_net_read_text")
        else:
            raise ValueError("path or text required")

    @classmethod
    def from_layers(cls, layers, precision: int = 9) -> "Network":
        import io
        buf = io.StringIO()
        formats.write_nnet(layers, buf, precision=precision)
        return cls(text=buf.getvalue())

    def write(self, path: str) -> None:
        check(lib().tnet_net_write(self.h, path.encode()), "tnet_net_write")

    def components(self):
        out = []
        for i in range(lib().tnet_net_num_components(self.h)):
            tag = C.create_string_buffer(64)
            ni, no = C.c_int(), C.c_int()
            check(lib().tnet_net_component(self.h, i, tag, 64, C.byref(ni), C.byref(no)), "component")
            out.append((tag.value.decode(), ni.value, no.value))
        return out

    @property
    def n_in(self) -> int:
        return self.components()[0][1]

    @property
    def n_out(self) -> int:
        return self.components()[-1][2]

    def get_params(self, i: int):
        tag, ni, no = self.components()[i]
        W = np.empty((ni, no), np.float32)
        b = np.empty(no, np.float32)
        check(lib().tnet_net_get_params(self.h, i, W.ctypes.data, b.ctypes.data), "get_params")
        return W, b

    def linear_params(self):
        return [self.get_params(i) for i, c in enumerate(self.components()) if c[0] == "<biasedlinearity>"]

    def set_params(self, i: int, W: np.ndarray, b: np.ndarray) -> None:
        W = np.ascontiguousarray(W, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        check(lib().tnet_net_set_params(self.h, i, W.ctypes.data, b.ctypes.data), "set_params")

    def set_learn_rate(self, lr: float, factors: Optional[str] = None) -> None:
        check(lib().tnet_net_set_learn_rate(self.h, lr, factors.encode() if factors else None), "learn_rate")

    def set_momentum(self, m: float) -> None:
        check(lib().tnet_net_set_momentum(self.h, m), "momentum")

    def set_weightcost(self, wc: float) -> None:
        check(lib().tnet_net_set_weightcost(self.h, wc), "weightcost")

    def set_grad_div_frm(self, div: bool) -> None:
        check(lib().tnet_net_set_grad_div_frm(self.h, int(div)), "graddivfrm")

    def propagate(self, X: DeviceArray, Y: Optional[DeviceArray] = None) -> DeviceArray:
        if Y is None:
            Y = DeviceArray(X.rows, self.n_out)
        check(lib().tnet_net_propagate(self.h, X.ptr, X.rows, X.stride, Y.ptr, Y.stride), "propagate")
        return Y

    def backpropagate(self, E: DeviceArray) -> None:
        check(lib().tnet_net_backpropagate(self.h, E.ptr, E.rows, E.stride), "backpropagate")

    def train_bunch(self, obj: "Objective", X: DeviceArray, labels: DeviceArray, train: bool = True) -> None:
        check(lib().tnet_net_train_bunch(self.h, obj.h, X.ptr, X.rows, X.stride, labels.ptr, int(train)),
              "train_bunch")

    def recurrent_params(self, i: int = 0):
        """(W [(n_in + n_out) x n_out], bias) of a <recurrent> component."""
        _, ni, no = self.components()[i]
        W = np.empty((ni + no, no), np.float32)
        b = np.empty(no, np.float32)
        check(lib().tnet_net_recurrent_get(self.h, i, W.ctypes.data, b.ctypes.data), "recurrent_get")
        return W, b

    def rbm_params(self, i: int = 0):
        """(W [n_vis x n_hid], vis_bias, hid_bias, (vis_type, hid_type)) of an <rbm> component."""
        _, ni, no = self.components()[i]
        W = np.empty((ni, no), np.float32)
        vb = np.empty(ni, np.float32)
        hb = np.empty(no, np.float32)
        t = np.zeros(2, np.int32)
        check(lib().tnet_net_rbm_get(self.h, i, W.ctypes.data, vb.ctypes.data, hb.ctypes.data, t.ctypes.data),
              "rbm_get")
        names = ("bern", "gauss")
        return W, vb, hb, (names[t[0]], names[t[1]])

    def set_rbm_params(self, i: int, W=None, vis_bias=None, hid_bias=None, types=None) -> None:
        keep = []
        args = []
        for a in (W, vis_bias, hid_bias):
            a = None if a is None else np.ascontiguousarray(a, np.float32)
            keep.append(a)
            args.append(None if a is None else a.ctypes.data)
        vt, ht = (-1, -1) if types is None else tuple(0 if x == "bern" else 1 for x in types)
        check(lib().tnet_net_rbm_set(self.h, i, args[0], args[1], args[2], vt, ht), "rbm_set")

    def rbm_update(self, i: int, pos_vis: "DeviceArray", pos_hid: "DeviceArray", neg_vis: "DeviceArray",
                   neg_hid: "DeviceArray") -> None:
        """CuRbm::RbmUpdate (generic, unstacked form)."""
        check(lib().tnet_net_rbm_update(self.h, i, pos_vis.ptr, pos_hid.ptr, neg_vis.ptr, neg_hid.ptr, pos_vis.rows,
                                        pos_vis.stride, pos_hid.stride), "rbm_update")

    def set_comm(self, comm: Optional["Comm"]) -> None:
        """train_bunch all-reduces the weight gradients over `comm` (None: local update)."""
        self._comm = comm
        check(lib().tnet_net_set_comm(self.h, comm.h if comm else None), "set_comm")

    def train_empty(self, comm: "Comm", global_rows: int) -> None:
        """Data-parallel step of a rank without a bunch (zero gradient, same update)."""
        check(lib().tnet_net_train_empty(self.h, comm.h, global_rows), "train_empty")

    def keep_output(self, keep: bool = True) -> None:
        check(lib().tnet_net_keep_output(self.h, int(keep)), "keep_output")

    def output(self, i: int, rows: int) -> np.ndarray:
        no = self.components()[i][2]
        out = np.empty((rows, no), np.float32)
        check(lib().tnet_net_output(self.h, i, out.ctypes.data, no), "output")
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().tnet_net_free(self.h)
                self.h = None
        except Exception:
            pass


class Objective:
    """CuObjectiveFunction (src/CuTNetLib/cuObjectiveFunction.h:20-157)."""

    XENT, MSE = 0, 1

    def __init__(self, kind: int = 0):
        self.h = check_ptr(lib().tnet_obj_create(kind), "tnet_obj_create")

    def evaluate(self, out: DeviceArray, des: DeviceArray, err: DeviceArray) -> None:
        check(lib().tnet_obj_evaluate(self.h, out.ptr, out.rows, out.cols, out.stride, des.ptr, des.stride, err.ptr,
                                      err.stride), "evaluate")

    def evaluate_labels(self, out: DeviceArray, labels: DeviceArray, err: DeviceArray) -> None:
        check(lib().tnet_obj_evaluate_labels(self.h, out.ptr, out.rows, out.cols, out.stride, labels.ptr, err.ptr,
                                             err.stride), "evaluate_labels")

    def stats(self):
        e, c = C.c_double(), C.c_double()
        f = C.c_long()
        check(lib().tnet_obj_stats(self.h, C.byref(e), C.byref(f), C.byref(c)), "stats")
        return e.value, f.value, c.value

    def report(self) -> str:
        buf = C.create_string_buffer(512)
        check(lib().tnet_obj_report(self.h, buf, 512), "report")
        return buf.value.decode()

    def reset(self) -> None:
        check(lib().tnet_obj_reset(self.h), "reset")

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().tnet_obj_free(self.h)
                self.h = None
        except Exception:
            pass


class Trainer:
    """The TNetCu SGD loop (src/TNetCu.cc:375-442) over a CuCache."""

    def __init__(self, net: Network, obj: Objective, bunchsize=256, cachesize=12800, seed=0, randomize=True,
                 crossval=False):
        self.net, self.obj = net, obj
        self.h = check_ptr(lib().tnet_trainer_create(net.h, obj.h, bunchsize, cachesize, seed, int(randomize),
                                                     int(crossval)), "tnet_trainer_create")

    def add_utterance(self, feats: np.ndarray, labels: np.ndarray) -> None:
        feats, labels = _utterance(feats, labels, "Trainer.add_utterance")
        check(lib().tnet_trainer_add_utterance(self.h, feats.ctypes.data, feats.shape[0], feats.shape[1],
                                               feats.shape[1], labels.ctypes.data), "add_utterance")

    def finish(self) -> None:
        check(lib().tnet_trainer_finish(self.h), "finish")

    def train_corpus(self, feats: Sequence[np.ndarray], labels: Sequence[np.ndarray]) -> None:
        for x, l in zip(feats, labels):
            self.add_utterance(x, l)
        self.finish()

    @property
    def steps(self) -> int:
        return lib().tnet_trainer_steps(self.h)

    @property
    def empty_steps(self) -> int:
        return lib().tnet_trainer_empty_steps(self.h)

    def replay(self, n: int) -> None:
        check(lib().tnet_trainer_replay(self.h, n), "replay")

    def set_transform(self, transform: Optional["Network"], start_ext: int = 0, end_ext: int = 0) -> None:
        """--FEATURETRANSFORM network + --STARTFRMEXT/--ENDFRMEXT (TNetCu.cc:384-393)."""
        self._transform = transform   # borrowed by the C++ trainer: keep it alive
        check(lib().tnet_trainer_set_transform(self.h, transform.h if transform else None, start_ext, end_ext),
              "set_transform")

    def add_reader(self, reader: "FeatureReader", max_utts: int = -1) -> int:
        """the TNetCu cache-fill loop (TNetCu.cc:376-419) over a native FeatureReader; returns frames added"""
        n = lib().tnet_trainer_add_reader(self.h, reader.h, max_utts)
        if n < 0:
            check(int(n), "add_reader")
        return int(n)

    def set_comm(self, comm: Optional["Comm"]) -> None:
        self._comm = comm
        check(lib().tnet_trainer_set_comm(self.h, comm.h if comm else None), "set_comm")

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().tnet_trainer_free(self.h)
                self.h = None
        except Exception:
            pass


class RbmTrainer:
    """The TRbmCu CD-1 loop (src/TRbmCu.cc:291-357) over a one-<rbm> network."""

    def __init__(self, net: Network, bunchsize=256, cachesize=12800, seed=0, randomize=True, learn_rate=0.1,
                 momentum=0.5, weightcost=0.0002):
        self.net = net
        self.h = check_ptr(lib().tnet_rbm_trainer_create(net.h, bunchsize, cachesize, seed, int(randomize),
                                                         learn_rate, momentum, weightcost), "tnet_rbm_trainer_create")

    def add_utterance(self, feats: np.ndarray) -> None:
        feats, _ = _utterance(feats, None, "RbmTrainer.add_utterance")
        check(lib().tnet_rbm_trainer_add_utterance(self.h, feats.ctypes.data, feats.shape[0], feats.shape[1],
                                                   feats.shape[1]), "rbm add_utterance")

    def finish(self) -> None:
        check(lib().tnet_rbm_trainer_finish(self.h), "rbm finish")

    def train_corpus(self, feats: Sequence[np.ndarray]) -> None:
        for x in feats:
            self.add_utterance(x)
        self.finish()

    @property
    def steps(self) -> int:
        return lib().tnet_rbm_trainer_steps(self.h)

    def stats(self):
        """(sum of squared reconstruction errors, frames)"""
        e = C.c_double()
        n = C.c_long()
        check(lib().tnet_rbm_trainer_stats(self.h, C.byref(e), C.byref(n)), "rbm stats")
        return e.value, n.value

    def report(self) -> str:
        buf = C.create_string_buffer(512)
        check(lib().tnet_rbm_trainer_report(self.h, buf, 512), "rbm report")
        return buf.value.decode()

    def prefill(self, feats: np.ndarray) -> int:
        feats, _ = _utterance(feats, None, "RbmTrainer.prefill")
        n = lib().tnet_rbm_trainer_prefill(self.h, feats.ctypes.data, feats.shape[0], feats.shape[1], feats.shape[1])
        if n < 0:
            check(-1, "rbm prefill")
        return n

    def replay(self, n: int) -> None:
        check(lib().tnet_rbm_trainer_replay(self.h, n), "rbm replay")

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().tnet_rbm_trainer_free(self.h)
                self.h = None
        except Exception:
            pass


class RnnTrainer:
    """The TRecurrentCu frame-by-frame loop (src/TRecurrentCu.cc:319-375)."""

    def __init__(self, net: Network, obj: Objective, bptt: int = 4, crossval: bool = False):
        self.net, self.obj = net, obj
        self.h = check_ptr(lib().tnet_rnn_trainer_create(net.h, obj.h, bptt, int(crossval)), "tnet_rnn_trainer_create")

    def train_utterance(self, feats: np.ndarray, labels: np.ndarray) -> None:
        feats, labels = _utterance(feats, labels, "RnnTrainer.train_utterance")
        check(lib().tnet_rnn_trainer_utterance(self.h, feats.ctypes.data, feats.shape[0], feats.shape[1],
                                               feats.shape[1], labels.ctypes.data), "rnn utterance")

    def train_corpus(self, feats, labels) -> None:
        for x, l in zip(feats, labels):
            self.train_utterance(x, l)

    @property
    def frames(self) -> int:
        return lib().tnet_rnn_trainer_frames(self.h)

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().tnet_rnn_trainer_free(self.h)
                self.h = None
        except Exception:
            pass


def shard_utterances(items: Sequence, rank: int, world: int) -> list:
    """Utterance sharding of the data-parallel path: round-robin over ranks in list order, the
    way the reference Platform deals utterances to its worker threads (Platform.h:206-236,
    `thr = (thr+1) % num_thr_`)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return list(items)[rank::world]


class Comm:
    """Data-parallel communicator: RCCL (one process per GPU), or a host transport (Comm.host)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().tnet_comm_unique_id(buf), "unique_id")
        return buf.raw

    def __init__(self, rank: int, world: int, uid: bytes):
        self.h = check_ptr(lib().tnet_comm_create(rank, world, C.c_char_p(uid)), "tnet_comm_create")

    @classmethod
    def host(cls, rank: int, world: int, allreduce: Callable[[np.ndarray], None]) -> "Comm":
        """Host-transport communicator: `allreduce(a)` must sum the numpy array `a` (float32 or
        float64) over ranks in place, e.g. through torch.distributed with the gloo backend."""
        self = cls.__new__(cls)

        def _fn(user, buf, n, is_double):
            try:
                ct = C.c_double if is_double else C.c_float
                a = np.ctypeslib.as_array(C.cast(buf, C.POINTER(ct)), shape=(n,))
                allreduce(a)
                return 0
            except Exception:  # an exception cannot cross the C boundary
                import traceback
                traceback.print_exc()
                return 1

        self._fn = HOST_ALLREDUCE_FN(_fn)  # keep the trampoline alive as long as the communicator
        self.h = check_ptr(lib().tnet_comm_create_host(rank, world, C.cast(self._fn, C.c_void_p), None),
                           "tnet_comm_create_host")
        return self

    def plan_round(self, n: int, final: bool, cap: int = 1 << 16):
        """One round of the data-parallel step plan (collective): (ranks_at_step, all_final)."""
        steps = C.c_long(0)
        allf = C.c_int(0)
        buf = np.zeros(cap, np.int32)
        check(lib().tnet_dp_plan_round(self.h, n, int(final), C.byref(steps), buf.ctypes.data_as(C.POINTER(C.c_int)),
                                       cap, C.byref(allf)), "dp_plan_round")
        return buf[: steps.value].copy(), bool(allf.value)

    def set_step_rows(self, global_rows: int) -> None:
        """Rows of the global bunch for the next steps' GRADDIVFRM division (0 = rows x world)."""
        check(lib().tnet_comm_set_step_rows(self.h, global_rows), "set_step_rows")

    def capture(self, on: bool = True) -> None:
        """arm the reduction check for ONE step (tnet_comm_capture): the next step's gradient blocks are copied
        to the host before and after their reduction"""
        check(lib().tnet_comm_capture(self.h, int(on)), "comm_capture")

    def captured(self):
        """[(local, reduced)] per gradient block of the last armed step, in submission order; `reduced` holds
        NaN outside the ranges this rank applies"""
        out = []
        for i in range(lib().tnet_comm_captured(self.h)):
            n = C.c_long(0)
            check(lib().tnet_comm_captured_block(self.h, i, None, None, 0, C.byref(n)), "captured_block")
            loc, red = np.empty(n.value, np.float32), np.empty(n.value, np.float32)
            check(lib().tnet_comm_captured_block(self.h, i, loc.ctypes.data, red.ctypes.data, n.value, C.byref(n)),
                  "captured_block")
            out.append((loc, red))
        return out

    def transport_ranks(self) -> int:
        r = C.c_int(0)
        check(lib().tnet_comm_transport_ranks(self.h, C.byref(r)), "transport_ranks")
        return r.value

    def allreduce_device(self, a: "DeviceArray") -> None:
        check(lib().tnet_comm_allreduce_device(self.h, a.ptr, a.rows * a.stride), "allreduce_device")

    def allreduce_host(self, v: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(v, np.float64).copy()
        check(lib().tnet_comm_allreduce_host(self.h, v.ctypes.data_as(C.POINTER(C.c_double)), v.size), "allreduce")
        return v

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().tnet_comm_free(self.h)
                self.h = None
        except Exception:
            pass


class FeatureReader:
    """FeatureRepository + LabelRepository (src/KaldiLib/Features.cc, Labels.cc) in native code with a
    read-ahead thread pool (csrc/host/htkio.cpp, include/tnet_train.h tnet_reader_*).  Iterating yields
    (logical name, features [rows x cols] incl. the context rows, class ids [rows - start_ext - end_ext]
    or None, sample period, parameter kind); the arrays are copies."""

    def __init__(self, scp: str, mlf: Optional[str] = None, label_map: Optional[str] = None,
                 label_dir: Optional[str] = None, label_ext: Optional[str] = "lab", start_ext: int = 0,
                 end_ext: int = 0, swap: bool = True, target_kind: int = 12, deriv_order: int = 0,
                 deriv_win: Optional[Sequence[int]] = None, threads: int = 4, depth: int = 16,
                 cmn_dir: Optional[str] = None, cmn_mask: Optional[str] = None, cvn_dir: Optional[str] = None,
                 cvn_mask: Optional[str] = None, cvg_file: Optional[str] = None):
        """cmn_* / cvn_* / cvg_file: CMEANDIR / CMEANMASK, VARSCALEDIR / VARSCALEMASK, VARSCALEFN"""
        enc = lambda s: s.encode() if s is not None else None  # noqa: E731
        self._win = (C.c_int * len(deriv_win))(*deriv_win) if deriv_win else None
        self.start_ext, self.end_ext = start_ext, end_ext
        self.h = check_ptr(lib().tnet_reader_create_norm(
            enc(scp), int(swap), start_ext, end_ext, target_kind, deriv_order,
            C.cast(self._win, C.c_void_p) if self._win else None, enc(mlf), enc(label_map), enc(label_dir),
            enc(label_ext), enc(cmn_dir), enc(cmn_mask), enc(cvn_dir), enc(cvn_mask), enc(cvg_file), threads, depth),
            "reader_create")

    def __len__(self) -> int:
        return int(lib().tnet_reader_size(self.h))

    def next_raw(self):
        """the next utterance as (name, feats, labels, period, kind) views into the reader's buffer
        (valid until the next call), or None at the end of the list"""
        fp, lp = C.c_void_p(), C.c_void_p()
        rows, cols, nl, per, kind = C.c_int(), C.c_int(), C.c_int(), C.c_int(), C.c_int()
        name = C.create_string_buffer(4096)
        st = lib().tnet_reader_next(self.h, C.byref(fp), C.byref(rows), C.byref(cols), C.byref(lp), C.byref(nl),
                                    C.byref(per), C.byref(kind), name, len(name))
        if st == 0:
            return None
        check(st if st < 0 else 0, "reader_next")
        n = rows.value * cols.value
        x = np.ctypeslib.as_array(C.cast(fp, C.POINTER(C.c_float)), (n,)).reshape(rows.value, cols.value) if n else \
            np.zeros((rows.value, cols.value), np.float32)
        lab = np.ctypeslib.as_array(C.cast(lp, C.POINTER(C.c_int)), (nl.value,)) if lp.value else None
        return name.value.decode(), x, lab, per.value, kind.value

    def __iter__(self):
        while True:
            u = self.next_raw()
            if u is None:
                return
            name, x, lab, per, kind = u
            yield name, x.copy(), (lab.copy() if lab is not None else None), per, kind

    def rewind(self) -> None:
        check(lib().tnet_reader_rewind(self.h), "reader_rewind")

    def __del__(self):
        if getattr(self, "h", None):
            try:
                lib().tnet_reader_free(self.h)
            except Exception:
                pass
            self.h = None


def htk_read(record: str, start_ext: int = 0, end_ext: int = 0, swap: bool = True):
    """one HTK record ("logical=physical[s,e]" or a path) through the native reader:
    (features [rows x cols], sample period, parameter kind)"""
    rows, cols, per, kind = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    check(lib().tnet_htk_read(record.encode(), int(swap), start_ext, end_ext, None, 0, C.byref(rows), C.byref(cols),
                              C.byref(per), C.byref(kind)), "htk_read")
    out = np.empty((rows.value, cols.value), np.float32)
    check(lib().tnet_htk_read(record.encode(), int(swap), start_ext, end_ext, out.ctypes.data, out.size, C.byref(rows),
                              C.byref(cols), C.byref(per), C.byref(kind)), "htk_read")
    return out, per.value, kind.value


def mask_match(mask: str, label: str):
    """ProcessMask (StkMatch.cc:453-490) through the native label mask: None when `mask` does not match
    `label`, else the characters its '%'s capture"""
    buf = C.create_string_buffer(4096)
    r = lib().tnet_mask_match(mask.encode("latin-1"), label.encode("latin-1"), buf, len(buf))
    check(min(r, 0), "mask_match")
    return buf.value.decode("latin-1") if r == 1 else None


def mlf_lookup(patterns, labels):
    """LabelContainer Insert(patterns[k], k) in order, then Find(label) for each label (MlfStream.cc:43-265)
    through the native MLF index: the record numbers, -1 where none"""
    P = (C.c_char_p * max(1, len(patterns)))(*[p.encode("latin-1") for p in patterns])
    L = (C.c_char_p * max(1, len(labels)))(*[x.encode("latin-1") for x in labels])
    out = np.full(max(1, len(labels)), -2, np.int32)
    check(lib().tnet_mlf_lookup(C.cast(P, C.c_void_p), len(patterns), C.cast(L, C.c_void_p), len(labels),
                                out.ctypes.data), "mlf_lookup")
    return out[:len(labels)].tolist()
