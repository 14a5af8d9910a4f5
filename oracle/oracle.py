"""ctypes wrapper around liboracle.so (oracle/tnet_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker.  The product package (nnet-asr_amd/tnet_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = C.CDLL(path)
        L.orc_sgemm.argtypes = [C.c_char, C.c_char, C.c_int, C.c_int, C.c_int, C.c_float, f32p, C.c_int,
                                f32p, C.c_int, C.c_float, f32p, C.c_int]
        L.orc_sigmoid.argtypes = [f32p, f32p, C.c_long]
        L.orc_diff_sigmoid.argtypes = [f32p, f32p, f32p, C.c_long]
        L.orc_softmax.argtypes = [f32p, f32p, C.c_int, C.c_int]
        L.orc_add_col_sum.argtypes = [C.c_float, f32p, C.c_int, C.c_int, C.c_float, f32p]
        L.orc_xent_eval.argtypes = [f32p, i32p, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_double),
                                    C.POINTER(C.c_long)]
        L.orc_epoch_schedule.argtypes = [i32p, C.c_int, C.c_int, C.c_int, C.c_long, C.c_int, i32p, C.c_long]
        L.orc_epoch_schedule.restype = C.c_long
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        L.orc_epoch_schedule_x.argtypes = [i32p, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, i32p, C.c_long,
                                           C.POINTER(C.c_uint64)]
        L.orc_epoch_schedule_x.restype = C.c_long
        L.orc_rand_seed.argtypes = [C.c_long, C.c_long, u32p, u32p, u32p, u32p]
        L.orc_rand_seed.restype = C.c_uint64
        L.orc_rand_uniform.argtypes = [f32p, C.c_long, u32p, u32p, u32p, u32p]
        L.orc_gauss_rand.argtypes = [f32p, C.c_long, u32p, u32p, u32p, u32p]
        L.orc_rbm_step.argtypes = [C.c_int, C.c_int, f32p, f32p, f32p, f32p, f32p, f32p, f32p, C.c_int, C.c_int,
                                   C.c_int, C.c_float, C.c_float, C.c_float, u32p, u32p, u32p, u32p, C.c_void_p,
                                   C.POINTER(C.c_double)]
        L.orc_rbm_step.restype = C.c_int
        L.orc_rnn_utterance.argtypes = [C.c_int, C.c_int, C.c_int, f32p, f32p, f32p, f32p, f32p, f32p, f32p, f32p,
                                        i32p, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_int,
                                        C.POINTER(C.c_double), C.POINTER(C.c_long)]
        L.orc_rnn_utterance.restype = C.c_int
        L.orc_mlp_step.argtypes = [C.c_int, i32p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, f32p, i32p,
                                   C.c_int, C.c_float, C.c_float, C.c_float, C.c_int, C.c_int, f32p, f32p,
                                   C.POINTER(C.c_double), C.POINTER(C.c_long)]
        L.orc_mlp_forward.argtypes = [C.c_int, i32p, C.c_void_p, C.c_void_p, f32p, C.c_int, f32p]
        L.orc_write_random_nnet.argtypes = [C.c_char_p, i32p, C.c_int, C.c_ulonglong]
        _LIB = L
    return _LIB


def _ptrs(arrs):
    return (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def sgemm(ta, tb, A, B, alpha=1.0, beta=0.0, Cm=None):
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    M = A.shape[1] if ta == "T" else A.shape[0]
    K = A.shape[0] if ta == "T" else A.shape[1]
    N = B.shape[0] if tb == "T" else B.shape[1]
    if Cm is None:
        Cm = np.zeros((M, N), np.float32)
    lib().orc_sgemm(ta.encode(), tb.encode(), M, N, K, alpha, A, A.shape[1], B, B.shape[1], beta, Cm, N)
    return Cm


def sigmoid(x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    lib().orc_sigmoid(y, x, x.size)
    return y


def diff_sigmoid(e, y):
    e = np.ascontiguousarray(e, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    out = np.empty_like(e)
    lib().orc_diff_sigmoid(out, e, y, e.size)
    return out


def softmax(x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    lib().orc_softmax(y, x, x.shape[0], x.shape[1])
    return y


def add_col_sum(M, alpha=1.0, beta=0.0, v=None):
    M = np.ascontiguousarray(M, np.float32)
    if v is None:
        v = np.zeros(M.shape[1], np.float32)
    lib().orc_add_col_sum(alpha, M, M.shape[0], M.shape[1], beta, v)
    return v


def xent_eval(y, labels):
    y = np.ascontiguousarray(y, np.float32)
    labels = np.ascontiguousarray(labels, np.int32)
    err = np.empty_like(y)
    xe = C.c_double(0.0)
    cor = C.c_long(0)
    lib().orc_xent_eval(y, labels, y.shape[0], y.shape[1], err.ctypes.data, C.byref(xe), C.byref(cor))
    return err, xe.value, cor.value


def epoch_schedule(lens, cachesize, bunch, seed, randomize=True):
    lens = np.ascontiguousarray(lens, np.int32)
    cap = int(lens.sum()) // bunch + 1
    out = np.zeros(cap * bunch, np.int32)
    nb = lib().orc_epoch_schedule(lens, len(lens), cachesize, bunch, seed, int(randomize), out, cap)
    if nb < 0:
        raise ValueError("utterance leftover fills the whole cache (the reference asserts cache_space > 0)")
    return out[: nb * bunch].reshape(nb, bunch)


class MLP:
    """Oracle MLP state: weights W[l] [n_in x n_out], biases, momentum buffers."""

    def __init__(self, Ws, bs):
        self.W = [np.ascontiguousarray(w, np.float32).copy() for w in Ws]
        self.b = [np.ascontiguousarray(x, np.float32).copy() for x in bs]
        self.cW = [np.zeros_like(w) for w in self.W]
        self.cb = [np.zeros_like(x) for x in self.b]
        self.dims = np.array([self.W[0].shape[0]] + [w.shape[1] for w in self.W], np.int32)
        self.xent = 0.0
        self.correct = 0
        self.frames = 0

    @classmethod
    def from_layers(cls, layers):
        lin = [L for L in layers if L.tag == "<biasedlinearity>"]
        return cls([L.W for L in lin], [L.b for L in lin])

    def step(self, X, labels, lr, mmt=0.0, wc=0.0, graddivfrm=True, cpu_semantics=False):
        X = np.ascontiguousarray(X, np.float32)
        labels = np.ascontiguousarray(labels, np.int32)
        B = X.shape[0]
        Y = np.empty((B, self.dims[-1]), np.float32)
        E = np.empty_like(Y)
        xe = C.c_double(0.0)
        cor = C.c_long(0)
        lib().orc_mlp_step(len(self.W), self.dims, _ptrs(self.W), _ptrs(self.b), _ptrs(self.cW), _ptrs(self.cb),
                           X, labels, B, lr, mmt, wc, int(graddivfrm), int(cpu_semantics), Y, E,
                           C.byref(xe), C.byref(cor))
        self.xent += xe.value
        self.correct += cor.value
        self.frames += B
        return Y, E

    def forward(self, X):
        X = np.ascontiguousarray(X, np.float32)
        Y = np.empty((X.shape[0], self.dims[-1]), np.float32)
        lib().orc_mlp_forward(len(self.W), self.dims, _ptrs(self.W), _ptrs(self.b), X, X.shape[0], Y)
        return Y


def write_random_nnet(path, dims, seed=2):
    d = np.ascontiguousarray(dims, np.int32)
    if lib().orc_write_random_nnet(path.encode(), d, len(d), seed) != 0:
        raise OSError(f"cannot write {path}")


# ---------------------------------------------------------------------------------------------
# CuRand / CuRbm restatement (curand.tcc, curandkernels.cu, cuRbm.cc, TRbmCu.cc)
# ---------------------------------------------------------------------------------------------
class RandState:
    """HybridTaus state of a rows x cols target, seeded as CuRand::SeedGpu after srand48(seed)."""

    def __init__(self, seed, rows, cols):
        n = rows * cols
        self.rows, self.cols = rows, cols
        self.z = [np.zeros(n, np.uint32) for _ in range(4)]
        self.x_after = int(lib().orc_rand_seed(seed, n, *self.z))

    def uniform(self):
        out = np.empty(self.rows * self.cols, np.float32)
        lib().orc_rand_uniform(out, out.size, *self.z)
        return out.reshape(self.rows, self.cols)

    def gauss(self):
        out = np.empty(self.rows * self.cols, np.float32)
        lib().orc_gauss_rand(out, out.size, *self.z)
        return out.reshape(self.rows, self.cols)


def epoch_schedule_x(lens, cachesize, bunch, x0, randomize=True):
    """Epoch bunch schedule with the lrand48 stream starting at raw state x0."""
    lens = np.ascontiguousarray(lens, np.int32)
    cap = int(lens.sum()) // bunch + 1
    out = np.zeros(cap * bunch, np.int32)
    xe = C.c_uint64()
    nb = lib().orc_epoch_schedule_x(lens, len(lens), cachesize, bunch, x0, int(randomize), out, cap, C.byref(xe))
    if nb < 0:
        raise ValueError("utterance leftover fills the whole cache (the reference asserts cache_space > 0)")
    return out[: nb * bunch].reshape(nb, bunch)


class RBM:
    """Oracle RBM state: W [V x H], visible / hidden biases and their momentum buffers."""

    def __init__(self, W, vb, hb, vis_type="gauss", hid_type="bern"):
        self.W = np.ascontiguousarray(W, np.float32).copy()
        self.vb = np.ascontiguousarray(vb, np.float32).copy()
        self.hb = np.ascontiguousarray(hb, np.float32).copy()
        self.cW = np.zeros_like(self.W)
        self.cvb = np.zeros_like(self.vb)
        self.chb = np.zeros_like(self.hb)
        self.vis_gauss = vis_type == "gauss"
        self.hid_gauss = hid_type == "gauss"
        self.mse = 0.0
        self.frames = 0

    @classmethod
    def from_layer(cls, L):
        return cls(L.W, L.extra["vis_bias"], L.b, L.extra["vis_type"], L.extra["hid_type"])

    def step(self, pos_vis, rand: RandState, lr, mmt, wc):
        pos_vis = np.ascontiguousarray(pos_vis, np.float32)
        B, V = pos_vis.shape
        H = self.W.shape[1]
        neg = np.empty((B, V), np.float32)
        e2 = C.c_double(0.0)
        st = lib().orc_rbm_step(V, H, self.W, self.vb, self.hb, self.cW, self.cvb, self.chb, pos_vis, B,
                                int(self.vis_gauss), int(self.hid_gauss), lr, mmt, wc, *rand.z,
                                neg.ctypes.data, C.byref(e2))
        if st != 0:
            raise MemoryError("orc_rbm_step")
        self.mse += e2.value
        self.frames += B
        return neg


class RNN:
    """Oracle state of [<recurrent> nIn->H, <biasedlinearity> H->S, <softmax>] (TRecurrentCu)."""

    def __init__(self, Wr, br, W2, b2):
        self.Wr = np.ascontiguousarray(Wr, np.float32).copy()
        self.br = np.ascontiguousarray(br, np.float32).copy()
        self.W2 = np.ascontiguousarray(W2, np.float32).copy()
        self.b2 = np.ascontiguousarray(b2, np.float32).copy()
        self.cbr = np.zeros_like(self.br)
        self.cW2 = np.zeros_like(self.W2)
        self.cb2 = np.zeros_like(self.b2)
        self.xent = 0.0
        self.correct = 0
        self.frames = 0

    def utterance(self, feats, labels, bptt, lr, mmt=0.0, wc=0.0, gdf=True):
        feats = np.ascontiguousarray(feats, np.float32)
        labels = np.ascontiguousarray(labels, np.int32)
        T, nIn = feats.shape
        H, S = self.W2.shape
        xe = C.c_double(0.0)
        cor = C.c_long(0)
        st = lib().orc_rnn_utterance(nIn, H, S, self.Wr, self.br, self.cbr, self.W2, self.b2, self.cW2, self.cb2,
                                     feats, labels, T, bptt, lr, mmt, wc, int(gdf), C.byref(xe), C.byref(cor))
        if st != 0:
            raise MemoryError("orc_rnn_utterance")
        self.xent += xe.value
        self.correct += cor.value
        self.frames += T


# --------------------------------------------------------------------------------------
# feature front end (--FEATURETRANSFORM networks): numpy restatement
# --------------------------------------------------------------------------------------

def frontend_component(L, x):
    """One front-end component forward, restating src/CuTNetLib/cuCRBEDctFeat.h:16-304 (and the
    CUDA kernels it calls, src/CuBaseLib/cukernels.cu:347-379, cumath.cc:76-113).  Returns float32;
    the block product accumulates in float64."""
    x = np.asarray(x, dtype=np.float32)
    T = x.shape[0]
    if L.tag == "<expand>":                                     # _expand: edge-clamped row offsets
        off = np.asarray(L.extra["offsets"], dtype=np.int64)
        rows = np.clip(np.arange(T)[:, None] + off[None, :], 0, T - 1)   # [T x k]
        return x[rows].reshape(T, -1)
    if L.tag in ("<copy>", "<transpose>"):                      # _rearrange: out of range -> +inf
        if L.tag == "<copy>":
            idx = np.asarray(L.extra["indices"], dtype=np.int64)
        else:                                                   # cuCRBEDctFeat.h:109-123
            n, ctx = L.n_in, int(L.extra["context"])
            ch = n // ctx
            idx = np.array([c + f * ch for c in range(ch) for f in range(ctx)], dtype=np.int64)
        ok = (idx >= 0) & (idx < x.shape[1])
        y = np.full((T, idx.shape[0]), np.inf, dtype=np.float32)
        y[:, ok] = x[:, idx[ok]]
        return y
    if L.tag == "<blocklinearity>":
        B = np.asarray(L.W, dtype=np.float64)                   # [bi x bo]
        bi, bo = B.shape
        nb = x.shape[1] // bi
        xb = x.astype(np.float64).reshape(T, nb, bi)
        return np.einsum("tbi,io->tbo", xb, B).reshape(T, nb * bo).astype(np.float32)
    if L.tag == "<bias>":
        return (x + np.asarray(L.b, dtype=np.float32)[None, :]).astype(np.float32)
    if L.tag == "<window>":
        return (x * np.asarray(L.extra["window"], dtype=np.float32)[None, :]).astype(np.float32)
    if L.tag == "<log>":
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.log(x).astype(np.float32)
    raise ValueError("not a front-end component: " + L.tag)


def frontend_forward(layers, x, start_ext=0, end_ext=0):
    """TNetCu's per-utterance front end (TNetCu.cc:384-393): frame extension by edge repetition
    (src/KaldiLib/Features.cc:776-850), transform network, trim start_ext/end_ext rows."""
    x = np.asarray(x, dtype=np.float32)
    y = np.concatenate([np.repeat(x[:1], start_ext, 0), x, np.repeat(x[-1:], end_ext, 0)], axis=0)
    for L in layers:
        y = frontend_component(L, y)
    return y[start_ext:y.shape[0] - end_ext]
