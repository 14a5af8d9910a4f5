#!/usr/bin/env python3
"""bench.py -- training frames/sec of the MI355X TNet SGD path (BASELINE.json metric).

Workload (N=1 line): the metric's 440 -> 2048x4 -> 4000 sigmoid MLP, softmax + cross-entropy,
bunch 1024 frames per GPU, GRADDIVFRM=T, fp32 end to end; synthetic 440-dim N(0,1) frames with
uniform class ids resident in a GPU CuCache.  One "step" = one bunch:
gather from the shuffled cache -> forward -> softmax/xent -> backward -> SGD update, exactly the
TNetCu per-bunch loop (src/TNetCu.cc:427-441).

Multi-GPU (launched by torch.distributed.run): one process per GPU, utterance-sharded caches
(weak scaling: 1024 frames per GPU per step), per-layer RCCL all-reduce of the gradients over
xGMI, global-bunch GRADDIVFRM normalisation.  torch is used only for the gloo rendezvous /
barrier / max-reduce of the timings (tnet_amd maps torch's ROCm runtime before the library whenever
torch is installed: one HIP runtime and one RCCL per process, whatever the import order).  After the
timed region every rank checksums its parameters and the ranks compare them: replicas that differ
(a broken exchange) end the run with a non-zero exit instead of a number; before that, one extra step verifies the
reductions themselves (rccl_check: every layer's RCCL-reduced gradient against a float64 gloo sum of the ranks'
local gradients, tnet_amd/dpcheck.py -- a wrong reduction hands every rank the same wrong sum, which the replica
checksum cannot see; exit 4 on a mismatch).

Extra JSON fields: roofline (dominant kernel = the 2048x2048 affine-layer GEMMs, timed with hipEvents
on the library stream over K further steps of the same workload right after the timed region: one
event pair per run of back-to-back roofline launches -- the 3 hidden forward GEMMs, and the 6 hidden
backward + update GEMMs -- and none in the value region, since every event pair adds stream time),
kernels (per-kernel breakdown from extra all-events steps after the timed region), cpu_baseline (the
reference CPU TNet on this host, rank 0 at N=1).
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402

import tnet_amd  # noqa: E402
from tnet_amd import Comm, Network, Objective, Trainer, formats  # noqa: E402
from tnet_amd._lib import check, lib  # noqa: E402

CONFIGS = {
    "dnn4": [440, 2048, 2048, 2048, 2048, 4000],        # metric: 440 -> 2048x4 -> senones
    "dnn5": [440, 2048, 2048, 2048, 2048, 2048, 4000],  # BASELINE config 3
    "mlp3": [598, 1024, 135],                           # BASELINE config 2
}
PEAK_FP32_MFMA = 157.3  # TFLOP/s, MI355X dense fp32 matrix (MI355X_MICROARCH.md)
PEAK_HBM = 8000.0       # GB/s


def flops_per_frame(dims):
    W = sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))
    return 2.0 * (3 * W - dims[0] * dims[1])  # fwd all, bwd-error all but first, dW all


def build_network(dims, seed=2):
    """Topology from a compact zero-weight text, then gen_mlp_init-style weights uploaded."""
    parts = []
    for i in range(len(dims) - 1):
        ni, no = dims[i], dims[i + 1]
        parts.append(f"<biasedlinearity> {no} {ni}\nm {no} {ni}\n" + ("0 " * ni + "\n") * no + f"v {no} " +
                     "0 " * no + "\n")
        parts.append(f"<{'softmax' if i == len(dims) - 2 else 'sigmoid'}> {no} {no}\n")
    net = Network(text="".join(parts))
    rng = np.random.default_rng(seed)
    for k in range(len(dims) - 1):
        W = (0.1 * rng.standard_normal((dims[k], dims[k + 1]))).astype(np.float32)
        b = (np.zeros(dims[k + 1]) if k == len(dims) - 2 else rng.random(dims[k + 1]) / 5.0 - 4.1).astype(np.float32)
        net.set_params(2 * k, W, b)
    return net


def synth_frames(n, dim, n_cls, seed):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((n, dim)).astype(np.float32), rng.integers(0, n_cls, n).astype(np.int32)


def pmc_traffic():
    """roofline.traffic: HBM bytes per launch of the roofline kernel set, from the newest committed
    PMC summary (profiles/r*_pmc_gemm2048.json, tools/profile_round.sh + tools/roofline_evidence.py:
    FETCH_SIZE x2 + WRITE_SIZE of the same kernels, measured in separate rocprofv3 --pmc passes --
    counters cannot be read inside this process)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_gemm2048.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d["traffic_MB_per_launch"] * 1e6, os.path.relpath(files[-1], REPO)


def param_checksum(net):
    """(sha256 of every parameter's bytes, float64 sum): replicas of a data-parallel run must be
    bit-identical (every rank applies the same reduced gradient / gathers the same shards)."""
    import hashlib
    h = hashlib.sha256()
    tot = 0.0
    for W, b in net.linear_params():
        for a in (W, b):
            a = np.ascontiguousarray(a, np.float32)
            h.update(a.tobytes())
            tot += float(a.sum(dtype=np.float64))
    return h.hexdigest()[:16], repr(tot)


def roofline_shape(dims):
    """the dominant kernel's layer shape: the 2048x2048 hidden layers of the metric / dnn5 networks, else
    the layer with the most weights (MLP3: the 598x1024 input layer)"""
    shapes = [(dims[i], dims[i + 1]) for i in range(len(dims) - 1)]
    if (2048, 2048) in shapes:
        return ":2048x2048"
    ni, no = max(shapes, key=lambda s: s[0] * s[1])
    return f":{ni}x{no}"


def parse_kernel_report(text):
    out = {}
    for line in text.strip().splitlines():
        tag, n, ms, work = line.split()
        if tag.startswith("@runs:"):
            out["@runs"] = {"runs": int(tag[6:]), "launches": int(n), "ms": float(ms), "work": float(work)}
            continue
        out[tag] = {"launches": int(n), "ms": float(ms), "work": float(work)}
    return out


def mapped_runtime():
    """the HIP runtime / RCCL this process actually mapped (with torch installed,
    tnet_amd binds torch's bundled libamdhip64 / librccl, whose collective kernels' footprint is in
    profiles/r04_rccl_footprint.json)"""
    seen = {}
    try:
        for line in open("/proc/self/maps"):
            p = line.split()[-1]
            for key in ("librccl", "libamdhip64"):
                if key in p:
                    seen[key] = os.path.realpath(p)
    except OSError:
        pass
    return seen


def dp_mode(world):
    """the RCCL exchange's form (RcclExchange: all-reduce unless TNET_DP_SHARD=1)"""
    shard = os.environ.get("TNET_DP_SHARD", "0") == "1"
    return (" (RCCL reduce-scatter, sharded SGD apply, all-gather)" if shard else " (RCCL all-reduce)")


def prewarm_steps(ms, dims, bunch):
    """Training steps of the same network shape on a SCRATCH network, objective, trainer and 8-bunch synthetic cache
    (seeds of their own, no exchange), for `ms` of wall time, synchronised every 8 steps: the GPU meets the step's
    own kernel and memory-traffic mix before the warm-up steps (the GEMM-only prewarm left the 20 / 5 window 1-2 %
    under the steady state: profiles/r05_prewarm_ab.json).  Nothing of the measured run's state is touched.
    Returns the time spent (ms)."""
    if ms <= 0:
        return 0.0
    net = build_network(dims, seed=7)
    net.set_learn_rate(0.008)
    net.set_grad_div_frm(True)
    obj = Objective()
    cache = 8 * bunch
    tr = Trainer(net, obj, bunchsize=bunch, cachesize=cache, seed=99, randomize=True)
    X, L = synth_frames(cache, dims[0], dims[-1], seed=4242)
    if lib().tnet_trainer_prefill(tr.h, X.ctypes.data, X.shape[0], X.shape[1], X.shape[1], L.ctypes.data) != cache:
        raise SystemExit("prewarm: prefill took a partial cache")
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        tr.replay(8)
        tnet_amd.synchronize()
    spent = (time.perf_counter() - t0) * 1e3
    del tr, obj, net, X, L
    return spent


def prewarm(ms):
    """Scratch GEMMs of the step's own 2048^2 shape on the library stream for `ms` of wall time (synchronised
    every 8 launches), on buffers of their own: the GPU leaves its idle clock state before the warm-up steps,
    and nothing of the training state (weights, cache, generator) is touched.  Returns the time spent (ms)."""
    if ms <= 0:
        return 0.0
    S = lib().tnet_stream()
    A, Bm, C = (tnet_amd.DeviceArray(1024, 2048), tnet_amd.DeviceArray(2048, 2048), tnet_amd.DeviceArray(1024, 2048))
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            check(lib().tnet_sgemm(b"N", b"N", 1024, 2048, 2048, 1.0, A.ptr, A.stride, Bm.ptr,
                                   Bm.stride, 0.0, C.ptr, C.stride, S), "prewarm sgemm")
        tnet_amd.synchronize()
    spent = (time.perf_counter() - t0) * 1e3
    del A, Bm, C
    return spent


def reduction_checks(args, comm, trainer, dist, rank, world):
    """rccl_check: one extra step after the measured regions whose gradient reductions
    are compared with a float64 gloo sum of the same local gradients (tnet_amd.dpcheck), in the exchange form the run
    uses and -- for an RCCL run at N > 1 in the default all-reduce form, or at any N with --rccl-check-shard 2 -- once
    more in the sharded form (reduce-scatter + sharded apply + all-gather) on a second communicator created with
    TNET_DP_SHARD=1.  The armed steps run the production schedule: the exchange copies each block on the device, on
    the reduction's own stream, and the copies are read back after the step (GradExchange::CaptureLocal).

    The second form is a check of a mode the run did NOT time: whatever goes wrong with it (its communicator, the swap
    into the trainer, the armed step) is recorded under that mode with ok false and an error text, and never ends the
    run -- only a mismatch in the timed mode does (exit 4).  The ranks agree (gloo) that every rank created the second
    communicator before any of them trains on it, so a creation failure on one rank cannot leave the others waiting
    inside a collective."""
    from tnet_amd import dpcheck

    def allreduce64(a):
        if dist is not None:
            import torch
            dist.all_reduce(torch.from_numpy(a))

    def gather(res):
        if dist is None:
            return [res]
        got = [None] * world
        dist.all_gather_object(got, res)
        return got

    def all_ok(flag):
        if dist is None:
            return flag
        import torch
        t = torch.tensor([0.0 if flag else 1.0], dtype=torch.float64)
        dist.all_reduce(t)
        return float(t.item()) == 0.0

    shard = os.environ.get("TNET_DP_SHARD", "0") == "1"
    timed = "reduce-scatter+all-gather" if shard else "all-reduce"
    modes = {timed: dpcheck.merge_ranks(gather(dpcheck.check_step(comm, trainer, allreduce64)))}
    modes[timed]["timed"] = True
    want_shard = (args.comm == "rccl" and not shard and
                  ((world > 1 and args.rccl_check_shard >= 1) or args.rccl_check_shard == 2))
    if want_shard:
        name = "reduce-scatter+all-gather"
        comm2, err = None, None
        os.environ["TNET_DP_SHARD"] = "1"  # read once, at the communicator's creation
        try:
            uid = [Comm.unique_id() if rank == 0 else None]
            if dist is not None:
                dist.broadcast_object_list(uid, src=0)
            comm2 = Comm(rank, world, uid[0])
        except Exception as e:  # noqa: BLE001  (recorded, never fatal: not the timed mode)
            err = f"communicator: {type(e).__name__}: {str(e)[:300]}"
        finally:
            os.environ.pop("TNET_DP_SHARD", None)
        if not all_ok(err is None):
            modes[name] = {"ok": False, "timed": False,
                           "error": err or "another rank failed to create the sharded-form communicator"}
        else:
            res, swapped = None, False
            try:
                trainer.set_comm(comm2)
                swapped = True
                res = dpcheck.check_step(comm2, trainer, allreduce64)
            except Exception as e:  # noqa: BLE001
                err = f"armed step: {type(e).__name__}: {str(e)[:300]}"
            finally:
                try:
                    tnet_amd.synchronize()
                    if swapped:
                        trainer.set_comm(comm)
                except Exception as e:  # noqa: BLE001
                    err = err or f"swap back: {type(e).__name__}: {str(e)[:300]}"
            got = gather({"res": res, "err": err})
            errs = [g["err"] for g in got if g["err"]]
            if errs:
                modes[name] = {"ok": False, "timed": False, "error": errs[0]}
            else:
                modes[name] = dpcheck.merge_ranks([g["res"] for g in got])
                modes[name]["timed"] = False
        if comm2 is not None:
            try:
                comm2.__del__()
            except Exception:  # noqa: BLE001
                pass
    return {"ranks": world, "transport": args.comm if world > 1 else "rccl (one rank)",
            "transport_ranks": comm.transport_ranks(), "librccl": mapped_runtime().get("librccl"),
            "tolerance": dpcheck.TOLERANCE, "capture": "device copies on the reduction's stream (no host sync in the "
                                                       "armed step), read back after it",
            "modes": modes, "timed_mode": timed,
            "max_rel_err": max(m.get("max_rel_err", float("inf")) for m in modes.values()),
            "ok": modes[timed]["ok"], "all_modes_ok": all(m["ok"] for m in modes.values())}


def main():
    # stdout carries exactly the one JSON result line: the native libraries' own prints (RCCL's version
    # banner at communicator creation, on every rank) go to stderr with everything else
    result_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default window: 100 timed steps (~110 ms); a 20-step window (~22 ms) reads 1-2 % lower on the
    # same box (profiles/r02_*): the clock is still settling after a short warmup
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="dnn4", choices=sorted(CONFIGS))
    ap.add_argument("--bunch", type=int, default=1024)
    ap.add_argument("--cache", type=int, default=65536, help="frames resident per GPU")
    ap.add_argument("--lr", type=float, default=1.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="N>1 gradient transport: RCCL over xGMI (the measured path), or 'host' (gloo through "
                         "host memory) to rehearse the multi-process launch on a one-GPU box")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on GPU 0 (with --comm host)")
    ap.add_argument("--force-dp", action="store_true",
                    help="diagnostic: run the data-parallel path (gradient GEMMs + RCCL all-reduce + SGD apply) "
                         "even at N=1, on a one-rank RCCL communicator")
    ap.add_argument("--kernel-timing", type=int, default=1,
                    help="hipEvent timing in the roofline region (K steps after the timed region): 0 off, 1 the "
                         "roofline kernels (2048x2048 GEMMs), one event pair per RUN of back-to-back roofline "
                         "launches (each pair costs stream time), 2 a pair around every roofline launch")
    ap.add_argument("--prewarm-ms", type=float, default=200.0,
                    help="before the warm-up steps: this long of scratch 1024x2048x2048 GEMMs (no training state "
                         "touched) to bring the GPU out of its idle clock state -- from idle the step takes 1.17 ms "
                         "and settles at 1.01 ms only after ~20 ms of load (profiles/r04_warmup_trace.json), longer "
                         "than a 5-step warm-up (20 / 5 window: 966-982 k without, 994-999 k at 40 ms, 1.007-1.009 M "
                         "at 200 ms; 100 / 20: 1.020 M -- profiles/r04_prewarm_ab.json); 0: off")
    ap.add_argument("--prewarm-form", default="steps", choices=["steps", "gemm"],
                    help="steps: training steps of the same shape on a scratch network / trainer (the step's own "
                         "kernel and traffic mix); gemm: the round-4 scratch 2048^2 GEMMs")
    ap.add_argument("--rccl-check-shard", type=int, default=1,
                    help="N > 1 over RCCL: also check the sharded exchange form on a second communicator swapped into "
                         "the trainer (0: off; 2: also at one rank, with --force-dp -- the swap rehearsed on one GPU)")
    ap.add_argument("--breakdown-steps", type=int, default=20,
                    help="extra steps after the timed region with every launch event-timed (kernels field)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dims = CONFIGS[args.config]
    B = args.bunch

    # one GPU per rank: device local_rank; a launcher that leaves each rank only its own device visible
    # gives device 0.  Anything in between would put two ranks on one GPU and report an oversubscribed
    # whole-node number, so it is an error (--same-device is the explicit rehearsal form).
    ndev = ctypes.c_int(0)
    check(lib().tnet_device_count(ctypes.byref(ndev)), "device_count")
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if args.same_device or ndev.value == 1:
        dev = 0
    elif ndev.value >= local_world:
        dev = local_rank
    else:
        raise SystemExit(f"{ndev.value} GPUs visible to rank {rank} for {local_world} local ranks: "
                         "one GPU per rank needed (or --same-device for a host-transport rehearsal)")
    check(lib().tnet_select_gpu(dev), "select_gpu")
    dist = None
    comm = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811  (gloo only: rendezvous, barrier, max)
        dist.init_process_group("gloo")
        if args.comm == "host":
            import torch

            def allreduce(a):
                t = torch.from_numpy(a)
                dist.all_reduce(t)

            comm = Comm.host(rank, world, allreduce)
        else:
            uid = [Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = Comm(rank, world, uid[0])
    elif args.force_dp:
        comm = Comm(0, 1, Comm.unique_id())

    net = build_network(dims)
    net.set_learn_rate(args.lr)
    net.set_grad_div_frm(True)
    obj = Objective()
    trainer = Trainer(net, obj, bunchsize=B, cachesize=args.cache, seed=123 + rank, randomize=True)
    if comm is not None:
        trainer.set_comm(comm)
    X, L = synth_frames(args.cache, dims[0], dims[-1], seed=1000 + rank)
    taken = lib().tnet_trainer_prefill(trainer.h, X.ctypes.data, X.shape[0], X.shape[1], X.shape[1], L.ctypes.data)
    if taken != args.cache:
        raise SystemExit(f"prefill took {taken} rows, expected {args.cache}")
    del X, L

    def barrier():
        tnet_amd.synchronize()
        if dist is not None:
            dist.barrier()

    prewarm_ms = (prewarm_steps(args.prewarm_ms, dims, B) if args.prewarm_form == "steps" else
                  prewarm(args.prewarm_ms))
    trainer.replay(args.warmup)
    barrier()
    # timed region: K steps, no events on the stream (value, ms_per_step)
    t0 = time.perf_counter()
    trainer.replay(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    # roofline region: the next K steps of the same workload with one hipEvent pair around each run of
    # back-to-back roofline kernels (each pair adds ~3 us of stream time, so not inside the value region)
    buf = ctypes.create_string_buffer(1 << 16)
    kern = {}
    roof_shape = roofline_shape(dims)
    if args.kernel_timing:
        # "gemm_*<shape>": the GEMM launches of the roofline shape only (not the data-parallel SGD applies of
        # that shape, which run on the apply stream); runs also close at every exchange step
        check(lib().tnet_kernel_timing_filter(("gemm_*" + roof_shape).encode()), "timing_filter")
        check(lib().tnet_kernel_timing(2 if args.kernel_timing == 1 else 1), "kernel_timing")
        trainer.replay(args.steps)
        check(lib().tnet_kernel_timing(0), "kernel_timing")
        check(lib().tnet_kernel_timing_report(buf, len(buf)), "kernel_timing_report")
        kern = parse_kernel_report(buf.value.decode())
    # per-kernel breakdown (every launch event-timed) in extra steps outside the timed region
    breakdown = {}
    if args.breakdown_steps > 0:
        check(lib().tnet_kernel_timing_filter(b""), "timing_filter")
        check(lib().tnet_kernel_timing(1), "kernel_timing")
        trainer.replay(args.breakdown_steps)
        check(lib().tnet_kernel_timing(0), "kernel_timing")
        check(lib().tnet_kernel_timing_report(buf, len(buf)), "kernel_timing_report")
        breakdown = parse_kernel_report(buf.value.decode())
    # the reduction check: one more step, after every measured region (synchronous copies)
    rccl_check = reduction_checks(args, comm, trainer, dist, rank, world) if comm is not None else None
    if rccl_check is not None and not rccl_check["ok"]:  # the TIMED mode's reductions are wrong: no number
        print("bench: the reduced gradients differ from the gloo float64 sum of the local gradients: " +
              json.dumps(rccl_check), file=sys.stderr)
        raise SystemExit(4)
    if rccl_check is not None and not rccl_check["all_modes_ok"]:
        print("bench: WARNING the untimed sharded-form check failed (recorded in rccl_check.modes): " +
              json.dumps(rccl_check["modes"]), file=sys.stderr)
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    replicas = param_checksum(net)
    if dist is not None:
        got = [None] * world
        dist.all_gather_object(got, replicas)
        if any(g != got[0] for g in got):
            print("bench: parameter replicas differ across ranks after the run: " + json.dumps(got), file=sys.stderr)
            raise SystemExit(3)

    frames = world * args.steps * B
    value = frames / dt
    ms_per_step = 1000.0 * dt / args.steps

    # ---- roofline of the dominant kernel: the 2048x2048 affine-layer GEMMs (fwd + bwd + fused update)
    hid = [v for k, v in kern.items() if k.startswith("gemm_") and k.endswith(roof_shape)]
    roof = None
    if hid:
        # run mode: exact totals of the event-bracketed runs (every launch in a run is a roofline GEMM)
        tot = kern.get("@runs") or {"launches": sum(v["launches"] for v in hid), "ms": sum(v["ms"] for v in hid),
                                    "work": sum(v["work"] for v in hid)}
        launches, ms, flops = tot["launches"], tot["ms"], tot["work"]
        achieved = flops / (ms * 1e-3) / 1e12
        traffic, traffic_src = pmc_traffic() if roof_shape == ":2048x2048" else (None, None)
        ni, no = (int(v) for v in roof_shape[1:].split("x"))
        roof = {"bound": "mfma", "kernel": f"gemm_f32 {roof_shape[1:]} (fwd/bwd/update; a paired update + backward "
                                           "launch counts as its two GEMMs)", "achieved": round(achieved, 2),
                "peak": PEAK_FP32_MFMA, "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_MFMA, 4),
                "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                # fwd: X, Y, W; bwd: E, W, y below, E below; upd: X, E, W read + write
                "algorithmic_bytes_per_launch": 4.0 * ((B * ni + B * no + ni * no) + (B * no + 2 * B * ni + ni * no) +
                                                       (B * ni + B * no + 2 * ni * no)) / 3,
                "launches": launches, "avg_launch_us": round(1000.0 * ms / launches, 2),
                "timing": (f"hipEvent pairs on the library stream around each run of back-to-back roofline launches "
                           f"({kern['@runs']['runs']} runs), {args.steps} steps right after the value region"
                           if "@runs" in kern else
                           f"hipEvent pairs on the library stream around each roofline launch, {args.steps} steps "
                           "right after the value region"),
                "flops_per_launch": flops / launches}
    breakdown.pop("@runs", None)
    all_gemm_ms = sum(v["ms"] for k, v in breakdown.items() if k.startswith("gemm_"))
    all_ms = sum(v["ms"] for v in breakdown.values())
    kernels = {k: {"launches": v["launches"], "avg_us": round(1000 * v["ms"] / v["launches"], 2),
                   "rate": round(v["work"] / (v["ms"] * 1e-3) / (1e12 if k.startswith("gemm") else 1e9), 2),
                   "rate_unit": "TFLOP/s" if k.startswith("gemm") else "GB/s"} for k, v in sorted(breakdown.items())}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import cpu_baseline
        try:
            cpu = cpu_baseline.reference_cpu_baseline(dims, bunch=B, threads=args.cpu_threads or None)
        except Exception as e:  # measurement infrastructure failure must not kill the GPU line
            cpu = {"error": str(e)[:300]}
        if cpu is None:
            cpu = cpu_baseline.port_cpu_baseline(dims, bunch=B)

    if rank == 0:
        line = {
            # BASELINE.json's metric for its config (dnn4); the other configs name their own network
            "metric": ("training frames/sec (whole node), 440\u21922048\u00d74\u2192senone MLP, 1/2/4/8 MI355X"
                       if args.config == "dnn4" else
                       f"training frames/sec (whole node), {'x'.join(map(str, dims))} MLP"),
            "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "prewarm": {"ms": round(prewarm_ms, 1), "form": args.prewarm_form,
                        "what": ("training steps of the same shape on a scratch network / trainer / cache"
                                 if args.prewarm_form == "steps" else "scratch 1024x2048x2048 GEMMs") +
                        " before the warm-up steps (no state of the measured run touched): the GPU out of its idle "
                        "clock state, whose ramp outlasts a 5-step warm-up (profiles/r04_warmup_trace.json, "
                        "profiles/r05_prewarm_ab.json); --prewarm-ms 0 reports the cold window"},
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"TNet SGD step, {'x'.join(map(str, dims))} sigmoid MLP + softmax xent",
                       "bunch_per_gpu": B, "global_bunch": B * world, "frames_resident_per_gpu": args.cache,
                       "parallelism": f"dp{world}" + ((dp_mode(world) if args.comm == "rccl" else
                                                       " (host all-reduce rehearsal)")
                                                      if world > 1 or args.force_dp else ""),
                       "flops_per_frame": flops_per_frame(dims),
                       "achieved_tflops_whole_step": round(value * flops_per_frame(dims) / 1e12 / world, 2),
                       "whole_step_frac_of_fp32_peak": round(value * flops_per_frame(dims) / 1e12 / world /
                                                             PEAK_FP32_MFMA, 4),
                       "gemm_share_of_kernel_time": round(all_gemm_ms / all_ms, 4) if all_ms else None},
            "roofline": roof,
            "cpu_baseline": cpu,
            "replica_check": {"ranks": world, "identical": True, "param_sha256_16": replicas[0],
                              "param_sum": replicas[1]},
            "rccl_check": rccl_check,
            "runtime": mapped_runtime(),
            "kernels": kernels,
            "kernels_note": f"every launch event-timed, {args.breakdown_steps} extra steps after the timed region "
                            "(event pairs add stream time: the value region has none, the roofline region times "
                            "only the roofline kernels)",
        }
        os.write(result_fd, (json.dumps(line) + "\n").encode())
    # release the library objects in dependency order (trainer -> objective / network -> communicator)
    # while the HIP runtime and the process group are still up
    tnet_amd.synchronize()
    for name in ("trainer", "obj", "net", "comm"):
        if os.environ.get("TNET_BENCH_TRACE_TEARDOWN"):
            print(f"teardown {name}", file=sys.stderr, flush=True)
        locals_ = {"trainer": trainer, "obj": obj, "net": net, "comm": comm}
        o = locals_[name]
        if o is not None:
            o.__del__()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if os.environ.get("TNET_BENCH_TRACE_TEARDOWN"):
        print("teardown done", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
