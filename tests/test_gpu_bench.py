"""bench.py keeps the driver's contract: one JSON line from rank 0 with BASELINE.json's metric, the
required fields, the roofline object, and (N > 1) the whole-job value of every rank's frames over the
slowest rank's time.  Small windows and caches: this checks the contract and the multi-process launch,
not the number (the number is bench.py's own run, profiles/)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric": str, "value": float, "unit": str, "n_gpus": int, "steps": int, "warmup": int,
            "ms_per_step": float, "higher_is_better": bool, "scaling": str, "dtype": str, "data": str,
            "config": dict}


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _check_contract(d, n, steps, warmup):
    for k, t in REQUIRED.items():
        assert isinstance(d[k], t), (k, d[k])
    assert "vs_baseline" in d and d["vs_baseline"] is None  # BASELINE.md publishes no frames/s figure
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["unit"] == "frames/s" and d["higher_is_better"] and d["scaling"] == "weak"
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value = every rank's frames over the slowest rank's time
    bunch = d["config"]["bunch_per_gpu"]
    assert abs(d["value"] - n * bunch * 1000.0 / d["ms_per_step"]) <= 0.01 * d["value"]
    assert d["config"]["global_bunch"] == n * bunch


def test_bench_contract_one_gpu():
    cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--cache", "4096",
           "--breakdown-steps", "1"]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    _check_contract(d, 1, 3, 1)
    r = d["roofline"]
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s" and r["peak"] == 157.3
    assert 0 < r["frac"] <= 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert "traffic" in r and d["kernels"]


def test_bench_two_ranks_rehearsal():
    """the torch.distributed.run launch the driver uses at N > 1, rehearsed on one GPU (both ranks on
    device 0, gradients summed through host memory): rendezvous, barriers, max-over-ranks timing, teardown"""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--cache", "4096", "--comm", "host", "--same-device", "--kernel-timing", "0",
           "--breakdown-steps", "0"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    _check_contract(d, 2, 2, 1)
    assert d["roofline"] is None  # kernel timing off
    # the reduction check's C++ capture path (HostExchange) at world 2: both ranks' gradients of one step
    c = d["rccl_check"]
    assert c["ok"] and c["ranks"] == 2 and c["transport"] == "host" and c["transport_ranks"] == 2
    assert list(c["modes"]) == ["all-reduce"] and c["modes"]["all-reduce"]["blocks"] == 10
    assert c["max_rel_err"] <= 1e-6


@pytest.mark.parametrize("shard", ["0", "1"])
def test_bench_force_dp_reduction_check(shard):
    """--force-dp at N = 1 (a one-rank RCCL communicator): the reduction check runs through RcclExchange's capture
    (both exchange forms) and the one-rank reduction equals the local gradient exactly"""
    cmd = [sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--cache", "4096",
           "--force-dp", "--kernel-timing", "0", "--breakdown-steps", "0", "--prewarm-ms", "0"]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TNET_DP_SHARD=shard))
    assert p.returncode == 0, p.stderr[-3000:]
    c = _line(p.stdout)["rccl_check"]
    mode = "reduce-scatter+all-gather" if shard == "1" else "all-reduce"
    assert c["ok"] and c["ranks"] == 1 and c["transport_ranks"] == 1 and list(c["modes"]) == [mode]
    assert c["max_rel_err"] == 0.0 and c["modes"][mode]["blocks"] == 10
    assert c["librccl"] and "rccl" in c["librccl"]


def test_shuffle_ahead_bit_identical():
    """the next pass's permutation drawn ahead on a host thread (CuCache, default) and drawn in Randomize itself
    (TNET_SHUFFLE_AHEAD=0) train the same parameters bit for bit over several passes of a 4-bunch cache: the ahead
    shuffle starts from the trainer stream's state and is taken only while the stream still stands there"""
    cmd = [sys.executable, "bench.py", "--config", "mlp3", "--steps", "13", "--warmup", "2", "--no-cpu-baseline",
           "--cache", "4096", "--kernel-timing", "0", "--breakdown-steps", "0", "--prewarm-ms", "0"]
    sha = []
    for env in ({}, {"TNET_SHUFFLE_AHEAD": "0"}):
        p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
        assert p.returncode == 0, p.stderr[-3000:]
        sha.append(_line(p.stdout)["replica_check"]["param_sha256_16"])
    assert sha[0] == sha[1]


@pytest.mark.parametrize("config", ["mlp3", "dnn4"])
def test_dp_exchange_schedules_bit_identical(config):
    """the round-5 exchange schedule (MLP3: the whole reduction inline on the compute stream + one merged apply;
    dnn4: each apply on the comm stream behind its reduction) and the round-4 one (TNET_DP_INLINE=0
    TNET_DP_APPLY_COMM=0: per-layer submissions, applies on their own stream) train the same parameters bit for bit
    (only the streams and launch grouping differ, never the arithmetic)"""
    cmd = [sys.executable, "bench.py", "--config", config, "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--cache", "4096", "--force-dp", "--kernel-timing", "0", "--breakdown-steps", "0", "--prewarm-ms", "0"]
    sha = []
    for env in ({}, {"TNET_DP_INLINE": "0", "TNET_DP_APPLY_COMM": "0"}):
        p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
        assert p.returncode == 0, p.stderr[-3000:]
        d = _line(p.stdout)
        assert d["rccl_check"]["ok"]
        sha.append(d["replica_check"]["param_sha256_16"])
    assert sha[0] == sha[1]


def test_bench_sharded_check_swap_at_one_rank():
    """the second-communicator swap bench.py makes for the sharded-form check at N > 1, rehearsed
    at one rank (--force-dp --rccl-check-shard 2): both forms' armed steps run the production schedule (device
    captures, no host sync inside the step), both compare exactly at one rank, the trainer is handed back its own
    communicator, and the replica checksum still runs after the swap"""
    cmd = [sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--cache", "4096",
           "--force-dp", "--kernel-timing", "0", "--breakdown-steps", "0", "--prewarm-ms", "0",
           "--rccl-check-shard", "2"]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    c = d["rccl_check"]
    assert set(c["modes"]) == {"all-reduce", "reduce-scatter+all-gather"}, c
    assert c["timed_mode"] == "all-reduce" and c["modes"]["all-reduce"]["timed"]
    for m in c["modes"].values():
        assert m["ok"] and m["max_rel_err"] == 0.0 and m["blocks"] == 10, m
    assert c["ok"] and c["all_modes_ok"] and d["replica_check"]["identical"]
