#!/usr/bin/env python3
"""VERDICT r5 item 1 evidence: the armed reduction-check step runs the production schedule.

Run under `rocprofv3 --hip-trace --marker-trace`: a one-rank RCCL data-parallel dnn4 trainer (bench.py --force-dp's
setup, small cache) trains a few steps, then ONE step armed for the reduction check inside a roctx range "armed_step"
(both exchange forms: the all-reduce communicator and a second, sharded one swapped in); the captured blocks are read
back after the range.  `summarize` then lists every HIP API call inside each range: no hipStreamSynchronize /
hipDeviceSynchronize / blocking hipMemcpy may appear between the step's first and last call.

  rocprofv3 --hip-trace --marker-trace --output-format csv -d DIR -o armed -- python3 tools/armed_step_trace.py run
  python3 tools/armed_step_trace.py summarize DIR > profiles/r06_armed_step_hip_trace.json
"""
import ctypes
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
sys.path.insert(0, REPO)

SYNC = ("hipStreamSynchronize", "hipDeviceSynchronize", "hipEventSynchronize", "hipMemcpy", "hipMemcpy2D",
        "hipMemcpyDtoH", "hipMemcpyHtoD", "hipStreamQuery")


def run():
    import numpy as np
    import bench
    import tnet_amd
    from tnet_amd import Comm, Objective, Trainer, dpcheck
    from tnet_amd._lib import lib

    # rocprofiler-sdk's roctx (the legacy libroctx64 is not seen by rocprofv3's --marker-trace); hipGetDeviceCount
    # calls bracket each range too, as sentinels in the HIP trace
    roctx = ctypes.CDLL("/opt/rocm/lib/librocprofiler-sdk-roctx.so")
    roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
    ndev = ctypes.c_int(0)

    def sentinel():
        for _ in range(3):
            lib().tnet_device_count(ctypes.byref(ndev))
    dims = bench.CONFIGS["dnn4"]
    net = bench.build_network(dims)
    net.set_learn_rate(1.0)
    net.set_grad_div_frm(True)
    obj = Objective()
    tr = Trainer(net, obj, bunchsize=1024, cachesize=8192, seed=123, randomize=True)
    comm = Comm(0, 1, Comm.unique_id())
    tr.set_comm(comm)
    X, L = bench.synth_frames(8192, dims[0], dims[-1], seed=1000)
    assert lib().tnet_trainer_prefill(tr.h, X.ctypes.data, X.shape[0], X.shape[1], X.shape[1], L.ctypes.data) == 8192
    tr.replay(3)
    tnet_amd.synchronize()
    out = {}
    os.environ["TNET_DP_SHARD"] = "1"
    comm2 = Comm(0, 1, Comm.unique_id())
    os.environ.pop("TNET_DP_SHARD")
    for name, c in (("all-reduce", comm), ("reduce-scatter+all-gather", comm2)):
        tr.set_comm(c)
        tr.replay(1)
        tnet_amd.synchronize()
        c.capture(True)
        sentinel()
        roctx.roctxRangePushA(f"armed_step:{name}".encode())
        tr.replay(1)
        roctx.roctxRangePop()
        sentinel()
        blocks = c.captured()
        c.capture(False)
        out[name] = dpcheck.compare_reduction(blocks, lambda a: None)
    tr.set_comm(comm)
    tnet_amd.synchronize()
    print(json.dumps(out))
    del tr, obj, net, comm2, comm


def summarize(d):
    import csv

    def rows(pattern):
        files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
        if not files:
            raise SystemExit(f"no {pattern} under {d}")
        with open(files[0]) as f:
            return list(csv.DictReader(f))

    hip = rows("*hip_api_trace.csv")
    hip.sort(key=lambda h: int(h["Start_Timestamp"]))
    ranges = []
    try:
        for m in rows("*marker_api_trace.csv"):
            msg = m.get("Function") or m.get("Message") or ""
            if msg.startswith("armed_step"):
                ranges.append((msg, int(m["Start_Timestamp"]), int(m["End_Timestamp"])))
    except SystemExit:
        pass
    if not ranges:  # the sentinels: three hipGetDeviceCount calls on either side of each armed step
        idx = [i for i, h in enumerate(hip) if h["Function"] == "hipGetDeviceCount"]
        runs, cur = [], []
        for i in idx:
            if cur and i != cur[-1] + 1:
                runs.append(cur)
                cur = []
            cur.append(i)
        if cur:
            runs.append(cur)
        runs = [r for r in runs if len(r) == 3]
        for k, name in zip(range(0, len(runs) - 1, 2), ("armed_step:all-reduce", "armed_step:reduce-scatter+all-gather")):
            ranges.append((name + " (sentinels)", int(hip[runs[k][-1]]["End_Timestamp"]),
                           int(hip[runs[k + 1][0]]["Start_Timestamp"])))
    res = {}
    for msg, t0, t1 in ranges:
        inside = [h for h in hip if t0 <= int(h["Start_Timestamp"]) <= t1]
        counts = {}
        for h in inside:
            counts[h["Function"]] = counts.get(h["Function"], 0) + 1
        res[msg] = {"range_us": (t1 - t0) / 1e3, "hip_calls": len(inside), "by_function": counts,
                    "host_syncs": {k: v for k, v in counts.items() if k in SYNC}}
    print(json.dumps({"what": "HIP API calls inside each armed reduction-check step (rocprofv3 --hip-trace "
                              "--marker-trace, tools/armed_step_trace.py): the production schedule has no host "
                              "synchronisation inside a step", "ranges": res,
                      "ok": bool(res) and all(not r["host_syncs"] for r in res.values())}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2])
