"""The data-parallel reduction check (bench.py rccl_check): one training step whose gradient reductions are verified
against an independent sum.

The product's exchange (trainer.cpp RcclExchange) reduces every layer's gradient in place with RCCL over xGMI, on a
communication stream ordered by fence-free events.  A wrong reduction (a stale operand, a missed wait) would hand
every rank the SAME wrong sum, so the replicas stay identical and bench.py's parameter checksum cannot see it.
Here the exchange is armed for one step (Comm.capture): each gradient block is copied on the device right before its
reduction (the rank's local gradient) and right after it (the reduced values over the ranges the rank applies), on
the stream the reduction runs on, into buffers allocated when arming -- the armed step runs the production schedule,
with no host synchronisation and no allocation inside it -- and read back after the step; the local copies are then
summed over the ranks in float64 through a second transport (gloo) and compared with what RCCL produced.  The reference's reduction this stands for is the CPU Platform's row-sliced, double-accumulated sum
of the threads' gradients (src/TNetLib/Platform.h:307-335).

Tolerance: ||rccl - sum64|| / ||sum64|| <= 1e-5 per block over the compared elements (a float32 sum of N terms in
any order is within ~N * 6e-8 of the exact sum in that norm).
"""
from typing import Callable, List, Sequence, Tuple

import numpy as np

TOLERANCE = 1e-5


def compare_reduction(blocks: Sequence[Tuple[np.ndarray, np.ndarray]],
                      allreduce64: Callable[[np.ndarray], None]) -> dict:
    """blocks: [(local float32, reduced float32 with NaN outside this rank's applied ranges)] in submission order
    (every rank holds the same block sequence); allreduce64(a) sums a float64 array over the ranks in place.
    Returns this rank's {"blocks", "elements", "max_rel_err", "worst_block"} (collective: every rank must call)."""
    worst, worst_i, elements = 0.0, -1, 0
    for i, (loc, red) in enumerate(blocks):
        if loc.shape != red.shape:
            raise ValueError(f"block {i}: local {loc.shape} vs reduced {red.shape}")
        ref = np.ascontiguousarray(loc, np.float64).copy()
        allreduce64(ref)
        m = ~np.isnan(red)
        elements += int(m.sum())
        diff = red[m].astype(np.float64) - ref[m]
        nrm = float(np.linalg.norm(ref[m]))
        err = float(np.linalg.norm(diff)) / nrm if nrm > 0 else float(np.linalg.norm(diff))
        if not np.isfinite(err):
            err = float("inf")
        if err > worst or worst_i < 0:
            worst, worst_i = err, i
    return {"blocks": len(blocks), "elements": elements, "max_rel_err": worst, "worst_block": worst_i}


def check_step(comm, trainer, allreduce64: Callable[[np.ndarray], None]) -> dict:
    """arm `comm`, train ONE step through `trainer` (Trainer.replay), compare the step's reductions"""
    comm.capture(True)
    trainer.replay(1)
    blocks = comm.captured()
    comm.capture(False)
    if not blocks:
        raise RuntimeError("reduction check: the step submitted no gradient blocks")
    return compare_reduction(blocks, allreduce64)


def merge_ranks(results: List[dict]) -> dict:
    """the per-rank results of one mode (all_gather_object) -> the worst over ranks"""
    worst = max(results, key=lambda r: r["max_rel_err"])
    return {"blocks": results[0]["blocks"], "elements_per_rank": [r["elements"] for r in results],
            "max_rel_err": worst["max_rel_err"], "worst_block": worst["worst_block"],
            "ok": all(r["max_rel_err"] <= TOLERANCE for r in results)}
