"""The newbob learning-rate scheduler of tools/train/training_scheduler_xent.sh:56-214, restated.

SURVEY.md section 8(f) row 4 ("epoch scheduler compatibility"): the reference trains one process per
epoch and talks to the driver only through its command line and the ``Report()`` line it prints, so
the scheduler is host-side orchestration.  This module keeps the script's protocol exactly:

* the command lines it builds (``-H <best> -I <mlf> -L '*/' -X lab -S <scp> --LEARNINGRATE=...
  --BUNCHSIZE --CACHESIZE --RANDOMIZE --OUTPUTLABELMAP --TARGETMMF --STARTFRMEXT --ENDFRMEXT
  [--FEATURETRANSFORM]``, cross-validation with ``--RANDOMIZE=FALSE --CROSSVALIDATE=TRUE``,
  training_scheduler_xent.sh:70-150);
* the err/frm parse (the last ``Xent:`` line, ``sed 's|.*err\\/frm:\\([0-9\\.]*\\) .*|\\1|'``,
  :44-52) -- ``parse_xent``;
* the CPU learning-rate division by BUNCHSIZE when THREADS is set (:96-98);
* accept / reject, start halving below START_HALVING_INC relative improvement, stop below
  END_HALVING_INC once halving (after MIN_ITER), KEEP_LRATE_ITER (:160-205) -- ``Newbob.decide``;
* the weight file names ``<base>_iterNN_lr<%.5g>_tr<%.5g>_cv<%.5g>`` and ``_rejected`` (:152-172).

The awk arithmetic of the script is double precision; ``%.5g`` is C printf -- Python's ``%``
formatting is the same printf.  ``awk print`` of the halved learning rate uses OFMT ``%.6g``
(:209), which ``_awk_num`` reproduces, because the next epoch's --LEARNINGRATE is that text.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

_XENT_LINE = re.compile(r"Xent:")
_ERRFRM = re.compile(r".*err/frm:([0-9.]*) .*")


def parse_xent(stdout: str) -> Optional[str]:
    """training_scheduler_xent.sh:49: grep 'Xent:' | tail -n 1 | sed 's|.*err\\/frm:\\([0-9\\.]*\\) .*|\\1|'.
    Returns the text (as the script keeps it) or None when no line matched (the script exits)."""
    lines = [l for l in stdout.splitlines() if _XENT_LINE.search(l)]
    if not lines:
        return None
    m = _ERRFRM.match(lines[-1])
    return m.group(1) if m else lines[-1]          # sed leaves a non-matching line unchanged


def _awk_num(x: float) -> str:
    """awk's print of a number: integers as integers, else OFMT %.6g."""
    if x == int(x) and abs(x) < 1e16:
        return str(int(x))
    return "%.6g" % x


@dataclass
class Iteration:
    iter: int
    lrate: str
    xent_train: str
    xent_cv: str
    accepted: bool
    nnet: str


@dataclass
class Newbob:
    """State machine of training_scheduler_xent.sh:99-205 (decisions only; ``run`` drives binaries)."""
    learnrate: object            # the LEARNRATE text (or a number)
    bunchsize: int = 512
    threads: Optional[int] = None
    max_iter: int = 20
    min_iter: int = 1
    keep_lrate_iter: int = 0
    end_halving_inc: float = 0.1
    start_halving_inc: float = 0.5
    halving_factor: float = 0.5
    history: List[Iteration] = field(default_factory=list)

    def __post_init__(self):
        # :96-98 -- CPU (THREADS set) sums gradients over the bunch, so the rate is per frame
        if self.threads:
            self.lrate = _awk_num(float(self.learnrate) / self.bunchsize)
        else:                                                           # the text as given
            self.lrate = self.learnrate if isinstance(self.learnrate, str) else repr(self.learnrate)
        self.do_halving = False
        self.xent_best: Optional[float] = None
        self.xent_prev: Optional[float] = None
        self.done = False

    def initial(self, xent_cv: str) -> None:
        self.xent_best = float(xent_cv)
        self.xent_best_text = xent_cv

    def decide(self, it: int, xent_train: str, xent_cv: str, nnet: str) -> bool:
        """One iteration's bookkeeping after its train + CV runs; returns whether the weights are
        accepted.  Sets ``done`` when the script would ``break`` and updates ``lrate``."""
        cv = float(xent_cv)
        lr_used = self.lrate
        if it < self.keep_lrate_iter:                                   # :160-167
            accepted = True
            self.xent_prev, self.xent_best, self.xent_best_text = self.xent_best, cv, xent_cv
            self.history.append(Iteration(it, lr_used, xent_train, xent_cv, accepted, nnet))
            return accepted
        if cv < self.xent_best:                                         # :170-179
            accepted = True
            self.xent_prev, self.xent_best, self.xent_best_text = self.xent_best, cv, xent_cv
        else:
            accepted = False
            self.xent_prev = self.xent_best
        self.history.append(Iteration(it, lr_used, xent_train, xent_cv, accepted, nnet))
        # :182-184 end training if halving already and not improving much
        if self.do_halving and 1.0 - self.xent_best / self.xent_prev < self.end_halving_inc and it > self.min_iter:
            self.done = True
            return accepted
        # :188-190 start halving when not improving much
        if 1.0 - cv / self.xent_prev < self.start_halving_inc:
            self.do_halving = True
        if self.do_halving:                                             # :192-195
            self.lrate = _awk_num(float(self.lrate) * self.halving_factor)
        return accepted


def _g5(x: str) -> str:
    """bash's builtin ``printf '%.5g' $x``: the text goes through strtold and is printed from the
    80-bit long double (so "3.47165" prints 3.4717, where the double 3.4716499.. would give 3.4716).
    C's %g: E-style exponent X after rounding; fixed with 4-X decimals if -4 <= X < 5; trailing
    zeros dropped."""
    import numpy as np
    v = np.longdouble(str(x))
    if v == 0:
        return "0"
    mant, exp = np.format_float_scientific(v, precision=4, unique=False).split("e")
    e = int(exp)
    if -4 <= e < 5:
        out = np.format_float_positional(v, precision=4 - e, unique=False, fractional=True, trim="-")
        return out.rstrip(".")
    mant = mant.rstrip("0").rstrip(".")
    return f"{mant}e{'-' if e < 0 else '+'}{abs(e):02d}"


def run(driver: Sequence[str], nn_init: str, mlf_train: str, mlf_cv: str, scp_train: str, scp_cv: str,
        phonelist: str, learnrate, workdir: str, bunchsize: int = 512, cachesize: int = 16384,
        randomize: bool = True, frm_ext: int = 0, feature_transform: Optional[str] = None,
        threads: Optional[int] = None, max_iter: int = 20, min_iter: int = 1, keep_lrate_iter: int = 0,
        end_halving_inc: float = 0.1, start_halving_inc: float = 0.5, halving_factor: float = 0.5,
        extra: Sequence[str] = (), config: Optional[str] = None, env: Optional[dict] = None,
        log: Optional[Callable[[str], None]] = None) -> Newbob:
    """training_scheduler_xent.sh end to end with ``driver`` (TNet / TNetCu / TNetCu_amd argv[0:])."""
    nb = Newbob(learnrate, bunchsize, threads, max_iter, min_iter, keep_lrate_iter, end_halving_inc,
                start_halving_inc, halving_factor)
    os.makedirs(os.path.join(workdir, "weights"), exist_ok=True)
    name = os.path.basename(nn_init)
    base = os.path.join(workdir, "weights", name[:-5] if name.endswith(".init") and len(name) > 5 else name)
    common = ["-L", "*/", "-X", "lab", f"--BUNCHSIZE={bunchsize}", f"--CACHESIZE={cachesize}",
              f"--OUTPUTLABELMAP={phonelist}", f"--STARTFRMEXT={frm_ext}", f"--ENDFRMEXT={frm_ext}"]
    if feature_transform:
        common.append(f"--FEATURETRANSFORM={feature_transform}")
    if config:                                                          # ${STK_CONF:+-C $STK_CONF}
        common += ["-C", config]
    if threads:
        common.append(f"--THREADS={threads}")
    common += list(extra)

    def go(args):
        p = subprocess.run(list(driver) + args + common, capture_output=True, text=True, cwd=workdir, env=env)
        x = parse_xent(p.stdout)
        if p.returncode != 0 or x is None:
            raise RuntimeError("Error, No xentopy returned, terminating...\n" + p.stdout[-2000:] + p.stderr[-2000:])
        if log:
            log(p.stdout)
        return x

    cv_args = ["--RANDOMIZE=FALSE", "--CROSSVALIDATE=TRUE"]
    nb.initial(go(["-H", nn_init, "-I", mlf_cv, "-S", scp_cv] + cv_args))
    nb.initial_cv = nb.xent_best
    best = nn_init
    width = len(str(max_iter))
    for k in range(1, max_iter + 1):
        it = str(k).rjust(width, "0")                                   # seq -w
        nxt = f"{base}_iter{it}"
        tr = go(["-H", best, "-I", mlf_train, "-S", scp_train, f"--LEARNINGRATE={nb.lrate}",
                 f"--RANDOMIZE={'TRUE' if randomize else 'FALSE'}", f"--TARGETMMF={nxt}"])
        cv = go(["-H", nxt, "-I", mlf_cv, "-S", scp_cv] + cv_args)
        named = f"{nxt}_lr{_g5(nb.lrate)}_tr{_g5(tr)}_cv{_g5(cv)}"
        shutil.move(nxt, named)
        if nb.decide(k, tr, cv, named):
            best = named
        else:
            shutil.move(named, named + "_rejected")
        if nb.done:
            break
    # :208-211 copy out the best network
    if nb.history:
        last = nb.history[-1]
        final = f"{base}_final_iters{str(last.iter).rjust(width, '0')}_tr{_g5(last.xent_train)}_cv{_g5(nb.xent_best_text)}"
        shutil.copyfile(best, final)
        nb.final = final
    nb.best = best
    return nb
