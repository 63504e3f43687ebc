#!/usr/bin/env python3
"""How rounding-sensitive is one input of one-stage interior-point DDP (ddp(ocp, u, x0, bp),
D:98-186)?  Runs the oracle restatement (oracle/noc_oracle.py: ddp) once as is and SEEDS times with
every derivative array and every total cost perturbed by one ulp at random on every evaluation --
the size of the difference between two correct fp64 implementations of the same formulas (the
device kernels evaluate the derivatives with generated straight-line code, the oracle with
torch.func autodiff; their costs sum in different orders).  Prints the iteration counts, the
final controls' max |dU| and the final cost's relative spread against the unperturbed run: the
envelope inside which ANY correct implementation's result lies for this input.  CPU only.
Usage: ddp_jitter_envelope.py [problem N seed bp SEEDS]  (default pendulum 20 5 5e-5 30)"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ip-parallel-optimal-control_amd"), ROOT]
import numpy as np
from noc import problems
from oracle import noc_oracle as O, problems as PR


class Jitter(O.NumpyProblem):
    def __init__(self, tocp, seed):
        super().__init__(tocp)
        self.rng = np.random.default_rng(seed)

    def _j(self, a):
        a = np.asarray(a, dtype=np.float64)
        towards = np.where(self.rng.random(a.shape) < 0.5, np.inf, -np.inf)
        return np.where(self.rng.random(a.shape) < 0.5, np.nextafter(a, towards), a)

    def derivatives(self, X, U, bp):
        return tuple(self._j(t) for t in super().derivatives(X, U, bp))

    def total_cost(self, X, U, bp):
        return float(self._j(super().total_cost(X, U, bp)))


def envelope(name="pendulum", N=20, seed=5, bp=5e-5, seeds=30):
    x0, u0 = problems.initial_conditions(name, N, 1, seed=seed)
    ocp = PR.pendulum_ocp(1.0 / N) if name == "pendulum" else PR.cartpole_ocp(1.0 / N)
    base = O.NumpyProblem(ocp)
    X0, U0, it0, p0 = O.ddp(base, u0[0], x0[0], bp)
    c0 = base.total_cost(X0, U0, bp)
    its, dus, dcs = [], [], []
    for s in range(100, 100 + seeds):
        X, U, it, _ = O.ddp(Jitter(ocp, s), u0[0], x0[0], bp)
        its.append(int(it))
        dus.append(float(np.max(np.abs(U - U0))))
        dcs.append(float(abs(base.total_cost(X, U, bp) - c0) / abs(c0)))
    return dict(problem=name, N=N, seed=seed, bp=bp, seeds=seeds, oracle_iterations=int(it0),
                oracle_cost=float(c0), jittered_iterations=sorted(its),
                max_abs_dU=max(dus), median_abs_dU=float(np.median(dus)),
                max_rel_dcost=max(dcs), median_rel_dcost=float(np.median(dcs)))


if __name__ == "__main__":
    a = sys.argv[1:]
    out = envelope(a[0], int(a[1]), int(a[2]), float(a[3]), int(a[4])) if len(a) >= 5 else envelope()
    print(json.dumps(out, indent=1))
