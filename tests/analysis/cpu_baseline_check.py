"""SURVEY §8d / BASELINE.md §3 check, run in the BUILD container only (the reference cannot travel):
the oracle (oracle/nmgp_oracle.py, the bench's cpu_baseline leg) must run the PM2.5-shaped DSVI
iteration within +-10% of the reference's own CPU time before it stands in for the reference on the
GPU box.  Both run the same minibatch (D=5, M=256, B=2000, fp64) with the same thread count:
forward + loss.backward() + Adam step, 3 warm-up then >=10 timed iterations, median reported.
The reference is imported with the two torch-2.x shims of SURVEY §8c (torch.solve, torch.symeig).
Writes profiles/r02_cpu_oracle_vs_reference.json."""
import collections
import json
import os
import platform
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
REF = "/root/reference"


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def batch():
    D, n = 5, 400
    rng = np.random.default_rng(0)
    xs = [np.sort(rng.uniform(0, 1, n))[:, None] for _ in range(D)]
    ys = [rng.standard_normal(n)[:, None] for _ in range(D)]
    return xs, ys, np.linspace(0, 1, 256)


def reference_step(xs, ys, z):
    _Sol = collections.namedtuple("solve", ["solution", "LU"])
    torch.solve = lambda input, A: _Sol(torch.linalg.solve(A, input), None)
    torch.symeig = lambda A, eigenvectors=False, upper=True: torch.linalg.eigh(A, UPLO="U" if upper else "L")
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(REF, "code"))
    import nmgp_dsvi as R
    m = R.NMGP(number_observations=10000, dim_outputs=5, Z=torch.from_numpy(z).unsqueeze(1), seed=22)
    for k in ["length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"]:
        getattr(m, k).data.fill_(-1.0)
        getattr(m, k).requires_grad = False
    opt = torch.optim.Adam(m.parameters(), lr=0.01)
    Xt = [torch.from_numpy(x) for x in xs]
    Yt = [torch.from_numpy(y) for y in ys]

    def step():                          # code/nmgp_dsvi.py:832-854
        opt.zero_grad()
        loss = m(Xt, Yt)
        loss.backward(retain_graph=True)
        opt.step()
    return step


def oracle_step(xs, ys, z):
    from oracle import nmgp_oracle as O
    p = O.new_params(5, 256, seed=22)
    frozen = {"length_scales_tildeell_log", "length_scales_L0_log", "length_scales_L1_log"}
    for k in frozen:
        p[k] = torch.tensor(-1.0, dtype=torch.float64)
    p = {k: v.clone().requires_grad_() for k, v in p.items()}
    state = {}

    def step():                          # bench.py cpu_baseline
        for v in p.values():
            v.grad = None
        loss, _ = O.forward(p, [x[:, 0] for x in xs], [y[:, 0] for y in ys], z, 10000.0, O.TorchNoise())
        loss.backward()
        O.adam_step(p, {k: v.grad for k, v in p.items() if k not in frozen}, state, 0.01)
    return step


def main():
    threads = int(os.environ.get("NMGP_CPU_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    xs, ys, z = batch()
    iters = 13
    torch.manual_seed(0)
    steps = {"reference": reference_step(xs, ys, z), "oracle": oracle_step(xs, ys, z)}
    times = {k: [] for k in steps}
    for it in range(iters):              # interleaved: both see the same load / clock conditions
        for k, f in steps.items():
            t0 = time.time()
            f()
            times[k].append(time.time() - t0)
    ref, orc = times["reference"][3:], times["oracle"][3:]
    r, o = statistics.median(ref), statistics.median(orc)
    rec = {"config": "PM2.5-shaped DSVI iteration (D=5, M=256, B=2000, fp64): forward + backward + Adam",
           "threads": threads, "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
           "reference_median_s": round(r, 4), "oracle_median_s": round(o, 4), "oracle_over_reference": round(o / r, 3),
           "within_10pct": abs(o / r - 1.0) <= 0.10, "timed_iterations": len(ref),
           "reference_s": [round(t, 4) for t in ref], "oracle_s": [round(t, 4) for t in orc]}
    print(json.dumps(rec))
    with open(os.path.join(ROOT, "profiles", "r02_cpu_oracle_vs_reference.json"), "w") as fh:
        json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
