"""A/B of the nested walker's lanes per walker (MCG_NEST_LANES) on the bench's nested leg (C2
target, D = 32, nlive 32,768, k 2,048, nmcmc 200), the C3 shell (D = 16) and the D = 8 / 64 shell: the same dead
points bit for bit, and the wall time of each setting (interleaved, median of 5).
  python scripts/probes/nest_lanes_ab.py"""
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import os, sys, time, json, hashlib
import numpy as np
sys.path[:0] = [os.path.join(%r, "mcmc-ocaml_amd"), %r]
from bench import c2_target
from mcmc_amd import Context, nested, targets as T
cases = []
D = 32
mu, sg, _ = c2_target(D)
cases.append(("c2d32", T.diag_gauss(mu, sg), T.box(-10 * np.ones(D), 10 * np.ones(D)), 32768, 2048, 200))
cases.append(("c3shell16", T.gauss_shell(np.zeros(16), 2.0, 0.1), T.box(-6 * np.ones(16), 6 * np.ones(16)), 131072, 4096, 100))
for D in (8, 64):
    cases.append(("shell%%d" %% D, T.gauss_shell(np.zeros(D), 2.0, 0.1), T.box(-6 * np.ones(D), 6 * np.ones(D)), 16384, 1024, 100))
res = {}
for name, lik, pri, nlive, k, nmcmc in cases:
    walls = []
    for rep in range(5):
        with Context(seed=7) as ctx:
            t = time.perf_counter()
            out = nested.nested_evidence(lik, pri, nlive=nlive, nmcmc=nmcmc, k=k, mode_hopping_frac=0.1, ctx=ctx)
            walls.append(time.perf_counter() - t)
    h = hashlib.sha1(np.ascontiguousarray(out.ll).tobytes() + np.ascontiguousarray(out[2]).tobytes()).hexdigest()[:16]
    res[name] = dict(logz=out[0], n_dead=int(out.n_dead), n_gen=int(out.n_gen), wall_med=sorted(walls)[2], hash=h)
print(json.dumps(res))
''' % (ROOT, ROOT)

out = {}
for rnd in range(2):
    for lanes in ("narrow", "wide"):
        env = dict(os.environ, MCG_NEST_LANES=lanes)
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stdout, r.stderr)
            sys.exit(r.returncode)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        out.setdefault(lanes, []).append(line)
        print("lanes", lanes, "round", rnd, line, flush=True)
