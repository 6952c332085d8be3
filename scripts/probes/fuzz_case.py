"""Re-run one tests/test_gpu_fuzz.py MH case and show where the GPU and oracle states differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mcmc-ocaml_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402
from mcmc_amd import targets as T  # noqa: E402

O.build()
i = int(sys.argv[1])
case = F.MH_CASES[i]
print(case)
got = {}


def fake_assert(g, o):
    got["g"], got["o"] = g, o


F.assert_same = fake_assert
F.test_mh_random_combinations_bit_exact(O, T, case)
g, o = got["g"], got["o"]
for key in ("ll0", "lp0", "bits", "rec_x", "rec_ll", "rec_lp", "x", "ll"):
    a, b = np.asarray(g[key]), np.asarray(o[key])
    if a.shape != b.shape:
        print(key, "shape", a.shape, b.shape)
        continue
    bad = np.argwhere(a != b)
    print(key, a.shape, "mismatches", len(bad), bad[:8].tolist())
x, lx = np.asarray(g["x"]), np.asarray(o["x"])
bad = np.argwhere(x != lx)
if len(bad):
    d, c = bad[0]
    print("first: dim", d, "chain", c, "gpu", x[d, c], "oracle", lx[d, c], "last rec gpu", np.asarray(g["rec_x"])[-1][d, c])
    print("dims", sorted(set(bad[:, 0].tolist()))[:20], "chains", len(set(bad[:, 1].tolist())))
print("nacc", g["nacc"], int(o["nacc"].sum()))
