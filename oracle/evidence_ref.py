"""Restatement of Evidence.Make(MO).evidence_direct / evidence_lebesgue (evidence.ml:66-221) and
the Kd_tree.tree_of_objects it builds on (kd_tree.ml:72-175) -- TEST INFRASTRUCTURE ONLY (the
checker of libmcg's mcg_evidence_direct / mcg_evidence_lebesgue).

Written as the reference is, on Python lists of samples (value tuple, ll, lp): stable list
partitions, an explicit tree with object lists, collect_subvolumes with List.rev_append order.
Pure-Python loops: for the small sample sets of the tests."""
import math
from functools import cmp_to_key


def _cmp(a, b):
    return (a > b) - (a < b)


def bounds_of_objects(objs):                       # kd_tree.ml:93-106
    low = list(objs[0][0])
    high = list(low)
    for v, _, _ in objs[1:]:
        for i in range(len(low)):
            if v[i] < low[i]:
                low[i] = v[i]
            if v[i] > high[i]:
                high[i] = v[i]
    return low, high


def bounds_volume(low, high):                      # kd_tree.ml:177-182
    v = 1.0
    for lo, hi in zip(low, high):
        v = v * (hi - lo)
    return v + 0.0


def find_ith(key, i, objs):                        # kd_tree.ml:72-87 (the order statistic)
    return sorted(objs, key=key)[i]


def tree_of_objects(objs):                         # kd_tree.ml:155-175 -> (objs, left, right) | None
    if not objs:
        return None
    if len(objs) == 1 or all(o[0] == objs[0][0] for o in objs[1:]):
        return (objs, None, None)
    n = len(objs)
    low, high = bounds_of_objects(objs)
    dim, dxm = -1, -math.inf
    for i in range(len(low)):                      # longest_dim (kd_tree.ml:120-130)
        if high[i] - low[i] > dxm:
            dim, dxm = i, high[i] - low[i]
    key = lambda o: o[0][dim]
    pvt = find_ith(key, n // 2, objs)
    lte = [o for o in objs if key(o) <= key(pvt)]
    gt = [o for o in objs if key(o) > key(pvt)]
    if not gt:                                     # adjust_for_empty_split (kd_tree.ml:144-153)
        mx = lte[0]
        for o in lte[1:]:
            if key(o) > key(mx):
                mx = o
        gt = [o for o in lte if key(o) >= key(mx)]
        lte = [o for o in lte if key(o) < key(mx)]
    return (objs, tree_of_objects(lte), tree_of_objects(gt))


def collect_subvolumes(nmax, t):                   # evidence.ml:80-86
    if t is None:
        return []
    objs, left, right = t
    if len(objs) < nmax:
        return [t]
    return list(reversed(collect_subvolumes(nmax, left))) + collect_subvolumes(nmax, right)


def mean_sample(f, objs):
    s = 0.0
    for o in objs:
        s = s + f(o)
    return s / len(objs)


def median_sample(f, objs):
    ss = sorted(objs, key=f)
    n = len(ss)
    if n % 2 == 0:
        return 0.5 * (f(ss[n // 2 - 1]) + f(ss[n // 2]))
    return f(ss[n // 2])


def _samples(pts, ll, lp):
    return [(tuple(float(v) for v in p), float(a), float(b)) for p, a, b in zip(pts, ll, lp)]


def evidence_direct(pts, ll, lp, n=64):            # evidence.ml:145-156
    samples = _samples(pts, ll, lp)
    srt = sorted(samples, key=cmp_to_key(lambda a, b: _cmp(a[0], b[0])))
    rev = []                                       # rev_remove_dups compare_samples
    for k, x in enumerate(srt):
        if k + 1 == len(srt) or x[0] != srt[k + 1][0]:
            rev.insert(0, x)
    t = tree_of_objects(rev)
    integral = 0.0
    for objs, _, _ in collect_subvolumes(n, t):
        low, high = bounds_of_objects(objs)
        integral = integral + bounds_volume(low, high) * mean_sample(lambda o: math.exp(o[1] + o[2]), objs)
    return integral


def evidence_lebesgue(pts, ll, lp, n=64, eps=0.1):  # evidence.ml:194-221
    samples = sorted(_samples(pts, ll, lp), key=lambda o: -o[1])
    col = []
    for k, x in enumerate(samples):                # collect_samples_up_to_eps
        col.append(x)
        if k + 1 < len(samples) and math.exp(-samples[k + 1][1]) - math.exp(-x[1]) > eps:
            break
    mean_il = mean_sample(lambda o: math.exp(-o[1]), col)
    rev = []                                       # remove_dups_rev
    for k, x in enumerate(col):
        if k + 1 == len(col) or x[1] != col[k + 1][1]:
            rev.insert(0, x)
    t = tree_of_objects(rev)
    pm = 0.0
    for objs, _, _ in collect_subvolumes(n, t):
        low, high = bounds_of_objects(objs)
        pm = pm + math.exp(median_sample(lambda o: o[2], objs)) * bounds_volume(low, high)
    return pm / mean_il


def evidence_harmonic_mean(ll):                    # evidence.ml:101-107, linear space
    linv = 0.0
    for v in ll:
        linv = linv + 1.0 / math.exp(v)
    return len(ll) / linv
