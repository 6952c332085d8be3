import sys, numpy as np
sys.path.insert(0, 'mcmc-ocaml_amd'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import oracle as O
from mcmc_amd import targets as T
from test_gpu_nested import unit_square_gauss, oracle_nested, gpu_nested
lik, pri = unit_square_gauss(T)
g = gpu_nested(lik, pri, 3, nlive=64, nmcmc=20, mode_hopping_frac=0.1, k=1)
o = oracle_nested(O, lik, pri, 3, nlive=64, nmcmc=20, mode_hop=0.1, k=1)
np.savez('gpurun_out/dbg_nested.npz', gll=g.ll, oll=o['ll'], gpts=g[2], opts=o['pts'], gn=g.n_dead, on=o['n_dead'])
d = np.nonzero(g.ll != o['ll'])[0]
print('n_dead', g.n_dead, o['n_dead'], 'first diff idx', d[:10])
for i in d[:5]:
    print(i, repr(g.ll[i]), repr(o['ll'][i]), g[2][i], o['pts'][i])
