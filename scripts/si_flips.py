import os, sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'riemannian-interior-point-trust-region-method_amd'); sys.path.insert(0, 'tests')
import __graft_entry__ as g; g.build()
import torch, si
from oracle import si_oracle as SI
from parity import BRANCH_KEYS
DS = 'tests/golden/si_1'
D = SI.SIData.load(DS)
PTS = 'abcdefghijklmnopqrst'
xs, ys = zip(*[SI.load_start(DS, p) for p in PTS])
xs, ys = np.stack(xs), np.stack(ys)
eng = si.SIBatch(5, D.N, 16, 20)
eng.load(D.X, D.XP, D.h, si.expand_constset(np.loadtxt(os.path.join(DS, 'constset.csv'))))
opt = {"TRS_solver": "tCG", "manviofun": si.si_manviofun, "tolresid": 0.0, "maxtime": 1e9, "maxiter": 10}
res = eng.solve(xs, ys, opt)
for b in range(20):
    gl = res.log(b)
    rl = SI.solve(D, xs[b], ys[b], dict(tolresid=0.0, maxtime=1e9, maxiter=10, manviofun=SI.si_manvio)).log
    first = None
    for k in BRANCH_KEYS:
        m = min(len(gl[k]), len(rl[k]))
        f = next((i for i in range(m) if gl[k][i] != rl[k][i]), None)
        if f is not None and (first is None or f < first[0]):
            first = (f, k)
    if first is None:
        print(b, 'no flip'); continue
    r, k = first
    print(b, 'row', r, k, 'gpu', gl[k][r], 'ora', rl[k][r], 'normdx', gl['normdx'][r], rl['normdx'][r], 'TR', gl['TR_radius'][r], rl['TR_radius'][r],
          'dx', gl['dxtype'][r], rl['dxtype'][r], 'ared/pred', gl['ared/pred'][r], rl['ared/pred'][r])
