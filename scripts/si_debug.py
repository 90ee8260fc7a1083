import os, sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'riemannian-interior-point-trust-region-method_amd')
import __graft_entry__ as g; g.build()
import torch, si
from oracle import si_oracle as SI
DS = 'tests/golden/si_1'
D = SI.SIData.load(DS)
x0, y0 = SI.load_start(DS, 'a')
P = SI.SIVectorized(D)
rs = np.random.RandomState(3)
cases = {}
v = P.manifold.projection(x0, rs.randn(3, 5, 5))
for name, y, vv in [('y0_v', np.zeros(16), v), ('y1_v', y0, v),
                    ('y0_vJ', np.zeros(16), v * np.array([1, 0, 0])[:, None, None]),
                    ('y0_vR', np.zeros(16), v * np.array([0, 1, 0])[:, None, None]),
                    ('y0_vQ', np.zeros(16), v * np.array([0, 0, 1])[:, None, None])]:
    eng = si.SIBatch(5, D.N, 16, 1)
    eng.load(D.X, D.XP, D.h, si.expand_constset(np.loadtxt(os.path.join(DS, 'constset.csv'))))
    out = eng.hvp(x0[None], y[None], 0.1, vv[None]).cpu().numpy()[0]
    cases[name] = (out, y, vv)
np.savez('gpurun_out/si_debug.npz', **{k: v[0] for k, v in cases.items()})
for k, (out, y, vv) in cases.items():
    _, _, Hw, _ = P.begin_inner(x0, y, 0.1)
    ref = Hw(vv)
    print(k, [float(np.linalg.norm(out[c] - ref[c]) / (np.linalg.norm(ref[c]) + 1e-300)) for c in range(3)])
