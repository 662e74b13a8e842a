import sys, numpy as np
sys.path.insert(0,'/root/repo/tests'); sys.path.insert(0,'/root/repo/oracle'); sys.path.insert(0,'/root/repo/sift-scale-space-extrema-detection_amd')
import oracle as orc, sift_amd
from golden_util import Golden
g = Golden('blob256x256_o3_s4'); P=g.params
p = sift_amd.make_params(P['num_octaves'], P['scales_per_octave'])
ctx = sift_amd.Context(0)
ctx.build_scale_space(g.img, p)
r = orc.OracleRun(g.img, orc.make_params(3,4), orc.CONV_SEPARABLE)
for o in range(3):
    for s in range(6):
        D = ctx.plane(sift_amd.PLANE_DOG, o, s).astype(np.float64)
        d = np.abs(D - r.dog[o][s]); i = np.unravel_index(np.argmax(d), d.shape)
        print('dog', o, s, 'maxdiff %.3e at %s' % (d.max(), i), 'n>1e-6:', int((d>1e-6).sum()))
    for s in range(7):
        G = ctx.plane(sift_amd.PLANE_GAUSS, o, s).astype(np.float64)
        d = np.abs(G - r.gauss[o][s]); print('gauss', o, s, 'maxdiff %.3e' % d.max())
c, low = ctx.find_extrema()
print('low', low, 'oracle', r.n_low, 'cands', len(c), r.cand_rec.shape[0], ctx.counts())
# oracle extrema on GPU fp32 DoG planes
flat = np.concatenate([ctx.plane(sift_amd.PLANE_DOG, o, s).astype(np.float64).ravel() for o in range(3) for s in range(6)])
import ctypes
lowc = ctypes.c_long(0)
n = orc.lib().oracle_find_extrema(ctypes.byref(orc.make_params(3,4)), 256, 256, flat.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), None, None, 0, ctypes.byref(lowc))
print('oracle on gpu fp32 planes: cand', n, 'low', lowc.value)
