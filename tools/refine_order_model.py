"""Cache model of the fast refinement's DoG gathers (r2g): lines missed by
8 per-XCD LRU L2s (4 MiB each) over the 4K O4 S5 candidate list, in list
order vs (octave, band, scale) order.  Input: the oracle's candidate records
saved as rec.npy (octave, scale, x, y) -- e.g. oracle.extrema_lists on the
bench image (blob_image(3840, 2160, seed=42)).  usage: refine_order_model.py rec.npy
"""
import sys
import numpy as np, collections
rec = np.load(sys.argv[1] if len(sys.argv) > 1 else 'rec.npy')  # octave, scale, x, y
W, H, O, S = 3840, 2160, 4, 5
dims = []; h, w = 2*H, 2*W
for o in range(O):
    if o: h, w = (h+1)//2, (w+1)//2
    dims.append((h, w))
off = np.cumsum([0] + [h*w*(S+2) for h, w in dims])
o, s, x, y = rec[:,0].astype(np.int64), rec[:,1].astype(np.int64), rec[:,2].astype(np.int64), rec[:,3].astype(np.int64)
hh = np.array([d[0] for d in dims])[o]; ww = np.array([d[1] for d in dims])[o]
segs = []
for ds in (-1, 0, 1):
    for dy in (-1, 0, 1):
        base = (off[o] + ((s+ds)*hh + (y+dy))*ww) * 4
        a0 = (base + (x-1)*4) // 128; a1 = (base + (x+1)*4) // 128
        segs.append((a0, a1))
N = len(rec)
print('N', N, 'octave counts', np.bincount(o))
def lines_of(i):
    out = []
    for a0, a1 in segs:
        out.append(a0[i]);
        if a1[i] != a0[i]: out.append(a1[i])
    return out
total = sum(int((a0 != a1).sum()) + N for a0, a1 in segs)
allines = np.concatenate([np.concatenate([a0, a1]) for a0, a1 in segs])
print('touches (lines)', total, 'MB', total*128/1e6, 'distinct', len(np.unique(allines)), 'MB', len(np.unique(allines))*128/1e6)
def sim(order, name, cap=32768, nx=8, blk=256):
    # XCD-contiguous ranges of blocks, LRU per XCD
    nb = (N + blk - 1)//blk
    q, r = divmod(nb, nx)
    miss = 0
    for xc in range(nx):
        b0 = xc*q + min(xc, r); b1 = b0 + q + (1 if xc < r else 0)
        lru = collections.OrderedDict()
        for i in order[b0*blk:min(N, b1*blk)]:
            for a0, a1 in segs:
                for a in ((a0[i],) if a0[i] == a1[i] else (a0[i], a1[i])):
                    if a in lru: lru.move_to_end(a)
                    else:
                        miss += 1; lru[a] = 1
                        if len(lru) > cap: lru.popitem(last=False)
    print('%-28s misses %d = %.0f MB' % (name, miss, miss*128/1e6), flush=True)
sim(np.arange(N), 'list order, XCD ranges')
# (o, band of B rows, s, y, x) order
for B in (8, 32, 128):
    key = ((o*10000 + y//B)*10 + s)*100000000 + y*100000 + x
    sim(np.argsort(key, kind='stable'), 'o, %d-row band, s' % B)
