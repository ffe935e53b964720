"""Debug: 4-plane dense stats vs the exact numpy model on the clustered alignment."""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import weightedld_amd as W
from test_gpu_screen import clustered, exact_model_dense
buf = clustered(1500, 2000, 3, 1900, 0.9)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
L = buf.shape[0]
iu = np.triu_indices(L, 1)
for rep in range(3):
    ctx = W.Context(0, W.KERNEL_MFMA)
    ctx.load(buf, w)
    st = ctx.stats()
    d = ctx.dense(L)
    m = exact_model_dense(buf, w, st["weight_shift"])
    v = m[3][iu] == 1
    bad = v & ~((d[0][iu].view(np.uint32) == m[0][iu].view(np.uint32)) | (np.isnan(d[0][iu]) & np.isnan(m[0][iu])))
    a, b = iu[0][bad], iu[1][bad]
    print("rep", rep, "planes", st["mfma_planes"], "shift", st["weight_shift"], "bad", int(bad.sum()))
    for x, y in list(zip(a, b))[:20]:
        print("  a=%d b=%d tile=(%d,%d) a%%64=%d b%%64=%d gpu=%g model=%g" % (x, y, x // 64, y // 64, x % 64, y % 64, d[0][x, y], m[0][x, y]))
    ctx.close()
q = np.rint(np.ldexp(w.astype(np.float64), st["weight_shift"])).astype(np.int64)
print("q range", q.min(), q.max(), "weights min/max", w.min(), w.max())
