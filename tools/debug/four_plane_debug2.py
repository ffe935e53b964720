"""Debug: repeat 4-plane dense runs (AUTO context, as in the test) vs the exact model."""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import weightedld_amd as W
import _oracle as O
from test_gpu_screen import clustered, exact_model_dense
buf = clustered(1500, 2000, 3, 1900, 0.9)
w = W.henikoff_weights(W.SiteSet.from_buffer(buf))
L = buf.shape[0]
iu = np.triu_indices(L, 1)
ctx = W.Context(0, W.KERNEL_AUTO)
ctx.load(buf, w)
st = ctx.stats()
m = exact_model_dense(buf, w, st["weight_shift"])
od = O.all_pairs_dense(buf, w)
v = m[3][iu] == 1
print("model vs oracle max |d diff|", np.abs(m[0][iu][v] - od[0][iu][v]).max(), flush=True)
for rep in range(20):
    d = ctx.dense(L)
    bad = v & ~((d[0][iu].view(np.uint32) == m[0][iu].view(np.uint32)) | (np.isnan(d[0][iu]) & np.isnan(m[0][iu])))
    bad2 = v & (np.abs(d[0][iu] - od[0][iu]) > 1e-5)
    a, b = iu[0][bad], iu[1][bad]
    print("rep", rep, "bad vs model", int(bad.sum()), "bad vs oracle", int(bad2.sum()),
          [(int(x), int(y)) for x, y in list(zip(a, b))[:6]], flush=True)
