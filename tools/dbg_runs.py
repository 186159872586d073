import sys, numpy as np, torch
sys.path.insert(0, "reed-solomon-erasure_amd"); sys.path.insert(0, ".")
import reed_solomon_erasure as R
from reed_solomon_erasure.core import last_kernel
from oracle import oracle as O
lib = R._lib.load()
k, p, field, lost = 10, 4, 8, (0, 1)
T, es, n, stripes = k + p, 1, 16384 + 4096 + 64, 32
rng = np.random.default_rng(1)
oc = O.Codec(field, k, p)
flat = np.zeros((stripes, T, n), np.uint8)
for s in range(stripes):
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] + [np.zeros(n, np.uint8) for _ in range(p)]
    oc.encode(sh); flat[s] = np.stack(sh)
lib.rse_set_option(9, 2)
pres = np.ones((stripes, T), bool); pres[:, list(lost)] = False
work = flat.copy(); work[~pres] = 0
d = torch.from_numpy(work.reshape(-1)).cuda()
r = R.core.ReedSolomon(k, p, field)
p0 = lib.rse_get_option(12)
r.reconstruct_batch(d, n, stripes, pres, data_only=False)
torch.cuda.synchronize()
print("pattern launches", lib.rse_get_option(12) - p0, "last", last_kernel(), "jit modules", lib.rse_get_option(10))
print("ok bytes", (d.cpu().numpy().reshape(stripes, T, -1) == flat).all())
# same pattern through reconstruct_data_flat (flat_reconstruct directly)
work2 = flat.copy(); work2[~pres] = 0
d2 = torch.from_numpy(work2.reshape(-1)).cuda()
p0 = lib.rse_get_option(12)
for it in range(2):
    r.reconstruct_data_flat(d2, n, stripes, pres[0].tolist())
    torch.cuda.synchronize()
    print("data_flat", it, "pattern launches", lib.rse_get_option(12) - p0, "last", last_kernel(), "modules", lib.rse_get_option(10))
torch.cuda.synchronize()
print("flat pattern launches", lib.rse_get_option(12) - p0, "last", last_kernel())
