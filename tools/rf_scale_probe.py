import time, sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
from ate_replication_causalml_amd.models import forest as F
dev = torch.device('cuda', 0)
for n, p, nt in [(200000, 100, 64), (1000000, 100, 64), (1000000, 500, 64)]:
    rs = np.random.RandomState(0)
    X = rs.randn(n, p).astype(np.float64)
    y = (X[:, 0] + 0.5 * X[:, 1] + rs.randn(n) > 0).astype(np.float64)
    t = time.perf_counter()
    Xd = torch.as_tensor(X, device=dev)
    edges = F.bin_edges_device(Xd)
    Xb = F.bin_matrix(Xd, *edges, dev)
    torch.cuda.synchronize()
    tb = time.perf_counter()
    F.fit_forest_binned(Xb, edges, F.KIND_CLASS, y=torch.as_tensor(y, device=dev), ntree=nt,
                        seed=1)
    torch.cuda.synchronize()
    tg = time.perf_counter()
    f = F.rf_classifier(X, y, num_trees=nt, seed=1, backend="gpu")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    pr = f.oob_proba()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"n={n} p={p} trees={nt}: device bin {tb-t:.2f}s grow {tg-tb:.2f}s "
          f"rf_classifier {t1-tg:.2f}s oob {t2-t1:.2f}s", flush=True)
