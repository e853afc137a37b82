import torch
dev = torch.device("cuda", 0)
A = torch.randn(2, 43, 43, device=dev, dtype=torch.float64)
K = A @ A.transpose(1, 2) + 43 * torch.eye(43, device=dev, dtype=torch.float64)
rk = torch.randn(2, 43, device=dev, dtype=torch.float64)
def t(name, fn):
    fn(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            fn()
        print(name, "OK", flush=True)
    except Exception as e:
        print(name, "FAIL", str(e).splitlines()[0], flush=True)
    torch.cuda.synchronize()
t("cholesky_ex", lambda: torch.linalg.cholesky_ex(K))
L, _ = torch.linalg.cholesky_ex(K)
t("cholesky_solve", lambda: torch.cholesky_solve(rk[:, :, None], L))
t("cholesky", lambda: torch.linalg.cholesky(K))
t("solve_triangular", lambda: torch.linalg.solve_triangular(L, rk[:, :, None], upper=False))
m = torch.rand(2, 1000, device=dev) < 0.5
t("any", lambda: m.any(0))
v = torch.randn(1000, device=dev, dtype=torch.float64)
t("amin_where", lambda: torch.stack([torch.where(m[a], v, torch.full_like(v, 1.0)).amin() for a in range(2)]))
t("index_add", lambda: torch.zeros(2, 5, 5, device=dev).index_add_(0, torch.zeros(3, dtype=torch.long, device=dev), torch.ones(3, 5, 5, device=dev)))
