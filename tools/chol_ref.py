import torch, time
for n in (3000, 6000, 12000):
    A = torch.randn(n, n, dtype=torch.float64, device='cuda')
    A = A @ A.T + n * torch.eye(n, dtype=torch.float64, device='cuda')
    for _ in range(2): torch.linalg.cholesky(A)
    torch.cuda.synchronize()
    t0 = time.perf_counter(); R = 5
    for _ in range(R): L = torch.linalg.cholesky(A)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / R
    print(f"n={n} torch.linalg.cholesky fp64: {dt*1e3:.3f} ms  {n**3/3/dt/1e12:.2f} TFLOP/s", flush=True)
    B = torch.randn(n, n, dtype=torch.float64, device='cuda')
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(R): C = A @ B
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / R
    print(f"n={n} dgemm: {dt*1e3:.3f} ms {2*n**3/dt/1e12:.2f} TFLOP/s", flush=True)
