"""CPU, world_size 2 over gloo: the landmark-sharding decomposition the
multi-GPU path relies on.  Each rank owns a contiguous point
range; camera column norms (-> global Jacobi scale), the reduced camera
matrix S and its right-hand side are sums of per-shard contributions, with
the camera diagonal D_c^2 added on rank 0 only -- exactly the all-reduce
protocol of sfm_amd/csrc/ba_solver.hip.  The sum must equal the single-process
system."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from sfm_amd import scene
    from oracle import ffi as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C, P = 8, 240
    per = P // world
    sh = scene.generate(C, P, views=4, seed=99, p_begin=rank * per, p_end=(rank + 1) * per)
    ones_c, ones_p = np.ones((C, 6)), np.ones((per, 3))
    # 1. local camera column norms -> all-reduce -> global Jacobi scale
    _, _, cc, cp = O.reduced_system(sh.uv, sh.cam_idx, sh.pt_idx, sh.K, sh.rot, sh.t, sh.X, ones_c, ones_p,
                                    np.zeros(6 * C), np.zeros(3 * per), add_cam_diag=False)
    cct = torch.tensor(cc)
    dist.all_reduce(cct)
    scale_c = 1.0 / (1.0 + np.sqrt(cct.numpy()))
    scale_p = 1.0 / (1.0 + np.sqrt(cp))
    D_c = np.full(6 * C, 0.05)
    D_p = np.full(3 * per, 0.02)
    # 2. local reduced system with D_c^2 on rank 0 only -> all-reduce
    S, rhs, _, _ = O.reduced_system(sh.uv, sh.cam_idx, sh.pt_idx, sh.K, sh.rot, sh.t, sh.X, scale_c, scale_p,
                                    D_c, D_p, add_cam_diag=(rank == 0))
    St, rt = torch.tensor(S), torch.tensor(rhs)
    dist.all_reduce(St)
    dist.all_reduce(rt)
    if rank == 0:
        q.put((St.numpy(), rt.numpy(), scale_c))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_reduced_system_equals_global():
    from sfm_amd import scene
    from oracle import ffi as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    S_sh, rhs_sh, scale_c = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    C, P = 8, 240
    full = scene.generate(C, P, views=4, seed=99)
    _, _, cc, cp = O.reduced_system(full.uv, full.cam_idx, full.pt_idx, full.K, full.rot, full.t, full.X,
                                    np.ones((C, 6)), np.ones((P, 3)), np.zeros(6 * C), np.zeros(3 * P), False)
    sc = 1.0 / (1.0 + np.sqrt(cc))
    assert np.allclose(sc, scale_c, rtol=1e-13)
    S, rhs, _, _ = O.reduced_system(full.uv, full.cam_idx, full.pt_idx, full.K, full.rot, full.t, full.X, sc,
                                    1.0 / (1.0 + np.sqrt(cp)), np.full(6 * C, 0.05), np.full(3 * P, 0.02), True)
    assert np.allclose(S_sh, S, rtol=1e-11, atol=1e-12 * np.abs(S).max())
    assert np.allclose(rhs_sh, rhs, rtol=1e-11, atol=1e-12 * np.abs(rhs).max())


# ---- the distributed reduced-camera factor (sfm_ba_set_distributed_factor,
# ba_solver.hip dist_factor_enqueue): the same protocol on the host, numpy
# for the device kernels, gloo for the collectives ----
def _panel_layout(n, pw):
    """Panel J = columns [pw J, pw J + pw) of the augmented (n+1)-row system,
    rows c0_J..n, owner J % world, at offset poff[J] of the panel image --
    dist_prepare's arithmetic."""
    npan = (n + 1 + pw - 1) // pw
    count, poff, tot = [], [], 0
    for J in range(npan):
        c0, c1 = J * pw, min((J + 1) * pw, n + 1)
        count.append((c1 - c0) * (n + 1 - c0))
        poff.append(tot)
        tot += count[-1]
    return npan, count, poff, tot


def _pack(A, n, pw, J, buf, off):
    c0, c1 = J * pw, min((J + 1) * pw, n + 1)
    rows = n + 1 - c0
    for c in range(c0, c1):
        buf[off + (c - c0) * rows: off + (c - c0 + 1) * rows] = A[c0:n + 1, c]


def _unpack(A, n, pw, J, buf, off):
    c0, c1 = J * pw, min((J + 1) * pw, n + 1)
    rows = n + 1 - c0
    for c in range(c0, c1):
        A[c0:n + 1, c] = buf[off + (c - c0) * rows: off + (c - c0 + 1) * rows]


def _unpack_add(A, n, pw, J, buf, off):
    c0, c1 = J * pw, min((J + 1) * pw, n + 1)
    rows = n + 1 - c0
    for c in range(c0, c1):
        A[c0:n + 1, c] += buf[off + (c - c0) * rows: off + (c - c0 + 1) * rows]


def _dist_worker(rank, world, port, q, pw):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from sfm_amd import scene
    from oracle import ffi as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C, P = 8, 240
    lo, hi = rank * P // world, (rank + 1) * P // world
    sh = scene.generate(C, P, views=4, seed=99, p_begin=lo, p_end=hi)
    scale_c, scale_p = np.full((C, 6), 0.5), np.full((hi - lo, 3), 0.5)
    S, rhs, _, _ = O.reduced_system(sh.uv, sh.cam_idx, sh.pt_idx, sh.K, sh.rot, sh.t, sh.X, scale_c, scale_p,
                                    np.full(6 * C, 0.05), np.full(3 * (hi - lo), 0.02), add_cam_diag=(rank == 0))
    n = 6 * C
    # this rank's partial augmented system: lower triangle, row n = rhs
    A = np.zeros((n + 1, n + 1))
    A[:n, :n] = np.tril(S)
    A[n, :n] = rhs
    A[n, n] = 1.0
    npan, count, poff, tot = _panel_layout(n, pw)
    # every rank's partial panels, its own ones left zero: the owner updates
    # its partial in place and adds the others' sum just before its factor
    send = np.zeros(tot)
    for J in range(npan):
        if J % world != rank:
            _pack(A, n, pw, J, send, poff[J])
    recv = {}

    def reduce_panel(k):
        if k < npan:
            t = torch.from_numpy(send[poff[k]:poff[k] + count[k]].copy())
            dist.reduce(t, dst=k % world)
            if k % world == rank:
                recv[k] = t.numpy()

    def factor(k):
        c0, c1 = k * pw, min((k + 1) * pw, n + 1)
        _unpack_add(A, n, pw, k, recv.pop(k), 0)
        D = A[c0:c1, c0:c1]
        if c1 <= n:
            L = np.linalg.cholesky(np.tril(D) + np.tril(D, -1).T)
            A[c0:c1, c0:c1] = L
            A[c1:n + 1, c0:c1] = np.linalg.solve(L, A[c1:n + 1, c0:c1].T).T
        else:  # the last panel holds row n: factor the real part, z below it
            m = n - c0
            Lr = np.linalg.cholesky(np.tril(D[:m, :m]) + np.tril(D[:m, :m], -1).T)
            A[c0:n, c0:n] = Lr
            A[n, c0:n] = np.linalg.solve(Lr, A[n, c0:n])
            A[n, n] = 1.0

    def update(k, J):
        c0, c1 = k * pw, min((k + 1) * pw, n + 1)
        j0, j1 = J * pw, min((J + 1) * pw, n + 1)
        Lk = A[c0:n + 1, c0:c1]
        A[j0:n + 1, j0:j1] -= Lk[j0 - c0:, :] @ Lk[j0 - c0:j1 - c0, :].T

    reduce_panel(0)
    reduce_panel(1)
    if rank == 0:
        factor(0)
    for k in range(npan):
        c0 = k * pw
        buf = torch.zeros(count[k], dtype=torch.float64)
        if k % world == rank:
            _pack(A, n, pw, k, buf.numpy(), 0)
        dist.broadcast(buf, src=k % world)
        reduce_panel(k + 2)
        if k % world != rank:
            _unpack(A, n, pw, k, buf.numpy(), 0)
        # look-ahead: the next owner's panel first, then the rest
        if k + 1 < npan and (k + 1) % world == rank:
            update(k, k + 1)
            factor(k + 1)
        for J in range(k + 2, npan):
            if J % world == rank:
                update(k, J)
    # replicated back substitution L^T y = z
    L = np.tril(A[:n, :n])
    y = np.linalg.solve(L.T, A[n, :n])
    q.put((rank, L, y))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,pw", [(2, 8), (2, 16), (3, 8)])
def test_distributed_factor_protocol_equals_global_solve(world, pw):
    """The ranks' partial systems reduced panel by panel into the owners of
    block-cyclic panels (the owner's own partial updated in place, the
    others' sum added just before its factor), per panel the owner's factor
    + a broadcast, every rank updating its own later panels in look-ahead
    order: every rank ends with the factor of the global system and the same
    solution as np.linalg.solve on it."""
    from sfm_amd import scene
    from oracle import ffi as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, q, pw)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    C, P = 8, 240
    full = scene.generate(C, P, views=4, seed=99)
    S, rhs, _, _ = O.reduced_system(full.uv, full.cam_idx, full.pt_idx, full.K, full.rot, full.t, full.X,
                                    np.full((C, 6), 0.5), np.full((P, 3), 0.5), np.full(6 * C, 0.05),
                                    np.full(3 * P, 0.02), True)
    # (the reduced system of a free-gauge BA is ill-conditioned: the factor
    # is checked by its reconstruction and the solution by its residual, both
    # backward-stable quantities, plus a loose forward comparison)
    L_ref = np.linalg.cholesky(S)
    y_ref = np.linalg.solve(S, rhs)
    for _, L, y in res:
        assert np.abs(L @ L.T - S).max() <= 1e-12 * np.abs(S).max()
        assert np.abs(S @ y - rhs).max() <= 1e-10 * np.abs(rhs).max()
        assert np.allclose(L, L_ref, rtol=1e-6, atol=1e-9 * np.abs(L_ref).max())
        assert np.allclose(y, y_ref, rtol=1e-5, atol=1e-9 * np.abs(y_ref).max())
        assert np.array_equal(L, res[0][1]) and np.array_equal(y, res[0][2])  # every rank the same factor
