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
