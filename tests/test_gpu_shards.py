"""GPU, several ranks on ONE GPU: the landmark-sharded solve
with real cross-rank sums.  RCCL allows one rank per GPU, so the ranks'
all-reduces go through the host-callback hook (sfm_ba_set_host_comm) over
gloo; everything else -- sharded reduced systems, packed S all-reduce,
rank-0-only camera terms, replicated factorisation and LM decisions,
per-rank point back substitution -- is the device code the multi-GPU bench
runs over RCCL.  Each sharded solve must take the single-process solve's
accept/reject sequence, with parameters within 1e-6 and cost within 1e-9
(the reduction order differs, so not bitwise), and every rank must hold
bitwise identical cameras.  All three BA_TYPE modes (CTracker.h:67)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

C, P, VIEWS, SEED = 40, 6000, 8, 0x5F3D2017 + 21


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, mode):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    import sfm_amd
    from sfm_amd import scene
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    per = P // world
    sc = scene.generate(C, P, views=VIEWS, seed=SEED, p_begin=rank * per, p_end=(rank + 1) * per)

    def allreduce(arr, op):
        t = torch.from_numpy(arr)  # shares the callback's buffer
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == 1 else dist.ReduceOp.SUM)

    with sfm_amd.BundleAdjuster(0) as ba:
        ba.set_host_comm(world, rank, allreduce)
        ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
        sm, tr = ba.solve(mode=mode)
        rot, t, X = ba.parameters()
    q.put((rank, sm.num_iterations, sm.final_cost, [x["step_is_successful"] for x in tr], rot, t, X))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,mode", [(2, 2), (3, 2), (2, 1), (2, 0)])
def test_sharded_solve_on_one_gpu_matches_single(world, mode):
    import sfm_amd
    from sfm_amd import scene
    full = scene.generate(C, P, views=VIEWS, seed=SEED)
    with sfm_amd.BundleAdjuster(0) as ba:
        ba.set_problem(full.uv, full.cam_idx, full.pt_idx, full.K, full.rot, full.t, full.X)
        sm, tr = ba.solve(mode=mode)
        rot1, t1, X1 = ba.parameters()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0

    def rel(a, b):
        return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3)))

    for r in res:
        assert r[1] == sm.num_iterations
        assert r[3] == [x["step_is_successful"] for x in tr]
        assert abs(r[2] - sm.final_cost) <= 1e-9 * sm.final_cost
        assert np.array_equal(r[4], res[0][4]) and np.array_equal(r[5], res[0][5])  # replicated cameras
    assert rel(res[0][4], rot1) < 1e-6 and rel(res[0][5], t1) < 1e-6
    X_sh = np.concatenate([r[6] for r in res])
    assert rel(X_sh, X1) < 1e-6
