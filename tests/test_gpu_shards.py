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


def _collect(procs, q, world, timeout):
    """Each worker's result from the queue; a worker that raised puts
    ("error", rank, traceback) instead, and then (or at the deadline) the
    workers -- the ones left waiting in a collective -- are ended, so a
    failing rank fails the test at once instead of hanging it."""
    import queue
    import time
    deadline = time.monotonic() + timeout
    res = []
    try:
        while len(res) < world:
            left = deadline - time.monotonic()
            if left <= 0:
                raise AssertionError(f"only {len(res)} of {world} ranks reported within {timeout} s")
            try:
                r = q.get(timeout=min(left, 5.0))
            except queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                if dead:
                    raise AssertionError(f"a rank exited with {dead[0]} before reporting")
                continue
            if r[0] == "error":
                raise AssertionError(f"rank {r[1]} failed:\n{r[2]}")
            res.append(r)
    except BaseException:
        for p in procs:
            if p.is_alive():
                p.kill()
        for p in procs:
            p.join(10)
        raise
    return sorted(res, key=lambda r: r[0])


def _guarded(fn):
    """Worker body wrapper: an exception goes into the queue (last arg)."""
    def run(rank, *args):
        try:
            fn(rank, *args)
        except BaseException:
            import traceback
            args[-1].put(("error", rank, traceback.format_exc()))
            raise
    return run


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, mode, dist_pt=0):
    _guarded(_worker_body)(rank, world, port, mode, dist_pt, q)


def _gloo_collectives(dist, torch, calls=None):
    """allreduce / broadcast / reduce_scatter over gloo for
    BundleAdjuster.set_host_collectives (arrays shared with the callback)."""
    def allreduce(arr, op):
        if calls is not None:
            calls["allreduce"] = calls.get("allreduce", 0) + 1
            calls["max_count"] = max(calls.get("max_count", 0), arr.size)
        dist.all_reduce(torch.from_numpy(arr), op=dist.ReduceOp.MAX if op == 1 else dist.ReduceOp.SUM)

    def broadcast(arr, root):
        if calls is not None:
            calls["broadcast"] = calls.get("broadcast", 0) + 1
        dist.broadcast(torch.from_numpy(arr), src=root)

    def reduce_scatter(buf, out):
        if calls is not None:
            calls["reduce_scatter"] = calls.get("reduce_scatter", 0) + 1
        dist.reduce_scatter_tensor(torch.from_numpy(out), torch.from_numpy(buf))

    def reduce(arr, root):
        if calls is not None:
            calls["reduce"] = calls.get("reduce", 0) + 1
        dist.reduce(torch.from_numpy(arr), dst=root)

    return allreduce, broadcast, reduce_scatter, reduce


def _worker_body(rank, world, port, mode, dist_pt, q):
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
        if dist_pt:
            ba.set_host_collectives(world, rank, *_gloo_collectives(dist, torch))
            ba.set_distributed_factor(dist_pt)
        else:
            ba.set_host_comm(world, rank, allreduce)
        ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
        sm, tr = ba.solve(mode=mode)
        rot, t, X = ba.parameters()
    q.put((rank, sm.num_iterations, sm.final_cost, [x["step_is_successful"] for x in tr], rot, t, X))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,mode,dist_pt", [(2, 2, 0), (3, 2, 0), (2, 1, 0), (2, 0, 0), (2, 2, 1), (3, 2, 1),
                                                (2, 2, 2), (4, 2, 1)])
def test_sharded_solve_on_one_gpu_matches_single(world, mode, dist_pt):
    """dist_pt > 0: the distributed reduced-camera factor (1-D block-cyclic
    panels of dist_pt tiles: C = 40 gives a 4-tile system, so 2-4 ranks own
    1-2 panels each) through the broadcast / reduce-scatter hook."""
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
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode, dist_pt)) for r in range(world)]
    for p in procs:
        p.start()
    res = _collect(procs, q, world, 150)
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


# ---- BASELINE config C4 (2000 cams / 1M points / 10M obs), the config the
# 8-GPU scaling run uses: the sharded path at full size with two ranks ----
C4_C, C4_P = 2000, 1_000_000
C4_SEED = 0x5F3D2017 + 4          # scene.config("C4")


def _c4_worker(rank, world, port, q, dist_pt=0):
    _guarded(_c4_worker_body)(rank, world, port, dist_pt, q)


def _c4_worker_body(rank, world, port, dist_pt, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    import sfm_amd
    from sfm_amd import scene
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scene.generate(C4_C, C4_P, seed=C4_SEED, p_begin=rank * C4_P // world, p_end=(rank + 1) * C4_P // world)
    calls = {"n": 0, "max_count": 0}

    def allreduce(arr, op):
        calls["n"] += 1
        calls["max_count"] = max(calls["max_count"], arr.size)
        t = torch.from_numpy(arr)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == 1 else dist.ReduceOp.SUM)

    dcalls = {}
    with sfm_amd.BundleAdjuster(0) as ba:
        if dist_pt:
            ba.set_host_collectives(world, rank, *_gloo_collectives(dist, torch, dcalls))
            ba.set_distributed_factor(dist_pt)
        else:
            ba.set_host_comm(world, rank, allreduce)
        ba.set_problem(sc.uv, sc.cam_idx, sc.pt_idx, sc.K, sc.rot, sc.t, sc.X)
        dist.barrier()  # both shards resident before either solves
        sm, tr = ba.solve()
        rot, t, X = ba.parameters()
    if dist_pt:
        calls = {"n": dcalls.get("allreduce", 0), "max_count": dcalls.get("max_count", 0),
                 "broadcast": dcalls.get("broadcast", 0), "reduce": dcalls.get("reduce", 0)}
    q.put((rank, sm.num_iterations, sm.final_cost, [x["step_is_successful"] for x in tr],
           [x["cost"] for x in tr], rot, t, X, calls["n"], calls["max_count"], calls, sm.num_linear_solves))
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def c4_single():
    import sfm_amd
    from sfm_amd import scene
    full = scene.generate(C4_C, C4_P, seed=C4_SEED)
    with sfm_amd.BundleAdjuster(0) as ba:
        ba.set_problem(full.uv, full.cam_idx, full.pt_idx, full.K, full.rot, full.t, full.X)
        sm, tr = ba.solve()
        rot1, t1, X1 = ba.parameters()
    return sm, tr, rot1, t1, X1


def _run_c4_ranks(world, dist_pt):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q, dist_pt)) for r in range(world)]
    for p in procs:
        p.start()
    res = _collect(procs, q, world, 540)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3])
def test_c4_distributed_factor_matches_single_rank(c4_single, world):
    """C4 in 2 / 3 landmark shards on one GPU with the DISTRIBUTED reduced-
    camera factor: the ranks' partial 12000x12000
    systems reduced panel by panel into the owners of 1-D block-cyclic panels
    of 4 tiles (47 panels), each factored by its owner and broadcast, every
    rank updating its own later panels, the back substitution replicated.  Against the single-
    rank solve: the same accept/reject sequence, per-iteration and final
    cost within 1e-9, parameters within 1e-6, cameras bitwise equal across
    the ranks -- and no packed-S all-reduce went through the hook."""
    sm, tr, rot1, t1, X1 = c4_single
    res = _run_c4_ranks(world, 4)

    def rel(a, b):
        return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3)))

    n = 6 * C4_C
    nblk = (n + 1 + 63) // 64
    panels = (nblk + 3) // 4
    for r in res:
        calls = r[10]
        assert r[9] <= 28 * C4_C                    # only the camera sums (U_c, b_c) and scalars were all-reduced
        assert calls["reduce"] == r[11] * panels    # one per panel and linear solve
        assert calls["broadcast"] == r[11] * panels
        assert r[1] == sm.num_iterations
        assert r[3] == [x["step_is_successful"] for x in tr]
        for a, b in zip(r[4], [x["cost"] for x in tr]):
            assert abs(a - b) <= 1e-9 * b
        assert abs(r[2] - sm.final_cost) <= 1e-9 * sm.final_cost
        assert np.array_equal(r[5], res[0][5]) and np.array_equal(r[6], res[0][6])
    assert rel(res[0][5], rot1) < 1e-6 and rel(res[0][6], t1) < 1e-6
    assert rel(np.concatenate([r[7] for r in res]), X1) < 1e-6


@pytest.mark.timeout(600)
def test_c4_two_rank_sharded_solve_matches_single_rank():
    """C4 split into two landmark shards (500k points / 5M observations each)
    on one GPU, cross-rank sums through sfm_ba_set_host_comm: the 12000x12000
    reduced system goes through the packed all-reduce (72M doubles, 576 MB),
    every rank factors it and back-substitutes its own 500k points.  Against
    the single-rank C4 solve: the same accept/reject sequence, per-iteration
    and final cost within 1e-9, parameters within 1e-6, and bitwise equal
    cameras on both ranks (the replicated LM decisions)."""
    import sfm_amd
    from sfm_amd import scene
    full = scene.generate(C4_C, C4_P, seed=C4_SEED)
    with sfm_amd.BundleAdjuster(0) as ba:
        ba.set_problem(full.uv, full.cam_idx, full.pt_idx, full.K, full.rot, full.t, full.X)
        sm, tr = ba.solve()
        rot1, t1, X1 = ba.parameters()
    del full
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = _collect(procs, q, world, 540)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0

    def rel(a, b):
        return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3)))

    n = 6 * C4_C
    for r in res:
        assert r[9] == n * (n + 1) // 2 + n        # the packed S + rhs went through the hook
        assert r[1] == sm.num_iterations
        assert r[3] == [x["step_is_successful"] for x in tr]
        for a, b in zip(r[4], [x["cost"] for x in tr]):
            assert abs(a - b) <= 1e-9 * b
        assert abs(r[2] - sm.final_cost) <= 1e-9 * sm.final_cost
        assert np.array_equal(r[5], res[0][5]) and np.array_equal(r[6], res[0][6])
    assert rel(res[0][5], rot1) < 1e-6 and rel(res[0][6], t1) < 1e-6
    assert rel(np.concatenate([r[7] for r in res]), X1) < 1e-6
