"""Multi-process host logic of the sharded multi-GPU path (ipm355.dist) on CPU with `gloo`,
world size 2 and 3: sharding covers every instance exactly once, and the single all_gather
returns every rank's results to every rank (the solve itself is stubbed -- no GPU here)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ipm355 import dist as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = D.solve_sharded(None, n, solve_fn=lambda i: (1000.0 + i * 0.5, 10 + (i % 7)))
        np.save(os.path.join(out_dir, f"r{rank}.npy"), res)
    finally:
        dist.destroy_process_group()


def test_shard_partition():
    for n in (0, 1, 7, 64):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in D.shard(n, r, world))
            assert got == list(range(n))
    with pytest.raises(ValueError):
        D.shard(4, 2, 2)


@pytest.mark.parametrize("world,n", [(2, 64), (3, 10)])
def test_all_gather_results_gloo(tmp_path, world, n):
    mp.start_processes(_worker, args=(world, _free_port(), n, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    ref = np.array([[1000.0 + i * 0.5, 10 + (i % 7)] for i in range(n)])
    for r in range(world):
        res = np.load(tmp_path / f"r{r}.npy")
        assert res.shape == (n, 3)
        np.testing.assert_array_equal(res[:, :2], ref)       # every rank sees every instance
        assert np.all(res[:, 2] >= 0)


def test_single_process_gather_without_init():
    res = D.gather_results({0: (1.0, 2, 0.1), 2: (3.0, 4, 0.2)}, 3)
    assert res[0, 0] == 1.0 and res[2, 1] == 4 and np.isnan(res[1, 0])


def test_launch_local_end_to_end(tmp_path):
    """The self-launcher bench.py --gpus N uses (ipm355.dist.launch_local): N fresh rank processes
    with torchrun's env contract, solve_sharded over gloo, x* gathered -> every rank has every row."""
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_worker.py")
    rc = D.launch_local(2, [sys.executable, worker, "9", str(tmp_path)])
    assert rc == 0
    for r in range(2):
        tab = np.load(tmp_path / f"tab{r}.npy")
        X = np.load(tmp_path / f"x{r}.npy")
        np.testing.assert_array_equal(tab[:, 0], 100.0 + np.arange(9))
        np.testing.assert_array_equal(tab[:, 1], 7 + np.arange(9) % 3)
        np.testing.assert_array_equal(X, np.arange(9)[:, None] * np.arange(5)[None, :])
        assert (tmp_path / f"env{r}.txt").read_text() == f"{r} {r} 2"


def test_launch_local_failing_rank_terminates_the_others(tmp_path):
    import sys
    code = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(3)\n"
            "time.sleep(60)\n")
    rc = D.launch_local(2, [sys.executable, "-c", code])
    assert rc == 3


class _FakeSolver:
    """Records where solve_sharded places each instance (every rank used GPU 0)."""
    seen = []

    def __init__(self, device=None, **kw):
        import types
        self.dev = types.SimpleNamespace(index=device)
        _FakeSolver.seen.append(device)
        self.inner_iters, self.phase1_solver, self.xstar = [3], None, np.zeros(2)

    def solve(self):
        return 1.5


def test_solve_sharded_places_solvers_on_the_rank_device(monkeypatch):
    _FakeSolver.seen = []
    monkeypatch.setenv("LOCAL_RANK", "3")
    res = D.solve_sharded(lambda i: {}, 2, _FakeSolver)
    assert _FakeSolver.seen == [3, 3]
    np.testing.assert_array_equal(res[:, 0], [1.5, 1.5])
    _FakeSolver.seen = []
    D.solve_sharded(lambda i: {}, 1, _FakeSolver, device=5)
    assert _FakeSolver.seen == [5]


def test_shard_solves_every_instance_once_with_solve_kwargs(monkeypatch):
    """ipm355.dist.Shard (the config-4 product path): built once (inputs resident), solve() passes
    its keyword arguments (e.g. iteration_budget) to every instance and reports value, Newton
    iterations (phase 1 included) and seconds per instance index."""
    calls = []

    class _Budgeted(_FakeSolver):
        def solve(self, **kw):
            calls.append(kw)
            return 2.5

    monkeypatch.setenv("LOCAL_RANK", "0")
    sh = D.build_shard(lambda i: {}, 3, _Budgeted)
    assert sh.indices == [0, 1, 2] and not sh.concurrent
    out = sh.solve(iteration_budget=7)
    assert sorted(out) == [0, 1, 2] and all(v[0] == 2.5 and v[1] == 3 for v in out.values())
    assert calls == [{"iteration_budget": 7}] * 3
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")     # (restored after the test)
    assert D.configure_queues(16) in (True, False)


def test_shard_concurrent_groups_instances_by_stream():
    """with more instances than torch's pool of 32 streams per device, two instances
    share a stream and hence a native handle (Handle.get caches one per (device, stream)).
    Shard.solve must never drive one stream from two host threads at once: instances sharing a
    stream run one after another in that stream's thread (host logic only: fake streams and
    solvers that fail if two threads enter the same stream)."""
    import threading
    import time
    from ipm355 import dist as D

    class FakeStream:
        def __init__(self, sid):
            self.cuda_stream = sid

        def synchronize(self):
            pass

    active, lock, seen = {}, threading.Lock(), set()

    class FakeSolver:
        def __init__(self, sid):
            self.sid, self.inner_iters = sid, [3]

        def solve(self):
            with lock:
                assert not active.get(self.sid), "two threads drive one stream"
                active[self.sid] = True
                seen.add(threading.get_ident())
            time.sleep(0.005)
            with lock:
                active[self.sid] = False
            return float(self.sid)

    sh = object.__new__(D.Shard)
    sh.indices, sh.dev, sh.concurrent = list(range(40)), 0, True
    sh.streams = [FakeStream(i % 32) for i in range(40)]
    sh.solvers = [FakeSolver(i % 32) for i in range(40)]
    out = sh.solve()
    assert sorted(out) == list(range(40))
    assert all(out[i][0] == float(i % 32) and out[i][1] == 3 for i in range(40))
    assert len(seen) > 1          # still concurrent across distinct streams
