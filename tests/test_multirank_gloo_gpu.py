"""The landmark-sharded solver with one OS process per rank, on a one-GPU box.

Two processes, each with its own solver handle on device 0, join a gloo process group (torch.distributed,
127.0.0.1) and exchange through the host-callback communicator (sg_ba_comm_init_host): every all-reduce the
solver makes — the load-time structure flag and Cholesky envelope (max), then per LM iteration the camera
blocks and cost scalars, the packed band of S and its rhs, and the step scalars (sum) — leaves the device,
goes through gloo between the processes and comes back, in the order the RCCL communicator issues them.
RCCL itself needs one GPU per rank, which a one-GPU box does not have; the solver's exchange path and its
compute path are the ones a multi-GPU run takes.  Parity: the sharded solve against the one-rank solve of the
whole problem in the parent process (summation order differs only), with the tolerances of
test_multirank_local_gpu.py's two-shard C2 test.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, iters):
    sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))
    import torch
    import torch.distributed as dist
    from slamgpu import ba
    from slamgpu.capi import default_solver_options
    from slamgpu.scene import make_config

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    calls = {"sum": 0, "max": 0}

    def allreduce(arr, op):
        calls[op] += 1
        dist.all_reduce(torch.from_numpy(arr), op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)

    m = make_config("C2")
    full = ba.problem_from_map_frames(m, 48, 50, 2.0)
    shard = ba.shard_problem(full, rank, world)
    g = ba.BundleAdjuster(device=0)
    g.comm_init_host(world, rank, allreduce)
    g.load(shard)
    info = g.info()
    s = g.solve(default_solver_options(max_num_iterations=iters))
    g.close()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), q=shard.q, t=shard.t, X=shard.X,
             pmi=shard.point_map_index, num_iterations=s["num_iterations"],
             num_successful=s["num_successful_steps"], initial_cost=s["initial_cost"],
             final_cost=s["final_cost"], ok=s["ok"], nranks=info["nranks"], band=info["band_tiles"],
             sums=calls["sum"], maxes=calls["max"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_two_processes_gloo_c2_match_one_rank(tmp_path, gpu_lib):
    import torch.multiprocessing as mp
    from slamgpu import ba
    from slamgpu.capi import default_solver_options
    from slamgpu.scene import make_config

    iters = 5
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), iters), nprocs=2, join=True,
                       start_method="spawn")
    r = [np.load(tmp_path / ("rank%d.npz" % k)) for k in range(2)]
    m = make_config("C2")
    pa = ba.problem_from_map_frames(m, 48, 50, 2.0)
    one = pa.copy()
    g = ba.BundleAdjuster()
    g.load(one)
    s1 = g.solve(default_solver_options(max_num_iterations=iters))
    band = g.info()["band_tiles"]
    g.close()
    for x in r:
        assert int(x["nranks"]) == 2 and int(x["band"]) == band   # the envelope union reached every rank
        assert int(x["ok"]) == 1
        assert int(x["num_iterations"]) == s1["num_iterations"]
        assert int(x["num_successful"]) == s1["num_successful_steps"]
        # load: structure flag + envelope (max); per iteration: camera blocks, packed S band, step scalars (sum)
        assert int(x["maxes"]) == 2 and int(x["sums"]) >= 3 * iters
    # the replicated decision and factorisation: both processes hold the same frames
    np.testing.assert_array_equal(r[0]["q"], r[1]["q"])
    np.testing.assert_array_equal(r[0]["t"], r[1]["t"])
    assert abs(float(r[0]["initial_cost"]) - s1["initial_cost"]) <= 1e-12 * s1["initial_cost"]
    assert abs(float(r[0]["final_cost"]) - s1["final_cost"]) <= 1e-12 * s1["final_cost"]
    np.testing.assert_allclose(r[0]["q"], one.q, rtol=0, atol=1e-10)
    np.testing.assert_allclose(r[0]["t"], one.t, rtol=0, atol=1e-6)
    where = {int(mi): i for i, mi in enumerate(pa.point_map_index)}
    X = np.full_like(pa.X, np.nan)
    for x in r:
        for j, mi in enumerate(x["pmi"]):
            i = where[int(mi)]
            X[4 * i:4 * i + 4] = x["X"][4 * j:4 * j + 4]
    assert not np.isnan(X).any()
    np.testing.assert_allclose(X, one.X, rtol=0, atol=1e-10)


def test_host_communicator_failure_is_reported(gpu_lib):
    """A transport that fails (the callback returns nonzero) fails the call with SG_ECOMM instead of hanging or
    solving with a partial sum; the handle stays usable for a one-rank problem afterwards."""
    from slamgpu import ba
    from slamgpu.capi import SlamGpuError
    from slamgpu.scene import make_config

    m = make_config("C1")
    pa = ba.problem_from_map_frames(m, m.num_frames - 2, m.num_frames, 2.0)
    shard = ba.shard_problem(pa, 0, 2)

    def broken(arr, op):
        raise RuntimeError("transport down")

    g = ba.BundleAdjuster()
    g.comm_init_host(2, 0, broken)
    with pytest.raises(SlamGpuError) as e:
        g.load(shard)
    assert "code -71" in str(e.value) and "communicator" in str(e.value)
    g.close()


@pytest.mark.parametrize("launch", ["torchrun", "self"])
def test_bench_two_ranks_host_transport(launch):
    """bench.py's N > 1 path, rehearsed on one GPU through the host transport (--comm host): one process per rank,
    barriers, max-over-ranks timing, rank-0 JSON.  `torchrun` is the driver's form (torch.distributed.run around
    bench.py); `self` is a plain `bench.py --gpus 2`, which must start its two rank processes itself instead of
    running one rank and printing n_gpus 1.  The line is the strong-scaling figure of the
    metric's own config-2 problem, sharded over the two ranks, and the bench survives a chain whose exchange timer
    is the largest per-iteration entry (it did not: KeyError 'exchange')."""
    import json
    import subprocess
    args = [os.path.join(ROOT, "bench.py"),
            "--gpus", "2", "--steps", "5", "--warmup", "2", "--comm", "host", "--other", "0", "--cpu-runs", "0",
            "--cpu-seconds", "0", "--frontend", "0", "--solve-all", "0", "--model-scaling", "0", "--weak", "0"]
    if launch == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["metric"] == "local-BA iters/sec (50 KF, 20k pts)"
    assert line["config"]["landmarks"] == 19449 and line["value"] > 0
    assert line["solver"]["nranks"] == 2 and line["solver"]["num_allreduces"] > 0
