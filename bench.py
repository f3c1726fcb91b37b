#!/usr/bin/env python3
"""Benchmark: local bundle-adjustment LM iterations/sec on MI355X (BASELINE.json metric).

One "step" = one Levenberg-Marquardt iteration of the reference's local BA (slam.cpp:482-521, Ceres 1.8
LM + SPARSE_SCHUR restated on the GPU): linearize (if the previous step was accepted), damp + Schur
complement, reduced camera Cholesky, back-substitution, candidate cost, accept/reject — all on device.

Workload (N = 1): BASELINE config 2 — 50 keyframes / ~20k landmarks / ~130k observations, synthetic
scene (slamgpu/scene.py, seed 2), SolveFrames(map, 48, 50, 2.0).  fp64 arithmetic (the reference's own
precision).  Termination is disabled inside the timed region so that exactly K iterations run.

N > 1 (torchrun, one rank per GPU): weak scaling — 50 keyframes and N x 20k landmarks sharded over the
ranks by first observing frame (sg_problem_shard), RCCL all-reduce of the camera system per iteration;
value = N * K / time, i.e. the unit is one LM iteration's worth of config-2 work (20k landmarks).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-robot_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector / matrix peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--points", type=int, default=20000, help="landmarks per GPU")
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (0: skip)")
    ap.add_argument("--sweep-obs", type=int, default=2_000_000,
                    help="observations in the scaled Jacobian-sweep measurement (0: skip)")
    ap.add_argument("--frontend", type=int, default=1,
                    help="also measure the front end at N=1: KLT tracks/sec (config 3) and the 256-bit "
                         "Hamming matcher (config 4)")
    return ap.parse_args()


FP32_PEAK_TFLOPS = 157.3     # MI355X FP32 vector peak
INT_PEAK_TOPS = 78.6         # 32-bit integer VALU lane-ops/s: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz


def pmc_traffic(kernel, largest_grid=False):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (tools/pmc_traffic.sh -> profiles/<round>_pmc_traffic.json, newest file wins).  Among several launch
    shapes of one kernel the smallest grid is the config-2 / bench launch, the largest the scaled sweep."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None
    groups = [g for g in json.load(open(files[-1]))["kernels"].values() if g["kernel"] == kernel]
    if not groups:
        return None
    g = (max if largest_grid else min)(groups, key=lambda g: g["grid_size"])
    return g["traffic_bytes"]


def bench_tracker(local, cpu_seconds):
    """BASELINE config 3: 640x480 synthetic video, 2000 tracks, 3-level pyramid, 7x7 window, forward/backward
    TrackFeature (matcher.cpp:173-206).  Inputs resident on the device; value = tracks / kernel time."""
    from slamgpu.tracker import HessianTracker
    from slamgpu.video import make_frames, seed_points
    frames = make_frames(2)
    pts = seed_points(2000)
    W, depth, reps = 7, 3, 50
    t = HessianTracker(window=W, depth=depth, device=local, retry_levels=0)
    t.MakePyramid(frames[0], 0)
    t.MakePyramid(frames[1], 1)
    _, pyr_ms = t.kernel_ms()
    t.load_features(pts, pts)
    t.run(0, 1, 3)
    t.results()
    t.run(0, 1, reps)
    out, acc, its = t.results()
    track_ms, _ = t.kernel_ms()
    ms = track_ms / reps
    value = len(pts) / (ms * 1e-3)
    flops = float(its.sum()) * 108.0 * W * W        # 108 W^2 flops per Newton iteration
    ach = flops / (ms * 1e-3) / 1e12
    res = {"metric": "KLT tracks/sec (640x480, 2000 tracks, 3 levels, 7x7, forward+backward)",
           "value": value, "unit": "tracks/s", "ms_per_frame_tracking": ms, "ms_pyramid": pyr_ms,
           "tracks_per_s_with_pyramid": len(pts) / ((ms + pyr_ms) * 1e-3),
           "accepted_frac": float(acc.mean()), "newton_iterations": int(its.sum()),
           # one wave per track and ~2 waves per SIMD: the launch lasts as long as its longest serial
           # Newton chain, so the per-iteration latency of that chain is the number that bounds the kernel
           "newton_iterations_max_track": int(its.max()),
           "us_per_newton_iteration_on_longest_track": ms * 1e3 / max(int(its.max()), 1),
           "roofline": {"bound": "valu", "achieved": ach, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": ach / FP32_PEAK_TFLOPS, "traffic": pmc_traffic("k_track_fb"), "kernel": "k_track_fb",
                        "note": "108*W^2 flops per Newton iteration (6 probes of bilinear sampling, moments, "
                                "score); one wave per feature"}}
    if cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        pf, dims = oracle.make_pyramid(frames[0], depth)
        pt, _ = oracle.make_pyramid(frames[1], depth)
        threads = min(16, os.cpu_count() or 1)
        done, tc = 0, 0.0
        while tc < cpu_seconds:
            tt = time.perf_counter()
            oracle.track_fb(pf, pt, dims, W, pts, pts, np.full(len(pts), depth, np.int32), nthreads=threads)
            tc += time.perf_counter() - tt
            done += len(pts)
        res["cpu_baseline"] = {"value": done / tc, "unit": "tracks/s", "cores": threads, "kind": "port",
                               "sample": "%d forward/backward tracks (oracle/oracle_track.cpp, OpenMP over "
                                         "tracks) in %.1f s" % (done, tc)}
    return res


def bench_hamming(local, cpu_seconds):
    """BASELINE config 4: 10k x 10k 256-bit descriptors, all pairs, best + second-best per query."""
    from slamgpu.matcher import HammingMatcher, make_descriptor_sets
    A, B, truth = make_descriptor_sets(10000)
    m = HammingMatcher(device=local)
    m.load(B, A)
    m.run(3)
    m.results()
    reps = 20
    m.run(reps)
    bi, bd, sd, ms = m.results()
    pairs = float(len(A)) * len(B)
    ops = pairs * 16.0       # per pair: 8 x v_xor_b32 + 8 x v_bcnt_u32_b32 (accumulating) on 32-bit lanes
    ach = ops / (ms * 1e-3) / 1e12
    res = {"metric": "256-bit Hamming all-pairs query-rows/sec (10k x 10k)", "value": len(B) / (ms * 1e-3),
           "unit": "rows/s", "pairs_per_s": pairs / (ms * 1e-3), "ms": ms,
           "recall_of_true_matches": float((bi[truth >= 0] == truth[truth >= 0]).mean()),
           "roofline": {"bound": "valu-int", "achieved": ach, "peak": INT_PEAK_TOPS, "unit": "Tops/s",
                        "frac": ach / INT_PEAK_TOPS, "traffic": pmc_traffic("k_hamming_slices"),
                        "kernel": "k_hamming_slices"}}
    if cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = min(16, os.cpu_count() or 1)
        done, tc = 0, 0.0
        while tc < cpu_seconds:
            tt = time.perf_counter()
            oracle.hamming_match(B, A, nthreads=threads)
            tc += time.perf_counter() - tt
            done += len(B)
        res["cpu_baseline"] = {"value": done / tc, "unit": "rows/s", "cores": threads, "kind": "port",
                               "sample": "%d query rows x 10k (oracle, popcnt, OpenMP) in %.1f s" % (done, tc)}
    return res


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def main():
    args = parse()
    ws, rank, local = dist_env()
    import torch
    from slamgpu import ba
    from slamgpu.capi import default_solver_options
    from slamgpu.scene import make_scene

    dist = None
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=ws)
    n_gpus = ws

    # ---- workload: config 2 per GPU (weak scaling over landmarks)
    scene = make_scene(num_frames=args.frames, num_points=args.points * n_gpus, seed=2, run_max=14)
    full = ba.problem_from_map_frames(scene, args.frames - 2, args.frames, 2.0)
    prob = ba.shard_problem(full, rank, n_gpus) if n_gpus > 1 else full

    solver = ba.BundleAdjuster(device=local)
    if n_gpus > 1:
        uid = ba.BundleAdjuster.unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8, device=f"cuda:{local}")
        dist.broadcast(t, 0)
        solver.comm_init(bytes(t.cpu().tolist()), n_gpus, rank)
    solver.load(prob)
    total_iters = args.warmup + 2 * args.steps + 16
    opts = default_solver_options(max_num_iterations=total_iters, disable_termination=1)
    solver.begin(opts)
    solver.iterate(args.warmup)
    solver.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    # ---- timed region: exactly K LM iterations
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    solver.iterate(args.steps)
    solver.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    summary_after = solver.summary()

    # ---- per-kernel HIP-event timing over a second timed region of the same workload
    s0 = solver.summary()
    solver.set_timing(True)
    solver.iterate(args.steps)
    solver.sync()
    ktimes = solver.kernel_times()
    solver.set_timing(False)
    s1 = solver.summary()
    n_lin = s1["num_successful_steps"] - s0["num_successful_steps"]
    work = solver.kernel_work()

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    per_iter_ms = {k: v[0] * v[1] / max(args.steps, 1) for k, v in ktimes.items()}
    dominant = max(per_iter_ms, key=per_iter_ms.get)
    # dominant kernel roofline (fp64 arithmetic)
    dom_ms = ktimes[dominant][0]
    dom_bytes, dom_flops = work[dominant]
    if dom_flops > 0 and dominant in ("cholesky",):
        ach = dom_flops / (dom_ms * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / FP64_PEAK_TFLOPS, "traffic": pmc_traffic("k_cholesky_window"), "kernel": dominant,
                "note": "single-workgroup dense banded Cholesky of the reduced camera system (n=%d)"
                        % (6 * (args.frames - 2))}
    else:
        ach = dom_bytes / (dom_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": ach / HBM_PEAK_GBS, "traffic": pmc_traffic("k_" + dominant), "kernel": dominant}
    # Jacobian/Hessian sweep (north-star kernel): bytes per linearization / mean active launch time.
    lin_total_ms = ktimes["linearize"][0] * ktimes["linearize"][1]
    sweep = None
    if n_lin > 0:
        ach = work["linearize"][0] * n_lin / (lin_total_ms * 1e-3) / 1e9
        sweep = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": ach / HBM_PEAK_GBS, "bytes_per_launch": work["linearize"][0],
                 "traffic": pmc_traffic("k_linearize"),
                 "active_launches": n_lin, "launches": ktimes["linearize"][1]}

    # scaled sweep: the same kernel on a problem large enough to amortise launch latency
    sweep_scaled = None
    if args.sweep_obs > 0:
        npts = max(args.sweep_obs // 10, 1000)
        big = make_scene(num_frames=200, num_points=npts, seed=5, run_max=18)
        bp = ba.problem_from_map_frames(big, 198, 200, 2.0)
        bs = ba.BundleAdjuster(device=local)
        bs.load(bp)
        bs.begin(default_solver_options())
        bs.sweep(3)
        bs.sync()
        bs.set_timing(True)
        bs.sweep(20)
        bs.sync()
        kt = bs.kernel_times()["linearize"]
        wb = bs.kernel_work()["linearize"][0]
        ach = wb / (kt[0] * 1e-3) / 1e9
        sweep_scaled = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS, "obs": bp.num_obs, "points": bp.num_points,
                        "ms_per_launch": kt[0], "bytes_per_launch": wb,
                        "traffic": pmc_traffic("k_linearize", largest_grid=True)}
        bs.close()

    # CPU baseline: the oracle (C++ restatement of the same LM) on the host cores, bounded sample
    cpu = None
    if args.cpu_seconds > 0 and n_gpus == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        threads = min(16, os.cpu_count() or 1)
        po = full.copy()
        o = default_solver_options(max_num_iterations=5, disable_termination=1)
        done_iters, t_cpu = 0, 0.0
        while t_cpu < args.cpu_seconds:
            tt = time.perf_counter()
            s = oracle.solve(po, o, nthreads=threads)
            t_cpu += time.perf_counter() - tt
            done_iters += s["num_lm_iterations"]
        cpu = {"value": done_iters / t_cpu, "unit": "iters/s", "cores": threads, "kind": "port",
               "sample": "%d LM iterations of config 2 (oracle/oracle_ba.cpp, dual-number Jacobians, "
                         "OpenMP) in %.1f s, chunks of 5 iterations each re-linearising at start"
                         % (done_iters, t_cpu)}

    frontend = None
    if args.frontend and n_gpus == 1:
        cs = min(args.cpu_seconds, 4.0)
        frontend = {"tracker": bench_tracker(local, cs), "hamming": bench_hamming(local, cs)}

    value = n_gpus * args.steps / elapsed
    line = {
        "metric": "local-BA iters/sec (50 KF, 20k pts)",  # BASELINE metric; KLT tracks/sec under "frontend"
        "value": value,
        "unit": "iters/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded scene generator, slamgpu/scene.py)",
        "config": {"workload": "config 2: SolveFrames(48 of 50 KF) local BA, LM iteration",
                   "keyframes": args.frames, "landmarks_per_gpu": prob.num_points,
                   "observations_per_gpu": prob.num_obs, "free_frames": int(full.frame_rot_free.sum()),
                   "parallelism": "landmark-shard x%d (RCCL all-reduce of the camera system)" % n_gpus
                   if n_gpus > 1 else "single GPU"},
        "roofline": roof,
        "roofline_sweep": sweep,
        "roofline_sweep_scaled": sweep_scaled,
        "kernel_ms_per_iter": {k: round(v, 5) for k, v in per_iter_ms.items()},
        "cpu_baseline": cpu,
        "speedup_vs_cpu": (value / cpu["value"]) if cpu else None,
        "lm_state": {"final_cost": summary_after["final_cost"], "radius": summary_after["trust_region_radius"]},
        "frontend": frontend,
        "traffic_source": "HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes "
                          "(tools/pmc_traffic.sh, profiles/*_pmc_traffic.json; FETCH_SIZE doubled on gfx950)",
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
