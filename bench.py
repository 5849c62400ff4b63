#!/usr/bin/env python3
"""Benchmark: registered scans/s on synthetic 64x1800 HDL-64-style scans (BASELINE.json configs[1]).

One "step" = one batch of B independent scan-to-map registration jobs (config C4-style independent
jobs, default B = 1024 per GPU: larger batches overlap the sub-batches' low-occupancy phases
better, 90.7k -> 92.8k scans/s from 512 to 1024) through the whole hot path on one GPU: range-image projection, LOAM feature
extraction, scan-to-map Gauss-Newton registration against a 100k-point local corner+surf map
(imageProjection.cpp:183-225 -> featureExtraction.h:79-294 -> mapOptmization.h:263-1489).
Inputs (raw scans, guesses, map grid) are resident in HBM before the timed region starts.

Multi-GPU (launched by torch.distributed.run): every rank processes its own B jobs (weak scaling,
no data-path collective); after each step the 32-byte pose records of all jobs are all-gathered
over RCCL (the only collective of the path).

Rank 0 prints ONE JSON line with the metric, a roofline block for the dominant kernel (HIP events
on the library's stream over the timed region) and a cpu_baseline block (the CPU oracle restating
the reference path, timed on a bounded sample of the same jobs at N=1), plus the pose RMSE of the
GPU path against that CPU reference on the sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "registered scans/sec + pose RMSE vs ref, 64×1800 synthetic Velodyne"
WORKLOAD = {"C1": "VLP-16-style scans, local corner+surf map",
            "C2": "HDL-64-style scans, ~100k-pt local corner+surf map",
            "C3": "Ouster-style scans, ~500k-pt local corner+surf map (mapping leaves 0.1/0.2)",
            "C5": "dense scans, ~5.8M-pt map inside the crop box (mapping leaves 0.05)"}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# Algorithmic bytes per unit for each kernel family (DESIGN.md "Kernels and rooflines").
def kernel_bytes(name, tot):
    n_in, n, Q, IQ, M, F, S = tot["n_in"], tot["n"], tot["Q"], tot["IQ"], tot["M"], tot["F"], tot["S"]
    return {
        "gn_knn": 116.0 * IQ,                 # query 16 B + the 5 neighbours found 80 B + 5 positions out 20 B
        "gn_residual": 116.0 * IQ,            # query 16 B + 5 positions 20 B + 5 neighbour gathers 80 B
        "project": 24.0 * n_in + 4.0 * n,     # raw point read + owner claim
        "extract": 4.0 * 2 * n + 28.0 * n,    # owners, owning point, xyzi+col+range write
        "features": 41.0 * n,                 # range/col/cloud read, label + candidate write
        "voxel_ring": 17.0 * n + 16.0 * S,    # label + candidate point read (<= n), per-ring DS write
        "voxel_scan": 16.0 * F + 16.0 * Q,    # corner + surf clouds read, DS queries written
    }.get(name, 0.0)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="jobs per GPU per step")
    ap.add_argument("--config", default="C2", choices=["C1", "C2", "C3", "C5"])
    ap.add_argument("--cpu-sample", type=int, default=96, help="jobs timed on the CPU oracle (N=1)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="worker threads of the all-cores CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--deskew", action="store_true",
                    help="enable the IMU deskew path (SURVEY 8f row 3): one imuDeskewInfo table per job")
    ap.add_argument("--dist", action="store_true",
                    help="use the torch.distributed (RCCL) path even at world size 1 (tests)")
    ap.add_argument("--profile", default="dominant", choices=["all", "dominant", "off"],
                    help="HIP-event kernel timing inside the timed region: every kernel, only the roofline "
                         "kernels (default), or none")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "hbm_traffic.json"),
                    help="per-launch HBM bytes of the dominant kernel from rocprofv3 PMC passes")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or args.dist:
        import torch  # noqa: F401  (load torch's HIP runtime first; the library shares it)
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl", init_method="env://")

    from feature_base_pointcloud_registration_amd import api, shard, synth

    cfg = args.config
    H, W, *_ = synth.CONFIGS[cfg]
    B = args.batch
    P = synth.config_params(cfg, max_batch=B)
    corner_map, surf_map = synth.config_map(cfg)
    jobs = synth.make_jobs(cfg, B, base_seed=1000 + rank * B)
    scans = [j[0] for j in jobs]
    guesses = np.stack([j[1] for j in jobs]).astype(np.float32)
    gts = np.stack([j[2] for j in jobs])

    dev = local_rank if world > 1 else 0
    stream_gbps = api.stream_copy_bandwidth(dev) if rank == 0 else None  # achievable HBM copy rate
    ctx = api.Context(P, device=dev)
    ctx.set_map(corner_map, surf_map)
    if args.deskew:  # per-job IMU tables: 200 Hz queue around each job's scan time
        tabs = [api.imu_deskew_info(synth.imu_queue(10.0 * j - 0.05, 10.0 * j + 0.16, gyro=(0.0, 0.0, 0.0), seed=j), 10.0 * j,
                                    10.0 * j + 0.1)[0] for j in range(B)]
        ctx.set_deskew(tabs)
    ctx.batch_stage(scans, guesses)

    gather_buf = None
    if dist is not None:
        import torch
        gather_buf = torch.zeros(B * 8, dtype=torch.float32, device=f"cuda:{local_rank}")

    def step():
        ctx.batch_launch()
        if dist is not None:
            ctx.batch_export(gather_buf.data_ptr())
            ctx.batch_wait()
            shard.gather_records(dist, gather_buf, world)

    for _ in range(args.warmup):
        step()
    ctx.batch_wait()
    kernels = ["gn_knn", "gn_residual", "gn_solve", "project", "extract", "features", "voxel_ring", "concat",
               "voxel_scan", "gn_init", "crop", "gn_finalize"]
    # one untimed profiled step: per-kernel device times (HIP events) and the dominant kernel
    ctx.set_profiling(True)
    step()
    ctx.batch_wait()
    ctx.set_profiling(False)
    prof = {k: ctx.kernel_time(k) for k in kernels}
    modelled = [k for k in kernels if kernel_bytes(k, dict.fromkeys(["n_in", "n", "Q", "IQ", "M", "F", "S"], 1.0)) > 0]
    dom = max(modelled, key=lambda k: prof[k][0])
    if dist is not None:
        import torch
        torch.cuda.synchronize()
        dist.barrier()
    # timed region: HIP events only around the roofline kernel by default (--profile all: every kernel)
    if args.profile == "all":
        ctx.set_profiling(True)
    elif args.profile == "dominant":
        ctx.set_profiling(True, [dom])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.batch_wait()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    poses, stats = ctx.batch_results()
    tb, tg = ctx.batch_bytes()
    ktot = {k: ctx.kernel_time(k) for k in kernels}
    timed = {k: (ktot[k][0] - prof[k][0], ktot[k][1] - prof[k][1]) for k in kernels}  # timed region only

    if rank != 0:
        ctx.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    total_jobs = world * B * args.steps
    value = total_jobs / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    # per-step workload counts (identical every step: the same staged batch is re-registered)
    tot = dict(n_in=float(sum(len(s) for s in scans)), n=float(stats["n_points"].sum()),
               Q=float((stats["n_corner_ds"] + stats["n_surf_ds"]).sum()),
               IQ=float(((stats["n_corner_ds"] + stats["n_surf_ds"]) * stats["iterations"]).sum()),
               M=float((stats["n_corner_map"] + stats["n_surf_map"]).sum()),
               F=float((stats["n_corner"] + stats["n_surf"]).sum()), S=float(stats["n_surf"].sum()))
    if timed[dom][1] > 0:  # live events over the timed region
        dom_ms, dom_launches, steps_measured, live = timed[dom][0], timed[dom][1], args.steps, True
    else:                  # --profile off: the profiled step
        dom_ms, dom_launches, steps_measured, live = prof[dom][0], prof[dom][1], 1, False
    launches_per_step = dom_launches / max(steps_measured, 1)
    bytes_per_launch = kernel_bytes(dom, tot) / max(launches_per_step, 1e-9)
    avg_launch_s = dom_ms / 1000.0 / max(dom_launches, 1)
    achieved = bytes_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    traffic = None
    if os.path.exists(args.pmc_json):
        try:
            with open(args.pmc_json) as f:
                pm = json.load(f)
            if pm.get("config") == cfg and pm.get("batch") == B and dom in pm.get("kernels", {}):
                traffic = pm["kernels"][dom]["hbm_bytes_per_launch"]
        except Exception:
            traffic = None

    # pose accuracy vs ground truth (sanity) and vs the CPU reference path (metric)
    err_gt = np.abs(poses[:, 3:] - gts[:, 3:].astype(np.float32)).max()
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "scans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"{cfg}: {H}x{W} {WORKLOAD[cfg]}; "
                        f"{B} independent scan-to-map jobs per GPU per step (C4-style independent jobs)",
            "jobs_per_gpu_per_step": B,
            "mean_points_per_scan": round(tot["n_in"] / B, 1),
            "mean_local_map_points": round(tot["M"] / B, 1),
            "mean_queries_per_scan": round(tot["Q"] / B, 1),
            "mean_gn_iterations": round(float(stats["iterations"].mean()), 3),
            "parallelism": f"scan-shard x{world}, RCCL pose all-gather" if world > 1 else "single GPU",
            "imu_deskew": bool(args.deskew),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "stream_copy_GBps": round(stream_gbps, 1),
            "frac_vs_stream_copy": round(achieved / stream_gbps, 5),
            "traffic": traffic,
            "bytes_per_launch": bytes_per_launch,
            "avg_launch_us": round(avg_launch_s * 1e6, 3),
            "launches_per_step": launches_per_step,
            "timing": "HIP events on the library stream over the timed region" if live else
                      "HIP events on the library stream, profiled untimed step",
        },
        "kernel_ms_per_step": {k: round(v[0], 4) for k, v in prof.items()},  # profiled untimed step
        "path_bytes_per_step": tb,
        "path_achieved_GBps": round(tb / (elapsed / args.steps) / 1e9, 2),
        "path_frac_of_peak": round(tb / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 5),
        "max_abs_trans_err_vs_gt_m": float(err_gt),
        "registration_status_ok": int((stats["status"] == 0).sum()),
    }

    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import pyoracle as O  # CPU restatement of the reference path: baseline + accuracy reference
        S = min(args.cpu_sample, B)
        omap = O.Map(P, corner_map, surf_map)
        ref = np.zeros((S, 6), np.float32)
        ref_iters, ref_nsel = np.zeros(S), np.zeros(S)
        O.stage_ms(reset=True)
        t1 = time.perf_counter()
        for j in range(S):
            stream = O.Stream(P)  # independent job: fresh FeatureExtraction state
            ref[j], st = stream.process_scan(omap, scans[j], 0.0, guesses[j], n_threads=P.number_of_cores)
            ref_iters[j], ref_nsel[j] = st["iterations"], st["n_sel"]
        cpu_s = time.perf_counter() - t1
        stage = O.stage_ms()
        dt = poses[:S, 3:] - ref[:, 3:]
        dr = np.angle(np.exp(1j * (poses[:S, :3].astype(np.float64) - ref[:, :3])))
        result["cpu_baseline"] = {
            "value": round(S / cpu_s, 3),
            "unit": "scans/s",
            "cores": int(P.number_of_cores),
            "kind": "port",
            "sample": f"first {S} of the {B} {cfg} jobs, whole path (projection, features, "
                      f"registration incl. per-scan KD-tree build), OpenMP {P.number_of_cores} threads "
                      f"(numberOfCores), host nproc={os.cpu_count()}",
            # per-stage oracle time (A2/A4, A6-A9, A11, A12, A13 KD build, A13-A18 GN)
            "stage_ms_per_scan": {k: round(v / S, 3) for k, v in stage.items()},
            "mean_gn_iterations": float(ref_iters.mean()),
            "mean_n_sel": float(ref_nsel.mean()),
        }
        result["pose_rmse_vs_ref"] = {
            "trans_m": float(np.sqrt(np.mean(np.sum(dt.astype(np.float64) ** 2, axis=1)))),
            "rot_rad": float(np.sqrt(np.mean(np.sum(dr ** 2, axis=1)))),
            "max_trans_m": float(np.abs(dt).max()),
            "max_rot_rad": float(np.abs(dr).max()),
            "n": S,
        }
        result["gpu_vs_cpu_speedup"] = round(value / (S / cpu_s), 2)
        # all-cores batch: one independent job per worker thread, one OpenMP thread each
        # (ctypes releases the GIL inside the oracle calls)
        import concurrent.futures
        nth = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))

        def one(j):
            return O.Stream(P).process_scan(omap, scans[j], 0.0, guesses[j], n_threads=1)[0]

        t2 = time.perf_counter()
        with concurrent.futures.ThreadPoolExecutor(nth) as ex:
            list(ex.map(one, range(S)))
        cpu_all_s = time.perf_counter() - t2
        result["cpu_baseline_all_cores"] = {
            "value": round(S / cpu_all_s, 3), "unit": "scans/s", "cores": nth, "kind": "port",
            "sample": f"the same {S} jobs, {nth} independent single-threaded jobs at a time"}
    print(json.dumps(result), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
