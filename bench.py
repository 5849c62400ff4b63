#!/usr/bin/env python3
"""Benchmark: registered scans/s on synthetic 64x1800 HDL-64-style scans (BASELINE.json configs[1]).

One "step" = one batch of B independent scan-to-map registration jobs (config C4-style independent
jobs, default B = 1024 per GPU: larger batches overlap the sub-batches' low-occupancy phases
better, 90.7k -> 92.8k scans/s from 512 to 1024) through the whole hot path on one GPU: range-image projection, LOAM feature
extraction, scan-to-map Gauss-Newton registration against a 100k-point local corner+surf map
(imageProjection.cpp:183-225 -> featureExtraction.h:79-294 -> mapOptmization.h:263-1489).
Inputs (raw scans, guesses, map grid) are resident in HBM before the timed region starts.

Multi-GPU (launched by torch.distributed.run): every rank processes its own B jobs (weak scaling,
the default) or a contiguous block of --total-jobs N (strong scaling: C4 = 1024 jobs over 8 GPUs,
128 per GPU); there is no data-path collective.  After each step the 32-byte pose records of all
jobs are all-gathered over RCCL (the only collective of the path) and, after the
timed region, checked against every rank's own results.

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
# VALU roof: wave-level VALU instructions per second.  MI355X_MICROARCH.md: a wave64 VALU instruction
# occupies a SIMD-32 for 2 cycles, 1024 SIMDs x 2.4 GHz / 2 = 1228.8 G instr/s; measured on the box
# (fbr_valu_peak, tools/valu_calib.py -> profiles/valu_calib.json): 1079 G instr/s of independent
# v_fma_f32 at 8 waves per SIMD (2.26 cycles per instruction at the 2.38 GHz effective clock), ~490
# with one wave per SIMD.  The measured peak is the roof.  (SQ_ACTIVE_INST_VALU counts one
# quad-cycle per VALU instruction whatever the issue rate -- the calibration's PMC pass -- so it is
# an instruction count, not busy time.)
VALU_PEAK_GINST_SPEC = 1024 * 2.4 / 2.0


def valu_peak_ginst():
    try:
        with open(os.path.join(REPO, "profiles", "valu_calib.json")) as f:
            return float(json.load(f)["measured_peak_ginst_per_s"]), "profiles/valu_calib.json (measured v_fma_f32)"
    except Exception:
        return VALU_PEAK_GINST_SPEC, "MI355X_MICROARCH.md (2 cycles per wave64 VALU instruction)"


VALU_PEAK_GINST, VALU_PEAK_SOURCE = valu_peak_ginst()

# Algorithmic bytes per unit for each kernel family: the minimal HBM traffic the kernel's job needs
# (DESIGN.md §4 holds the same table; SURVEY §8(d)'s per-unit figures).  Units per step: n_in raw
# points, HW range-image cells, n valid points, C corner picks, S per-ring surf DS points, F = C + S
# feature points, Q DS queries, IQ query-iterations (IQc of them corner ones).  The traffic the
# design itself adds on top (scratch it stages, caches it keeps) is design_bytes below: reported
# beside the algorithmic figure, never folded into the roofline fraction.
# Batch scans are 16-B device records (x, y, z, ring; fbr_kernels.h) unless FBR_PACKED_SCANS=0 keeps
# the 24-B fbr_point_xyzirt scans.
SCAN_REC_B = 24.0 if os.environ.get("FBR_PACKED_SCANS", "1") == "0" else 16.0


def kernel_bytes(name, tot):
    n_in, HW, n, C = tot["n_in"], tot["HW"], tot["n"], tot["C"]
    S, F, Q, IQ = tot["S"], tot["F"], tot["Q"], tot["IQ"]
    R = SCAN_REC_B
    return {
        "project": R * n_in + 4.0 * n,           # raw point record read + first-wins owner claim
        "extract": 4.0 * HW + 4.0 * n + R * n + 24.0 * n,  # owner image read + claimed cells reset, owning
                                                          # raw point gather, xyzi+col+range write
        "features": 9.0 * n + 32.0 * C,          # range + col read, label written; corner points read + written
        "voxel_ring": 17.0 * n + 16.0 * S,       # label + candidate point read, per-ring DS write
        "concat": 32.0 * F,                      # per-ring corner / surf outputs read + job clouds written
        "voxel_scan": 16.0 * F + 16.0 * Q,       # corner + surf clouds read, DS queries written
        "gn_knn": 36.0 * IQ,                     # query 16 B read, 5 map indices 20 B written; the map rows
                                                 # are cache hits (C2's map is 1.5 MB)
        "gn_residual": 36.0 * IQ,                # query 16 B + 5 indices 20 B read; neighbour gathers are
                                                 # cache hits (SURVEY §8(d)'s 96 B per query-iteration is
                                                 # these two kernels with the gathers counted)
    }.get(name, 0.0)


def design_bytes(name, tot):
    """HBM traffic the design adds to a kernel's algorithmic bytes (design choices, not the job):
    features stages each ring's curvature through its scratch slot (4 B written, 4 B read back per
    point); gn_knn writes a 1-B same-neighbours flag and reads the previous iteration's 5 indices as
    its warm start; gn_residual reads the flag and fit state (2 B) and the fit cache (plane 16 B,
    line 24 B: read when the neighbours are unchanged, written when refitted)."""
    n, Q, IQ, IQc = tot["n"], tot["Q"], tot["IQ"], tot.get("IQc", 0.0)
    return {
        "features": 8.0 * n,
        "gn_knn": 1.0 * IQ + 20.0 * (IQ - Q),
        "gn_residual": 2.0 * IQ + 16.0 * IQ + 8.0 * IQc,
    }.get(name, 0.0)


BYTE_MODEL = {
    "project": "%d B per raw point record + 4 B owner claim per valid point" % SCAN_REC_B,
    "extract": "4 B per range-image cell + 4 B owner reset + %d B raw-record gather + 24 B written per valid point"
               % SCAN_REC_B,
    "features": "9 B per valid point (range + col read, label written) + 32 B per corner pick",
    "voxel_ring": "17 B per valid point + 16 B per per-ring DS point",
    "concat": "32 B per feature point",
    "voxel_scan": "16 B per feature point + 16 B per DS query",
    "gn_knn": "36 B per query-iteration (query 16 B read, 5 indices 20 B written); map rows are L2/MALL hits",
    "gn_residual": "36 B per query-iteration (query 16 B, 5 indices 20 B read); neighbour gathers are L2/MALL hits",
}
DESIGN_MODEL = {
    "features": "8 B per valid point: the ring's curvature staged through its scratch slot",
    "gn_knn": "1 B same-neighbours flag per query-iteration + 20 B warm start (previous 5 indices) per warm-started one",
    "gn_residual": "2 B flag / fit state + 16 B plane fit cache per query-iteration, + 8 B per corner one (24 B line)",
}

# rocprofv3 kernel symbols behind each launcher name (tools/roofline_check.py maps a profile's rows)
KERNEL_SYMBOLS = {"project": ["k_project"], "extract": ["k_rowcount", "k_compact"], "features": ["k_features"],
                  "voxel_ring": ["k_voxel_ring"], "concat": ["k_concat"], "voxel_scan": ["k_voxel_grid"],
                  "gn_knn": ["k_gn_knn"], "gn_residual": ["k_gn_residual"], "gn_solve": ["k_gn_solve"],
                  "gn_loop": ["k_gn_loop_knn", "k_gn_loop_residual"],
                  "gn_init": ["k_gn_init"], "gn_finalize": ["k_gn_finalize"], "crop": ["k_crop_count"]}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="jobs per GPU per step (weak scaling)")
    ap.add_argument("--total-jobs", type=int, default=0,
                    help="strong scaling: N jobs per step split into contiguous per-rank blocks (C4: 1024)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend of the pose-record gather (gloo: host records, tests)")
    ap.add_argument("--gather", default="torch", choices=["torch", "native"],
                    help="pose-record all-gather for N > 1: torch.distributed (--backend), or the library's own "
                         "RCCL communicator (fbr_comm_create / fbr_batch_allgather; the process group, gloo, "
                         "then only carries the RCCL id, barriers and the timing)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on device 0 (world-size > 1 rehearsal on a one-GPU box)")
    ap.add_argument("--records-out", default=None, help="rank 0 writes the gathered records (.npy)")
    ap.add_argument("--latency", type=int, default=50,
                    help="single-stream line: N pose-chained scans through fbr_process_scan (the reference's "
                         "operating mode, imageProjection.cpp:206-218), rank 0 at N=1; 0 disables")
    ap.add_argument("--ingest", type=int, default=4,
                    help="ingest-inclusive line: REPS x B jobs from host memory through fbr_process_batch "
                         "(pinned double-buffered staging; the first batch's upload and the last batch's "
                         "compute overlap nothing, so few REPS understate the streaming rate), rank 0 at "
                         "N=1; 0 disables")
    ap.add_argument("--config", default="C2", choices=["C1", "C2", "C3", "C5"])
    ap.add_argument("--pipeline-depth", type=int, default=0,
                    help="fbr_params.pipeline_depth: batch launch slots (0 = the library default, 3)")
    ap.add_argument("--cpu-sample", type=int, default=96, help="jobs timed on the CPU oracle (N=1)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="worker threads of the CPU-share baseline (the GPU box's CPU share per GPU is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exact-line", type=int, default=1,
                    help="rank 0 at N=1: a second context with exact_voxel_order = 1 (PCL's point order inside voxels, "
                         "bit-identical poses) reports its throughput and parity block; 0 disables")
    ap.add_argument("--exact-voxel-order", type=int, default=0,
                    help="fbr_params.exact_voxel_order of the main line (1: std::sort's in-voxel point order)")
    ap.add_argument("--deskew", action="store_true",
                    help="enable the IMU deskew path (SURVEY 8f row 3): one imuDeskewInfo table per job")
    ap.add_argument("--dist", action="store_true",
                    help="use the torch.distributed (RCCL) path even at world size 1 (tests)")
    ap.add_argument("--profile", default="all", choices=["all", "dominant", "off"],
                    help="kernel timing inside the timed region (dispatch start/end timestamps through HIP "
                         "events): every kernel (default), only the roofline kernel, or none")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "hbm_traffic.json"),
                    help="per-launch HBM bytes of the dominant kernel from rocprofv3 PMC passes")
    ap.add_argument("--sq-json", default=os.path.join(REPO, "profiles", "sq_decomp.json"),
                    help="per-kernel wave-state / instruction-mix decomposition (tools/sq_decomp.py)")
    ap.add_argument("--valu-json", default=os.path.join(REPO, "profiles", "valu_pmc.json"),
                    help="per-launch VALU instructions of every kernel from a rocprofv3 SQ pass (tools/valu_pmc.py)")
    return ap.parse_args()


def ingest_line(ctx, scans, guesses, resident_poses, reps, B):
    """Scans/s with the raw scans starting in host memory: reps x B jobs through fbr_process_batch
    (pinned staging + copy stream, batch k+1's upload overlapping batch k's compute), next to the
    pageable path (fbr_batch_stage's synchronous copies, then the batch) for one batch."""
    ctx.process_batch(scans[:min(B, 8)], guesses[:min(B, 8)])  # allocates the staging ring
    t0 = time.perf_counter()
    p, st = ctx.process_batch(scans * reps, np.tile(guesses, (reps, 1)))
    t_pipe = time.perf_counter() - t0
    h2d = ctx.ingest_bytes()
    same = bool((p[:B].view(np.int32) == resident_poses.view(np.int32)).all())
    t1 = time.perf_counter()
    ctx.batch_stage(scans, guesses)
    ctx.batch_launch()
    ctx.batch_wait()
    ctx.batch_results()
    t_page = time.perf_counter() - t1
    return {
        "value": round(reps * B / t_pipe, 3), "unit": "scans/s",
        "jobs": reps * B, "path": "fbr_process_batch: pinned staging ring, copy stream, double-buffered inputs",
        "h2d_bytes_per_scan": round(h2d / (reps * B), 1),
        "h2d_GBps": round(h2d / t_pipe / 1e9, 2),
        "pageable_one_batch_scans_per_s": round(B / t_page, 3),
        "poses_equal_resident": same,
    }


def mask_check(ctx, scans, poses, stats, P, S, O, launches=5):
    """Whole feature masks of the headline batch (fbr_batch_set_full_masks / fbr_batch_labels): the
    first S jobs' cloudLabel against the oracle's bit for bit, the full-mask launches' poses and
    statistics against the timed ones (the default launches resolve only the observable surf
    picks), and the rate of full-mask launches (untimed by the headline)."""
    B = len(scans)
    ctx.batch_set_full_masks(True)
    t0 = time.perf_counter()
    for _ in range(launches):
        ctx.batch_launch()
    ctx.batch_wait()
    t_full = time.perf_counter() - t0
    pf, sf = ctx.batch_results()
    eq = 0
    for j in range(S):
        lab = ctx.batch_labels(j)
        ref = O.Stream(P).features(scans[j])["label"]
        eq += int(len(lab) == len(ref) and np.array_equal(lab, ref))
    ctx.batch_set_full_masks(False)
    return {"n": S, "mask_bit_equal": eq,
            "poses_equal_timed": bool((pf.view(np.int32) == poses.view(np.int32)).all()),
            "stats_equal_timed": bool(np.array_equal(sf, stats)),
            "full_mask_scans_per_s": round(launches * B / t_full, 1),
            "path": "fbr_batch_set_full_masks + fbr_batch_labels on the staged headline batch"}


def latency_line(cfg, corner_map, surf_map, n, cpu_scans=0):
    """The reference's operating mode: one scan at a time, each registration starting from the
    previous result (imageProjection.cpp:206-218), host scan in, pose out.  Reports wall ms per
    scan (host upload to pose back), kernel launches / blocking host syncs / GN flag polls per scan,
    and the oracle's per-scan time and pose on the same chain for the first cpu_scans scans."""
    from feature_base_pointcloud_registration_amd import api, synth
    H, W, *_ = synth.CONFIGS[cfg]
    P = synth.config_params(cfg, max_batch=1)
    traj = synth.trajectory(7, n + 3)
    scans = [synth.scan(p, H, W, seed=500 + k) for k, p in enumerate(traj)]
    _, guess0 = synth.job(7)
    ms = []
    poses = []
    with api.Context(P) as c:
        c.set_map(corner_map, surf_map)
        pose = guess0.copy()
        for k in range(3):  # warm-up (first-call allocations, code loading)
            pose, _ = c.process_scan(scans[k], 0.2 * k, pose)
        warm_pose = pose.copy()
        api.debug_counters(reset=True)
        api.host_times(reset=True)
        api.wait_stats(reset=True)
        iters = []
        for k in range(3, n + 3):
            t = time.perf_counter()
            pose, st = c.process_scan(scans[k], 0.2 * k, pose)
            ms.append(1e3 * (time.perf_counter() - t))
            poses.append(pose.copy())
            iters.append(int(st["iterations"]))
        launches, syncs, polls = api.debug_counters()
        ht = api.host_times()
        fallbacks, long_waits, wait_max_s, queries = api.wait_stats()
    ms = np.array(ms)
    out = {"scans": n, "ms_per_scan_mean": round(float(ms.mean()), 4), "ms_per_scan_p50": round(float(np.median(ms)), 4),
           "ms_per_scan_p99": round(float(np.percentile(ms, 99)), 4),
           "ms_per_scan_max": round(float(ms.max()), 4),
           # the slowest scans of the chain: (index in the chain, ms, GN iterations)
           "slowest": [(int(i), round(float(ms[i]), 4), iters[i]) for i in np.argsort(ms)[::-1][:3]],
           "gn_iterations_mean": round(float(np.mean(iters)), 3),
           # host waits on device results (GN iteration flags, the direct result): fallbacks (not
           # visible although the stream drained), waits > 1 ms, the longest, stream queries
           "result_waits": {"fallbacks": fallbacks, "over_1ms": long_waits, "max_ms": round(1e3 * wait_max_s, 4),
                            "stream_queries": queries},
           "launches_per_scan": round(launches / n, 2), "host_syncs_per_scan": round(syncs / n, 2),
           "gn_flag_polls_per_scan": round(polls / n, 2),
           # host wall time inside fbr_process_scan per scan: scan upload (staging copy + enqueue),
           # stage enqueue (launches, GN flag polls), result wait, whole call
           "host_ms_per_scan": {k: round(1e3 * v / n, 4) for k, v in zip(("upload", "enqueue", "result_wait", "call"), ht)},
           "path": "fbr_process_scan (host scan -> HBM, projection, features, registration, pose back)"}
    if cpu_scans:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import pyoracle as O
        st = O.Stream(P)
        omap = O.Map(P, corner_map, surf_map)
        po = guess0.copy()
        for k in range(3):
            po, _ = st.process_scan(omap, scans[k], 0.2 * k, po, n_threads=P.number_of_cores)
        t = time.perf_counter()
        dmax = float(np.abs(po.astype(np.float64) - warm_pose).max())
        for k in range(3, 3 + cpu_scans):
            po, _ = st.process_scan(omap, scans[k], 0.2 * k, po, n_threads=P.number_of_cores)
            dmax = max(dmax, float(np.abs(po.astype(np.float64) - poses[k - 3]).max()))
        out["cpu_oracle_ms_per_scan"] = round(1e3 * (time.perf_counter() - t) / cpu_scans, 3)
        out["cpu_oracle_threads"] = int(P.number_of_cores)
        out["chain_max_abs_pose_diff_vs_oracle"] = dmax
    return out


def exact_line(cfg, corner_map, surf_map, scans, guesses, ref=None, ref_iters=None, ref_nsel=None, B=256, steps=5):
    """The same workload on a second context with fbr_params.exact_voxel_order = 1 (in this process,
    beside the default-mode context): every VoxelGrid sums a voxel's points in std::sort's order
    (csrc/fbr_introsort.h), so the poses equal the oracle's bit for bit.  B = 256 jobs; its parity
    block over the oracle sample of the main line (the same first jobs)."""
    from feature_base_pointcloud_registration_amd import api, synth
    B = min(B, len(scans))
    P = synth.config_params(cfg, max_batch=B, exact_voxel_order=1)
    with api.Context(P) as c:
        c.set_map(corner_map, surf_map)
        c.batch_stage(scans[:B], guesses[:B])
        for _ in range(2):
            c.batch_launch()
        c.batch_wait()
        t0 = time.perf_counter()
        for _ in range(steps):
            c.batch_launch()
        c.batch_wait()
        dt = time.perf_counter() - t0
        poses, stats = c.batch_results()
    out = {"value": round(B * steps / dt, 3), "unit": "scans/s", "ms_per_step": round(1e3 * dt / steps, 4),
           "jobs_per_step": B,
           "path": "fbr_params.exact_voxel_order = 1: std::sort's partition phase emulated in every VoxelGrid "
                   "(per-ring, mapping DS, start-up map), then the stable radix sort"}
    if ref is not None:
        S = min(len(ref), B)
        out["parity_vs_ref"] = {
            "n": S, "iterations_equal": int((stats["iterations"][:S] == ref_iters[:S]).sum()),
            "n_sel_equal": int((stats["n_sel"][:S] == ref_nsel[:S]).sum()),
            "pose_bit_equal": int((poses[:S].view(np.int32) == ref[:S].view(np.int32)).all(axis=1).sum())}
        out["pose_max_abs_diff_vs_ref"] = float(np.abs(poses[:S].astype(np.float64) - ref[:S]).max())
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    dev = 0 if args.same_device else local_rank
    if world > 1 or args.dist:
        import torch  # noqa: F401  (load torch's HIP runtime first; the library shares it)
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if args.gather == "native":
            args.backend = "gloo"  # torch carries no records: the C-ABI's RCCL communicator does
        dist.init_process_group(backend=args.backend, init_method="env://")

    from feature_base_pointcloud_registration_amd import api, shard, synth

    cfg = args.config
    H, W, *_ = synth.CONFIGS[cfg]
    if args.total_jobs:  # strong split (C4): rank r owns the contiguous block [j0, j1)
        j0, j1 = shard.job_block(rank, world, args.total_jobs)
        counts = [shard.job_block(r, world, args.total_jobs)[1] - shard.job_block(r, world, args.total_jobs)[0]
                  for r in range(world)]
    else:                # weak: every rank its own --batch jobs
        j0, j1 = rank * args.batch, (rank + 1) * args.batch
        counts = [args.batch] * world
    B = j1 - j0
    Bpad = max(counts)   # all-gather blocks are padded to the largest rank's
    P = synth.config_params(cfg, max_batch=B, pipeline_depth=args.pipeline_depth,
                            exact_voxel_order=args.exact_voxel_order)
    corner_map, surf_map = synth.config_map(cfg)
    jobs = synth.make_jobs(cfg, B, base_seed=1000 + j0)  # job j uses seed 1000 + j
    scans = [j[0] for j in jobs]
    guesses = np.stack([j[1] for j in jobs]).astype(np.float32)
    gts = np.stack([j[2] for j in jobs])

    stream_gbps = api.stream_copy_bandwidth(dev) if rank == 0 else None  # achievable HBM copy rate
    ctx = api.Context(P, device=dev)
    ctx.set_map(corner_map, surf_map)
    if args.deskew:  # per-job IMU tables: 200 Hz queue around each job's scan time
        tabs = [api.imu_deskew_info(synth.imu_queue(10.0 * j - 0.05, 10.0 * j + 0.16, gyro=(0.0, 0.0, 0.0), seed=j), 10.0 * j,
                                    10.0 * j + 0.1)[0] for j in range(B)]
        ctx.set_deskew(tabs)
    ctx.batch_stage(scans, guesses)

    gather_buf = None
    ext_streams = {}  # library stream handle -> torch.cuda.ExternalStream
    if dist is not None:
        import torch
        if args.backend == "nccl":
            gather_buf = torch.zeros(Bpad * shard.RECORD_FLOATS, dtype=torch.float32, device=f"cuda:{dev}")
    gathered = [None]
    native = dist is not None and args.gather == "native"
    launches, native_done = [0], [-1]
    if native:
        obj = [api.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = api.Comm(ctx, obj[0], world, rank, Bpad)
        recv = torch.zeros(world * Bpad * shard.RECORD_FLOATS, dtype=torch.float32, device=f"cuda:{dev}")

    def native_gather(upto):
        """fbr_batch_allgather of every launch <= upto not yet gathered (the same ids on every rank;
        consecutive gathers are ordered on the device by the library)."""
        while native_done[0] < upto:
            native_done[0] += 1
            # recv is read on torch's stream: the next gather waits for those reads
            comm.allgather(native_done[0], recv.data_ptr(), torch.cuda.current_stream().cuda_stream)
            gathered[0] = recv

    def gather_ready():
        """All-gather the records of the latest launch the library has fully enqueued (launches are
        pipelined: after launch n that is launch n-1).  The export waits for the previous gather
        (torch's stream still reading gather_buf); the gather waits for the export."""
        cur = torch.cuda.current_stream()
        lid, sh = ctx.batch_export_ready(gather_buf.data_ptr(), cur.cuda_stream)
        if lid < 0:
            return False
        if sh not in ext_streams:
            ext_streams[sh] = torch.cuda.ExternalStream(sh, device=f"cuda:{dev}")
        cur.wait_stream(ext_streams[sh])
        gathered[0] = shard.gather_records(dist, gather_buf, world)
        return True

    def gather_rest():  # after the last launch: every launch not yet gathered, in order
        if native:
            native_gather(launches[0] - 1)
            return
        ctx.batch_flush()
        while gather_ready():
            pass

    def step():
        ctx.batch_launch()
        launches[0] += 1
        if dist is None:
            return
        if native:  # launch n returns once n - 2 is fully enqueued: gather it without a host wait
            native_gather(launches[0] - 3)
        elif args.backend == "nccl":
            gather_ready()
        else:  # gloo: host records
            poses_h, stats_h = ctx.batch_results()
            rec = np.zeros(Bpad * shard.RECORD_FLOATS, np.float32)
            rec[:B * shard.RECORD_FLOATS] = shard.encode_records(poses_h, stats_h["iterations"], stats_h["status"])
            gathered[0] = shard.gather_records(dist, torch.from_numpy(rec), world)

    for _ in range(args.warmup):
        step()
    if dist is not None and (native or args.backend == "nccl"):
        gather_rest()
    ctx.batch_wait()
    kernels = ["gn_knn", "gn_residual", "gn_solve", "project", "extract", "features", "voxel_ring", "concat",
               "voxel_scan", "gn_init", "crop", "gn_finalize", "gn_loop"]
    # one untimed profiled step: per-kernel device times (HIP events) and the dominant kernel
    ctx.set_profiling(True)
    step()
    if dist is not None and (native or args.backend == "nccl"):
        gather_rest()
    ctx.batch_wait()
    ctx.set_profiling(False)
    prof = {k: ctx.kernel_time(k) for k in kernels}
    modelled = [k for k in kernels if kernel_bytes(k, dict.fromkeys(["n_in", "HW", "n", "C", "S", "F", "Q", "IQ", "IQc"], 1.0)) > 0]
    dom = max(modelled, key=lambda k: prof[k][0])  # the roofline kernel: the profiled step's largest
    if dist is not None:
        import torch
        torch.cuda.synchronize()
        dist.barrier()
    # timed region: every kernel's dispatches carry start / end events (--profile dominant: only the
    # roofline kernel's, off: none)
    if args.profile == "all":
        ctx.set_profiling(True)
    elif args.profile == "dominant":
        ctx.set_profiling(True, [dom])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dist is not None and (native or args.backend == "nccl"):  # the last launches' records
        gather_rest()
    ctx.batch_wait()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    records_check = None
    if dist is not None:
        tdev = f"cuda:{dev}" if args.backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # the last step's gathered records, rank-ordered, against every rank's own results
        allrec = shard.unpad_records(gathered[0].cpu().numpy(), counts)
        p_l, s_l = ctx.batch_results()
        mine = shard.encode_records(p_l, s_l["iterations"], s_l["status"])
        off = sum(counts[:rank]) * shard.RECORD_FLOATS
        bad = int((allrec[off:off + len(mine)].view(np.int32) != mine.view(np.int32)).sum())
        bt = torch.tensor([bad], dtype=torch.int64, device=tdev)
        dist.all_reduce(bt)
        records_check = {"jobs": int(sum(counts)), "mismatched_words": int(bt.item())}
        if rank == 0 and args.records_out:
            np.save(args.records_out, allrec)

    poses, stats = ctx.batch_results()
    tb, tg = ctx.batch_bytes()
    ktot = {k: ctx.kernel_time(k) for k in kernels}
    timed = {k: (ktot[k][0] - prof[k][0], ktot[k][1] - prof[k][1]) for k in kernels}  # timed region only
    # the roofline kernel stays the profiled step's largest (dom above): in the timed region three
    # launches overlap, and a long-lived low-occupancy kernel (the mapping DS, one 1024-thread
    # workgroup per CU) accumulates as much live time as the kNN while costing the step a third of
    # it; every kernel's live fraction is reported in roofline.kernels either way

    if native:
        comm.close()
    if rank != 0:
        ctx.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    total_jobs = sum(counts) * args.steps
    value = total_jobs / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    # per-step workload counts (identical every step: the same staged batch is re-registered)
    tot = dict(n_in=float(sum(len(s) for s in scans)), HW=float(B * H * W), n=float(stats["n_points"].sum()),
               C=float(stats["n_corner"].sum()), S=float(stats["n_surf"].sum()),
               F=float((stats["n_corner"] + stats["n_surf"]).sum()),
               Q=float((stats["n_corner_ds"] + stats["n_surf_ds"]).sum()),
               IQ=float(((stats["n_corner_ds"] + stats["n_surf_ds"]) * stats["iterations"]).sum()),
               IQc=float((stats["n_corner_ds"] * stats["iterations"]).sum()),
               M=float((stats["n_corner_map"] + stats["n_surf_map"]).sum()))

    # per-launch VALU instructions (rocprofv3 SQ pass of the same config and batch, tools/valu_pmc.py)
    valu = {}
    if os.path.exists(args.valu_json):
        try:
            with open(args.valu_json) as f:
                vj = json.load(f)
            if vj.get("config") == cfg and vj.get("batch") == B:
                valu = vj.get("kernels", {})
        except Exception:
            valu = {}

    def kernel_roofline(k):
        if timed[k][1] > 0:  # live: the timed region's dispatches
            ms, launches, steps_measured, live = timed[k][0], timed[k][1], args.steps, True
        else:                # not timed live (--profile dominant/off): the profiled step
            ms, launches, steps_measured, live = prof[k][0], prof[k][1], 1, False
        lps = launches / max(steps_measured, 1)
        bpl = kernel_bytes(k, tot) / max(lps, 1e-9)
        dpl = design_bytes(k, tot) / max(lps, 1e-9)
        avg_s = ms / 1000.0 / max(launches, 1)
        ach = bpl / avg_s / 1e9 if avg_s > 0 else 0.0
        r = dict(bytes_per_launch=bpl, avg_launch_us=round(avg_s * 1e6, 3), launches_per_step=lps,
                 achieved_GBps=round(ach, 2), frac=round(ach / HBM_PEAK_GBS, 5),
                 ms_per_step=round(ms / max(steps_measured, 1), 4), live=live)
        if dpl > 0:  # the design's own traffic, beside (not inside) the algorithmic fraction
            r["design_bytes_per_launch"] = dpl
            r["design_model"] = DESIGN_MODEL[k]
            r["frac_with_design_bytes"] = round((bpl + dpl) / avg_s / 1e9 / HBM_PEAK_GBS, 5) if avg_s > 0 else 0.0
        if k in valu and avg_s > 0:  # the launch's wave-level VALU instructions over its live duration
            ipl = valu[k]["insts_valu_per_launch"]
            r["valu_insts_per_launch"] = ipl
            r["valu_achieved_ginst_s"] = round(ipl / avg_s / 1e9, 2)
            r["valu_frac"] = round(ipl / avg_s / 1e9 / VALU_PEAK_GINST, 5)
            if valu[k].get("avg_us_alone"):  # the same against the SQ pass's own (serialised) duration
                r["valu_frac_alone"] = round(ipl / (valu[k]["avg_us_alone"] * 1e-6) / 1e9 / VALU_PEAK_GINST, 4)
        return r

    kroof = {k: kernel_roofline(k) for k in modelled}
    # what each kernel's waves wait on (SQ passes of the same config and batch, tools/sq_decomp.py)
    if os.path.exists(args.sq_json):
        try:
            with open(args.sq_json) as f:
                sj = json.load(f)
            if sj.get("config") == cfg and sj.get("batch") == B:
                for k, e in sj["kernels"].items():
                    if k in kroof:
                        kroof[k]["wave_state_alone"] = {kk: round(v, 3) for kk, v in e["wave_state"].items()}
        except Exception:
            pass
    bytes_per_launch, launches_per_step = kroof[dom]["bytes_per_launch"], kroof[dom]["launches_per_step"]
    avg_launch_s, achieved, live = kroof[dom]["avg_launch_us"] * 1e-6, kroof[dom]["achieved_GBps"], kroof[dom]["live"]
    # the roof the dominant kernel is closer to: VALU issue when its VALU fraction exceeds its HBM one
    valu_bound = "valu_frac" in kroof[dom] and kroof[dom]["valu_frac"] > kroof[dom]["frac"]
    traffic = None
    if os.path.exists(args.pmc_json):
        try:
            with open(args.pmc_json) as f:
                pm = json.load(f)
            if pm.get("config") == cfg and pm.get("batch") == B:
                # every kernel's counter bytes per launch (FETCH_SIZE + WRITE_SIZE, one launch alone)
                # against its algorithmic bytes: the wasted-traffic ratio
                for k, e in pm.get("kernels", {}).items():
                    if k in kroof and kroof[k]["bytes_per_launch"] > 0:
                        kroof[k]["traffic"] = e["hbm_bytes_per_launch"]
                        kroof[k]["traffic_over_algorithmic"] = round(e["hbm_bytes_per_launch"] / kroof[k]["bytes_per_launch"], 3)
                if dom in pm.get("kernels", {}):
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
        "scaling": "strong" if args.total_jobs else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"{cfg}: {H}x{W} {WORKLOAD[cfg]}; " + (
                f"{args.total_jobs} independent scan-to-map jobs per step split over {world} GPU(s) (C4)"
                if args.total_jobs else f"{B} independent scan-to-map jobs per GPU per step (C4-style independent jobs)"),
            "jobs_per_step": int(sum(counts)),
            "jobs_per_gpu_per_step": B,
            "mean_points_per_scan": round(tot["n_in"] / B, 1),
            "mean_local_map_points": round(tot["M"] / B, 1),
            "mean_queries_per_scan": round(tot["Q"] / B, 1),
            "mean_gn_iterations": round(float(stats["iterations"].mean()), 3),
            "parallelism": (f"scan-shard x{world}, " + ("RCCL pose all-gather through the C-ABI (fbr_batch_allgather)"
                                                         if native else f"{'RCCL' if args.backend == 'nccl' else 'gloo'} "
                                                                        "pose all-gather (torch.distributed)")
                            if dist is not None else "single GPU"),
            "imu_deskew": bool(args.deskew),
            "exact_voxel_order": int(args.exact_voxel_order),
            "timed_region": ("fbr_batch_launch of a staged batch, every stage on the device: projection, features, "
                             "per-ring and mapping VoxelGrids, CropBox statistics, Gauss-Newton registration, "
                             "results; excludes the host-to-device copy of the raw scans and guesses "
                             "(fbr_batch_stage: inputs resident in HBM as 16-B x, y, z, ring records packed "
                             "by host threads, as the ingest path's records are), reported separately as "
                             "the ingest line"),
        },
        "roofline": {
            "bound": "valu" if valu_bound else "hbm",
            "kernel": dom,
            "achieved": kroof[dom]["valu_achieved_ginst_s"] if valu_bound else round(achieved, 2),
            "peak": round(VALU_PEAK_GINST, 2) if valu_bound else HBM_PEAK_GBS,
            "unit": "G wave64 VALU instr/s" if valu_bound else "GB/s",
            "frac": kroof[dom]["valu_frac"] if valu_bound else round(achieved / HBM_PEAK_GBS, 5),
            "valu_frac": kroof[dom].get("valu_frac"),
            "valu_frac_alone": kroof[dom].get("valu_frac_alone"),
            "valu_peak_source": VALU_PEAK_SOURCE,
            "valu_peak_spec_ginst_s": VALU_PEAK_GINST_SPEC,
            "hbm_achieved_GBps": round(achieved, 2),
            "hbm_frac": round(achieved / HBM_PEAK_GBS, 5),
            "valu_source": os.path.relpath(args.valu_json, REPO) if valu else None,
            "stream_copy_GBps": round(stream_gbps, 1),
            "hbm_frac_vs_stream_copy": round(achieved / stream_gbps, 5),
            "traffic": traffic,
            "bytes_per_launch": bytes_per_launch,
            "avg_launch_us": round(avg_launch_s * 1e6, 3),
            "launches_per_step": launches_per_step,
            "timing": ("kernel dispatch start/end timestamps (hipExtLaunchKernel events) over the timed region"
                       if live else "kernel dispatch start/end timestamps, profiled untimed step"),
            "rocprof_symbols": KERNEL_SYMBOLS[dom],
            "byte_model": BYTE_MODEL[dom],
            "design_bytes_per_launch": kroof[dom].get("design_bytes_per_launch", 0.0),
            "design_model": DESIGN_MODEL.get(dom),
            "kernels": {k: {kk: v for kk, v in r.items() if kk != "live"} for k, r in kroof.items()},
        },
        "kernel_ms_per_step": {k: round(v[0], 4) for k, v in prof.items()},  # profiled untimed step
        "path_bytes_per_step": tb,
        "path_achieved_GBps": round(tb / (elapsed / args.steps) / 1e9, 2),
        "path_frac_of_peak": round(tb / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 5),
        "max_abs_trans_err_vs_gt_m": float(err_gt),
        "registration_status_ok": int((stats["status"] == 0).sum()),
    }
    if records_check is not None:
        result["records_check"] = records_check

    if world == 1 and args.latency > 0:
        result["latency"] = latency_line(cfg, corner_map, surf_map, args.latency,
                                         cpu_scans=0 if args.no_cpu_baseline else 10)

    if world == 1 and args.ingest > 0:
        result["ingest"] = ingest_line(ctx, scans, guesses, poses, args.ingest, B)

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
        # correspondence-level parity (SURVEY §7 hard part 3): a flipped gate (sqdist < 1, lambda ratio
        # 3, s > 0.1, plane 0.2, degeneracy 100) in any iteration shows up as a different final n_sel,
        # iteration count or pose bits
        it_g, ns_g = stats["iterations"][:S], stats["n_sel"][:S]
        result["parity_vs_ref"] = {
            "n": S,
            "iterations_equal": int((it_g == ref_iters).sum()),
            "n_sel_equal": int((ns_g == ref_nsel).sum()),
            "n_sel_absdiff_max": int(np.abs(ns_g - ref_nsel).max()),
            "pose_bit_equal": int((poses[:S].view(np.int32) == ref.view(np.int32)).all(axis=1).sum()),
            "iterations_hist": {int(k): int(v) for k, v in zip(*np.unique(it_g, return_counts=True))},
        }
        result["feature_masks"] = mask_check(ctx, scans, poses, stats, P, S, O)
        result["pose_rmse_vs_ref"] = {
            "trans_m": float(np.sqrt(np.mean(np.sum(dt.astype(np.float64) ** 2, axis=1)))),
            "rot_rad": float(np.sqrt(np.mean(np.sum(dr ** 2, axis=1)))),
            "max_trans_m": float(np.abs(dt).max()),
            "max_rot_rad": float(np.abs(dr).max()),
            "n": S,
        }
        result["gpu_vs_cpu_speedup"] = round(value / (S / cpu_s), 2)
        # CPU-share batch: one independent job per worker thread, one OpenMP thread each
        # (ctypes releases the GIL inside the oracle calls)
        import concurrent.futures
        nth = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))

        def one(j):
            return O.Stream(P).process_scan(omap, scans[j], 0.0, guesses[j], n_threads=1)[0]

        t2 = time.perf_counter()
        with concurrent.futures.ThreadPoolExecutor(nth) as ex:
            list(ex.map(one, range(S)))
        cpu_all_s = time.perf_counter() - t2
        result["cpu_baseline_cpu_share"] = {
            "value": round(S / cpu_all_s, 3), "unit": "scans/s", "cores": nth, "kind": "port",
            "sample": f"the same {S} jobs, {nth} independent single-threaded jobs at a time: the CPU share a "
                      f"one-GPU box gives this job ({nth} threads), not the host's {os.cpu_count()} cores"}
    if world == 1 and args.exact_line and not args.no_cpu_baseline:
        result["exact_voxel_order"] = exact_line(cfg, corner_map, surf_map, scans, guesses, ref, ref_iters, ref_nsel)
    print(json.dumps(result), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
