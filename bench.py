#!/usr/bin/env python3
"""bench.py -- Mrays/s of the MI355X path-tracing core (BASELINE.json metric).

A step is one pass of the hot path over one batch: every pixel of a 1920x1080 frame of
Scenes/bounce.txt (camera 0, recursion 10) gets 256 camera samples (configs[1]).  Scene
buffers and the fp64 framebuffer stay resident in HBM; only the timed kernels run inside
the timed region.  One ray = one Scene.RayTrace call (Raytracer.cs:77); one sample = one
GetColor(x, y) (misses included, FullRaytracer.cs:343).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): weak
scaling.  A step is one frame of N * 256 samples per pixel; the frame's rows are dealt to the
ranks as interleaved 8-row bands (rank r: bands r, r+N, ...), each rank renders its rows with
all of the frame's samples (the same work as one GPU's step at N = 1), and the band
accumulators are gathered onto rank 0 with one RCCL gather per step and added into the frame
(the progressive merge of FullRaytracer.cs:326-344), overlapped with the next step's render.
`--split samples` instead gives every rank the whole frame with a disjoint sample range and
reduces the accumulators onto rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (scene fixture, camera, width, height, spp)
    "bounce1080": ("bounce.txt", 0, 1920, 1080, 256),
    "die1080": ("die.txt", 0, 1920, 1080, 1024),
    "bounce256": ("bounce.txt", 0, 256, 256, 16),
    # C4: procedural 1M-triangle height field in the bounce room (raytracercore_amd/scenes.py)
    "mesh1080": ("@mesh", 0, 1920, 1080, 64),
    # C5: die.txt at 4K, 4096 spp per frame over 8 GPUs = 512 spp per GPU per step (sample-sharded)
    "die4k": ("die.txt", 0, 3840, 2160, 512),
}


def load_scene(rc, scene_file):
    if scene_file == "@mesh":
        from raytracercore_amd.scenes import mesh_scene_text

        return rc.SceneLoader.from_text(mesh_scene_text())
    return rc.SceneLoader.from_file(rc.scene_path(scene_file))
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 vector = fp32 MFMA dense peak
BASELINE_METRIC = "Mrays/sec (primary+secondary) and samples/sec at 1080p, Cornell box"  # BASELINE.json


def scene_counts(scene):
    import raytracercore_amd as rc

    kinds = [p.kind for p in scene.prims]
    n_xf = sum(1 for p in scene.prims if p.kind == rc.RT_PRIM_SPHERE and p.flags & rc.RT_FLAG_TRANSFORMED)
    return kinds.count(rc.RT_PRIM_TRIANGLE), kinds.count(rc.RT_PRIM_SPHERE), kinds.count(rc.RT_PRIM_PLANE), n_xf


def flops_per_ray(st) -> float:
    """SURVEY.md §8(d) compute view, exactly: 20*N_node + 45*N_tri + 30*N_sph + 150 FLOP per ray segment,
    with N_* the node visits / primitive tests per ray segment measured by the instrumented kernel
    (rectangles, boxes' faces and frame faces count as triangles, the BVH order's outer faces too;
    C2: 45*19 + 30*3 + 150 = 1095)."""
    return 20.0 * st["nodes"] + 45.0 * (st["tris"] + st.get("outer", 0.0)) + 30.0 * st["sphs"] + 150.0


def bytes_per_ray(st, scene) -> float:
    """SURVEY.md §8(d) B_ray: 32 + 16 + 32*N_node + 48*N_tri + 16*N_sph (+144 transformed) + 48.
    The BVH kernels' outer faces (st["outer"]) are not in N_tri here: their records are wave-uniform
    scalar loads, one per wave rather than per ray, so they add no per-ray memory traffic."""
    n_tri, n_sph, n_pln, n_xf = scene_counts(scene)
    xf_share = n_xf / n_sph if n_sph else 0.0
    return 32 + 16 + 32.0 * st["nodes"] + 48.0 * st["tris"] + st["sphs"] * (16.0 + 144.0 * xf_share) + 48


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s
MALL_RANDOM_GBS = 8600.0  # MI355X_MICROARCH.md: uniformly random rows of an Infinity-Cache-resident table


def roofline(cfg, fpr, bpr, rays, ms, counters=None):
    """C4 (1M triangles, a ~220 MB BVH + triangle set) is bound by memory: its
    B_ray stream is priced against HBM.  C1-C3/C5 (scene on chip) are bound by fp32 VALU issue:
    the algorithmic FLOP per ray segment x rays per launch / kernel time against the fp32 vector
    peak.  `counters` (profiles/traffic/<config>.json, tools/pmc_summary.py over the same command)
    adds the hardware view: SQ_INSTS_VALU_FLOPS_FP32 x 64 per launch / kernel time and the VALU
    issue rate per SIMD-cycle."""
    secs = ms * 1e-3
    if cfg == "mesh1080":
        gbs = bpr * rays / secs / 1e9
        return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                "infinity_cache_view": {"peak": MALL_RANDOM_GBS, "frac": round(gbs / MALL_RANDOM_GBS, 4),
                                        "basis": "MI355X_MICROARCH.md: uniformly random rows of a table resident "
                                                 "in the 256 MiB Infinity Cache, 8.6 TB/s"},
                "note": f"SURVEY B_ray {bpr:.0f} B per ray segment (node visits and triangle tests measured by the "
                        f"instrumented kernel) x {rays:.4g} rays per launch / path-kernel time.  The contract "
                        f"prices these bytes against HBM (8 TB/s), but the ~220 MB scene is resident in the 256 MB "
                        f"Infinity Cache (MALL): the misses of the 4 MB L2s are served by the MALL, not HBM, and "
                        f"the PMC traffic (FETCH_SIZE, which counts MALL hits) is fabric bytes, not HBM bytes.  "
                        f"What bounds the kernel is the vector-memory pipeline (L1 tag lookups, L2 latency: "
                        f"DESIGN 3.3a), so this is a fabric-bandwidth figure, not an HBM one"}
    tf = fpr * rays / secs / 1e12
    out = {"bound": "valu_fp32", "achieved": round(tf, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": round(tf / FP32_PEAK_TFLOPS, 4), "traffic": None,
           "note": f"fp32 VALU kernel, no MFMA (gfx950 fp32 vector peak {FP32_PEAK_TFLOPS} TFLOP/s); SURVEY 8(d) "
                   f"{fpr:.0f} FLOP per ray segment x {rays:.4g} rays per launch / path-kernel time; the scene is "
                   f"compiled into the kernel (SGPR/literal operands), so the only HBM stream is the per-item "
                   f"partials (traffic)"}
    if counters and "valu_flops_fp32" in counters:
        hw = counters["valu_flops_fp32"] * 64 / secs / 1e12
        out["counter_view"] = {
            "achieved": round(hw, 3), "frac": round(hw / FP32_PEAK_TFLOPS, 4), "unit": "TFLOP/s",
            "valu_issue_per_simd_cycle": counters.get("valu_issue_per_simd_cycle"),
            "valu_lane_utilisation": counters.get("valu_lane_utilisation"),
            "basis": "SQ_INSTS_VALU_FLOPS_FP32 x 64 per launch (PMC, tools/pmc_summary.py) / live path-kernel time"}
    return out


def path_stats(gpu, W, H, spp, seed, d_rays):
    """One untimed instrumented launch: traversal work per ray segment (N_node, N_tri, N_sph of the
    SURVEY formulas) and, for the BVH kernels, where the lane slots of the loop go."""
    import torch

    dev = d_rays.device
    d_sum = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
    d_n = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_m = torch.zeros(W * H, dtype=torch.int32, device=dev)
    gpu.set_stats(True)
    d_rays.zero_()
    gpu.render_device(0, 0, W, H, spp, seed, 1 << 40, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(),
                      d_rays.data_ptr(), 0)
    st = gpu.get_stats()
    gpu.set_stats(False)
    rays = max(1, int(d_rays.item()))
    # (the brute-force kernels' cycle-counter split is not reported: read on the generic STATS
    # kernel with s_memtime around sections whose loads are still in flight, it disagreed with the
    # duplicated-section costs of the timed kernel)
    out = {"nodes": st["node_visits"] / rays, "tris": st["tri_tests"] / rays, "sphs": st["sph_tests"] / rays,
           "outer": st["outer_tests"] / rays,
           "wave_iters_per_ray": round(st["wave_iters"] * 64 / rays, 4), "lane_slots": None}
    if gpu.info().traversal in (2, 3):  # BVH kernels: the three "cycle" counters count lane slots
        slots = st["wave_iters"] * 64
        node, leaf, idle, wait = st["node_visits"], st["cyc_start"], st["cyc_trace"], st["cyc_shade"]
        out["lane_slots"] = {k: round(v / rays, 3) for k, v in (
            ("node_step", node), ("leaf_step", leaf), ("traversing_idle", idle), ("waiting_for_shading", wait),
            ("no_work", slots - node - leaf - idle - wait))}
        out["stack"] = {"overflow_pushes_per_ray": round(st["stack_overflow_pushes"] / rays, 4),
                        "max_depth": st["max_stack_depth"]}
    return out


def host_cores():
    """The host CPUs this process may use (affinity mask, any cgroup CPU quota, the job's CPU share),
    the machine's CPU count and the CPU model string (nproc and the model are recorded)."""
    total = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = total
    quota = None
    try:  # cgroup v2: "max 100000" or "<quota> <period>"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    share = None  # the CPU share a job scheduler allots (the GPU box exports it as OMP_NUM_THREADS)
    try:
        share = int(os.environ["OMP_NUM_THREADS"]) or None
    except (KeyError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    threads = min(v for v in (usable, quota, share) if v)
    return {"nproc": total, "affinity": usable, "cgroup_quota": quota, "job_share": share, "threads": threads,
            "cpu_model": model}


def cpu_baseline(cfg_name: str, threads: int = 0):
    """The oracle (C++ fp64 restatement of the reference algorithm, FullRaytracer's tile passes)
    on every host core this process may use, over a bounded sample of the workload."""
    from oracle.oracle import OracleScene
    import raytracercore_amd as rc

    hc = host_cores()
    threads = threads or hc["threads"]
    scene_file, cam, W, H, spp_cfg = CONFIGS[cfg_name]
    if scene_file == "@mesh":  # 1M triangles: the reference's collect-all-leaves query is slow, so
        from raytracercore_amd.scenes import mesh_scene_text  # a half-size frame at 1 spp

        orc = OracleScene.from_text(mesh_scene_text())
        W, H, spp = W // 2, H // 2, 1
    else:
        orc = OracleScene.from_file(rc.scene_path(scene_file))
        # C1 (bounce256) in full; the larger frames at 16 spp (a few seconds on 16 host threads)
        spp = spp_cfg if W * H <= 65536 else 16
    orc.set_size(W, H)
    orc.select_camera(cam)
    _, n, m, rays, secs, used = orc.render_frame(spp, seed=0, threads=threads)
    return {
        "value": round(rays / secs / 1e6, 3),
        "unit": "Mrays/s",
        "cores": used,
        "kind": "port",
        "host": hc,
        "sample": f"{scene_file} camera {cam} {W}x{H} x {spp} spp (1 spp per tile pass, FullRaytracer tiling), "
                  f"{rays} rays in {secs:.2f} s on {used} threads ({hc['cpu_model']}, nproc {hc['nproc']}); "
                  f"samples/s {W * H * spp / secs:.4g}; C++ fp64 restatement, not the C# binary",
    }


def frame_split(args) -> int:
    """--split frame: the product's multi-GPU path, timed.  One process, rt_frame over devices
    0..N-1 (rtcore_api.hip rt_frame_render: every device renders its interleaved 8-row band set with
    all of the step's samples, one RCCL ncclGather over xGMI onto device 0, one copy to pinned host
    memory, the host merge into SampleSet-order buffers).  A step is one frame of N x spp samples
    per pixel (the same per-GPU work at every N, like the default split), and its time includes the
    gather, the device -> host copy and the host merge: a host-buffer (PCIe-inclusive) rate, not the
    HBM-resident `value` of the default split.  Run as ONE process (not under torchrun)."""
    import numpy as np

    import raytracercore_amd as rc

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--split frame drives every GPU from one process: run it without torchrun")
    n = args.gpus
    if rc.device_count() < n:
        raise SystemExit(f"--split frame: {n} GPUs asked, {rc.device_count()} visible")
    scene_file, cam, W, H, spp = CONFIGS[args.config]
    if args.spp > 0:
        spp = args.spp
    scene = load_scene(rc, scene_file)
    frame = rc.GpuFrame(scene, cam, n_gpus=n, size=(W, H))
    frame_spp = spp * n
    acc = (np.zeros((W, H, 3), np.float64), np.zeros((W, H), np.uint32), np.zeros((W, H), np.uint32))
    for k in range(args.warmup):
        frame.render(frame_spp, args.seed, k * frame_spp, out=acc)
    # two-stage pipeline (rt_frame_submit / rt_frame_collect): step k+1 renders on the devices while
    # step k is gathered, copied to the host and merged; every step is collected inside the timing
    rays = 0
    step_ms = []
    first, last = args.warmup, args.warmup + args.steps
    t0 = time.perf_counter()
    frame.submit(frame_spp, args.seed, first * frame_spp)
    for k in range(first, last):
        s0 = time.perf_counter()
        if k + 1 < last:
            frame.submit(frame_spp, args.seed, (k + 1) * frame_spp)
        rays += frame.collect(acc)[3]
        step_ms.append((time.perf_counter() - s0) * 1e3)
    elapsed = time.perf_counter() - t0
    expect = frame_spp * (args.warmup + args.steps)
    tot = acc[1].astype(np.int64) + acc[2].astype(np.int64)
    if not np.all(tot == expect):
        raise SystemExit(f"sample bookkeeping mismatch: {np.unique(tot)} != {expect}")
    frame.close()
    out = {
        "metric": "Mrays/sec (primary+secondary), multi-GPU product path (rt_frame, host buffers)",
        "value": round(rays / elapsed / 1e6, 2), "unit": "Mrays/s", "n_gpus": n, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: the reference's own scene file (tests/golden/scenes) with seeded camera samples",
        "config": {"workload": f"{scene_file} camera {cam} {W}x{H} x {spp} spp per GPU per step",
                   "parallelism": f"rt_frame: one process, {n} GPU(s), interleaved 8-row band sets, "
                                  + ("one ncclGather over xGMI per step" if n > 1 else "a one-rank RCCL gather")
                                  + ", merge into host SampleSet buffers overlapped with the next step's render"},
        "step_ms_min": round(min(step_ms), 3), "step_ms_max": round(max(step_ms), 3),
        "roofline": None,
        "note": "host-buffer rate (includes the gather, the device -> host copy of 32 B per pixel and the host "
                "merge, the last step's exposed); the HBM-resident rate of the same per-GPU work is the default "
                "split's `value`",
    }
    print(json.dumps(out), flush=True)
    return 0


def launch_ranks(args_list, n: int) -> int:
    """`--gpus N` (N > 1) without a launcher: start N fresh rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run would) and return the worst
    exit status.  Runs before anything here touches the GPU; the children are new processes, not an
    exec of this one.  Rank 0's JSON line is the only one printed."""
    import socket
    import subprocess

    with socket.socket() as sk:  # a free port on the loopback for the rendezvous
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(args_list), env=env))
    # a rank that fails leaves the others waiting in the rendezvous or a collective: stop them
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="bounce1080", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override samples per pixel per step")
    ap.add_argument("--traversal", default="auto", choices=["auto", "brute", "bvh", "bvh2", "grouped"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--split", default="bands", choices=["bands", "samples", "frame"],
                    help="multi-GPU split: interleaved row bands + gather (default) or sample ranges + reduce, "
                         "one rank per GPU over torch.distributed; or `frame`: ONE process drives --gpus GPUs "
                         "through the library's own rt_frame (the product path a C# host calls: band sets, "
                         "ncclGather to device 0, merge into host SampleSet buffers)")
    ap.add_argument("--dump", default="", help="rank 0 writes the frame accumulators of the warm-up and timed "
                                               "steps (sum, samples, misses) to this .npz (tests)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be at least 1")
    if args.split == "frame":
        return frame_split(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(sys.argv[1:], args.gpus)
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')}: launch one rank per GPU")

    import numpy as np
    import torch
    import torch.distributed as dist

    import raytracercore_amd as rc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RTCORE_BENCH_SAME_DEVICE") == "1":  # rehearsal of the N-rank path on one GPU
        local = 0
    if world > 1:
        if os.environ.get("RTCORE_BENCH_SAME_DEVICE") == "1":  # RCCL refuses two ranks on one GPU
            dist.init_process_group(backend="gloo")
        else:
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"world size {dist.get_world_size()} != --gpus {args.gpus}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    scene_file, cam, W, H, spp = CONFIGS[args.config]
    if args.spp > 0:
        spp = args.spp
    scene = load_scene(rc, scene_file)
    trav = {"auto": rc.RT_TRAVERSAL_AUTO, "brute": rc.RT_TRAVERSAL_BRUTE, "bvh": rc.RT_TRAVERSAL_BVH,
            "bvh2": rc.RT_TRAVERSAL_BVH2, "grouped": rc.RT_TRAVERSAL_GROUPED}[args.traversal]
    gpu = rc.GpuRaytracer(scene, cam, device=local, size=(W, H), traversal=trav)
    info = gpu.info()
    npix = W * H
    # frame accumulators on rank 0 (SampleSet[w, h]: sum RGB fp64 planes, samples, misses)
    f_sum = torch.zeros(3 * npix, dtype=torch.float64, device=dev)
    f_n = torch.zeros(npix, dtype=torch.int32, device=dev)
    f_m = torch.zeros(npix, dtype=torch.int32, device=dev)
    d_rays = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    from raytracercore_amd import sharding

    if args.split == "bands":
        # rank r renders the band set (BAND, N, r) of a frame of N * spp samples per pixel: the same
        # per-GPU work at every N (weak scaling), one RCCL gather of the band slots per step
        band = sharding.BAND
        plane = sharding.slot_rows(H, world, band) * W
        rows = sharding.row_index(H, world, band, device=dev)
        frame_spp = spp * world
        # two slot sets: step k renders into set k % 2 while set (k-1) % 2 is gathered and merged
        slots = [torch.zeros(4 * plane, dtype=torch.float64, device=dev) for _ in range(2)]
        glists = [[torch.empty_like(slots[0]) for _ in range(world)] if (rank == 0 and world > 1) else None
                  for _ in range(2)]

        def step(k: int) -> None:
            slot = slots[k % 2]
            slot.zero_()
            s_, n_, m_ = sharding.slot_views(slot, plane)
            gpu.render_bands_device(band, world, rank, frame_spp, args.seed, k * frame_spp, s_.data_ptr(),
                                    n_.data_ptr(), m_.data_ptr(), plane, d_rays.data_ptr(), stream)

        def start_merge(k: int):
            return k, sharding.gather_slots(slots[k % 2], glists[k % 2], dist, async_op=True)

        def apply_merge(k: int) -> None:
            if rank == 0:
                got = glists[k % 2] if world > 1 else [slots[k % 2]]
                sharding.scatter_slots(f_sum, f_n, f_m, got, rows, W, plane)
        expect_per_step = frame_spp
        parallelism = (f"row bands x{world} (interleaved {band}-row bands, {frame_spp} spp per frame), "
                       + ("RCCL gather per step" if world > 1 else "one GPU, no collective"))
    else:
        # sample sharding: every rank renders the whole frame with its own sample range; one RCCL
        # reduce per accumulator plane per step
        sets = [(torch.zeros_like(f_sum), torch.zeros_like(f_n), torch.zeros_like(f_m)) for _ in range(2)]

        def step(k: int) -> None:
            base = sharding.sample_base(k, rank, world, spp)
            d_sum, d_n, d_m = sets[k % 2]
            d_sum.zero_()
            d_n.zero_()
            d_m.zero_()
            gpu.render_device(0, 0, W, H, spp, args.seed, base, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(),
                              d_rays.data_ptr(), stream)

        def start_merge(k: int):
            return k, sharding.merge_accumulators(sets[k % 2], dist, async_op=True)

        def apply_merge(k: int) -> None:
            if rank == 0:
                d_sum, d_n, d_m = sets[k % 2]
                f_sum.add_(d_sum)
                f_n.add_(d_n)
                f_m.add_(d_m)
        expect_per_step = spp * world
        parallelism = f"sample-sharded x{world}, " + ("RCCL reduce per step" if world > 1 else "one GPU, no collective")

    def finish_merge(pending) -> None:
        k, works = pending
        for w in works:
            w.wait()  # the compute stream waits for the collective, not the host
        apply_merge(k)

    def run(first: int, count: int) -> list:
        # each launch records its own hipEvent pair around the path kernel (a ring of 64 per scene):
        # the steps queue without a host sync and their kernel times are read every 64 steps
        kernel_ms = []
        pending = None
        queued = 0
        for k in range(first, first + count):
            step(k)
            queued += 1
            if queued == gpu.KERNEL_TIME_RING:
                kernel_ms += gpu.kernel_times(queued)
                queued = 0
            if pending is not None:
                finish_merge(pending)
            pending = start_merge(k)
        if pending is not None:
            finish_merge(pending)
        if queued:
            kernel_ms += gpu.kernel_times(queued)
        return kernel_ms

    run(0, args.warmup)
    torch.cuda.synchronize(dev)
    d_rays.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    kernel_ms = run(args.warmup, args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    rays = d_rays.clone()
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
    elapsed = float(elapsed.item())
    total_rays = int(rays.item())
    total_samples = npix * spp * args.steps * world
    avg_ms = sum(kernel_ms) / len(kernel_ms)

    # bookkeeping of the timed and warm-up steps (before the untimed diagnostic steps below)
    if rank == 0:
        n_all = f_n.cpu().numpy().astype(np.int64)
        m_all = f_m.cpu().numpy().astype(np.int64)
        expect = expect_per_step * (args.steps + args.warmup)
        if not np.all(n_all + m_all == expect):
            raise SystemExit(f"sample bookkeeping mismatch: {np.unique(n_all + m_all)} != {expect}")
        if args.dump:
            np.savez(args.dump, sum=f_sum.cpu().numpy().reshape(3, H, W), samples=n_all.reshape(H, W),
                     misses=m_all.reshape(H, W))

    multi = None
    if world > 1:
        # where an N-GPU step's time goes, from untimed steps after the timed region: every rank's
        # path-kernel time, and the render, collective and merge phases run one at a time
        ks = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(ks, torch.tensor([avg_ms], dtype=torch.float64, device=dev))
        k_all = [float(t.item()) for t in ks]
        phases = []
        for j in range(3):
            k = args.warmup + args.steps + j
            torch.cuda.synchronize(dev)
            dist.barrier()
            p0 = time.perf_counter()
            step(k)
            torch.cuda.synchronize(dev)
            p1 = time.perf_counter()
            dist.barrier()  # the collective starts when every rank has rendered
            p2 = time.perf_counter()
            _, works = start_merge(k)
            for w in works:
                w.wait()
            torch.cuda.synchronize(dev)
            p3 = time.perf_counter()
            apply_merge(k)
            torch.cuda.synchronize(dev)
            p4 = time.perf_counter()
            phases.append(torch.tensor([p1 - p0, p3 - p2, p4 - p3], dtype=torch.float64, device=dev))
        ph = torch.stack(phases).median(dim=0).values
        dist.all_reduce(ph, op=dist.ReduceOp.MAX)
        multi = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                 "kernel_ms_per_rank": [round(v, 3) for v in k_all],
                 "kernel_ms_min": round(min(k_all), 3), "kernel_ms_max": round(max(k_all), 3),
                 "render_ms": round(float(ph[0]) * 1e3, 3),
                 ("gather_ms" if args.split == "bands" else "reduce_ms"): round(float(ph[1]) * 1e3, 3),
                 ("scatter_ms" if args.split == "bands" else "add_ms"): round(float(ph[2]) * 1e3, 3),
                 "basis": "median of 3 untimed steps after the timed region, phases run one at a time "
                          "(max over ranks); in the timed steps the collective of step k overlaps the "
                          "render of step k+1"}

    if rank == 0:
        my_rays_per_step = total_rays / (args.steps * world)  # the average rank's launch
        build = gpu.build_stats()  # of the timed launches (before the instrumented one below)
        # the BVH kernels' lane-slot split depends on the launch's length (its tail), so they are
        # instrumented at the timed launch's spp; the brute-force kernels at 1/16 of it
        st = path_stats(gpu, W, H, spp if info.traversal in (2, 3) else max(1, spp // 16), args.seed, d_rays)
        fpr = flops_per_ray(st)
        bpr = bytes_per_ray(st, scene)
        counters = None
        traffic_file = os.path.join(ROOT, "profiles", "traffic", f"{args.config}.json")
        # PMC figures of this launch shape (tools/profile.sh); the profiles are of the 1-GPU launch
        if os.path.exists(traffic_file) and args.spp == 0 and world == 1:
            counters = json.load(open(traffic_file))
        metric = BASELINE_METRIC if args.config == "bounce1080" else \
            f"Mrays/sec (primary+secondary) and samples/sec, {scene_file} {W}x{H}"
        out = {
            "metric": metric,
            "value": round(total_rays / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: the reference's own scene file (tests/golden/scenes) with seeded camera samples",
            "config": {"workload": f"{scene_file} camera {cam} {W}x{H} x {spp} spp per GPU per step",
                       "traversal": ["auto", "brute", "bvh4", "bvh2", "grouped"][info.traversal], "recursion": scene.params.recursion,
                       "kernel_build": "scene-specialised (hiprtc)" if build.get("jit_status") == 1.0 else "generic",
                       "parallelism": parallelism},
            "samples_per_s": round(total_samples / elapsed, 1),
            # the reference's only published figure: 6.240 spp/s at 700x700 on bounce.txt,
            # i.e. 3.06 M camera samples/s, on an unknown ~32-thread CPU; a different metric from
            # Mrays/s, so vs_baseline stays null
            "published_reference": {"samples_per_s": 3.0576e6, "source": "Screenshots/app.png status bar"},
            "rays_per_sample": round(total_rays / total_samples, 4),
            "kernel_ms": round(avg_ms, 3),
            "roofline": roofline(args.config, fpr, bpr, my_rays_per_step, avg_ms, counters),
            "path_stats": {"per_ray": {k: round(st[k], 3) for k in ("nodes", "tris", "sphs", "outer")},
                           "flop_per_ray": round(fpr, 1), "bytes_per_ray": round(bpr, 1),
                           "rays_per_launch": round(my_rays_per_step),
                           "lane_slots_per_ray": st["wave_iters_per_ray"],
                           **({"lane_slots": st["lane_slots"]} if st["lane_slots"] else {}),
                           **({"stack": st["stack"]} if "stack" in st else {})},
            "multi_gpu": multi,
            "scene_build": {"builder": ["auto", "host", "gpu"][info.bvh_builder],
                            **{k: round(v, 2) for k, v in build.items()}},
        }
        if counters is not None:
            rf = out["roofline"]
            rf["traffic"] = counters["traffic_bytes"]
            if rf["bound"] == "hbm":
                # the measured view beside the algorithmic one (frac, the headline, is SURVEY B_ray):
                # PMC bytes past L2 per launch / kernel time.  The ~220 MB scene fits the 256 MB
                # Infinity Cache, so part of these bytes are MALL hits, not HBM reads.
                gbs = rf["traffic"] / (avg_ms * 1e-3) / 1e9
                rf["measured"] = {"achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "unit": "GB/s",
                                  "basis": "PMC 2 x FETCH_SIZE + WRITE_SIZE per launch (L2 -> fabric, includes "
                                           "Infinity Cache hits) / path-kernel time"}
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_threads)
        print(json.dumps(out), flush=True)
    gpu.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
