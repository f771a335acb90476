#!/usr/bin/env python3
"""Benchmark: rendered Mpix/s, forward+backward, 1M Gaussians @ 1920x1080 (BASELINE.json).

One step = one optimizer step's batch of camera views (BASELINE config 4): for each
view this rank owns, forward + backward of the differentiable rasterizer through the drop-in
surface (diff_gaussian_rasterization.GaussianRasterizer + autograd), gradients accumulated into
the replicated Gaussian parameters (by default inside dgr.deferred_backward: each view's render
backward right after its forward, the views alternating over two HIP streams, and ONE batched
preprocess backward for the step's views); then, with N>1 ranks, ONE RCCL all_reduce(SUM) of the
236 B/Gaussian parameter-gradient bucket.  Every view is BASELINE config 2's workload (1M
Gaussians, SH degree 3, one 1920x1080 ring view, fwd+bwd).

Default (strong scaling, config 4 as §8e defines it): `--views-total 8` views per step at every N,
view v on rank v mod N -- 8 views on one GPU, 1 view + the all-reduce per GPU at N=8, so the N=1
and N=8 lines describe the same 8-view step.  `--views-per-rank K` (weak scaling): K views per
rank at every N, the same K at N=1.

Run: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no WORLD_SIZE in the
environment, this process runs the PMC passes (rank 0's workload) and then starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py ...` as a child (it never
touches the GPU itself, and never re-execs), relays rank 0's JSON line and exits with the child's
code; under an external torch.distributed.run WORLD_SIZE must equal N.  One rank per GPU over RCCL
("nccl"); GSR_DIST_BACKEND=gloo is the one-GPU rehearsal of the same ranks.
Prints ONE JSON line on rank 0.
"""
import argparse
import contextlib
import ctypes
import glob
import hashlib
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-npu_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import synthetic  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMD-32 units, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md), at the 2.4 GHz the PMC runs measure (GRBM_GUI_ACTIVE / kernel time)
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2  # 1,228.8 G wave-instructions/s
N_RING = 8  # distinct ring cameras (synthetic.Camera)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--views-total", type=int, default=8,
                    help="views per step over all ranks (strong scaling; view v on rank v mod N)")
    ap.add_argument("--views-per-rank", type=int, default=0,
                    help="> 0: weak scaling, this many views per rank at every N (overrides --views-total)")
    ap.add_argument("--antialiasing", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every usable host core (affinity mask, bounded by a cgroup CPU quota)")
    ap.add_argument("--cpu-reps", type=int, default=10,
                    help="CPU baseline runs (median reported; ~1 s each at the default workload)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event timing")
    ap.add_argument("--no-aux", action="store_true", help="skip the §8f side measurements (distCUDA2)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the in-run rocprofv3 --pmc passes (traffic then from the stamped profiles/ file)")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false",
                    help="render the views of a step one after the other on one stream")
    ap.add_argument("--no-prefix-stream", action="store_true",
                    help="run the forward's binning prefix on the caller's stream, not the library's priority stream")
    ap.add_argument("--per-view", dest="batch_views", action="store_false",
                    help="render the views one GaussianRasterizer call at a time (alternating over two streams, "
                         "deferred_backward) instead of the default: this rank's views as ONE MultiViewRasterizer "
                         "batch (binning prefix batched over the views, one backward preprocess pass)")
    ap.add_argument("--no-deferred", dest="deferred", action="store_false",
                    help="--per-view: every view's full backward on its own (default: per-view render backward, "
                         "ONE batched preprocess backward per step, dgr.deferred_backward)")
    ap.add_argument("--order", choices=("interleave", "lookahead", "forward-first"), default="interleave",
                    help="issue order of the step's views: forward+backward per view, the next view's forward "
                         "before this view's backward, or every forward before every backward")
    ap.add_argument("--no-fused-accumulation", action="store_true",
                    help="accumulate the views' gradients with autograd's separate add instead of in the kernel")
    ap.add_argument("--no-overlap-allreduce", action="store_true",
                    help="N > 1: all-reduce the gradients after the backward instead of overlapped with it")
    ap.add_argument("--allreduce-chunks", type=int, default=4,
                    help="N > 1: Gaussian ranges of the overlapped gradient all-reduce")
    ap.add_argument("--no-single-view", action="store_true",
                    help="skip the config2_single_view leg (plain GaussianRasterizer fwd+bwd of view 0, own roofline)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)  # workload under a --pmc pass
    # the pmc child of rank 0 of an N-rank run (started before the process group): rank 0's views
    ap.add_argument("--pmc-world", type=int, default=0, help=argparse.SUPPRESS)
    # the ranks' copy of the launcher's PMC figures (JSON file), read by rank 0
    ap.add_argument("--pmc-file", default="", help=argparse.SUPPRESS)
    # launch check (CPU test): each rank prints {"rank", "world", "local_rank"} and exits, no GPU
    ap.add_argument("--rank-probe", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def tile_diff_cells(W, H):
    """(gx + 1) (gy + 1) when the library takes the tile ranges from the rects' difference array
    (gsr_common.h use_tile_diff: <= 255 x 255 tiles, <= 8,704 cells, <= 8,192 tiles), else 0."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    cells = (gx + 1) * (gy + 1)
    return cells if gx <= 255 and gy <= 255 and cells <= 8704 and gx * gy <= 8192 else 0


def algorithmic_bytes(P, M, L, N, T, P_vis, views_per_bwd=1, diff_cells=0):
    """Compulsory HBM bytes per launch of each kernel (split per kernel).
    views_per_bwd: views whose preprocess backward one launch covers (deferred_backward batches a
    step's views: the parameters are read and their gradients written once, the per-view radii and
    render gradients V times).  diff_cells: the tile ranges come from the rects' difference array
    (tile_hist: packed rects in, 16 workgroups' arrays added out; the tile sort writes no tile ids)."""
    params = 4 * (11 + 3 * M)  # means 12 + scales 12 + rot 16 + opacity 4 + SH 12M
    return {
        # params in; key, radius, tile count, rect out per Gaussian; splat record 48 + conic 16 +
        # means2D 8 + rgb 12 + depth 4 + clamped 1 per visible Gaussian
        "preprocess_fwd": P * (params + 20) + P_vis * 89,
        # depth keys in, sorted ids out; rects gathered and laid out in depth order, tile counts out
        "depth_sort": P * 28,
        "scan": P * 8,                                          # depth-ordered tile counts in, offsets out
        # ids, offsets, rects, record starts in; (tile, (record slot, id)) per instance + valid bits out
        "emit_instances": P * 20 + L * 12 + L // 8,
        # with the difference array (slotless, emission fused into pass 1): depth-ordered ids, offsets and
        # packed rects in per Gaussian, the 4-B id word out (pass 1), in and out (pass 2); without it,
        # (tile, slot, id) in and out
        "tile_sort": P * 12 + L * 12 if diff_cells else L * 24,
        # tile_hist: packed rects in, 16 workgroup arrays added; else a pass over the sorted tile ids
        "tile_ranges": P * 4 + 16 * 4 * diff_cells if diff_cells else L * 4 + T * 8,
        # the mean of its two launches per view: the forward's (ranges in, launch order out -- with the
        # difference array: its cells in, every 8-B range and the order out) and the backward's
        # (per-tile work in, launch order out)
        "tile_order": ((4 * diff_cells + 12 * T if diff_cells else 12 * T) + 8 * T) // 2,
        "render_fwd": L * 44 + N * 24 + T * 8,                  # id + 40 B record per instance; 24 B/pixel out
        # id + record per instance, 24 B/pixel in; the 40-B gradient record (GSR_GRAD_REC 10 floats) out
        # per visible Gaussian (SURVEY §8d's per-Gaussian record, written once here, read once below)
        "render_bwd": L * 44 + N * 24 + T * 8 + P_vis * 40,
        # params + radii + the 40-B render gradient records in, parameter gradients out
        "preprocess_bwd": P * params + views_per_bwd * (P * 4 + P_vis * 40) + P * (40 + 12 * M),
    }


def lib_sha256():
    """Identity of the native library this process rasterizes with (stamps PMC traffic figures)."""
    import diff_gaussian_rasterization as dgr
    h = hashlib.sha256()
    with open(dgr._C.LIB_PATH, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


PMC_CHILD_STEPS = 2  # the --pmc-child workload: 1 warm-up + 1 step
PMC_COUNTED_STEPS = 1  # the steps after the child's marker kernel (tools/pmc_summary.MARKER)


def workload_stamp(args, world, views_rank):
    """What a PMC figure was measured on: traffic per launch belongs to exactly this workload."""
    return {"P": args.P, "width": args.width, "height": args.height, "views_per_rank": views_rank,
            "world": world, "mode": "batch" if args.batch_views else ("per-view deferred" if args.deferred
                                                                     else "per-view"),
            "antialiasing": bool(args.antialiasing)}


def pmc_traffic(args, world, timeout=240):
    """HBM traffic and VALU wave-instructions of every rasterizer operation, measured now on this
    build: three rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE -- together they exceed the 4 TCC
    counters of one pass -- and SQ_INSTS_VALU) over this script's own workload (`--pmc-child`:
    this rank's views, PMC_CHILD_STEPS steps of which the dispatches after the warm-up's marker
    kernel are counted, nothing else), each a child process under a time
    limit; bytes = 2 FETCH_SIZE + WRITE_SIZE (KiB) per MI355X_MICROARCH.md §HBM.  Returns the
    pmc_summary totals over all dispatches of each operation (the caller divides by the number of
    calls), or None if rocprofv3 is absent or a pass fails."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return None
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_summary
    tmp = tempfile.mkdtemp(prefix="gsr_pmc_")
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "1", "--warmup", "1",
             "--P", str(args.P), "--width", str(args.width), "--height", str(args.height),
             "--views-total", str(args.views_total), "--views-per-rank", str(args.views_per_rank),
             "--pmc-world", str(world)]
    for flag, on in (("--antialiasing", args.antialiasing), ("--per-view", not args.batch_views),
                     ("--no-deferred", not args.deferred), ("--no-overlap", not args.overlap)):
        if on:
            child.append(flag)
    # a clean environment for the child: no rank variables (it is one process, not a rank)
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK")}
    env["TMPDIR"] = tmp
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU"):
            r = subprocess.run([exe, "--pmc", counter, "--output-format", "csv", "-d", os.path.join(tmp, counter),
                                "-o", "run", "--"] + child, env=env, cwd=ROOT, timeout=timeout,
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            if r.returncode != 0:
                return None
        with open(os.devnull, "w") as devnull:
            old, sys.stdout = sys.stdout, devnull
            try:
                pmc_summary.main(tmp)
            finally:
                sys.stdout = old
        t = json.load(open(os.path.join(tmp, "pmc_traffic.json")))
        v = json.load(open(os.path.join(tmp, "pmc_valu.json")))
        return {"bytes_total": t["bytes_total"], "winst_total": v["winst_total"],
                "marked": bool(t.get("marked")) and bool(v.get("marked"))}
    except Exception:
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def single_view_leg(args, timeout=400):
    """config2_single_view: the plain single-view step train.py runs -- one GaussianRasterizer
    forward + full backward of view 0 per step (bench.py --views-total 1 --per-view --no-deferred),
    its own per-kernel times, roofline and PMC traffic, in a child process."""
    cmd = [sys.executable, os.path.abspath(__file__), "--views-total", "1", "--per-view", "--no-deferred",
           "--no-aux", "--no-cpu-baseline", "--no-single-view", "--steps", str(max(args.steps, 20)),
           "--warmup", str(args.warmup), "--P", str(args.P), "--width", str(args.width),
           "--height", str(args.height)] + (["--antialiasing"] if args.antialiasing else []) \
        + (["--no-pmc"] if args.no_pmc else []) + (["--no-profile"] if args.no_profile else [])
    try:
        r = subprocess.run(cmd, cwd=ROOT, timeout=timeout, capture_output=True, text=True)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        d = json.loads(line)
        return {k: d[k] for k in ("value", "unit", "ms_per_step", "ms_per_step_median", "ms_per_step_mean", "value_mean",
                                       "roofline")} | {
            "workload": d["config"]["workload"], "execution": d["config"]["execution"]}
    except Exception as e:
        return {"value": None, "error": f"{type(e).__name__}: {e}"}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(args, argv, port, pmc_file=None):
    """The child command of `bench.py --gpus N` (N > 1): torch.distributed.run with one rank per
    GPU on this node, each rank running this script with the same arguments (`argv`), plus the
    launcher's PMC figures for rank 0 (or --no-pmc when there are none)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    if pmc_file:
        cmd += ["--pmc-file", pmc_file]
    elif "--no-pmc" not in argv:
        cmd.append("--no-pmc")
    return cmd


def launch_ranks(args, argv, timeout=3000):
    """`bench.py --gpus N` without WORLD_SIZE: the PMC passes of rank 0's workload first (child
    processes under rocprofv3, before any rank exists), then N ranks through torch.distributed.run
    as ONE child process of this one -- this process never initialises the GPU and never re-execs.
    The ranks inherit stdout, so rank 0's JSON line is the line this command prints; returns the
    child's exit code."""
    backend = os.environ.get("GSR_DIST_BACKEND", "nccl")
    if backend == "nccl":
        ndev = torch.cuda.device_count()  # counts devices without initialising HIP on this image
        if ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs for RCCL, this node has {ndev} "
                  "(GSR_DIST_BACKEND=gloo rehearses the ranks on fewer)", file=sys.stderr)
            return 2
    pmc_file = None
    if not args.pmc_child and not args.no_pmc and not args.no_profile and not args.rank_probe:
        pmc = pmc_traffic(args, args.gpus)
        if pmc is not None:
            fd, pmc_file = tempfile.mkstemp(prefix="gsr_pmc_", suffix=".json")
            with os.fdopen(fd, "w") as f:
                json.dump(pmc, f)
    cmd = rank_launch_cmd(args, argv, free_port(), pmc_file)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, start_new_session=True)
    try:
        return proc.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, 9)
        proc.wait()
        print(f"bench.py: the {args.gpus}-rank run exceeded {timeout} s", file=sys.stderr)
        return 124
    finally:
        if pmc_file:
            os.unlink(pmc_file)


def rank_views(args, rank, views_world):
    """(scaling, n_ring, this rank's ring views, views per step over all ranks): weak scaling
    (--views-per-rank K) gives every rank K distinct cameras of a ring of max(8, K x world) views;
    strong scaling deals the fixed --views-total batch round-robin."""
    from diff_gaussian_rasterization import multiview
    if args.views_per_rank > 0:
        n_ring = max(N_RING, args.views_per_rank * views_world)
        views = multiview.views_for_rank(rank, views_world, args.views_per_rank, n_views=n_ring)
        return "weak", n_ring, views, views_world * len(views)
    n_ring = max(N_RING, args.views_total)
    return "strong", n_ring, multiview.views_of_batch(rank, views_world, args.views_total), args.views_total


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if not args.pmc_child:
        if env_world is None and args.gpus > 1:
            sys.exit(launch_ranks(args, argv))
        if env_world is not None and int(env_world) != args.gpus:
            print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}", file=sys.stderr)
            sys.exit(2)
    if args.rank_probe:  # (no GPU call: the views come from host arithmetic only)
        r, w = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
        scaling, n_ring, views, views_step = rank_views(args, r, w)
        print(json.dumps({"rank": r, "world": w, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "argv": argv,
                          "scaling": scaling, "n_ring": n_ring, "views": views, "views_step": views_step}),
              flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.pmc_child:  # one process replaying rank 0's share of a `--pmc-world`-rank step
        world, rank, local_rank = 1, 0, 0
    views_world = args.pmc_world if (args.pmc_child and args.pmc_world > 0) else world
    # PMC passes of this rank's workload, on rank 0 only, before the process group exists and before
    # this process touches the GPU (the child replays rank 0's views of the N-rank step)
    pmc = None
    if rank == 0 and args.pmc_file:  # measured by the `--gpus N` launcher before the ranks started
        with open(args.pmc_file) as f:
            pmc = json.load(f)
    elif rank == 0 and not args.pmc_child and not args.no_pmc and not args.no_profile:
        pmc = pmc_traffic(args, world)
    # GSR_DIST_BACKEND=gloo (rehearsal only): several ranks on one GPU exercise the N>1 path of
    # this script on a one-GPU box; the driver's multi-GPU runs use the default, RCCL ("nccl").
    backend = os.environ.get("GSR_DIST_BACKEND", "nccl")
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)

    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import multiview
    lib = dgr._C.lib
    lib.gsr_profile_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    lib.gsr_profile_kernel_name.restype = ctypes.c_char_p
    lib.gsr_set_prefix_stream(0 if args.no_prefix_stream else 1)

    H, W, P = args.height, args.width, args.P
    scene = synthetic.make_scene(P, seed=0)
    params = {k: v.to(dev).requires_grad_(True) for k, v in scene.items()}
    M = params["shs"].shape[1]
    # weak scaling: K views per rank, distinct cameras over all ranks; strong: a fixed batch of views
    # per step, dealt round-robin
    mode, n_ring, views, _ = rank_views(args, rank, views_world)
    scaling = mode
    views_step = world * len(views) if mode == "weak" else args.views_total
    cams, grads = [], []
    for v in views:
        cam = synthetic.Camera(W, H, view=v, n_views=n_ring)
        s = dgr.GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
            bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.world_view_transform.to(dev),
            projmatrix=cam.full_proj_transform.to(dev), sh_degree=3, campos=cam.camera_center.to(dev),
            prefiltered=False, debug=False, antialiasing=args.antialiasing)
        cams.append(s)
        gc, gi = synthetic.make_grads(H, W, seed=1 + v)
        grads.append((gc.to(dev), gi.to(dev)))

    ar_events = []  # (start, end) around the all-reduce, recorded only in the instrumented pass below

    # Views alternate between two HIP streams: the forward of view v+1 (preprocess, the
    # latency-bound sorts and scans, render) runs while the backward of view v occupies the GPU.
    # The backward passes add into the same .grad buffers in view order (dgr.accumulate_grads_in_place
    # orders them with an event), the forward of every view reads only the parameters.
    main_stream = torch.cuda.current_stream(dev)
    streams = [main_stream] + ([torch.cuda.Stream(dev)] if (args.overlap and len(cams) > 1) else [])

    # the screen-space gradient receptacles (gaussian_renderer's screenspace_points), one per view
    means2Ds = [torch.zeros_like(params["means3D"], requires_grad=True) for _ in cams]

    # --batch-views: this rank's views as ONE MultiViewRasterizer node (each view's forward, then
    # every view's render backward and one preprocess backward over the Gaussians for the batch)
    mv = dgr.MultiViewRasterizer(cams) if args.batch_views else None
    means2D_batch = torch.zeros((len(cams), P, 3), device=dev, requires_grad=True) if mv else None
    gc_batch = torch.stack([g[0] for g in grads]) if mv else None
    gi_batch = torch.stack([g[1] for g in grads]) if mv else None

    # N > 1: the gradient all-reduce overlapped with the batched backward (multiview.
    # overlapped_allreduce: the preprocess backward in Gaussian ranges, each range reduced while the
    # next computes) unless --no-overlap-allreduce; comm=False: no collective (compute-only pass)
    overlap_ar = world > 1 and not args.no_overlap_allreduce and (args.batch_views or args.deferred)

    def step(record_allreduce=False, overlap=True, comm=True):
        for p in params.values():
            p.grad = None
        for m in means2Ds:
            m.grad = None
        ovl = overlap_ar and comm and not record_allreduce
        with (multiview.overlapped_allreduce(chunks=args.allreduce_chunks) if ovl else contextlib.nullcontext()):
            if mv is not None:
                means2D_batch.grad = None
                color, radii, inv = mv(means3D=params["means3D"], means2D=means2D_batch, shs=params["shs"],
                                       opacities=params["opacities"], scales=params["scales"],
                                       rotations=params["rotations"])
                torch.autograd.backward([color, inv], [gc_batch, gi_batch])
            else:
                n_st = len(streams) if overlap else 1
                for st in streams[1:n_st]:
                    st.wait_stream(main_stream)  # the step's start (parameters, previous step's collective)
                with (dgr.deferred_backward() if args.deferred else contextlib.nullcontext()):
                    views_loop(n_st)
        if ovl or not comm:
            return
        if record_allreduce:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        nbytes = multiview.allreduce_grads(params)
        if record_allreduce:
            e1.record()
            ar_events.append((e0, e1, nbytes))

    def views_loop(n_st):
        def forward(i):
            st = streams[i % n_st]
            with torch.cuda.stream(st):
                rast = dgr.GaussianRasterizer(raster_settings=cams[i])
                # views after the first add their gradients into the parameters' .grad inside the
                # backward kernel (dgr.accumulate_grads_in_place) instead of autograd's separate add
                with dgr.accumulate_grads_in_place(not args.no_fused_accumulation):
                    color, radii, inv = rast(means3D=params["means3D"], means2D=means2Ds[i], shs=params["shs"],
                                             opacities=params["opacities"], scales=params["scales"],
                                             rotations=params["rotations"])
            return st, color, inv

        def backward(i, out):
            st, color, inv = out
            with torch.cuda.stream(st):
                torch.autograd.backward([color, inv], list(grads[i]))

        n = len(cams)
        if args.order == "interleave":  # forward, backward, next view
            for i in range(n):
                backward(i, forward(i))
        elif args.order == "lookahead":  # the next view's forward is issued before this view's backward
            prev = forward(0)
            for i in range(1, n):
                cur = forward(i)
                backward(i - 1, prev)
                prev = cur
            backward(n - 1, prev)
        else:  # every forward, then every backward
            outs = [forward(i) for i in range(n)]
            for i in range(n):
                backward(i, outs[i])
        for st in streams[1:n_st]:
            main_stream.wait_stream(st)

    if args.pmc_child:  # the workload of one --pmc pass (pmc_traffic): nothing printed, nothing timed
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        # the marker (tools/pmc_summary.MARKER): the summary counts the dispatches after it only --
        # the warm-up holds a first call's binning re-run, geometry dispatches no timed step has
        try:
            torch.cuda._sleep(1)
        except Exception:  # no marker: the summary then counts every step (PMC_CHILD_STEPS)
            pass
        torch.cuda.synchronize()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        return

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # step boundaries on the main stream (for the per-step median; recording costs nothing measurable)
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.steps):
        step()
        marks[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = multiview.max_over_ranks(t1 - t0, dev)
    step_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)]
    median_ms = multiview.max_over_ranks(statistics.median(step_ms) / 1e3, dev) * 1e3

    # per-kernel HIP-event timings: a second, instrumented run of the same steps (the events
    # recorded around every launch cost ~3% of the step, so they stay out of the timed region)
    kern = {}
    if not args.no_profile:
        # one stream: every kernel's duration is its own, not shared with an overlapping view's
        # (the library's internal binning streams off as well)
        lib.gsr_set_prefix_stream(0)
        lib.gsr_profile_enable(1)
        for _ in range(args.steps):
            step(overlap=False)
        torch.cuda.synchronize()
        lib.gsr_set_prefix_stream(0 if args.no_prefix_stream else 1)
        nk = 16
        tot = (ctypes.c_double * nk)()
        cnt = (ctypes.c_int * nk)()
        n = lib.gsr_profile_read(tot, cnt, nk)
        lib.gsr_profile_enable(0)
        for k in range(n):
            if cnt[k]:
                kern[lib.gsr_profile_kernel_name(k).decode()] = {"avg_ms": tot[k] / cnt[k], "launches": cnt[k]}

    # all-reduce share of the step, separate passes: the collective alone (events around
    # a non-overlapped allreduce_grads), and the step without any collective (compute only); the
    # exposed communication is the timed step minus the compute-only step
    allreduce = None
    if world > 1:
        for _ in range(min(args.steps, 5)):
            step(record_allreduce=True)
        torch.cuda.synchronize()
        ar_ms = sum(a.elapsed_time(b) for a, b, _ in ar_events) / len(ar_events)
        ar_ms = multiview.max_over_ranks(ar_ms / 1e3, dev) * 1e3
        n_c = min(args.steps, 10)
        dist.barrier()
        tc0 = time.perf_counter()
        for _ in range(n_c):
            step(comm=False)
        torch.cuda.synchronize()
        dist.barrier()
        compute_ms = multiview.max_over_ranks((time.perf_counter() - tc0) / n_c, dev) * 1e3
        step_ms = elapsed / args.steps * 1e3
        allreduce = {"ms_standalone": round(ar_ms, 4), "bytes_per_rank": ar_events[0][2],
                     "algbw_GBps": round(ar_events[0][2] / (ar_ms * 1e-3) / 1e9, 1),
                     "overlapped": overlap_ar, "chunks": args.allreduce_chunks if overlap_ar else 1,
                     "compute_only_ms_per_step": round(compute_ms, 4),
                     "exposed_ms": round(max(step_ms - compute_ms, 0.0), 4),
                     "fraction_of_step": round(max(step_ms - compute_ms, 0.0) / step_ms, 3),
                     "standalone_fraction_of_step": round(ar_ms / step_ms, 3)}

    # geometry of the workload (one extra forward per view outside the timed region)
    with torch.no_grad():
        Ls, vis = [], []
        for s in cams:  # per-view geometry, averaged like the per-kernel times are
            out = dgr._C.rasterize_gaussians(s.bg, params["means3D"], torch.Tensor([]), params["opacities"],
                                             params["scales"], params["rotations"], 1.0, torch.Tensor([]),
                                             s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, params["shs"], 3,
                                             s.campos, False, args.antialiasing, False)
            Ls.append(int(out[0]))
            vis.append(int((out[2] > 0).sum().item()))
        L = round(sum(Ls) / len(Ls))
        P_vis = round(sum(vis) / len(vis))
    N = H * W
    T = ((W + 15) // 16) * ((H + 15) // 16)
    pix_total = views_step * N * args.steps
    # the median step is the headline (value, ms_per_step); the mean over the bracketed
    # K steps (wall clock between the barriers, max over ranks) is reported beside it
    value_mean = pix_total / elapsed / 1e6
    value = views_step * N / (median_ms * 1e-3) / 1e6
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    roofline = None
    if kern:
        batched_bwd = args.batch_views or args.deferred
        ab = algorithmic_bytes(P, M, L, N, T, P_vis, views_per_bwd=min(len(cams), 16) if batched_bwd else 1,
                               diff_cells=tile_diff_cells(W, H))
        if args.batch_views:  # a batch's views share every launch (grid.y = view, up to 8 views per launch)
            vb = min(len(cams), 8)
            for k in ("depth_sort", "scan", "emit_instances", "tile_sort", "tile_ranges", "tile_order", "render_fwd",
                      "render_bwd"):
                ab[k] *= vb
            # the batched preprocess reads the parameters once for its views
            params_b = P * 4 * (11 + 3 * M)
            # (and writes no means2D / depth / rgb / conic_opacity: 40 B per visible Gaussian and view,
            # read by nothing -- preprocess_bwd recomputes the conic)
            ab["preprocess_fwd"] = params_b + vb * (ab["preprocess_fwd"] - params_b - P_vis * 40)
        # the dominant kernel: the largest share of the step (mean launch time x launches per step)
        dom = max(kern, key=lambda k: kern[k]["avg_ms"] * kern[k]["launches"])
        achieved = ab[dom] / (kern[dom]["avg_ms"] * 1e-3) / 1e9
        sha = lib_sha256()
        stamp = workload_stamp(args, world, len(cams))
        # calls of each operation during the PMC child's counted steps: launches per step (instrumented
        # pass) x the steps after its marker (x all its steps when no marker was seen); traffic per
        # launch = the op's bytes over those dispatches / its calls
        n_pmc = PMC_COUNTED_STEPS if (pmc and pmc.get("marked")) else PMC_CHILD_STEPS
        calls = {k: v["launches"] / args.steps * n_pmc for k, v in kern.items()}
        traffic_all, valu_all, traffic_src, vsrc = None, None, None, None
        if pmc:
            traffic_all = {k: round(v / calls[k]) for k, v in pmc["bytes_total"].items() if calls.get(k)}
            valu_all = {k: round(v / calls[k]) for k, v in pmc["winst_total"].items() if calls.get(k)}
            traffic_src = "rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE (this run, this workload)"
            vsrc = "rocprofv3 --pmc SQ_INSTS_VALU (this run, this workload)"
            # the stamped figures, for profiles/ (bench.py accepts them only for this build + workload)
            os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
            tag = "single" if (not args.batch_views and not args.deferred and len(cams) == 1) else "step"
            json.dump({"lib_sha256": sha, "workload": stamp, "bytes_per_launch": traffic_all,
                       "winst_per_launch": valu_all, "source": "bench.py --pmc-child passes"},
                      open(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}.json"), "w"), indent=1)
        else:  # committed figures, only if measured on this very library build AND this workload
            for name in ("pmc_step.json", "pmc_single.json"):
                try:
                    st = json.load(open(os.path.join(ROOT, "profiles", name)))
                except Exception:
                    continue
                if st.get("lib_sha256") == sha and st.get("workload") == stamp:
                    traffic_all, valu_all = st["bytes_per_launch"], st["winst_per_launch"]
                    traffic_src = vsrc = f"profiles/{name} (same build, same workload)"
                    break
            if traffic_all is None:
                traffic_src = "not measured: no PMC pass in this run and no stamped file for this build + workload"
        traffic = (traffic_all or {}).get(dom)
        valu = None  # secondary roofline: render kernels are VALU-issue bound, not HBM bound
        if valu_all:
            valu = {k: {"winst_per_launch": valu_all[k],
                        "achieved_Ginst_s": round(valu_all[k] / (kern[k]["avg_ms"] * 1e-3) / 1e9, 1),
                        "frac": round(valu_all[k] / (kern[k]["avg_ms"] * 1e-3) / 1e9 / VALU_PEAK_GINST, 3)}
                    for k in kern if k in valu_all}
            valu = {"peak_Ginst_s": VALU_PEAK_GINST, "source": vsrc, "kernels": valu}
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_source": traffic_src, "lib_sha256": sha[:16], "workload_stamp": stamp,
                    "algorithmic_bytes": ab[dom],
                    "kernels": {k: {"avg_ms": round(v["avg_ms"], 4), "launches": v["launches"],
                                    "GBps": round(ab[k] / (v["avg_ms"] * 1e-3) / 1e9, 1),
                                    "algorithmic_bytes": ab[k], "traffic": (traffic_all or {}).get(k),
                                    "traffic_over_algorithmic": round((traffic_all or {})[k] / ab[k], 3)
                                    if (traffic_all or {}).get(k) and ab.get(k) else None}
                                for k, v in kern.items()},
                    "valu": valu}

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(args, scene, cams[0], grads[0])

    aux = None
    if not args.no_aux and world == 1:
        aux = {"distCUDA2": aux_knn(params["means3D"].detach(), args), "fused_ssim": aux_ssim(H, W, dev, args),
               "separate_sh": aux_separate_sh(dgr, params, cams[0], grads[0], H * W),
               "sparse_adam": aux_sparse_adam(dgr, params, cams[0], grads[0], args),
               "train_iteration": aux_train_iteration(dgr, params, cams[0], H, W),
               "config3_scale": aux_config3_scale(dgr, dev)}

    coll = "RCCL (nccl)" if backend == "nccl" else f"{backend} (one-GPU rehearsal, not RCCL)"
    if mode == "strong":
        workload = (f"BASELINE config 4: {args.views_total} views per step of config 2 ({P} Gaussians, SH deg 3, "
                    f"{W}x{H}, fwd+bwd each), view v on rank v mod {world}"
                    + ((f", one {coll} grad all-reduce per step" + (f" overlapped with the backward "
                                                                     f"({args.allreduce_chunks} Gaussian ranges)"
                                                                     if overlap_ar else ""))
                       if world > 1 else ", grads accumulated on one GPU"))
    else:
        workload = (f"{args.views_per_rank} views per rank per step of config 2 ({P} Gaussians, SH deg 3, {W}x{H}, "
                    f"fwd+bwd each)" + (f", one {coll} grad all-reduce per step" if world > 1 else ""))
    res = {
        "metric": "rendered Mpix/s fwd+bwd, 1M Gaussians @1080p",
        "value": round(value, 2),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        # the median of the steps' stream times (events at the step boundaries, max over ranks)
        "ms_per_step": round(median_ms, 4),
        "ms_per_step_median": round(median_ms, 4),
        # the mean over the K timed steps: wall clock between the barriers / K (max over ranks)
        "ms_per_step_mean": round(elapsed / args.steps * 1e3, 4),
        "value_mean": round(value_mean, 2),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seed-0 Gaussian cloud, SURVEY.md §8d; ring camera views)",
        "config": {"workload": workload, "P": P, "width": W, "height": H, "views_per_step": views_step,
                   "views_per_rank": len(views), "num_rendered": L, "num_rendered_per_view": Ls,
                   "visible": P_vis, "antialiasing": args.antialiasing, "parallelism": f"views-dp{world}",
                   "backend": backend if world > 1 else None,
                   "forward_views_reruns": dgr._C.views_reruns,
                   "execution": ("one MultiViewRasterizer batch: the binning prefix of all views batched "
                                 "(one launch per stage, grid.y = view), then every view's render forward, every "
                                 "view's render backward, one preprocess backward for the batch"
                                 if args.batch_views else
                                 ("views alternating over 2 HIP streams" if args.overlap else "views on one stream")
                                 + ("; per view forward + render backward, one batched preprocess backward per "
                                    "step (deferred_backward)" if args.deferred
                                    else "; per view forward + full backward"))},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "aux": aux,
        "allreduce": allreduce,
    }
    if world == 1 and not args.pmc_child and not args.no_single_view and (args.batch_views or len(cams) > 1):
        res["config2_single_view"] = single_view_leg(args)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def aux_knn(points, args, reps=5):
    """simple_knn.distCUDA2 on the scene's P means: mean time per call
    (it synchronises once inside, to size its grid), plus the brute-force C oracle on a
    bounded sample as the CPU baseline."""
    from simple_knn._C import distCUDA2
    for _ in range(2):
        distCUDA2(points)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        distCUDA2(points)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    P = points.shape[0]
    out = {"points": P, "ms": round(ms, 3), "Mpoints_per_s": round(P / ms / 1e3, 1), "cpu_baseline": None}
    if not args.no_cpu_baseline:
        try:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle
            n = 20000
            threads = cpu_threads(args)
            sample = points[:n].cpu().numpy()
            t = time.perf_counter()
            oracle.knn_dist2(sample, nthreads=threads)
            dt = time.perf_counter() - t
            out["cpu_baseline"] = {"value": round(n / dt / 1e6, 4), "unit": "Mpoints/s", "cores": threads,
                                   "kind": "port", "sample": f"brute-force oracle on the first {n} points"}
        except Exception as e:
            out["cpu_baseline"] = {"value": None, "sample": f"failed: {e}"}
    return out


def aux_separate_sh(dgr, params, s, grad, npix, reps=10):
    """The headline step through the separate-DC surface train.py uses once SparseGaussianAdam is
    exported (rasterizer(dc=features_dc, shs=features_rest), gaussian_renderer/__init__.py:90-100):
    same view, same scene, SH coefficient 0 and the rest as two parameter tensors."""
    dc = params["shs"].detach()[:, :1].contiguous().requires_grad_(True)
    rest = params["shs"].detach()[:, 1:].contiguous().requires_grad_(True)
    gc, gi = grad
    rast = dgr.GaussianRasterizer(raster_settings=s)

    def step():
        for p in (*params.values(), dc, rest):
            p.grad = None  # as the headline step: no gradient accumulation kernels
        means2D = torch.zeros_like(params["means3D"], requires_grad=True)
        color, radii, inv = rast(means3D=params["means3D"], means2D=means2D, dc=dc, shs=rest,
                                 opacities=params["opacities"], scales=params["scales"], rotations=params["rotations"])
        torch.autograd.backward([color, inv], [gc, gi])
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    return {"ms_per_step": round(ms, 4), "Mpix_per_s": round(npix / ms / 1e3, 2)}


def aux_sparse_adam(dgr, params, s, grad, args, reps=10):
    """SparseGaussianAdam.step(radii > 0, P) (train.py:180-183) over the six parameter groups of a
    degree-3 model (xyz 3, f_dc 3, f_rest 45, opacity 1, scaling 3, rotation 4 floats per Gaussian)
    with the bench view's gradients and visibility.  HBM-bound: 28 B per visible element (p, g, m, v
    read; p, m, v written) + 1 B of flags per Gaussian and group.  CPU baseline: the numpy
    restatement (oracle/adam_oracle.py) on the same arrays."""
    gc, gi = grad
    P = params["means3D"].shape[0]
    rast = dgr.GaussianRasterizer(raster_settings=s)
    sh = params["shs"].detach()
    groups = {"xyz": params["means3D"].detach().clone(), "f_dc": sh[:, :1].contiguous(),
              "f_rest": sh[:, 1:].contiguous(), "opacity": params["opacities"].detach().clone(),
              "scaling": params["scales"].detach().clone(), "rotation": params["rotations"].detach().clone()}
    groups = {k: torch.nn.Parameter(v) for k, v in groups.items()}
    means2D = torch.zeros_like(groups["xyz"], requires_grad=True)
    color, radii, inv = rast(means3D=groups["xyz"], means2D=means2D, dc=groups["f_dc"], shs=groups["f_rest"],
                             opacities=groups["opacity"], scales=groups["scaling"], rotations=groups["rotation"])
    torch.autograd.backward([color, inv], [gc, gi])
    visible = radii > 0
    opt = dgr.SparseGaussianAdam([{"params": [p], "lr": 1e-4, "name": k} for k, p in groups.items()], lr=0.0,
                                 eps=1e-15)
    for _ in range(2):
        opt.step(visible, P)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        opt.step(visible, P)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    n_vis = int(visible.sum())
    per_g = sum(p.numel() for p in groups.values()) // P
    nbytes = 28 * n_vis * per_g + len(groups) * P
    out = {"gaussians": P, "visible": n_vis, "floats_per_gaussian": per_g, "ms_step": round(ms, 4),
           "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1), "hbm_frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3),
           "cpu_baseline": None}
    if not args.no_cpu_baseline:
        try:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import adam_oracle
            host = {k: (p.detach().cpu().numpy(), p.grad.cpu().numpy(), opt.state[p]["exp_avg"].cpu().numpy(),
                        opt.state[p]["exp_avg_sq"].cpu().numpy()) for k, p in groups.items()}
            vis = visible.cpu().numpy()
            t = time.perf_counter()
            for pa, ga, ma, va in host.values():
                adam_oracle.adam_update(pa, ga, ma, va, vis, 1e-4, 0.9, 0.999, 1e-15, P, pa.size // P)
            dt = time.perf_counter() - t
            out["cpu_baseline"] = {"value": round(dt * 1e3, 1), "unit": "ms per step", "cores": 1, "kind": "port",
                                   "sample": "one step of all six groups, numpy restatement (single thread)"}
        except Exception as e:
            out["cpu_baseline"] = {"value": None, "sample": f"failed: {e}"}
    return out


def aux_train_iteration(dgr, params, s, H, W, reps=10):
    """One train.py iteration with --optimizer_type sparse_adam at the bench scale (train.py:97-183):
    parameter activations (gaussian_model.py:111-135), render with dc= (gaussian_renderer/
    __init__.py:90-100), loss 0.8 L1 + 0.2 (1 - fused SSIM) (train.py:119-124), backward,
    SparseGaussianAdam.step(radii > 0, P).  Densification and logging are not part of it.  The
    target is a perturbed render of the same view (synthetic data)."""
    from fused_ssim import fused_ssim
    P = params["means3D"].shape[0]
    sh = params["shs"].detach()
    raw = {"xyz": params["means3D"].detach().clone(), "f_dc": sh[:, :1].contiguous(),
           "f_rest": sh[:, 1:].contiguous(), "opacity": torch.logit(params["opacities"].detach()),
           "scaling": torch.log(params["scales"].detach()), "rotation": params["rotations"].detach().clone()}
    raw = {k: torch.nn.Parameter(v) for k, v in raw.items()}
    lr = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20, "opacity": 2.5e-2, "scaling": 5e-3, "rotation": 1e-3}
    opt = dgr.SparseGaussianAdam([{"params": [p], "lr": lr[k], "name": k} for k, p in raw.items()], lr=0.0, eps=1e-15)
    rast = dgr.GaussianRasterizer(raster_settings=s)

    def render():
        means2D = torch.zeros_like(raw["xyz"], requires_grad=True)
        return rast(means3D=raw["xyz"], means2D=means2D, dc=raw["f_dc"], shs=raw["f_rest"],
                    opacities=torch.sigmoid(raw["opacity"]), scales=torch.exp(raw["scaling"]),
                    rotations=torch.nn.functional.normalize(raw["rotation"]))

    with torch.no_grad():
        gt = (render()[0] + 0.05 * torch.randn((3, H, W), device=raw["xyz"].device)).clamp(0, 1)

    def iteration():
        img, radii, _ = render()
        loss = 0.8 * (img - gt).abs().mean() + 0.2 * (1.0 - fused_ssim(img[None], gt[None]))
        loss.backward()
        opt.step(radii > 0, P)
        opt.zero_grad(set_to_none=True)
    for _ in range(3):
        iteration()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        iteration()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    return {"gaussians": P, "resolution": [W, H], "ms_per_iteration": round(ms, 4),
            "iterations_per_s": round(1e3 / ms, 1), "Mpix_per_s": round(H * W / ms / 1e3, 1)}


def aux_config3_scale(dgr, dev, P=6_000_000, W=1297, H=840, reps=5):
    """BASELINE config 3's scale (Mip-NeRF360 'garden': ~6M Gaussians, SH degree 3, images_4 at
    1297x840; the dataset is absent offline): one train.py iteration (aux_train_iteration) on a
    seed-0 synthetic cloud of 6M Gaussians seen by ring view 0 at that resolution, with its
    num_rendered and the peak device memory of the iterations (parameters, Adam state,
    rasterizer state buffers, SSIM).  tests/test_config3_scale.py checks this view against the
    oracle."""
    try:
        scene = synthetic.make_scene(P, seed=0)
        params = {k: v.to(dev) for k, v in scene.items()}
        del scene
        cam = synthetic.Camera(W, H, view=0)
        s = dgr.GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, bg=torch.zeros(3, device=dev),
            scale_modifier=1.0, viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev),
            sh_degree=3, campos=cam.camera_center.to(dev), prefiltered=False, debug=False, antialiasing=False)
        with torch.no_grad():
            e = torch.Tensor([])
            L = int(dgr._C.rasterize_gaussians(s.bg, params["means3D"], e, params["opacities"], params["scales"],
                                               params["rotations"], 1.0, e, s.viewmatrix, s.projmatrix, s.tanfovx,
                                               s.tanfovy, H, W, params["shs"], 3, s.campos, False, False, False)[0])
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(dev)
        out = aux_train_iteration(dgr, params, s, H, W, reps=reps)
        out.update({"num_rendered": L, "peak_device_GiB": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2),
                    "workload": f"BASELINE config 3 scale: {P} synthetic Gaussians (seed 0, SH deg 3), ring view 0 "
                                f"at {W}x{H} (garden images_4), one train.py sparse-Adam iteration"})
        del params
        torch.cuda.empty_cache()
        return out
    except Exception as e:  # the side leg must never take the headline result down
        return {"value": None, "error": f"{type(e).__name__}: {e}"}


def aux_ssim(H, W, dev, args, reps=20):
    """fused_ssim on one (1, 3, H, W) image pair: forward (map + partials) and
    backward, timed with events on the current stream; HBM-bound, so priced in algorithmic bytes
    (forward: 2 images in, map + 3 partial planes out; backward: 2 images + dL/dmap + 3 partial
    planes in, dL/dimg1 out: 13 planes of 4 B per pixel and channel)."""
    import fused_ssim
    lib = fused_ssim._lib
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.rand((1, 3, H, W), device=dev, generator=g)
    b = (a + 0.1 * torch.randn(a.shape, device=dev, generator=g)).clamp(0, 1)
    up = torch.randn(a.shape, device=dev, generator=g)
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m, dA, dB, dC, grad = (torch.empty_like(a) for _ in range(5))
    stream = torch.cuda.current_stream(dev).cuda_stream
    n = a.numel() // (H * W)

    # the C ABI directly on preallocated planes, so the events see kernel time, not Python
    def fwd():
        return lib.gsr_ssim_forward(n, H, W, C1, C2, a.data_ptr(), b.data_ptr(), m.data_ptr(), dA.data_ptr(),
                             dB.data_ptr(), dC.data_ptr(), stream)

    def bwd():
        return lib.gsr_ssim_backward(n, H, W, C1, C2, a.data_ptr(), b.data_ptr(), up.data_ptr(), dA.data_ptr(),
                              dB.data_ptr(), dC.data_ptr(), grad.data_ptr(), stream)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
    for _ in range(3):
        if fwd() or bwd():
            raise RuntimeError(lib.gsr_last_error().decode())
    ms_f, ms_b = timed(fwd), timed(bwd)
    ms = ms_f + ms_b
    nbytes = 13 * 4 * a.numel()
    out = {"shape": list(a.shape), "ms_fwd_bwd": round(ms, 4), "ms_fwd": round(ms_f, 4), "ms_bwd": round(ms_b, 4),
           "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
           "hbm_frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3), "cpu_baseline": None}
    if not args.no_cpu_baseline:
        try:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import ssim_oracle
            threads = cpu_threads(args)
            torch.set_num_threads(threads)
            ac, bc, uc = a.cpu(), b.cpu(), up.cpu()
            t = time.perf_counter()
            ssim_oracle.ssim_and_grad(ac, bc, dtype=torch.float32, upstream=uc)
            dt = time.perf_counter() - t
            out["cpu_baseline"] = {"value": round(dt * 1e3, 1), "unit": "ms (fwd+bwd)", "cores": threads,
                                   "kind": "port", "sample": "the same image pair, float32 torch-CPU restatement"}
        except Exception as e:
            out["cpu_baseline"] = {"value": None, "sample": f"failed: {e}"}
    return out


def host_cpus():
    """The host cores this process may use, and how that was found (the CPU baseline
    runs on all host cores of the GPU box, with the count and CPU model reported).  The affinity
    mask bounds it; a cgroup CPU quota (cpu.max: quota / period) bounds it further -- on a shared
    box the mask may list the whole machine while the quota grants a share of it, and threads
    beyond the quota only time-slice."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    n = min(aff, quota) if quota else aff
    return n, {"nproc_affinity": aff, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(), "cpu_model": model}


def cpu_threads(args):
    """--cpu-threads, or every usable host core (host_cpus)."""
    return args.cpu_threads or host_cpus()[0]


def cpu_baseline(args, scene, s, grad):
    """The CPU restatement behind the product's own C ABI (oracle/libgsr_cpu.so: gsr_forward with
    resize callbacks, then gsr_backward on the state buffers -- the host calling sequence of the
    HIP library; the oracle's OpenMP code underneath) on the bench's first view: one
    forward+backward per run, --cpu-reps runs, the median reported."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cpu_abi
        threads = cpu_threads(args)
        gc, gi = grad
        gc, gi = gc.cpu(), gi.cpu()
        cpu = cpu_abi.CpuRasterizer(nthreads=threads)
        times = []
        for _ in range(max(1, args.cpu_reps)):
            t = time.perf_counter()
            cpu.forward_backward(scene["means3D"], scene["opacities"], s.bg.cpu(), s.viewmatrix.cpu(),
                                 s.projmatrix.cpu(), s.campos.cpu(), s.tanfovx, s.tanfovy, s.image_height,
                                 s.image_width, gc, gi, shs=scene["shs"], sh_degree=3, scales=scene["scales"],
                                 rotations=scene["rotations"], antialiasing=args.antialiasing)
            times.append(time.perf_counter() - t)
        dt = statistics.median(times)
        return {"value": round(s.image_height * s.image_width / dt / 1e6, 3), "unit": "Mpix/s", "cores": threads,
                "kind": "port", **host_cpus()[1], "seconds": round(dt, 3), "runs_s": [round(x, 3) for x in times],
                "sample": f"one full fwd+bwd of one bench view ({args.P} Gaussians, {s.image_width}x"
                          f"{s.image_height}) by the C/OpenMP restatement through gsr_forward/gsr_backward "
                          f"(oracle/libgsr_cpu.so), median of {len(times)} runs"}
    except Exception as e:  # the baseline must never take the GPU result down
        return {"value": None, "unit": "Mpix/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}


if __name__ == "__main__":
    main()
