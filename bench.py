#!/usr/bin/env python3
"""bench.py -- primary rays/s of the MI355X BIH ray tracer.

Workload (BASELINE.json configs[2]): 1,000,000-triangle
random soup (splitmix64 seed 1), 1920x1080, 4 jittered primary rays per
pixel, reference camera, cuRAND-XORWOW seed 1984.  One step = one frame
pass.  With N GPUs (the north star's decomposition) every frame is
cut into interleaved 4-row bands dealt round-robin to the ranks; each rank
renders its bands with global pixel indices (so the frame is byte-identical
to a one-GPU render) and ONE RCCL gather per frame brings the bands to rank 0,
which lays them out in frame order (bihrt.tiling.BandGather) -- strong
scaling, value = rays per frame x steps / max-over-ranks time.  A side leg
renders whole frames per rank (weak scaling, no collective).  At N = 1 the
"band_share" leg times each rank's share of an 8-GPU split on this GPU.  The BIH is built once before the timed
region (its device time is reported as build_ms; the reference rebuilds it
every frame, Renderer.cpp:415-503 -- the "with_rebuild" leg times that).

Single process:   python bench.py
Multi-GPU:        python bench.py --gpus N        (starts the N ranks itself), or
                  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
Rank 0 prints one JSON line.  Every per-call device buffer is sized before the
timed region (bih_reserve) and the warm-up issues every call size the timed
loop issues; the line reports the allocations the headline made
(device_allocs_in_headline, expected 0).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))

METRIC = "primary rays/sec at 1920×1080, 1M-tri scene; achieved HBM GB/s vs peak"   # BASELINE.json
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
NODE_B, LEAF_B, TRI_B = 16, 8, 40   # SURVEY.md 8d algorithmic bytes
FB_B, RNG_B = 4, 48


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (one rank each).  Without a launcher (no WORLD_SIZE in the "
                         "environment) N > 1 starts the N ranks itself (torch.distributed.run, before this "
                         "process touches the GPU) and relays rank 0's line; under a launcher it must equal "
                         "WORLD_SIZE.  Default: WORLD_SIZE, else 1")
    # the defaults are the driver's command (--gpus 1 --steps 20 --warmup 5);
    # --steps 500 --warmup 50 gives the steady state of a long frame loop
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--band", type=int, default=4,
                    help="rows per band of the N > 1 row split (a multiple of the 4-row packet tile; 4 balances the ranks best: 1080 rows = 270 bands)")
    ap.add_argument("--in-flight", type=int, default=3,
                    help="frames in flight: consecutive frames on this many streams, so the "
                         "next frame fills the tail of the one before (1 = one frame at a time)")
    ap.add_argument("--mode", choices=["weak", "strong"], default="strong",
                    help="N > 1: row bands of every frame + RCCL gather to rank 0 (strong, the "
                         "north star's decomposition) or whole frames per rank (weak) as the "
                         "headline; the other runs as a side leg")
    ap.add_argument("--gather-packed", type=int, default=1,
                    help="N > 1 strong: send the bands as 4-bit hit counts (8x fewer bytes over "
                         "xGMI; rank 0 expands them to the same RGBA words); needs spp 4")
    ap.add_argument("--group", type=int, default=16,
                    help="consecutive frames per render call (bih_render_device_frames: one launch "
                         "of each kernel for the group; each frame is still the reference's frame "
                         "at its index); the with_rebuild and moving_camera legs use 1")
    ap.add_argument("--share-world", type=int, default=8,
                    help="N=1: time each of the bands one of this many GPUs would render (the "
                         "strong decomposition's per-rank work) -> projected per-GPU efficiency")
    ap.add_argument("--share-reps", type=int, default=3,
                    help="band_share legs: windows timed per share (and for the full frame); the median is kept")
    ap.add_argument("--traverse", choices=["anyhit", "reference"], default="anyhit")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on rank 0 (N=1)")
    ap.add_argument("--cpu-row-step", type=int, default=4,
                    help="rows of frame 0 timed on all host threads (every k-th row)")
    ap.add_argument("--cpu-serial-row-step", type=int, default=16,
                    help="rows timed single-threaded (reference walk)")
    ap.add_argument("--cpu-debug-row-step", type=int, default=1080,
                    help="rows timed single-threaded with the reference's host debug rules "
                         "(CPUTraverseTree visits ~40k nodes per ray at 1M triangles: one row)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--parity-row-step", type=int, default=16,
                    help="rows of frames 7 and 15 of the timed call shape checked against the oracle")
    ap.add_argument("--traffic", type=int, default=1,
                    help="N=1: measure HBM traffic per launch with rocprofv3 PMC passes "
                         "(child processes, before this process touches the GPU)")
    ap.add_argument("--kernel-samples", type=int, default=20,
                    help="isolated launches timed with the library's kernel events (roofline launch_ms)")
    ap.add_argument("--step-events", type=int, default=0,
                    help="record torch events around every timed render (kernel_ms per leg)")
    ap.add_argument("--whitted-frames", type=int, default=3,
                    help="N=1: frames of config C4 (8-bounce Whitted, 3840x2160, same soup) to time; 0 = skip")
    ap.add_argument("--c5", type=int, default=1,
                    help="config C5 leg: 10M-triangle soup at 3840x2160 with the headline's call shape "
                         "and decomposition (row bands + gather at N > 1); 0 = skip")
    ap.add_argument("--c5-tris", type=int, default=10_000_000)
    ap.add_argument("--no-reference-leg", action="store_true")
    ap.add_argument("--dynamic-leg", type=int, default=1,
                    help="time the per-frame rebuild with geometry that changes every step (two soups)")
    ap.add_argument("--host-loop", type=int, default=1,
                    help="N=1: time INTEGRATION.md's host loop (bih_rebuild + bih_render into a host "
                         "framebuffer), pageable and page-locked")
    ap.add_argument("--no-rebuild-leg", action="store_true",
                    help="skip the leg that rebuilds the BIH every frame (as the reference does)")
    ap.add_argument("--headline-only", action="store_true",
                    help="time the headline leg only (no side legs), e.g. under rocprofv3 so that "
                         "its kernel average is the headline's launches")
    ap.add_argument("--stub", action="store_true",
                    help="launcher test: ranks join a gloo group, check the world size and rank 0 prints "
                         "a JSON line; no GPU work")
    return ap.parse_args()


def visible_gpu_count():
    """GPUs this process may use, counted WITHOUT any HIP call (the launcher
    must not initialise the runtime before it starts the ranks): the KFD
    topology nodes that have SIMDs (/sys/class/kfd/kfd/topology/nodes/*/
    properties, simd_count > 0; CPU nodes have none), else amdsmi's processor
    handles, limited by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES.  None when neither source is readable.
    BIH_KFD_TOPOLOGY overrides the topology directory (tests)."""
    root = os.environ.get("BIH_KFD_TOPOLOGY", "/sys/class/kfd/kfd/topology/nodes")
    n = None
    try:
        names = os.listdir(root)
    except OSError:
        names = None
    if names is not None:
        n = 0
        for d in names:
            try:
                with open(os.path.join(root, d, "properties")) as f:
                    kv = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if int(kv.get("simd_count", "0")) > 0:
                n += 1
    if n is None:
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            try:
                n = len(amdsmi.amdsmi_get_processor_handles())
            finally:
                amdsmi.amdsmi_shut_down()
        except Exception:
            return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher: start the N ranks as child
    processes (torch.distributed.run on 127.0.0.1, one process per GPU) before
    this process makes any GPU call; rank 0's JSON line goes to our stdout.
    Exit 2 if the devices cannot be counted without HIP or fewer than N are
    visible (N ranks sharing one GPU over gloo, BIH_BENCH_SHARE_GPU=1, need
    one); otherwise the child's exit status."""
    import socket
    import subprocess
    n = visible_gpu_count()
    need = 1 if os.environ.get("BIH_BENCH_SHARE_GPU") == "1" else args.gpus
    if n is None:
        print("bench.py: cannot count the GPUs without HIP (no KFD topology, no amdsmi)", file=sys.stderr)
        return 2
    if n < need:
        print(f"bench.py: --gpus {args.gpus} but {n} devices are visible", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run(cmd, env=env)
    if p.returncode != 0:
        print(f"bench.py: {args.gpus}-rank run failed (exit {p.returncode})", file=sys.stderr)
    return p.returncode


def stub_worker(args, rank, world):
    """The launcher's test worker: the group forms over gloo with the world
    size asked for; rank 0 prints one JSON line."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    assert dist.get_world_size() == args.gpus == world, (dist.get_world_size(), args.gpus, world)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"stub": True, "world_size": dist.get_world_size(), "backend": dist.get_backend(),
                          "rank_sum": t.item()}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def call_sizes(n, g):
    """Frames per call when n frames are issued in calls of g (the last one takes the rest)."""
    return [min(g, n - k) for k in range(0, n, g)]


class Workload:
    """One scene and image on this rank: the tree, the renderer, one output
    buffer per stream in flight, and (strong decomposition at N > 1) one band
    gather per stream and call size.  Every per-call device buffer is sized
    before any timing (bih_reserve, gathers pre-built for every call size)."""

    def __init__(self, C, tris, W, H, cam=None, shapes=(1,)):
        self.C, self.W, self.H = C, W, H
        torch, bihrt, a = C.torch, C.bihrt, C.args
        self.tris = tris
        self.d_tris = torch.from_numpy(tris).to(f"cuda:{C.local}")
        self.arrays = bihrt.GPUArrayManager.from_device(self.d_tris.data_ptr(), tris.shape[0], device=C.local,
                                                        stream=C.sptr)
        # the bench never writes its soup after the build: a rebuild (the
        # with_rebuild leg) need not read the new tree's header back
        # (BIH_PARAM_STATIC_SOUP; the same tree bit for bit)
        self.arrays.set_param(bihrt.PARAM_STATIC_SOUP, 1)
        self.info = self.arrays.info()
        self.cam = cam if cam is not None else bihrt.camera_reference(W, H)
        self.r = bihrt.Renderer(self.arrays, W, H, spp=a.spp, seed=1984, camera=self.cam)
        self.mrows = C.tiling.max_rows(H, a.band, C.world)
        G = C.G
        self.outs = [torch.zeros(G * H * W, dtype=torch.int32, device="cuda") for _ in range(C.F)]
        self.gathers, self.frame_img = {}, None
        if C.world > 1:
            packed = bool(a.gather_packed) and a.spp == 4 and W % 8 == 0
            for j in range(C.F):
                for m in sorted(set(shapes)):
                    self.gathers[(j, m)] = C.tiling.BandGather(C.dist, H, W, a.band, C.rank, C.world,
                                                               torch.device("cuda", C.local), frames=m,
                                                               packed=packed)
            self.frame_img = [torch.zeros(G * H * W, dtype=torch.int32, device="cuda") if C.rank == 0 else None
                              for _ in range(C.F)]
        # every per-call buffer of both decompositions' call shapes, up front
        rows_all = C.tiling.band_rows(H, a.band, 0, 1)
        self.arrays.reserve(W, H, a.spp, rows_all, G)
        if C.world > 1:
            self.arrays.reserve(W, H, a.spp, C.tiling.band_rows(H, a.band, C.rank, C.world), G)
        torch.cuda.synchronize()

    def plan(self, mode, g):
        """(rows of this rank, frame of step k from `base`, frames per step job-wide)"""
        C, a = self.C, self.C.args
        if mode == "weak" or C.world == 1:
            return (C.tiling.band_rows(self.H, a.band, 0, 1),
                    (lambda base, k: C.tiling.frame_of_step(base, k, C.rank, C.world, g)), C.world)
        return C.tiling.band_rows(self.H, a.band, C.rank, C.world), (lambda base, k: base + k), 1

    def step(self, mode, rows, c, frame, traverse, ev=None, rebuild=False, nf=None, m=1, first=0):
        """One render call (call index c): frames frame .. frame+m-1, on
        stream first + c % nf.  `rebuild`: bih_rebuild before the render; a
        callable is called with c first (on the tree's stream: the
        dynamic_rebuild leg writes the call's soup into the tree's input)."""
        C = self.C
        nf = nf or C.F
        j = first + c % nf
        s = C.streams[j]
        o = self.outs[j].data_ptr()
        strong = mode == "strong" and C.world > 1
        # frames of a call packed at the rank's padded rows (the gather sends them as one block)
        stride = (self.mrows if strong else self.H) * self.W
        r = self.r

        def render():
            if m == 1:
                r.render_device(o, frame, rows=rows, traverse=traverse, stream=s.cuda_stream)
            elif traverse == C.bihrt.TRAVERSE_ANYHIT:
                r.render_device_frames(o, frame, m, stride, rows=rows, stream=s.cuda_stream)
            else:
                for f in range(m):
                    r.render_device(o + 4 * f * stride, frame + f, rows=rows, traverse=traverse,
                                    stream=s.cuda_stream)

        if ev is None and not rebuild and not strong:
            render()     # the render alone: no torch work on the stream, no stream context
            return
        if callable(rebuild):
            rebuild(c)
        with C.torch.cuda.stream(s):
            if rebuild:
                self.arrays.rebuild()
            if ev is not None:
                ev[0].record(s)
            render()
            if ev is not None:
                ev[1].record(s)
            if strong:
                # call c's gather runs on stream j while call c+1 renders on j+1
                self.gathers[(j, m)](self.outs[j], self.frame_img[j])

    def timed(self, mode, traverse, base, rebuild=False, nf=None, g=None, rows=None, steps=None, first=0):
        """Times exactly `steps` frames per rank (args.steps), in calls of g
        frames (the last call takes the rest).  Untimed first: args.warmup
        frames in calls of g, then one call of every timed call size the
        warm-up did not issue.  Frames run on without a gap from the warm-up
        into the timed calls.  Returns (max-over-ranks seconds, kernel ms per
        frame or None, frames per step job-wide)."""
        C, a = self.C, self.C.args
        g = g or C.G
        steps = steps or a.steps
        rows_p, frame_of, fps = self.plan(mode, g)
        rows = rows or rows_p
        calls = call_sizes(steps, g)
        warm = call_sizes(a.warmup, g)
        warm += [m for m in sorted(set(calls)) if m not in warm]
        # every stream in play takes a call before the timed ones: a stream's
        # first kernel creates its hardware queue (~7 ms)
        while len(warm) < (nf or C.F):
            warm.append(calls[0])
        k = c = 0
        for m in warm:
            self.step(mode, rows, c, frame_of(base, k), traverse, rebuild=rebuild, nf=nf, m=m, first=first)
            k, c = k + m, c + 1
        C.sync_all()
        allocs0 = self.arrays.info().device_allocs
        # per-call torch events only when asked (--step-events): recording them
        # costs host time per call, which the row-band shares feel
        evs = [(C.torch.cuda.Event(enable_timing=True), C.torch.cuda.Event(enable_timing=True))
               for _ in calls] if a.step_events else []
        strong = mode == "strong" and C.world > 1
        self.timed_calls = []
        t0 = time.perf_counter()
        for i, m in enumerate(calls):
            self.step(mode, rows, c, frame_of(base, k), traverse, evs[i] if evs else None, rebuild=rebuild,
                      nf=nf, m=m, first=first)
            # (bookkeeping after the call is issued: which buffer holds which frames)
            self.timed_calls.append({"j": first + c % (nf or C.F), "f0": frame_of(base, k), "m": m, "c": c,
                                     "rows": rows, "strong": strong})
            k, c = k + m, c + 1
        C.sync_all()
        el = C.max_over_ranks(time.perf_counter() - t0)
        # device allocations inside the timed calls (bih_reserve sized every
        # per-call buffer; the warm-up built the camera's structures): 0
        self.timed_allocs = self.arrays.info().device_allocs - allocs0
        kms = [x.elapsed_time(y) / m for (x, y), m in zip(evs, calls)] if evs else []
        return el, (sum(kms) / len(kms) if kms else None), fps

    def capture(self, i, qs):
        """Host copies of frames qs (indices inside the call; -1 = its last) of
        timed call i (-1 = the last) as the timed loop left them in their
        output buffer, untimed, after the loop: [(frame, global rows, u32
        (rows, W))].  Strong decomposition: rank 0's gathered full frames
        (other ranks hold only their bands: nothing)."""
        import numpy as np
        C, H, W = self.C, self.H, self.W
        tc = self.timed_calls[i]
        res = []
        for q in sorted({q % tc["m"] for q in qs}):
            if tc["strong"]:
                if C.rank != 0:
                    continue
                t = self.frame_img[tc["j"]][q * H * W:(q + 1) * H * W]
                ys = np.arange(H)
            else:
                nr = tc["rows"].nrows
                t = self.outs[tc["j"]][q * H * W:q * H * W + nr * W]
                ys = rows_global(tc["rows"], H)
            res.append((tc["f0"] + q, ys, t.cpu().numpy().view(np.uint32).reshape(ys.size, W).copy()))
        return res

    def close(self):
        self.arrays.close()
        del self.d_tris


class Ctx:
    pass


def rows_global(rows, H):
    """Global row of each local row of a bih_rows tiling (include/bih.h)."""
    import numpy as np
    r = np.arange(rows.nrows)
    return rows.row0 + (r // rows.band_h) * rows.band_h * rows.band_step + r % rows.band_h


class TimedOutputs:
    """What the timed calls wrote, checked: frames the
    timer timed, captured right after each leg, go to the oracle on rank 0
    at N = 1 (`pending`, checked in cpu_baseline: the only place bench.py may
    run the oracle) or are compared on the GPU side with another render of the
    same frames (`checks`: the 8 band shares reassembled against the full
    frame; at N > 1 rank 0's gathered frames against its own one-GPU render)."""

    def __init__(self):
        self.pending, self.checks = [], []

    def oracle(self, leg, caps, row_step, cam=None, soup="A", W=None, H=None):
        for f, ys, img in caps:
            pick = np.arange(0, ys.size, row_step)
            self.pending.append({"leg": leg, "frame": int(f), "ys": ys[pick], "img": img[pick], "cam": cam,
                                 "soup": soup, "W": W, "H": H, "row_step": row_step})

    def gpu(self, leg, frame, equal, what):
        self.checks.append({"leg": leg, "frame": int(frame), "equal": bool(equal), "against": what})

    def summary(self):
        allc = self.checks
        return {"all_equal": bool(allc) and all(c["equal"] for c in allc), "checks": allc,
                "unchecked": [{"leg": p["leg"], "frame": p["frame"]} for p in self.pending],
                "oracle_seconds": getattr(self, "oracle_seconds", None)}



def main():
    args = parse()
    if args.gpus and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if args.gpus is None:
        args.gpus = world
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.stub:
        stub_worker(args, rank, world)
        return
    import torch

    # a rank of an N > 1 run needs its own device (counted, not initialised)
    if world > 1 and os.environ.get("BIH_BENCH_SHARE_GPU") != "1" and torch.cuda.device_count() <= local:
        print(f"bench.py: rank {rank}: LOCAL_RANK {local} but {torch.cuda.device_count()} devices are visible",
              file=sys.stderr)
        sys.exit(3)

    # PMC traffic passes run as child processes before this one initialises
    # the GPU (rocprofv3 must start the program itself)
    traffic = None
    if world == 1 and args.traffic:
        traffic = measure_traffic(args)

    # rehearsal of the N > 1 path on a one-GPU box: all ranks on cuda:0 over gloo
    shared = os.environ.get("BIH_BENCH_SHARE_GPU") == "1"
    if shared:
        local = 0
    torch.cuda.set_device(local)
    dist = None
    backend = None
    if world > 1:
        import torch.distributed as dist
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        backend = dist.get_backend()
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    import bihrt
    from bihrt import tiling

    C = Ctx()
    C.args, C.rank, C.world, C.local, C.dist, C.torch, C.bihrt, C.tiling = (args, rank, world, local, dist,
                                                                             torch, bihrt, tiling)
    W, H, SPP = args.width, args.height, args.spp
    # explicit streams: the build and untimed work on streams[0]; call k of a
    # timed leg on streams[k % in_flight] with its own output buffers, so that
    # consecutive calls overlap (libbih_amd orders what they share)
    C.F = F = max(1, args.in_flight)
    C.G = G = max(1, args.group)
    C.streams = streams = [torch.cuda.Stream() for _ in range(F)]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    C.sptr = sptr = stream.cuda_stream

    def sync_all():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(el):
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        if dist is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    C.sync_all, C.max_over_ranks = sync_all, max_over_ranks
    # every call size a leg issues (gathers are built for each up front)
    shapes = set(call_sizes(args.steps, G)) | set(call_sizes(args.warmup, G)) | {1, G}

    # scene: generated on the host (deterministic), resident in HBM before timing
    tris = bihrt.scenes.soup(args.tris, seed=1)
    wl = Workload(C, tris, W, H, shapes=shapes)
    r, arrays, info, cam = wl.r, wl.arrays, wl.info, wl.cam
    out = wl.outs[0]
    trav = bihrt.TRAVERSE_ANYHIT if args.traverse == "anyhit" else bihrt.TRAVERSE_REFERENCE

    mode = args.mode if world > 1 else "weak"
    rows, frame_of, _ = wl.plan(mode, G)
    rays_per_frame = W * H * SPP
    elapsed, kernel_ms, fps = wl.timed(mode, trav, 0)
    value = fps * rays_per_frame * args.steps / elapsed
    allocs_headline = wl.timed_allocs
    # the frames the headline's timed calls wrote: the first and last frame of
    # each call (N = 1: against the oracle -- the last frame of the first,
    # G-frame call on every row, the others on every 16th row; N > 1 strong:
    # rank 0's gathered frames against its own one-GPU render, below)
    tout = TimedOutputs()
    head_caps = []
    for i in range(len(wl.timed_calls)):
        head_caps += [(i, cap) for cap in wl.capture(i, [0, -1])]
    if world == 1:
        for i, cap in head_caps:
            full = i == 0 and cap[0] == wl.timed_calls[0]["f0"] + wl.timed_calls[0]["m"] - 1
            tout.oracle("headline", [cap], 1 if full else args.parity_row_step)

    # The roofline's kernel time, from the timed window's own shape: the same
    # calls on the same streams again (frames further on), with the library's
    # HIP events around each render kernel (bih_set_timing; they cost host
    # time per call, so not in the headline itself).  The union of the
    # launches' kernel intervals over the window's frames is the kernel time
    # per frame; overlapping launches (the alternating-stream grid) are not
    # double counted.
    window = None
    if trav == bihrt.TRAVERSE_ANYHIT:
        r.set_timing(True)
        elw, _, _ = wl.timed(mode, trav, 10000)
        r.set_timing(False)
        n_calls = len(wl.timed_calls)
        try:
            hist = r.render_history(min(n_calls, 3)) if n_calls <= 3 else None
        except bihrt.BihError:
            hist = None
        if hist is not None:
            iv = sorted((float(a), float(b)) for a, b, _ in hist)
            union, cur = 0.0, None
            for a0, b0 in iv:
                if cur is None or a0 > cur[1]:
                    if cur is not None:
                        union += cur[1] - cur[0]
                    cur = [a0, b0]
                else:
                    cur[1] = max(cur[1], b0)
            union += cur[1] - cur[0]
            frames_w = sum(tc["m"] for tc in wl.timed_calls)
            window = {"calls": [tc["m"] for tc in wl.timed_calls], "frames": frames_w,
                      "kernel_intervals_ms": [[round(a, 5), round(b, 5)] for a, b in iv],
                      "kernel_union_ms": union, "kernel_ms_per_frame": union / frames_w,
                      "kernel_sum_ms": sum(b - a for a, b in iv),
                      "ms_per_step": 1e3 * elw / args.steps,
                      "source": "HIP events around each k_render_bins launch of a replica of the timed window "
                                "(same calls, streams and shapes; bih_render_history), union of the intervals"}

    if args.headline_only:
        args.no_reference_leg = args.no_rebuild_leg = True
    ref_leg = None
    if not args.no_reference_leg:
        other = bihrt.TRAVERSE_REFERENCE if trav == bihrt.TRAVERSE_ANYHIT else bihrt.TRAVERSE_ANYHIT
        el2, kms2, fps2 = wl.timed(mode, other, 1000)
        ref_leg = {"traverse": "reference" if other == bihrt.TRAVERSE_REFERENCE else "anyhit",
                   "value": fps2 * rays_per_frame * args.steps / el2,
                   "ms_per_step": 1e3 * el2 / args.steps,
                   "kernel_ms": kms2}

    # one frame at a time (frame latency): informational when frames overlap
    serial_leg = None
    if F > 1 and not args.headline_only:
        el5, kms5, fps5 = wl.timed(mode, trav, 4000, nf=1, g=1)
        if world == 1:
            tout.oracle("one_in_flight", wl.capture(-1, [-1]), args.parity_row_step)
        serial_leg = {"value": fps5 * rays_per_frame * args.steps / el5, "unit": "rays/s",
                      "ms_per_step": 1e3 * el5 / args.steps, "kernel_ms": kms5,
                      "note": "in_flight 1, one frame per call: each frame starts after the previous one ends"}

    # N = 1: the strong decomposition's per-rank work at --share-world GPUs.
    # Rank q of Q renders the interleaved bands band_rows(H, B, q, Q) of every
    # frame; each share is timed alone here, with the same call shape and
    # pipelining as the full frame it is compared with (measured again right
    # before the shares, so both see the same box state).  Projected per-GPU
    # efficiency = full-frame ms / (Q x slowest share ms): what the row tiling
    # costs per GPU before the gather.
    share_leg = None
    Q = args.share_world
    if world == 1 and Q > 1 and not args.headline_only:
        for q in range(Q):
            arrays.reserve(W, H, SPP, tiling.band_rows(H, args.band, q, Q), G)
        # (each window timed --share-reps times, the median kept: a share's
        # window is ~0.17 ms, where one slow window would decide the ratio)
        full_ms = median_ms(wl, "weak", trav, 7000, args.share_reps, args.steps)
        full_cap = wl.capture(-1, [-1])
        tout.oracle("band_share_full_frame", full_cap, args.parity_row_step)
        shares, parts = [], []
        for q in range(Q):
            # (the same frames as the full frame: each share's last frame
            # reassembles into the full frame's last frame)
            shares.append(median_ms(wl, "weak", trav, 7000, args.share_reps, args.steps,
                                    rows=tiling.band_rows(H, args.band, q, Q)))
            parts.append(wl.capture(-1, [-1])[0])
        check_shares(tout, "band_share", full_cap[0], parts, H, args.band, Q, tiling)
        share_leg = {"world": Q, "band": args.band, "share_ms_per_step": shares,
                     "full_frame_ms_per_step": full_ms,
                     "projected_efficiency": full_ms / (Q * max(shares)),
                     "note": f"each of the {Q} ranks' interleaved {args.band}-row bands rendered alone "
                             f"on this GPU, {G} frames per call and {F} calls in flight as the full frame "
                             f"timed beside it, each window timed {args.share_reps} times (median); "
                             f"efficiency = full ms / ({Q} x slowest share ms); excludes "
                             f"the gather to rank 0 ({H * W * 4 * (Q - 1) // Q / 1e6:.1f} MB over xGMI per "
                             "frame, 8x less packed)"}

    # config C2 (BASELINE.json configs[1]): a ~70k-triangle mesh at 1920x1080.
    # The Stanford bunny is not available offline; the stand-in is the
    # closed 69,432-triangle torus (bihrt.scenes.torus), same camera, same
    # frame sequence and calls as the headline
    c2_leg = None
    if world == 1 and not args.headline_only:
        w2 = Workload(C, bihrt.scenes.torus(), W, H, cam=cam, shapes=shapes)
        el2, _, _ = w2.timed("weak", bihrt.TRAVERSE_ANYHIT, 0)
        tout.oracle("c2_torus", w2.capture(-1, [-1]), args.parity_row_step, soup="torus")
        c2_leg = {"config": "C2 stand-in: 69,432-triangle closed torus (bunny unavailable offline), 1920x1080, "
                            "4 spp, any-hit, call shape as the headline",
                  "tris": int(w2.tris.shape[0]), "value": rays_per_frame * args.steps / el2, "unit": "rays/s",
                  "ms_per_step": 1e3 * el2 / args.steps,
                  "note": "parity: tests/test_gpu_parity.py::test_c2_torus_1080p (oracle rows, exact walk)"}
        w2.close()
        del w2

    # config C5 (BASELINE.json configs[4]): the 10M-triangle soup at
    # 3840x2160 with the headline's call shape; at N > 1 the headline's
    # decomposition (row bands of every frame + one gather to rank 0 per call)
    c5_leg = None
    if args.c5 and not args.headline_only:
        t5 = bihrt.scenes.soup(args.c5_tris, seed=1)
        W5, H5 = 3840, 2160
        w5 = Workload(C, t5, W5, H5, shapes=shapes)
        el5, _, fps5 = w5.timed(mode, bihrt.TRAVERSE_ANYHIT, 0)
        # N = 1: each of the --share-world ranks' interleaved bands of C5's
        # frame alone (C5 is "row-tiled across 8 x MI355X"; north_star), as
        # band_share does for the headline: projected per-GPU efficiency
        share5 = None
        if world == 1 and Q > 1:
            for q in range(Q):
                w5.arrays.reserve(W5, H5, SPP, tiling.band_rows(H5, args.band, q, Q), G)
            full5 = median_ms(w5, "weak", bihrt.TRAVERSE_ANYHIT, 7000, args.share_reps, args.steps)
            full5_cap = w5.capture(-1, [-1])
            sh5, parts5 = [], []
            for q in range(Q):
                sh5.append(median_ms(w5, "weak", bihrt.TRAVERSE_ANYHIT, 7000, args.share_reps, args.steps,
                                     rows=tiling.band_rows(H5, args.band, q, Q)))
                parts5.append(w5.capture(-1, [-1])[0])
            check_shares(tout, "c5_band_share", full5_cap[0], parts5, H5, args.band, Q, tiling)
            share5 = {"world": Q, "band": args.band, "share_ms_per_step": sh5, "full_frame_ms_per_step": full5,
                      "projected_efficiency": full5 / (Q * max(sh5)),
                      "note": f"each of the {Q} ranks' interleaved {args.band}-row bands of the 3840x2160 frame "
                              f"rendered alone on this GPU, {G} frames per call, as the full frame timed beside "
                              "it; excludes the gather"}
        w5.arrays.rebuild()
        torch.cuda.synchronize()
        b5 = w5.arrays.info().build_ms
        st5 = w5.arrays.bins_stats()
        c5_leg = {"config": f"C5: {args.c5_tris}-triangle soup (splitmix64 seed 1), {W5}x{H5}, {SPP} spp, "
                            "any-hit, call shape as the headline",
                  "tris": int(t5.shape[0]), "value": fps5 * W5 * H5 * SPP * args.steps / el5, "unit": "rays/s",
                  "ms_per_step": 1e3 * el5 / args.steps, "n_gpus": world, "scaling": mode,
                  "parallelism": parallelism(mode, args.band, world),
                  "build_ms": w5.info.build_ms, "rebuild_ms": b5,
                  "bins": {"usable": bool(st5.usable), "list_entries": int(st5.list_entries)},
                  "band_share": share5,
                  "note": "parity: tests/test_gpu_parity.py::test_10m_4k_* (oracle rows, exact walk)"}
        w5.close()
        del w5, t5
        torch.cuda.synchronize()

    # config C4 (BASELINE.json configs[3]): 8-bounce Whitted mirror rays at
    # 3840x2160 on the same soup and tree (bih_render_whitted_device)
    whitted_leg = None
    if world == 1 and args.whitted_frames > 0 and not args.headline_only:
        whitted_leg = whitted(args, bihrt, torch, arrays, SPP, sptr)

    # N > 1: the other decomposition, informational
    side_leg = None
    if world > 1 and not args.headline_only:
        other_mode = "strong" if mode == "weak" else "weak"
        el4, kms4, fps4 = wl.timed(other_mode, trav, 3000)
        side_leg = {"mode": other_mode,
                    "scaling": other_mode,
                    "value": fps4 * rays_per_frame * args.steps / el4, "unit": "rays/s",
                    "ms_per_step": 1e3 * el4 / args.steps, "kernel_ms": kms4,
                    "parallelism": parallelism(other_mode, args.band, world)}

    # a camera that moves every frame: the per-camera structures (primary-ray
    # records, frustum bins and tile queue) are rebuilt inside every step
    moving_leg = None
    if not args.no_rebuild_leg:
        from bihrt import Camera
        base_cam = cam.as_list()
        cams = []
        for k in range(8):
            c = list(base_cam)
            d = (0.002 * k, 0.001 * k, -0.003 * k)
            for j in range(3):
                c[j] += d[j]
                c[3 + j] += d[j]
            cams.append(Camera.from_list(c))
        rows_m, frame_of_m, fps_m = wl.plan(mode, 1)
        for k in range(max(args.warmup, len(cams))):
            r.camera = cams[k % len(cams)]
            wl.step(mode, rows_m, k, frame_of_m(6000, k), trav)
        k0 = max(args.warmup, len(cams))
        sync_all()
        t0 = time.perf_counter()
        for k in range(k0, k0 + args.steps):
            r.camera = cams[k % len(cams)]
            wl.step(mode, rows_m, k, frame_of_m(6000, k), trav)
        sync_all()
        el6 = max_over_ranks(time.perf_counter() - t0)
        kl = k0 + args.steps - 1
        wl.timed_calls = [{"j": kl % C.F, "f0": frame_of_m(6000, kl), "m": 1, "c": kl, "rows": rows_m,
                           "strong": mode == "strong" and world > 1}]
        if world == 1:
            tout.oracle("moving_camera", wl.capture(-1, [0]), args.parity_row_step,
                        cam=cams[kl % len(cams)].as_list())
        r.camera = cam
        moving_leg = {"value": fps_m * rays_per_frame * args.steps / el6, "unit": "rays/s",
                      "ms_per_step": 1e3 * el6 / args.steps,
                      "note": "step = render with a camera that moved since the last frame (8 cameras in "
                              "turn): primary-ray records, frustum bins and tile queue rebuilt per step"}

    # the reference rebuilds the BIH every frame (Renderer::Render,
    # Renderer.cpp:415-503): time rebuild + render per step as well
    rebuild_leg = None
    if not args.no_rebuild_leg:
        # the renders on the other streams than the tree's (streams[0], where
        # the rebuilds go), so that a rebuild never queues behind a render
        # (BIH_REBUILD_STREAMS=all: every stream, as the other legs)
        sep = C.F > 1 and os.environ.get("BIH_REBUILD_STREAMS", "") != "all"
        el3, _, fps3 = wl.timed(mode, trav, 2000, rebuild=True, g=1, nf=C.F - 1 if sep else None,
                                first=1 if sep else 0)
        if world == 1:
            tout.oracle("with_rebuild", wl.capture(-1, [0]), args.parity_row_step)
        rebuild_leg = {"value": fps3 * rays_per_frame * args.steps / el3, "unit": "rays/s",
                       "ms_per_step": 1e3 * el3 / args.steps,
                       "build_ms": arrays.info().build_ms,
                       "render_streams": (C.F - 1) if sep else C.F,
                       "note": "step = bih_rebuild + render"
                               + (" + gather" if mode == "strong" and world > 1 else "")}

    # The reference's frame loop with geometry that changes: before every step
    # the tree's device soup is overwritten (soup A and soup B in turn, the
    # same size, on the tree's stream), then bih_rebuild -- which must now
    # read the new tree's header back (no BIH_PARAM_STATIC_SOUP: the content
    # hash changes) -- and the render, whose camera structures (records,
    # frustum bins, tile queue) are rebuilt for the new tree.
    dyn_leg = None
    if not args.no_rebuild_leg and args.dynamic_leg:
        tris_b = bihrt.scenes.soup(args.tris, seed=2)
        d_a = wl.d_tris.clone()
        d_b = torch.from_numpy(tris_b).to(wl.d_tris.device)
        torch.cuda.synchronize()
        arrays.set_param(bihrt.PARAM_STATIC_SOUP, 0)

        def swap_soup(c):
            with torch.cuda.stream(streams[0]):      # the tree's stream: ordered before the rebuild
                wl.d_tris.copy_(d_b if c % 2 else d_a)

        sep = C.F > 1
        el7, _, fps7 = wl.timed(mode, trav, 12000, rebuild=swap_soup, g=1, nf=C.F - 1 if sep else None,
                                first=1 if sep else 0)
        last_c = wl.timed_calls[-1]["c"]
        if world == 1:
            tout.oracle("dynamic_rebuild", wl.capture(-1, [0]), args.parity_row_step,
                        soup="B" if last_c % 2 else "A")
        dyn_leg = {"value": fps7 * rays_per_frame * args.steps / el7, "unit": "rays/s",
                   "ms_per_step": 1e3 * el7 / args.steps, "soups": "1M soups A (seed 1) and B (seed 2) in turn",
                   "device_allocs_in_leg": wl.timed_allocs,
                   "note": "step = overwrite the tree's device soup with the other soup + bih_rebuild (header "
                           "read back: the soup changed) + render; the camera structures are rebuilt for "
                           "every new tree (src/App.cpp:174-183 -> src/Renderer.cpp:415-501 with moving "
                           "geometry)"}
        # soup A back, and the tree of soup A
        swap_soup(0)
        arrays.rebuild()
        arrays.set_param(bihrt.PARAM_STATIC_SOUP, 1)
        torch.cuda.synchronize()
        del d_a, d_b
        if world == 1:
            C.tris_b = tris_b

    # INTEGRATION.md's C loop: bih_rebuild + bih_render into a host
    # framebuffer, one frame per call (bih_build tree: the library's own copy
    # of the soup).  Pageable framebuffer, then the same buffer page-locked
    # once (bih_host_register): bih_render's device-to-host copy then runs at
    # DMA rate.
    host_leg = None
    if world == 1 and not args.headline_only and args.host_loop:
        hg = bihrt.GPUArrayManager(tris)
        hr = bihrt.Renderer(hg, W, H, spp=SPP, seed=1984, camera=cam)
        fbuf = np.zeros((H, W), np.uint32)
        hg.reserve(W, H, SPP, None, 1)
        res_h = {}
        f = 15000
        for kind, reb in (("pageable", True), ("pinned", True), ("pinned_render_only", False),
                          ("pageable_render_only", False)):
            if kind.startswith("pinned"):
                bihrt.host_register(fbuf)
            for k in range(max(3, args.warmup)):
                if reb:
                    hg.rebuild()
                hr.render(f, out=fbuf)
                f += 1
            t0 = time.perf_counter()
            for k in range(args.steps):
                if reb:
                    hg.rebuild()
                hr.render(f, out=fbuf)
                f += 1
            elh = time.perf_counter() - t0
            if kind in ("pageable", "pinned"):
                tout.oracle(f"host_loop_{kind}", [(f - 1, np.arange(H), fbuf.copy())], args.parity_row_step)
            res_h[kind] = {"ms_per_step": 1e3 * elh / args.steps, "value": rays_per_frame * args.steps / elh}
            if kind.startswith("pinned"):
                bihrt.host_unregister(fbuf)
        host_leg = dict(res_h)
        host_leg.update({
            "pinned_speedup": res_h["pageable"]["ms_per_step"] / res_h["pinned"]["ms_per_step"],
            "pinned_speedup_render_only": (res_h["pageable_render_only"]["ms_per_step"] /
                                           res_h["pinned_render_only"]["ms_per_step"]),
            "unit": "rays/s",
            "note": "step = bih_rebuild + bih_render (one frame, 8.3 MB into a host framebuffer, synchronous) "
                    "as INTEGRATION.md's C loop; pinned = the same buffer after bih_host_register; "
                    "*_render_only: bih_render alone (reference: D2D copy into the GL buffer, "
                    "src/Renderer.cpp:645-655)"})
        hg.close()
        del hg, hr

    # the dominant kernel's launch duration: HIP events the library records
    # on the render stream right around the render kernel (bih_last_render_ms),
    # over isolated launches (each call synchronised before the next) -- the
    # figure rocprofv3's kernel trace reports for the same kernel
    # (the headline's launches: a call of G frames, one k_render_bins launch;
    # the calls rotate over the headline's streams as its do, so the render
    # runs through the XORWOW ring -- k_render_bins<L, 0>, the headline's
    # instance; a run of calls on one stream switches to the stamped state)
    kms_iso, tails_iso = [], []
    r.set_timing(True)
    for k in range(args.kernel_samples):
        wl.step(mode, rows, k, frame_of(5000, k * G), trav, m=G)
        torch.cuda.synchronize()
        km, tm = r.last_render_times()
        kms_iso.append(km)
        tails_iso.append(tm)
    r.set_timing(False)
    kernel_launch_ms = sum(kms_iso) / len(kms_iso) if kms_iso else None

    # per-ray work counters of one frame (untimed): exact integers, equal to
    # the oracle's (tests/test_gpu_parity.py::test_per_ray_counters_match_oracle)
    stat_frame = args.warmup
    nloc = rows.nrows * W * SPP
    st = torch.zeros(3 * nloc, dtype=torch.int32, device="cuda")
    r.render_device(out.data_ptr(), stat_frame, rows=rows, traverse=trav, stats_ptr=st.data_ptr(),
                    stream=sptr)
    torch.cuda.synchronize()
    sums = st.view(-1, 3).to(torch.int64).sum(0)
    del st
    if dist is not None and mode == "strong":
        dist.all_reduce(sums)
    n_node, n_leaf, n_tri = [int(x) for x in sums.tolist()]
    rays_all = rays_per_frame
    b_ray = (NODE_B * n_node + LEAF_B * n_leaf + TRI_B * n_tri) / rays_all + (FB_B + RNG_B) / SPP
    launch_rays = rows.nrows * W * SPP * (G if trav == 0 else 1)   # rays of one headline launch
    # per-launch duration of the kernel: with frames in flight a launch's
    # events also count the time it queues behind the other stream's frame,
    # so the isolated launches give the duration (what rocprofv3 reports for
    # `--headline-only --in-flight 1`)
    launch_ms = kernel_launch_ms if kernel_launch_ms else (serial_leg["kernel_ms"] if serial_leg else kernel_ms)
    work_gbs = b_ray * launch_rays / (launch_ms * 1e-3) / 1e9 if launch_ms else None
    achieved = traffic["bytes_per_launch"] / (launch_ms * 1e-3) / 1e9 if traffic else None

    bst = arrays.bins_stats()
    # algorithmic bytes of one k_render_bins launch: every list entry of the
    # frame read once per frame (48 B: 3 edge functions + pixel mask), one 64-B
    # intersector record per packet-level intersector call, the XORWOW state
    # (20 B) and the framebuffer word (4 B) per pixel; and the compulsory
    # bytes of the same launch (what must cross HBM at least once when the
    # list stays cached across the launch's frames: list + records + RNG in
    # and out once, a framebuffer per frame)
    alg = None
    bc = (traffic or {}).get("bin_counters")
    if bc and trav == 0 and bst.usable and launch_ms:
        pix = rows.nrows * W
        gl = G if trav == 0 else 1       # frames per k_render_bins launch
        alg_bytes = gl * (48 * int(bst.list_entries) + 64 * bc["mt"] + 24 * pix)
        comp_bytes = 48 * int(bst.list_entries) + 64 * bc["mt"] + 2 * 20 * pix + gl * 4 * pix
        alg = {"bytes_per_launch": alg_bytes, "frames_per_launch": gl,
               "terms": {"list_entries": int(bst.list_entries), "intersector_calls": bc["mt"],
                         "pixels": pix, "entries_pretested": bc["entries"], "live_lanes": bc["lanes"],
                         "live_packets": bc["packets"]},
               "formula": "frames per launch x (48 x list entries + 64 x intersector calls + "
                          "(20 + 4) x pixels), per-frame terms of one frame (tools/fast_counters.py)",
               "gbs": alg_bytes / (launch_ms * 1e-3) / 1e9,
               "compulsory_bytes_per_launch": comp_bytes,
               "compulsory_formula": "48 x list entries + 64 x intersector calls + 2 x 20 x pixels "
                                     "(XORWOW in, out) + frames per launch x 4 x pixels",
               "compulsory_gbs": comp_bytes / (launch_ms * 1e-3) / 1e9}
        if window:
            # per frame over the timed window's own kernel time (union of its launches)
            kpf = window["kernel_ms_per_frame"]
            alg["bytes_per_frame"] = alg_bytes / gl
            alg["window_gbs"] = alg_bytes / gl / (kpf * 1e-3) / 1e9
            alg["window_compulsory_gbs"] = comp_bytes / gl / (kpf * 1e-3) / 1e9
        # What the kernel itself addresses per frame at the headline's call
        # shape (counter build, a 16-frame call with the hit cache warm): the
        # entries it pre-tests (48 B), its packet-level intersector records
        # (64 B), each live lane's hit-cache record (52 B) and the per-pixel RNG
        # and framebuffer words (24 B) -- a lower bound (whole 64-entry chunks
        # are loaded).  Since round 6's hit cache most lanes no longer walk
        # their tile's list, so the model above (every list entry once per
        # frame, kept from earlier rounds for comparability) counts far more
        # than the kernel reads.
        hs = bc.get("headline_shape")
        if hs and window:
            per = (48 * hs["entries"] + 64 * hs["mt"] + 52 * hs["lanes"]) / G + 24 * pix
            alg["addressed_bytes_per_frame"] = per
            alg["addressed_gbs"] = per / (window["kernel_ms_per_frame"] * 1e-3) / 1e9
            alg["addressed_terms_per_frame"] = {k: hs[k] / G for k in ("entries", "mt", "lanes", "cache-hits")
                                                if k in hs}
            alg["addressed_formula"] = ("(48 x entries pre-tested + 64 x intersector calls + 52 x live lanes) per "
                                        "frame of a 16-frame call + 24 x pixels (counter build)")
    # the issue roofline of the same kernel: VALU wave-instructions (PMC,
    # SQ_INSTS_VALU per launch of the headline shape) at 2 cycles each on a
    # SIMD (a wave64 VALU op issues over 2 cycles: MI355X_MICROARCH.md), over
    # 1024 SIMDs x 2.4 GHz for the kernel time per frame
    issue = None
    sq = (traffic or {}).get("sq")
    if sq and trav == 0 and (window or launch_ms):
        gl = G
        kpf = window["kernel_ms_per_frame"] if window else launch_ms / gl
        valu_f, salu_f = sq["SQ_INSTS_VALU"] / gl, sq["SQ_INSTS_SALU"] / gl
        issue = {"valu_per_frame": valu_f, "salu_per_frame": salu_f,
                 "valu_issue_frac": valu_f * 2 / (1024 * 2.4e9 * kpf * 1e-3),
                 "kernel_ms_per_frame": kpf,
                 "formula": "SQ_INSTS_VALU per frame x 2 cycles / (1024 SIMDs x 2.4 GHz x kernel ms per frame)",
                 "source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU per dispatch of the headline's "
                           f"{G}-frame k_render_bins launches (tools/prof_render.py)"}
    bins = {"usable": bool(bst.usable), "tiles": [bst.tiles_x, bst.tiles_y],
            "list_entries": int(bst.list_entries), "global_entries": int(bst.global_entries),
            "entry_bytes": 48,
            "note": "frustum bins of the bench camera (bih_bins_get_stats): per 4x4-pixel tile the "
                    "triangles whose edge pre-test a sample of the tile can pass"}

    # N > 1 strong: rank 0's gathered headline frames against rank 0's own
    # one-GPU render of the same frames (whole frames, one call each)
    if world > 1 and mode == "strong" and rank == 0:
        full_rows = tiling.band_rows(H, args.band, 0, 1)
        arrays.reserve(W, H, SPP, full_rows, G)
        for i, (f, ys, img) in head_caps:
            r.render_device_frames(out.data_ptr(), f, 1, H * W, rows=full_rows, stream=sptr)
            torch.cuda.synchronize()
            ref = out[: H * W].cpu().numpy().view(np.uint32).reshape(H, W)
            tout.gpu("headline", f, np.array_equal(img, ref),
                     "rank 0's gathered frame vs its own one-GPU render of the same frame, every pixel")

    cpu = None
    parity = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu, parity = cpu_baseline(args, tris, wl, trav, W, H, SPP, torch, np, tout, getattr(C, "tris_b", None))

    rccl = None
    if backend == "nccl":
        try:
            rccl = ".".join(str(x) for x in torch.cuda.nccl.version())
        except Exception:
            rccl = None
    ach = (alg["window_gbs"] if alg and "window_gbs" in alg else alg["gbs"] if alg else achieved)
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": mode,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: 1M-triangle soup, splitmix64 seed 1, centroids U([0,2.667]x[-1,1]x[0,2]) "
                    "+ U(-0.02,0.02)^3 vertices (SURVEY.md 8d C3)",
            "config": {
                "workload": f"{args.tris}-triangle random soup, {W}x{H}, {SPP} spp primary rays, "
                            "reference camera, XORWOW seed 1984",
                "tris": args.tris, "unique_codes": info.n_unique, "width": W, "height": H,
                "spp": SPP, "traverse": args.traverse,
                "parallelism": parallelism(mode, args.band, world),
                "frames_in_flight": F,
                "frames_per_call": G,
                "calls": call_sizes(args.steps, G),
                "warmup_calls": call_sizes(args.warmup, G) + [m for m in sorted(set(call_sizes(args.steps, G)))
                                                              if m not in call_sizes(args.warmup, G)],
            },
            "world_size": world,
            "backend": backend,
            "rccl_version": rccl,
            "device_allocs_in_headline": allocs_headline,
            "kernel_ms": kernel_ms,
            "build_ms": info.build_ms,
            # roofline of the dominant kernel: HBM is the only roofline this
            # integer/f32 path has (no MFMA work).  `achieved` = the launch's
            # algorithmic bytes over its duration; `traffic` =
            # the HBM bytes the PMC counters measured per launch (the list stays
            # in cache across the launch's frames, so traffic is far below the
            # algorithmic bytes); `frac_compulsory` prices the bytes that must
            # cross HBM once per launch.  What limits the kernel is `limiter`.
            "roofline": {
                "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": ach / HBM_PEAK_GBS if ach is not None else None,
                "traffic": traffic["bytes_per_launch"] if traffic else None,
                "achieved_source": ("algorithmic bytes per frame (roofline.algorithmic) / kernel ms per frame of "
                                    "the timed window's shape (roofline.window: union of its launches' HIP-event "
                                    "intervals)" if (alg and window) else
                                    "algorithmic bytes per launch (roofline.algorithmic) / launch_ms" if alg else
                                    "measured bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE) / launch_ms"
                                    if achieved is not None else "traffic not measured"),
                "algorithmic": alg,
                "frac_algorithmic": alg["gbs"] / HBM_PEAK_GBS if alg else None,
                "frac_compulsory": alg["compulsory_gbs"] / HBM_PEAK_GBS if alg else None,
                "achieved_measured": achieved,
                "frac_measured": achieved / HBM_PEAK_GBS if achieved is not None else None,
                "launch_ms": launch_ms,
                "window": window,
                "issue": issue,
                "frac_isolated_launches": alg["gbs"] / HBM_PEAK_GBS if alg else None,
                "frac_addressed": (alg["addressed_gbs"] / HBM_PEAK_GBS) if alg and "addressed_gbs" in alg else None,
                "fallback_ms": (sum(tails_iso) / len(tails_iso)) if tails_iso else None,
                "frames_per_launch": G if trav == 0 else 1,
                "launch_ms_source": (f"HIP events around the render kernel on its stream "
                                     f"(bih_last_render_times), mean of {len(kms_iso)} isolated launches "
                                     f"of the headline's calls ({G if trav == 0 else 1} frames each)")
                                    if kernel_launch_ms else "headline leg",
                "limiter": "instruction issue and memory latency of the list walk, not HBM "
                           "(DESIGN.md section 4: SQ counters)",
                "kernel": (traffic or {}).get("kernel") or
                          ("k_render_bins (any-hit: frustum-bin list walk; k_render_fallback finishes "
                           "undecided packets)" if trav == 0 else "k_render_packet_asm (reference walk)"),
            },
            "work_equivalent": {
                "bytes_per_ray": b_ray,
                "counters_per_ray": {"nodes": n_node / rays_all, "leaves": n_leaf / rays_all,
                                     "tris": n_tri / rays_all},
                "gbs": work_gbs,
                "roofline_rays_per_s": HBM_PEAK_GBS * 1e9 / b_ray,
                "rays_vs_roofline_rays": value / (HBM_PEAK_GBS * 1e9 / b_ray),
                "note": "SURVEY 8d B_ray = 16 n_node + 8 n_leaf + 40 n_tri + 52/spp over the exact "
                        "walk's per-ray counters (the reference algorithm's node/leaf/triangle "
                        "visits, equal to the oracle's); the roofline rays/s is 8 TB/s / B_ray. "
                        "The shortcut passes reach the same pixels with far fewer visits, so this "
                        "prices work the kernel does not do: it is not a bandwidth",
            },
            "traffic_detail": traffic,
            "bins": bins,
            "cpu_baseline": cpu,
            "other_traversal": ref_leg,
            "with_rebuild": rebuild_leg,
            "dynamic_rebuild": dyn_leg,
            "host_loop": host_leg,
            "moving_camera": moving_leg,
            "one_in_flight": serial_leg,
            "other_decomposition": side_leg,
            "band_share": share_leg,
            "whitted_c4": whitted_leg,
            "c2_torus": c2_leg,
            "c5_10m_4k": c5_leg,
        }
        if parity is not None:
            res["parity_timed_call_shape"] = parity
            res["parity_sample_rows_equal"] = parity["all_equal"]
        # what the timed calls themselves wrote
        ts = tout.summary()
        res["timed_outputs_equal"] = ts["all_equal"] if ts["checks"] else None
        res["timed_outputs"] = ts
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def whitted(args, bihrt, torch, arrays, SPP, sptr):
    """Config C4: frames of 8-bounce mirror rays at 3840x2160 on the bench soup."""
    WW, WH = 3840, 2160
    rw = bihrt.Renderer(arrays, WW, WH, spp=SPP, seed=1984)
    wout = torch.zeros(WW * WH, dtype=torch.int32, device="cuda")
    whits = torch.zeros(WW * WH * SPP, dtype=torch.int32, device="cuda")
    rw.render_whitted_device(wout.data_ptr(), 0, hits_ptr=whits.data_ptr(), stream=sptr)
    torch.cuda.synchronize()
    traced = int(torch.clamp(whits.to(torch.int64) + 1, max=9).sum())
    hist = torch.bincount(whits.view(-1), minlength=10).tolist()
    del whits
    rw.set_timing(True)
    t0 = time.perf_counter()
    for k in range(args.whitted_frames):
        rw.render_whitted_device(wout.data_ptr(), 1 + k, stream=sptr)
    torch.cuda.synchronize()
    wel = (time.perf_counter() - t0) / args.whitted_frames
    wk, _ = rw.last_render_times()
    rw.set_timing(False)
    # work of one more frame (untimed, counters on): per bounce the rays, the
    # nodes their walks entered and the triangles they tested; algorithmic
    # bytes = 16 B per node record + 36 B per triangle record ({v0, e1, e2})
    # + 28 B per ray read from its queue and, for rays that hit, written to
    # the next one -- over the trace kernels' time (wk)
    arrays.set_param(bihrt.PARAM_WHITTED_COUNTERS, 1)
    rw.render_whitted_device(wout.data_ptr(), 1 + args.whitted_frames, stream=sptr)
    work = rw.whitted_work()
    arrays.set_param(bihrt.PARAM_WHITTED_COUNTERS, 0)
    torch.cuda.synchronize()
    del wout
    nodes, tris_t, rays = sum(work["nodes"]), sum(work["tris"]), sum(work["rays"])
    alg = 16 * nodes + 36 * tris_t + 28 * rays + 28 * sum(work["rays"][1:])
    work_leg = {"per_bounce": work, "nodes_per_ray": nodes / max(1, rays), "tris_per_ray": tris_t / max(1, rays),
                "algorithmic_bytes": alg,
                "formula": "16 x nodes + 36 x triangles tested + 28 x rays read + 28 x rays written",
                "algorithmic_gbs": alg / (wk * 1e-3) / 1e9 if wk else None,
                "frac_of_hbm_peak": alg / (wk * 1e-3) / 1e9 / HBM_PEAK_GBS if wk else None,
                "note": "records are re-read from L2/MALL far more than from HBM (the tree and soup are "
                        "52 MB): the bound is the per-lane gather rate of the walk, not HBM bandwidth"}
    return {"config": "C4: 1M soup, 3840x2160, 4 spp, 8 bounces of mirror rays",
            "ms_per_frame": 1e3 * wel, "primary_rays_per_s": WW * WH * SPP / wel,
            "rays_traced_per_frame": traced, "rays_traced_per_s": traced / wel,
            "trace_kernels_ms": wk, "hit_histogram": hist, "frames": args.whitted_frames,
            "work": work_leg,
            "note": "k_wh_gen + 9 x k_wh_trace (closest hit, per-lane walk, ballot/mbcnt "
                    "compaction of live rays between bounces) + k_wh_shade; bit-exact vs the "
                    "oracle (tests/test_whitted.py)"}


def median_ms(wl, mode, trav, base, reps, steps, rows=None):
    """Median over `reps` timed windows of the same call shape (ms per frame)."""
    v = sorted(1e3 * wl.timed(mode, trav, base, rows=rows)[0] / steps for _ in range(max(1, reps)))
    return v[len(v) // 2]


def check_shares(tout, leg, full, parts, H, band, Q, tiling):
    """The Q band shares' last frames (each rendered alone, timed) laid out
    in frame order (tiling.assemble) equal the full-frame leg's last frame,
    the same frame index, on every pixel."""
    f, _, img = full
    frames = {p[0] for p in parts}
    ok = frames == {f} and all(p[2].shape[0] == p[1].size for p in parts)
    if ok:
        got = tiling.assemble([p[2] for p in parts], H, band, Q)
        ok = bool(np.array_equal(got, img))
    tout.gpu(leg, f, ok, f"the {Q} shares' last frames reassembled (tiling.assemble) vs the full-frame "
                         "leg's last frame, every pixel")


def parallelism(mode, band, world):
    if world == 1:
        return "1 GPU, whole frames"
    if mode == "weak":
        return f"whole frames in groups of consecutive frames, round-robin over {world} GPUs, no collective"
    return (f"row bands of {band} rows interleaved over {world} GPUs + one RCCL gather of the bands "
            "to rank 0 per render call")


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads(args):
    """Host threads for the OpenMP legs: every CPU this process may run on
    (sched_getaffinity), unless OMP_NUM_THREADS names the box's CPU share
    (the GPU pool sets it to 16 per GPU) or --cpu-threads overrides."""
    aff = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n = args.cpu_threads or (min(aff, omp) if omp > 0 else aff)
    return n, aff, omp


def cpu_baseline(args, tris, wl, trav, W, H, SPP, torch, np, tout=None, tris_b=None):
    """The oracle (strict-IEEE C restatement of the reference's render path,
    oracle/bih_oracle.c) timed on the host, on bounded row samples of frame 0
    of the same workload:
      value   -- the reference walk (TraverseTree, CUDAKernels.cu:227-368,
                 MODE_GPU_REF) with OpenMP over the host threads;
      anyhit  -- the same walk stopped at the first hit (MODE_GPU_ANYHIT),
                 OpenMP;
      serial  -- the reference walk on one thread;
      host_debug_serial -- the reference's own serial host loop and rules
                 (DebugRender / CPUTraverseTree, Renderer.cpp:202-412,
                 MODE_HOST_DEBUG), one thread: config C1's semantics.
    Then the parity of the timed call shape: one call of G frames through the
    path the headline times (bih_render_device_frames, frames 0..G-1), its
    frame 0 compared with the rows the four CPU legs rendered, frames 7 and
    G-1 with oracle rows (cudaRender carries the XORWOW state across frames,
    CUDAKernels.cu:411-419)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads, aff, omp = cpu_threads(args)
    ot = oracle.OracleTree(tris)
    legs = {}
    imgs = []

    def leg(name, mode, step, nthreads, row0=0):
        nrows = math.ceil((H - row0) / step)
        img, st = ot.render(W, H, spp=SPP, frame=0, rows=(row0, nrows, step), mode=mode,
                            threads=nthreads)
        imgs.append((0, row0, step, img))
        legs[name] = {"value": st.rays / st.render_seconds, "unit": "rays/s", "cores": st.threads,
                      "seconds": st.render_seconds, "rays": st.rays,
                      "sample": f"rows {row0}::{step} of frame 0 ({nrows} rows x {W} px x {SPP} spp)",
                      "per_ray": {"nodes": st.node_visits / st.rays, "leaves": st.leaf_visits / st.rays,
                                  "tris": st.tri_tests / st.rays}}

    leg("reference_walk", oracle.MODE_GPU_REF, args.cpu_row_step, threads)
    leg("anyhit", oracle.MODE_GPU_ANYHIT, args.cpu_row_step, threads)
    leg("serial", oracle.MODE_GPU_REF, args.cpu_serial_row_step, 1)
    leg("host_debug_serial", oracle.MODE_HOST_DEBUG, args.cpu_debug_row_step, 1,
        row0=args.cpu_debug_row_step // 2)
    G = max(1, args.group)
    ps = args.parity_row_step
    for f in sorted({min(7, G - 1), G - 1} - {0}):
        img, _ = ot.render(W, H, spp=SPP, frame=f, rows=(0, math.ceil(H / ps), ps),
                           mode=oracle.MODE_GPU_ANYHIT, threads=threads)
        imgs.append((f, 0, ps, img))
    # the timed call shape, untimed: G frames in one call on the headline's stream 0
    from bihrt.tiling import band_rows
    wl.step("weak", band_rows(H, args.band, 0, 1), 0, 0, trav, m=G)
    torch.cuda.synchronize()
    frames = wl.outs[0][: G * H * W].cpu().numpy().view(np.uint32).reshape(G, H, W)
    checks = [{"frame": f, "rows": f"{row0}::{step}", "equal": bool(np.array_equal(frames[f][row0:H:step], img))}
              for f, row0, step, img in imgs]
    parity = {"call": f"bih_render_device_frames, frames 0..{G - 1} in one call", "checks": checks,
              "all_equal": all(c["equal"] for c in checks)}
    # the frames the timed legs wrote (TimedOutputs.pending), against the
    # oracle of their soup, camera and frame
    if tout is not None and tout.pending:
        trees = {"A": ot}
        t0 = time.perf_counter()
        for p in tout.pending:
            key = p["soup"]
            if key not in trees:
                import bihrt
                trees[key] = oracle.OracleTree(tris_b if key == "B" else bihrt.scenes.torus())
            t = trees[key]
            ys = p["ys"]
            step = int(ys[1] - ys[0]) if ys.size > 1 else 1
            cam = np.array(p["cam"], np.float32) if p["cam"] is not None else None
            if ys.size and np.array_equal(ys, ys[0] + step * np.arange(ys.size)):
                ref, _ = t.render(W, H, spp=SPP, frame=p["frame"], cam=cam, rows=(int(ys[0]), int(ys.size), step),
                                  mode=oracle.MODE_GPU_ANYHIT, threads=threads)
            else:
                ref = np.concatenate([t.render(W, H, spp=SPP, frame=p["frame"], cam=cam, rows=(int(y), 1, 1),
                                               mode=oracle.MODE_GPU_ANYHIT, threads=threads)[0] for y in ys])
            rows_txt = "every row" if step == 1 and ys.size == H else f"rows {int(ys[0])}::{step}"
            tout.gpu(p["leg"], p["frame"], np.array_equal(ref, p["img"]),
                     f"oracle (soup {key}{', moved camera' if cam is not None else ''}), {rows_txt}")
        tout.oracle_seconds = time.perf_counter() - t0
        tout.pending = []
    main = legs["reference_walk"]
    res = {"value": main["value"], "unit": "rays/s", "cores": main["cores"], "kind": "port",
           "sample": main["sample"] + ", oracle/bih_oracle.c reference walk (TraverseTree rules), "
                     f"OpenMP {main['cores']} threads",
           "seconds": main["seconds"],
           "cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": aff,
           "omp_num_threads_env": omp or None,
           "threads_rule": "min(sched_getaffinity, OMP_NUM_THREADS) -- the box's CPU share",
           "legs": legs}
    return res, parity


def measure_traffic(args):
    """FETCH_SIZE and WRITE_SIZE (KB, rocprofv3, one counter per pass) of the
    render kernel over tools/prof_render.py on this workload; gfx950
    correction: FETCH_SIZE x 2 (MI355X_MICROARCH.md, HBM section).  These are
    L2-to-fabric bytes: Infinity Cache hits are included."""
    import csv
    import glob
    import re
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    res = {}
    tmp = tempfile.mkdtemp(prefix="bih_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    traverse = args.traverse
    # the headline's renders run with calls in flight on several streams, so
    # through the XORWOW ring (k_render_bins<L, 0>) and the shared grid; the
    # traffic driver rotates its calls over as many streams (and keeps the
    # ring even if it did not)
    env["BIH_STAMPED"] = "0"
    sq = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU SQ_INSTS_SALU"):
        out = os.path.join(tmp, ctr.split()[0])
        cmd = [prof, "--pmc"] + ctr.split() + ["-d", out, "-o", ctr.split()[0], "--output-format", "csv", "--",
               sys.executable, os.path.join(ROOT, "tools", "prof_render.py"), "--frames", "6",
               "--tris", str(args.tris), "--width", str(args.width), "--height", str(args.height),
               "--spp", str(args.spp), "--traverse", traverse, "--group", str(max(1, args.group)),
               "--streams", str(max(1, args.in_flight))]
        try:
            p = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, timeout=300)
        except (OSError, subprocess.TimeoutExpired):
            if ctr.startswith("SQ"):
                continue
            return None
        if p.returncode != 0:
            if ctr.startswith("SQ"):
                continue
            return None
        # the dominant render kernel: k_render_bins (any-hit with frustum
        # bins; the plain instance <L, 0>, not the first launch's cost
        # measuring <L, 2>), else the BIH packet kernel; per dispatch (a
        # counter may come split over dimensions: summed)
        per = {}
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"]
                if "k_render_bins" in name:
                    if not re.search(r"k_render_bins<\d+, 0>", name):
                        continue
                    key = "k_render_bins"
                elif "k_render_packet_asm" in name:
                    key = "k_render_packet_asm"
                else:
                    continue
                did = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(per))
                cname = row.get("Counter_Name", ctr)
                per[(key, did, cname)] = per.get((key, did, cname), 0.0) + float(row["Counter_Value"])
        for cname in ctr.split():
            vals = {}
            for (key, _, cn), v in sorted(per.items(), key=lambda kv: int(kv[0][1]) if kv[0][1].isdigit() else 0):
                if cn == cname:
                    vals.setdefault(key, []).append(v)
            key = "k_render_bins" if "k_render_bins" in vals else "k_render_packet_asm"
            if not vals.get(key):
                if ctr.startswith("SQ"):
                    continue
                return None
            kernel_name = key
            # (the first launch reads the camera's structures from HBM for the
            # first time: left out when there are others)
            v = vals[key][1:] if len(vals[key]) > 2 else vals[key]
            (sq if ctr.startswith("SQ") else res)[cname] = sum(v) / len(v)
    shutil.rmtree(tmp, ignore_errors=True)
    fetch = 2.0 * res["FETCH_SIZE"] * 1024.0
    write = res["WRITE_SIZE"] * 1024.0
    return {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
            "raw_kb": res, "correction": "FETCH_SIZE x2 (gfx950), KB x 1024", "kernel": kernel_name,
            "sq": sq if len(sq) == 2 else None,
            "bin_counters": bin_counters(args, env)}


FC_LIB = os.path.join(ROOT, "bih-gpu-raytracer_amd", "lib", "variants", "libbih_amd_fc.so")


def bin_counters(args, env):
    """Work counters of k_render_bins on this workload's frame: a child
    process renders two frames with the BIH_FAST_COUNTERS=1 build of the same
    sources (lib/variants/libbih_amd_fc.so, built by __graft_entry__.build)
    and prints them (tools/fast_counters.py).  Frame 1's line is returned."""
    import subprocess
    if not os.path.exists(FC_LIB):
        return None

    def run(extra):
        cmd = [sys.executable, os.path.join(ROOT, "tools", "fast_counters.py"), "--tris", str(args.tris),
               "--width", str(args.width), "--height", str(args.height)] + extra
        try:
            p = subprocess.run(cmd, env=dict(env, BIH_LIB=FC_LIB), capture_output=True, text=True,
                               timeout=300)
        except (OSError, subprocess.TimeoutExpired):
            return None
        lines = [l for l in p.stderr.splitlines() if l.startswith("bin-counters")]
        if p.returncode != 0 or not lines:
            return None
        tok = lines[-1].split("|")[0].split()[1:]
        return {k: int(v) for k, v in zip(tok[0::2], tok[1::2])}

    res = run(["--frames", "2"])
    if res is not None and args.group > 1:
        # the headline's call shape: the third call of G frames (hit cache
        # warm), totals over its G frames
        res["headline_shape"] = run(["--frames", "3", "--group", str(args.group)])
    return res


if __name__ == "__main__":
    main()
